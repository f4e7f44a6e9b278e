"""bench.py's multi-GPU launch path on the CPU: `bench.py --gpus N` without a
launcher spawns N ranks under torch.distributed.run (SMI_BENCH_PROBE=1 makes
each rank report its RANK / WORLD_SIZE / LOCAL_RANK and exit before any GPU
call), and the strong-scaling split of the C3 / C5 global batch."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_flag_spawns_ranks():
    env = dict(os.environ, SMI_BENCH_PROBE='1')
    env.pop('WORLD_SIZE', None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--steps', '1'],
                         env=env, capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    rows = [json.loads(line) for line in out.stdout.splitlines() if line.startswith('{')]
    assert sorted(r['rank'] for r in rows) == [0, 1]
    assert all(r['world'] == 2 for r in rows)
    assert sorted(r['local_rank'] for r in rows) == [0, 1]


def test_strong_scaling_split():
    sys.path.insert(0, ROOT)
    import bench
    for cfg in ('c3', 'c5'):
        lc, ec, dims = bench.make_config(cfg)
        assert dims['B_global'] == 1024
        for n in (1, 2, 4, 8):
            assert dims['B_global'] % n == 0
    lc, ec, dims = bench.make_config('c2')
    assert dims['B_global'] == 64 and lc.replay.batch_size == 64
