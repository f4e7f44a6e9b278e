"""Data-parallel PPOLearner.learn() at the benched widths, pinned to the same
fp64 truth and envelope as the single-GPU full-size cases
(tests/golden/envelope_<case>.npz, tests/parity.py).

Two processes share cuda:0 and exchange over torch.distributed (gloo: RCCL
refuses two ranks on one GPU; on a multi-GPU node the same code runs over
'nccl' = RCCL/xGMI, as bench.py does).  Each rank learns its half of the
global batch (segments sharded on the batch axis).  Required:
  * the ranks end bit-identical (parameters, ZFilter);
  * rank 0's parameters, advantages (both halves), returns and ZFilter sums lie
    within the fp32 envelope of the fp64 oracle's learn() on the GLOBAL batch;
  * every statistic is self-consistent in fp64 with the global state.
Cases: C3 (LSTM 100, heads 300x200, obs 42, act 8, 10 + 10 epochs) as 2 x 512
segments, adapt over two learns and clip; C5 (C3 + camera stem, FC 256) as
2 x 64 segments; and the strong-scaled compositions of BASELINE configs[2]:
the c3_adapt fixture as 4 x 256 and 8 x 128 segments (one process per rank, all
on cuda:0: ranks share the GPU, the exchange is gloo over host memory).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, outdir):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from surreal_amd import synthetic
    from surreal_amd.learner import TorchDistAllReduce
    from tests import parity as P
    from tests.test_gpu_parity_pinned import _used, fixture_learner
    meta, fx, c, st, learner = fixture_learner(case, dp=TorchDistAllReduce())
    B = learner.batch_size
    lo, hi = rank * B, (rank + 1) * B
    res = []
    for it in range(len(c['batch_seeds'])):
        full = P.case_batch(case, it)

        def cut(x):
            if x is None:
                return None
            if isinstance(x, dict):
                return {k: cut(v) for k, v in x.items()}
            if isinstance(x, list):
                return [cut(v) for v in x]
            return x[lo:hi].contiguous()
        cap = P.learn_capture(learner, synthetic.to_device(cut(full), 'cuda:0'))
        adv, ret = _used(learner)
        r = {'stats': learner.last_stats(), 'adv': torch.from_numpy(adv), 'ret': torch.from_numpy(ret)}
        if rank == 0:
            r['cap'] = cap
        else:
            r['final'] = cap['final']
        res.append(r)
    torch.save(res, os.path.join(outdir, f'rank{rank}.pt'))
    dist.destroy_process_group()


@pytest.mark.timeout(900)
@pytest.mark.parametrize('case,world', [('c3_adapt', 2), ('c3_clip', 2), ('c5', 2),
                                        ('c3_adapt', 4), ('c3_adapt', 8)])
def test_dp_ranks_match_global_fixture(case, world):
    from tests import parity as P
    from tests.helpers import oracle_batch
    with tempfile.TemporaryDirectory() as outdir:
        mp.spawn(_worker, args=(world, _free_port(), case, outdir), nprocs=world, join=True)
        out = [torch.load(os.path.join(outdir, f'rank{r}.pt'), weights_only=True)
               for r in range(world)]
    meta, fx = P.load_fixture(case)
    c = P.CASES[case]
    lc = c['cfg']()
    st = P.init_state(case)
    report = {}
    for it in range(len(c['batch_seeds'])):
        r0 = out[0][it]
        fin = r0['cap']['final']
        for rk in range(1, world):
            rr = out[rk][it]
            for k in ('actor', 'critic', 'lstm', 'cnn'):
                if k in fin:
                    assert torch.equal(fin[k], rr['final'][k]), (it, rk, k)
            for a, b in zip(fin['zf'], rr['final']['zf']):
                assert torch.equal(a, b), (it, rk)
            assert rr['stats'] == r0['stats'], (it, rk)
        assert r0['stats']['epochs_run'] == meta['epochs_run'][it]
        adv = np.concatenate([out[rk][it]['adv'].numpy() for rk in range(world)])
        ret = np.concatenate([out[rk][it]['ret'].numpy() for rk in range(world)])
        from tests.test_gpu_parity_pinned import check_fixture_state
        check_fixture_state(meta, fx, st, it, fin, adv, ret, fin['zf'], report, tag='_dp')
        batch = P.case_batch(case, it)
        rec = P.recompute_stats(lc, c['D'], c['A'], c['pixel'], oracle_batch(batch), r0['cap'],
                                adv, ret, r0['stats']['epochs_run'])
        P.check_stats(r0['stats'], rec, report, tag=f'_dp@{it}')
    P.print_report(report, f'{case}_dp{world}')
