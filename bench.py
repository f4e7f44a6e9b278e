"""Learner throughput benchmark (driver contract: see DESIGN.md §6 Measurement).

A step = one PPOLearner.learn() over one synthetic batch already resident in
HBM (reward scaling, critic forward + windowed GAE, the policy epochs with the
device-side KL early stop, the value epochs, z_update).

--config c3 (default; BASELINE configs[2], "1024-actor batch, data parallel
over 2/4/8 GPUs"): the reference PPO defaults — LSTM policy
(rnn_hidden 100, horizon 5), heads 300x200, n_step 25, adapt mode, z-filter —
with robosuite SawyerLift state dims (obs 42, act 8; SURVEY §8 notes 42 is an
assumption): 1024 segments per learn() in total, split over the GPUs
(--scaling strong, the default; --scaling weak keeps 1024 per GPU).
--config c2 (BASELINE configs[1]): HalfCheetah dims, 64x64 MLP, 64 x 50 per GPU.
--config c5 (BASELINE configs[4]): C3 plus the pixel stem — camera0
3x84x84 uint8 -> conv 16@8s4 -> 32@4s2 -> FC 256, LSTM input 42 + 256 — the
same 1024 segments split over the GPUs.
--config c4 (BASELINE configs[3]): the DDPG learner (see run_ddpg).

With --gpus N the learner is data parallel: one process per GPU
(launched by torch.distributed.run, or spawned by this script when no launcher
set WORLD_SIZE), each rank holds its shard of the segments and the ranks
all-reduce advantage moments, per-epoch gradients/statistics and the ZFilter
sums over RCCL (torch.distributed 'nccl'); every rank applies the update of the
global batch.

Prints ONE JSON line on rank 0: the metric (timed region = K plain learn()
calls, no instrumentation), a roofline object for the dominant kernel
(per-launch HIP events recorded by libsurreal_mi on the learner's stream in a
separate instrumented pass of min(K, 5) learn() calls right after the timed
region) and the CPU baseline (the oracle restatement, timed on this host on a
bounded sample).
"""
import argparse
import copy
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'PPO learner env-steps/sec/node (GAE+update) at 1/2/4/8 GPUs; % HBM roofline'
FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: v_mfma_f32_* dense peak
HBM_PEAK_GBS = 8000.0


def make_config(name):
    """(learner_config, env_config, dims) of a bench workload; dims['B_global']
    is the workload's segment count (the global batch under --scaling strong)."""
    from surreal_amd.config import PPO_DEFAULT_LEARNER_CONFIG, gym_env_config, pixel_env_config
    lc = copy.deepcopy(PPO_DEFAULT_LEARNER_CONFIG)
    if name == 'c2':
        lc.model.actor_fc_hidden_sizes = [64, 64]
        lc.model.critic_fc_hidden_sizes = [64, 64]
        lc.algo.use_z_filter = True
        lc.algo.n_step = 50
        lc.algo.gamma = 0.99
        lc.algo.advantage.lam = 0.95
        lc.algo.ppo_mode = 'adapt'
        lc.algo.rnn.if_rnn_policy = False
        lc.replay.batch_size = 64
        return lc, gym_env_config(17, 6), dict(D=17, A=6, rnn_hidden=None, B_global=64)
    # c3: the reference defaults (ppo_configs.py:15-94) + z-filter on
    lc.model.actor_fc_hidden_sizes = [300, 200]
    lc.model.critic_fc_hidden_sizes = [300, 200]
    lc.algo.use_z_filter = True
    lc.algo.n_step = 25
    lc.algo.ppo_mode = 'adapt'
    lc.algo.rnn.if_rnn_policy = True
    lc.algo.rnn.rnn_hidden = 100
    lc.algo.rnn.rnn_layer = 1
    lc.algo.rnn.horizon = 5
    lc.replay.batch_size = 1024
    if name == 'c5':
        lc.model.cnn_feature_dim = 256
        return lc, pixel_env_config(42, 8, (3, 84, 84)), dict(D=42, A=8, rnn_hidden=100,
                                                               pixel=(3, 84, 84), B_global=1024)
    return lc, gym_env_config(42, 8), dict(D=42, A=8, rnn_hidden=100, B_global=1024)


def spawn_ranks(n):
    """bench.py --gpus N without a launcher: run N ranks under
    torch.distributed.run as a CHILD process (this parent has made no GPU call:
    torch is imported, nothing initialised) and exit with its code."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(('127.0.0.1', 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


# kernel class (smi_kernel_timing) -> kernel-name patterns of its launches
CLASS_KERNELS = {
    'gemm_dw': ('gemm_dwd_kernel', 'gemm_dwd_group_kernel', 'gemm_dw128_kernel', 'gemm_kernel<2,'),
    'gemm_fwd': ('gemm_panel_kernel<0,', 'gemm_kernel<0,', 'gemm_smallk_fwd_kernel'),
    'gemm_dx': ('gemm_panel_kernel<1,', 'gemm_kernel<1,', 'dx_smallk_kernel'),
    'lstm_fwd': ('lstm_fwd',), 'lstm_bwd': ('lstm_bwd',),
    'cnn_fwd': ('cnn_fwd_kernel',), 'cnn_bwd': ('cnn_bwd_kernel',),
}
PMC_TRAFFIC = {'c3': 'profiles/r06/pmc_traffic_c3_r6.json',
               'c5': 'profiles/r02/pmc_traffic_c5_r2.json'}


def pmc_traffic(config, cls):
    """HBM bytes per launch of a kernel class from the committed PMC passes of
    this bench command (tools/pmc_bench.sh -> tools/pmc_traffic.py: FETCH_SIZE
    x2 + WRITE_SIZE, MI355X_MICROARCH.md 'HBM'), launch-weighted over the
    class's kernels; None when no such profile exists."""
    path = os.path.join(ROOT, PMC_TRAFFIC.get(config, ''))
    pats = CLASS_KERNELS.get(cls)
    if not pats or not os.path.isfile(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    n = b = 0
    for name, v in d.items():
        if any(p in name for p in pats) and v.get('launches'):
            n += v['launches']
            b += v['launches'] * v['hbm_bytes_per_launch']
    return (round(b / n) if n else None), os.path.relpath(path, ROOT)


MFMA_CLASSES = ('gemm_fwd', 'gemm_dx', 'gemm_dw', 'lstm_fwd', 'lstm_bwd', 'cnn_fwd', 'cnn_bwd')


def kernel_table(kt, n_inst):
    """per-class launches / time per step and achieved TFLOP/s (MFMA classes)
    or GB/s (HBM-bound classes, whose work unit is algorithmic bytes)"""
    from surreal_amd import _lib as L
    out = {}
    for n, (c, ms, w) in kt.items():
        row = {'launches_per_step': round(c / n_inst, 2), 'avg_ms': round(ms / c, 5),
               'ms_per_step': round(ms / n_inst, 4)}
        if n in L.KT_BYTES:
            gbs = w / (ms * 1e-3) / 1e9
            row.update({'GBps': round(gbs, 1), 'hbm_frac': round(gbs / HBM_PEAK_GBS, 4),
                        'bytes_per_launch': int(w / c)})
        elif n == 'gemm_splitk_reduce':
            row['note'] = 'split-K partial reducer (memory-bound; work counted = elements reduced)'
        else:
            row['tflops'] = round(w / (ms * 1e-3) / 1e12, 3)
        out[n] = row
    return out


def kernels_sum_note(kernels, ms):
    """Label of the per-class table: its classes come from an instrumented pass
    (eager launches, one library event pair per launch), so their sum is not the
    timed step; the table is for per-class shares and launch durations."""
    tot = sum(r['ms_per_step'] for r in kernels.values())
    return {'ms_per_step': round(tot, 4), 'ratio_to_timed_step': round(tot / ms, 4) if ms else None,
            'note': 'instrumented eager pass (per-launch events); sums of its classes are inflated '
                    'by the event records and exclude non-library launches; not the timed step'}


def mfma_dominant(kt):
    """the MFMA kernel class with the most time (roofline.kernel)"""
    cands = [n for n in kt if n in MFMA_CLASSES]
    return max(cands, key=lambda n: kt[n][1]) if cands else None


def roofline_hbm(kt, n_inst):
    """'% HBM roofline' of the streaming kernels inside the benched learn():
    algorithmic bytes per launch / measured launch time vs 8 TB/s.  At C3 these
    working sets are cache-resident (<= 10 MB), so the in-workload fraction is
    bounded by launch latency, not by HBM; tools/bench_hbm.py sweeps the same
    kernels over > 256 MB working sets."""
    from surreal_amd import _lib as L
    rows = {}
    for n, (c, ms, w) in kt.items():
        if n not in L.KT_BYTES:
            continue
        gbs = w / (ms * 1e-3) / 1e9
        rows[n] = {'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                   'frac': round(gbs / HBM_PEAK_GBS, 4), 'bytes_per_launch': int(w / c),
                   'avg_us': round(ms / c * 1e3, 2), 'launches_per_step': round(c / n_inst, 2)}
    if not rows:
        return None
    tot_b = sum(kt[n][2] for n in rows)
    tot_ms = sum(kt[n][1] for n in rows)
    agg = tot_b / (tot_ms * 1e-3) / 1e9
    # the largest per-launch working set against the 256 MB MALL: below it the
    # streams are (partly) cache-resident and the fraction is launch latency
    big = max(r['bytes_per_launch'] for r in rows.values())
    where = ('cache-resident at these batch sizes (largest launch %.1f MB <= 256 MB MALL)' % (big / 1e6)
             if big <= 256e6 else 'largest launch %.0f MB > 256 MB MALL: HBM-resident streams' % (big / 1e6))
    return {'kernels': rows, 'aggregate': {'achieved': round(agg, 1), 'unit': 'GB/s',
                                           'frac': round(agg / HBM_PEAK_GBS, 4),
                                           'ms_per_step': round(tot_ms / n_inst, 4)},
            'note': f'in-workload ({where}); > 256 MB sweeps: tools/bench_hbm.py, profiles/'}


def calibrate(dev, mfma_iters=20000, stream_mb=1024, reps=5):
    """Fixed-work calibration launches right before the timed region
    (calib_kernels.hip): what this box delivers today, so a slow box reads as a
    slow box and not as a code regression.  MFMA: 512 workgroups (2 per CU) x 4
    waves x iters x 4 v_mfma_f32_32x32x2_f32 on random register operands; HBM:
    a float4 read + write stream over 2 x stream_mb MB (> the 256 MB MALL).
    Best of `reps` launches each (HIP events on the current stream)."""
    from surreal_amd import _lib as L
    st = L.stream(dev)
    n_wg = 512
    out = torch.empty(n_wg * 256, device=dev)
    stamps = torch.zeros(2 * n_wg, dtype=torch.int64, device=dev)
    n = stream_mb * (1 << 20) // 4
    x = torch.rand(n, device=dev)
    y = torch.empty_like(x)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn):
        best = None
        fn()                                     # warm (code object, first touch)
        for _ in range(reps):
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        return best
    ms_m = timed(lambda: L.call('smi_calib_mfma', n_wg, mfma_iters, L.ptr(out), L.ptr(stamps), st))
    ms_s = timed(lambda: L.call('smi_calib_stream', L.ptr(x), L.ptr(y), n, st))
    s = stamps.view(n_wg, 2).cpu().numpy().astype(np.float64)
    clk = np.median(s[:, 0] / np.maximum(s[:, 1], 1)) * 100.0
    flops = n_wg * 4 * mfma_iters * 4 * 4096.0
    tf = flops / (ms_m * 1e-3) / 1e12
    tbps = 8.0 * n / (ms_s * 1e-3) / 1e12
    del x, y
    return {'calib_mfma_tflops': round(tf, 2), 'calib_mfma_frac': round(tf / FP32_MFMA_PEAK_TFLOPS, 4),
            'calib_mfma_clock_mhz': round(float(clk), 1),
            'calib_hbm_tbps': round(tbps, 3), 'calib_hbm_frac': round(tbps * 1e3 / HBM_PEAK_GBS, 4),
            'note': f'fixed-work launches right before the timed region (best of {reps}): '
                    f'{n_wg} x 4 waves x {mfma_iters} x 4 v_mfma_f32_32x32x2_f32 on random register '
                    f'operands; float4 read+write stream over 2 x {stream_mb} MB'}


class ClockProbe(object):
    """The shader clock over the timed region: one sleeping wave on a side
    stream stamps s_memtime / s_memrealtime from before the first timed launch
    until a stop kernel enqueued on the learner's stream after the last one
    (bounded by max_s of wall time, so it always exits)."""

    stop_in_region = True      # its stop kernel must precede the closing barrier

    def __init__(self, dev, max_s=30.0):
        from surreal_amd import _lib as L
        self.L, self.dev = L, dev
        self.flag = torch.zeros(4, dtype=torch.int32, device=dev)
        self.out = torch.zeros(3, dtype=torch.int64, device=dev)
        self.side = torch.cuda.Stream(device=dev)
        self.max_ticks = int(max_s * 1e8)
        torch.cuda.synchronize(dev)

    def start(self):
        L = self.L
        L.call('smi_clock_probe', L.ptr(self.flag), self.max_ticks, L.ptr(self.out),
               ctypes_stream(self.side))

    def stop(self):
        """enqueue the stop kernel on the learner's stream after the last timed
        launch, BEFORE the closing barrier (a device-wide synchronize waits for
        the probe's stream too)"""
        L = self.L
        L.call('smi_clock_probe_stop', L.ptr(self.flag), 1, L.stream(self.dev))

    def read(self):
        self.side.synchronize()
        m, r, to = (int(v) for v in self.out.cpu().tolist())
        if to or r <= 0:
            return None
        return {'clock_mhz': round(m / r * 100.0, 1), 'window_ms': round(r / 1e5, 3),
                'source': 'one sleeping wave on a side stream: d s_memtime / d s_memrealtime x '
                          '100 MHz from before the first timed step to a stop kernel enqueued '
                          'after the last (inside the timed region: one ~2 us launch)'}


class SmiClockSampler(object):
    """The GPU's current gfx clock over the timed region, sampled by a host
    thread from the SMU through amdsmi (gpu_metrics current_gfxclk, MHz) every
    `period_s`; reported as the mean and range of the samples.  No kernel runs
    beside the timed launches.  The period is 50 ms: each sample is a gpu_metrics
    read plus Python work under the GIL, and at 2 ms the thread slowed the C4
    step (host-side replay sampling every 0.25 ms)."""

    stop_in_region = False     # stopped after the closing barrier and the clock read

    def __init__(self, dev, period_s=0.05):
        import threading
        import amdsmi
        self.amdsmi = amdsmi
        amdsmi.amdsmi_init()
        hs = amdsmi.amdsmi_get_processor_handles()
        idx = torch.device(dev).index or 0
        vis = os.environ.get('HIP_VISIBLE_DEVICES') or os.environ.get('ROCR_VISIBLE_DEVICES')
        if vis:
            idx = int(vis.split(',')[idx])
        self.h = hs[idx] if idx < len(hs) else hs[0]
        self.period = period_s
        self.samples = []
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._run, daemon=True)
        self.read_one()                                  # fail here, not in the thread

    def read_one(self):
        m = self.amdsmi.amdsmi_get_gpu_metrics_info(self.h)
        v = m.get('current_gfxclk')
        if isinstance(v, (list, tuple)):
            v = [x for x in v if isinstance(x, (int, float)) and 0 < x < 10000]
            v = sum(v) / len(v) if v else None
        return v if isinstance(v, (int, float)) and 0 < v < 10000 else None

    def _run(self):
        while not self._stop.wait(self.period):
            self._sample()

    def _sample(self):
        v = self.read_one()
        if v is not None:
            self.samples.append(float(v))

    def start(self):
        self._th.start()                # (thread start-up before the timed region)
        self._sample()                  # at the start of the timed region

    def stop(self):
        # called after the closing barrier, with no sample: a gpu_metrics read
        # (or the thread's wake-up) between the last issue and the barrier is
        # host time inside the timed region (C4: 0.267 -> 0.31-0.37 ms per
        # step with a read there, profiles/r06/clock_ab)
        self._stop.set()

    def read(self):
        self._th.join(timeout=5)
        try:
            self.amdsmi.amdsmi_shut_down()
        except Exception:
            pass
        if not self.samples:
            return None
        return {'clock_mhz': round(float(np.mean(self.samples)), 1),
                'min_mhz': round(min(self.samples), 1), 'max_mhz': round(max(self.samples), 1),
                'samples': len(self.samples),
                'source': f'amdsmi gpu_metrics current_gfxclk at the start of the timed region and '
                          f'every {self.period * 1e3:.0f} ms through it (host thread; '
                          'SMU-reported, reads up to ~5 % below the in-kernel s_memtime clock of '
                          'calib.calib_mfma_clock_mhz); an in-kernel probe wave beside the timed '
                          'launches cost 15 % of the C3 step (profiles/r06/clock_ab), so none runs'}


def make_clock(mode, dev):
    """--clock probe | smi | none"""
    if mode == 'probe':
        return ClockProbe(dev)
    if mode == 'smi':
        try:
            return SmiClockSampler(dev)
        except Exception as e:          # amdsmi not usable here: report, do not fail the bench
            print(f'clock sampler unavailable: {e!r}', file=sys.stderr)
    return None


def ctypes_stream(s):
    import ctypes
    return ctypes.c_void_p(s.cuda_stream)


def attach_calib(out, calib, clock):
    """clock_mhz (shader clock over the timed region) and the calibration
    rates next to the headline, which stays unnormalised"""
    if clock is not None:
        out['clock_mhz'] = clock['clock_mhz']
        out['clock'] = clock
    if calib is not None:
        out['calib_mfma_tflops'] = calib['calib_mfma_tflops']
        out['calib_hbm_tbps'] = calib['calib_hbm_tbps']
        out['calib'] = calib


def mlp_flops_per_row(d, h1, h2, o):
    fwd = 2 * (d * h1 + h1 * h2 + h2 * o)
    bwd = fwd + 2 * (h1 * h2 + h2 * o)        # dW of all layers + dX of layers 2, 3
    return fwd, bwd


def cpu_model():
    """The host CPU model (lscpu 'Model name', read from /proc/cpuinfo)."""
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return None


def host_threads():
    """Threads the CPU baseline uses: this process's CPU share (OMP_NUM_THREADS
    on the GPU box, where os.cpu_count() reports the whole machine)."""
    env = os.environ.get('OMP_NUM_THREADS')
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _time_oracle(ref, batches, budget_s, max_calls=200, warmup=3, min_calls=20):
    """BASELINE.md's protocol: `warmup` untimed calls, then the median of at
    least `min_calls` timed calls (more while `budget_s` lasts, at most
    `max_calls`)"""
    for i in range(warmup):
        ref.learn(batches[i % len(batches)])
    times = []
    t_end = time.perf_counter() + budget_s
    i = 0
    while (time.perf_counter() < t_end or len(times) < min_calls) and len(times) < max_calls:
        t0 = time.perf_counter()
        ref.learn(batches[i % len(batches)])
        times.append(time.perf_counter() - t0)
        i += 1
    return statistics.median(times), len(times)


def cpu_baseline(name, lc, dims, budget_s=12.0, one_thread_budget_s=6.0):
    """The oracle's PPOLearnerRef.learn() (torch CPU fp32) timed on this host:
    with all the process's threads on the full benched batch (C3: 1024
    segments; C2: 64; C5: a 16-segment slice — the fp32 pixel stem costs ~0.25
    s per segment on the CPU), plus a 1-thread figure on a 64-segment slice (8
    for C5).  Learner env-steps/s on the CPU is close to batch-size independent
    at these sizes; each sample is stated."""
    from oracle import ppo_ref as R
    from surreal_amd import synthetic
    from tests.helpers import oracle_batch
    D, A = dims['D'], dims['A']
    T = lc.algo.n_step

    def make(B):
        c = copy.deepcopy(lc)
        c.replay.batch_size = B
        ref = R.PPOLearnerRef(c, D, A, pixel=dims.get('pixel'))
        bs = [oracle_batch(synthetic.ppo_batch(B, T, D, A, seed=i, rnn_hidden=dims['rnn_hidden'],
                                                pixel=dims.get('pixel'))) for i in range(2)]
        return ref, bs
    threads = host_threads()
    # C5's fp32 pixel stem costs ~0.25 s per segment on 16 threads: its samples
    # are 4 / 1 segments so that 3 + 20 calls stay within a minute or two
    B_all = {'c5': 4}.get(name, dims['B_global'])
    torch.set_num_threads(threads)
    ref, bs = make(B_all)
    med, n = _time_oracle(ref, bs, budget_s)
    B_one = 1 if name == 'c5' else min(64, B_all)
    torch.set_num_threads(1)
    ref1, bs1 = make(B_one)
    med1, n1 = _time_oracle(ref1, bs1, one_thread_budget_s, max_calls=20)
    torch.set_num_threads(threads)
    return {'value': round(B_all * T / med, 1), 'unit': 'env-steps/s', 'cores': threads, 'kind': 'port',
            'cpu_model': cpu_model(), 'os_cpu_count': os.cpu_count(),
            'sample': f'oracle PPOLearnerRef.learn() (torch CPU fp32, {threads} threads) on a '
                      f'{B_all}-segment x {T}-step batch of the {name.upper()} workload, {n} timed '
                      f'calls after 3 warm-ups (>= 20 calls, ~{budget_s:.0f} s budget), median '
                      f'{med * 1e3:.1f} ms',
            'value_1thread': round(B_one * T / med1, 1),
            'sample_1thread': f'same learn() on 1 thread, {B_one}-segment slice, {n1} timed calls '
                              f'after 3 warm-ups, median {med1 * 1e3:.1f} ms'}


DDPG_METRIC = 'DDPG learner env-steps/sec (replay sample + n-step target + critic/actor update)'


def run_ddpg(args):
    """--config c4 (BASELINE configs[3]): DDPGLearner, batch 512,
    HalfCheetah dims (obs 17, act 6), actor 300x200, critic 400x300, n_step 3,
    fed by UniformReplay over a 333,333-row shard resident in HBM.  A step =
    one CPython-exact index draw (MT19937 kernel) + row gather + learn().
    With WORLD_SIZE > 1 (SURVEY §8(e) DDPG row): the 512-row batch is sharded.
    Every rank holds the same replicated ring and MT19937 state, draws the same
    512 global indices (the single learner's CPython-exact stream) and gathers
    its 512 / N rows; the gradients are averaged over the ranks (DDPGLearner
    dp=TorchDistAllReduce), which equals the single learner's update on the
    512 rows: strong scaling, value = 512 x steps / max-over-ranks time."""
    dist, world, rank, _ = init_dist()
    from surreal_amd import _lib as L
    from surreal_amd.config import DDPG_DEFAULT_LEARNER_CONFIG, gym_env_config
    from surreal_amd.ddpg import DDPGLearner
    from surreal_amd.learner import TorchDistAllReduce
    from surreal_amd.replay import UniformReplay
    dev = torch.device('cuda', torch.cuda.current_device())
    D, A, B, NREP = 17, 6, 512, 333333
    lc = copy.deepcopy(DDPG_DEFAULT_LEARNER_CONFIG)
    lc.replay.batch_size = B
    lc.replay.memory_size = NREP
    lc.replay.sampling_start_size = 1000
    ec = gym_env_config(D, A)
    if B % world:
        raise SystemExit(f'--config c4: batch {B} does not split over {world} ranks')
    rep = UniformReplay(lc, ec, seed=0, device=dev)       # replicated ring, one index stream
    rows = np.random.RandomState(0).randn(NREP, rep.width).astype(np.float32)
    rows[:, D:D + A] = np.tanh(rows[:, D:D + A])
    rows[:, 2 * D + A + 1] = (rows[:, 2 * D + A + 1] > 1.6).astype(np.float32)
    rep.insert_rows(rows)
    graph = os.environ.get('SMI_DDPG_GRAPH', '0') == '1' and dist is None  # measured neutral
    dp = TorchDistAllReduce() if dist is not None else None
    llc = copy.deepcopy(lc)
    llc.replay.batch_size = B // world                     # this rank's shard of the batch
    learner = DDPGLearner(llc, ec, seed=1, device=dev, use_graph=graph, dp=dp)
    buf = torch.empty(B // world, rep.width, device=dev)

    def step():
        _, got = rep.sample(B, out=buf, rank=rank, world=world)
        learner.learn(rep.split(got))

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    calib = None if args.no_calib else calibrate(dev)
    for _ in range(args.warmup):
        step()
    barrier()
    probe = None if args.no_calib else make_clock(args.clock, dev)
    if probe is not None:
        probe.start()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if probe is not None and probe.stop_in_region:
        probe.stop()
    barrier()
    elapsed = time.perf_counter() - t0
    if probe is not None and not probe.stop_in_region:
        probe.stop()
    clock = probe.read() if probe is not None else None
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # instrumented pass on an eager learner (graph replays carry no per-kernel
    # events): same launches, same shapes
    n_inst = min(args.steps, 5)
    learner_e = DDPGLearner(llc, ec, seed=1, device=dev, dp=dp) if graph else learner

    def step_e():
        _, got = rep.sample(B, out=buf, rank=rank, world=world)
        learner_e.learn(rep.split(got))

    step_e()
    torch.cuda.synchronize()
    L.kernel_timing(True)
    for _ in range(n_inst):
        step_e()
    torch.cuda.synchronize()
    L.kernel_timing(False)
    kt = L.kernel_timing_report()
    kernels = kernel_table(kt, n_inst)
    dom = mfma_dominant(kt)
    c, ms_k, fl = kt[dom]
    ach = fl / (ms_k * 1e-3) / 1e12
    out = {
        'metric': DDPG_METRIC, 'value': round(B * args.steps / elapsed, 1),
        'unit': 'env-steps/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 4), 'higher_is_better': True,
        'scaling': 'strong', 'vs_baseline': None, 'dtype': 'f32',
        'data': 'synthetic replay rows (seeded); random-init weights of the named architecture',
        'config': {'workload': 'C4: DDPG learner, batch 512 sampled CPython-exactly from a '
                               '333,333-row replay shard, obs 17, act 6, actor 300x200, critic '
                               '400x300, n_step 3, hard target update',
                   'batch': B, 'batch_per_rank': B // world, 'replay_rows': NREP,
                   'parallelism': f'dp{world}' if world > 1 else 'single',
                   'update': 'hipGraph replay' if graph else 'eager launches'},
        'roofline': {'kernel': dom, 'bound': 'mfma', 'achieved': round(ach, 3),
                     'peak': FP32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                     'frac': round(ach / FP32_MFMA_PEAK_TFLOPS, 4), 'traffic': None,
                     'avg_ms': round(ms_k / c, 5), 'algorithmic_flops_per_launch': int(fl / c)},
        'kernels': kernels,
        'kernels_sum': kernels_sum_note(kernels, elapsed / args.steps * 1e3),
    }
    attach_calib(out, calib, clock)
    if dist is not None:
        barrier()
        dist.destroy_process_group()
    if rank != 0:
        return
    if not args.no_cpu_baseline and world == 1:
        out['cpu_baseline'] = cpu_baseline_ddpg(lc, rows, D, A, B, args.cpu_budget)
    print(json.dumps(out), flush=True)


def cpu_baseline_ddpg(lc, rows, D, A, B, budget_s=12.0):
    """The oracle DDPGLearnerRef.optimize() (torch CPU fp32) fed by CPython
    random.randint index draws over the same replay rows, timed per step."""
    import random
    from oracle import ddpg_ref as R
    threads = host_threads()
    torch.set_num_threads(threads)
    ref = R.DDPGLearnerRef(lc, D, A)
    table = torch.from_numpy(rows)
    random.seed(0)

    def step():
        idx = [random.randint(0, len(rows) - 1) for _ in range(B)]
        r = table[idx]
        ref.optimize(r[:, :D], r[:, D:D + A], r[:, D + A:D + A + 1], r[:, D + A + 1:2 * D + A + 1],
                     r[:, 2 * D + A + 1:2 * D + A + 2])

    for _ in range(3):                                     # 3 warm-ups
        step()
    times = []
    t_end = time.perf_counter() + budget_s
    while (time.perf_counter() < t_end or len(times) < 20) and len(times) < 2000:
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {'value': round(B / med, 1), 'unit': 'env-steps/s', 'cores': threads, 'kind': 'port',
            'cpu_model': cpu_model(), 'os_cpu_count': os.cpu_count(),
            'sample': f'oracle DDPGLearnerRef.optimize() (torch CPU fp32, {threads} threads) + '
                      f'random.randint sampling, batch {B} of the C4 workload, {len(times)} timed '
                      f'steps after 3 warm-ups (>= 20, ~{budget_s:.0f} s), median {med * 1e3:.2f} ms'}


def init_dist():
    """One process per GPU (RANK/LOCAL_RANK/WORLD_SIZE from the launcher).
    Returns (dist or None, world, rank, device)."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    if world > 1:
        import torch.distributed as dist
        ndev = torch.cuda.device_count()
        local_rank = local_rank % max(ndev, 1)       # rehearsal: several ranks per GPU
        torch.cuda.set_device(local_rank)
        # 'nccl' = RCCL over xGMI; SMI_DIST_BACKEND=gloo rehearses the same
        # code path with several ranks on one GPU (RCCL refuses that)
        backend = os.environ.get('SMI_DIST_BACKEND', 'nccl')
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local_rank))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device('cuda', torch.cuda.current_device())
    return dist, world, rank, dev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', choices=['c2', 'c3', 'c4', 'c5'], default='c3')
    ap.add_argument('--ppo-mode', choices=['adapt', 'clip'], default=None,
                    help='override the workload\'s PPO surrogate (A/B only; C2-C5 are adapt)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-calib', action='store_true',
                    help='skip the fixed-work calibration launches and the clock measurement')
    ap.add_argument('--clock', choices=['smi', 'probe', 'none'], default='smi',
                    help='GPU clock over the timed region: amdsmi samples from a host thread '
                         '(smi), an in-kernel s_memtime probe wave on a side stream (probe; '
                         'A/B only), or none')
    ap.add_argument('--cpu-budget', type=float, default=12.0)
    ap.add_argument('--local-segments', type=int, default=None,
                    help='segments per rank (overrides --scaling): e.g. 128 runs on one GPU '
                         'the share one rank of an 8-GPU strong-scaling C3 job computes')
    ap.add_argument('--scaling', choices=['strong', 'weak'], default=None,
                    help='strong (default for c3/c5): the workload\'s global batch split over '
                         'the ranks; weak (c2, c4): the per-GPU batch fixed')
    ap.add_argument('--no-host-batch', action='store_true',
                    help='skip the host-fed line (numpy batches through the StagingArena)')
    ap.add_argument('--graph', choices=['on', 'off'], default='on',
                    help='learn() as a hipGraph replay of its device sequence '
                         '(PPOLearner(use_graph=True), bit-identical to eager); with ranks > 1 '
                         'over RCCL the all-reduces are captured too (gloo runs eager)')
    args = ap.parse_args()

    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        return spawn_ranks(args.gpus)
    if os.environ.get('SMI_BENCH_PROBE') == '1':     # launch-path test (tests/test_cpu_bench.py)
        print(json.dumps({'rank': int(os.environ.get('RANK', '0')),
                          'world': int(os.environ.get('WORLD_SIZE', '1')),
                          'local_rank': int(os.environ.get('LOCAL_RANK', '0'))}), flush=True)
        return 0
    if args.config == 'c4':
        return run_ddpg(args)
    dist, world, rank, dev = init_dist()
    from surreal_amd import _lib as L
    from surreal_amd import synthetic
    from surreal_amd.learner import PPOLearner, TorchDistAllReduce
    lc, ec, dims = make_config(args.config)
    if args.ppo_mode:               # A/B of the clip surrogate (the workloads are adapt)
        lc.algo.ppo_mode = args.ppo_mode
    scaling = args.scaling or ('weak' if args.config == 'c2' else 'strong')
    if scaling == 'strong':
        if dims['B_global'] % world:
            raise SystemExit(f'global batch {dims["B_global"]} does not split over {world} ranks')
        lc.replay.batch_size = dims['B_global'] // world
    if args.local_segments:
        lc.replay.batch_size = args.local_segments
        scaling = 'weak'
    B, T = lc.replay.batch_size, lc.algo.n_step
    D, A = dims['D'], dims['A']
    dp = TorchDistAllReduce() if dist is not None else None
    learner = PPOLearner(lc, ec, seed=1, device=dev, dp=dp, use_graph=args.graph == 'on')
    pool = [synthetic.to_device(synthetic.ppo_batch(B, T, D, A, seed=rank * 1000 + i,
                                                    rnn_hidden=dims['rnn_hidden'],
                                                    pixel=dims.get('pixel')), dev)
            for i in range(4)]

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    calib = None if args.no_calib else calibrate(dev)
    for i in range(args.warmup):
        learner.learn(pool[i % len(pool)])
    barrier()
    probe = None if args.no_calib else make_clock(args.clock, dev)
    if probe is not None:
        probe.start()
    # timed region: the learner exactly as a caller runs it (no instrumentation)
    t0 = time.perf_counter()
    for k in range(args.steps):
        learner.learn(pool[k % len(pool)])
    if probe is not None and probe.stop_in_region:
        probe.stop()
    barrier()
    elapsed = time.perf_counter() - t0
    if probe is not None and not probe.stop_in_region:
        probe.stop()
    clock = probe.read() if probe is not None else None
    if dist is not None:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    epochs_run = learner.last_stats()['epochs_run']
    host_fed = None
    if not args.no_host_batch:
        # the same learns fed as the reference's learn() is fed: numpy batches
        # (the aggregator's output) staged by the learner itself -- one pinned
        # buffer, one H2D per batch (StagingArena, ppo.py:420-484) -- timed like
        # the headline; reported beside it, never as `value`
        hpool = [synthetic.ppo_batch(B, T, D, A, seed=rank * 1000 + i, rnn_hidden=dims['rnn_hidden'],
                                     pixel=dims.get('pixel')) for i in range(4)]
        for i in range(2):
            learner.learn(hpool[i % len(hpool)])
        barrier()
        t0 = time.perf_counter()
        for k in range(args.steps):
            learner.learn(hpool[k % len(hpool)])
        barrier()
        he = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([he], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            he = float(t.item())
        host_fed = {'value': round(world * B * T * args.steps / he, 1), 'unit': 'env-steps/s',
                    'ms_per_step': round(he / args.steps * 1e3, 4),
                    'note': 'numpy batches -> StagingArena (every array packed into one pinned '
                            'buffer, one async H2D) -> learn(): PCIe-inclusive, not the headline'}
    # instrumented pass (separate, after the timed region): per-launch HIP
    # events of the MFMA kernels recorded by the library on the learner's
    # stream, and per-phase torch events -> roofline / kernels / phases
    n_inst = min(args.steps, 5)
    learner.kernel_events = {}
    if dp is not None:
        dp.timing = []
    L.kernel_timing(True)
    for k in range(n_inst):
        learner.learn(pool[k % len(pool)])
    barrier()
    L.kernel_timing(False)
    ev = learner.kernel_events
    learner.kernel_events = None
    allreduce = None
    if dp is not None:
        # per-rank time inside the stream-ordered all-reduces (max over ranks)
        ar_ms = sum(s_.elapsed_time(e_) for s_, e_, _ in dp.timing) / n_inst
        ar_n = len(dp.timing) / n_inst
        ar_b = sum(b_ for _, _, b_ in dp.timing) / n_inst
        dp.timing = None
        t = torch.tensor([ar_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        allreduce = {'ms_per_step_max_over_ranks': round(float(t.item()), 4),
                     'calls_per_step': ar_n, 'bytes_per_step': int(ar_b),
                     'backend': dist.get_backend()}

    # per-kernel (MFMA engine) classes from the library's own events, and the
    # learner-level launches/phases from torch events on the same stream
    kt = L.kernel_timing_report()
    kernels = kernel_table(kt, n_inst)
    # phases from a pass of their own (eager launches, no per-kernel events: the
    # library's events inside the phases inflated them ~20 % over the wall time)
    learner.kernel_events = {}
    for k in range(n_inst):
        learner.learn(pool[k % len(pool)])
    barrier()
    ev = learner.kernel_events
    learner.kernel_events = None
    phases = {n: round(float(np.sum([s.elapsed_time(e) for s, e in v])) / n_inst, 4)
              for n, v in ev.items()}
    rhbm = roofline_hbm(kt, n_inst)
    if mfma_dominant(kt):
        dom = mfma_dominant(kt)
        c, ms, fl = kt[dom]
        ach = fl / (ms * 1e-3) / 1e12
        traffic, tsrc = pmc_traffic(args.config, dom)
        roof = {'kernel': dom, 'bound': 'mfma', 'achieved': round(ach, 3),
                'peak': FP32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s', 'frac': round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
                'traffic': traffic, 'avg_ms': round(ms / c, 5),
                'algorithmic_flops_per_launch': int(fl / c)}
        if traffic is not None:
            roof['traffic_unit'] = 'HBM bytes per launch'
            roof['traffic_source'] = tsrc + ' (PMC passes of this command, launch-weighted over the class)'
    else:
        # C2: the fused single-CU epoch kernel dominates
        kdur = {n: float(np.mean([s.elapsed_time(e) for s, e in v])) for n, v in ev.items()}
        dom = max(kdur, key=kdur.get)
        a_h1, a_h2 = lc.model.actor_fc_hidden_sizes
        c_h1, c_h2 = lc.model.critic_fc_hidden_sizes
        af, ab = mlp_flops_per_row(D, a_h1, a_h2, A)
        cf, cb = mlp_flops_per_row(D, c_h1, c_h2, 1)
        E_v = lc.algo.consts.epoch_baseline
        flops = {
            'ppo_fused_kernel': B * (af * (epochs_run + 2) + ab * epochs_run) + B * E_v * (cf + cb),
            'critic_gae_kernel': B * (T + 1) * cf,
            'ppo_epoch_grad_kernel': B * (af + ab + cf + cb),
        }
        fl = flops.get(dom, 0)
        ach = fl / (kdur[dom] * 1e-3) / 1e12
        roof = {'kernel': dom, 'bound': 'mfma', 'achieved': round(ach, 6), 'peak': FP32_MFMA_PEAK_TFLOPS,
                'unit': 'TFLOP/s', 'frac': round(ach / FP32_MFMA_PEAK_TFLOPS, 8), 'traffic': None,
                'avg_ms': round(kdur[dom], 5), 'algorithmic_flops_per_launch': int(fl)}
    ms = elapsed / args.steps * 1e3
    value = world * B * T * args.steps / elapsed
    split = (f'{dims["B_global"]} segments split over {world} GPU(s) ({B} per GPU)'
             if scaling == 'strong' else f'{B} segments per GPU')
    if args.config == 'c5':
        wl = ('C5: C3 (LSTM 100, horizon 5, heads 300x200, n_step 25, adapt, z-filter, 10/10 '
              'epochs, obs 42, act 8) + pixel stem: camera0 3x84x84 uint8 -> conv 16@8s4 -> '
              '32@4s2 -> FC 256; ' + split)
    elif args.config == 'c3':
        wl = ('C3: synthetic PPO learner batch, reference PPO defaults (LSTM 100, horizon 5, heads '
              '300x200, n_step 25, adapt, z-filter, 10/10 epochs), SawyerLift state dims (obs 42, '
              'act 8), ' + split)
    else:
        wl = ('C2: synthetic PPO learner batch, HalfCheetah dims (obs 17, act 6), 64x64 MLP, '
              '64 segments x n_step 50 per GPU, adapt mode, z-filter, 10/10 epochs')
    out = {
        'metric': METRIC, 'value': round(value, 1), 'unit': 'env-steps/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms, 4),
        'higher_is_better': True, 'scaling': scaling, 'vs_baseline': None, 'dtype': 'f32',
        'data': 'synthetic (seeded, SURVEY §8(d)); random-init weights of the named architecture',
        'config': {'workload': wl, 'segments_per_gpu': B, 'n_step': T,
                   'env_steps_per_learn_per_gpu': B * T, 'global_segments': world * B,
                   'parallelism': f'dp{world}' if world > 1 else 'single',
                   'epochs_run_last': epochs_run, 'ppo_mode': lc.algo.ppo_mode,
                   'launch': 'hipGraph replay' if learner._graph is not None else 'eager'},
        'roofline': roof,
        'kernels': kernels,
        'kernels_sum': kernels_sum_note(kernels, ms),
        'phase_ms_per_step': phases,
    }
    attach_calib(out, calib, clock)
    if rhbm is not None:
        out['roofline_hbm'] = rhbm
    if allreduce is not None:
        out['allreduce'] = allreduce
    if host_fed is not None:
        out['host_fed'] = host_fed
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(args.config, make_config(args.config)[0], dims,
                                           args.cpu_budget)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    sys.exit(main() or 0)
