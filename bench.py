"""Learner throughput benchmark (driver contract: see README/DESIGN.md §Measurement).

A step = one PPOLearner.learn() over one synthetic batch already resident in
HBM: reward scaling, critic forward over B*(T+1) rows + windowed GAE, the fused
policy/value epoch loop (ref_pol, <=10 actor updates with KL early stop, 10
critic updates), z_update.  Workload at N=1 = BASELINE config 2 (HalfCheetah
dims obs 17 / act 6, 64x64 MLP, 64 segments x 50 steps).  With --gpus N the
learner is data parallel: each rank holds a 64-segment shard of
one global N*64-segment batch and the ranks all-reduce advantage moments, the
per-epoch gradient/statistic exchange buffer and the ZFilter column sums over
RCCL (torch.distributed 'nccl') — weak scaling, every rank applies the update
of the global batch.

Prints ONE JSON line on rank 0 with the metric, a roofline object for the
dominant kernel (HIP events on the learner's stream, inside the timed region)
and the CPU baseline (the oracle restatement timed on this host).
"""
import argparse
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


def c2_config():
    from surreal_amd.config import PPO_DEFAULT_LEARNER_CONFIG, gym_env_config
    import copy
    lc = copy.deepcopy(PPO_DEFAULT_LEARNER_CONFIG)
    lc.model.actor_fc_hidden_sizes = [64, 64]
    lc.model.critic_fc_hidden_sizes = [64, 64]
    lc.algo.use_z_filter = True
    lc.algo.n_step = 50
    lc.algo.gamma = 0.99
    lc.algo.advantage.lam = 0.95
    lc.algo.ppo_mode = 'adapt'
    lc.algo.rnn.if_rnn_policy = False
    lc.replay.batch_size = 64
    return lc, gym_env_config(17, 6)


def mlp_flops_per_row(d, h1, h2, o):
    fwd = 2 * (d * h1 + h1 * h2 + h2 * o)
    bwd = fwd + 2 * (h1 * h2 + h2 * o)        # dW of all layers + dX of layers 2, 3
    return fwd, bwd


def cpu_baseline(lc, ec, budget_s=12.0):
    from oracle import ppo_ref as R
    from surreal_amd import synthetic
    from tests.helpers import oracle_batch
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    B, T = lc.replay.batch_size, lc.algo.n_step
    D, A = ec.obs_spec['low_dim']['flat_inputs'][0], ec.action_spec['dim'][0]
    ref = R.PPOLearnerRef(lc, D, A)
    batches = [oracle_batch(synthetic.ppo_batch(B, T, D, A, seed=i)) for i in range(4)]
    for i in range(2):
        ref.learn(batches[i % 4])
    times = []
    t_end = time.perf_counter() + budget_s
    i = 0
    while time.perf_counter() < t_end or len(times) < 5:
        t0 = time.perf_counter()
        ref.learn(batches[i % 4])
        times.append(time.perf_counter() - t0)
        i += 1
    med = statistics.median(times)
    return {'value': B * T / med, 'unit': 'env-steps/s', 'cores': threads, 'kind': 'port',
            'sample': f'oracle PPOLearnerRef.learn() on the C2 batch, {len(times)} calls '
                      f'(~{budget_s:.0f} s), median {med * 1e3:.2f} ms, torch CPU fp32, '
                      f'{threads} threads'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-budget', type=float, default=12.0)
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local_rank))
    else:
        torch.cuda.set_device(0)
    dev = torch.device('cuda', torch.cuda.current_device())

    from surreal_amd import synthetic
    from surreal_amd.learner import PPOLearner, TorchDistAllReduce
    lc, ec = c2_config()
    B, T = lc.replay.batch_size, lc.algo.n_step
    D, A = 17, 6
    dp = TorchDistAllReduce() if dist is not None else None
    learner = PPOLearner(lc, ec, seed=1, device=dev, dp=dp)
    pool = [synthetic.to_device(synthetic.ppo_batch(B, T, D, A, seed=rank * 1000 + i), dev)
            for i in range(8)]

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    for i in range(args.warmup):
        learner.learn(pool[i % len(pool)])
    barrier()
    learner.kernel_events = {}
    epochs = []
    t0 = time.perf_counter()
    for k in range(args.steps):
        learner.learn(pool[k % len(pool)])
    barrier()
    elapsed = time.perf_counter() - t0
    ev = learner.kernel_events
    learner.kernel_events = None
    if dist is not None:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    epochs_run = learner.last_stats()['epochs_run']

    # per-kernel average durations (ms) from the live events
    kdur = {n: float(np.mean([s.elapsed_time(e) for s, e in v])) for n, v in ev.items()}
    dominant = max(kdur, key=kdur.get)
    a_h1, a_h2 = lc.model.actor_fc_hidden_sizes
    c_h1, c_h2 = lc.model.critic_fc_hidden_sizes
    af, ab = mlp_flops_per_row(D, a_h1, a_h2, A)
    cf, cb = mlp_flops_per_row(D, c_h1, c_h2, 1)
    E_v = lc.algo.consts.epoch_baseline
    flops = {
        # ref fwd + (epochs_run + 1) fwd + epochs_run bwd (policy)  +  E_v (fwd + bwd) (value)
        'ppo_fused_kernel': B * (af * (epochs_run + 2) + ab * epochs_run) + B * E_v * (cf + cb),
        'critic_gae_kernel': B * (T + 1) * cf,
        # data parallel: one grad launch per phase (policy fwd/bwd and/or value fwd/bwd)
        'ppo_epoch_grad_kernel': B * (af + ab + cf + cb),
    }
    if dominant in flops:
        ach = flops[dominant] / (kdur[dominant] * 1e-3) / 1e12
        roof = {'kernel': dominant, 'bound': 'mfma', 'achieved': round(ach, 6),
                'peak': FP32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                'frac': round(ach / FP32_MFMA_PEAK_TFLOPS, 8), 'traffic': None,
                'avg_ms': round(kdur[dominant], 5),
                'algorithmic_flops_per_launch': int(flops[dominant])}
    else:
        byt = B * D * 4 * 2
        ach = byt / (kdur[dominant] * 1e-3) / 1e9
        roof = {'kernel': dominant, 'bound': 'hbm', 'achieved': round(ach, 3), 'peak': HBM_PEAK_GBS,
                'unit': 'GB/s', 'frac': round(ach / HBM_PEAK_GBS, 8), 'traffic': None,
                'avg_ms': round(kdur[dominant], 5)}
    ms = elapsed / args.steps * 1e3
    value = world * B * T * args.steps / elapsed
    out = {
        'metric': METRIC, 'value': round(value, 1), 'unit': 'env-steps/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms, 4),
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32',
        'data': 'synthetic (seeded, SURVEY §8(d)); random-init 64x64 actor/critic',
        'config': {'workload': 'C2: synthetic PPO learner batch, HalfCheetah dims (obs 17, act 6), '
                               '64x64 MLP, 64 segments x n_step 50 per GPU, adapt mode, z-filter, '
                               '10/10 epochs', 'segments_per_gpu': B, 'n_step': T,
                   'env_steps_per_learn_per_gpu': B * T, 'global_segments': world * B, 'parallelism': f'dp{world}' if world > 1 else 'single',
                   'epochs_run_last': epochs_run},
        'roofline': roof,
        'kernels_avg_ms': {k: round(v, 5) for k, v in kdur.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(lc, ec, args.cpu_budget)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
