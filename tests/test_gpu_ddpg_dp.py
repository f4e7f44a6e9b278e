"""Data-parallel DDPG as SURVEY §8(e) specifies it: the B = 512 batch sharded
across ranks from ONE CPython-exact MT19937 stream (uniform_replay.py:43-47),
gradients averaged (dp=TorchDistAllReduce).

Two processes share cuda:0 and exchange over torch.distributed (gloo: RCCL
refuses two ranks on one GPU; a multi-GPU node runs the same code over
'nccl' = RCCL/xGMI, as bench.py --config c4 does).  Every rank holds the same
replicated replay ring and the same MT19937 seed, draws the same 512 global
indices per step on the device and gathers its 256-row slice
(UniformReplay.sample(rank=, world=)).  Required:
  * the concatenated per-rank indices of every step equal
    `random.seed(s); [random.randint(0, n - 1) for _ in range(512)]` of ONE
    learner (bit-exact sampling);
  * the ranks end bit-identical (parameters, targets, statistics);
  * rank 0's parameters and statistics lie within the fp32 envelope of the
    fp64 oracle's single-learner step on the 512 sampled rows
    (tests/test_gpu_ddpg.py ddpg_envelope_check), including the TD3 smoothing
    noise, which every rank draws for the global batch and slices."""
import os
import random
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests.test_gpu_dp_procs import _free_port

pytestmark = pytest.mark.gpu

B, D, A, NREP, SEED, STEPS = 512, 17, 6, 5000, 7, 3


def _cfg(target, td3, clip=False, batch=B):
    from tests.test_gpu_ddpg import _cfg as base
    lc = base(batch, target, clip)
    lc.replay.memory_size = NREP
    if clip:                       # small enough that clip_grad_value_ acts on the averaged gradient
        lc.algo.network.critic_gradient_value_clip = 0.02
        lc.algo.network.actor_gradient_value_clip = 0.005
    if td3:
        lc.algo.network.use_double_critic = True
        lc.algo.network.use_action_regularization = True
    return lc


def _rows():
    """the replicated replay contents (every rank inserts the same rows)"""
    w = 2 * D + A + 2
    rows = np.random.RandomState(5).randn(NREP, w).astype(np.float32)
    rows[:, D:D + A] = np.tanh(rows[:, D:D + A])
    rows[:, 2 * D + A + 1] = (rows[:, 2 * D + A + 1] > 1.0).astype(np.float32)
    return rows


def _split(rows):
    return {'obs': rows[:, :D], 'actions': rows[:, D:D + A], 'rewards': rows[:, D + A:D + A + 1],
            'obs_next': rows[:, D + A + 1:2 * D + A + 1], 'dones': rows[:, 2 * D + A + 1:]}


def _worker(rank, world, port, target, td3, clip, outdir):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from surreal_amd.config import gym_env_config
    from surreal_amd.ddpg import DDPGLearner
    from surreal_amd.learner import TorchDistAllReduce
    from surreal_amd.replay import UniformReplay
    from tests.test_gpu_ddpg import _ddpg_state
    ec = gym_env_config(D, A)
    rep = UniformReplay(_cfg(target, td3, clip), ec, seed=SEED, device='cuda:0')
    rep.insert_rows(_rows())
    learner = DDPGLearner(_cfg(target, td3, clip, batch=B // world), ec, seed=2, device='cuda:0',
                          dp=TorchDistAllReduce())
    init = {k: v for k, v in _ddpg_state(learner).items() if k in ('actor', 'critic', 'critic2')}
    res = []
    for it in range(STEPS):
        idx, rows = rep.sample(B, rank=rank, world=world)
        np.random.seed(100 + it)
        learner.learn(rep.split(rows))
        res.append({'idx': idx.cpu(), 'state': _ddpg_state(learner), 'stats': learner.last_stats()})
    torch.save({'init': init, 'res': res}, os.path.join(outdir, f'rank{rank}.pt'))
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize('target,td3,clip', [('hard', False, False), ('soft', True, False),
                                             ('hard', False, True), ('soft', True, True)])
def test_two_process_ddpg_dp_matches_single_learner(target, td3, clip):
    from tests.test_gpu_ddpg import ddpg_envelope_check
    world = 2
    with tempfile.TemporaryDirectory() as outdir:
        mp.spawn(_worker, args=(world, _free_port(), target, td3, clip, outdir), nprocs=world, join=True)
        out = [torch.load(os.path.join(outdir, f'rank{r}.pt'), weights_only=True) for r in range(world)]
    # one learner's index stream (uniform_replay.py:43-47)
    random.seed(SEED)
    rows = _rows()
    batches = []
    for it in range(STEPS):
        want = [random.randint(0, NREP - 1) for _ in range(B)]
        got = torch.cat([out[r]['res'][it]['idx'] for r in range(world)]).tolist()
        assert got == want, f'step {it}: the sharded draw differs from random.randint'
        batches.append(_split(rows[np.asarray(want)]))
        r0, r1 = out[0]['res'][it], out[1]['res'][it]
        for k in r0['state']:
            assert torch.equal(r0['state'][k], r1['state'][k]), (it, k)
        assert r0['stats'] == r1['stats']
    gpu = [(out[0]['res'][it]['state'], out[0]['res'][it]['stats']) for it in range(STEPS)]
    ddpg_envelope_check(_cfg(target, td3, clip), D, A, out[0]['init'], batches, gpu, tag='_dp2')
