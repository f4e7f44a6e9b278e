"""Data-parallel DDPGLearner.learn() (dp=TorchDistAllReduce, SURVEY §8(e) DDPG
row) in two processes that share cuda:0 and exchange over torch.distributed
(gloo: RCCL refuses two ranks on one GPU; a multi-GPU node runs the same code
over 'nccl' = RCCL/xGMI).  Each rank learns on its half of the batch; both
ranks must end with bit-identical parameters equal to the CPU oracle's
optimize() on the concatenated batch (tolerances as in test_gpu_ddpg.py),
including the TD3 smoothing noise, which every rank draws for the global batch
from numpy's global RNG and slices to its own rows."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests.test_gpu_dp_procs import _free_port

pytestmark = pytest.mark.gpu

B_LOC, D, A = 256, 17, 6


def _cfg(target, td3, clip=False):
    from tests.test_gpu_ddpg import _cfg as base
    lc = base(B_LOC, target, clip)
    if clip:                       # small enough that clip_grad_value_ acts on the averaged gradient
        lc.algo.network.critic_gradient_value_clip = 0.02
        lc.algo.network.actor_gradient_value_clip = 0.005
    if td3:
        lc.algo.network.use_double_critic = True
        lc.algo.network.use_action_regularization = True
    return lc


def _worker(rank, world, port, target, td3, clip, outdir):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from surreal_amd import synthetic
    from surreal_amd.config import gym_env_config
    from surreal_amd.ddpg import DDPGLearner
    from surreal_amd.learner import TorchDistAllReduce
    learner = DDPGLearner(_cfg(target, td3, clip), gym_env_config(D, A), seed=2, device='cuda:0',
                          dp=TorchDistAllReduce())
    init = {'actor': learner.model.actor.flat.cpu(), 'critic': learner.model.critic.flat.cpu()}
    if td3:
        init['critic2'] = learner.model2.critic.flat.cpu()
    res = []
    for it in range(3):
        b = synthetic.ddpg_batch(B_LOC * world, D, A, seed=it)
        lo, hi = rank * B_LOC, (rank + 1) * B_LOC
        np.random.seed(100 + it)
        learner.learn({k: v[lo:hi].contiguous().cuda() for k, v in b.items()})
        r = {'actor': learner.model.actor.flat.cpu(), 'critic': learner.model.critic.flat.cpu(),
             'tcritic': learner.model_target.critic.flat.cpu(), 'stats': learner.last_stats()}
        if td3:
            r['critic2'] = learner.model2.critic.flat.cpu()
        res.append(r)
    torch.save({'init': init, 'res': res}, os.path.join(outdir, f'rank{rank}.pt'))
    dist.destroy_process_group()


@pytest.mark.parametrize('target,td3,clip', [('hard', False, False), ('soft', True, False),
                                             ('hard', False, True), ('soft', True, True)])
def test_two_process_ddpg_dp_matches_oracle(target, td3, clip):
    from oracle import ddpg_ref as R
    from surreal_amd import synthetic
    from tests.test_gpu_ppo import _compare_params
    world = 2
    with tempfile.TemporaryDirectory() as outdir:
        mp.spawn(_worker, args=(world, _free_port(), target, td3, clip, outdir), nprocs=world, join=True)
        out = [torch.load(os.path.join(outdir, f'rank{r}.pt'), weights_only=True) for r in range(world)]
    lc = _cfg(target, td3, clip)
    lc.replay.batch_size = B_LOC * world
    ref = R.DDPGLearnerRef(lc, D, A)
    R.load_flat(ref.actor.params(), out[0]['init']['actor'])
    R.load_flat(ref.critic.params(), out[0]['init']['critic'])
    if td3:
        R.load_flat(ref.critic2.params(), out[0]['init']['critic2'])
    ref.hard_update()
    report = {}
    for it in range(3):
        b = synthetic.ddpg_batch(B_LOC * world, D, A, seed=it)
        np.random.seed(100 + it)
        rs = ref.optimize(b['obs'], b['actions'], b['rewards'], b['obs_next'], b['dones'])
        r0, r1 = out[0]['res'][it], out[1]['res'][it]
        for k in ('actor', 'critic', 'tcritic') + (('critic2',) if td3 else ()):
            assert torch.equal(r0[k], r1[k]), (it, k)
        for k in rs:
            assert abs(r0['stats'][k] - rs[k]) <= 1e-4 * abs(rs[k]) + 1e-5, (it, k, r0['stats'][k], rs[k])
        _compare_params(f'critic{it}', r0['critic'], R.flat_of(ref.critic.params()), 1e-3, it + 1, report)
        _compare_params(f'actor{it}', r0['actor'], R.flat_of(ref.actor.params()), 1e-4, it + 1, report,
                        max_frac=1e-2 if td3 else 5e-3)
        _compare_params(f'tcritic{it}', r0['tcritic'], R.flat_of(ref.critic_t.params()), 1e-3, it + 1,
                        report)
        if td3:
            _compare_params(f'critic2_{it}', r0['critic2'], R.flat_of(ref.critic2.params()), 1e-3,
                            it + 1, report)
    print('ddpg dp report:', report)
