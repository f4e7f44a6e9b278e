"""World-size-2 gloo test (CPU) of the MATH of the DDPG data-parallel
decomposition that DDPGLearner(dp=...) implements (SURVEY §8(e) DDPG row).  It
runs a torch restatement of the rank-local step, not the product's HIP learner
(no GPU here); tests/test_gpu_ddpg_dp.py runs DDPGLearner(dp=...) itself,
with and without gradient clipping.  Each rank holds half
of the batch, computes the reference's mean-loss gradients on it, averages
them over the ranks (through the product's TorchDistAllReduce) before
clip_grad_value + Adam, and draws the TD3 smoothing noise for the global batch
from numpy's global RNG, keeping its own rows.  After each step both ranks
must hold identical parameters equal to the single-process oracle on the
concatenated batch (fp32 reassociation + Adam sign-flip budget)."""
import copy
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from oracle import ddpg_ref as R
from tests.test_cpu_dist import _free_port

B_LOC, D, A, STEPS = 64, 17, 6, 3


def _cfg(B, td3):
    from surreal_amd.config import DDPG_DEFAULT_LEARNER_CONFIG
    lc = copy.deepcopy(DDPG_DEFAULT_LEARNER_CONFIG)
    lc.replay.batch_size = B
    lc.algo.network.target_update = {'type': 'soft', 'tau': 1e-3}
    lc.algo.network.clip_critic_gradient = True
    if td3:
        lc.algo.network.use_double_critic = True
        lc.algo.network.use_action_regularization = True
    return lc


def _batch(it):
    g = torch.Generator().manual_seed(it)
    return {'obs': torch.randn(B_LOC * 2, D, generator=g),
            'actions': torch.rand(B_LOC * 2, A, generator=g) * 2 - 1,
            'rewards': torch.randn(B_LOC * 2, 1, generator=g),
            'obs_next': torch.randn(B_LOC * 2, D, generator=g),
            'dones': (torch.rand(B_LOC * 2, 1, generator=g) < 0.1).float()}


def _step(ref, group, b, W, r):
    """DDPGLearnerRef.optimize with the DP reductions of DDPGLearner(dp=...)."""
    def mean_grads(module):
        for p in module.parameters():
            group.allreduce_(p.grad)
            p.grad.mul_(1.0 / W)

    obs, actions, rewards, obs_next, done = (b[k] for k in ('obs', 'actions', 'rewards',
                                                             'obs_next', 'dones'))
    with torch.no_grad():
        a_t = ref.actor_t(obs_next)
        q_t = ref.critic_t(obs_next, a_t)
        if ref.action_reg:
            noise = np.clip(np.random.normal(0, 0.2, size=(ref.batch_size * W, ref.act_dim)),
                            -0.5, 0.5)[r * ref.batch_size:(r + 1) * ref.batch_size]
            a_t = (a_t + torch.tensor(noise, dtype=torch.float32)).clamp(-1, 1)
        y = rewards + pow(ref.gamma, ref.n_step) * q_t * (1.0 - done)
        if ref.double:
            y = torch.min(y, rewards + pow(ref.gamma, ref.n_step) *
                          ref.critic2_t(obs_next, a_t) * (1.0 - done))
    crits = [(ref.critic, ref.critic_optim)] + ([(ref.critic2, ref.critic_optim2)] if ref.double else [])
    for crit, opt in crits:
        crit.zero_grad()
        nn.MSELoss()(crit(obs, actions), y).backward()
        mean_grads(crit)
        if ref.clip_critic:
            nn.utils.clip_grad_value_(crit.parameters(), ref.critic_clip_value)
        opt.step()
    ref.actor.zero_grad()
    (-ref.critic(obs, ref.actor(obs)).mean()).backward()
    mean_grads(ref.actor)
    if ref.clip_actor:
        nn.utils.clip_grad_value_(ref.actor.parameters(), ref.actor_clip_value)
    ref.actor_optim.step()
    ref.target_update()


def _worker(rank, world, port, td3, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from surreal_amd.learner import TorchDistAllReduce
    group = TorchDistAllReduce()
    ref = R.DDPGLearnerRef(_cfg(B_LOC, td3), D, A, seed=5)
    res = []
    for it in range(STEPS):
        b = {k: v[rank * B_LOC:(rank + 1) * B_LOC] for k, v in _batch(it).items()}
        np.random.seed(100 + it)
        _step(ref, group, b, world, rank)
        res.append([R.flat_of(ref.actor.params()), R.flat_of(ref.critic.params()),
                    R.flat_of(ref.critic_t.params())])
    out[rank] = res
    dist.destroy_process_group()


def _close(got, want, lr, steps):
    d = (got - want).abs()
    scale = float(want.abs().max())
    flips = d > 1e-5 * scale
    assert float(d.max()) <= 2 * lr * steps + 1e-5 * scale, float(d.max())
    assert flips.float().mean().item() < 1e-2


@pytest.mark.parametrize('td3', [False, True])
def test_gloo_world2_ddpg_dp_equals_global_batch(td3):
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), td3, out), nprocs=world, join=True)
        res = [out[r] for r in range(world)]
    lc = _cfg(B_LOC * world, td3)
    ref = R.DDPGLearnerRef(lc, D, A, seed=5)
    net = lc.algo.network
    for it in range(STEPS):
        np.random.seed(100 + it)
        b = _batch(it)
        ref.optimize(b['obs'], b['actions'], b['rewards'], b['obs_next'], b['dones'])
        for k in range(3):
            assert torch.equal(res[0][it][k], res[1][it][k]), (it, k)
        _close(res[0][it][0], R.flat_of(ref.actor.params()), net.lr_actor, it + 1)
        _close(res[0][it][1], R.flat_of(ref.critic.params()), net.lr_critic, it + 1)
        _close(res[0][it][2], R.flat_of(ref.critic_t.params()), net.lr_critic, it + 1)
