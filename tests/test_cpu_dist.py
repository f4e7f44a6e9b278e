"""World-size-2 gloo test (CPU) of the data-parallel decomposition the HIP
phase kernels implement: each rank holds its shard of the
segments, weights per-row gradients by 1/B_global, SUM-all-reduces gradients
(through the product's TorchDistAllReduce), the advantage moments, the KL used
for early stopping / the adapt penalty, and the ZFilter column sums.  The
result must equal the single-process oracle on the concatenated batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ppo_ref as R


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_learn(ref, group, obs, obs_next, actions, rewards, dones, pds, B_g):
    """PPOLearnerRef._optimize with the DP reductions (non-RNN)."""
    pd = ref.pd
    with torch.no_grad():
        x = torch.cat([obs, obs_next], 1).reshape(-1, obs.shape[-1])
        values = ref.model.forward_critic(x).view(obs.shape[0], ref.n_step + 1)
        adv_raw, ret = R.gae_and_return(values, rewards, dones, ref.gamma, ref.lam, ref.n_step,
                                        ref.horizon, False, False)
        adv_raw, ret = adv_raw.view(-1), ret.view(-1, 1)
        mom = torch.tensor([adv_raw.double().sum(), (adv_raw.double() ** 2).sum(),
                            float(adv_raw.numel())], dtype=torch.float64)
        group.allreduce_(mom)
        mean = mom[0] / mom[2]
        std = torch.sqrt((mom[1] - mom[2] * mean * mean) / (mom[2] - 1))
        adv = ((adv_raw - mean.float()) / max(float(std), 1e-4)).view(-1, 1)
    o0, a0, b0 = obs[:, 0, :], actions[:, 0, :], pds[:, 0, :]
    with torch.no_grad():
        ref_pol = ref.ref_target_model.forward_actor(o0)

    def global_kl(pol):
        k = pd.kl(ref_pol, pol).sum().reshape(1)
        group.allreduce_(k)
        return float(k) / B_g

    runs = 0
    with torch.no_grad():
        kl = global_kl(ref.model.forward_actor(o0))
    for e in range(ref.epoch_policy):
        pol = ref.model.forward_actor(o0)
        lp = pd.likelihood(a0, pol)
        bp = pd.likelihood(a0, b0)
        if ref.ppo_mode == 'clip':
            ratio = lp / bp
            c = torch.clamp(ratio, 1 - ref.clip_epsilon, 1 + ref.clip_epsilon)
            loss = torch.cat([-ratio * adv, -c * adv], 1).max(1)[0].sum() / B_g
        else:
            surr = -(adv * (lp / torch.clamp(bp, min=1e-2))).sum() / B_g
            coef = ref.beta + (2 * ref.eta * (kl - 2 * ref.kl_target) if kl - 2 * ref.kl_target > 0 else 0)
            loss = surr + coef * pd.kl(ref_pol, pol).sum() / B_g
        for p in ref.model.actor_params():
            p.grad = None
        loss.backward()
        for p in ref.model.actor_params():
            group.allreduce_(p.grad)
        torch.nn.utils.clip_grad_norm_(ref.model.actor_params(), ref.actor_clip)
        ref.actor_optim.step()
        runs += 1
        with torch.no_grad():
            kl = global_kl(ref.model.forward_actor(o0))
        if kl > ref.kl_target * 4:
            break
    for _ in range(ref.epoch_baseline):
        v = ref.model.forward_critic(o0)
        loss = (v - ret).pow(2).sum() / B_g
        for p in ref.model.critic_params():
            p.grad = None
        loss.backward()
        for p in ref.model.critic_params():
            group.allreduce_(p.grad)
        torch.nn.utils.clip_grad_norm_(ref.model.critic_params(), ref.critic_clip)
        ref.critic_optim.step()
    with torch.no_grad():
        zs = torch.stack([o0.sum(0), (o0 * o0).sum(0)])
        group.allreduce_(zs)
        ref.model.z_filter.running_sum += zs[0]
        ref.model.z_filter.running_sumsq += zs[1]
        ref.model.z_filter.count += float(B_g)
    return runs


def _worker(rank, world, port, mode, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from surreal_amd import synthetic
    from surreal_amd.learner import TorchDistAllReduce
    from tests.helpers import oracle_batch, ppo_config
    group = TorchDistAllReduce()
    B_loc, T, D, A = 16, 6, 5, 3
    lc = ppo_config(B=B_loc, T=T, mode=mode, use_z_filter=True, hidden=(16, 16))
    ref = R.PPOLearnerRef(lc, D, A, seed=3)
    b = oracle_batch(synthetic.ppo_batch(B_loc * world, T, D, A, seed=9))
    sl = slice(rank * B_loc, (rank + 1) * B_loc)
    runs = _dp_learn(ref, group, b['obs'][sl], b['obs_next'][sl], b['actions'][sl],
                     b['rewards'][sl], b['dones'][sl], b['pds'][sl], B_loc * world)
    out[rank] = (ref.model.actor.flat().numpy(), ref.model.critic.flat().numpy(),
                 ref.model.z_filter.running_sum.numpy().copy(), runs)
    dist.destroy_process_group()


@pytest.mark.parametrize('mode', ['clip', 'adapt'])
def test_gloo_world2_dp_equals_single_process(mode):
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), mode, out), nprocs=world, join=True)
    from surreal_amd import synthetic
    from tests.helpers import oracle_batch, ppo_config
    torch.set_num_threads(1)
    lc = ppo_config(B=32, T=6, mode=mode, use_z_filter=True, hidden=(16, 16))
    ref = R.PPOLearnerRef(lc, 5, 3, seed=3)
    stats = ref.learn(oracle_batch(synthetic.ppo_batch(32, 6, 5, 3, seed=9)))
    a0, c0, z0, r0 = out[0]
    a1, c1, z1, r1 = out[1]
    assert np.array_equal(a0, a1) and np.array_equal(c0, c1) and r0 == r1
    assert r0 == stats['epochs_run']
    ra, rc = ref.model.actor.flat().numpy(), ref.model.critic.flat().numpy()
    scale_a, scale_c = np.abs(ra).max(), np.abs(rc).max()
    assert np.max(np.abs(a0 - ra)) <= 1e-5 * scale_a + 2 * 3e-4 * 1e-3
    assert np.max(np.abs(c0 - rc)) <= 1e-5 * scale_c + 2 * 3e-4 * 1e-3
    assert np.allclose(z0, ref.model.z_filter.running_sum.numpy(), rtol=1e-5, atol=1e-5)
