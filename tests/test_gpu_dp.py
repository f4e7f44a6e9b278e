"""Data-parallel PPO learner on the GPU: ranks are simulated in one process
(one GPU box = one device), driving each learner's phase generator in lockstep
and summing the exchange buffers exactly as the RCCL all-reduce does.  The
result must equal the CPU oracle's single-process learn() on the concatenated
global batch (tolerances as in test_gpu_ppo.py), and every rank must hold
bit-identical parameters afterwards."""
import numpy as np
import pytest
import torch

from oracle import ppo_ref as R
from surreal_amd import synthetic
from surreal_amd.learner import PPOLearner
from tests.helpers import copy_weights_to_oracle, env_config, max_rel_err, oracle_batch, ppo_config

pytestmark = pytest.mark.gpu


class _Group(object):
    def __init__(self, n):
        self.world_size = n

    def allreduce_(self, t):
        raise AssertionError('ranks are driven through _learn_phases in this test')


def _shard(batch, lo, hi):
    def cut(x):
        if x is None:
            return None
        if isinstance(x, dict):
            return {k: cut(v) for k, v in x.items()}
        if isinstance(x, list):
            return [cut(v) for v in x]
        return x[lo:hi].contiguous()
    return cut(batch)


def _lockstep(learners, shards):
    gens = [l._learn_phases(s) for l, s in zip(learners, shards)]
    nphase = 0
    while True:
        bufs, done = [], 0
        for g in gens:
            try:
                bufs.append(next(g))
            except StopIteration:
                done += 1
        if done:
            assert done == len(gens)
            return nphase
        total = bufs[0].clone()
        for b in bufs[1:]:
            total += b
        for b in bufs:
            b.copy_(total)
        nphase += 1


@pytest.mark.parametrize('mode,world,B_loc,rf', [('clip', 2, 32, False), ('adapt', 2, 32, False),
                                                 ('adapt', 4, 16, False), ('clip', 3, 7, False),
                                                 ('adapt', 2, 32, True), ('clip', 3, 7, True)])
def test_dp_equals_global_batch(mode, world, B_loc, rf):
    # rf: RewardFilter on (reward_scale 2): each rank whitens with the shared
    # pre-update stats and the update uses the all-reduced global sums
    T, D, A = 12, 17, 6
    kw = dict(use_r_filter=True, reward_scale=2.0) if rf else {}
    lc = ppo_config(B=B_loc, T=T, mode=mode, use_z_filter=True, **kw)
    learners = [PPOLearner(lc, env_config(D, A), seed=21, dp=_Group(world)) for _ in range(world)]
    lcg = ppo_config(B=B_loc * world, T=T, mode=mode, use_z_filter=True, **kw)
    ref = R.PPOLearnerRef(lcg, D, A)
    copy_weights_to_oracle(learners[0], ref)
    report = {}
    # every arm on the bar every learn() parity test uses: the fp32 envelope
    # around the fp64 oracle on the GLOBAL batch (tests/parity.py;
    # test_gpu_parity_pinned.py).  With the RewardFilter the whitened rewards
    # also carry the filter's fp32 rounding (rank sums in fp64, the
    # reference's one fp32 sum), which the envelope's ulp variants cover.
    from tests import parity as P
    st0 = P.gpu_state(learners[0])
    st0.pop('zf', None)
    r64, vs = P.envelope(st0, lcg, D, A, None, n_ulp=4)
    for it in range(2):
        batch = synthetic.ppo_batch(B_loc * world, T, D, A, seed=300 + it)
        dev = synthetic.to_device(batch, 'cuda')
        shards = [_shard(dev, r * B_loc, (r + 1) * B_loc) for r in range(world)]
        nphase = _lockstep(learners, shards)
        assert nphase == int(rf) + 1 + max(11, 10) + 1   # [reward sums,] moments, epochs, z-filter
        rstats = ref.learn(oracle_batch(batch))
        stats = learners[0].last_stats()
        assert stats['epochs_run'] == rstats['epochs_run']
        ob = oracle_batch(batch)
        r64.learn(ob)
        for k, v in enumerate(vs):
            v.learn(ob, 300 + it)
        for name, got, ref_of in (('actor', learners[0].model.actor.flat, lambda r: r.model.actor.flat()),
                                  ('critic', learners[0].model.critic.flat, lambda r: r.model.critic.flat())):
            w, sc = P.width(ref_of(r64).double().numpy(), [ref_of(v.ref).double().numpy() for v in vs])
            P.check(f'{name}@{it}', got.cpu(), ref_of(r64).double().numpy(), w, sc, report)
        zf, zf64 = learners[0].model.z_filter, r64.model.z_filter
        for b in ('running_sum', 'running_sumsq'):
            w, sc = P.width(getattr(zf64, b).double().numpy(), [getattr(v.ref.model.z_filter, b).double().numpy() for v in vs])
            P.check(f'zf_{b}@{it}', getattr(zf, b).cpu(), getattr(zf64, b).double().numpy(), w, sc, report)
        assert float(zf.count.item()) == float(ref.model.z_filter.count.item())
        for l in learners[1:]:
            assert torch.equal(l.model.actor.flat, learners[0].model.actor.flat)
            assert torch.equal(l.model.critic.flat, learners[0].model.critic.flat)
            assert torch.equal(l.model.z_filter.running_sum, learners[0].model.z_filter.running_sum)
        if rf:
            for b in ('running_sum', 'running_sumsq', 'count'):
                got, exp = float(getattr(learners[0].reward_filter, b).item()), float(getattr(r64.reward_filter, b).item())
                assert abs(got - exp) <= 1e-6 * abs(exp) + 1e-6, (it, b, got, exp)
                assert all(torch.equal(getattr(l.reward_filter, b), getattr(learners[0].reward_filter, b))
                           for l in learners)
            continue
        for k in ('_surr_loss', '_pol_kl', '_entropy', '_val_loss', '_avg_return_targ',
                  '_avg_behave_likelihood', '_avg_is_weight', '_ref_behave_diff',
                  'grad_norm_actor', 'grad_norm_critic', '_val_explained_var'):
            assert abs(stats[k] - rstats[k]) <= 1e-4 * abs(rstats[k]) + 1e-6, (it, k, stats[k], rstats[k])
    P.print_report(report)


def test_dp_world1_matches_fused_path():
    # the phase kernels with one rank reproduce the fused single-launch kernel
    T, D, A, B = 10, 17, 6, 48
    lc = ppo_config(B=B, T=T, mode='adapt', use_z_filter=True)
    fused = PPOLearner(lc, env_config(D, A), seed=4)
    phased = PPOLearner(lc, env_config(D, A), seed=4, dp=_Group(1))
    for it in range(2):
        b = synthetic.to_device(synthetic.ppo_batch(B, T, D, A, seed=it), 'cuda')
        fused.learn(b)
        _lockstep([phased], [b])
        sf, sp = fused.last_stats(), phased.last_stats()
        assert sf['epochs_run'] == sp['epochs_run']
        assert max_rel_err(phased.model.actor.flat.cpu(), fused.model.actor.flat.cpu()) < 1e-4
        assert max_rel_err(phased.model.critic.flat.cpu(), fused.model.critic.flat.cpu()) < 1e-4


def _capture_worker(rank, port, outdir):
    import os
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1)
    from surreal_amd.learner import TorchDistAllReduce
    from tests.test_gpu_boundary import _same, _state
    dp = TorchDistAllReduce()
    lc = ppo_config(B=128, T=25, mode='adapt', use_z_filter=True, hidden=(300, 200), lam=1.0,
                    epochs=(4, 4), rnn=True, rnn_hidden=100, horizon=5)
    lc.parameter_publish.exp_interval = 2 * lc.replay.batch_size
    ec = env_config(42, 8)
    eager = PPOLearner(lc, ec, seed=4, dp=dp)
    graph = PPOLearner(lc, ec, seed=4, dp=dp, use_graph=True)
    same = []
    for it in range(5):
        b = synthetic.to_device(synthetic.ppo_batch(128, 25, 42, 8, seed=70 + it, rnn_hidden=100), 'cuda')
        eager.learn(b)
        graph.learn(b)
        eager.publish_parameter(it)
        graph.publish_parameter(it)
        torch.cuda.synchronize()
        ok = _same(_state(eager), _state(graph)) and eager.last_stats() == graph.last_stats()
        ok = ok and all(torch.equal(v, graph.optimizer_state()[k]) for k, v in eager.optimizer_state().items())
        same.append(bool(ok))
    torch.save({'capturable': dp.capturable, 'captured': graph._graph is not None, 'same': same},
               os.path.join(outdir, 'res.pt'))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_learn_captured_with_rccl_allreduce_bit_exact():
    """A data-parallel learner over RCCL (backend 'nccl', world 1 on this one-GPU
    box) replays learn() as ONE hipGraph with the all-reduces captured between
    its launches: bit-identical to the same data-parallel learner run eagerly,
    over several learns with a publish between them (a rank of a
    strong-scaled job issues ~400 launches and 33 collectives per learn)."""
    import os
    import tempfile
    import torch.multiprocessing as mp
    from tests.test_gpu_dp_procs import _free_port
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_capture_worker, args=(_free_port(), d), nprocs=1, join=True)
        res = torch.load(os.path.join(d, 'res.pt'), weights_only=True)
    assert res['capturable'] and res['captured'], res
    assert all(res['same']), res
