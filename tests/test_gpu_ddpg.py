"""DDPG learner step (ddpg.py:244-428) on the MFMA GEMM layers vs the CPU
oracle, plus the uniform replay (CPython-exact indices) feeding it.  Tolerance
as test_gpu_ppo.py (1e-5 relative, scale floor, Adam sign-flip budget)."""
import copy
import random

import numpy as np
import pytest
import torch

from oracle import ddpg_ref as R
from surreal_amd import _lib as L
from surreal_amd import synthetic
from surreal_amd.config import DDPG_DEFAULT_LEARNER_CONFIG, gym_env_config
from surreal_amd.ddpg import DDPGLearner
from tests.helpers import max_rel_err
from tests.test_gpu_ppo import _compare_params

pytestmark = pytest.mark.gpu


def _cfg(B=512, target='hard', clip_critic=False, layernorm=False):
    lc = copy.deepcopy(DDPG_DEFAULT_LEARNER_CONFIG)
    lc.replay.batch_size = B
    lc.model.use_layernorm = layernorm
    lc.algo.network.clip_critic_gradient = clip_critic
    if target == 'soft':
        lc.algo.network.target_update = {'type': 'soft', 'tau': 1e-3}
    else:
        lc.algo.network.target_update = {'type': 'hard', 'interval': 2}
    return lc


def _sync_weights(learner, ref):
    R.load_flat(ref.actor.params(), learner.model.actor.flat.cpu())
    R.load_flat(ref.critic.params(), learner.model.critic.flat.cpu())
    ref.hard_update()


def _fp32_as_good_as_torch(got, ref32, ref64, slack=1e-6, mag=None):
    """GEMM parity: the HIP result must be within 2x the error of torch's own
    fp32 CPU result against the fp64 truth (+ slack of the scale), and within
    1e-5 relative on the tensor's scale.  Reductions over >~20k rows (weight
    gradients of the B*E = 21504-row C3 batch) accumulate k-ordered MFMA chains
    per split-K slab where torch's CPU kernel blocks more finely: they get
    slack 4e-6 (still inside the 1e-5 parity bar).  `mag` (the largest sum of
    |terms| of one output) replaces the result's scale where the sums cancel:
    fp32 summation error is relative to the magnitudes summed, not to the
    cancelled result (a bias gradient over 4096 rows of +-1)."""
    got, ref32, ref64 = (np.asarray(t, dtype=np.float64) for t in (got, ref32, ref64))
    scale = np.abs(ref64).max() if mag is None else max(float(mag), np.abs(ref64).max())
    e_gpu = np.abs(got - ref64).max()
    e_cpu = np.abs(ref32 - ref64).max()
    assert e_gpu <= 2 * e_cpu + slack * scale, (e_gpu, e_cpu, scale)
    assert e_gpu <= 1e-5 * scale


@pytest.mark.parametrize('rows,k,n', [(512, 17, 300), (70, 406, 300), (512, 300, 1), (3, 5, 7),
                                      (21504, 100, 300), (5376, 42, 400), (20000, 200, 8),
                                      (8192, 17, 300), (4099, 64, 33), (21504, 42, 400),
                                      (300, 2592, 64), (2688, 2592, 256), (4096, 300, 1),
                                      (3000, 17, 6), (21504, 200, 1), (777, 100, 3), (9, 256, 5)])
def test_linear_ops_vs_torch(rows, k, n):
    L.ensure_workspace(torch.device('cuda'))      # split-K paths (dW; few-tile long-K forward)
    g = torch.Generator().manual_seed(rows + k)
    x = torch.randn(rows, k, generator=g)
    lin = torch.nn.Linear(k, n)
    W, b = lin.weight.detach(), lin.bias.detach()
    dy = torch.randn(rows, n, generator=g)
    xd, wd, bd = x.cuda(), W.cuda().contiguous(), b.cuda()
    y = torch.empty(rows, n, device='cuda')
    st = L.stream()
    L.call('smi_linear_forward', L.ptr(xd), k, rows, k, L.ptr(wd), k, L.ptr(bd), n, 1, L.ptr(y), n, st)
    _fp32_as_good_as_torch(y.cpu(), torch.relu(x @ W.t() + b),
                           torch.relu(x.double() @ W.double().t() + b.double()))
    dyd = dy.cuda()
    dx = torch.empty(rows, k, device='cuda')
    L.call('smi_linear_backward_input', L.ptr(dyd), n, rows, n, L.ptr(wd), k, k, L.ptr(xd), k,
           L.ptr(dx), k, st)
    _fp32_as_good_as_torch(dx.cpu(), (dy @ W) * (x > 0), (dy.double() @ W.double()) * (x > 0))
    dw = torch.empty(n, k, device='cuda')
    db = torch.empty(n, device='cuda')
    L.call('smi_linear_backward_weight', L.ptr(dyd), n, rows, n, L.ptr(xd), k, k, L.ptr(dw), k,
           L.ptr(db), 0, st)
    sl = 4e-6 if rows > 16384 else 1e-6
    mw = float((dy.abs().t() @ x.abs()).max())
    mb = float(dy.abs().sum(0).max())
    _fp32_as_good_as_torch(dw.cpu(), dy.t() @ x, dy.double().t() @ x.double(), sl, mw)
    _fp32_as_good_as_torch(db.cpu(), dy.sum(0), dy.double().sum(0), sl, mb)
    # accumulate into existing gradients (split-K reducer path for long reductions)
    L.call('smi_linear_backward_weight', L.ptr(dyd), n, rows, n, L.ptr(xd), k, k, L.ptr(dw), k,
           L.ptr(db), 1, st)
    _fp32_as_good_as_torch(dw.cpu(), 2 * (dy.t() @ x), 2 * (dy.double().t() @ x.double()), sl,
                           2 * mw)
    _fp32_as_good_as_torch(db.cpu(), 2 * dy.sum(0), 2 * dy.double().sum(0), sl, 2 * mb)


def test_dw_group_vs_torch():
    """smi_dw_group_begin / _flush: weight gradients queued between them run as
    one grouped launch at the flush.  Mixed group: the DDPG layer shapes, an
    accumulating call, one output too large to group (launches at once), and
    more calls than a group holds (the overflow launches at once)."""
    L.ensure_workspace(torch.device('cuda'))
    shapes = [(512, 17, 400, 0), (512, 406, 300, 1), (512, 301, 1, 0), (512, 17, 300, 0),
              (512, 300, 600, 0), (512, 300, 200, 0), (512, 201, 6, 1), (4099, 64, 33, 0)]
    g = torch.Generator().manual_seed(11)
    st = L.stream()
    cases = []
    for rows, k, n, acc in shapes:
        x, dy = torch.randn(rows, k, generator=g), torch.randn(rows, n, generator=g)
        w0, b0 = torch.randn(n, k, generator=g), torch.randn(n, generator=g)
        dev = [t.cuda() for t in (x, dy, w0, b0)]
        cases.append((rows, k, n, acc, x, dy, w0, b0, dev))
    L.call('smi_dw_group_begin')
    for rows, k, n, acc, x, dy, w0, b0, (xd, dyd, dw, db) in cases:
        L.call('smi_linear_backward_weight', L.ptr(dyd), n, rows, n, L.ptr(xd), k, k, L.ptr(dw), k,
               L.ptr(db), acc, st)
    L.call('smi_dw_group_flush', st)
    for rows, k, n, acc, x, dy, w0, b0, (xd, dyd, dw, db) in cases:
        mw = float((dy.abs().t() @ x.abs()).max()) + acc * float(w0.abs().max())
        mb = float(dy.abs().sum(0).max()) + acc * float(b0.abs().max())
        _fp32_as_good_as_torch(dw.cpu(), acc * w0 + dy.t() @ x,
                               acc * w0.double() + dy.double().t() @ x.double(), 1e-6, mw)
        _fp32_as_good_as_torch(db.cpu(), acc * b0 + dy.sum(0), acc * b0.double() + dy.double().sum(0),
                               1e-6, mb)


@pytest.mark.parametrize('rows,n', [(512, 300), (512, 400), (70, 200), (3, 37), (1, 1024)])
def test_layernorm_kernels_vs_torch(rows, n):
    """smi_layernorm_forward / _backward (ReLU before the norm) against
    torch.nn.functional.layer_norm in fp64 autograd, at 2x the error of torch's
    own fp32 CPU layer_norm (or 1e-6 of scale)."""
    g = torch.Generator().manual_seed(rows * 7 + n)
    z = torch.randn(rows, n, generator=g, dtype=torch.float64)
    x = torch.relu(z)
    gamma = 1 + 0.1 * torch.randn(n, generator=g, dtype=torch.float64)
    beta = 0.1 * torch.randn(n, generator=g, dtype=torch.float64)
    dy = torch.randn(rows, n, generator=g, dtype=torch.float64)

    def ref(dtype):
        xx = x.to(dtype).clone().requires_grad_(True)
        gg, bb = gamma.to(dtype).clone().requires_grad_(True), beta.to(dtype).clone().requires_grad_(True)
        y = torch.nn.functional.layer_norm(xx, (n,), gg, bb, 1e-5)
        y.backward(dy.to(dtype))
        dx = xx.grad * (x > 0).to(dtype)                      # through the ReLU
        return [t.detach().double() for t in (y, dx, gg.grad, bb.grad)]
    r64, r32 = ref(torch.float64), ref(torch.float32)
    dev = 'cuda'
    xd, gd, bd, dyd = (t.float().to(dev) for t in (x, gamma, beta, dy))
    y, mu, rs = torch.empty(rows, n, device=dev), torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    dx, dg, db = torch.empty(rows, n, device=dev), torch.empty(n, device=dev), torch.empty(n, device=dev)
    st = L.stream(torch.device(dev))
    L.call('smi_layernorm_forward', L.ptr(xd), n, rows, n, L.ptr(gd), L.ptr(bd), 1e-5, L.ptr(y), n,
           L.ptr(mu), L.ptr(rs), st)
    L.call('smi_layernorm_backward', L.ptr(dyd), n, L.ptr(xd), n, L.ptr(mu), L.ptr(rs), L.ptr(gd), rows,
           n, 1, L.ptr(dx), n, L.ptr(dg), L.ptr(db), st)
    torch.cuda.synchronize()
    for name, got, a, b in zip(('y', 'dx', 'dgamma', 'dbeta'), (y, dx, dg, db), r32, r64):
        got = got.double().cpu()
        scale = float(b.abs().max())
        e_gpu, e_cpu = float((got - b).abs().max()), float((a - b).abs().max())
        assert e_gpu <= 2 * e_cpu + 1e-6 * scale, (name, e_gpu, e_cpu, scale)
    assert torch.allclose(mu.double().cpu(), x.mean(1), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize('target,clip_critic,layernorm', [('hard', False, False), ('soft', True, False),
                                                          ('hard', False, True), ('soft', True, True)])
def test_ddpg_learn_matches_oracle(target, clip_critic, layernorm):
    B, D, A = 512, 17, 6
    lc = _cfg(B, target, clip_critic, layernorm)
    learner = DDPGLearner(lc, gym_env_config(D, A), seed=2)
    ref = R.DDPGLearnerRef(lc, D, A)
    _sync_weights(learner, ref)
    report = {}
    for it in range(3):
        b = synthetic.ddpg_batch(B, D, A, seed=it)
        rs = ref.optimize(b['obs'], b['actions'], b['rewards'], b['obs_next'], b['dones'])
        learner.learn({k: v.cuda() for k, v in b.items()})
        s = learner.last_stats()
        for k in rs:
            assert abs(s[k] - rs[k]) <= 1e-4 * abs(rs[k]) + 1e-5, (it, k, s[k], rs[k])
        _compare_params(f'critic{it}', learner.model.critic.flat.cpu(), R.flat_of(ref.critic.params()),
                        1e-3, it + 1, report)
        # the DDPG actor gradient is the critic's input gradient pushed back
        # through the actor (ddpg.py:325-329): more of its entries are fp32
        # rounding noise than in PPO, so the Adam sign-flip budget is 0.5 %
        _compare_params(f'actor{it}', learner.model.actor.flat.cpu(), R.flat_of(ref.actor.params()),
                        1e-4, it + 1, report, max_frac=5e-3)
        _compare_params(f'tcritic{it}', learner.model_target.critic.flat.cpu(),
                        R.flat_of(ref.critic_t.params()), 1e-3, it + 1, report)
    print('ddpg parity report:', report)


@pytest.mark.parametrize('target,action_reg', [('hard', False), ('soft', True)])
def test_ddpg_td3_matches_oracle(target, action_reg):
    """TD3 options (ddpg.py:267-283,312-320): twin critic with min target, and
    target-policy smoothing noise drawn from numpy's global RNG on the host (the
    reference's own generator: both sides are seeded identically per step)."""
    B, D, A = 512, 17, 6
    lc = _cfg(B, target, False)
    lc.algo.network.use_double_critic = True
    lc.algo.network.use_action_regularization = action_reg
    learner = DDPGLearner(lc, gym_env_config(D, A), seed=2)
    ref = R.DDPGLearnerRef(lc, D, A)
    _sync_weights(learner, ref)
    R.load_flat(ref.critic2.params(), learner.model2.critic.flat.cpu())
    ref.hard_update()
    report = {}
    for it in range(3):
        b = synthetic.ddpg_batch(B, D, A, seed=it)
        np.random.seed(100 + it)
        rs = ref.optimize(b['obs'], b['actions'], b['rewards'], b['obs_next'], b['dones'])
        np.random.seed(100 + it)
        learner.learn({k: v.cuda() for k, v in b.items()})
        s = learner.last_stats()
        for k in rs:
            assert abs(s[k] - rs[k]) <= 1e-4 * abs(rs[k]) + 1e-5, (it, k, s[k], rs[k])
        _compare_params(f'critic{it}', learner.model.critic.flat.cpu(), R.flat_of(ref.critic.params()),
                        1e-3, it + 1, report)
        _compare_params(f'critic2_{it}', learner.model2.critic.flat.cpu(),
                        R.flat_of(ref.critic2.params()), 1e-3, it + 1, report)
        # min(y1, y2) picks per row; rows with y1 ~ y2 within fp32 noise may pick
        # differently in any two implementations (like a ReLU mask flip), on
        # top of the DDPG actor's sign-flip budget: 1 %
        _compare_params(f'actor{it}', learner.model.actor.flat.cpu(), R.flat_of(ref.actor.params()),
                        1e-4, it + 1, report, max_frac=1e-2)
        _compare_params(f'tcritic2_{it}', learner.model_target2.critic.flat.cpu(),
                        R.flat_of(ref.critic2_t.params()), 1e-3, it + 1, report)
    print('ddpg td3 parity report:', report)


def test_replay_sample_feeds_learner_with_cpython_indices():
    from surreal_amd.replay import UniformReplay
    D, A, B = 17, 6, 512
    lc = _cfg(B)
    lc.replay.memory_size = 5000
    lc.replay.sampling_start_size = 100
    ec = gym_env_config(D, A)
    rep = UniformReplay(lc, ec, seed=1234)
    rows = np.random.RandomState(0).randn(3000, rep.width).astype(np.float32)
    rows[:, D:D + A] = np.tanh(rows[:, D:D + A])
    rep.insert_rows(rows)
    assert rep.start_sample_condition()
    idx, got = rep.sample(B)
    random.seed(1234)
    exp = [random.randint(0, 3000 - 1) for _ in range(B)]
    assert idx.cpu().tolist() == exp
    assert torch.equal(got.cpu(), torch.from_numpy(rows[exp]))
    learner = DDPGLearner(lc, ec, seed=0)
    learner.learn(rep.split(got))
    assert np.isfinite(list(learner.last_stats().values())).all()


def test_replay_bulk_insert_wraps_like_single_inserts():
    """uniform_replay.py:36-41: insert() appends until memory_size, then
    overwrites the oldest slot; a bulk insert of more rows than slots keeps the
    last memory_size rows in the same slots as repeated single inserts."""
    from surreal_amd.replay import UniformReplay
    D, A = 5, 2
    lc = _cfg(8)
    lc.replay.memory_size = 7
    ec = gym_env_config(D, A)
    bulk = UniformReplay(lc, ec, seed=1)
    single = UniformReplay(lc, ec, seed=1)
    rs = np.random.RandomState(3)
    for n in (3, 18, 1, 9):
        rows = rs.randn(n, bulk.width).astype(np.float32)
        bulk.insert_rows(rows)
        for r in rows:
            single.insert_rows(r[None])
        assert torch.equal(bulk.table.cpu(), single.table.cpu()), n
        assert len(bulk) == len(single) and bulk._next_idx == single._next_idx


@pytest.mark.parametrize('target', ['hard', 'soft'])
def test_ddpg_graph_replay_bit_exact(target):
    """hipGraph replay of the update (use_graph=True) runs the same launch
    sequence on the same buffers: parameters, target networks and statistics
    are bit-identical to the eager learner over several steps (hard target
    interval 2 exercises the host-side target update between replays)."""
    B, D, A = 512, 17, 6
    lc = _cfg(B, target)
    eager = DDPGLearner(lc, gym_env_config(D, A), seed=3)
    graph = DDPGLearner(lc, gym_env_config(D, A), seed=3, use_graph=True)
    for it in range(5):
        b = {k: v.cuda() for k, v in synthetic.ddpg_batch(B, D, A, seed=10 + it).items()}
        eager.learn(b)
        graph.learn(b)
        torch.cuda.synchronize()
        for name in ('actor', 'critic'):
            assert torch.equal(getattr(eager.model, name).flat, getattr(graph.model, name).flat), (it, name)
            assert torch.equal(getattr(eager.model_target, name).flat,
                               getattr(graph.model_target, name).flat), (it, name)
        assert eager.last_stats() == graph.last_stats(), it
    assert graph._graph is not None
