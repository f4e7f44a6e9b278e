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


# --------------------------------------------------- learn() on the envelope
# The C4 step on the same bar as the PPO learner (tests/parity.py): the fp64
# oracle is the truth; the envelope is the fp32 oracle over row orders (given,
# reversed, shuffled) and the fp64 oracle with one fp32 rounding of relative
# noise on its inputs and initial weights (6 seeds).  Parameters (actor,
# critic, critic2, target critics) must satisfy max|GPU - fp64| <= 2 *
# envelope + 1e-6 * scale; a statistic (a mean over the step's rows, taken at
# the step's starting parameters) likewise, or within 1e-5 of its magnitude.
DDPG_ORDERS = ('given', 'reversed', 'shuffled')


class _DVariant(object):
    def __init__(self, kind, key, lc, D, A, init, pixel=None):
        self.kind, self.key = kind, key
        self.pixel = pixel
        self.ref = R.DDPGLearnerRef(lc, D, A, dtype=torch.float32 if kind == 'order' else torch.float64,
                                    pixel=pixel)
        self.gen = torch.Generator().manual_seed(777 + 13 * key if kind == 'ulp' else 0)
        _load_ddpg(self.ref, init, self._noisy if kind == 'ulp' else None)

    def _noisy(self, x):
        x = torch.as_tensor(x).to(torch.float32).double()
        return x * (1 + 2.0 ** -24 * torch.randn(x.shape, generator=self.gen, dtype=torch.float64))

    def optimize(self, b, it):
        B = b['rewards'].shape[0]
        if self.kind == 'order':
            p = (np.arange(B) if self.key == 'given' else np.arange(B)[::-1].copy()
                 if self.key == 'reversed' else np.random.RandomState(50 + it).permutation(B))
            self.ref.noise_perm = p
            x = {k: torch.as_tensor(np.asarray(v)[p]) for k, v in b.items()}
        else:
            x = {k: (torch.as_tensor(v) if k in ('pix', 'pix_next') else self._noisy(v))
                 for k, v in b.items()}
            x['dones'] = torch.as_tensor(b['dones'], dtype=torch.float64)
        obs, obs_next = x['obs'], x['obs_next']
        if self.pixel is not None:                  # camera frames: uint8, exact in every execution
            obs, obs_next = (obs, x['pix']), (obs_next, x['pix_next'])
        return self.ref.optimize(obs, x['actions'], x['rewards'], obs_next, x['dones'])


def _load_ddpg(ref, init, noisy=None):
    f = (lambda t: t) if noisy is None else noisy
    R.load_flat(ref.actor.params(), f(init['actor']))
    R.load_flat(ref.critic.params(), f(init['critic']))
    if 'critic2' in init:
        R.load_flat(ref.critic2.params(), f(init['critic2']))
    if 'perc' in init:
        R.load_flat(list(ref.perc.parameters()), f(init['perc']))
    if 'perc2' in init:
        R.load_flat(list(ref.perc2.parameters()), f(init['perc2']))
    # the constructor syncs actor / critic(s) only (ddpg.py:174-178); the target
    # perceptions keep their own init, taken from the learner
    ref.hard_update(perception=False)
    if 'perc_t' in init:
        R.load_flat(list(ref.perc_t.parameters()), f(init['perc_t']))
    if 'perc2_t' in init:
        R.load_flat(list(ref.perc2_t.parameters()), f(init['perc2_t']))


def _ddpg_state(learner):
    out = {'actor': learner.model.actor.flat.detach().cpu().clone(),
           'critic': learner.model.critic.flat.detach().cpu().clone(),
           'critic_t': learner.model_target.critic.flat.detach().cpu().clone(),
           'actor_t': learner.model_target.actor.flat.detach().cpu().clone()}
    if learner.use_double_critic:
        out['critic2'] = learner.model2.critic.flat.detach().cpu().clone()
        out['critic2_t'] = learner.model_target2.critic.flat.detach().cpu().clone()
    if learner.is_pixel_input:
        out['perc'] = learner.model.perception.flat.detach().cpu().clone()
        out['perc_t'] = learner.model_target.perception.flat.detach().cpu().clone()
        if learner.use_double_critic:
            out['perc2'] = learner.model2.perception.flat.detach().cpu().clone()
            out['perc2_t'] = learner.model_target2.perception.flat.detach().cpu().clone()
    return out


def _ddpg_ref_state(ref):
    out = {'actor': R.flat_of(ref.actor.params()), 'critic': R.flat_of(ref.critic.params()),
           'critic_t': R.flat_of(ref.critic_t.params()), 'actor_t': R.flat_of(ref.actor_t.params())}
    if ref.double:
        out['critic2'] = R.flat_of(ref.critic2.params())
        out['critic2_t'] = R.flat_of(ref.critic2_t.params())
    if ref.pixel is not None:
        out['perc'] = R.flat_of(list(ref.perc.parameters()))
        out['perc_t'] = R.flat_of(list(ref.perc_t.parameters()))
        if ref.double:
            out['perc2'] = R.flat_of(list(ref.perc2.parameters()))
            out['perc2_t'] = R.flat_of(list(ref.perc2_t.parameters()))
    return {k: v.double().numpy() for k, v in out.items()}


def ddpg_envelope_run(lc, D, A, iters=3, batches=None, n_ulp=6, learn_input=None, seed=2,
                      pixel=None):
    """the HIP learner vs the fp64 oracle within the envelope over `iters`
    steps.  batches: list of numpy dicts (obs, actions, rewards (B,1),
    obs_next, dones (B,1)); learn_input(learner, it) -> what learner.learn()
    gets (default: the batch on the device)."""
    B = lc.replay.batch_size
    from surreal_amd.config import pixel_env_config
    ec = pixel_env_config(D, A, pixel) if pixel is not None else gym_env_config(D, A)
    learner = DDPGLearner(lc, ec, seed=seed)
    init = {k: v for k, v in _ddpg_state(learner).items()
            if k in ('actor', 'critic', 'critic2', 'perc', 'perc2', 'perc_t', 'perc2_t')}
    if batches is None:
        batches = [{k: v.numpy() for k, v in synthetic.ddpg_batch(B, D, A, seed=it).items()}
                   for it in range(iters)]
    gpu = []
    for it, b in enumerate(batches):
        np.random.seed(100 + it)                    # the TD3 smoothing noise's stream
        if learn_input is None and pixel is not None:
            dev = {k: torch.as_tensor(b[k], dtype=torch.float32).cuda()
                   for k in ('actions', 'rewards', 'dones')}
            for k, pk in (('obs', 'pix'), ('obs_next', 'pix_next')):
                dev[k] = {'low_dim': {'flat_inputs': torch.as_tensor(b[k], dtype=torch.float32).cuda()},
                          'pixel': {'camera0': torch.as_tensor(b[pk]).cuda()}}
            learner.learn(dev)
        elif learn_input is None:
            learner.learn({k: torch.as_tensor(v, dtype=torch.float32).cuda() for k, v in b.items()})
        else:
            learner.learn(learn_input(learner, it))
        gpu.append((_ddpg_state(learner), learner.last_stats()))
    ddpg_envelope_check(lc, D, A, init, batches, gpu, n_ulp=n_ulp, pixel=pixel)
    return learner


def ddpg_envelope_check(lc, D, A, init, batches, gpu, n_ulp=6, pixel=None, tag=''):
    """gpu[it] = (_ddpg_state, last_stats()) of a HIP learner after step it
    (started from `init`, np.random seeded 100 + it before each step) against
    the fp64 oracle's optimize() over the same batches, within the envelope of
    equally valid fp32 executions (tests/parity.py)."""
    from tests import parity as P
    r64 = R.DDPGLearnerRef(lc, D, A, dtype=torch.float64, pixel=pixel)
    _load_ddpg(r64, init)
    vs = [_DVariant('order', k, lc, D, A, init, pixel) for k in DDPG_ORDERS]
    vs += [_DVariant('ulp', k, lc, D, A, init, pixel) for k in range(1, n_ulp + 1)]
    report = {}
    for it, b in enumerate(batches):
        np.random.seed(100 + it)
        f64 = lambda k: torch.as_tensor(b[k], dtype=torch.float32).double()  # noqa: E731
        o64, on64 = f64('obs'), f64('obs_next')
        if pixel is not None:
            o64, on64 = (o64, torch.as_tensor(b['pix'])), (on64, torch.as_tensor(b['pix_next']))
        s64 = r64.optimize(o64, f64('actions'), f64('rewards'), on64, f64('dones'))
        svs = []
        for v in vs:
            np.random.seed(100 + it)
            svs.append(v.optimize(b, it))
        got, s = gpu[it]
        p64 = _ddpg_ref_state(r64)
        pvs = [_ddpg_ref_state(v.ref) for v in vs]
        for k in p64:
            w, sc = P.width(p64[k], [x[k] for x in pvs])
            P.check(f'{k}{tag}@{it}', got[k], p64[k], w, sc, report)
        for k in s64:
            w = max(abs(x[k] - s64[k]) for x in svs)
            e, sc = abs(s[k] - s64[k]), max(abs(s64[k]), 1e-30)
            bar = max(2 * w + 1e-6 * sc, 1e-5 * sc)
            ok = e <= bar
            report[f'stat{tag}:{k}@{it}'] = (e / sc, bar / sc, ok, w / sc)
            if not ok:
                report.setdefault('_fail', []).append(f'stat{tag}:{k}@{it}')
    P.print_report(report)
    return report


@pytest.mark.parametrize('target,clip_critic,layernorm', [('hard', False, False), ('soft', True, False),
                                                          ('hard', False, True), ('soft', True, True)])
def test_ddpg_learn_envelope(target, clip_critic, layernorm):
    # BASELINE configs[3]: batch 512, HalfCheetah dims, actor 300x200, critic 400x300, n 3
    ddpg_envelope_run(_cfg(512, target, clip_critic, layernorm), 17, 6, iters=3)


@pytest.mark.parametrize('target,action_reg', [('hard', False), ('soft', True)])
def test_ddpg_td3_envelope(target, action_reg):
    """TD3 options (ddpg.py:267-283,312-320): twin critic with min target, and
    target-policy smoothing noise from numpy's global RNG on the host (the
    reference's own generator: every execution is seeded identically per step,
    row-permuted executions permute the noise rows with the batch rows)."""
    lc = _cfg(512, target, False)
    lc.algo.network.use_double_critic = True
    lc.algo.network.use_action_regularization = action_reg
    ddpg_envelope_run(lc, 17, 6, iters=3)


@pytest.mark.parametrize('target,td3', [('hard', False), ('soft', True)])
def test_ddpg_pixel_envelope(target, td3):
    """DDPG with camera observations (ddpg_net.py:34-43,57-79; ddpg.py:207-223,
    287-333,409-428): 3 stacked RGB frames (9 x 84 x 84 uint8, frame_stacks 3,
    ddpg_configs.py:114) -> CNNStemNetwork (16@8s4, 32@4s2, FC 200) concatenated
    with the low-dim state before actor and critic; the perception trains with
    the critic optimizer (no value clip: the reference clips model.critic only),
    the actor reads it detached, the targets copy / track it.  TD3: the twin has
    its own perception and target perception."""
    B, D, A, cam = 64, 17, 6, (9, 84, 84)
    lc = _cfg(B, target, False)
    if td3:
        lc.algo.network.use_double_critic = True
        lc.algo.network.use_action_regularization = True
    batches = []
    for it in range(3):
        b = {k: v.numpy() for k, v in synthetic.ddpg_batch(B, D, A, seed=70 + it).items()}
        g = torch.Generator().manual_seed(170 + it)
        b['pix'] = torch.randint(0, 256, (B,) + cam, generator=g, dtype=torch.uint8).numpy()
        b['pix_next'] = torch.randint(0, 256, (B,) + cam, generator=g, dtype=torch.uint8).numpy()
        batches.append(b)
    learner = ddpg_envelope_run(lc, D, A, batches=batches, pixel=cam, n_ulp=3)
    assert learner.is_pixel_input


def test_ddpg_host_path_ssar_envelope():
    """experience lists as ExpSenderWrapperSSAR sends them ->
    DDPGLearner._prefetcher_preprocess (SSARAggregator, aggregator.py:52-103) ->
    preprocess (the host -> device copy, ddpg.py:186-242) -> learn(), on the
    envelope bar against the oracle fed the same aggregated arrays."""
    from oracle import aggregator_ref as AR
    B, D, A = 512, 17, 6
    lc = _cfg(B, 'hard', False)
    ec = gym_env_config(D, A)
    host = [AR.make_ssar_exp_list(AR.ssar_exp_arrays(B, D, A, 900 + it)) for it in range(3)]

    def learn_input(learner, it):            # the learner's own host path
        return learner.preprocess(learner._prefetcher_preprocess(host[it]))
    # the oracle sees the aggregator's output as the reference's preprocess
    # converts it (float32 tensors)
    from surreal_amd.aggregator import SSARAggregator
    aggs = []
    for it in range(3):
        a = SSARAggregator(ec.obs_spec, ec.action_spec).aggregate(host[it])
        aggs.append({'obs': np.asarray(a['obs']['low_dim']['flat_inputs'], np.float32),
                     'actions': np.asarray(a['actions'], np.float32),
                     'rewards': np.asarray(a['rewards'], np.float32),
                     'obs_next': np.asarray(a['obs_next']['low_dim']['flat_inputs'], np.float32),
                     'dones': np.asarray(a['dones'], np.float32)})
        assert aggs[-1]['rewards'].shape == (B, 1) and aggs[-1]['dones'].shape == (B, 1)
    ddpg_envelope_run(lc, D, A, batches=aggs, learn_input=learn_input)


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
