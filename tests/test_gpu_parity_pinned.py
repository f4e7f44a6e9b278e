"""PPOLearner.learn() pinned at the configurations bench.py measures.

Bars (tests/parity.py has the full statement):
  * trajectory quantities — advantages as the epochs use them, raw advantages,
    returns, post-step actor / critic / LSTM / CNN parameters, ZFilter sums,
    first-step raw gradients — against the fp64 oracle within the fp32
    ENVELOPE: max|GPU - fp64| <= 2 * max_variants max|variant - fp64| +
    1e-6 * scale;
  * every last_stats() entry by SELF-CONSISTENCY: recomputed in fp64 from the
    GPU's own state at the point the reference computes it (ppo.py:194-331,
    553-575) and required within 1e-5 (north_star) of its magnitude;
  * the number of policy epochs run equal in every execution.

Cases: C2 (B 64 x T 50, 64x64 MLP, clip and adapt, 2 learn() calls), the MLP
phase path at B = 1024, a KL early stop, stacked LSTMs, the host-numpy input
path (experience lists -> _prefetcher_preprocess -> learn()) at the reference
--unit-test shape (BASELINE configs[0]), at C2 and with pixels — their oracle
envelopes run live; and the full-size cases, whose fp64 truth and envelope
widths were computed in the build container (tests/golden/make_envelopes.py ->
tests/golden/envelope_<case>.npz): C3 (the full 1024-segment batch bench.py
times, adapt x 2 learns and clip), C5 (C3 + the 84x84 camera stem at 128
segments, one GPU's share at N = 8), and the raw first-step policy / value
gradients at C3 and at C5 widths.  tests/test_gpu_dp_pinned.py runs the same
fixtures through two data-parallel ranks.
"""
import copy

import numpy as np
import pytest
import torch

from oracle import aggregator_ref as AR
from surreal_amd import synthetic
from surreal_amd.aggregator import StagingArena
from surreal_amd.config import PPO_DEFAULT_LEARNER_CONFIG, gym_env_config, pixel_env_config
from surreal_amd.learner import PPOLearner
from tests import parity as P
from tests.helpers import env_config, oracle_batch, ppo_config

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _env(D, A, pixel):
    return pixel_env_config(D, A, pixel) if pixel is not None else env_config(D, A)


def copy_learner_state(src, dst):
    """dst continues exactly as src would (parameters, filters, Adam state,
    adaptive hyper-parameters): the twin of learn_capture_fused"""
    with torch.no_grad():
        for a, b in ((src.model, dst.model), (src.ref_target_model, dst.ref_target_model)):
            b.actor.flat.copy_(a.actor.flat)
            b.critic.flat.copy_(a.critic.flat)
            b.stem_flat.copy_(a.stem_flat)
            if src.use_z_filter:
                b.z_filter.load_state_dict(a.z_filter.state_dict())
        for k, v in src.optimizer_state().items():
            dst.optimizer_state()[k].copy_(v)
    dst.beta, dst.clip_epsilon = src.beta, src.clip_epsilon
    dst._write_hyper()


def _is_fused(learner, batch):
    if learner.if_rnn_policy or learner.if_pixel_input or learner.dp is not None:
        return False
    return learner.batch_size <= 256


def _used(learner):
    """advantages / returns exactly as the epochs used them"""
    b = learner._bufs
    return b['adv_used'].cpu().numpy(), (b['ret_used'] if 'ret_used' in b else b['ret']).cpu().numpy()


def _check_stats(lc, D, A, pixel, ob, cap, learner, report, tag):
    s = learner.last_stats()
    adv, ret = _used(learner)
    rec = P.recompute_stats(lc, D, A, pixel, ob, cap, adv, ret, s['epochs_run'])
    P.check_stats(s, rec, report, tag=tag)


# ------------------------------------------------------------- live cases
def _host_batch(learner, B, T, D, A, seed, rnn_hidden, pixel):
    arr = AR.ppo_exp_arrays(B, T, D, A, seed, rnn_hidden=rnn_hidden, pixel=pixel)
    return learner._prefetcher_preprocess(AR.make_ppo_exp_list(arr))


def pinned_live(lc, D, A, iters=1, pixel=None, seed=0, rnn_hidden=None, source='synthetic',
                n_ulp=6, orders=('given', 'reversed', ('shuffled', 1))):
    """envelope computed here (small configurations).  source 'synthetic':
    device batches; 'host': experience lists aggregated on the host and handed
    to learn() as numpy (the single-H2D arena)."""
    B, T = lc.replay.batch_size, lc.algo.n_step
    learner = PPOLearner(lc, _env(D, A, pixel), seed=seed + 7, device=DEV)
    learner.export_advantages = True
    st = P.gpu_state(learner)
    st.pop('zf', None)
    r64, vs = P.envelope(st, lc, D, A, pixel, n_ulp, orders)
    report = {}
    for it in range(iters):
        if source == 'host':
            batch = _host_batch(learner, B, T, D, A, seed * 100 + it, rnn_hidden, pixel)
            ob = oracle_batch(batch)
            dev_batch = batch
        else:
            batch = synthetic.ppo_batch(B, T, D, A, seed=seed * 100 + it, rnn_hidden=rnn_hidden,
                                        pixel=pixel, rnn_layers=lc.algo.rnn.rnn_layer)
            ob = oracle_batch(batch)
            dev_batch = synthetic.to_device(batch, DEV)
        s64 = r64.learn(ob)
        svs = [v.learn(ob, seed * 100 + it) for v in vs]
        if _is_fused(learner, dev_batch):
            def clone():
                twin = PPOLearner(lc, _env(D, A, pixel), seed=seed + 7, device=DEV)
                copy_learner_state(learner, twin)
                return twin
            cap = P.learn_capture_fused(learner, dev_batch, clone)
        else:
            cap = P.learn_capture(learner, dev_batch)
        s = learner.last_stats()
        runs = [s['epochs_run'], s64['epochs_run']] + [x['epochs_run'] for x in svs]
        assert len(set(runs)) == 1, (it, runs)
        seg = lambda name: [v.per_segment(getattr(v.ref, name).double().numpy()) for v in vs]  # noqa: E731
        adv, ret = _used(learner)
        w, sc = P.width(r64.last_adv.double().numpy(), seg('last_adv'))
        P.check(f'adv@{it}', adv, r64.last_adv.double().numpy(), w, sc, report)
        w, sc = P.width(r64.last_ret.double().numpy(), seg('last_ret'))
        P.check(f'ret@{it}', ret, r64.last_ret.double().numpy(), w, sc, report)
        if 'adv_raw' in learner._bufs and learner._bufs['adv_raw'].dim() == 1:
            w, sc = P.width(r64.last_adv_raw.double().numpy(), seg('last_adv_raw'))
            P.check(f'adv_raw@{it}', learner._bufs['adv_raw'].cpu(), r64.last_adv_raw.double().numpy(),
                    w, sc, report)
        p64 = P.oracle_params(r64)
        pvs = [P.oracle_params(v.ref) for v in vs]
        fin = cap['final']
        for k in p64:
            w, sc = P.width(p64[k], [x[k] for x in pvs])
            P.check(f'{k}@{it}', fin[k], p64[k], w, sc, report)
        if learner.use_z_filter:
            zf, z64 = learner.model.z_filter, r64.model.z_filter
            for b in ('running_sum', 'running_sumsq'):
                r = getattr(z64, b).double().numpy()
                w, sc = P.width(r, [getattr(v.ref.model.z_filter, b).double().numpy() for v in vs])
                P.check(f'zf_{b}@{it}', getattr(zf, b).cpu(), r, w, sc, report)
            assert float(zf.count.item()) == float(vs[0].ref.model.z_filter.count.item())
        _check_stats(lc, D, A, pixel, ob, cap, learner, report, f'@{it}')
    P.print_report(report)
    return report


@pytest.mark.parametrize('mode', ['clip', 'adapt'])
def test_pinned_c2(mode):
    # BASELINE configs[1]: HalfCheetah dims, 64x64 MLP, 64 segments x n_step 50
    pinned_live(ppo_config(B=64, T=50, mode=mode, use_z_filter=True), 17, 6, iters=2)


@pytest.mark.parametrize('mode', ['clip', 'adapt'])
def test_pinned_mlp_large_batch_phase_path(mode):
    # low-dim MLP policy with B > 256: the multi-workgroup phase sequence
    pinned_live(ppo_config(B=1024, T=50, mode=mode, use_z_filter=True), 17, 6, iters=2, seed=4)


def test_pinned_c2_early_stop():
    lc = ppo_config(B=64, T=20, mode='adapt', use_z_filter=True, lr=(3e-2, 1e-3),
                    kl_target=0.002)
    rep = pinned_live(lc, 17, 6, iters=2, seed=3)
    assert rep


@pytest.mark.parametrize('layers,Hd', [(2, 100), (3, 24)])
def test_pinned_stacked_lstm(layers, Hd):
    # nn.LSTM(num_layers = rnn_layer) (ppo_net.py:146-149)
    lc = ppo_config(B=64, T=10, mode='adapt', use_z_filter=True, hidden=(64, 64), lam=1.0,
                    epochs=(3, 3), rnn=True, rnn_hidden=Hd, horizon=3, rnn_layer=layers)
    pinned_live(lc, 42, 8, iters=2, rnn_hidden=Hd, seed=8 + layers, n_ulp=16)


def test_host_path_reference_unit_test_shape():
    # BASELINE configs[0]: the reference's --unit-test settings
    # (main/ppo_configs.py:225-227: batch 2) on the default PPO config
    lc = copy.deepcopy(PPO_DEFAULT_LEARNER_CONFIG)
    lc.replay.batch_size = 2
    lc.replay.sampling_start_size = 2
    pinned_live(lc, 17, 6, iters=3, rnn_hidden=100, seed=5, source='host')


@pytest.mark.parametrize('mode', ['clip', 'adapt'])
def test_host_path_c2(mode):
    pinned_live(ppo_config(B=64, T=50, mode=mode, use_z_filter=True), 17, 6, iters=2, seed=6,
                source='host')


def test_host_path_pixel_lstm():
    lc = ppo_config(B=3, T=6, mode='adapt', use_z_filter=True, hidden=(16, 16), lam=1.0,
                    epochs=(2, 2), rnn=True, rnn_hidden=12, horizon=2, cnn_feat=16)
    pinned_live(lc, 5, 2, iters=2, pixel=(3, 84, 84), rnn_hidden=12, seed=7, source='host')


# --------------------------------------------------------- fixture cases
def fixture_learner(case, dp=None):
    meta, fx = P.load_fixture(case)
    c = P.CASES[case]
    lc = c['cfg']()
    st = P.init_state(case)
    assert P.digest([st[k] for k in sorted(st)]) == meta['init_digest'], 'initial weights differ'
    if dp is not None:
        lc.replay.batch_size //= dp.world_size
    learner = PPOLearner(lc, _env(c['D'], c['A'], c['pixel']), seed=0, device=DEV, dp=dp)
    P.load_state_into_learner(learner, st)
    learner.export_advantages = True
    return meta, fx, c, st, learner


def check_fixture_state(meta, fx, st, it, fin, adv, ret, zf, report, tag=''):
    for name in ('adv', 'ret'):
        r, w, sc = P.truth(meta, fx, name, it, st)
        P.check(f'{name}{tag}@{it}', adv if name == 'adv' else ret, r, w, sc, report)
    for k in ('actor', 'critic', 'lstm', 'cnn'):
        if f'{k}@{it}' in fx:
            r, w, sc = P.truth(meta, fx, k, it, st)
            P.check(f'{k}{tag}@{it}', fin[k], r, w, sc, report)
            # the update itself (GPU - init vs fp64 - init): relative L2 over the
            # entries the fp64 update moved and the cosine, on bars that a frozen
            # or mis-stepped tensor cannot meet (tests/parity.py update_metrics)
            w_rel, w_cos, thr, _ = meta['update'][f'{k}@{it}']
            st0 = np.asarray(st[k], dtype=np.float64)
            P.check_update(f'{k}{tag}@{it}', np.asarray(fin[k], np.float64) - st0,
                           fx[f'{k}@{it}'].astype(np.float64), thr, w_rel, w_cos, report)
    for b, v in zip(('running_sum', 'running_sumsq'), zf[:2]):
        r, w, sc = P.truth(meta, fx, f'zf_{b}', it, st)
        P.check(f'zf_{b}{tag}@{it}', v, r, w, sc, report)


def pinned_fixture(case):
    meta, fx, c, st, learner = fixture_learner(case)
    lc = learner.learner_config
    report = {}
    for it in range(len(c['batch_seeds'])):
        batch = P.case_batch(case, it)
        assert P.batch_digest(batch) == meta['batch_digest'][it], 'synthetic batch differs'
        cap = P.learn_capture(learner, synthetic.to_device(batch, DEV))
        s = learner.last_stats()
        assert s['epochs_run'] == meta['epochs_run'][it], (s['epochs_run'], meta['epochs_run'][it])
        adv, ret = _used(learner)
        check_fixture_state(meta, fx, st, it, cap['final'], adv, ret, cap['final']['zf'], report)
        _check_stats(lc, c['D'], c['A'], c['pixel'], oracle_batch(batch), cap, learner, report,
                     f'@{it}')
    P.print_report(report, case)


@pytest.mark.timeout(300)
def test_pinned_c3_full_batch_adapt():
    # the exact workload bench.py --config c3 times (1024 segments, 10 + 10 epochs)
    pinned_fixture('c3_adapt')


@pytest.mark.timeout(300)
def test_pinned_c3_full_batch_clip():
    pinned_fixture('c3_clip')


@pytest.mark.timeout(300)
def test_pinned_c3_rank_of_eight():
    # bench.py --config c3 --local-segments 128: one rank's share of the C3 job at
    # N = 8 (the VALU LSTM recurrence, the adaptive dW split), 10 + 10 epochs
    pinned_fixture('c3_l128')


@pytest.mark.timeout(300)
def test_pinned_c5_full_batch():
    # bench.py --config c5 --local-segments 128: C3 + camera0 3x84x84 -> CNN (FC 256)
    pinned_fixture('c5')


@pytest.mark.timeout(300)
def test_pinned_c5_short():
    # C5 at 2 + 2 epochs: the pixel stem's update pinned on tight bars (the
    # 10 + 10 fixture needs a raised relative-L2 mask, tests/parity.py)
    pinned_fixture('c5_short')


def gpu_first_step_grads(learner, phase):
    """the raw gradient a backward phase left in the exchange buffer:
    [actor head | lstm | cnn] then [critic head | lstm | cnn]"""
    xbuf = learner._bufs['rnn_xbuf'].cpu().double().numpy()
    m = learner.model
    nAh, nCh = m.actor.flat.numel(), m.critic.flat.numel()
    nL = m.rnn_stem.flat.numel() if learner.if_rnn_policy else 0
    nCnn = m.cnn_stem.flat.numel() if learner.if_pixel_input else 0
    off, head = (0, 'actor') if phase == 'policy' else (nAh + nL + nCnn, 'critic')
    nh = nAh if phase == 'policy' else nCh
    out = {head: xbuf[off:off + nh]}
    if nL:
        out['lstm'] = xbuf[off + nh:off + nh + nL]
    if nCnn:
        out['cnn'] = xbuf[off + nh + nL:off + nh + nL + nCnn]
    return out


@pytest.mark.timeout(300)
@pytest.mark.parametrize('case', ['c3_grad_policy', 'c3_grad_value', 'c3_l128_grad_policy',
                                  'c3_l128_grad_value', 'c5_grad_policy', 'c5_grad_value'])
def test_pinned_first_step_gradients(case):
    """Raw gradients of the first policy update (epochs 1 + 0) or the first
    value update (0 + 1) before any Adam amplification: the per-step accuracy
    of the forward, loss, head backward, BPTT, CNN backward and the weight-
    gradient GEMMs, at the full C3 batch (21504 rows) and at C5 widths."""
    meta, fx, c, st, learner = fixture_learner(case)
    batch = P.case_batch(case, 0)
    assert P.batch_digest(batch) == meta['batch_digest'][0]
    learner.learn(synthetic.to_device(batch, DEV))
    got = gpu_first_step_grads(learner, c['grad'])
    report = {}
    for k, v in got.items():
        r, w, sc = P.truth(meta, fx, f'grad_{k}', 0, st)
        P.check(f'grad_{k}', v, r, w, sc, report)
    P.print_report(report, case)


# ------------------------------------------------------ staging (a2 / f2)
def test_staging_arena_single_copy_bit_exact():
    """The arena's device tensors equal torch.as_tensor(x, float32) of every
    aggregated array (uint8 camera frames unchanged), over several batches
    with slot reuse."""
    B, T, D, A, Hd, pix = 5, 7, 9, 3, 10, (3, 16, 16)
    spec = {'low_dim': {'flat_inputs': (D,)}, 'pixel': {'camera0': pix}}
    ec = gym_env_config(D, A)
    from surreal_amd.aggregator import MultistepAggregatorWithInfo
    agg = MultistepAggregatorWithInfo(spec, ec.action_spec)
    arena = StagingArena(DEV)
    for it in range(5):
        host = agg.aggregate(AR.make_ppo_exp_list(
            AR.ppo_exp_arrays(B, T, D, A, it, rnn_hidden=Hd, pixel=pix)))
        dev = arena.stage(host)
        torch.cuda.synchronize()
        pairs = [(dev['obs']['low_dim']['flat_inputs'], host['obs']['low_dim']['flat_inputs']),
                 (dev['obs_next']['low_dim']['flat_inputs'], host['obs_next']['low_dim']['flat_inputs']),
                 (dev['actions'], host['actions']), (dev['rewards'], host['rewards']),
                 (dev['dones'], host['dones']), (dev['persistent_infos'][0], host['persistent_infos'][0]),
                 (dev['onetime_infos'][0], host['onetime_infos'][0]),
                 (dev['onetime_infos'][1], host['onetime_infos'][1])]
        for d, h in pairs:
            assert d.dtype == torch.float32 and d.is_cuda
            assert torch.equal(d.cpu(), torch.as_tensor(h, dtype=torch.float32))
        for k in ('obs', 'obs_next'):
            d, h = dev[k]['pixel']['camera0'], host[k]['pixel']['camera0']
            assert d.dtype == torch.uint8 and torch.equal(d.cpu(), torch.as_tensor(h))
        np.testing.assert_equal(dev['dones'].cpu().numpy(), np.asarray(host['dones'], np.float32))
