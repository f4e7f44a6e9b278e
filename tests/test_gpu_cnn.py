"""Pixel stem (CNNStemNetwork, surreal/model/model_builders/builders.py:8-33,
applied to obs/255 by ppo_net.py:268-275,368-375) on the HIP kernels.

* u8 scaling: the fused /255 is bit-equal to torch's uint8 / 255.0 for all 256
  values (one-hot conv-1 filter makes conv-1 outputs the scaled pixels).
* smi_cnn_forward / smi_cnn_backward vs torch.nn.Conv2d/Linear on CPU in fp32
  and fp64 (the same GEMM parity bar as test_gpu_ddpg.py), including the
  time-major row -> (pix[b][t] | pix_next[b]) mapping the learner uses and a
  row count that makes workgroups loop over several images.
* PPOModel forward with camera + low-dim + LSTM vs the oracle model.
* PPOLearner.learn() with pixels + LSTM (SURVEY C5 structure, reduced widths)
  vs oracle.PPOLearnerRef: clip/adapt, with and without low-dim observations.
"""
import numpy as np
import pytest
import torch

from oracle import ppo_ref as R
from surreal_amd import _lib as L
from surreal_amd import synthetic
from surreal_amd.config import pixel_env_config
from surreal_amd.learner import PPOLearner
from surreal_amd.model import PPOModel
from tests.helpers import (copy_weights_to_oracle, load_lstm_flat, load_seq_flat, lstm_flat,
                           oracle_batch, ppo_config, seq_flat)
from tests.test_gpu_ddpg import _fp32_as_good_as_torch
from tests.test_gpu_ppo import _compare_params

pytestmark = pytest.mark.gpu
DEV = 'cuda'
CAM = (3, 84, 84)


def _geom(C, H, W):
    H1, W1 = (H - 8) // 4 + 1, (W - 8) // 4 + 1
    H2, W2 = (H1 - 4) // 2 + 1, (W1 - 4) // 2 + 1
    return H1, W1, H2, W2


def _run_fwd(flat, pix, pixn, B, T, rows, F, with_a1=True):
    C, H, W = CAM
    H1, W1, H2, W2 = _geom(C, H, W)
    a1 = torch.empty(rows, 16, H1 * W1, device=DEV) if with_a1 else None
    a2 = torch.empty(rows, 32 * H2 * W2, device=DEV)
    feat = torch.empty(rows, F, device=DEV)
    L.call('smi_cnn_forward', L.ptr(flat), L.ptr(pix), L.ptr(pixn) if pixn is not None else None,
           B, T, rows, C, H, W, F, L.ptr(a1) if with_a1 else None, L.ptr(a2), L.ptr(feat), F,
           L.stream())
    return a1, a2, feat


def test_u8_scaling_bit_exact():
    C, H, W = CAM
    F = 8
    net = R.cnn_stem_ref(C, H, W, F)
    with torch.no_grad():
        for p in net.parameters():
            p.zero_()
        net[0].weight[:, 0, 0, 0] = 1.0            # conv-1 output = scaled pixel (0, 4oy, 4ox)
    flat = seq_flat(net).to(DEV)
    H1, W1, _, _ = _geom(C, H, W)
    img = torch.zeros(1, C, H, W, dtype=torch.uint8)
    vals = torch.arange(H1 * W1) % 256
    img[0, 0, 0:4 * H1:4, 0:4 * W1:4] = vals.reshape(H1, W1).to(torch.uint8)
    pix = img.to(DEV)
    a1, _, _ = _run_fwd(flat, pix, None, 1, 1, 1, F)
    got = a1[0, 0].cpu()
    exp = vals.to(torch.uint8) / 255.0
    assert torch.equal(got, exp), (got - exp).abs().max()


def _images(B, T, seed):
    g = torch.Generator().manual_seed(seed)
    pix = torch.randint(0, 256, (B, T) + CAM, generator=g, dtype=torch.uint8)
    pixn = torch.randint(0, 256, (B, 1) + CAM, generator=g, dtype=torch.uint8)
    return pix, pixn


def _timemajor_images(pix, pixn, S):
    B, T = pix.shape[:2]
    rows = [pix[:, t] if t < T else pixn[:, 0] for t in range(S)]
    return torch.stack(rows, 0).reshape(S * B, *CAM)


@pytest.mark.parametrize('B,T,S,F', [(5, 7, 8, 256), (3, 2, 2, 40), (24, 25, 26, 256)])
def test_cnn_forward_backward_vs_torch(B, T, S, F):
    C, H, W = CAM
    torch.manual_seed(B * 100 + S)
    net = R.cnn_stem_ref(C, H, W, F)
    net64 = R.cnn_stem_ref(C, H, W, F).double()
    net64.load_state_dict({k: v.double() for k, v in net.state_dict().items()})
    flat = seq_flat(net).to(DEV)
    pix, pixn = _images(B, T, S)
    rows = S * B
    x = _timemajor_images(pix, pixn, S)
    pix_d, pixn_d = pix.to(DEV), pixn.to(DEV)      # kept alive until the kernels ran
    a1, a2, feat = _run_fwd(flat, pix_d, pixn_d, B, T, rows, F)
    # torch reference (CPU): activations of each stage
    xs = x / 255.0
    r1 = torch.relu(net[0](xs))
    r2 = torch.relu(net[2](r1))
    out = net(xs)
    xs64 = x.double() / 255.0
    r1_64 = torch.relu(net64[0](xs64))
    r2_64 = torch.relu(net64[2](r1_64))
    out64 = net64(xs64)
    _fp32_as_good_as_torch(a1.cpu().reshape(r1.shape), r1.detach(), r1_64.detach(), 2e-6)
    _fp32_as_good_as_torch(a2.cpu(), r2.detach().reshape(rows, -1),
                           r2_64.detach().reshape(rows, -1), 2e-6)
    _fp32_as_good_as_torch(feat.cpu(), out.detach(), out64.detach(), 2e-6)
    # backward of sum(out * dy): dz = dy * relu'(out).  The reference backward
    # uses the GPU forward's ReLU masks (A1 > 0, A2 > 0): a pre-activation
    # within fp32 noise of 0 may take either side in any two implementations,
    # and the backward is exactly linear given the masks.
    g = torch.Generator().manual_seed(7)
    dy = torch.randn(rows, F, generator=g)
    dz = (dy * (out.detach() > 0)).contiguous()
    dz_d = dz.to(DEV)
    nbytes = int(L.lib().smi_cnn_scratch_bytes(rows, C, H, W, F))
    scratch = torch.empty(nbytes // 4 + 1, device=DEV)
    grad = torch.full_like(flat, float('nan'))
    L.call('smi_cnn_backward', L.ptr(flat), L.ptr(pix_d), L.ptr(pixn_d), B, T, rows,
           C, H, W, F, L.ptr(a1), L.ptr(a2), L.ptr(dz_d), F, L.ptr(grad), L.ptr(scratch), nbytes,
           L.stream())
    m1 = (a1.cpu().reshape(r1.shape) > 0)
    m2 = (a2.cpu() > 0)

    def masked_grads(model, dt):
        model.zero_grad()
        z1 = model[0](x.to(dt) / 255.0) * m1.to(dt)
        z2 = model[2](z1).reshape(rows, -1) * m2.to(dt)
        (model[5](z2) * dz.to(dt)).sum().backward()
        return [p.grad.detach() for p in model.parameters()]

    g32 = masked_grads(net, torch.float32)
    g64 = masked_grads(net64, torch.float64)
    got = grad.cpu()
    o = 0
    for a32, a64 in zip(g32, g64):
        n = a32.numel()
        _fp32_as_good_as_torch(got[o:o + n].reshape(a32.shape), a32, a64, 4e-6)
        o += n
    assert o == got.numel()


def _pixel_cfg(mode, B, T, H, Hd, hidden, F, zf=True, epochs=(10, 10), lr=(3e-4, 3e-4), rnn=True):
    return ppo_config(B=B, T=T, mode=mode, use_z_filter=zf, hidden=hidden, lam=1.0 if rnn else 0.95,
                      epochs=epochs, rnn=rnn, rnn_hidden=Hd, horizon=H, lr=lr, cnn_feat=F)


def test_ppo_model_pixel_forward_vs_oracle():
    B, S, D, A, Hd, F = 6, 4, 7, 3, 16, 32
    lc = _pixel_cfg('adapt', B, S, 2, Hd, (16, 16), F)
    ec = pixel_env_config(D, A, CAM)
    m = PPOModel(ec.obs_spec, A, lc.model, True, -1.0, True, True, lc.algo.rnn, DEV,
                 torch.Generator().manual_seed(1))
    ref = R.PPOModelRef(D, A, [16, 16], [16, 16], -1.0, True, True, Hd, 1, CAM, F)
    ref.actor.load_flat(m.actor.flat.cpu())
    ref.critic.load_flat(m.critic.flat.cpu())
    load_lstm_flat(ref.rnn_stem, m.rnn_stem.flat.cpu())
    load_seq_flat(ref.cnn_stem, m.cnn_stem.flat.cpu())
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, S, D, generator=g)
    with torch.no_grad():
        m.z_filter.running_sum.copy_(torch.randn(D, generator=g).to(DEV))
        m.z_filter.running_sumsq.copy_((torch.rand(D, generator=g) * 5 + 3).to(DEV))
        m.z_filter.count.fill_(2.0)
    ref.z_filter.load_state_dict({k: v.cpu() for k, v in m.z_filter.state_dict().items()})
    pix, _ = _images(B, S, 5)
    h0 = 0.1 * torch.randn(1, B, Hd, generator=g)
    c0 = 0.1 * torch.randn(1, B, Hd, generator=g)
    obs = {'low_dim': {'flat_inputs': x.to(DEV)}, 'pixel': {'camera0': pix.to(DEV)}}
    got_a = m.forward_actor(obs, (h0.to(DEV), c0.to(DEV))).cpu()
    got_c = m.forward_critic(obs, (h0.to(DEV), c0.to(DEV))).cpu()
    exp_a = ref.forward_actor((x, pix), (h0, c0)).detach()
    exp_c = ref.forward_critic((x, pix), (h0, c0)).detach()
    assert got_a.shape == exp_a.shape and got_c.shape == exp_c.shape
    assert float((got_a - exp_a).abs().max()) <= 1e-5 * float(exp_a.abs().max()) + 1e-6
    assert float((got_c - exp_c).abs().max()) <= 1e-5 * float(exp_c.abs().max()) + 1e-6


def _run_pixel(mode, B, T, H, D, A, Hd, hidden, F, iters=2, zf=True, epochs=(10, 10),
               lr=(3e-4, 3e-4), rnn=True):
    lc = _pixel_cfg(mode, B, T, H, Hd, hidden, F, zf and D > 0, epochs, lr, rnn)
    ec = pixel_env_config(D, A, CAM)
    learner = PPOLearner(lc, ec, seed=9)
    ref = R.PPOLearnerRef(lc, D, A, pixel=CAM)
    copy_weights_to_oracle(learner, ref)
    report = {}
    for it in range(iters):
        batch = synthetic.ppo_batch(B, T, D, A, seed=50 + it, rnn_hidden=Hd if rnn else None,
                                    pixel=CAM)
        rstats = ref.learn(oracle_batch(batch))
        learner.learn(synthetic.to_device(batch, DEV))
        stats = learner.last_stats()
        assert stats['epochs_run'] == rstats['epochs_run'], (it, stats['epochs_run'],
                                                             rstats['epochs_run'])
        keys = ['_surr_loss', '_entropy', '_pol_kl', '_val_loss', '_avg_return_targ',
                '_avg_behave_likelihood', '_avg_is_weight', '_ref_behave_diff', 'grad_norm_actor',
                'grad_norm_critic', '_avg_log_sig']
        keys += ['_clip_surr_loss'] if mode == 'clip' else ['_kl_loss_adapt']
        for k in keys:
            assert abs(stats[k] - rstats[k]) <= 2e-4 * abs(rstats[k]) + 2e-6, (it, k, stats[k],
                                                                               rstats[k])
        ups = rstats['epochs_run']
        _compare_params(f'actor{it}', learner.model.actor.flat.cpu(), ref.model.actor.flat(),
                        lr[0], ups, report)
        _compare_params(f'critic{it}', learner.model.critic.flat.cpu(), ref.model.critic.flat(),
                        lr[1], epochs[1], report)
        if rnn:
            _compare_params(f'lstm{it}', learner.model.rnn_stem.flat.cpu(),
                            lstm_flat(ref.model.rnn_stem), max(lr), ups + epochs[1], report)
        # CNN stem: more entries whose gradient cancels to rounding noise (FC
        # weights of units alive in a handful of rows), which Adam's first steps
        # normalise to +-lr in either implementation; the raw gradients are held
        # to 1e-4 of scale by test_pixel_rnn_gradients_match_autograd
        _compare_params(f'cnn{it}', learner.model.cnn_stem.flat.cpu(), seq_flat(ref.model.cnn_stem),
                        max(lr), ups + epochs[1], report, max_frac=5e-3)
    return report


# Pixel learn() parity is asserted over a few epochs of one learn(): beyond
# that, ReLU-mask flips of pre-activations within fp32 noise of 0 plus Adam's
# sign-normalised steps make ANY two fp32 implementations drift apart by ~lr
# per affected entry (tools/dbg_px.py).  Raw gradients are held
# to 1e-4 of scale by test_pixel_rnn_gradients_match_autograd.
@pytest.mark.parametrize('mode', ['clip', 'adapt'])
def test_pixel_rnn_learn_matches_oracle(mode):
    rep = _run_pixel(mode, B=6, T=6, H=2, D=7, A=3, Hd=16, hidden=(16, 16), F=32, iters=1,
                     epochs=(3, 3))
    print('pixel rnn parity:', rep)


def test_pixel_only_rnn_learn_matches_oracle():
    # pixel-only: the LSTM sees CNN features alone, so entries whose gradient is
    # ~Adam eps (1e-8) dominate the drift from the second step on
    # (tools/dbg_px2.py); one policy and one value update are asserted
    rep = _run_pixel('adapt', B=5, T=5, H=2, D=0, A=2, Hd=12, hidden=(16, 16), F=24, iters=1,
                     epochs=(1, 1))
    print('pixel-only rnn parity:', rep)


def test_pixel_rnn_c5_widths_one_update():
    # SURVEY C5 widths (camera 3x84x84, FC 256, LSTM 100 over low-dim 42 + 256,
    # heads 300x200, A 8, T 25, horizon 5) at 16 segments; one policy and one
    # value update (the Adam-amplification argument of test_gpu_rnn.py).
    rep = _run_pixel('adapt', B=16, T=25, H=5, D=42, A=8, Hd=100, hidden=(300, 200), F=256,
                     iters=1, epochs=(1, 1))
    print('pixel rnn C5-widths parity:', rep)


@pytest.mark.parametrize('rnn', [True, False])
def test_pixel_gradients_match_autograd(rnn):
    """Raw gradients of the last value update (before Adam) vs the oracle's
    autograd at C5 widths: critic head, LSTM (rnn) and CNN stem; rnn=False is
    the non-RNN pixel model (heads over [zfilter(low_dim) | cnn])."""
    B, T, D, A, F = 16, 25, 42, 8, 256
    H, Hd = (5, 100) if rnn else (25, 0)
    lc = _pixel_cfg('adapt', B, T, H, Hd, (300, 200), F, epochs=(1, 1), rnn=rnn)
    learner = PPOLearner(lc, pixel_env_config(D, A, CAM), seed=9)
    ref = R.PPOLearnerRef(lc, D, A, pixel=CAM)
    copy_weights_to_oracle(learner, ref)
    batch = synthetic.ppo_batch(B, T, D, A, seed=1, rnn_hidden=Hd if rnn else None, pixel=CAM)
    ref.learn(oracle_batch(batch))
    learner.learn(synthetic.to_device(batch, DEV))
    xbuf = learner._bufs['rnn_xbuf'].cpu().double()
    nAh = learner.model.actor.flat.numel()
    nL = learner.model.rnn_stem.flat.numel() if rnn else 0
    nK = learner.model.cnn_stem.flat.numel()
    nCh = learner.model.critic.flat.numel()
    o = nAh + nL + nK
    g_critic = xbuf[o:o + nCh]
    g_lstm = xbuf[o + nCh:o + nCh + nL]
    g_cnn = xbuf[o + nCh + nL:o + nCh + nL + nK]

    def flat_grad(ps):
        return torch.cat([p.grad.detach().reshape(-1) for p in ps]).double()
    rc = flat_grad(ref.model.critic.model.parameters())
    rk = flat_grad(ref.model.cnn_stem.parameters())
    checks = [('critic', g_critic, rc), ('cnn', g_cnn, rk)]
    if rnn:
        rl = flat_grad([ref.model.rnn_stem.weight_ih_l0, ref.model.rnn_stem.weight_hh_l0,
                        ref.model.rnn_stem.bias_ih_l0, ref.model.rnn_stem.bias_hh_l0])
        checks.append(('lstm', g_lstm, rl))
    for name, got, exp in checks:
        scale = float(exp.abs().max())
        err = (got - exp).abs()
        print(name, 'max abs err / scale', float(err.max()) / scale,
              'frac > 1e-5 scale', float((err > 1e-5 * scale).double().mean()))
        assert float(err.max()) <= 1e-4 * scale, name


@pytest.mark.parametrize('mode', ['clip', 'adapt'])
def test_pixel_mlp_learn_matches_oracle(mode):
    # non-RNN pixel model (ppo_net.py:155-166: heads over [zfilter(low_dim) | cnn]),
    # ppo.py's non-RNN branch: one GAE window of n_step, step 0 trains
    # (with one training row per segment the CNN gradients sum few terms; the
    # raw gradients are held to 1e-4 of scale by the autograd test below)
    rep = _run_pixel(mode, B=24, T=6, H=6, D=7, A=3, Hd=0, hidden=(32, 24), F=32, iters=1,
                     epochs=(1, 1), rnn=False)
    print('pixel mlp parity:', rep)
