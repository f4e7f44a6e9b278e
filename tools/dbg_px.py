"""Developer tool: raw last-value-update gradients (critic / lstm / cnn) vs the
oracle's autograd for pixel+LSTM configs over several epoch counts."""
import sys
import torch
sys.path.insert(0, '/root/repo')
from oracle import ppo_ref as R  # noqa: E402
from surreal_amd import synthetic  # noqa: E402
from surreal_amd.config import pixel_env_config  # noqa: E402
from surreal_amd.learner import PPOLearner  # noqa: E402
from tests import test_gpu_cnn as TC  # noqa: E402
from tests.helpers import copy_weights_to_oracle, oracle_batch, lstm_flat, seq_flat  # noqa: E402

CAM = (3, 84, 84)


def run(B, T, H, D, A, Hd, hidden, F, epochs, zf=True):
    lc = TC._pixel_cfg('adapt', B, T, H, Hd, hidden, F, zf, epochs)
    learner = PPOLearner(lc, pixel_env_config(D, A, CAM), seed=9)
    ref = R.PPOLearnerRef(lc, D, A, pixel=CAM)
    copy_weights_to_oracle(learner, ref)
    batch = synthetic.ppo_batch(B, T, D, A, seed=50, rnn_hidden=Hd, pixel=CAM)
    rst = ref.learn(oracle_batch(batch))
    learner.learn(synthetic.to_device(batch, 'cuda'))
    xbuf = learner._bufs['rnn_xbuf'].cpu().double()
    nAh = learner.model.actor.flat.numel()
    nL = learner.model.rnn_stem.flat.numel()
    nK = learner.model.cnn_stem.flat.numel()
    nCh = learner.model.critic.flat.numel()
    o = nAh + nL + nK
    segs = {'critic': xbuf[o:o + nCh], 'lstm': xbuf[o + nCh:o + nCh + nL],
            'cnn': xbuf[o + nCh + nL:o + nCh + nL + nK]}
    fg = lambda ps: torch.cat([p.grad.detach().reshape(-1) for p in ps]).double()  # noqa: E731
    refs = {'critic': fg(ref.model.critic.model.parameters()),
            'lstm': fg([ref.model.rnn_stem.weight_ih_l0, ref.model.rnn_stem.weight_hh_l0,
                        ref.model.rnn_stem.bias_ih_l0, ref.model.rnn_stem.bias_hh_l0]),
            'cnn': fg(ref.model.cnn_stem.parameters())}
    out = {}
    for k in segs:
        sc = float(refs[k].abs().max())
        out[k] = round(float((segs[k] - refs[k]).abs().max()) / sc, 8)
    pe = {}
    for k, got, exp in (('critic', learner.model.critic.flat.cpu(), ref.model.critic.flat()),
                        ('lstm', learner.model.rnn_stem.flat.cpu(), lstm_flat(ref.model.rnn_stem)),
                        ('cnn', learner.model.cnn_stem.flat.cpu(), seq_flat(ref.model.cnn_stem))):
        pe[k] = round(float((got.double() - exp.double()).abs().max()), 8)
    print(epochs, 'grad err/scale', out, 'param max abs diff', pe, 'runs', rst['epochs_run'],
          flush=True)


base = dict(B=24, T=10, H=3, D=17, A=6, Hd=40, hidden=(32, 48), F=32)
for ep in ((1, 1), (1, 2), (1, 3), (1, 10), (2, 1), (10, 1)):
    run(epochs=ep, **base)
run(epochs=(1, 2), zf=False, **base)
