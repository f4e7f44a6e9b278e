"""Diagnostic (GPU box): is the reference-policy forward (PREP phase) bitwise
equal to the learner's first policy forward (POLICY_FWD, epoch 0) when the
two models are identical?  (The reference computes both with the same torch
code, so its KL gradient at epoch 0 is exactly zero.)  Reads the RNN scratch
regions refmu and OUT (carve order of ppo_rnn.hip rnn_scratch)."""
import sys

import torch

sys.path.insert(0, '.')
from surreal_amd import synthetic  # noqa: E402
from surreal_amd.learner import PPOLearner  # noqa: E402
from tests.helpers import env_config, ppo_config  # noqa: E402


def al64(n):
    return (n + 63) & ~63


def main(B=64, zf=True):
    T, H, D, A, Hd, h1, h2 = 25, 5, 42, 8, 100, 300, 200
    lc = ppo_config(B=B, T=T, mode='adapt', use_z_filter=zf, hidden=(h1, h2), lam=1.0,
                    epochs=(0, 0), rnn=True, rnn_hidden=Hd, horizon=H)
    learner = PPOLearner(lc, env_config(D, A), seed=8)
    batch = synthetic.to_device(synthetic.ppo_batch(B, T, D, A, seed=1, rnn_hidden=Hd), 'cuda')
    learner.learn(batch)
    torch.cuda.synchronize()
    s = learner._bufs['rnn_scratch']
    E, S1 = T - H + 1, T + 1
    NE, NG, G4 = E * B, S1 * B, 4 * Hd
    sizes = [('Xz', NG * D), ('Xr', NE * D), ('xproj', NG * G4), ('hbuf', (S1 + 1) * B * Hd),
             ('cbuf', (E + 1) * B * Hd), ('gates', NE * G4), ('HA1', NG * h1), ('HA2', NG * h2),
             ('OUT', NG * A), ('dOUT', NE * A), ('dH1', NE * h1), ('dH2', NE * h2), ('dh', NE * Hd),
             ('dgates', NE * G4), ('values', B * S1), ('adv', NE), ('ret', NE), ('refmu', NE * A)]
    off, reg = 0, {}
    for n, k in sizes:
        reg[n] = (off, k)
        off += al64(k)
    o, k = reg['OUT']
    out = s[o:o + NE * A].cpu()
    o, k = reg['refmu']
    ref = s[o:o + k].cpu()
    d = (out - ref).abs()
    print(f'B={B} zf={zf}: refmu vs learner mu: max |diff| {float(d.max()):.3e}, '
          f'entries differing {int((d > 0).sum())}/{d.numel()}')


if __name__ == '__main__':
    main(64, True)
    main(64, False)
