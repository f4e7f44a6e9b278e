"""Diagnostic (GPU box): raw gradients of one policy + one value update at C3
widths, GPU vs oracle fp32 vs oracle fp64, per parameter tensor.
Prints max|g - g64| / max|g64| for the GPU and for CPU fp32, and the share of
entries whose relative error exceeds 1e-4."""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from oracle import ppo_ref as R  # noqa: E402
from surreal_amd import synthetic  # noqa: E402
from surreal_amd.learner import PPOLearner  # noqa: E402
from tests.helpers import copy_weights_to_oracle, env_config, oracle_batch, ppo_config  # noqa: E402


def main(B=1024, mode='adapt', phase='policy'):
    T, H, D, A, Hd = 25, 5, 42, 8, 100
    lc = ppo_config(B=B, T=T, mode=mode, use_z_filter=True, hidden=(300, 200), lam=1.0,
                    epochs=(1, 0) if phase == 'policy' else (0, 1), rnn=True, rnn_hidden=Hd, horizon=H)
    learner = PPOLearner(lc, env_config(D, A), seed=9)
    refs = []
    for dt in (torch.float32, torch.float64):
        r = R.PPOLearnerRef(lc, D, A, dtype=dt)
        copy_weights_to_oracle(learner, r)
        refs.append(r)
    batch = synthetic.ppo_batch(B, T, D, A, seed=1, rnn_hidden=Hd)
    for r in refs:
        r.learn(oracle_batch(batch))
    learner.learn(synthetic.to_device(batch, 'cuda'))
    xbuf = learner._bufs['rnn_xbuf'].cpu().double()
    nAh = learner.model.actor.flat.numel()
    nL = learner.model.rnn_stem.flat.numel()
    nCh = learner.model.critic.flat.numel()
    gpu = {'actor': xbuf[:nAh], 'lstm_pol': xbuf[nAh:nAh + nL],
           'critic': xbuf[nAh + nL:nAh + nL + nCh], 'lstm_val': xbuf[nAh + nL + nCh:nAh + nL + nCh + nL]}

    def grads(r):
        m = r.model
        f = lambda ps: torch.cat([p.grad.detach().reshape(-1) for p in ps]).double()  # noqa: E731
        lstm = [m.rnn_stem.weight_ih_l0, m.rnn_stem.weight_hh_l0, m.rnn_stem.bias_ih_l0,
                m.rnn_stem.bias_hh_l0]
        return {'actor': f(list(m.actor.model.parameters()) + [m.actor.log_var]) if phase == 'policy' else None,
                'critic': f(m.critic.model.parameters()) if phase != 'policy' else None,
                'lstm_pol': f(lstm), 'lstm_val': f(lstm)}
    g32, g64 = grads(refs[0]), grads(refs[1])
    h1, h2 = 300, 200

    def parts(name):
        if name.startswith('lstm'):
            return [('W_ih', 4 * Hd * D), ('W_hh', 4 * Hd * Hd), ('b_ih', 4 * Hd), ('b_hh', 4 * Hd)]
        out = A if name == 'actor' else 1
        p = [('W1', h1 * Hd), ('b1', h1), ('W2', h2 * h1), ('b2', h2), ('W3', out * h2), ('b3', out)]
        return p + ([('log_var', A)] if name == 'actor' else [])
    for name in (('actor', 'lstm_pol') if phase == 'policy' else ('critic', 'lstm_val')):
        o = 0
        for pn, n in parts(name):
            a, b, c = gpu[name][o:o + n], g32[name][o:o + n], g64[name][o:o + n]
            sc = float(c.abs().max())
            eg = (a - c).abs()
            ec = (b - c).abs()
            rel_g = (eg / (c.abs() + 1e-12))
            rel_c = (ec / (c.abs() + 1e-12))
            print(f'{name:9s} {pn:8s} n={n:7d} scale={sc:.3e}  gpu {float(eg.max()) / sc:.2e} '
                  f'cpu32 {float(ec.max()) / sc:.2e}   elems rel>1e-4: gpu {float((rel_g > 1e-4).double().mean()):.4f} '
                  f'cpu32 {float((rel_c > 1e-4).double().mean()):.4f}')
            o += n


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1024, sys.argv[2] if len(sys.argv) > 2 else 'adapt',
         sys.argv[3] if len(sys.argv) > 3 else 'policy')
