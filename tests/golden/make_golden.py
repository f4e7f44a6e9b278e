"""Generates the committed golden fixtures of tests/golden/.

Nothing here imports or runs the reference (denied: SURVEY.md §8(c)); the
fixtures come from
  * the Python standard library `random` — the generator the reference's
    UniformReplay.sample calls directly (surreal/replay/uniform_replay.py:44);
  * closed-form known answers derived by hand from the reference formulas
    (SURVEY.md §8(c) items 1-8), evaluated in float64 numpy.
Run:  python tests/golden/make_golden.py
"""
import json
import math
import os
import random

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def sampler_streams():
    cases = []
    for seed in (0, 1, 2, 12345, 2 ** 40 + 7):
        for n in (1, 2, 3, 1000, 333333):
            random.seed(seed)
            draws = [random.randint(0, n - 1) for _ in range(700)]   # crosses a 624-word twist
            cases.append({'seed': seed, 'n': n, 'draws': draws})
    states = []
    for seed in (0, 2 ** 40 + 7):
        random.seed(seed)
        st = random.getstate()[1]
        states.append({'seed': seed, 'head': list(st[:8]), 'tail': list(st[620:624]),
                       'pos': st[624]})
    return {'generator': 'CPython %s random' % '.'.join(map(str, __import__('sys').version_info[:3])),
            'cases': cases, 'states': states}


def gae_kats():
    """Closed forms of ppo.py:371-418 (float64)."""
    rng = np.random.RandomState(7)
    out = []
    B, T = 4, 6
    # (1) gamma = lam = 1, no dones: adv = sum r + V_T - V_0, ret = sum r + V_T
    r = rng.randn(B, T)
    V = rng.randn(B, T + 1)
    out.append({'name': 'gamma1_lam1', 'gamma': 1.0, 'lam': 1.0, 'B': B, 'T': T,
                'rewards': r.tolist(), 'dones': np.zeros((B, T)).tolist(), 'values': V.tolist(),
                'adv': (r.sum(1) + V[:, T] - V[:, 0]).tolist(),
                'ret': (r.sum(1) + V[:, T]).tolist()})
    # (2) rewards = 0, V == c: td = (g-1)c, adv = (g-1)c sum (g l)^t, ret = c g^T
    g, lam, c = 0.9, 0.8, 1.5
    ks = np.arange(T)
    out.append({'name': 'zero_rewards_const_values', 'gamma': g, 'lam': lam, 'B': B, 'T': T,
                'rewards': np.zeros((B, T)).tolist(), 'dones': np.zeros((B, T)).tolist(),
                'values': np.full((B, T + 1), c).tolist(),
                'adv': [float((g - 1) * c * np.sum((g * lam) ** ks))] * B,
                'ret': [float(c * g ** T)] * B})
    # (3) done at T-1 zeroes the bootstrap value
    r = rng.randn(B, T)
    V = rng.randn(B, T + 1)
    d = np.zeros((B, T)); d[:, T - 1] = 1.0
    Vm = V.copy(); Vm[:, 1:] *= 1 - d
    gl = (g ** ks) * (lam ** ks)
    td = r + g * Vm[:, 1:] - Vm[:, :-1]
    out.append({'name': 'done_last_step', 'gamma': g, 'lam': lam, 'B': B, 'T': T,
                'rewards': r.tolist(), 'dones': d.tolist(), 'values': V.tolist(),
                'adv': (td * gl).sum(1).tolist(),
                'ret': ((g ** ks) * r).sum(1).tolist()})
    return out


def diag_gauss_kats():
    A = 5
    mu = np.linspace(-0.5, 0.5, A)
    sd = np.linspace(0.2, 0.9, A)
    return {
        'A': A, 'mu': mu.tolist(), 'sd': sd.tolist(),
        # loglik at a = mu: -0.5 A log(2 pi) - sum log sd
        'loglik_at_mean': float(-0.5 * A * math.log(2 * math.pi) - np.log(sd).sum()),
        # entropy: 0.5 sum log sd + 0.5 A log(2 pi e)
        'entropy': float(0.5 * np.log(sd).sum() + 0.5 * A * math.log(2 * math.pi * math.e)),
        # KL(p || p) = 0
        'kl_self': 0.0,
        # KL of shifted mean, same std: sum d^2 / (2 sd^2)
        'shift': 0.25,
        'kl_shift': float(np.sum(0.25 ** 2 / (2 * sd ** 2))),
    }


def zfilter_kat():
    # one update with a constant column c over B rows:
    # mean = c B / (B + 1e-5); sumsq = 1e-5 + B c^2
    B, c, eps = 64, 2.0, 1e-5
    count = eps + B
    mean = c * B / count
    var = (eps + B * c * c) / count - mean * mean
    return {'B': B, 'c': c, 'mean': mean, 'var': var, 'count': count}


def adam_kat():
    # one Adam step from zero moments: m_hat = g, v_hat = g^2  ->  p1 = p0 - lr g/(|g| + eps)
    lr, eps = 1e-3, 1e-8
    p0 = np.array([0.5, -0.25, 1.0, 0.0])
    g = np.array([0.1, -2.0, 1e-3, 0.3])
    return {'lr': lr, 'eps': eps, 'p0': p0.tolist(), 'g': g.tolist(),
            'p1': (p0 - lr * g / (np.abs(g) + eps)).tolist()}


def clip_kat():
    # ratio == 1 (learn == behave): clip loss = -mean(adv), surr = -mean(adv)
    adv = np.array([0.5, -1.0, 2.0, 0.25])
    return {'adv': adv.tolist(), 'clip_loss': float(-adv.mean())}


def main():
    with open(os.path.join(HERE, 'sampler_streams.json'), 'w') as f:
        json.dump(sampler_streams(), f)
    kats = {'gae': gae_kats(), 'diag_gauss': diag_gauss_kats(), 'zfilter': zfilter_kat(),
            'adam': adam_kat(), 'clip': clip_kat()}
    with open(os.path.join(HERE, 'known_answers.json'), 'w') as f:
        json.dump(kats, f, indent=1)


if __name__ == '__main__':
    main()
