"""CPU tests: the oracle restatement against the committed golden fixtures
(CPython random streams, hand-derived known answers) — no GPU needed."""
import json
import math
import os

import numpy as np
import torch

from oracle import ppo_ref as R
from oracle import sampler_ref as SR

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_mt19937_oracle_matches_cpython_streams():
    gold = _load('sampler_streams.json')
    for c in gold['cases']:
        draws, words = SR.randint_stream(c['seed'], c['n'], len(c['draws']))
        assert draws.tolist() == c['draws'], (c['seed'], c['n'])
        assert words >= len(c['draws'])
    for s in gold['states']:
        st = SR.seed_state(s['seed'])
        assert st[:8].tolist() == s['head'] and st[620:624].tolist() == s['tail']
        assert int(st[624]) == s['pos']


def test_rejection_consumes_extra_words():
    # n = 3 -> k = 2 bits, r = 3 is rejected: more words than draws
    _, words = SR.randint_stream(0, 3, 700)
    assert words > 700
    # CPython uses k = n.bit_length() (not (n-1).bit_length()): for n = 1024,
    # k = 11 and about half of the words are rejected
    _, words1 = SR.randint_stream(0, 1024, 700)
    assert words1 > 1.5 * 700


def test_gae_oracle_known_answers():
    for case in _load('known_answers.json')['gae']:
        T = case['T']
        v = torch.tensor(case['values']).float()
        r = torch.tensor(case['rewards']).float()
        d = torch.tensor(case['dones']).float()
        adv, ret = R.gae_and_return(v, r, d, case['gamma'], case['lam'], T, T, False, False)
        assert np.allclose(adv.view(-1).numpy(), case['adv'], rtol=1e-5, atol=1e-5), case['name']
        assert np.allclose(ret.view(-1).numpy(), case['ret'], rtol=1e-5, atol=1e-5), case['name']


def test_rnn_window_with_full_horizon_equals_nonrnn():
    # SURVEY §8(c) KAT 4: horizon == T gives E = 1 and the non-RNN formula
    g = torch.Generator().manual_seed(0)
    B, T = 8, 10
    v = torch.randn(B, T + 1, generator=g)
    r = torch.randn(B, T, generator=g)
    d = (torch.rand(B, T, generator=g) < 0.2).float()
    a1, r1 = R.gae_and_return(v.clone(), r, d, 0.99, 0.95, T, T, True, False)
    a2, r2 = R.gae_and_return(v.clone(), r, d, 0.99, 0.95, T, T, False, False)
    assert torch.allclose(a1.view(-1), a2.view(-1), rtol=1e-6, atol=1e-6)
    assert torch.allclose(r1.view(-1), r2.view(-1), rtol=1e-6, atol=1e-6)


def test_diag_gauss_oracle_known_answers():
    k = _load('known_answers.json')['diag_gauss']
    mu, sd = torch.tensor(k['mu']).float(), torch.tensor(k['sd']).float()
    p = torch.cat([mu, sd]).view(1, -1)
    pd = R.DiagGaussRef(k['A'])
    assert abs(pd.loglikelihood(mu.view(1, -1), p).item() - k['loglik_at_mean']) < 1e-5
    assert abs(pd.entropy(p).item() - k['entropy']) < 1e-5
    assert abs(pd.kl(p, p).item()) < 1e-6
    q = torch.cat([mu + k['shift'], sd]).view(1, -1)
    assert abs(pd.kl(p, q).item() - k['kl_shift']) < 1e-5


def test_zfilter_oracle_known_answer():
    k = _load('known_answers.json')['zfilter']
    zf = R.ZFilterRef(3)
    zf.z_update(torch.full((k['B'], 3), k['c']))
    assert np.allclose(zf.running_mean(), k['mean'], rtol=1e-6)
    assert abs(zf.count.item() - k['count']) < 1e-3


def test_adam_closed_form_against_torch():
    k = _load('known_answers.json')['adam']
    p = torch.nn.Parameter(torch.tensor(k['p0']).float())
    opt = torch.optim.Adam([p], lr=k['lr'], eps=k['eps'])
    p.grad = torch.tensor(k['g']).float()
    opt.step()
    assert np.allclose(p.detach().numpy(), k['p1'], rtol=1e-6, atol=1e-7)


def test_clip_loss_ratio_one_known_answer():
    k = _load('known_answers.json')['clip']
    adv = torch.tensor(k['adv']).float().view(-1, 1)
    ratio = torch.ones_like(adv)
    surr = -ratio * adv
    csurr = -torch.clamp(ratio, 0.8, 1.2) * adv
    loss = torch.cat([surr, csurr], 1).max(1)[0].mean()
    assert abs(loss.item() - k['clip_loss']) < 1e-7


def test_oracle_learner_runs_and_early_stops():
    from surreal_amd import synthetic
    from tests.helpers import oracle_batch, ppo_config
    lc = ppo_config(B=16, T=6, mode='adapt', lr=(5e-2, 1e-3), kl_target=0.001)
    ref = R.PPOLearnerRef(lc, 17, 6)
    s = ref.learn(oracle_batch(synthetic.ppo_batch(16, 6, 17, 6, seed=1)))
    assert s['epochs_run'] < 10                   # KL > 4 * kl_target stopped the loop
    assert s['_pol_kl'] > 4 * 0.001
