"""The statistic self-consistency check of the pinned GPU tests
(tests/parity.py recompute_stats), validated on the CPU oracle itself: the
oracle's own last-learn() statistics (fp32, oracle/ppo_ref.py restating
ppo.py:194-331,553-575) must be reproduced in fp64 from the oracle's own
captured states within the same 1e-5 bar the GPU is held to.  This pins the
bookkeeping (which parameters each statistic is taken at, which advantages,
the reference policy) independently of the GPU."""
import numpy as np
import pytest
import torch

from oracle import ppo_ref as R
from surreal_amd import synthetic
from tests import parity as P
from tests.helpers import lstm_flat, oracle_batch, ppo_config, seq_flat


def _oracle_state(ref, m=None):
    m = m if m is not None else ref.model
    st = {'actor': m.actor.flat().clone(), 'critic': m.critic.flat().clone()}
    if m.rnn:
        st['lstm'] = lstm_flat(m.rnn_stem).clone()
    if m.cnn_stem is not None:
        st['cnn'] = seq_flat(m.cnn_stem).clone()
    if m.use_z_filter:
        st['zf'] = tuple(getattr(m.z_filter, b).clone() for b in ('running_sum', 'running_sumsq', 'count'))
    return st


def _capture_oracle_learn(ref, ob):
    cap = {'ref': _oracle_state(ref, ref.ref_target_model), 'pol_in': [], 'val_in': [],
           'pol_final': None, 'hyper': (ref.clip_epsilon, ref.beta)}
    pu, vu = ref._policy_update, ref._value_update

    def policy_update(*a, **k):
        cap['pol_in'].append(_oracle_state(ref))
        return pu(*a, **k)

    def value_update(*a, **k):
        if cap['pol_final'] is None:
            cap['pol_final'] = _oracle_state(ref)
        cap['val_in'].append(_oracle_state(ref))
        return vu(*a, **k)
    ref._policy_update, ref._value_update = policy_update, value_update
    cap['zf_epochs'] = _oracle_state(ref).get('zf')
    stats = ref.learn(ob)
    ref._policy_update, ref._value_update = pu, vu
    cap['final'] = _oracle_state(ref)
    if cap['pol_final'] is None:
        cap['pol_final'] = cap['final']
    return stats, cap


@pytest.mark.parametrize('kind,mode', [('mlp', 'clip'), ('mlp', 'adapt'), ('lstm', 'adapt'),
                                       ('lstm', 'clip'), ('pixel', 'adapt')])
def test_oracle_stats_are_self_consistent(kind, mode):
    D, A = 9, 3
    pixel, Hd = None, None
    if kind == 'mlp':
        lc = ppo_config(B=32, T=12, mode=mode, use_z_filter=True, hidden=(24, 16), epochs=(4, 3))
    else:
        Hd = 12
        lc = ppo_config(B=16, T=8, mode=mode, use_z_filter=True, hidden=(24, 16), lam=1.0,
                        epochs=(4, 3), rnn=True, rnn_hidden=Hd, horizon=3,
                        cnn_feat=8 if kind == 'pixel' else 256)
        if kind == 'pixel':
            pixel = (3, 36, 36)
    torch.manual_seed(0)
    ref = R.PPOLearnerRef(lc, D, A, seed=3, pixel=pixel)
    report = {}
    for it in range(2):
        batch = synthetic.ppo_batch(lc.replay.batch_size, lc.algo.n_step, D, A, seed=40 + it,
                                    rnn_hidden=Hd, pixel=pixel)
        ob = oracle_batch(batch)
        stats, cap = _capture_oracle_learn(ref, ob)
        adv = ref.last_adv.detach().numpy()
        ret = ref.last_ret.detach().numpy()
        rec = P.recompute_stats(lc, D, A, pixel, ob, cap, adv, ret, stats['epochs_run'])
        expect = {'_pol_kl', '_entropy', '_surr_loss', '_val_loss', '_val_explained_var',
                  '_avg_return_targ', '_avg_log_sig', '_avg_behave_likelihood', '_avg_is_weight',
                  '_ref_behave_diff', 'grad_norm_actor', 'grad_norm_critic',
                  '_clip_surr_loss' if mode == 'clip' else '_kl_loss_adapt'}
        assert expect <= set(rec), sorted(expect - set(rec))
        P.check_stats(stats, rec, report, tag=f'@{it}')
    P.print_report(report)
    assert np.isfinite([v[0] for v in report.values() if isinstance(v, tuple)]).all()
