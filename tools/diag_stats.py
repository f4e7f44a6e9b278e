"""Diagnostic (GPU box): last_stats() of the HIP learner vs the fp64 oracle and
the envelope (tests/test_gpu_parity_pinned.py) as the policy-epoch count grows,
C3 widths, clip mode."""
import sys

sys.path.insert(0, '.')
from surreal_amd import synthetic  # noqa: E402
from surreal_amd.learner import PPOLearner  # noqa: E402
from tests.helpers import env_config, oracle_batch, ppo_config  # noqa: E402
from tests.test_gpu_parity_pinned import STAT_KEYS, _envelope  # noqa: E402


def run(ep, mode, B=1024):
    T, H, D, A, Hd = 25, 5, 42, 8, 100
    lc = ppo_config(B=B, T=T, mode=mode, use_z_filter=True, hidden=(300, 200), lam=1.0,
                    epochs=ep, rnn=True, rnn_hidden=Hd, horizon=H)
    learner = PPOLearner(lc, env_config(D, A), seed=9)
    r64, vs = _envelope(learner, lc, D, A, None)
    batch = synthetic.ppo_batch(B, T, D, A, seed=200, rnn_hidden=Hd)
    ob = oracle_batch(batch)
    s64 = r64.learn(ob)
    svs = [v.learn(ob, 200) for v in vs]
    learner.learn(synthetic.to_device(batch, 'cuda'))
    s = learner.last_stats()
    out = []
    for k in STAT_KEYS + (('_clip_surr_loss',) if mode == 'clip' else ('_kl_loss_adapt',)):
        if k not in s64:
            continue
        sc = max(abs(s64[k]), 1e-30)
        eg = abs(s[k] - s64[k]) / sc
        ee = max(abs(x[k] - s64[k]) for x in svs) / sc
        out.append(f'{k}:{eg:.1e}/{ee:.1e}{"*" if eg > 2 * ee + 1e-6 else ""}')
    print(f'ep={ep} {mode}: ' + ' '.join(out), flush=True)


if __name__ == '__main__':
    mode = sys.argv[1] if len(sys.argv) > 1 else 'clip'
    for ep in ((1, 1), (2, 1), (3, 1), (5, 1), (10, 1)):
        run(ep, mode)
