"""Diagnostic (GPU box): post-step parameter error vs the fp64 oracle as the
number of policy / value epochs grows (C3 widths), GPU and CPU fp32, and the
entries where the GPU deviates most after the last count."""
import sys

import torch

sys.path.insert(0, '.')
from oracle import ppo_ref as R  # noqa: E402
from surreal_amd import synthetic  # noqa: E402
from surreal_amd.learner import PPOLearner  # noqa: E402
from tests.helpers import (copy_weights_to_oracle, env_config, lstm_flat, oracle_batch,  # noqa: E402
                           ppo_config)


def run(B, ep, mode, seed=1, show=False, unit=False):
    T, H, D, A, Hd = 25, 5, 42, 8, 100
    lc = ppo_config(B=B, T=T, mode=mode, use_z_filter=True, hidden=(300, 200), lam=1.0,
                    epochs=ep, rnn=True, rnn_hidden=Hd, horizon=H)
    if unit:     # the reference default config at the --unit-test batch (lr 1e-4, no z-filter)
        import copy
        from surreal_amd.config import PPO_DEFAULT_LEARNER_CONFIG
        lc = copy.deepcopy(PPO_DEFAULT_LEARNER_CONFIG)
        lc.replay.batch_size = B
        lc.algo.consts.epoch_policy, lc.algo.consts.epoch_baseline = ep
        D, A = 17, 6
    learner = PPOLearner(lc, env_config(D, A), seed=8)
    refs = []
    for dt in (torch.float32, torch.float64):
        r = R.PPOLearnerRef(lc, D, A, dtype=dt)
        copy_weights_to_oracle(learner, r)
        refs.append(r)
    init = {'actor': learner.model.actor.flat.cpu().double(),
            'critic': learner.model.critic.flat.cpu().double(),
            'lstm': learner.model.rnn_stem.flat.cpu().double()}
    batch = synthetic.ppo_batch(B, T, D, A, seed=seed, rnn_hidden=Hd)
    st = [r.learn(oracle_batch(batch)) for r in refs]
    learner.learn(synthetic.to_device(batch, 'cuda'))
    sg = learner.last_stats()
    got = {'actor': learner.model.actor.flat.cpu().double(),
           'critic': learner.model.critic.flat.cpu().double(),
           'lstm': learner.model.rnn_stem.flat.cpu().double()}
    line = [f'ep={ep} runs gpu/32/64={sg["epochs_run"]}/{st[0]["epochs_run"]}/{st[1]["epochs_run"]}']
    for k in got:
        p32 = (refs[0].model.actor.flat() if k == 'actor' else refs[0].model.critic.flat() if k == 'critic'
               else lstm_flat(refs[0].model.rnn_stem)).double()
        p64 = (refs[1].model.actor.flat() if k == 'actor' else refs[1].model.critic.flat() if k == 'critic'
               else lstm_flat(refs[1].model.rnn_stem)).double()
        sc = float(p64.abs().max())
        eg, ec = (got[k] - p64).abs(), (p32 - p64).abs()
        line.append(f'{k}: gpu {float(eg.max()) / sc:.2e} cpu {float(ec.max()) / sc:.2e} '
                    f'(>1e-5: {int((eg > 1e-5 * sc).sum())}/{int((ec > 1e-5 * sc).sum())})')
        if show:
            idx = torch.argsort(eg, descending=True)[:8]
            for i in idx.tolist():
                print(f'   {k}[{i}] init {float(init[k][i]): .6e} f64 {float(p64[i]): .6e} '
                      f'gpu {float(got[k][i]): .6e} cpu32 {float(p32[i]): .6e}  d64 {float(p64[i] - init[k][i]): .3e}')
    print(' | '.join(line), flush=True)


def envelope(B, ep, mode, unit=False, K=3, seed=1, amp=2.0 ** -24):
    """fp64 oracle runs on inputs perturbed by one fp32 rounding (relative
    2^-24 N(0,1) noise on every input and initial weight): the conditioning of
    the learn() map, vs the GPU and CPU32 errors."""
    T, H, D, A, Hd = 25, 5, 42, 8, 100
    lc = ppo_config(B=B, T=T, mode=mode, use_z_filter=True, hidden=(300, 200), lam=1.0,
                    epochs=ep, rnn=True, rnn_hidden=Hd, horizon=H)
    if unit:
        import copy
        from surreal_amd.config import PPO_DEFAULT_LEARNER_CONFIG
        lc = copy.deepcopy(PPO_DEFAULT_LEARNER_CONFIG)
        lc.replay.batch_size = B
        lc.algo.consts.epoch_policy, lc.algo.consts.epoch_baseline = ep
        D, A = 17, 6
    learner = PPOLearner(lc, env_config(D, A), seed=8)
    batch = synthetic.ppo_batch(B, T, D, A, seed=seed, rnn_hidden=Hd)
    ob = oracle_batch(batch)
    g = torch.Generator().manual_seed(123)

    def pert(x):
        if x is None:
            return None
        if isinstance(x, list):
            return [pert(v) for v in x]
        x = torch.as_tensor(x).double()
        return x * (1 + amp * torch.randn(x.shape, generator=g, dtype=torch.float64))
    outs = []
    for k in range(K + 2):
        dt = torch.float32 if k == K + 1 else torch.float64
        r = R.PPOLearnerRef(lc, D, A, dtype=dt)
        copy_weights_to_oracle(learner, r)
        if 0 < k <= K:
            with torch.no_grad():
                for p in list(r.model.parameters()):
                    p.copy_(pert(p))
                r.ref_target_model.update_target_params(r.model)
            b = {kk: (pert(v) if kk in ('obs', 'obs_next', 'actions', 'rewards', 'pds', 'onetime')
                      else v) for kk, v in ob.items()}
        else:
            b = ob
        r.learn(b)
        outs.append({'actor': r.model.actor.flat().double(), 'critic': r.model.critic.flat().double(),
                     'lstm': lstm_flat(r.model.rnn_stem).double()})
    learner.learn(synthetic.to_device(batch, 'cuda'))
    gpu = {'actor': learner.model.actor.flat.cpu().double(),
           'critic': learner.model.critic.flat.cpu().double(),
           'lstm': learner.model.rnn_stem.flat.cpu().double()}
    line = [f'envelope amp={amp:.1e} ep={ep}']
    for k in gpu:
        sc = float(outs[0][k].abs().max())
        env = max(float((outs[i][k] - outs[0][k]).abs().max()) for i in range(1, K + 1)) / sc
        line.append(f'{k}: gpu {float((gpu[k] - outs[0][k]).abs().max()) / sc:.2e} '
                    f'cpu32 {float((outs[K + 1][k] - outs[0][k]).abs().max()) / sc:.2e} f64-pert {env:.2e}')
    print(' | '.join(line), flush=True)


if __name__ == '__main__':
    mode = sys.argv[1] if len(sys.argv) > 1 else 'adapt'
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    unit = len(sys.argv) > 3 and sys.argv[3] == 'unit'
    if len(sys.argv) > 4 and sys.argv[4] == 'amp':
        for amp in (2.0 ** -24, 1e-6, 4e-6):
            envelope(B, (10, 5), mode, unit=unit, K=5, amp=amp)
        sys.exit(0)
    if len(sys.argv) > 4 and sys.argv[4] == 'solo':
        for ep in ((10, 3), (10, 4), (10, 5), (10, 6), (10, 8), (6, 10), (7, 10), (8, 10), (9, 10)):
            run(B, ep, mode, unit=unit)
        sys.exit(0)
    if len(sys.argv) > 4 and sys.argv[4] == 'grid':
        for ep in ((10, 1), (10, 2), (1, 10), (2, 10), (3, 10), (5, 10), (2, 2)):
            run(B, ep, mode, unit=unit)
        sys.exit(0)
    if len(sys.argv) > 4 and sys.argv[4] == 'env':
        for ep in ((1, 1), (10, 10)):
            envelope(B, ep, mode, unit=unit)
        sys.exit(0)
    for ep in ((1, 0), (0, 1), (1, 1), (2, 0), (3, 0), (5, 0), (10, 0), (0, 3), (0, 10)):
        run(B, ep, mode, unit=unit, show=unit and ep in ((1, 0), (0, 1)))
    run(B, (10, 10), mode, show=True, unit=unit)

