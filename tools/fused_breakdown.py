"""Developer tool: where does the fused PPO epoch kernel spend its time?

Times ppo_fused_kernel (HIP events, 20 launches each) for epoch mixes and
batch sizes so per-epoch policy / value costs and the prologue can be read off:
    python tools/fused_breakdown.py
    python tools/fused_breakdown.py --phases   # per-phase wall time inside the kernel
                                               # (needs the 'prof' build variant)
"""
import json
import os
import sys

_var = next((a.split('=', 1)[1] for a in sys.argv if a.startswith('--variant=')), None)
if '--phases' in sys.argv:
    _var = f'{_var}_prof' if _var else 'prof'
if _var:
    os.environ['SMI_LIB_VARIANT'] = _var

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def time_case(B, T, ep, ev, hidden=(64, 64), mode='adapt', reps=20):
    from surreal_amd import synthetic
    from surreal_amd.learner import PPOLearner
    from tests.helpers import env_config, ppo_config
    lc = ppo_config(B=B, T=T, mode=mode, use_z_filter=True, epochs=(ep, ev), hidden=hidden,
                    lr=(1e-5, 1e-5))
    learner = PPOLearner(lc, env_config(17, 6), seed=1)
    batch = synthetic.to_device(synthetic.ppo_batch(B, T, 17, 6, seed=0), 'cuda')
    for _ in range(3):
        learner.learn(batch)
    torch.cuda.synchronize()
    learner.kernel_events = {}
    for _ in range(reps):
        learner.learn(batch)
    torch.cuda.synchronize()
    out = {k: sum(s.elapsed_time(e) for s, e in v) / len(v) * 1e3 for k, v in learner.kernel_events.items()}
    return {k: round(v, 2) for k, v in out.items()}


POLICY_PHASES = {0: 'prologue', 8: 'fwd_tile', 9: 'row_kl', 1: 'fwd_sums', 10: 'row_loss',
                 11: 'gsig_sum', 12: 'dense_bwd', 2: 'logvar_grad', 3: 'loss_sums', 4: 'grad_norm',
                 5: 'adam', 6: 'store'}
VALUE_PHASES = {0: 'prologue', 2: 'fwd_bwd_sums', 4: 'grad_norm', 5: 'adam', 6: 'store'}


def phases(B=64, T=50, ep=10, ev=10, reps=20):
    import ctypes
    from surreal_amd import _lib as L
    time_case(B, T, ep, ev, reps=1)
    buf = (ctypes.c_ulonglong * 64)()
    L.lib().smi_phase_ticks(buf)                       # clear
    t = time_case(B, T, ep, ev, reps=reps)
    torch.cuda.synchronize()
    L.lib().smi_phase_ticks(buf)
    n = reps + 3                                       # warm-up learns are counted too
    pol = {name: round(buf[i] * 10e-3 / n, 2) for i, name in POLICY_PHASES.items()}
    val = {name: round(buf[32 + i] * 10e-3 / n, 2) for i, name in VALUE_PHASES.items()}
    print(json.dumps({'B': B, 'epochs': (ep, ev), 'kernel_us': t, 'policy_us': pol,
                      'value_us': val}), flush=True)


def main():
    if '--phases' in sys.argv:
        phases()
        phases(ep=1, ev=1)
        return
    res = []
    for (B, ep, ev, hid) in [(64, 10, 10, (64, 64)), (64, 10, 0, (64, 64)), (64, 0, 10, (64, 64)),
                             (64, 0, 0, (64, 64)), (64, 1, 0, (64, 64)), (64, 0, 1, (64, 64)),
                             (64, 5, 0, (64, 64)), (128, 10, 10, (64, 64)), (64, 10, 10, (32, 32))]:
        r = time_case(B, 50, ep, ev, hid)
        res.append({'B': B, 'epochs': (ep, ev), 'hidden': hid, 'us': r})
        print(json.dumps(res[-1]), flush=True)


if __name__ == '__main__':
    main()
