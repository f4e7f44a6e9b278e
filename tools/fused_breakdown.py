"""Developer tool: where does the fused PPO epoch kernel spend its time?

Times ppo_fused_kernel (HIP events, 20 launches each) for epoch mixes and
batch sizes so per-epoch policy / value costs and the prologue can be read off:
    python tools/fused_breakdown.py
"""
import json
import os
import sys

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


def main():
    res = []
    for (B, ep, ev, hid) in [(64, 10, 10, (64, 64)), (64, 10, 0, (64, 64)), (64, 0, 10, (64, 64)),
                             (64, 0, 0, (64, 64)), (64, 1, 0, (64, 64)), (64, 0, 1, (64, 64)),
                             (64, 5, 0, (64, 64)), (128, 10, 10, (64, 64)), (64, 10, 10, (32, 32))]:
        r = time_case(B, 50, ep, ev, hid)
        res.append({'B': B, 'epochs': (ep, ev), 'hidden': hid, 'us': r})
        print(json.dumps(res[-1]), flush=True)


if __name__ == '__main__':
    main()
