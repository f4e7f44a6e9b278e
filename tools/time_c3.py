"""Time PPOLearner.learn() at the C3 workload (1024 segments, LSTM 100, heads
300x200, T 25, horizon 5, D 42, A 8) with per-phase HIP events."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from surreal_amd import synthetic  # noqa: E402
from surreal_amd.learner import PPOLearner  # noqa: E402
from tests.helpers import env_config, ppo_config  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
lc = ppo_config(B=B, T=25, mode='adapt', use_z_filter=True, hidden=(300, 200), lam=1.0,
                rnn=True, rnn_hidden=100, horizon=5, lr=(1e-4, 1e-4))
learner = PPOLearner(lc, env_config(42, 8), seed=1, device='cuda:0')
pool = [synthetic.to_device(synthetic.ppo_batch(B, 25, 42, 8, seed=i, rnn_hidden=100), 'cuda:0')
        for i in range(3)]
for i in range(3):
    learner.learn(pool[i % 3])
torch.cuda.synchronize()
learner.kernel_events = {}
n = 10
t0 = time.perf_counter()
for i in range(n):
    learner.learn(pool[i % 3])
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / n
ev = learner.kernel_events
tot = {k: float(np.sum([s.elapsed_time(e) for s, e in v])) / n for k, v in ev.items()}
print(json.dumps({'B': B, 'ms_per_learn': dt * 1e3, 'env_steps_per_s': B * 25 / dt,
                  'phase_ms_per_learn': tot, 'epochs_run': learner.last_stats()['epochs_run']}))
