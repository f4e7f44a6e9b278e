"""Per-step phase split of the LSTM sequence kernels inside the C3 learn()
(developer tool; 'prof' build variant: python -c "from surreal_amd import build
as B; B.build(variant='prof')", run with SMI_LIB_VARIANT=prof).  Workgroup 0,
wave 0 accumulates wall-clock ticks (100 MHz) per phase of every step:
  fwd [0] recurrent MFMAs + pre-activation store  [1] barrier + x-part issue +
      cell update  [2] second barrier
  bwd [3] cell backward + stores  [4] barrier  [5] dh_rec MFMAs + barrier
  r4 prologues (round 6): [6] forward, [7] BPTT, kernel start to first barrier
Prints one JSON line: microseconds per step per phase."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('SMI_LIB_VARIANT', 'prof')
from surreal_amd import _lib as L  # noqa: E402
from surreal_amd import synthetic  # noqa: E402
from surreal_amd.learner import PPOLearner  # noqa: E402
from tests.helpers import env_config, ppo_config  # noqa: E402


def main():
    B, T, D, A, K = int(os.environ.get('B', 1024)), 25, 42, 8, 5
    lc = ppo_config(B=B, T=T, mode='adapt', use_z_filter=True, hidden=(300, 200), lam=1.0,
                    rnn=True, rnn_hidden=100, horizon=5)
    learner = PPOLearner(lc, env_config(D, A), seed=1, device='cuda')
    batch = synthetic.to_device(synthetic.ppo_batch(B, T, D, A, seed=0, rnn_hidden=100), 'cuda')
    lib = L.lib()
    # the MFMA forms' and the VALU recurrence's ticks (two objects: build.py UNITS)
    fns = [lib.smi_lstm_phase_ticks, lib.smi_lstm_v_phase_ticks]
    for f in fns:
        f.argtypes = [ctypes.c_void_p]
    bufs = [(ctypes.c_ulonglong * 8)() for _ in fns]
    learner.learn(batch)
    torch.cuda.synchronize()
    for f, b in zip(fns, bufs):
        f(ctypes.cast(b, ctypes.c_void_p))      # reset
    for _ in range(K):
        learner.learn(batch)
    torch.cuda.synchronize()
    for f, b in zip(fns, bufs):
        f(ctypes.cast(b, ctypes.c_void_p))
    buf = [bufs[0][i] + bufs[1][i] for i in range(8)]
    E = T - 5 + 1
    runs = learner.last_stats()['epochs_run']
    fwd_steps = K * ((T + 1) + E + (runs + 1) * E + 10 * E)
    bwd_steps = K * (runs + 10) * E
    us = lambda t, n: round(t * 0.01 / n, 4)  # noqa: E731  (10 ns ticks)
    print(json.dumps({'B': B, 'learns': K, 'fwd_steps': fwd_steps, 'bwd_steps': bwd_steps,
                      'fwd_us_per_step': {'mfma': us(buf[0], fwd_steps), 'cell': us(buf[1], fwd_steps),
                                          'barrier2': us(buf[2], fwd_steps)},
                      'bwd_us_per_step': {'cell': us(buf[3], bwd_steps), 'barrier': us(buf[4], bwd_steps),
                                          'mfma': us(buf[5], bwd_steps)},
                      # round 6: the r4 forms' prologues (kernel start to the first barrier),
                      # per launch (launches per learn: GAE + PREP + the policy forwards +
                      # 10 value, and one BPTT per update)
                      'r4_prologue_us_per_launch': {'fwd': us(bufs[0][6], K * (2 + runs + 1 + 10)),
                                                    'bwd': us(bufs[0][7], K * (runs + 10))}}),
          flush=True)


if __name__ == '__main__':
    main()
