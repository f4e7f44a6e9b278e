"""Phase split of the fused head kernels inside the C3 learn() (developer tool;
'prof' build variant, run with SMI_LIB_VARIANT=prof).  Thread 0 of every
workgroup adds its wall-clock ticks (100 MHz) per phase; prints one JSON line
with the mean microseconds per workgroup of each phase and of the workgroup's
whole lifetime:
  fwd  [0] X staged  [1] layer-1 k loop  [2] epilogue + barrier  [3] HA1 copy-out
       [4] layer-2 k loop  [5] epilogue + barrier  [6] HA2 copy-out + layer 3
       [7] W1^T / W2^T side job
  bwd  [0] dZ W3 pass  [1] dH1 k loop  [2] epilogue + barrier  [3] dH1 copy-out
       [4] dX k loop  [5] dX epilogue"""
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

FWD = ['x_stage', 'l1_kloop', 'l1_epi_barrier', 'ha1_copy', 'l2_kloop', 'l2_epi_barrier',
       'ha2_copy_l3', 'transposes']
BWD = ['dz_w3', 'dh1_kloop', 'epi_barrier', 'dh1_copy', 'dx_kloop', 'dx_epi']


def main():
    B, T, D, A, K = int(os.environ.get('B', 1024)), 25, 42, 8, 3
    lc = ppo_config(B=B, T=T, mode='adapt', use_z_filter=True, hidden=(300, 200), lam=1.0,
                    rnn=True, rnn_hidden=100, horizon=5)
    learner = PPOLearner(lc, env_config(D, A), seed=1, device='cuda')
    batch = synthetic.to_device(synthetic.ppo_batch(B, T, D, A, seed=0, rnn_hidden=100), 'cuda')
    lib = L.lib()
    lib.smi_head_phase_ticks.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 20)()
    learner.learn(batch)
    torch.cuda.synchronize()
    lib.smi_head_phase_ticks(ctypes.cast(buf, ctypes.c_void_p))      # reset
    for _ in range(K):
        learner.learn(batch)
    torch.cuda.synchronize()
    lib.smi_head_phase_ticks(ctypes.cast(buf, ctypes.c_void_p))
    out = {'B': B, 'learns': K}
    for k, names in ((0, FWD), (1, BWD)):
        n = max(int(buf[10 * k + 8]), 1)
        out['fwd' if k == 0 else 'bwd'] = {
            'workgroups': n, 'lifetime_us': round(buf[10 * k + 9] * 0.01 / n, 3),
            'phase_us': {nm: round(buf[10 * k + i] * 0.01 / n, 3) for i, nm in enumerate(names)}}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
