"""Phase split of the one-segment-per-workgroup VALU LSTM forward inside the
learner at a rank's batch (developer tool, 'prof' build variant:
python -c "from surreal_amd import build as B; B.build(variant='prof')", run
with SMI_LIB_VARIANT=prof).  Workgroup 0, thread 0 accumulates wall-clock ticks
(100 MHz) per phase of lstm_fwd_q_kernel:
  [0] x staging, c0 / h0, W_ih issued (first barrier)  [1] x parts on the
  matrix cores (second barrier)  [2] W_hh wait  [3] the step loop
and [4] the whole lstm_bwd_q_kernel (when the BPTT runs in its own launch).
Prints microseconds per launch per phase."""
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
    B, T, D, A, K = int(os.environ.get('B', 128)), 25, 42, 8, 5
    lc = ppo_config(B=B, T=T, mode='adapt', use_z_filter=True, hidden=(300, 200), lam=1.0,
                    rnn=True, rnn_hidden=100, horizon=5)
    learner = PPOLearner(lc, env_config(D, A), seed=1, device='cuda')
    batch = synthetic.to_device(synthetic.ppo_batch(B, T, D, A, seed=0, rnn_hidden=100), 'cuda')
    lib = L.lib()
    lib.smi_lstm_v_phase_ticks.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 8)()
    learner.learn(batch)
    torch.cuda.synchronize()
    lib.smi_lstm_v_phase_ticks(ctypes.cast(buf, ctypes.c_void_p))      # reset
    for _ in range(K):
        learner.learn(batch)
    torch.cuda.synchronize()
    lib.smi_lstm_v_phase_ticks(ctypes.cast(buf, ctypes.c_void_p))
    n_fwd = K * (learner.epoch_policy + 1 + learner.epoch_baseline)   # + the GAE / PREP launch
    names = ['x_stage_w_ih', 'x_parts_mfma', 'w_hh_wait', 'steps', 'bwd_whole']
    out = {'B': B, 'learns': K, 'fwd_launches': n_fwd,
           'us_per_fwd_launch': {nm: round(buf[i] * 0.01 / n_fwd, 3) for i, nm in enumerate(names[:4])},
           'bwd_total_us_all_launches': round(buf[4] * 0.01, 1)}
    print(json.dumps(out), flush=True)
    # the same kernel alone, back to back (hot instruction cache / L2), and with
    # a 1 GiB write between launches (cold): does the prologue cost come from
    # the launch's context in the learner?
    S, H = T + 1, 100
    g = torch.Generator(device='cpu').manual_seed(0)
    x = torch.randn(S, B, D, generator=g).cuda()
    w_ih, w_hh = (torch.randn(4 * H, D, generator=g) * 0.1).cuda(), (torch.randn(4 * H, H, generator=g) * 0.1).cuda()
    b_ih, b_hh = torch.zeros(4 * H, device='cuda'), torch.zeros(4 * H, device='cuda')
    h0, c0 = torch.zeros(B, H, device='cuda'), torch.zeros(B, H, device='cuda')
    hb, cb = torch.empty(S + 1, B, H, device='cuda'), torch.empty(S + 1, B, H, device='cuda')
    ga, xs = torch.empty(S, B, 4 * H, device='cuda'), torch.empty(S, B, 4 * H, device='cuda')
    junk = torch.empty(1 << 28, device='cuda')
    st = torch.cuda.current_stream().cuda_stream
    for mode in ('hot', 'cold'):
        n = 50
        for it in range(n + 1):
            if it == 1:
                torch.cuda.synchronize()
                lib.smi_lstm_v_phase_ticks(ctypes.cast(buf, ctypes.c_void_p))
            if mode == 'cold':
                junk.fill_(float(it))
            L.call('smi_lstm_forward_x', L.ptr(x), D, D, L.ptr(w_ih), L.ptr(b_ih), L.ptr(w_hh), L.ptr(b_hh),
                   L.ptr(h0), L.ptr(c0), S, B, H, L.ptr(hb), L.ptr(cb), L.ptr(ga), L.ptr(xs), st)
        torch.cuda.synchronize()
        lib.smi_lstm_v_phase_ticks(ctypes.cast(buf, ctypes.c_void_p))
        print(json.dumps({'standalone': mode, 'B': B, 'S': S,
                          'us_per_fwd_launch': {nm: round(buf[i] * 0.01 / n, 3) for i, nm in enumerate(names[:4])}}),
              flush=True)


if __name__ == '__main__':
    main()
