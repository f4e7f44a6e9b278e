"""Per-step phase breakdown of the LSTM sequence kernels (developer tool).
Needs the 'prof' build variant: python -c "from surreal_amd import build as B;
B.build(variant='prof')"; run with SMI_LIB_VARIANT=prof.
Prints microseconds per step for workgroup 0 / wave 0."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('SMI_LIB_VARIANT', 'prof')
from surreal_amd import _lib as L  # noqa: E402

B, S, H = int(os.environ.get('B', 1024)), 21, 100
dev = 'cuda'
lib = L.lib()
lib.smi_lstm_phase_ticks.argtypes = [ctypes.c_void_p]
st = L.stream()
g = torch.Generator(device=dev).manual_seed(0)
xproj = torch.randn(S, B, 4 * H, device=dev, generator=g) * 0.3
whh = torch.randn(4 * H, H, device=dev, generator=g) * 0.1
bhh = torch.randn(4 * H, device=dev, generator=g) * 0.1
h0 = torch.randn(B, H, device=dev, generator=g) * 0.1
c0 = torch.randn(B, H, device=dev, generator=g) * 0.1
hbuf = torch.empty(S + 1, B, H, device=dev)
cbuf = torch.empty(S + 1, B, H, device=dev)
gates = torch.empty(S, B, 4 * H, device=dev)
dh = torch.randn(S, B, H, device=dev, generator=g)
dgates = torch.empty(S, B, 4 * H, device=dev)
P = L.ptr
buf = (ctypes.c_ulonglong * 8)()


def run(n):
    for _ in range(n):
        L.call('smi_lstm_forward', P(xproj), P(whh), P(bhh), P(h0), P(c0), S, B, H, P(hbuf), P(cbuf),
               P(gates), st)
        L.call('smi_lstm_backward', P(dh), P(gates), P(cbuf), P(whh), S, B, H, P(dgates), st)


run(3)
torch.cuda.synchronize()
lib.smi_lstm_phase_ticks(ctypes.cast(buf, ctypes.c_void_p))
n = 20
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
run(n)
e.record()
torch.cuda.synchronize()
lib.smi_lstm_phase_ticks(ctypes.cast(buf, ctypes.c_void_p))
us = lambda i, steps: round(buf[i] * 0.01 / (n * steps), 3)  # noqa: E731  (100 MHz ticks)
print(json.dumps({'B': B, 'S': S, 'H': H, 'fwd+bwd_ms_per_pair': round(s.elapsed_time(e) / n, 4),
                  'fwd_us_per_step': {'mfma': us(0, S), 'epilogue': us(1, S), 'barrier': us(2, S)},
                  'bwd_us_per_step': {'elementwise': us(3, S), 'barrier': us(4, S),
                                      'mfma': us(5, S - 1)}}))
