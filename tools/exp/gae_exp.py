"""Developer experiment: HBM ceiling of the GAE byte mix vs the library kernel."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from surreal_amd import _lib as L  # noqa: E402

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libgae_exp.so'))
lib.exp_stream_launch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64] * 2 + [ctypes.c_void_p] * 2 + \
    [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
B, T, H = 1 << 21, 25, 5
E = T - H + 1
dev = 'cuda'
r = torch.randn(B * T, device=dev)
d = (torch.rand(B * T, device=dev) < 0.02).float()
v = torch.randn(B * (T + 1), device=dev)
adv = torch.empty(B * E, device=dev)
ret = torch.empty(B * E, device=dev)
sink = torch.zeros(4, device=dev)
nbytes = 4 * (2 * B * T + B * (T + 1) + 2 * B * E)
st = L.stream()


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters):
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


for grid in (1024, 2048, 4096, 8192):
    ms = timed(lambda: lib.exp_stream_launch(r.data_ptr(), d.data_ptr(), v.data_ptr(), B * T // 4,
                                             B * (T + 1) // 4, adv.data_ptr(), ret.data_ptr(),
                                             B * E // 4, sink.data_ptr(), grid, st))
    print(json.dumps({'kernel': 'stream_ceiling', 'grid': grid, 'ms': round(ms, 4),
                      'GBs': round(nbytes / ms / 1e6, 1)}), flush=True)
npart = L.lib().smi_gae_windows_max_partials(B, T)
part = torch.empty(2 * npart, dtype=torch.float64, device=dev)
npo = ctypes.c_int(0)
gt = torch.pow(0.99, torch.arange(T, dtype=torch.float32)).to(dev)
lt = torch.pow(0.95, torch.arange(T, dtype=torch.float32)).to(dev)
P = L.ptr
ms = timed(lambda: L.call('smi_gae_windows', P(v), None, P(r), P(d), B, T, H, P(gt), P(lt), 0.99,
                          0.99 ** H, P(adv), P(ret), P(part), ctypes.byref(npo), st))
print(json.dumps({'kernel': 'gae_windows_rnn_lib', 'variant': os.environ.get('SMI_LIB_VARIANT'),
                  'ms': round(ms, 4), 'GBs': round(nbytes / ms / 1e6, 1)}), flush=True)
