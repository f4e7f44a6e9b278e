"""Developer tool: time smi_cnn_forward / smi_cnn_backward at the C5 row counts
(JSON lines: rows, us per call, TF/s).  SMI_LIB_VARIANT selects a build variant."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from surreal_amd import _lib as L  # noqa: E402

C, H, W, F = 3, 84, 84, 256
dev = 'cuda'
n = int(L.lib().smi_cnn_param_count(C, H, W, F))
g = torch.Generator(device=dev).manual_seed(0)
flat = (torch.rand(n, device=dev, generator=g) - 0.5) * 0.05
st = L.stream()
for rows in (2688, 3328):
    pix = torch.randint(0, 256, (rows, C, H, W), device=dev, dtype=torch.uint8, generator=g)
    a1 = torch.empty(rows, 16, 400, device=dev)
    a2 = torch.empty(rows, 2592, device=dev)
    feat = torch.empty(rows, F, device=dev)
    dz = torch.randn(rows, F, device=dev, generator=g)
    nb = int(L.lib().smi_cnn_scratch_bytes(rows, C, H, W, F))
    scratch = torch.empty(nb // 4 + 1, device=dev)
    grad = torch.empty(n, device=dev)

    def fwd():
        L.call('smi_cnn_forward', L.ptr(flat), L.ptr(pix), None, rows, 1, rows, C, H, W, F,
               L.ptr(a1), L.ptr(a2), L.ptr(feat), F, st)

    def bwd():
        L.call('smi_cnn_backward', L.ptr(flat), L.ptr(pix), None, rows, 1, rows, C, H, W, F,
               L.ptr(a1), L.ptr(a2), L.ptr(dz), F, L.ptr(grad), L.ptr(scratch), nb, st)
    for name, fn, conv_flops in (('fwd', fwd, 2 * (16 * 400 * 192 + 32 * 81 * 256)),
                                 ('bwd', bwd, 2 * (2 * 32 * 81 * 256 + 16 * 400 * 192))):
        for _ in range(3):
            fn()
        L.kernel_timing(True)
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        L.kernel_timing(False)
        rep = L.kernel_timing_report()
        k = 'cnn_' + name
        c, ms, fl = rep[k]
        print(json.dumps({'variant': os.environ.get('SMI_LIB_VARIANT'), 'op': name, 'rows': rows,
                          'conv_us': round(ms / c * 1e3, 1),
                          'conv_tflops': round(fl / (ms * 1e-3) / 1e12, 1)}), flush=True)
