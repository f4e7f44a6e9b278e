"""Timing of the fused head passes (smi_head_forward / smi_head_backward_input)
at the learner's shapes: LSTM 100 -> 300 -> 200 -> 8 (policy, tanh) over
21504 rows (C3 policy epochs), -> 1 over 26624 rows (the GAE critic pass) and
2688 rows (one rank of N = 8).  The kernel choice comes from the environment
(SMI_HEAD_T, SMI_HEAD_FQ: read once per process), so A/B arms run as separate
processes.  Prints one JSON line per (pass, shape): median us and TF/s.
Usage: python tools/bench_head.py [--iters 50] [--tag NAME]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from surreal_amd import _lib as L  # noqa: E402

SHAPES = [(21504, 100, 300, 200, 8, 1), (26624, 100, 300, 200, 1, 0), (2688, 100, 300, 200, 8, 1)]


def timed(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ev = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        ev.append((s, e))
    torch.cuda.synchronize()
    t = sorted(s.elapsed_time(e) for s, e in ev)
    return t[len(t) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--tag', default=os.environ.get('SMI_HEAD_T', '1') + '/' +
                    os.environ.get('SMI_HEAD_FQ', 'auto'))
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    L.ensure_workspace(dev)
    st = L.stream(dev)
    P = L.ptr
    g = torch.Generator(device=dev).manual_seed(0)
    for rows, din, h1, h2, out, tanh_out in SHAPES:
        n = din * h1 + h1 + h1 * h2 + h2 + h2 * out + out
        prm = torch.randn(n, device=dev, generator=g) * 0.05
        x = torch.randn(rows, din, device=dev, generator=g)
        ha1 = torch.empty(rows, h1, device=dev)
        ha2 = torch.empty(rows, h2, device=dev)
        y = torch.empty(rows, out, device=dev)
        wT = torch.empty(din * h1 + h1 * h2, device=dev)
        dz = torch.randn(rows, out, device=dev, generator=g)
        dh2 = torch.empty(rows, h2, device=dev)
        dh1 = torch.empty(rows, h1, device=dev)
        dx = torch.empty(rows, din, device=dev)

        def fwd():
            L.call('smi_head_forward', P(prm), din, h1, h2, out, tanh_out, P(x), din, rows,
                   P(ha1), P(ha2), P(y), P(wT), st)

        def bwd():
            L.call('smi_head_backward_input', P(prm), din, h1, h2, out, P(wT), P(dz), rows,
                   P(ha1), P(ha2), P(dh2), P(dh1), 0, din, P(dx), din, None, 0, st)
        fwd()
        for name, fn, fl in (('fwd', fwd, 2.0 * rows * (din * h1 + h1 * h2 + h2 * out)),
                             ('bwd', bwd, 2.0 * rows * (out * h2 + h2 * h1 + h1 * din))):
            us = timed(fn, args.iters)
            print(json.dumps({'tag': args.tag, 'pass': name, 'rows': rows, 'out': out,
                              'us': round(us, 2), 'tflops': round(fl / us / 1e6, 2)}), flush=True)


if __name__ == '__main__':
    main()
