"""Per-shape timing of the MFMA GEMM engine (smi_linear_*) at the C3 learner
shapes (1024 segments x 21 steps = 21504 rows; LSTM 100, heads 300x200, obs
42, act 8).  Prints one JSON line per (op, shape): median ms and useful TF/s.
Usage: python tools/bench_gemm.py [--iters 20] [--only fwd,dx,dw]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from surreal_amd import _lib as L  # noqa: E402

R = 21504
SHAPES = [  # (name, in, out)
    ('xproj', 42, 400), ('head1', 100, 300), ('head2', 300, 200), ('head3', 200, 8),
    ('whh', 100, 400),
]


def timed(fn, iters):
    for _ in range(3):
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
    return t[len(t) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--only', default='fwd,dx,dw')
    args = ap.parse_args()
    ops = set(args.only.split(','))
    dev = torch.device('cuda', 0)
    L.ensure_workspace(dev)
    st = L.stream(dev)
    P = L.ptr
    g = torch.Generator(device=dev).manual_seed(0)
    for name, k, n in SHAPES:
        x = torch.randn(R, k, device=dev, generator=g)
        w = torch.randn(n, k, device=dev, generator=g) * 0.1
        b = torch.randn(n, device=dev, generator=g)
        y = torch.empty(R, n, device=dev)
        dy = torch.randn(R, n, device=dev, generator=g)
        dx = torch.empty(R, k, device=dev)
        dw = torch.empty(n, k, device=dev)
        db = torch.empty(n, device=dev)
        fl = 2.0 * R * k * n
        if 'fwd' in ops:
            ms = timed(lambda: L.call('smi_linear_forward', P(x), k, R, k, P(w), k, P(b), n, 1, P(y), n, st),
                       args.iters)
            print(json.dumps({'op': 'fwd', 'shape': name, 'M': R, 'K': k, 'N': n, 'ms': round(ms, 4),
                              'tflops': round(fl / ms / 1e9, 2)}), flush=True)
        if 'dx' in ops:
            ms = timed(lambda: L.call('smi_linear_backward_input', P(dy), n, R, n, P(w), k, k, P(x), k,
                                      P(dx), k, st), args.iters)
            print(json.dumps({'op': 'dx', 'shape': name, 'M': R, 'K': n, 'N': k, 'ms': round(ms, 4),
                              'tflops': round(fl / ms / 1e9, 2)}), flush=True)
        if 'dw' in ops:
            ms = timed(lambda: L.call('smi_linear_backward_weight', P(dy), n, R, n, P(x), k, k, P(dw), k,
                                      P(db), 0, st), args.iters)
            print(json.dumps({'op': 'dw', 'shape': name, 'M': n, 'K': R, 'N': k + 1, 'ms': round(ms, 4),
                              'tflops': round(fl / ms / 1e9, 2)}), flush=True)


if __name__ == '__main__':
    main()
