"""LSTM sequence kernels in isolation at a rank's share of the C3 batch
(default 128 segments, H 100, x width 42): microseconds per launch inside a
replayed hipGraph of 20 back-to-back launches (the learner's launch mode), for
smi_lstm_forward (xproj input), smi_lstm_forward_x (fused input projection)
and smi_lstm_backward at each step count, so the per-step cost and the fixed
(prologue) cost separate.  A/B knobs are environment variables
(SMI_LSTM_VALU, SMI_LSTM_Q, SMI_LSTM_XM).
Usage: python tools/bench_lstm.py [--segments 128] [--steps 1,13,25] [--reps 10]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from surreal_amd import _lib as L  # noqa: E402


def graph_us(fn, dev, n=20, reps=10):
    """median microseconds per launch of fn over replays of a graph of n launches"""
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / n)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--segments', type=int, default=128)
    ap.add_argument('--steps', default='1,13,25')
    ap.add_argument('--hidden', type=int, default=100)
    ap.add_argument('--din', type=int, default=42)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--dirty', action='store_true',
                    help='rewrite the weights before every launch (as the learner\'s Adam '
                         'does) and subtract the rewrite kernels\' own time')
    args = ap.parse_args()
    B, H, D = args.segments, args.hidden, args.din
    dev = torch.device('cuda', 0)
    L.ensure_workspace(dev)
    P = L.ptr
    g = torch.Generator(device=dev).manual_seed(0)
    SM = max(int(s) for s in args.steps.split(','))
    x = torch.randn(SM, B, D, device=dev, generator=g)
    wih = torch.randn(4 * H, D, device=dev, generator=g) * 0.1
    bih = torch.randn(4 * H, device=dev, generator=g) * 0.1
    xproj = torch.randn(SM, B, 4 * H, device=dev, generator=g) * 0.3
    whh = torch.randn(4 * H, H, device=dev, generator=g) * 0.1
    bhh = torch.randn(4 * H, device=dev, generator=g) * 0.1
    h0 = torch.randn(B, H, device=dev, generator=g) * 0.1
    c0 = torch.randn(B, H, device=dev, generator=g) * 0.1
    hbuf = torch.empty(SM + 1, B, H, device=dev)
    cbuf = torch.empty(SM + 1, B, H, device=dev)
    gates = torch.empty(SM, B, 4 * H, device=dev)
    dh = torch.randn(SM, B, H, device=dev, generator=g)
    dgates = torch.empty(SM, B, 4 * H, device=dev)
    knobs = {k: v for k, v in os.environ.items() if k.startswith('SMI_LSTM')}
    for S in (int(s) for s in args.steps.split(',')):
        def st():
            return torch.cuda.current_stream(dev).cuda_stream

        def fwd():
            L.call('smi_lstm_forward', P(xproj), P(whh), P(bhh), P(h0), P(c0), S, B, H, P(hbuf),
                   P(cbuf), P(gates), st())

        def fwdx():
            L.call('smi_lstm_forward_x', P(x), D, D, P(wih), P(bih), P(whh), P(bhh), P(h0), P(c0),
                   S, B, H, P(hbuf), P(cbuf), P(gates), P(xproj), st())

        def bwd():
            L.call('smi_lstm_backward', P(dh), P(gates), P(cbuf), P(whh), S, B, H, P(dgates), st())

        def dirty():
            for w in (whh, wih, bhh, bih):
                w.mul_(1.0)

        out = {'bench': 'lstm', 'segments': B, 'steps': S, 'hidden': H, 'din': D, 'knobs': knobs,
               'dirty': args.dirty}
        base = graph_us(dirty, dev, reps=args.reps) if args.dirty else 0.0
        for name, fn in (('fwd', fwd), ('fwd_x', fwdx), ('bwd', bwd)):
            f = (lambda fn=fn: (dirty(), fn())) if args.dirty else fn
            out[name + '_us'] = round(graph_us(f, dev, reps=args.reps) - base, 2)
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
