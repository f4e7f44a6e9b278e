"""LSTM sequence kernels in isolation at a rank's share of the C3 batch
(default 128 segments, 21 steps, H 100): median time per smi_lstm_forward /
smi_lstm_backward launch (HIP events on the calling stream) and per step.
SMI_LSTM_VALU=0/1 selects the MFMA / VALU recurrence forms for A/B.
Usage: python tools/bench_lstm.py [--segments 128] [--steps 21] [--iters 50]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from surreal_amd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--segments', type=int, default=128)
    ap.add_argument('--steps', type=int, default=21)
    ap.add_argument('--hidden', type=int, default=100)
    ap.add_argument('--iters', type=int, default=50)
    args = ap.parse_args()
    B, S, H = args.segments, args.steps, args.hidden
    dev = torch.device('cuda', 0)
    L.ensure_workspace(dev)
    st = L.stream(dev)
    P = L.ptr
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

    def fwd():
        L.call('smi_lstm_forward', P(xproj), P(whh), P(bhh), P(h0), P(c0), S, B, H, P(hbuf),
               P(cbuf), P(gates), st)

    def bwd():
        L.call('smi_lstm_backward', P(dh), P(gates), P(cbuf), P(whh), S, B, H, P(dgates), st)

    out = {'bench': 'lstm', 'segments': B, 'steps': S, 'hidden': H,
           'valu': os.environ.get('SMI_LSTM_VALU', 'auto')}
    for name, fn in (('fwd', fwd), ('bwd', bwd)):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ev = []
        for _ in range(args.iters):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            ev.append((s, e))
        torch.cuda.synchronize()
        t = sorted(s.elapsed_time(e) for s, e in ev)
        ms = t[len(t) // 2]
        out[name + '_us'] = round(ms * 1e3, 2)
        out[name + '_us_per_step'] = round(ms * 1e3 / S, 3)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
