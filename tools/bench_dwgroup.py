"""The grouped weight-gradient launch of one C3 backward phase in isolation:
the actor head's three layers (dW over 21504 rows: 300x101, 200x301, 8x201)
and the LSTM's fused W_ih | W_hh over [x_t | h_{t-1}] (400 x (42 | 100) + bias),
queued with smi_dw_group_begin / smi_linear_backward_weight and run by
smi_dw_group_flush, as ppo_rnn.hip's stem_backward does.  Prints the median
time per flush and the algorithmic TF/s; --rows / --segments change the row
count (128 segments: 2688 rows).  Used for A/B timing and rocprofv3 passes.
Usage: python tools/bench_dwgroup.py [--iters 50] [--segments 1024]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from surreal_amd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--segments', type=int, default=1024)
    ap.add_argument('--steps', type=int, default=21)
    ap.add_argument('--only', choices=('all', 'head', 'lstm'), default='all',
                    help='queue only the heads\' or only the LSTM\'s GEMMs')
    args = ap.parse_args()
    R = args.segments * args.steps
    dev = torch.device('cuda', 0)
    L.ensure_workspace(dev)
    st = L.stream(dev)
    P = L.ptr
    g = torch.Generator(device=dev).manual_seed(0)
    H, D, G4, h1, h2, A = 100, 42, 400, 300, 200, 8
    # head: X0 = LSTM outputs [R][H], HA1 [R][h1], HA2 [R][h2]; dZ [R][A]
    X0 = torch.randn(R, H, device=dev, generator=g)
    HA1 = torch.relu(torch.randn(R, h1, device=dev, generator=g))
    HA2 = torch.relu(torch.randn(R, h2, device=dev, generator=g))
    dZ = torch.randn(R, A, device=dev, generator=g) * 1e-3
    dH2 = torch.randn(R, h2, device=dev, generator=g) * 1e-3
    dH1 = torch.randn(R, h1, device=dev, generator=g) * 1e-3
    # LSTM: x_t [R][44] (ldx 44), h_{t-1} [R][H], dgates [R][4H]
    Xz = torch.randn(R, 44, device=dev, generator=g)
    hb = torch.randn(R, H, device=dev, generator=g)
    dg = torch.randn(R, G4, device=dev, generator=g) * 1e-3
    gW3, gb3 = torch.empty(A, h2, device=dev), torch.empty(A, device=dev)
    gW2, gb2 = torch.empty(h2, h1, device=dev), torch.empty(h2, device=dev)
    gW1, gb1 = torch.empty(h1, H, device=dev), torch.empty(h1, device=dev)
    fl = 2.0 * R * (A * h2 + h2 * h1 + h1 * H + G4 * (D + H)) + R * (A + h2 + h1 + G4)   # algorithmic (D = 42)
    lstm = torch.empty(G4 * D + G4 * H + 2 * G4, device=dev)
    gWih = torch.empty(G4, 44, device=dev)

    def phase():
        L.call('smi_dw_group_begin')
        if args.only != 'lstm':
            L.call('smi_linear_backward_weight', P(dZ), A, R, A, P(HA2), h2, h2, P(gW3), h2, P(gb3), 0, st)
            L.call('smi_linear_backward_weight', P(dH2), h2, R, h2, P(HA1), h1, h1, P(gW2), h1, P(gb2), 0, st)
            L.call('smi_linear_backward_weight', P(dH1), h1, R, h1, P(X0), H, H, P(gW1), H, P(gb1), 0, st)
        if args.only == 'head':
            L.call('smi_dw_group_flush', st)
            return
        # the LSTM's W_ih and W_hh as two GEMMs of the group (the learner fuses
        # them over [x_t | h_{t-1}] through the internal two-source form)
        # (x padded to 44 columns as the learner's [x_t | h_{t-1}] form reads it:
        # 16-byte rows, the streaming loop)
        L.call('smi_linear_backward_weight', P(dg), G4, R, G4, P(Xz), 44, 44, P(gWih), 44,
               P(lstm[G4 * D + G4 * H:]), 0, st)
        L.call('smi_linear_backward_weight', P(dg), G4, R, G4, P(hb), H, H, P(lstm[G4 * D:]), H,
               P(lstm[G4 * D + G4 * H + G4:]), 0, st)
        L.call('smi_dw_group_flush', st)
    for _ in range(5):
        phase()
    torch.cuda.synchronize()
    ev = []
    for _ in range(args.iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        phase()
        e.record()
        ev.append((s, e))
    torch.cuda.synchronize()
    t = sorted(s.elapsed_time(e) for s, e in ev)
    ms = t[len(t) // 2]
    if (os.environ.get('SMI_LIB_VARIANT') or '').startswith('dwtrace'):
        # one more phase, then the per-workgroup clock trace of its dW launch
        import ctypes
        import numpy as np
        phase()
        torch.cuda.synchronize()
        buf = np.zeros((8192, 6), dtype=np.uint64)
        n = L.lib().smi_diag_dw_trace(ctypes.c_void_p(buf.ctypes.data), 8192)
        tr = buf[:n]
        tr = tr[tr[:, 1] > 0]
        t0 = tr[:, 0].min()
        st_, en = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0      # us (100 MHz)
        dur = en - st_
        gi = ((tr[:, 3] >> 8) & 0xFF).astype(int)
        rows = ((tr[:, 3] >> 16) & 0xFFFF).astype(int)
        narrow = ((tr[:, 3] >> 32) & 1).astype(int)
        vec = ((tr[:, 3] >> 33) & 3).astype(int)
        xcc = (tr[:, 3] & 0xF).astype(int)
        cu = ((tr[:, 2] >> 8) & 0xF).astype(int) + 16 * ((tr[:, 2] >> 13) & 0x7).astype(int)
        grid = np.arange(0.0, float(en.max()) + 1.0, 1.0)
        conc = [int(((st_ <= x) & (en > x)).sum()) for x in grid]
        clk = (tr[:, 5] - tr[:, 4]).astype(np.float64) / np.maximum(dur, 1e-3) / 1e3   # GHz
        # residency: workgroups per CU at 20 us, and durations by that count
        key = xcc * 64 + cu
        at = (st_ <= 20.0) & (en > 20.0)
        per_cu = np.bincount(key[at], minlength=512)
        cnt = per_cu[key]
        # work per workgroup in full-tile rows (narrow tiles at 0.4), and us per 1000 of them
        work = rows * np.where(narrow == 1, 0.4, 1.0)
        out_extra = {
            'wgs_per_cu_at_20us_hist': {int(k): int(v) for k, v in enumerate(np.bincount(per_cu[per_cu > 0]))},
            'dur_med_by_cu_count': {int(k): round(float(np.median(dur[at & (cnt == k)])), 1)
                                    for k in np.unique(cnt[at])},
            'slab_rows_by_group': {int(k): sorted(set(int(r) for r in rows[gi == k]))[:4] for k in np.unique(gi)},
            'us_per_krow_p10_50_90': [round(float(np.percentile(1e3 * dur / np.maximum(work, 1), q)), 2)
                                      for q in (10, 50, 90)],
            'vec_by_group': {int(k): int(np.median(vec[gi == k])) for k in np.unique(gi)},
            'narrow_wgs': int(narrow.sum())}
        out = {**out_extra, 'clock_ghz_p10_50_90': [round(float(np.percentile(clk, q)), 3) for q in (10, 50, 90)],
               'trace_wgs': int(len(tr)), 'span_us': round(float(en.max()), 1),
               'dur_us_p10_50_90_max': [round(float(np.percentile(dur, q)), 1) for q in (10, 50, 90, 100)],
               'start_us_p50_90_max': [round(float(np.percentile(st_, q)), 1) for q in (50, 90, 100)],
               'per_group_dur_med': {int(k): round(float(np.median(dur[gi == k])), 1) for k in np.unique(gi)},
               'per_group_wgs': {int(k): int((gi == k).sum()) for k in np.unique(gi)},
               'per_xcc_wgs': {int(k): int((xcc == k).sum()) for k in np.unique(xcc)},
               'max_wgs_per_xcc_cu': int(np.bincount(xcc * 64 + cu).max()),
               'concurrency_every_5us': conc[::5]}
        print(json.dumps(out), flush=True)
    print(json.dumps({'bench': 'dw_group', 'rows': R, 'ms': round(ms, 4), 'gflop': round(fl / 1e9, 3),
                      'tflops': round(fl / ms / 1e9, 2), 'frac_f32_mfma': round(fl / ms / 1e9 / 157.3, 3)}),
          flush=True)


if __name__ == '__main__':
    main()
