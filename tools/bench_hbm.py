"""HBM-roofline sweep of the streaming kernels on the learner path.

Each kernel runs on working sets well beyond the 256 MiB Infinity Cache, timed
with HIP events on the stream it is launched on (median of --iters launches
after warm-up).  achieved GB/s = ALGORITHMIC bytes per launch / duration, where
the algorithmic bytes are the §8(d) per-unit figures:

  gae_windows (non-RNN, T=50, H=T)  r,d 8 B + V 4(T+1)/T B + adv,ret 8/T B per env-step
  gae_windows (RNN, T=25, H=5)      r,d 8 B + V 4(T+1)/T B + adv,ret 8E/T B per env-step
  zfilter_apply (D=42)              8 D B per row (read x, write out)
  zfilter_update (D=42)             4 D B per row (read x; 2D+1 floats written)
  diag_gauss kl+loglik+ent (A=8)    a 4A + p0 8A + p1 8A read, 3 x 4 B written per row
  adam_clip                         p,g,m,v read 16 B + p,m,v written 12 B per param: SURVEY
                                    §8(d)'s 28 B (the norm pass's second read of g, 4 B more
                                    moved, is NOT counted; frac_moved adds it); g spans 3 x 2^26
                                    floats (768 MiB, > 2 x the MALL) so that re-read cannot hit
                                    the Infinity Cache
  adam_noclip                       p,g,m,v read 16 B + p,m,v written 12 B per param
  gather_rows (W=42 floats)         8 idx + 2 x 4 W B per gathered row
  moments                           4 B per element

peak = 8000 GB/s (MI355X HBM3E spec, MI355X_MICROARCH.md).  Prints one JSON line
per kernel.  Usage: python tools/bench_hbm.py [--iters 20] [--only name,...]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from surreal_amd import _lib as L  # noqa: E402

PEAK = 8000.0


def timed(fn, iters, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    evs = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        evs.append((s, e))
    torch.cuda.synchronize()
    ts = sorted(s.elapsed_time(e) for s, e in evs)
    return ts[len(ts) // 2]


def report(name, nbytes, ms, **extra):
    gbs = nbytes / (ms * 1e-3) / 1e9
    out = {'kernel': name, 'algorithmic_bytes': int(nbytes), 'median_ms': round(ms, 4),
           'achieved_GBs': round(gbs, 1), 'peak_GBs': PEAK, 'frac': round(gbs / PEAK, 4)}
    out.update(extra)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--only', default='')
    args = ap.parse_args()
    only = set(args.only.split(',')) if args.only else None
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    L.ensure_workspace(dev)
    st = L.stream(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    P = L.ptr

    def want(n):
        return only is None or n in only

    for name, B, T, H in (('gae_windows_nonrnn', 1 << 20, 50, 50), ('gae_windows_rnn', 1 << 21, 25, 5)):
        if not want(name):
            continue
        E = T - H + 1
        r = torch.randn(B, T, device=dev, generator=g)
        d = (torch.rand(B, T, device=dev, generator=g) < 0.02).float()
        v = torch.randn(B, T + 1, device=dev, generator=g)
        gt = torch.pow(0.99, torch.arange(T, dtype=torch.float32)).to(dev)
        lt = torch.pow(0.95, torch.arange(T, dtype=torch.float32)).to(dev)
        adv = torch.empty(B, E, device=dev)
        ret = torch.empty(B, E, device=dev)
        npart = L.lib().smi_gae_windows_max_partials(B, T)
        parts = torch.empty(2 * npart, dtype=torch.float64, device=dev)
        np_out = ctypes.c_int(0)
        fn = lambda: L.call('smi_gae_windows', P(v), None, P(r), P(d), B, T, H, P(gt), P(lt), 0.99,  # noqa
                            float(0.99 ** H), P(adv), P(ret), P(parts), ctypes.byref(np_out), st)
        ms = timed(fn, args.iters)
        nbytes = B * T * 8 + B * (T + 1) * 4 + B * E * 8
        report(name, nbytes, ms, B=B, T=T, horizon=H, env_steps=B * T,
               bytes_per_env_step=round(nbytes / (B * T), 3))
        del r, d, v, adv, ret, parts

    D = 42
    if want('zfilter_apply'):
        rows = 1 << 22
        x = torch.randn(rows, D, device=dev, generator=g)
        out = torch.empty_like(x)
        zs, zq, zc = x[:1000].sum(0), (x[:1000] ** 2).sum(0), torch.tensor([1000.0], device=dev)
        fn = lambda: L.call('smi_zfilter_apply', P(x), P(out), rows, D, P(zs), P(zq), P(zc), 1e-5, st)  # noqa
        report('zfilter_apply', rows * D * 8, timed(fn, args.iters), rows=rows, dim=D)
        del x, out
    if want('zfilter_update'):
        rows = 1 << 22
        x = torch.randn(rows, D, device=dev, generator=g)
        zs, zq, zc = torch.zeros(D, device=dev), torch.zeros(D, device=dev), torch.ones(1, device=dev)
        fn = lambda: L.call('smi_zfilter_update', P(x), rows, D, D, P(zs), P(zq), P(zc), st)  # noqa
        report('zfilter_update', rows * D * 4, timed(fn, args.iters), rows=rows, dim=D)
        del x

    if want('diag_gauss'):
        rows, A = 1 << 23, 8
        a = torch.randn(rows, A, device=dev, generator=g)
        p0 = torch.rand(rows, 2 * A, device=dev, generator=g) + 0.5
        p1 = torch.rand(rows, 2 * A, device=dev, generator=g) + 0.5
        ll, kl, en = (torch.empty(rows, device=dev) for _ in range(3))
        fn = lambda: L.call('smi_diag_gauss', P(a), P(p0), P(p1), rows, A, P(ll), None, P(kl), P(en), st)  # noqa
        report('diag_gauss', rows * (4 * A + 16 * A + 12), timed(fn, args.iters), rows=rows, act_dim=A)
        del a, p0, p1, ll, kl, en

    if want('adam_clip'):
        n = 3 << 26
        p = torch.randn(n, device=dev, generator=g)
        gr = torch.randn(n, device=dev, generator=g)
        m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
        step = torch.zeros(1, dtype=torch.int32, device=dev)
        lr = torch.tensor([1e-4], device=dev)
        norm = torch.zeros(1, device=dev)
        fn = lambda: L.call('smi_adam_clip', P(p), P(gr), P(m), P(v), n, P(step), P(lr), 0.9,  # noqa
                            0.999, 1e-8, 0.0, 10.0, 0.0, None, P(norm), st)
        ms = timed(fn, args.iters)
        report('adam_clip', n * 28, ms, params=n,
               frac_moved=round(n * 32 / (ms * 1e-3) / 1e9 / PEAK, 4),
               note='28 B/param algorithmic (SURVEY 8(d)); frac_moved counts the norm pass (32 B)')
        fn2 = lambda: L.call('smi_adam_clip', P(p), P(gr), P(m), P(v), n, P(step), P(lr), 0.9,  # noqa
                             0.999, 1e-8, 0.0, 0.0, 0.0, None, None, st)
        report('adam_noclip', n * 28, timed(fn2, args.iters), params=n)
        del p, gr, m, v

    if want('gather_rows'):
        n_tab, W, batch = 1 << 22, 42, 1 << 21
        tab = torch.randn(n_tab, W, device=dev, generator=g)
        idx = torch.randint(0, n_tab, (batch,), device=dev, generator=g)
        out = torch.empty(batch, W, device=dev)
        fn = lambda: L.call('smi_gather_rows', P(tab), W, P(idx), batch, P(out), st)  # noqa
        report('gather_rows', batch * (8 + 8 * W), timed(fn, args.iters), table_rows=n_tab,
               cols=W, batch=batch)
        del tab, idx, out

    if want('moments'):
        n = 1 << 27
        x = torch.randn(n, device=dev, generator=g)
        o = torch.empty(3, dtype=torch.float64, device=dev)
        fn = lambda: L.call('smi_moments', P(x), n, None, 0, P(o), st)  # noqa
        report('moments', n * 4, timed(fn, args.iters), n=n)
        del x


if __name__ == '__main__':
    main()
