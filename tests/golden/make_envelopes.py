"""Generates tests/golden/envelope_<case>.npz (tests/parity.py, item 2): the
fp64 oracle's truth and the fp32 envelope widths of the full-size pinned
cases, computed once in the build container so the GPU box runs only the HIP
side of test_gpu_parity_pinned.py.

Usage: python tests/golden/make_envelopes.py [case ...]   (default: all cases)

The oracle is oracle/ppo_ref.py (the CPU restatement of surreal/learner/ppo.py,
test infrastructure); inputs are surreal_amd.synthetic batches and the
oracle's own seeded initial weights, both digest-checked by the GPU test.
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from tests import parity as P          # noqa: E402
from tests.helpers import oracle_batch  # noqa: E402


def _unclipped(grads, norm, clip_on, max_norm):
    """clip_grad_norm_ scaled the oracle's .grad in place: undo it (the GPU
    exports the raw gradient; the clip coefficient is applied inside Adam)"""
    if not clip_on:
        return grads
    coef = min(1.0, max_norm / (norm + 1e-6))
    return {k: v / coef for k, v in grads.items()}


def make(case):
    c = P.CASES[case]
    lc = c['cfg']()
    D, A, pixel = c['D'], c['A'], c['pixel']
    st = P.init_state(case)
    r64, vs = P.envelope(st, lc, D, A, pixel, c['n_ulp'], c['orders'])
    meta = {'case': case, 'init_digest': P.digest([st[k] for k in sorted(st)]),
            'batch_digest': [], 'epochs_run': [], 'width': {}, 'scale': {},
            'variants': len(vs), 'torch': torch.__version__, 'update': {}}
    arrays = {}
    na = lc.algo.network
    for it in range(len(c['batch_seeds'])):
        t0 = time.time()
        batch = P.case_batch(case, it)
        meta['batch_digest'].append(P.batch_digest(batch))
        ob = oracle_batch(batch)
        s64 = r64.learn(ob)
        svs = [v.learn(ob, c['batch_seeds'][it]) for v in vs]
        runs = [s64['epochs_run']] + [s['epochs_run'] for s in svs]
        assert len(set(runs)) == 1, (case, it, runs)
        meta['epochs_run'].append(int(s64['epochs_run']))
        out = {}
        if 'grad' in c:
            ph = c['grad']
            key = 'grad_norm_actor' if ph == 'policy' else 'grad_norm_critic'
            clip_on = na.clip_actor_gradient if ph == 'policy' else na.clip_critic_gradient
            mx = na.actor_gradient_norm_clip if ph == 'policy' else na.critic_gradient_norm_clip
            g64 = _unclipped(P.oracle_grads(r64, ph), s64[key], clip_on, mx)
            gvs = [_unclipped(P.oracle_grads(v.ref, ph), s[key], clip_on, mx)
                   for v, s in zip(vs, svs)]
            for k, v in g64.items():
                out[f'grad_{k}'] = (v, [g[k] for g in gvs])
        else:
            seg = lambda name: [v.per_segment(getattr(v.ref, name).double().numpy()) for v in vs]  # noqa: E731
            out['adv'] = (r64.last_adv.double().numpy(), seg('last_adv'))
            out['ret'] = (r64.last_ret.double().numpy(), seg('last_ret'))
            p64 = P.oracle_params(r64)
            pvs = [P.oracle_params(v.ref) for v in vs]
            for k in p64:
                out[k] = (p64[k], [x[k] for x in pvs])
            if lc.algo.use_z_filter:
                for b in ('running_sum', 'running_sumsq'):
                    out[f'zf_{b}'] = (getattr(r64.model.z_filter, b).double().numpy(),
                                      [getattr(v.ref.model.z_filter, b).double().numpy() for v in vs])
        for name, (r, variants) in out.items():
            key = f'{name}@{it}'
            w, s = P.width(r, variants)
            meta['width'][key], meta['scale'][key] = w, s
            if name in st:            # parameters: the envelope of the update measures
                st0 = np.asarray(st[name], dtype=np.float64)
                u64 = np.asarray(r, np.float64) - st0
                uvs = [np.asarray(v, np.float64) - st0 for v in variants]
                # the mask: entries the fp64 update moved by more than thr,
                # from half an Adam step up -- the first threshold at which the
                # envelope is informative (parity.py UPDATE_MASK_STEPS)
                for mult in P.UPDATE_MASK_STEPS:
                    thr = mult * P.update_thr(lc, name)
                    w_rel, w_cos, n = P.update_widths(u64, uvs, thr)
                    if 2.0 * w_rel + P.UPDATE_SLACK < P.UPDATE_TARGET_BAR:
                        break
                meta['update'][key] = [w_rel, w_cos, thr, n]
                print(f'  {key}: update relL2 width {w_rel:.3e}, 1-cos width {w_cos:.3e}, '
                      f'{n} entries moved > {thr:.1e} ({mult} x lr/2)', flush=True)
            r = np.asarray(r, dtype=np.float64)
            if name in st:            # parameters: fp32 difference from the initial state
                r = r - np.asarray(st[name], dtype=np.float64)
            arrays[key] = r.astype(np.float32)
        print(f'{case} learn {it}: {time.time() - t0:.1f} s, epochs_run {s64["epochs_run"]}', flush=True)
    P.save_fixture(case, meta, arrays)
    print(f'wrote {P.fixture_path(case)}', flush=True)


if __name__ == '__main__':
    torch.set_num_threads(os.cpu_count() or 1)
    for case in (sys.argv[1:] or list(P.CASES)):
        make(case)
