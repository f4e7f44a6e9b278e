"""Developer check: the GPU's raw critic gradient at the last value epoch of the
c3_adapt fixture's second learn against the fp64 autograd gradient at the
same captured state, per parameter block (where a statistic's error sits)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from surreal_amd import synthetic  # noqa: E402
from tests import parity as P  # noqa: E402
from tests.helpers import oracle_batch  # noqa: E402
from tests.test_gpu_parity_pinned import _used, fixture_learner  # noqa: E402

meta, fx, c, st, learner = fixture_learner('c3_adapt')
lc = c['cfg']()
out = {}
for it in range(2):
    batch = P.case_batch('c3_adapt', it)
    start = P.gpu_state(learner)
    last = None
    for buf in learner._learn_phases(synthetic.to_device(batch, 'cuda:0')):
        if getattr(learner, '_phase_tag', None) == 'value_grad':
            nA = learner.model.actor.flat.numel() + learner.model.rnn_stem.flat.numel()
            nC = learner.model.critic.flat.numel() + learner.model.rnn_stem.flat.numel()
            last = (P.gpu_state(learner), learner._bufs['rnn_xbuf'][nA:nA + nC].double().cpu().numpy())
    adv, ret = _used(learner)
    state, g_gpu = last
    for dt in (torch.float64, torch.float32):
        m = P._stat_model(lc, c['D'], c['A'], None, state, start.get('zf'), dt)
        ob = oracle_batch(batch)
        E = lc.algo.n_step - lc.algo.rnn.horizon + 1
        f = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float32).to(dt)  # noqa: E731
        obs_iter = f(ob['obs'])[:, :E].contiguous()
        cells = (f(ob['onetime'][0]).transpose(0, 1).contiguous(), f(ob['onetime'][1]).transpose(0, 1).contiguous())
        values = m.model.forward_critic(obs_iter, cells)
        if values.dim() == 3:
            values = values.squeeze(2)
        loss = (values - f(ret)).pow(2).mean()
        ps = list(m.model.critic_params())
        gs = torch.autograd.grad(loss, ps, allow_unused=True)
        names = [n for n, _ in m.model.critic.named_parameters()] if hasattr(m.model.critic, 'named_parameters') else []
        flat = torch.cat([g.reshape(-1) for g in gs if g is not None]).double().numpy()
        if dt == torch.float64:
            g64, sizes = flat, [g.numel() for g in gs if g is not None]
        else:
            g32 = flat
    blocks, o = [], 0
    for n in sizes:
        a, b, b32 = g_gpu[o:o + n], g64[o:o + n], g32[o:o + n]
        blocks.append({'n': n, 'norm64': float(np.linalg.norm(b)),
                       'gpu_err': float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30)),
                       'cpu32_err': float(np.linalg.norm(b32 - b) / (np.linalg.norm(b) + 1e-30))})
        o += n
    out[f'learn{it}'] = {'norm_gpu': float(np.linalg.norm(g_gpu)), 'norm64': float(np.linalg.norm(g64)),
                         'norm32': float(np.linalg.norm(g32)), 'blocks': blocks,
                         'len_gpu': int(g_gpu.size), 'len64': int(g64.size)}
print(json.dumps(out, indent=1), flush=True)
