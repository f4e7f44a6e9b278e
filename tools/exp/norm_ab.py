"""A/B of the clip-norm partials (developer check): the c3_adapt fixture's two
learns with the dW reducer's fused sums of squares (default) or the separate
sumsq pass (SMI_FUSED_NORM=0); prints the statistics of both learns as JSON."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from surreal_amd import synthetic  # noqa: E402
from tests import parity as P  # noqa: E402
from tests.test_gpu_parity_pinned import fixture_learner  # noqa: E402

meta, fx, c, st, learner = fixture_learner('c3_adapt')
out = []
for it in range(2):
    learner.learn(synthetic.to_device(P.case_batch('c3_adapt', it), 'cuda:0'))
    s = learner.last_stats()
    out.append({k: s[k] for k in ('grad_norm_critic', 'grad_norm_actor', '_val_loss', 'epochs_run')})
    out[-1]['critic_sum'] = float(learner.model.critic.flat.double().sum())
print(json.dumps({'fused': os.environ.get('SMI_FUSED_NORM', '1'), 'learns': out}), flush=True)
