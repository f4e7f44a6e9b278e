"""Developer tool: where do pixel-only CNN parameter differences sit?"""
import sys
import numpy as np
import torch
sys.path.insert(0, '/root/repo')
from oracle import ppo_ref as R  # noqa: E402
from surreal_amd import synthetic  # noqa: E402
from surreal_amd.config import pixel_env_config  # noqa: E402
from surreal_amd.learner import PPOLearner  # noqa: E402
from tests import test_gpu_cnn as TC  # noqa: E402
from tests.helpers import copy_weights_to_oracle, oracle_batch, seq_flat  # noqa: E402

CAM = (3, 84, 84)
for (D, epochs) in ((0, (1, 1)), (0, (2, 2)), (0, (1, 0)), (0, (0, 1)), (7, (2, 2))):
    B, T, H, A, Hd, F = 5, 5, 2, 2, 12, 24
    lc = TC._pixel_cfg('adapt', B, T, H, Hd, (16, 16), F, D > 0, epochs)
    learner = PPOLearner(lc, pixel_env_config(D, A, CAM), seed=9)
    ref = R.PPOLearnerRef(lc, D, A, pixel=CAM)
    copy_weights_to_oracle(learner, ref)
    batch = synthetic.ppo_batch(B, T, D, A, seed=50, rnn_hidden=Hd, pixel=CAM)
    ref.learn(oracle_batch(batch))
    learner.learn(synthetic.to_device(batch, 'cuda'))
    got = learner.model.cnn_stem.flat.cpu().double().numpy()
    exp = seq_flat(ref.model.cnn_stem).double().numpy()
    floor = 1e-2 * np.abs(exp).max()
    bad = np.abs(got - exp) / (np.abs(exp) + floor) > 1e-5
    segs = [('w1', 3072), ('b1', 16), ('w2', 8192), ('b2', 32), ('wf', F * 2592), ('bf', F)]
    o = 0
    out = {}
    for n, c in segs:
        out[n] = int(bad[o:o + c].sum())
        if n == 'wf':
            rows = bad[o:o + c].reshape(F, 2592).sum(1)
            out['wf_rows'] = rows.tolist()
        o += c
    print(D, epochs, out, 'maxdiff', float(np.abs(got - exp).max()), flush=True)
