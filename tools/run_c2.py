"""Developer tool: N learn() calls of the bench's C2 configuration, for
profilers that attach to a whole process (rocprofv3 --pmc / --kernel-trace):
    rocprofv3 --pmc SQ_WAVES -- python3 tools/run_c2.py 20
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(n):
    from surreal_amd import synthetic
    from surreal_amd.learner import PPOLearner
    from tests.helpers import env_config, ppo_config
    lc = ppo_config(B=64, T=50, mode='adapt', use_z_filter=True, epochs=(10, 10), lr=(1e-5, 1e-5))
    learner = PPOLearner(lc, env_config(17, 6), seed=1)
    batch = synthetic.to_device(synthetic.ppo_batch(64, 50, 17, 6, seed=0), 'cuda')
    for _ in range(n):
        learner.learn(batch)
    torch.cuda.synchronize()
    print('done', n, flush=True)


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
