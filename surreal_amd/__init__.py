"""surreal_amd — MI355X-native (gfx950) hot path of SURREAL's centralized learner.

Drop-in mirrors of the reference Python API whose compute runs in the HIP
kernels of libsurreal_mi.so (C ABI: include/surreal_mi.h):
  learner.PPOLearner / learner.DDPGLearner   surreal/learner/{ppo,ddpg}.py
  model.PPOModel / ZFilter / DiagGauss / RewardFilter   surreal/model/*
  replay.UniformReplay / FIFOReplay          surreal/replay/*
  aggregator.MultistepAggregatorWithInfo / SSARAggregator  surreal/learner/aggregator.py
"""
__version__ = '0.1.0'
