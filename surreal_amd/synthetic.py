"""Seeded synthetic learner batches shaped like the output of
MultistepAggregatorWithInfo.aggregate (surreal/learner/aggregator.py:151-184).

obs ~ N(0,1)*(1 + i/D) per feature; obs_next likewise; rewards ~ N(0,1);
dones ~ Bernoulli(0.02) with the last step forced to 1 for 5% of segments;
behaviour policy: mu ~ U(-0.5, 0.5), sigma = exp(init_log_sig) * U(0.8, 1.2);
actions are drawn from the behaviour policy (what PPOAgent.act samples,
surreal/agent/ppo_agent.py:103-151, via DiagGauss.sample) and clipped to
[-1, 1]; LSTM h, c ~ N(0, 0.1).  With pixel=(C, H, W), camera0 frames are
uniform uint8 (drawn after everything else, so the low-dim streams do not
change); D == 0 drops the low-dim modality.
"""
import numpy as np
import torch


def ppo_batch(B, T, D, A, seed=0, init_log_sig=-1.0, rnn_hidden=None, rnn_layers=1,
              obs_key='flat_inputs', pixel=None):
    g = torch.Generator().manual_seed(seed)
    scale = 1.0 + torch.arange(D, dtype=torch.float32) / D
    obs = torch.randn(B, T, D, generator=g) * scale
    obs_next = torch.randn(B, 1, D, generator=g) * scale
    rewards = torch.randn(B, T, generator=g)
    dones = (torch.rand(B, T, generator=g) < 0.02).float()
    last = torch.rand(B, generator=g) < 0.05
    dones[last, T - 1] = 1.0
    mu = torch.rand(B, T, A, generator=g) - 0.5
    sd = float(np.exp(init_log_sig)) * (0.8 + 0.4 * torch.rand(B, T, A, generator=g))
    actions = (mu + sd * torch.randn(B, T, A, generator=g)).clamp(-1.0, 1.0)
    pds = torch.cat([mu, sd], dim=-1)
    onetime = None
    if rnn_hidden:
        onetime = [0.1 * torch.randn(B, rnn_layers, rnn_hidden, generator=g),
                   0.1 * torch.randn(B, rnn_layers, rnn_hidden, generator=g)]
    o, on = {}, {}
    if D:
        o['low_dim'] = {obs_key: obs}
        on['low_dim'] = {obs_key: obs_next}
    if pixel is not None:
        o['pixel'] = {'camera0': torch.randint(0, 256, (B, T) + tuple(pixel), generator=g,
                                               dtype=torch.uint8)}
        on['pixel'] = {'camera0': torch.randint(0, 256, (B, 1) + tuple(pixel), generator=g,
                                                dtype=torch.uint8)}
    return {
        'obs': o,
        'obs_next': on,
        'actions': actions,
        'rewards': rewards,
        'dones': dones,
        'persistent_infos': [pds],
        'onetime_infos': onetime,
    }


def to_device(batch, device):
    def mv(x):
        if x is None:
            return None
        if isinstance(x, dict):
            return {k: mv(v) for k, v in x.items()}
        if isinstance(x, list):
            return [mv(v) for v in x]
        return x.to(device).contiguous()
    return mv(batch)


def ddpg_batch(B, D, A, seed=0):
    g = torch.Generator().manual_seed(seed)
    return {
        'obs': torch.randn(B, D, generator=g),
        'actions': (torch.rand(B, A, generator=g) * 2 - 1),
        'rewards': torch.randn(B, 1, generator=g),
        'obs_next': torch.randn(B, D, generator=g),
        'dones': (torch.rand(B, 1, generator=g) < 0.05).float(),
    }
