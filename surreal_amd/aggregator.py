"""Learner-side batch aggregation (host numpy), mirroring
surreal/learner/aggregator.py: MultistepAggregatorWithInfo (:106-262) for PPO
and SSARAggregator (:33-103) + FrameStackPreprocessor (:11-31) for DDPG.

Output dictionaries carry the same keys, shapes and dtypes as the reference.
`stage()` additionally packs an aggregated PPO batch into pinned host buffers
so the learner issues one async H2D copy per array.
"""
import collections

import numpy as np
import torch


class FrameStackPreprocessor(object):
    """aggregator.py:11-31: concatenate stacked pixel frames on axis 0."""

    def __init__(self, frame_stacks):
        self.frame_stacks = frame_stacks

    def preprocess_obs(self, obs):
        if 'pixel' in obs:
            for key in obs['pixel']:
                obs['pixel'][key] = np.concatenate(obs['pixel'][key], axis=0)
                assert len(obs['pixel'][key].shape) == 3

    def preprocess_list(self, exp_list):
        for exp in exp_list:
            for obs in (exp['obs'][0], exp['obs'][1]):
                self.preprocess_obs(obs)
        return exp_list


def _action_type(action_spec):
    t = action_spec.get('type', 'continuous')
    return getattr(t, 'name', t)


class SSARAggregator(object):
    """aggregator.py:33-103: list of (s, a, r, s', done) dicts -> batched arrays."""

    def __init__(self, obs_spec, action_spec):
        self.obs_spec = obs_spec
        self.action_spec = action_spec
        self.action_type = _action_type(action_spec)

    def aggregate(self, exp_list):
        obs0, obs1 = collections.OrderedDict(), collections.OrderedDict()
        actions, rewards, dones = [], [], []
        for exp in exp_list:
            for src, dst in ((exp['obs'][0], obs0), (exp['obs'][1], obs1)):
                for modality in src:
                    dst.setdefault(modality, collections.OrderedDict())
                    for key in src[modality]:
                        dst[modality].setdefault(key, []).append(np.asarray(src[modality][key]))
            actions.append(exp['action'])
            rewards.append(exp['reward'])
            dones.append(float(exp['done']))
        if self.action_type == 'continuous':
            actions = np.array(actions, dtype=np.float32)
        elif self.action_type == 'discrete':
            actions = np.array(actions, dtype=np.int32)
        else:
            raise NotImplementedError('action_spec unsupported ' + str(self.action_spec))
        for obs in (obs0, obs1):
            for modality in obs:
                for key in obs[modality]:
                    obs[modality][key] = np.array(obs[modality][key])
        return {'obs': obs0, 'obs_next': obs1, 'actions': np.array(actions),
                'rewards': np.expand_dims(rewards, axis=1),
                'dones': np.expand_dims(dones, axis=1)}


class MultistepAggregatorWithInfo(object):
    """aggregator.py:106-262: n-step sub-trajectories with agent infos.

    persistent_infos: list of (B, T, ...) arrays (the policy pd is [-1]);
    onetime_infos: None or list of (B, ...) arrays (LSTM h, c)."""

    def __init__(self, obs_spec, action_spec):
        self.obs_spec = obs_spec
        self.action_spec = action_spec
        self.action_type = _action_type(action_spec)

    def aggregate(self, exp_list):
        actions, rewards, dones, observations, next_obs = [], [], [], [], []
        for exp in exp_list:
            actions.append(np.stack(exp['actions']))
            rewards.append(np.array(exp['rewards']))
            dones.append(np.array(exp['dones']))
            observations.append(exp['obs'])
            next_obs.append([exp['obs_next']])
        observations = self._batch_obs(observations)
        next_obs = self._batch_obs(next_obs)
        if self.action_type not in ('continuous',):
            raise NotImplementedError('action_spec unsupported ' + str(self.action_spec))
        onetime_infos, persistent_infos = self._gather_action_infos(exp_list)
        return {'obs': observations, 'obs_next': next_obs, 'actions': np.stack(actions),
                'rewards': np.stack(rewards), 'persistent_infos': persistent_infos,
                'onetime_infos': onetime_infos, 'dones': np.stack(dones).astype('float32')}

    def _batch_obs(self, traj_list):
        batched = {}
        for modality in self.obs_spec.keys():
            batched[modality] = {}
            for key in self.obs_spec[modality].keys():
                batched[modality][key] = np.stack(
                    [np.stack([o[modality][key] for o in traj]) for traj in traj_list])
        return batched

    def _gather_action_infos(self, exp_list):
        first = exp_list[0]
        has_one = len(first['onetime_infos']) > 0
        has_pers = len(first['persistent_infos'][0]) > 0
        onetime = [[] for _ in range(len(first['onetime_infos']))] if has_one else None
        pers = [[] for _ in range(len(first['persistent_infos'][0]))] if has_pers else None
        for exp in exp_list:
            if has_one:
                for i in range(len(onetime)):
                    onetime[i].append(exp['onetime_infos'][i])
            if has_pers:
                for i in range(len(pers)):
                    pers[i].append(np.stack([step[i] for step in exp['persistent_infos']]))
        if has_one:
            onetime = [np.stack(x) for x in onetime]
        if has_pers:
            pers = [np.asarray(x) for x in pers]
        return onetime, pers


def stage(batch, device, pinned_cache=None):
    """Pinned-memory staging of an aggregated PPO batch + async H2D copies.

    Returns the same nested structure with float32 device tensors.  The copies
    are enqueued on the current stream (non_blocking) so learn() can follow
    without a host sync."""
    cache = pinned_cache if pinned_cache is not None else {}

    def put(key, arr):
        if arr is None:
            return None
        # camera observations stay uint8 (4x fewer bytes over PCIe; the conv
        # kernel applies the /255 of ppo_net.py:368-375)
        u8 = isinstance(key, tuple) and len(key) == 3 and key[1] == 'pixel'
        dt, ndt = (torch.uint8, np.uint8) if u8 else (torch.float32, np.float32)
        if isinstance(arr, torch.Tensor):
            return arr.to(device=device, dtype=dt, non_blocking=True)
        a = np.ascontiguousarray(arr, dtype=ndt)
        ent = cache.get(key)
        if ent is None or tuple(ent[0].shape) != a.shape:
            ent = [torch.empty(a.shape, dtype=dt).pin_memory(), torch.cuda.Event()]
            cache[key] = ent
        else:
            ent[1].synchronize()          # the previous async copy out of this buffer is done
        ent[0].numpy()[...] = a
        dev = ent[0].to(device=device, non_blocking=True)
        ent[1].record()
        return dev

    out = {}
    for name in ('obs', 'obs_next'):
        out[name] = {m: {k: put((name, m, k), v) for k, v in d.items()}
                     for m, d in batch[name].items()}
    for name in ('actions', 'rewards', 'dones'):
        out[name] = put(name, batch[name])
    pi = batch.get('persistent_infos')
    out['persistent_infos'] = None if pi is None else [put(('pi', i), x) for i, x in enumerate(pi)]
    oi = batch.get('onetime_infos')
    out['onetime_infos'] = None if oi is None else [put(('oi', i), x) for i, x in enumerate(oi)]
    return out
