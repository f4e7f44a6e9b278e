"""Learner-side batch aggregation (host numpy), mirroring
surreal/learner/aggregator.py: MultistepAggregatorWithInfo (:106-262) for PPO
and SSARAggregator (:33-103) + FrameStackPreprocessor (:11-31) for DDPG.

Output dictionaries carry the same keys, shapes and dtypes as the reference.
`StagingArena` packs an aggregated batch into one pinned host buffer and moves
it to the device with a single async H2D copy.
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


class StagingArena(object):
    """Learner-side staging of an aggregated batch (SURVEY.md §8(f) rank 2;
    the reference converts array by array with torch.tensor, ppo.py:420-484,
    after LearnerDataPrefetcher hands the batch over, data_fetcher.py:53-58).

    Every array of the batch is packed (converted to float32, camera frames kept
    uint8) into ONE pinned host buffer at 256-byte aligned offsets, and the
    whole buffer goes to the device in ONE async H2D copy on the current
    stream; the returned tensors are views into the device buffer.  Two slots
    alternate, so packing batch k+1 overlaps the copy / learn() of batch k; a
    slot's host side is reused only after its previous copy has completed (an
    event), and its device side is overwritten by a copy that is stream-ordered
    after every kernel that read it."""

    ALIGN = 256

    def __init__(self, device, slots=2):
        self.device = torch.device(device)
        self.slots = [None] * slots
        self.next = 0

    @staticmethod
    def _leaves(batch):
        out = []

        def walk(path, v):
            if v is None:
                return
            if isinstance(v, dict):
                for k in v:
                    walk(path + (k,), v[k])
            elif isinstance(v, (list, tuple)):
                for i, x in enumerate(v):
                    walk(path + (i,), x)
            else:
                out.append((path, v))
        for name in ('obs', 'obs_next', 'actions', 'rewards', 'dones', 'persistent_infos',
                     'onetime_infos'):
            walk((name,), batch.get(name))
        return out

    @staticmethod
    def _is_pixel(path):
        return len(path) == 3 and path[0] in ('obs', 'obs_next') and path[1] == 'pixel'

    def stage(self, batch):
        leaves = self._leaves(batch)
        layout, off = [], 0
        for path, v in leaves:
            dt = np.uint8 if self._is_pixel(path) else np.float32
            shape = tuple(v.shape)
            n = int(np.prod(shape)) * np.dtype(dt).itemsize
            layout.append((path, shape, dt, off, n))
            off += (n + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        total = max(off, self.ALIGN)
        key = tuple((p, s, d) for p, s, d, _, _ in layout)
        slot = self.slots[self.next]
        if slot is None or slot['key'] != key:
            slot = {'key': key, 'host': torch.empty(total, dtype=torch.uint8).pin_memory(),
                    'dev': torch.empty(total, dtype=torch.uint8, device=self.device),
                    'event': None}
            self.slots[self.next] = slot
        elif slot['event'] is not None:
            slot['event'].synchronize()       # this host buffer's previous copy is done
        self.next = (self.next + 1) % len(self.slots)
        hbytes = slot['host'].numpy()
        for (path, v), (_, shape, dt, o, n) in zip(leaves, layout):
            dst = hbytes[o:o + n].view(dt).reshape(shape)
            src = v.numpy() if isinstance(v, torch.Tensor) else v
            np.copyto(dst, src, casting='unsafe')
        slot['dev'].copy_(slot['host'], non_blocking=True)        # the single H2D
        ev = torch.cuda.Event()
        ev.record()
        slot['event'] = ev
        views = {}
        for path, shape, dt, o, n in layout:
            t = slot['dev'][o:o + n].view(torch.uint8 if dt == np.uint8 else torch.float32)
            views[path] = t.view(shape)
        return self._rebuild(batch, views)

    @staticmethod
    def _rebuild(batch, views):
        def build(path, v):
            if v is None:
                return None
            if isinstance(v, dict):
                return {k: build(path + (k,), v[k]) for k in v}
            if isinstance(v, (list, tuple)):
                return [build(path + (i,), x) for i, x in enumerate(v)]
            return views[path]
        out = dict(batch)
        for name in ('obs', 'obs_next', 'actions', 'rewards', 'dones', 'persistent_infos',
                     'onetime_infos'):
            out[name] = build((name,), batch.get(name))
        return out


def stage(batch, device, arena=None):
    """Stage an aggregated (host numpy) PPO batch on `device` through a
    StagingArena (one pinned buffer, one async H2D on the current stream)."""
    arena = arena if arena is not None else StagingArena(device)
    return arena.stage(batch)
