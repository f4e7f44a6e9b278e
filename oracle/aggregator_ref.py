"""ORACLE (test infrastructure only — see oracle/__init__.py).

Loop-for-loop restatement of the reference's learner-side batch aggregation
(surreal/learner/aggregator.py), kept in plain Python + numpy with the same
per-item np.stack / np.array calls, so the dtypes and byte layout that fall
out of numpy's promotion rules are the reference's:

  SSARAggregator.aggregate                  aggregator.py:52-103
  MultistepAggregatorWithInfo.aggregate     aggregator.py:151-184
    _batch_obs                              aggregator.py:186-205
    _stack_n_step_experience                aggregator.py:207-221
    _gather_action_infos                    aggregator.py:223-262

`make_ppo_exp_list` / `make_ssar_exp_list` build experience lists in the form
the reference's senders emit them (ExpSenderWrapperMultiStepMovingWindowWithInfo.send,
surreal/env/exp_sender_wrapper.py:230-264, fed by PPOAgent.act,
surreal/agent/ppo_agent.py:121-151; ExpSenderWrapperSSAR, exp_sender_wrapper.py:50-67):
python-float rewards, bool dones, per-step [pd] persistent infos, the first
step's [h, c] (rnn_layer, hidden) LSTM cells as one-time infos.
"""
import collections

import numpy as np


class MultistepAggregatorWithInfoRef:
    def __init__(self, obs_spec):
        self.obs_spec = obs_spec

    def aggregate(self, exp_list):                                   # :151-184
        observations, next_obs, actions, rewards, dones = [], [], [], [], []
        for exp in exp_list:
            a, r, d = self._stack_n_step_experience(exp)
            actions.append(a)
            rewards.append(r)
            dones.append(d)
            observations.append(exp['obs'])
            next_obs.append([exp['obs_next']])
        observations = self._batch_obs(observations)
        next_obs = self._batch_obs(next_obs)
        onetime_infos, persistent_infos = self._gather_action_infos(exp_list)
        return {'obs': observations, 'obs_next': next_obs, 'actions': np.stack(actions),
                'rewards': np.stack(rewards), 'persistent_infos': persistent_infos,
                'onetime_infos': onetime_infos, 'dones': np.stack(dones).astype('float32')}

    def _batch_obs(self, traj_list):                                  # :186-205
        out = {}
        for modality in self.obs_spec.keys():
            out[modality] = {}
            for key in self.obs_spec[modality].keys():
                per_traj = []
                for traj in traj_list:
                    steps = []
                    for ob in traj:
                        steps.append(ob[modality][key])
                    per_traj.append(np.stack(steps))
                out[modality][key] = np.stack(per_traj)
        return out

    @staticmethod
    def _stack_n_step_experience(exp):                               # :207-221
        return np.stack(exp['actions']), np.array(exp['rewards']), np.array(exp['dones'])

    @staticmethod
    def _gather_action_infos(exp_list):                              # :223-262
        persistent, onetime = None, None
        has_one = len(exp_list[0]['onetime_infos']) > 0
        has_pers = len(exp_list[0]['persistent_infos'][0]) > 0
        if has_one:
            onetime = [[] for _ in range(len(exp_list[0]['onetime_infos']))]
        if has_pers:
            persistent = [[] for _ in range(len(exp_list[0]['persistent_infos'][0]))]
        for exp in exp_list:
            if has_one:
                for i in range(len(onetime)):
                    onetime[i].append(exp['onetime_infos'][i])
            if has_pers:
                for i in range(len(persistent)):
                    per_step = []
                    for info_list in exp['persistent_infos']:
                        per_step.append(info_list[i])
                    persistent[i].append(np.stack(per_step))
        if has_one:
            onetime = [np.stack(x) for x in onetime]
        if has_pers:
            persistent = [np.asarray(x) for x in persistent]
        return onetime, persistent


class SSARAggregatorRef:
    def aggregate(self, exp_list, discrete=False):                    # :52-103
        obs0, obs1 = collections.OrderedDict(), collections.OrderedDict()
        actions, rewards, dones = [], [], []
        for exp in exp_list:
            for src, dst in ((exp['obs'][0], obs0), (exp['obs'][1], obs1)):
                for modality in src:
                    if modality not in dst:
                        dst[modality] = collections.OrderedDict()
                    for key in src[modality]:
                        if key not in dst[modality]:
                            dst[modality][key] = []
                        dst[modality][key].append(np.asarray(src[modality][key]))
            actions.append(exp['action'])
            rewards.append(exp['reward'])
            dones.append(float(exp['done']))
        actions = np.array(actions, dtype=np.int32 if discrete else np.float32)
        for obs in (obs0, obs1):
            for modality in obs:
                for key in obs[modality]:
                    obs[modality][key] = np.array(obs[modality][key])
        return {'obs': obs0, 'obs_next': obs1, 'actions': np.array(actions),
                'rewards': np.expand_dims(rewards, axis=1), 'dones': np.expand_dims(dones, axis=1)}


# ------------------------------------------------------------- experience lists
def ppo_exp_arrays(B, T, D, A, seed, rnn_hidden=None, rnn_layers=1, pixel=None):
    """The numbers behind a PPO experience list (seeded numpy): obs as float64
    (what a gym/robosuite env returns), actions float64 (DiagGauss.sample on a
    float32 pd), pds float32 (torch output), rewards float64, dones bool, LSTM
    cells float32."""
    rs = np.random.RandomState(seed)
    arr = {
        'obs': rs.randn(B, T, D),
        'obs_next': rs.randn(B, D),
        'pds': np.concatenate([rs.uniform(-.5, .5, (B, T, A)),
                               np.exp(-1.0) * rs.uniform(.8, 1.2, (B, T, A))], -1).astype(np.float32),
        'rewards': rs.randn(B, T),
        'dones': rs.uniform(size=(B, T)) < 0.05,
    }
    arr['actions'] = np.clip(arr['pds'][..., :A] + arr['pds'][..., A:] * rs.randn(B, T, A), -1, 1)
    if rnn_hidden:
        arr['h'] = (0.1 * rs.randn(B, rnn_layers, rnn_hidden)).astype(np.float32)
        arr['c'] = (0.1 * rs.randn(B, rnn_layers, rnn_hidden)).astype(np.float32)
    if pixel is not None:
        arr['pix'] = rs.randint(0, 256, (B, T) + tuple(pixel)).astype(np.uint8)
        arr['pix_next'] = rs.randint(0, 256, (B,) + tuple(pixel)).astype(np.uint8)
    return arr


def make_ppo_exp_list(arr, obs_key='flat_inputs'):
    """exp dicts as ExpSenderWrapperMultiStepMovingWindowWithInfo.send builds
    them (exp_sender_wrapper.py:237-263)."""
    B, T = arr['rewards'].shape
    exps = []
    for b in range(B):
        obs, actions, rewards, dones, pers = [], [], [], [], []
        for t in range(T):
            ob = {'low_dim': {obs_key: arr['obs'][b, t]}}
            if 'pix' in arr:
                ob['pixel'] = {'camera0': arr['pix'][b, t]}
            obs.append(ob)
            actions.append(arr['actions'][b, t])
            rewards.append(float(arr['rewards'][b, t]))
            dones.append(bool(arr['dones'][b, t]))
            pers.append([arr['pds'][b, t]])
        nxt = {'low_dim': {obs_key: arr['obs_next'][b]}}
        if 'pix' in arr:
            nxt['pixel'] = {'camera0': arr['pix_next'][b]}
        onetime = [arr['h'][b], arr['c'][b]] if 'h' in arr else []
        exps.append({'obs': obs, 'obs_next': nxt, 'actions': actions, 'rewards': rewards,
                     'dones': dones, 'persistent_infos': pers, 'onetime_infos': onetime,
                     'infos': [{}] * T, 'n_step': T})
    return exps


def ssar_exp_arrays(B, D, A, seed):
    rs = np.random.RandomState(seed)
    return {'obs': rs.randn(B, D), 'obs_next': rs.randn(B, D),
            'actions': rs.uniform(-1, 1, (B, A)), 'rewards': rs.randn(B),
            'dones': rs.uniform(size=B) < 0.1}


def make_ssar_exp_list(arr, obs_key='flat_inputs'):
    """exp dicts as ExpSenderWrapperSSAR.send builds them (exp_sender_wrapper.py:50-67)."""
    out = []
    for b in range(arr['rewards'].shape[0]):
        out.append({'obs': [{'low_dim': {obs_key: arr['obs'][b]}},
                            {'low_dim': {obs_key: arr['obs_next'][b]}}],
                    'action': arr['actions'][b], 'reward': float(arr['rewards'][b]),
                    'done': bool(arr['dones'][b]), 'info': {}})
    return out
