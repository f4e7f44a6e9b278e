"""Batched actor inference on the MI355X kernels.

The reference runs one actor process per environment, each calling act() on
ONE observation at a time (surreal/agent/ppo_agent.py:103-151,
ddpg_agent.py:153-182).  Here N agents share one GPU model: act() takes the N
agents' observations, stages them in one H2D copy, runs the policy forward for
all N rows (ZFilter -> [CNN] -> one LSTM step from each agent's own cells ->
actor MLP, on the same HIP kernels as the learner), copies the N policies back
in one D2H, and samples in numpy in agent order — so the action of agent i is
exactly what the i-th of N sequential reference agents sharing numpy's global
RNG would draw.  The returned action infos keep the reference's per-agent
format: onetime [h, c] (rnn_layer, hidden) cells before the step, persistent
[pd] (2A,).

Parameters come from the learner's modules (load_module_dict) or from a
published numpy dict (load_numpy: ModuleDict.load, distributed/module_dict.py:47-63).
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib as L
from .config import Config
from .model import PPOModel


def _np_state_to_torch(sd):
    """ModuleDict.load: every array cast to float32 (np_cast) and wrapped."""
    return {k: torch.from_numpy(np.asarray(v, dtype=np.float32)) for k, v in sd.items()}


class PPOAgentBatch(object):
    """N PPO actors (agent_mode 'training' | 'eval_stochastic' | 'eval_deterministic')."""

    def __init__(self, learner_config, env_config, n_agents, agent_mode='training', device=None,
                 seed=0):
        L.require_gpu()
        lc = learner_config if isinstance(learner_config, Config) else Config(learner_config)
        ec = env_config if isinstance(env_config, Config) else Config(env_config)
        self.n = int(n_agents)
        self.agent_mode = agent_mode
        self.action_dim = ec.action_spec['dim'][0]
        self.device = torch.device(device) if device is not None else torch.device('cuda')
        self._ctx = L.Context(self.device)      # own workspace (re-entrancy)
        algo = lc.algo
        self.rnn = algo.rnn if algo.rnn.if_rnn_policy else None
        self.model = PPOModel(ec.obs_spec, self.action_dim, lc.model, True, algo.consts.init_log_sig,
                              algo.use_z_filter, bool(ec.get('pixel_input', False)), algo.rnn,
                              self.device, torch.Generator().manual_seed(seed))
        log_sig_range = algo.consts.log_sig_range
        # per-agent log-sigma exploration noise, drawn as each reference agent
        # draws it at construction (ppo_agent.py:56-60)
        self.noise = np.zeros(self.n)
        if agent_mode == 'training':
            self.noise = np.array([np.random.uniform(low=-log_sig_range, high=log_sig_range)
                                   for _ in range(self.n)])
        self.cells = None
        if self.rnn is not None:
            L_, H = self.rnn.rnn_layer, self.rnn.rnn_hidden
            self.cells = (torch.zeros(L_, self.n, H, device=self.device),
                          torch.zeros(L_, self.n, H, device=self.device))

    def load_module_dict(self, module_dict):
        self.model.load_state_dict(module_dict['ppo'].state_dict())

    def load_numpy(self, numpy_dict):
        self.model.load_state_dict(_np_state_to_torch(numpy_dict['ppo']))

    def reset(self, agents=None):
        """ppo_agent.py:166-180 for the given agent indices (all by default)."""
        if self.cells is not None:
            idx = slice(None) if agents is None else list(agents)
            self.cells[0][:, idx] = 0
            self.cells[1][:, idx] = 0

    def act(self, obs):
        """obs: {modality: {key: array (N, ...)}} for the N agents.
        Returns (actions (N, A) float64, [action_info per agent]) in training
        mode (actions only otherwise), like N reference act() calls."""
        self._ctx.make_current()
        A = self.action_dim
        dev_obs = {}
        for mod, d in obs.items():
            dev_obs[mod] = {}
            for k, v in d.items():
                arr = np.asarray(v)
                dt = torch.uint8 if mod == 'pixel' else torch.float32
                t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.uint8 if mod == 'pixel'
                                                          else np.float32))
                dev_obs[mod][k] = t.to(self.device, non_blocking=False).to(dt)
        if self.cells is not None:
            h_prev = self.cells[0].transpose(0, 1).cpu().numpy()     # (N, L, H)
            c_prev = self.cells[1].transpose(0, 1).cpu().numpy()
            x = self.model._stem_input(dev_obs)                       # (N, D [+F])
            out, cells = self.model.rnn_stem(x.reshape(self.n, 1, -1).contiguous(), self.cells)
            self.cells = cells
            pd = self.model.actor(out.reshape(self.n, -1))
        else:
            pd = self.model.forward_actor(dev_obs)
        pd = pd.cpu().numpy()                                        # one D2H
        pd[:, A:] *= np.exp(self.noise)[:, None]          # float64 product, stored fp32 (as the reference)
        if self.agent_mode != 'eval_deterministic':
            act = np.random.randn(self.n, A) * pd[:, A:] + pd[:, :A]  # DiagGauss.sample, agent order
        else:
            act = pd[:, :A].copy()                                    # DiagGauss.maxprob
        np.clip(act, -1, 1, out=act)
        if self.agent_mode != 'training':
            return act
        infos = []
        for i in range(self.n):
            one = [h_prev[i], c_prev[i]] if self.cells is not None else []
            infos.append([one, [pd[i].copy()]])
        return act, infos


class DDPGAgentBatch(object):
    """N DDPG actors with their own exploration noise processes
    (ddpg_agent.py:103-182; action_noise.py:9-40) and, when configured, their
    own parameter-space noise (param_noise.py:9-72, ddpg_agent.py:134-151,172-173):
    every fetched parameter set is perturbed once per agent (numpy's global
    RNG, agents in order, each agent's state_dict keys in order), so each
    agent acts with its own perturbed perception + actor.  'adaptive_normal'
    keeps the unperturbed parameters, measures every compute_dist_interval-th
    act the distance between the unperturbed and perturbed actions, and scales
    each agent's sigma by alpha at the next fetch."""

    PN_DIST_INTERVAL = 10                     # AdaptiveNormalParameterNoise default

    def __init__(self, learner_config, env_config, n_agents, agent_mode='training', device=None,
                 seed=0, agent_ids=None, num_agents=None):
        """agent_ids / num_agents: the reference agents' ids and env_config.num_agents,
        which set each agent's exploration sigma (ddpg_agent.py:78-83: max_sigma / 3
        for a single agent, else max_sigma * id / num_agents)."""
        from .ddpg import DDPGModel
        L.require_gpu()
        lc = learner_config if isinstance(learner_config, Config) else Config(learner_config)
        ec = env_config if isinstance(env_config, Config) else Config(env_config)
        self.n = int(n_agents)
        self.agent_mode = agent_mode
        self.action_dim = ec.action_spec['dim'][0]
        self.device = torch.device(device) if device is not None else torch.device('cuda')
        self._ctx = L.Context(self.device)      # own workspace (re-entrancy)
        cs = lc.model.get('conv_spec', {})       # the learner's perception (ddpg.py:135-143)
        self.model = DDPGModel(ec.obs_spec, self.action_dim, lc.model.use_layernorm,
                               lc.model.actor_fc_hidden_sizes, lc.model.critic_fc_hidden_sizes,
                               conv_out_channels=cs.get('out_channels'),
                               conv_kernel_sizes=cs.get('kernel_sizes'), conv_strides=cs.get('strides'),
                               conv_hidden_dim=cs.get('hidden_output_dim'),
                               device=self.device, generator=torch.Generator().manual_seed(seed))
        self.frame_stack_concatenate_on_env = bool(ec.get('frame_stack_concatenate_on_env', True))
        exp = lc.algo.exploration
        self.param_noise_type = exp.get('param_noise_type')
        if self.param_noise_type not in (None, 'normal', 'adaptive_normal'):
            raise ValueError('Param noise type {} undefined.'.format(self.param_noise_type))
        if agent_mode == 'eval_deterministic':   # _init_noise returns early (ddpg_agent.py:121-122)
            self.param_noise_type = None
        if self.param_noise_type is not None:
            self.pn_sigma = np.full(self.n, float(exp.get('param_noise_sigma', 0.05)))
            self.pn_alpha = float(exp.get('param_noise_alpha', 1.15))
            self.pn_target = float(exp.get('param_noise_target_stddev', 0.005))
            self.pn_i = np.zeros(self.n, dtype=np.int64)        # acts since the last fetch
            self.pn_dist = [0.0] * self.n                      # total_action_distance
            self._pn_flats = None      # per agent: perturbed [perception | actor] device images
            self._pn_orig = None       # the fetched (unperturbed) images
            self._pn_stack = None      # [N][P] perturbed actors (batched acting)
            # SMI_PN_BATCHED=0: one forward per agent (A/B, and the pixel /
            # LayerNorm forms always)
            self._batched_pn = os.environ.get('SMI_PN_BATCHED', '1') != '0'
        if exp.noise_type not in ('normal', 'ou_noise'):
            raise ValueError('Noise type {} undefined.'.format(exp.noise_type))
        self.noise_type = exp.noise_type
        ids = np.arange(self.n) if agent_ids is None else np.asarray(agent_ids)
        total = self.n if num_agents is None else int(num_agents)
        self.sigma = (np.full(self.n, exp.max_sigma / 3.0) if total == 1
                      else exp.max_sigma * (ids.astype(np.float64) / total))
        self.theta = exp.theta
        self.dt = exp.dt
        self.x_prev = np.zeros((self.n, self.action_dim))

    def load_module_dict(self, module_dict):
        self.model.load_state_dict(module_dict['ddpg'].state_dict())

    def load_numpy(self, numpy_dict):
        """on_parameter_fetched (ddpg_agent.py:134-137): the published numpy
        parameters, perturbed per agent when parameter noise is configured"""
        if self.param_noise_type is None:
            self.model.load_state_dict(_np_state_to_torch(numpy_dict['ddpg']))
            return
        self._apply_param_noise(numpy_dict)

    def _acting_flats(self):
        m = self.model
        return [x.flat for x in (m.perception, m.actor) if x is not None]

    def _apply_param_noise(self, numpy_dict):
        sd = numpy_dict['ddpg']
        # the unperturbed set (AdaptiveNormalParameterNoise.original_model)
        self.model.load_state_dict(_np_state_to_torch(sd))
        self._pn_orig = [f.detach().clone() for f in self._acting_flats()]
        self._pn_flats = []
        for i in range(self.n):
            if self.param_noise_type == 'adaptive_normal':
                if self.pn_i[i] > 0:                            # param_noise.py:53-60
                    mean_dist = self.pn_dist[i] / self.pn_i[i]
                    if mean_dist > self.pn_target:
                        self.pn_sigma[i] /= self.pn_alpha
                    else:
                        self.pn_sigma[i] *= self.pn_alpha
                self.pn_i[i] = 0
            noisy = {}
            for k, v in sd.items():                             # param_noise.py:17-24 / 63-70
                v = np.asarray(v)
                noisy[k] = v + np.random.normal(0, self.pn_sigma[i], size=tuple(v.shape))
            self.model.load_state_dict(_np_state_to_torch(noisy))
            self._pn_flats.append([f.detach().clone() for f in self._acting_flats()])
        self._set_flats(self._pn_orig)
        # the N perturbed actors stacked [N][P] for one batched forward
        # (smi_mlp3_forward_stacked): low-dim observations, no LayerNorm
        m = self.model
        self._pn_stack = None
        if not m.is_pixel_input and not m.actor.use_layernorm and self._batched_pn:
            self._pn_stack = torch.stack([fl[-1] for fl in self._pn_flats]).contiguous()

    def _set_flats(self, imgs):
        for f, img in zip(self._acting_flats(), imgs):
            f.copy_(img)

    def reset(self, agents=None):
        idx = slice(None) if agents is None else list(agents)
        self.x_prev[idx] = 0.0

    def _noise(self):
        A = self.action_dim
        if self.noise_type == 'normal':                  # NormalActionNoise, per agent in order
            mu = np.zeros((self.n, A))
            return np.random.normal(mu, np.ones((self.n, A)) * self.sigma[:, None])
        # OrnsteinUhlenbeckActionNoise (mu = 0), per agent in order
        x = self.x_prev + self.theta * (np.zeros((self.n, A)) - self.x_prev) * self.dt + \
            (self.sigma[:, None] * np.sqrt(self.dt)) * np.random.normal(size=(self.n, A))
        self.x_prev = x
        return x

    def _act_param_noise(self, obs, x):
        """each agent's action from its own perturbed perception + actor (one
        forward per agent); adaptive: every PN_DIST_INTERVAL-th call the
        unperturbed model's actions give total_action_distance
        (param_noise.py:41-46: assigned, not accumulated, as the reference does)"""
        m = self.model
        if self._pn_stack is not None:
            a = self._act_stacked(x)
        else:      # pixel perception or LayerNorm actors: one forward per agent
            rows = []
            for i in range(self.n):
                self._set_flats(self._pn_flats[i])
                xi = self._perceive_row(obs, i) if m.is_pixel_input else x[i:i + 1]
                rows.append(m.forward_actor(xi))
            a = torch.cat(rows, 0)
            self._set_flats(self._pn_orig)
        if self.param_noise_type == 'adaptive_normal':
            due = [i for i in range(self.n) if self.pn_i[i] % self.PN_DIST_INTERVAL == 0]
            if due:
                a0 = m.forward_actor(x)                # x: the unperturbed perception
                for i in due:
                    self.pn_dist[i] = float(((a0[i] - a[i]) ** 2).sum() ** 0.5)
            self.pn_i += 1
        return a

    def _act_stacked(self, x):
        """the N agents' perturbed actors as ONE launch: row i of x through
        parameter set i of the [N][P] stack"""
        act = self.model.actor
        D, h1, h2, A = act.dims
        offs = (ctypes.c_int64 * 6)(*[act.off(p) for wb in (act.wb(0), act.wb(1), act.wb(2))
                                      for p in wb])
        x = x.contiguous()
        y = torch.empty(self.n, A, dtype=torch.float32, device=self.device)
        st = self._pn_stack
        L.call('smi_mlp3_forward_stacked', L.ptr(st), st.stride(0), offs, D, h1, h2, A, 2,
               L.ptr(x), x.stride(0), self.n, L.ptr(y), A, L.stream(self.device))
        return y

    def _perceive_row(self, obs, i):
        o = {'pixel': {'camera0': self._camera(obs['pixel']['camera0'])[i:i + 1]}}
        if self.model.low_dim:
            low = obs['low_dim'][list(obs['low_dim'])[0]]
            o['low_dim'] = {'flat_inputs': torch.from_numpy(
                np.ascontiguousarray(low, dtype=np.float32)[i:i + 1]).to(self.device)}
        return self.model.forward_perception(o)

    def _camera(self, frames):
        """camera0 of N agents -> a uint8 (N, C, H, W) device tensor; a list of
        per-agent frame lists is concatenated along channels first, as
        ddpg_agent.py:158-163 does when frames are not stacked by the env"""
        if not self.frame_stack_concatenate_on_env and isinstance(frames, (list, tuple)):
            frames = np.stack([np.concatenate(f, axis=0) for f in frames])
        a = np.asarray(frames)
        if a.dtype != np.uint8:
            if not (np.all(a == np.round(a)) and a.min() >= 0 and a.max() <= 255):
                raise TypeError('DDPG camera observations must hold uint8 pixel values')
            a = a.astype(np.uint8)
        return torch.from_numpy(np.ascontiguousarray(a)).to(self.device)

    def act(self, obs):
        """obs: (N, D) low-dim observations, or {'low_dim': {key: (N, D)}, 'pixel':
        {'camera0': (N, C, H, W) uint8}} -- the reference agent's forward_perception
        then forward_actor (ddpg_agent.py:153-182, ddpg_net.py:69-95), for N agents"""
        self._ctx.make_current()
        m = self.model
        if isinstance(obs, dict) and m.is_pixel_input:
            o = {'pixel': {'camera0': self._camera(obs['pixel']['camera0'])}}
            if m.low_dim:
                low = obs['low_dim'][list(obs['low_dim'])[0]]
                o['low_dim'] = {'flat_inputs': torch.from_numpy(
                    np.ascontiguousarray(low, dtype=np.float32)).to(self.device)}
            x = m.forward_perception(o)
        else:
            if isinstance(obs, dict):
                obs = obs['low_dim'][list(obs['low_dim'])[0]]
            if m.is_pixel_input:
                raise ValueError('this DDPG model reads camera0: pass {"pixel": {"camera0": ...}, ...}')
            x = torch.from_numpy(np.ascontiguousarray(obs, dtype=np.float32)).to(self.device)
        if x.dim() != 2 or x.shape[0] != self.n:
            raise ValueError(f'expected observations of {self.n} agents, got shape {tuple(x.shape)}')
        if self.param_noise_type is not None and self._pn_flats is not None:
            a = self._act_param_noise(obs, x).cpu().numpy().clip(-1, 1)
        else:
            a = m.forward_actor(x).cpu().numpy().clip(-1, 1)
        if self.agent_mode != 'eval_deterministic':
            a += self._noise()
        return a.clip(-1, 1)
