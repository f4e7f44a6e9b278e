"""Drop-in mirrors of surreal.model (ppo_net.py, z_filter.py, reward_filter.py,
model_builders/builders.py) whose compute runs in the HIP kernels of
libsurreal_mi.so.

Parameters live in ONE flat fp32 device buffer per network in the C-ABI "flat
MLP layout" (include/surreal_mi.h); every nn.Parameter is a view into it, so
state_dict()/load_state_dict() keep the usual (out, in) shapes while kernels,
Adam and all-reduces see a single contiguous buffer.

state_dict key names: torchx (which named the reference's layers) is not
available, so the Sequential-style names 'model.0.weight',
'model.2.weight', 'model.4.weight' (+ 'log_var') are this build's assumption.
"""
import math

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from .config import Config


def mlp_param_count(d_in, h1, h2, d_out, with_log_var):
    return h1 * d_in + h1 + h2 * h1 + h2 + d_out * h2 + d_out + (d_out if with_log_var else 0)


class _LinearView(nn.Module):
    """Holds weight/bias Parameters that are views of a flat buffer."""

    def __init__(self, flat, off, d_in, d_out):
        super().__init__()
        self.in_features, self.out_features = d_in, d_out
        self.weight = nn.Parameter(flat[off:off + d_out * d_in].view(d_out, d_in))
        off += d_out * d_in
        self.bias = nn.Parameter(flat[off:off + d_out])
        self.end = off + d_out

    def reset_parameters(self, generator=None):
        # torch.nn.Linear default init (kaiming_uniform a=sqrt(5); bias U(+-1/sqrt(fan_in)))
        with torch.no_grad():
            bound = 1.0 / math.sqrt(self.in_features)
            w = torch.empty(self.weight.shape).uniform_(-bound, bound, generator=generator)
            b = torch.empty(self.bias.shape).uniform_(-bound, bound, generator=generator)
            self.weight.copy_(w)
            self.bias.copy_(b)


class _FlatMLP(nn.Module):
    """Linear-ReLU-Linear-ReLU-Linear[-Tanh] over one flat device buffer."""

    def __init__(self, d_in, h1, h2, d_out, out_tanh, with_log_var, device, init_log_sig=0.0,
                 generator=None):
        super().__init__()
        self.dims = (d_in, h1, h2, d_out)
        self.out_tanh = out_tanh
        self.with_log_var = with_log_var
        n = mlp_param_count(d_in, h1, h2, d_out, with_log_var)
        flat = torch.zeros(n, dtype=torch.float32, device=device)
        l0 = _LinearView(flat, 0, d_in, h1)
        l2 = _LinearView(flat, l0.end, h1, h2)
        l4 = _LinearView(flat, l2.end, h2, d_out)
        layers = [l0, nn.ReLU(), l2, nn.ReLU(), l4]
        if out_tanh:
            layers.append(nn.Tanh())
        self.model = nn.Sequential(*layers)
        for lin in (l0, l2, l4):
            lin.reset_parameters(generator)
        if with_log_var:
            # builders.py:112 — log_var = zeros(1, D_act) + init_log_sig
            self.log_var = nn.Parameter(flat[l4.end:l4.end + d_out].view(1, d_out))
            with torch.no_grad():
                self.log_var.fill_(float(init_log_sig))
        self.__dict__['flat'] = flat     # plain attribute: not a parameter, not in state_dict

    def forward_flat(self, x2d, row_stride, zfilter=None):
        d_in, h1, h2, d_out = self.dims
        rows = x2d.shape[0]
        ocols = 2 * d_out if self.with_log_var else d_out
        out = torch.empty(rows, ocols, dtype=torch.float32, device=self.flat.device)
        if rows == 0:
            return out
        zf = zfilter
        L.call('smi_mlp_forward', L.ptr(self.flat), d_in, h1, h2, d_out, 2 if self.out_tanh else 0,
               1 if self.with_log_var else 0, L.ptr(x2d), rows, row_stride,
               1 if zf is not None else 0,
               L.ptr(zf.running_sum) if zf is not None else None,
               L.ptr(zf.running_sumsq) if zf is not None else None,
               L.ptr(zf.count) if zf is not None else None,
               float(zf.eps) if zf is not None else 0.0,
               L.ptr(out), L.stream(self.flat.device))
        return out


def _rows2d(x):
    """(N, D) view with a row stride, or a contiguous copy if rows are not evenly strided."""
    if x.dim() == 1:
        x = x.view(1, -1)
    x2 = x.reshape(-1, x.shape[-1]) if x.dim() > 2 else x
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    return x2, x2.stride(0)


class PPO_ActorNetwork(_FlatMLP):
    """builders.py:86-132: mean = tanh(MLP(obs)), std = exp(log_var) broadcast."""

    def __init__(self, D_obs, D_act, hidden_sizes=(64, 64), init_log_sig=0, device=None,
                 generator=None):
        super().__init__(D_obs, hidden_sizes[0], hidden_sizes[1], D_act, True, True, device,
                         init_log_sig, generator)

    def forward(self, obs, zfilter=None):
        shape = obs.shape
        x2, stride = _rows2d(obs)
        out = self.forward_flat(x2, stride, zfilter)
        if len(shape) == 3:
            out = out.view(shape[0], shape[1], -1)
        return out


class PPO_CriticNetwork(_FlatMLP):
    """builders.py:135-175: scalar value head."""

    def __init__(self, D_obs, hidden_sizes=(64, 64), device=None, generator=None):
        super().__init__(D_obs, hidden_sizes[0], hidden_sizes[1], 1, False, False, device, 0.0,
                         generator)

    def forward(self, obs, zfilter=None):
        shape = obs.shape
        x2, stride = _rows2d(obs)
        out = self.forward_flat(x2, stride, zfilter)
        if len(shape) == 3:
            out = out.view(shape[0], shape[1], 1)
        return out


class ZFilter(nn.Module):
    """z_filter.py:23-107: running sum / sumsq / count whitening, clamp +-5."""

    def __init__(self, obs_spec, eps=1e-5, device=None):
        super().__init__()
        self.eps = eps
        self.obs_spec = obs_spec
        self.in_size = sum(int(v[0]) for v in obs_spec['low_dim'].values())
        self.register_buffer('running_sum', torch.zeros(self.in_size, device=device))
        self.register_buffer('running_sumsq', eps * torch.ones(self.in_size, device=device))
        self.register_buffer('count', torch.tensor([eps], dtype=torch.float32, device=device))

    def z_update(self, x):                                  # z_filter.py:44-57
        if x is None:
            return
        x2, stride = _rows2d(x)
        L.call('smi_zfilter_update', L.ptr(x2), x2.shape[0], self.in_size, stride,
               L.ptr(self.running_sum), L.ptr(self.running_sumsq), L.ptr(self.count),
               L.stream(x.device))

    def forward(self, inputs):                              # z_filter.py:59-79
        if inputs is None:
            return None
        assert inputs.dim() >= 2
        x = inputs.contiguous()
        out = torch.empty_like(x)
        L.call('smi_zfilter_apply', L.ptr(x), L.ptr(out), x.numel() // x.shape[-1], x.shape[-1],
               L.ptr(self.running_sum), L.ptr(self.running_sumsq), L.ptr(self.count),
               float(self.eps), L.stream(x.device))
        return out

    def running_mean(self):
        return (self.running_sum / self.count).cpu().numpy()

    def running_std(self):
        return ((self.running_sumsq / self.count) -
                (self.running_sum / self.count).pow(2)).pow(0.5).cpu().numpy()

    def running_square(self):
        return (self.running_sumsq / self.count).cpu().numpy()


class RewardFilter(nn.Module):
    """reward_filter.py:5-63 (keeps the reference's `running_sumsq =` at :42)."""

    def __init__(self, eps=1e-5, device=None):
        super().__init__()
        self.eps = eps
        self.register_buffer('count', torch.tensor(eps, dtype=torch.float32, device=device))
        self.register_buffer('running_sum', torch.tensor(0.0, dtype=torch.float32, device=device))
        self.register_buffer('running_sumsq', torch.tensor(0.0, dtype=torch.float32, device=device))

    def _run(self, x, scale, mode):
        L.call('smi_reward_filter', L.ptr(x), x.numel(), float(scale), mode,
               L.ptr(self.running_sum), L.ptr(self.running_sumsq), L.ptr(self.count),
               float(self.eps), L.stream(x.device))

    def update(self, x):
        self._run(x.contiguous().clone(), 1.0, 2)

    def forward(self, inputs):
        out = inputs.contiguous().clone()
        self._run(out, 1.0, 1)
        return out

    def scale_forward_update_(self, rewards, scale):
        """In place: rewards*scale, whiten with pre-update stats, then update
        (ppo.py:452-456 as one launch)."""
        self._run(rewards, scale, 3)
        return rewards

    def reward_mean(self):
        return (self.running_sum / self.count).item()


class DiagGauss(object):
    """ppo_net.py:13-91 on device tensors (sample/maxprob stay host numpy)."""

    def __init__(self, action_dim):
        self.d = action_dim

    def _flat(self, a, prob):
        if a is not None and a.dim() == 3:
            a = a.reshape(-1, self.d)
        if prob.dim() == 3:
            prob = prob.reshape(-1, 2 * self.d)
        return (a.contiguous() if a is not None else None), prob.contiguous()

    def _run(self, a, p0, p1, want):
        rows = p0.shape[0]
        outs = {k: torch.empty(rows, dtype=torch.float32, device=p0.device) for k in want}
        L.call('smi_diag_gauss', L.ptr(a), L.ptr(p0), L.ptr(p1), rows, self.d,
               L.ptr(outs.get('loglik')), L.ptr(outs.get('lik')), L.ptr(outs.get('kl')),
               L.ptr(outs.get('ent')), L.stream(p0.device))
        return outs

    def loglikelihood(self, a, prob):
        a, prob = self._flat(a, prob)
        return self._run(a, prob, None, ['loglik'])['loglik'].view(-1, 1)

    def likelihood(self, a, prob):
        a, prob = self._flat(a, prob)
        return self._run(a, prob, None, ['lik'])['lik'].view(-1, 1)

    def kl(self, prob0, prob1):
        _, p0 = self._flat(None, prob0)
        _, p1 = self._flat(None, prob1)
        return self._run(None, p0, p1, ['kl'])['kl']

    def entropy(self, prob):
        _, p = self._flat(None, prob)
        return self._run(None, p, None, ['ent'])['ent']

    def sample(self, prob):
        if len(prob.shape) == 3:
            prob = prob.reshape(-1, self.d * 2)
        mean_nd, std_nd = prob[:, :self.d], prob[:, self.d:]
        return np.random.randn(prob.shape[0], self.d) * std_nd + mean_nd

    def maxprob(self, prob):
        if len(prob.shape) == 3:
            return prob[:, :, self.d]
        return prob[:, :self.d]


class PPOModel(nn.Module):
    """ppo_net.py:94-375 (low-dimensional observations).

    The LSTM stem (if_rnn_policy) and the pixel CNN stem (if_pixel_input) are
    SURVEY.md §8(f) rank 1 and are rejected loudly until their HIP kernels land.
    """

    def __init__(self, obs_spec, action_dim, model_config, use_cuda=True, init_log_sig=0,
                 use_z_filter=False, if_pixel_input=False, rnn_config=None, device=None,
                 generator=None):
        super().__init__()
        L.require_gpu()
        self.obs_spec = obs_spec
        self.action_dim = action_dim
        self.model_config = model_config
        self.use_z_filter = use_z_filter
        self.init_log_sig = init_log_sig
        self.if_pixel_input = if_pixel_input
        self.rnn_config = rnn_config if rnn_config is not None else Config({'if_rnn_policy': False})
        if if_pixel_input:
            raise NotImplementedError('surreal_amd: pixel CNN stem is not built yet (SURVEY §8(f) 1)')
        if self.rnn_config.get('if_rnn_policy', False):
            raise NotImplementedError('surreal_amd: LSTM policy stem is not built yet (SURVEY §8(f) 1)')
        self.device = torch.device(device) if device is not None else torch.device('cuda')
        self.low_dim = 0
        self.low_dim_keys = []
        if 'low_dim' in obs_spec:
            for k, v in obs_spec['low_dim'].items():
                self.low_dim += int(v[0])
                self.low_dim_keys.append(k)
        self.actor = PPO_ActorNetwork(self.low_dim, action_dim, model_config['actor_fc_hidden_sizes'],
                                      init_log_sig, self.device, generator)
        self.critic = PPO_CriticNetwork(self.low_dim, model_config['critic_fc_hidden_sizes'],
                                        self.device, generator)
        self.cnn_stem = None
        self.rnn_stem = None
        if use_z_filter:
            assert self.low_dim > 0, 'No low dimensional input, please turn off z-filter'
            self.z_filter = ZFilter(obs_spec, device=self.device)

    # ppo_net.py:168-178
    def _gather_low_dim_input(self, obs):
        if isinstance(obs, torch.Tensor):
            return obs
        if 'low_dim' not in obs:
            return None
        parts = [obs['low_dim'][k] for k in obs['low_dim']]
        return parts[0] if len(parts) == 1 else torch.cat(parts, -1)

    def clear_actor_grad(self):
        for p in self.actor.parameters():
            p.grad = None

    def clear_critic_grad(self):
        for p in self.critic.parameters():
            p.grad = None

    def get_actor_params(self):
        return self.actor.parameters()

    def get_critic_params(self):
        return self.critic.parameters()

    def update_target_params(self, net):                    # ppo_net.py:226-242
        with torch.no_grad():
            self.actor.flat.copy_(net.actor.flat)
            self.critic.flat.copy_(net.critic.flat)
            if self.use_z_filter:
                self.z_filter.load_state_dict(net.z_filter.state_dict())

    def update_target_z_filter(self, net):
        if self.use_z_filter:
            self.z_filter.load_state_dict(net.z_filter.state_dict())

    def forward_actor(self, obs, cells=None):
        x = self._gather_low_dim_input(obs)
        return self.actor(x, self.z_filter if self.use_z_filter else None)

    def forward_critic(self, obs, cells=None):
        x = self._gather_low_dim_input(obs)
        return self.critic(x, self.z_filter if self.use_z_filter else None)

    def forward_actor_expose_cells(self, obs, cells=None):
        return self.forward_actor(obs, cells), cells

    def z_update(self, obs):
        if not self.use_z_filter:
            raise ValueError('Z_update called when network is set to not use z_filter')
        self.z_filter.z_update(self._gather_low_dim_input(obs))
