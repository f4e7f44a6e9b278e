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


class _FlatViews(nn.Module):
    """Parameters that are views of a flat device buffer: state_dict() returns
    compact copies (each tensor its own storage), so pickling a state_dict —
    the reference Checkpoint (utils/checkpoint.py:234-246) and ModuleDict.dumps
    (distributed/module_dict.py:22-35) both do — does not drag the whole flat
    buffer along with every view.  load_state_dict() copies in place, into the
    flat buffer."""

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        super()._save_to_state_dict(destination, prefix, keep_vars)
        if not keep_vars:
            for name in self._parameters:
                key = prefix + name
                if key in destination:
                    destination[key] = destination[key].clone()


class _LinearView(_FlatViews):
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


class _FlatMLP(_FlatViews):
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


def lstm_param_count(input_size, hidden_size, num_layers=1):
    """floats of a stacked LSTM in the C-ABI layout (layer k >= 1 reads hidden_size)"""
    lib = L.lib()
    return int(lib.smi_lstm_param_count(input_size, hidden_size)) + \
        (num_layers - 1) * int(lib.smi_lstm_param_count(hidden_size, hidden_size))


class LSTMStem(_FlatViews):
    """nn.LSTM(input_size, hidden_size, num_layers, batch_first=True) of PPOModel
    (ppo_net.py:143-152) over ONE flat device buffer in the C-ABI LSTM layout:
    per layer [W_ih (4H, in) | W_hh (4H, H) | b_ih (4H) | b_hh (4H)] (torch's
    parameter order and gate order i, f, g, o; layer k >= 1 has in = H), layers
    one after another.  The Parameters are views named and shaped like torch's
    (weight_ih_l{k}, weight_hh_l{k}, bias_ih_l{k}, bias_hh_l{k}), so state_dict()
    matches nn.LSTM's.  forward() runs, per layer, the x-projection GEMM and the
    persistent LSTM sequence kernel; inputs are batch_first (B, S, in)."""

    def __init__(self, input_size, hidden_size, num_layers=1, batch_first=True, device=None,
                 generator=None, flat=None):
        super().__init__()
        if not 1 <= num_layers <= 3:
            raise NotImplementedError('surreal_amd: LSTM stem supports rnn_layer 1..3')
        if not batch_first:
            raise NotImplementedError('surreal_amd: the reference builds the LSTM batch_first')
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        H = hidden_size
        n = lstm_param_count(input_size, H, num_layers)
        if flat is None:
            flat = torch.zeros(n, dtype=torch.float32, device=device)
        assert flat.numel() == n
        o = 0
        for k in range(num_layers):
            D = input_size if k == 0 else H
            setattr(self, f'weight_ih_l{k}', nn.Parameter(flat[o:o + 4 * H * D].view(4 * H, D)))
            o += 4 * H * D
            setattr(self, f'weight_hh_l{k}', nn.Parameter(flat[o:o + 4 * H * H].view(4 * H, H)))
            o += 4 * H * H
            setattr(self, f'bias_ih_l{k}', nn.Parameter(flat[o:o + 4 * H]))
            o += 4 * H
            setattr(self, f'bias_hh_l{k}', nn.Parameter(flat[o:o + 4 * H]))
            o += 4 * H
        self.__dict__['flat'] = flat
        self.reset_parameters(generator)

    def layer_params(self, k):
        return tuple(getattr(self, f'{n}_l{k}') for n in ('weight_ih', 'weight_hh', 'bias_ih', 'bias_hh'))

    def reset_parameters(self, generator=None):
        # torch.nn.LSTM default init: every parameter U(-1/sqrt(H), 1/sqrt(H))
        k = 1.0 / math.sqrt(self.hidden_size)
        with torch.no_grad():
            for layer in range(self.num_layers):
                for p in self.layer_params(layer):
                    p.copy_(torch.empty(p.shape).uniform_(-k, k, generator=generator))

    def forward(self, x, cells=None):
        """x (B, S, in) -> (out (B, S, H), (h_n, c_n) each (num_layers, B, H))."""
        B, S, _ = x.shape
        H, NL = self.hidden_size, self.num_layers
        dev = self.flat.device
        st = L.stream(dev)
        if cells is None:
            h0 = torch.zeros(NL, B, H, device=dev)
            c0 = torch.zeros(NL, B, H, device=dev)
        else:
            h0 = cells[0].reshape(NL, B, H).contiguous()
            c0 = cells[1].reshape(NL, B, H).contiguous()
        inp = x.transpose(0, 1).contiguous()                      # time-major (S, B, in)
        hn, cn = [], []
        for k in range(NL):
            w_ih, w_hh, b_ih, b_hh = self.layer_params(k)
            D = inp.shape[-1]
            xproj = torch.empty(S, B, 4 * H, dtype=torch.float32, device=dev)
            L.call('smi_linear_forward', L.ptr(inp), D, S * B, D, L.ptr(w_ih), D, L.ptr(b_ih), 4 * H, 0,
                   L.ptr(xproj), 4 * H, st)
            hbuf = torch.empty(S + 1, B, H, dtype=torch.float32, device=dev)
            cbuf = torch.empty(S + 1, B, H, dtype=torch.float32, device=dev)
            L.call('smi_lstm_forward', L.ptr(xproj), L.ptr(w_hh), L.ptr(b_hh), L.ptr(h0[k]),
                   L.ptr(c0[k]), S, B, H, L.ptr(hbuf), L.ptr(cbuf), None, st)
            hn.append(hbuf[S].clone())
            cn.append(cbuf[S].clone())
            inp = hbuf[1:]                                        # (S, B, H), contiguous
        out = inp.transpose(0, 1).contiguous()
        return out, (torch.stack(hn), torch.stack(cn))


class _ParamView(_FlatViews):
    """weight/bias Parameters (torch Conv2d / Linear shapes) viewing a flat buffer."""

    def __init__(self, flat, off, wshape, nbias):
        super().__init__()
        nw = int(np.prod(wshape))
        self.weight = nn.Parameter(flat[off:off + nw].view(*wshape))
        self.bias = nn.Parameter(flat[off + nw:off + nw + nbias])
        self.end = off + nw + nbias

    def reset_parameters(self, generator=None):
        # torch Conv2d / Linear default init: U(+-1/sqrt(fan_in)) for weight and bias
        bound = 1.0 / math.sqrt(int(np.prod(self.weight.shape[1:])))
        with torch.no_grad():
            for p in (self.weight, self.bias):
                p.copy_(torch.empty(p.shape).uniform_(-bound, bound, generator=generator))


class CNNStemNetwork(nn.Module):
    """builders.py:8-33: conv 8x8/4 (C->16) -> ReLU -> conv 4x4/2 (16->32) -> ReLU
    -> Flatten -> Linear(D_out) -> ReLU, over ONE flat device buffer in the C-ABI
    CNN layout (include/surreal_mi.h, smi_cnn_*).  State-dict keys follow the
    Sequential positions: model.0 (conv), model.2 (conv), model.5 (linear).

    forward() takes the raw uint8 camera tensor, (N, C, H, W) or (B, S, C, H, W)
    — the obs/255 of ppo_net.py:368-375 is fused into the conv kernel (bit-equal
    to torch's uint8 / 255.0).  Inference only; the learner's phases run the
    backward (smi_ppo_rnn_phase)."""

    def __init__(self, D_obs, D_out, conv_channels=(16, 32), kernel_sizes=(8, 4), strides=(4, 2),
                 device=None, generator=None, flat=None):
        super().__init__()
        if list(conv_channels) != [16, 32] or list(kernel_sizes) != [8, 4] or list(strides) != [4, 2]:
            raise NotImplementedError('surreal_amd: CNN stem is built for the reference defaults '
                                      '(16@8s4, 32@4s2; builders.py:9)')
        C, H, W = (int(v) for v in D_obs)
        self.D_obs, self.D_out = (C, H, W), int(D_out)
        n = int(L.lib().smi_cnn_param_count(C, H, W, self.D_out))
        if flat is None:
            flat = torch.zeros(n, dtype=torch.float32, device=device)
        assert flat.numel() == n
        H1, W1 = (H - 8) // 4 + 1, (W - 8) // 4 + 1
        H2, W2 = (H1 - 4) // 2 + 1, (W1 - 4) // 2 + 1
        self.flat_dim = 32 * H2 * W2
        c1 = _ParamView(flat, 0, (16, C, 8, 8), 16)
        c2 = _ParamView(flat, c1.end, (32, 16, 4, 4), 32)
        fc = _ParamView(flat, c2.end, (self.D_out, self.flat_dim), self.D_out)
        self.model = nn.Sequential(c1, nn.ReLU(), c2, nn.ReLU(), nn.Flatten(), fc, nn.ReLU())
        for m in (c1, c2, fc):
            m.reset_parameters(generator)
        self.__dict__['flat'] = flat

    def forward(self, obs):
        if obs.dtype != torch.uint8:
            raise TypeError('CNNStemNetwork: camera observations must be uint8 (scaled by 1/255 '
                            'inside the kernel)')
        lead = obs.shape[:-3]
        x = obs.reshape(-1, *self.D_obs).contiguous()
        rows = x.shape[0]
        dev = self.flat.device
        a2 = torch.empty(rows, self.flat_dim, dtype=torch.float32, device=dev)
        out = torch.empty(rows, self.D_out, dtype=torch.float32, device=dev)
        C, H, W = self.D_obs
        L.call('smi_cnn_forward', L.ptr(self.flat), L.ptr(x), None, max(rows, 1), 1, rows,
               C, H, W, self.D_out, None, L.ptr(a2), L.ptr(out), self.D_out, L.stream(dev))
        return out.reshape(*lead, self.D_out)


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

    def scale_forward_partial_(self, rewards, scale, sums3):
        """Data parallel: rewards*scale and whitening as scale_forward_update_,
        the update deferred: this rank's {sum, sumsq, n} (fp64) go to sums3."""
        L.call('smi_reward_filter_partial', L.ptr(rewards), rewards.numel(), float(scale), 1,
               L.ptr(self.running_sum), L.ptr(self.running_sumsq), L.ptr(self.count),
               float(self.eps), L.ptr(sums3), L.stream(rewards.device))
        return rewards

    def commit_(self, sums3):
        """the reference update (reward_filter.py:33-42) from all-reduced sums"""
        L.call('smi_reward_filter_commit', L.ptr(sums3), L.ptr(self.running_sum),
               L.ptr(self.running_sumsq), L.ptr(self.count), L.stream(sums3.device))

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

    The LSTM stem (if_rnn_policy, rnn_layer 1..3) is the HIP LSTMStem and the pixel
    stem (if_pixel_input) the HIP CNNStemNetwork on obs['pixel']['camera0']
    (uint8).  With both, their parameters share one flat `stem_flat` buffer
    [lstm | cnn] (the layout smi_ppo_rnn_phase and the optimizers use).
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
        self.if_rnn = bool(self.rnn_config.get('if_rnn_policy', False))
        self.device = torch.device(device) if device is not None else torch.device('cuda')
        self.low_dim = 0
        self.low_dim_keys = []
        if 'low_dim' in obs_spec:
            for k, v in obs_spec['low_dim'].items():
                self.low_dim += int(v[0])
                self.low_dim_keys.append(k)
        self.cnn_stem = None
        self.rnn_stem = None
        F = int(model_config['cnn_feature_dim']) if if_pixel_input else 0
        d_in = self.low_dim + F
        n_cnn = 0
        if if_pixel_input:
            C, H, W = obs_spec['pixel']['camera0']
            n_cnn = int(L.lib().smi_cnn_param_count(C, H, W, F))
        n_rnn = 0
        if self.if_rnn:
            n_rnn = lstm_param_count(d_in, self.rnn_config['rnn_hidden'],
                                     self.rnn_config.get('rnn_layer', 1))
        stem = torch.zeros(n_rnn + n_cnn, dtype=torch.float32, device=self.device)
        if if_pixel_input:                                  # ppo_net.py:137-141
            self.cnn_stem = CNNStemNetwork(obs_spec['pixel']['camera0'], F, device=self.device,
                                           generator=generator, flat=stem[n_rnn:])
        if self.if_rnn:                                     # ppo_net.py:143-152,159-160
            self.rnn_stem = LSTMStem(d_in, self.rnn_config['rnn_hidden'],
                                     self.rnn_config.get('rnn_layer', 1), True, self.device, generator,
                                     flat=stem[:n_rnn])
            d_in = self.rnn_config['rnn_hidden']
        self.__dict__['stem_flat'] = stem          # [lstm | cnn]; empty for a plain MLP model
        self.actor = PPO_ActorNetwork(d_in, action_dim, model_config['actor_fc_hidden_sizes'],
                                      init_log_sig, self.device, generator)
        self.critic = PPO_CriticNetwork(d_in, model_config['critic_fc_hidden_sizes'],
                                        self.device, generator)
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

    def clear_actor_grad(self):                             # ppo_net.py:180-189
        for p in self.get_actor_params():
            p.grad = None

    def clear_critic_grad(self):                            # ppo_net.py:191-200
        for p in self.get_critic_params():
            p.grad = None

    def get_actor_params(self):                             # ppo_net.py:202-212
        ps = list(self.actor.parameters())
        if self.if_pixel_input:
            ps += list(self.cnn_stem.parameters())
        if self.if_rnn:
            ps += list(self.rnn_stem.parameters())
        return iter(ps)

    def get_critic_params(self):                            # ppo_net.py:214-224
        ps = list(self.critic.parameters())
        if self.if_pixel_input:
            ps += list(self.cnn_stem.parameters())
        if self.if_rnn:
            ps += list(self.rnn_stem.parameters())
        return iter(ps)

    def update_target_params(self, net):                    # ppo_net.py:226-242
        with torch.no_grad():
            self.actor.flat.copy_(net.actor.flat)
            self.critic.flat.copy_(net.critic.flat)
            self.stem_flat.copy_(net.stem_flat)             # lstm and/or cnn stems
            if self.use_z_filter:
                self.z_filter.load_state_dict(net.z_filter.state_dict())

    def update_target_z_filter(self, net):
        if self.use_z_filter:
            self.z_filter.load_state_dict(net.z_filter.state_dict())

    def _stem_input(self, obs):
        """cat([zfilter(low_dim), cnn(camera0/255)], -1) (ppo_net.py:262-275)."""
        x = self._gather_low_dim_input(obs)
        parts = []
        if x is not None:
            parts.append(self.z_filter.forward(x) if self.use_z_filter else x)
        if self.if_pixel_input:
            parts.append(self.cnn_stem(obs['pixel']['camera0']))
        return parts[0] if len(parts) == 1 else torch.cat(parts, -1)

    def _rnn_features(self, obs, cells):
        out, cells = self.rnn_stem(self._stem_input(obs).contiguous(), cells)
        return out, cells

    def forward_actor(self, obs, cells=None):               # ppo_net.py:253-282
        if self.if_rnn:
            return self.actor(self._rnn_features(obs, cells)[0])
        if self.if_pixel_input:
            return self.actor(self._stem_input(obs))
        return self.actor(self._gather_low_dim_input(obs),
                          self.z_filter if self.use_z_filter else None)

    def forward_critic(self, obs, cells=None):              # ppo_net.py:284-315
        if self.if_rnn:
            return self.critic(self._rnn_features(obs, cells)[0])
        if self.if_pixel_input:
            return self.critic(self._stem_input(obs))
        return self.critic(self._gather_low_dim_input(obs),
                           self.z_filter if self.use_z_filter else None)

    def forward_actor_expose_cells(self, obs, cells=None):  # ppo_net.py:317-352
        if not self.if_rnn:
            return self.forward_actor(obs, cells), cells
        x = self._stem_input(obs).reshape(1, 1, -1)
        out, cells = self.rnn_stem(x.contiguous(), cells)
        return self.actor(out.reshape(-1, self.rnn_config['rnn_hidden'])), cells

    def z_update(self, obs):
        if not self.use_z_filter:
            raise ValueError('Z_update called when network is set to not use z_filter')
        self.z_filter.z_update(self._gather_low_dim_input(obs))
