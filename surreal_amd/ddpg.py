"""DDPGModel / DDPGLearner mirrors (surreal/model/ddpg_net.py,
surreal/learner/ddpg.py) on the MFMA GEMM layers of linear_kernels.hip.

One DDPG learn() (ddpg.py:244-352, batch 512, actor 17-300-200-6, critic
17-400 | +6 -300-1) is ~45 launches on one stream and no host sync:
target actor + target critic forward, n-step target, critic forward, MSE
gradient, critic backward, Adam; actor forward, critic forward with the
updated critic, -mean(Q) gradient, backward through the critic's action block
and the actor, Adam; target update; statistics.  With use_layernorm
(off by default, ddpg_configs.py:21) every hidden ReLU is followed by a
LayerNorm block (smi_layernorm_*).  Pixel observations (env pixel_input,
ddpg_net.py:34-43,69-79): the perception CNNStemNetwork (16@8s4, 32@4s2, FC
conv_spec.hidden_output_dim) of each model turns camera0 (uint8, / 255 fused
into the conv kernel; 9 channels = 3 stacked RGB frames) into features that
are concatenated [cnn | low_dim] before the actor and critic; it trains with
the CRITIC's optimizer (get_critic_parameters, ddpg_net.py:57-61), the actor
reads it detached (ddpg.py:325-328), and it follows the target updates
(ddpg.py:414-428).

Parameter layouts (flat, torch (out, in) order; [g b] = LayerNorm weight / bias
with use_layernorm):
  actor : W1[h1][D] b1 [g1 b1'] W2[h2][h1] b2 [g2 b2'] W3[A][h2] b3
  critic: Wo[c1][D] bo [go bo'] Wc[c2][c1+A] bc [gc bc'] Wq[1][c2] bq
"""
import math
import os

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from .session import LearnerHooks
from .config import Config, ConfigError
from .model import CNNStemNetwork, _FlatViews, _LinearView

# group each backward's weight-gradient GEMMs into one launch (SMI_DDPG_DW_GROUP=0: A/B off)
_DW_GROUP = os.environ.get('SMI_DDPG_DW_GROUP', '1') != '0'

RELU, TANH, NONE = 1, 2, 0


class _LayerNormView(_FlatViews):
    """weight / bias of one LayerNorm block (torch.nn.LayerNorm(n) init: ones,
    zeros) as views of the network's flat buffer."""

    def __init__(self, flat, off, n):
        super().__init__()
        self.n = n
        self.weight = nn.Parameter(flat[off:off + n])
        self.bias = nn.Parameter(flat[off + n:off + 2 * n])
        with torch.no_grad():
            self.weight.fill_(1.0)
            self.bias.zero_()
        self.end = off + 2 * n


class _FlatNet(nn.Module):
    """Linear (spec (d_in, d_out)) and LayerNorm (spec ('ln', n)) blocks over one
    flat fp32 buffer, in the torch Sequential parameter order."""

    def __init__(self, specs, device, generator=None):
        super().__init__()
        n = sum(2 * sp[1] if sp[0] == 'ln' else sp[1] * sp[0] + sp[1] for sp in specs)
        flat = torch.zeros(n, dtype=torch.float32, device=device)
        self.__dict__['flat'] = flat
        self.layers, self.norms = [], []
        off = 0
        for sp in specs:
            if sp[0] == 'ln':
                ln = _LayerNormView(flat, off, sp[1])
                off = ln.end
                self.norms.append(ln)
            else:
                lin = _LinearView(flat, off, sp[0], sp[1])
                lin.reset_parameters(generator)
                off = lin.end
                self.layers.append(lin)

    def wb(self, k):
        lin = self.layers[k]
        return lin.weight, lin.bias

    def off(self, p):
        """offset of a parameter view in the flat buffer (= in a gradient image)"""
        return (p.data_ptr() - self.flat.data_ptr()) // 4


class ActorNetworkX(_FlatNet):
    """builders.py:35-56: Linear-ReLU[-LayerNorm]-Linear-ReLU[-LayerNorm]-Linear-Tanh."""

    def __init__(self, D_in, D_act, hidden_sizes=(300, 200), device=None, generator=None,
                 use_layernorm=False):
        h1, h2 = hidden_sizes
        ln = bool(use_layernorm)
        specs = [(D_in, h1)] + ([('ln', h1)] if ln else []) + [(h1, h2)] + \
            ([('ln', h2)] if ln else []) + [(h2, D_act)]
        super().__init__(specs, device, generator)
        self.use_layernorm = ln
        l0, l1, l2 = self.layers
        mods = [l0, nn.ReLU()] + ([self.norms[0]] if ln else []) + [l1, nn.ReLU()] + \
            ([self.norms[1]] if ln else []) + [l2, nn.Tanh()]
        self.model = nn.Sequential(*mods)
        self.dims = (D_in, h1, h2, D_act)


class CriticNetworkX(_FlatNet):
    """builders.py:58-84: obs -> Linear-ReLU[-LayerNorm]; cat(h, a) ->
    Linear-ReLU[-LayerNorm]-Linear."""

    def __init__(self, D_in, D_act, hidden_sizes=(400, 300), device=None, generator=None,
                 use_layernorm=False):
        c1, c2 = hidden_sizes
        ln = bool(use_layernorm)
        specs = [(D_in, c1)] + ([('ln', c1)] if ln else []) + [(c1 + D_act, c2)] + \
            ([('ln', c2)] if ln else []) + [(c2, 1)]
        super().__init__(specs, device, generator)
        self.use_layernorm = ln
        l0, l1, l2 = self.layers
        self.model_obs = nn.Sequential(*([l0, nn.ReLU()] + ([self.norms[0]] if ln else [])))
        self.model_concat = nn.Sequential(*([l1, nn.ReLU()] + ([self.norms[1]] if ln else []) + [l2]))
        self.dims = (D_in, c1, c2, D_act)


class DDPGModel(nn.Module):
    """ddpg_net.py:9-95 for low-dimensional observations."""

    def __init__(self, obs_spec, action_dim, use_layernorm, actor_fc_hidden_sizes,
                 critic_fc_hidden_sizes, conv_out_channels=None, conv_kernel_sizes=None,
                 conv_strides=None, conv_hidden_dim=None, critic_only=False, device=None,
                 generator=None):
        super().__init__()
        L.require_gpu()
        self.device = torch.device(device) if device is not None else torch.device('cuda')
        self.action_dim = action_dim
        self.is_pixel_input = 'pixel' in obs_spec
        self.low_dim = int(obs_spec['low_dim']['flat_inputs'][0]) if 'low_dim' in obs_spec else 0
        self.perception = None
        self.cnn_dim = 0
        if self.is_pixel_input:                          # ddpg_net.py:40-43
            self.cnn_dim = int(conv_hidden_dim if conv_hidden_dim is not None else 200)
            self.perception = CNNStemNetwork(
                obs_spec['pixel']['camera0'], self.cnn_dim,
                conv_out_channels or (16, 32), conv_kernel_sizes or (8, 4), conv_strides or (4, 2),
                device=self.device, generator=generator)
        # concatenated perception: [cnn features | low_dim] (ddpg_net.py:69-79)
        self.input_dim = self.cnn_dim + self.low_dim
        self.use_layernorm = bool(use_layernorm)
        self.actor = None if critic_only else ActorNetworkX(
            self.input_dim, action_dim, actor_fc_hidden_sizes, self.device, generator,
            use_layernorm)
        self.critic = CriticNetworkX(self.input_dim, action_dim, critic_fc_hidden_sizes,
                                     self.device, generator, use_layernorm)

    def get_actor_parameters(self):
        return self.actor.parameters()

    def get_critic_parameters(self):                    # ddpg_net.py:57-61
        ps = list(self.critic.parameters())
        if self.is_pixel_input:
            ps += list(self.perception.parameters())
        return iter(ps)

    def forward_perception(self, obs):                 # ddpg_net.py:69-79
        if isinstance(obs, torch.Tensor):
            return obs
        if not self.is_pixel_input:
            return obs['low_dim']['flat_inputs']
        net = _Net(self)
        pix = obs['pixel']['camera0']
        low = obs['low_dim']['flat_inputs'] if self.low_dim else None
        return net.perception_fwd(self, pix.contiguous(), low, pix.shape[0], None).clone()

    def forward_actor(self, obs):
        net = _Net(self)
        return net.actor_fwd(obs.contiguous(), obs.shape[0], store=None)

    def forward_critic(self, obs, action):
        net = _Net(self)
        return net.critic_fwd(self.critic, obs.contiguous(), action.contiguous(), obs.shape[0], None)

    def forward(self, obs_in, calculate_value=True, action=None):
        x = self.forward_perception(obs_in)
        if action is None:
            action = self.forward_actor(x)
        value = self.forward_critic(x, action) if calculate_value else None
        return action, value


def _p(t):
    return L.ptr(t)


def _check_rows(x, rows, width, what):
    """x must be a [>= rows][width] fp32 device matrix with unit column stride
    (the kernels read rows x width through its row stride)"""
    if (x.dim() != 2 or x.shape[0] < rows or x.shape[1] != width or x.stride(1) != 1
            or x.dtype != torch.float32):
        raise ValueError(f'{what} input: expected a float32 [{rows}][{width}] matrix, got '
                         f'{x.dtype} {tuple(x.shape)}')


class _Net(object):
    """Launch helpers over a DDPGModel's flat buffers."""

    def __init__(self, model, bufs=None):
        self.m = model
        self.st = L.stream(model.device)
        self.bufs = bufs if bufs is not None else {}

    def buf(self, name, shape):
        t = self.bufs.get(name)
        if t is None or tuple(t.shape) != tuple(shape):
            t = torch.zeros(shape, dtype=torch.float32, device=self.m.device)
            self.bufs[name] = t
        return t

    def lin(self, x, ldx, rows, k, w, ldw, b, n, act, y, ldy):
        L.call('smi_linear_forward', _p(x), ldx, rows, k, _p(w), ldw, _p(b), n, act, _p(y), ldy,
               self.st)

    def norm(self, net, j, x, rows, y, ldy, tag):
        """LayerNorm block j over x [rows][n] (post-ReLU) into y; mean / rstd kept
        under tag for the backward"""
        ln = net.norms[j]
        mu, rs = self.buf(tag + '_mu', (rows,)), self.buf(tag + '_rs', (rows,))
        L.call('smi_layernorm_forward', _p(x), x.stride(0), rows, ln.n, _p(ln.weight), _p(ln.bias),
               1e-5, _p(y), ldy, _p(mu), _p(rs), self.st)

    def norm_bwd(self, net, j, dy, x, rows, dx, g, tag):
        """backward of LayerNorm block j (and of the ReLU before it) from dy;
        dgamma / dbeta into the gradient image g (None: input gradient only)"""
        ln = net.norms[j]
        if g is None:
            dg, db = self.buf('ln_dg', (ln.n,)), self.buf('ln_db', (ln.n,))
        else:
            dg, db = g[net.off(ln.weight):], g[net.off(ln.bias):]
        L.call('smi_layernorm_backward', _p(dy), dy.stride(0), _p(x), x.stride(0),
               _p(self.bufs[tag + '_mu']), _p(self.bufs[tag + '_rs']), _p(ln.weight), rows, ln.n, 1,
               _p(dx), dx.stride(0), _p(dg), _p(db), self.st)

    def perception_fwd(self, model, pix, low, rows, store, keep=False):
        """[cnn(pix / 255) | low] (ddpg_net.py:69-79) into buffer store_P; keep:
        the conv activations stay for a backward (store_A1 / store_A2)"""
        cnn = model.perception
        C, H, W = cnn.D_obs
        F, D = model.cnn_dim, model.low_dim
        pre = store or 'ptmp'
        P = self.buf(pre + '_P', (rows, F + D))
        A1 = self.buf(pre + '_A1', (rows, 16 * ((H - 8) // 4 + 1) * ((W - 8) // 4 + 1))) if keep else None
        A2 = self.buf(pre + '_A2', (rows, cnn.flat_dim))
        if pix.dtype != torch.uint8:
            raise TypeError('DDPG camera observations must be uint8 (scaled by 1/255 in the kernel)')
        L.call('smi_cnn_forward', _p(cnn.flat), _p(pix), None, rows, 1, rows, C, H, W, F,
               _p(A1) if A1 is not None else None, _p(A2), _p(P), F + D, self.st)
        if D:
            L.call('smi_copy_cols', _p(low), low.stride(0), rows, D, _p(P[:, F:]), F + D, self.st)
        return P

    def perception_bwd(self, model, pix, rows, store, dH1, wo, ldwo, c1, grad):
        """the critic's first-layer input gradient over the cnn columns, masked by
        the FC ReLU, back through the CNN stem into grad (its flat layout)"""
        cnn = model.perception
        C, H, W = cnn.D_obs
        F, D = model.cnn_dim, model.low_dim
        P = self.bufs[store + '_P']
        dF = self.buf(store + '_dF', (rows, F))
        L.call('smi_linear_backward_input', _p(dH1), c1, rows, c1, _p(wo), ldwo, F, _p(P), F + D,
               _p(dF), F, self.st)
        nb = int(L.lib().smi_cnn_scratch_bytes(rows, C, H, W, F))
        scratch = self.buf('cnn_scratch', ((nb + 3) // 4,))
        L.call('smi_cnn_backward', _p(cnn.flat), _p(pix), None, rows, 1, rows, C, H, W, F,
               _p(self.bufs[store + '_A1']), _p(self.bufs[store + '_A2']), _p(dF), F, _p(grad),
               _p(scratch), nb, self.st)

    def actor_fwd(self, obs, rows, store='a', actor=None):
        actor = actor if actor is not None else self.m.actor
        D, h1, h2, A = actor.dims
        _check_rows(obs, rows, D, 'actor')
        pre = store or 'tmp'
        H1 = self.buf(pre + '_h1', (rows, h1))
        H2 = self.buf(pre + '_h2', (rows, h2))
        out = self.buf(pre + '_act', (rows, A))
        (w1, b1), (w2, b2), (w3, b3) = actor.wb(0), actor.wb(1), actor.wb(2)
        self.lin(obs, obs.stride(0), rows, D, w1, D, b1, h1, RELU, H1, h1)
        X1 = H1
        if actor.use_layernorm:
            X1 = self.buf(pre + '_n1', (rows, h1))
            self.norm(actor, 0, H1, rows, X1, h1, pre + '_ln1')
        self.lin(X1, h1, rows, h1, w2, h1, b2, h2, RELU, H2, h2)
        X2 = H2
        if actor.use_layernorm:
            X2 = self.buf(pre + '_n2', (rows, h2))
            self.norm(actor, 1, H2, rows, X2, h2, pre + '_ln2')
        self.lin(X2, h2, rows, h2, w3, h2, b3, A, TANH, out, A)
        return out if store else out.clone()

    def critic_fwd(self, critic, obs, act, rows, store):
        D, c1, c2, A = critic.dims
        _check_rows(obs, rows, D, 'critic')
        _check_rows(act, rows, A, 'critic action')
        pre = store or 'ctmp'
        CAT = self.buf(pre + '_cat', (rows, c1 + A))
        H2 = self.buf(pre + '_h2', (rows, c2))
        Q = self.buf(pre + '_q', (rows, 1))
        (wo, bo), (wc, bc), (wq, bq) = critic.wb(0), critic.wb(1), critic.wb(2)
        if critic.use_layernorm:
            H1 = self.buf(pre + '_h1', (rows, c1))
            self.lin(obs, obs.stride(0), rows, D, wo, D, bo, c1, RELU, H1, c1)
            self.norm(critic, 0, H1, rows, CAT, c1 + A, pre + '_ln1')
            L.call('smi_copy_cols', _p(act), act.stride(0), rows, A, _p(CAT[:, c1:]), c1 + A,
                   self.st)
        else:   # relu(obs W^T + b) and the action block of the concat in one launch
            L.call('smi_linear_forward_cat', _p(obs), obs.stride(0), rows, D, _p(wo), D, _p(bo), c1,
                   RELU, _p(CAT), c1 + A, _p(act), act.stride(0), A, self.st)
        self.lin(CAT, c1 + A, rows, c1 + A, wc, c1 + A, bc, c2, RELU, H2, c2)
        X2 = H2
        if critic.use_layernorm:
            X2 = self.buf(pre + '_n2', (rows, c2))
            self.norm(critic, 1, H2, rows, X2, c2, pre + '_ln2')
        self.lin(X2, c2, rows, c2, wq, c2, bq, 1, NONE, Q, 1)
        return Q if store else Q.clone()


class DDPGLearner(LearnerHooks):
    """ddpg.py:12-440 on MI355X (low-dim or pixel observations; optional
    layernorm, TD3 options)."""

    def __init__(self, learner_config, env_config, session_config=None, metrics=None,
                 device=None, seed=0, use_graph=False, dp=None, checkpoint_full_state=False,
                 checkpoint=None):
        """dp: None (one GPU) or a data-parallel group exposing `world_size`,
        `rank` and `allreduce_(tensor)` (in-place SUM, stream-ordered), e.g.
        learner.TorchDistAllReduce() over RCCL (SURVEY §8(e) DDPG row).  Each rank
        passes its own `replay.batch_size` rows; every gradient is averaged over
        the ranks before clip + Adam, which equals the reference's mean loss on
        the concatenated global batch (equal shards).  Initial weights are
        broadcast from rank 0 (learner.replicate_from_rank0), so parameters stay
        replicated whatever seed each rank passes.
        metrics / checkpoint: as PPOLearner's (session.py): learn() reports the
        statistics and calls periodic_checkpoint(global_steps=
        current_iteration) as ddpg.py:371-376 does."""
        L.require_gpu()
        self.checkpoint_full_state = bool(checkpoint_full_state)
        self.dp = dp if dp is not None and dp.world_size > 1 else None
        self.learner_config = lc = learner_config if isinstance(learner_config, Config) else Config(learner_config)
        self.env_config = ec = env_config if isinstance(env_config, Config) else Config(env_config)
        self.session_config = session_config
        self._init_hooks(metrics, checkpoint)
        self.device = torch.device(device) if device is not None else \
            torch.device('cuda', torch.cuda.current_device())
        L.ensure_workspace(self.device)
        self._ctx = L.Context(self.device)      # this learner's own workspace (re-entrancy)
        self.current_iteration = 0
        self.batch_size = lc.replay.batch_size
        self.discount_factor = lc.algo.gamma
        self.n_step = lc.algo.n_step
        self.is_pixel_input = ec.get('pixel_input', False)
        self.use_layernorm = lc.model.use_layernorm
        net = lc.algo.network
        self.use_double_critic = net.use_double_critic
        self.use_action_regularization = net.use_action_regularization
        tu = net.target_update
        self.target_update_type = tu.type
        if tu.type == 'soft':
            self.target_update_tau = tu.tau
        elif tu.type == 'hard':
            self.target_update_counter = 0
            self.target_update_interval = tu.interval
        else:
            raise ConfigError('Unsupported ddpg update type: {}'.format(tu.type))
        self.clip_actor_gradient = net.clip_actor_gradient
        self.actor_gradient_clip_value = net.actor_gradient_value_clip
        self.clip_critic_gradient = net.clip_critic_gradient
        self.critic_gradient_clip_value = net.critic_gradient_value_clip
        self.action_dim = ec.action_spec['dim'][0]
        gen = torch.Generator().manual_seed(seed)
        cs = lc.model.get('conv_spec', {})
        conv = dict(conv_out_channels=cs.get('out_channels'), conv_kernel_sizes=cs.get('kernel_sizes'),
                    conv_strides=cs.get('strides'), conv_hidden_dim=cs.get('hidden_output_dim'))
        mk = lambda: DDPGModel(ec.obs_spec, self.action_dim, self.use_layernorm,  # noqa: E731
                               lc.model.actor_fc_hidden_sizes, lc.model.critic_fc_hidden_sizes,
                               device=self.device, generator=gen, **conv)
        self.model = mk()
        self.model_target = mk()
        if self.use_double_critic:                      # ddpg.py:119-145 (critic_only twins)
            mk2 = lambda: DDPGModel(ec.obs_spec, self.action_dim, self.use_layernorm,  # noqa: E731
                                    lc.model.actor_fc_hidden_sizes,
                                    lc.model.critic_fc_hidden_sizes, critic_only=True,
                                    device=self.device, generator=gen, **conv)
            self.model2 = mk2()
            self.model_target2 = mk2()
        self.is_pixel_input = self.model.is_pixel_input
        from .learner import replicate_from_rank0
        flats = [self.model.actor.flat, self.model.critic.flat]
        if self.use_double_critic:
            flats.append(self.model2.critic.flat)
        if self.is_pixel_input:
            flats.append(self.model.perception.flat)
            if self.use_double_critic:
                flats.append(self.model2.perception.flat)
        if self.is_pixel_input:        # the target perceptions keep their own init (below)
            flats.append(self.model_target.perception.flat)
            if self.use_double_critic:
                flats.append(self.model_target2.perception.flat)
        replicate_from_rank0(self.dp, flats)
        # ddpg.py:174-178: the constructor hard-syncs the target actor and
        # critic(s) only; a target perception keeps its own random init until
        # the first target update
        self._hard_update(perception=False)
        dev = self.device
        self.opt = {}
        groups = [('critic', self.model.critic.flat, net.lr_critic, net.critic_regularization),
                  ('actor', self.model.actor.flat, net.lr_actor, net.actor_regularization)]
        if self.use_double_critic:                      # critic_optim2 (ddpg.py:163-168)
            groups.append(('critic2', self.model2.critic.flat, net.lr_critic,
                           net.critic_regularization))
        if self.is_pixel_input:                         # the perception joins the critic optimizer
            groups.append(('critic_cnn', self.model.perception.flat, net.lr_critic,
                           net.critic_regularization))
            if self.use_double_critic:
                groups.append(('critic2_cnn', self.model2.perception.flat, net.lr_critic,
                               net.critic_regularization))
        # gradient buffers packed for the data-parallel exchange: [critic | cnn |
        # critic2 | cnn2] (independent, one all-reduce) and [actor | 12 statistics]
        nc = self.model.critic.flat.numel()
        nq = self.model.perception.flat.numel() if self.is_pixel_input else 0
        na = self.model.actor.flat.numel()
        self._critic_pack = torch.zeros((nc + nq) * (2 if self.use_double_critic else 1), device=dev)
        self._actor_pack = torch.zeros(na + 12, device=dev)
        packs = {'critic': self._critic_pack[:nc], 'critic_cnn': self._critic_pack[nc:nc + nq],
                 'critic2': self._critic_pack[nc + nq:2 * nc + nq],
                 'critic2_cnn': self._critic_pack[2 * nc + nq:], 'actor': self._actor_pack[:na]}
        for name, flat, lr, wd in groups:
            self.opt[name] = {'m': torch.zeros_like(flat), 'v': torch.zeros_like(flat),
                              'step': torch.zeros(1, dtype=torch.int32, device=dev),
                              'lr': torch.tensor([lr], dtype=torch.float32, device=dev),
                              'wd': float(wd), 'g': packs[name]}
        self.stats_buf = self._actor_pack[na:]
        self._bufs = {}
        self.kernel_events = None
        # hipGraph replay of the update (learn() -> _optimize_graphed); the TD3
        # smoothing noise is a fresh host draw per step, so that option stays eager
        self.use_graph = bool(use_graph) and self.dp is None and not (
            self.use_double_critic and self.use_action_regularization)
        self._graph = None
        self._gin = None

    # ------------------------------------------------------------ helpers
    def _target_pairs(self, perception=True):
        """(target, source) flat buffers of the target update (ddpg.py:409-428)"""
        pairs = [(self.model_target.actor.flat, self.model.actor.flat),
                 (self.model_target.critic.flat, self.model.critic.flat)]
        if self.use_double_critic:
            pairs.append((self.model_target2.critic.flat, self.model2.critic.flat))
            if self.is_pixel_input and perception:
                pairs.append((self.model_target2.perception.flat, self.model2.perception.flat))
        if self.is_pixel_input and perception:
            pairs.append((self.model_target.perception.flat, self.model.perception.flat))
        return pairs

    def _hard_update(self, perception=True):
        with torch.no_grad():
            for t, s_ in self._target_pairs(perception):
                t.copy_(s_)

    def _dp_mean_(self, t):
        """Average a per-rank gradient / statistics buffer over the ranks."""
        if self.dp is not None:
            self.dp.allreduce_(t)
            t.mul_(1.0 / self.dp.world_size)

    def _adam(self, name, flat, clip_value, st):
        o = self.opt[name]
        L.call('smi_adam_clip', _p(flat), _p(o['g']), _p(o['m']), _p(o['v']), flat.numel(),
               _p(o['step']), _p(o['lr']), 0.9, 0.999, 1e-8, o['wd'], 0.0, float(clip_value),
               None, None, st)

    def preprocess(self, batch):                                         # ddpg.py:186-242
        """numpy -> device tensors; camera frames stay uint8 (the reference's
        .float() and the model's / 255, ddpg_net.py:90-95, happen in the conv
        kernel, bit-equal to torch's u8 -> float / 255)"""
        out = {}
        for k in ('obs', 'obs_next'):
            v = batch[k]
            if isinstance(v, dict):
                o = {}
                if 'pixel' in v:
                    o['pixel'] = {'camera0': torch.as_tensor(np.asarray(v['pixel']['camera0']),
                                                             dtype=torch.uint8).to(self.device)}
                if 'low_dim' in v:
                    o['low_dim'] = {'flat_inputs': torch.as_tensor(
                        v['low_dim']['flat_inputs'], dtype=torch.float32).to(self.device)}
                out[k] = o if 'pixel' in v else o['low_dim']['flat_inputs']
                continue
            out[k] = torch.as_tensor(v, dtype=torch.float32).to(self.device, non_blocking=True)
        for k in ('actions', 'rewards', 'dones'):
            out[k] = torch.as_tensor(batch[k], dtype=torch.float32).to(self.device, non_blocking=True)
        return Config(out)

    # --------------------------------------------------------- _optimize
    def _optimize(self, obs, actions, rewards, obs_next, done,           # ddpg.py:244-352
                  target_update=True):
        B = actions.shape[0]
        st = L.stream(self.device)
        net = _Net(self.model, self._bufs)
        tnet = _Net(self.model_target, self._bufs)
        D, h1, h2, A = self.model.actor.dims
        _, c1, c2, _ = self.model.critic.dims
        rs = rewards.stride(0) if rewards.dim() == 2 else 1
        pix = pix_n = None
        obs_next2 = obs_next
        if self.is_pixel_input:
            # forward_perception (ddpg_net.py:69-79) of every model that reads the
            # batch: the target model(s) on obs_next, the model(s) on obs (their
            # conv activations kept for the critic backward)
            pix, pix_n = obs['pixel']['camera0'].contiguous(), obs_next['pixel']['camera0'].contiguous()
            low = obs['low_dim']['flat_inputs'] if 'low_dim' in obs else None
            low_n = obs_next['low_dim']['flat_inputs'] if 'low_dim' in obs_next else None
            obs_next = tnet.perception_fwd(self.model_target, pix_n, low_n, B, 'tp')
            if self.use_double_critic:
                obs_next2 = tnet.perception_fwd(self.model_target2, pix_n, low_n, B, 't2p')
            obs2 = net.perception_fwd(self.model2, pix, low, B, 'q2p', keep=True) \
                if self.use_double_critic else None
            obs = net.perception_fwd(self.model, pix, low, B, 'cp', keep=True)
        else:
            obs2, obs_next2 = obs, obs_next
        # target: y = r + gamma^n * Q'(s', mu'(s')) * (1 - d)           (ddpg.py:266-284)
        a_t = tnet.actor_fwd(obs_next, B, store='ta')
        q_t = tnet.critic_fwd(self.model_target.critic, obs_next, a_t, B, store='tc')
        q_t2 = None
        if self.use_double_critic:
            # TD3 (ddpg.py:267-283): target policy smoothing noise is drawn on the
            # host from numpy's global RNG exactly as the reference does, and only
            # the twin target sees it (next_Q_target was computed before the noise)
            a_t2 = a_t
            if self.use_action_regularization:
                # data parallel: every rank draws the global batch's noise from
                # the same stream and keeps its own rows
                W, r = (self.dp.world_size, self.dp.rank) if self.dp is not None else (1, 0)
                noise = np.clip(np.random.normal(0, 0.2, size=(self.batch_size * W, self.action_dim)),
                                -0.5, 0.5)[r * self.batch_size:(r + 1) * self.batch_size]
                a_t2 = (a_t + torch.tensor(noise, dtype=torch.float32).to(self.device)).clamp(-1, 1)
            q_t2 = tnet.critic_fwd(self.model_target2.critic, obs_next2, a_t2.contiguous(), B,
                                   store='t2c')
        y = net.buf('y', (B, 1))
        r1 = rewards if rewards.is_contiguous() else rewards.contiguous()
        d1 = done if done.is_contiguous() else done.contiguous()
        L.call('smi_ddpg_target', _p(r1), _p(d1), _p(q_t), _p(q_t2) if q_t2 is not None else None,
               B, float(pow(self.discount_factor, self.n_step)), _p(y), st)
        # critic update (ddpg.py:287-310)
        crit = self.model.critic
        q = net.critic_fwd(crit, obs, actions, B, store='c')
        dq = net.buf('dq', (B, 1))
        L.call('smi_mse_grad', _p(q), 1, _p(y), B, _p(dq), _p(self.stats_buf[1:2]), st)
        g = self.opt['critic']['g']
        cnn = (self.model, pix, 'cp', self.opt['critic_cnn']['g']) if self.is_pixel_input else None
        self._critic_backward(net, crit, obs, B, dq, 'c', g, st, need_obs_grad=True, cnn=cnn)
        cclip = self.critic_gradient_clip_value if self.clip_critic_gradient else 0.0
        if self.use_double_critic:                      # second critic (ddpg.py:312-320)
            # its gradient does not depend on the first critic's step: both are
            # computed first and averaged over the ranks in one exchange
            crit2 = self.model2.critic
            q_2 = net.critic_fwd(crit2, obs2, actions, B, store='q2c')
            dq_2 = net.buf('dq_2', (B, 1))
            # the reference reports this critic's loss as 'critic_loss'
            L.call('smi_mse_grad', _p(q_2), 1, _p(y), B, _p(dq_2), _p(self.stats_buf[1:2]), st)
            cnn2 = (self.model2, pix, 'q2p', self.opt['critic2_cnn']['g']) if self.is_pixel_input \
                else None
            self._critic_backward(net, crit2, obs2, B, dq_2, 'q2c', self.opt['critic2']['g'], st,
                                  need_obs_grad=True, cnn=cnn2)
            L.call('smi_ddpg_stats', _p(actions), actions.stride(0), self.action_dim, _p(rewards),
                   rewards.stride(0) if rewards.dim() == 2 else 1, _p(y), _p(q_2), 1, B,
                   _p(self.stats_buf[8:12]), st)         # [.., .., .., Q_policy2]
        self._dp_mean_(self._critic_pack)
        self._adam('critic', crit.flat, cclip, st)
        if self.is_pixel_input:         # the perception: critic optimizer, no value clip
            self._adam('critic_cnn', self.model.perception.flat, 0.0, st)
        if self.use_double_critic:
            self._adam('critic2', self.model2.critic.flat, cclip, st)
            if self.is_pixel_input:
                self._adam('critic2_cnn', self.model2.perception.flat, 0.0, st)
        # actor update with the updated critic (ddpg.py:323-333)
        act = self.model.actor
        a = net.actor_fwd(obs, B, store='a')
        q2 = net.critic_fwd(crit, obs, a, B, store='c2')
        dq2 = net.buf('dq2', (B, 1))
        L.call('smi_neg_mean_grad', _p(q2), 1, B, _p(dq2), _p(self.stats_buf[0:1]), st)
        dA = self._critic_backward(net, crit, obs, B, dq2, 'c2', None, st, need_obs_grad=False)
        self._actor_backward(net, act, obs, B, dA, self.opt['actor']['g'], st)
        # statistics (ddpg.py:335-345); shard means -> global means together with
        # the actor gradient (one exchange)
        L.call('smi_ddpg_stats', _p(actions), actions.stride(0), A, _p(rewards), rs, _p(y), _p(q), 1,
               B, _p(self.stats_buf[2:6]), st)
        self._dp_mean_(self._actor_pack)
        self._adam('actor', act.flat,
                   self.actor_gradient_clip_value if self.clip_actor_gradient else 0.0, st)
        if target_update:
            self._target_update()

    def _critic_backward(self, net, crit, obs, B, dq, pre, g, st, need_obs_grad, cnn=None):
        """Backward through CriticNetworkX.  With g: weight grads into g (flat),
        the three weight-gradient GEMMs as one grouped launch (smi_dw_group_*);
        cnn = (model, pixels, perception store, gradient) continues through the
        model's perception (pixel inputs).  Always returns d loss / d action
        (B, A) when g is None."""
        if g is None or not _DW_GROUP:
            return self._critic_backward_body(net, crit, obs, B, dq, pre, g, st, cnn)
        L.call('smi_dw_group_begin')
        try:
            return self._critic_backward_body(net, crit, obs, B, dq, pre, g, st, cnn)
        finally:
            L.call('smi_dw_group_flush', st)   # always flush: nothing stays queued

    def _critic_backward_body(self, net, crit, obs, B, dq, pre, g, st, cnn=None):
        D, c1, c2, A = crit.dims
        ln = crit.use_layernorm
        CAT = net.bufs[pre + '_cat']
        H2 = net.bufs[pre + '_h2']
        X2 = net.bufs[pre + '_n2'] if ln else H2               # input of the Q layer
        (wo, bo), (wc, bc), (wq, bq) = crit.wb(0), crit.wb(1), crit.wb(2)
        dH2 = net.buf('dH2', (B, c2))
        if ln:      # d/d(norm output), then through the norm and the ReLU
            dN2 = net.buf('dN2', (B, c2))
            L.call('smi_linear_backward_input', _p(dq), 1, B, 1, _p(wq), c2, c2, None, 0, _p(dN2),
                   c2, st)
            net.norm_bwd(crit, 1, dN2, H2, B, dH2, g, pre + '_ln2')
        else:
            L.call('smi_linear_backward_input', _p(dq), 1, B, 1, _p(wq), c2, c2, _p(H2), c2,
                   _p(dH2), c2, st)
        if g is not None:
            L.call('smi_linear_backward_weight', _p(dq), 1, B, 1, _p(X2), c2, c2,
                   _p(g[crit.off(wq):]), c2, _p(g[crit.off(bq):]), 0, st)
            L.call('smi_linear_backward_weight', _p(dH2), c2, B, c2, _p(CAT), c1 + A, c1 + A,
                   _p(g[crit.off(wc):]), c1 + A, _p(g[crit.off(bc):]), 0, st)
            dH1 = net.buf('dH1c', (B, c1))
            if ln:
                dN1 = net.buf('dN1c', (B, c1))
                L.call('smi_linear_backward_input', _p(dH2), c2, B, c2, _p(wc), c1 + A, c1, None, 0,
                       _p(dN1), c1, st)
                net.norm_bwd(crit, 0, dN1, net.bufs[pre + '_h1'], B, dH1, g, pre + '_ln1')
            else:
                L.call('smi_linear_backward_input', _p(dH2), c2, B, c2, _p(wc), c1 + A, c1, _p(CAT),
                       c1 + A, _p(dH1), c1, st)
            L.call('smi_linear_backward_weight', _p(dH1), c1, B, c1, _p(obs), obs.stride(0), D,
                   _p(g[crit.off(wo):]), D, _p(g[crit.off(bo):]), 0, st)
            if cnn is not None:
                model, pix, store, gc = cnn
                net.perception_bwd(model, pix, B, store, dH1, wo, D, c1, gc)
            return None
        dA = net.buf('dA', (B, A))
        L.call('smi_linear_backward_input', _p(dH2), c2, B, c2, _p(wc[:, c1:]), c1 + A, A, None, 0,
               _p(dA), A, st)
        return dA

    def _actor_backward(self, net, act, obs, B, dA, g, st):
        """Backward through ActorNetworkX into g; its three weight-gradient
        GEMMs as one grouped launch (smi_dw_group_*)."""
        if not _DW_GROUP:
            return self._actor_backward_body(net, act, obs, B, dA, g, st)
        L.call('smi_dw_group_begin')
        try:
            self._actor_backward_body(net, act, obs, B, dA, g, st)
        finally:
            L.call('smi_dw_group_flush', st)

    def _actor_backward_body(self, net, act, obs, B, dA, g, st):
        D, h1, h2, A = act.dims
        ln = act.use_layernorm
        H1, H2, out = net.bufs['a_h1'], net.bufs['a_h2'], net.bufs['a_act']
        X1 = net.bufs['a_n1'] if ln else H1                     # inputs of layers 2 and 3
        X2 = net.bufs['a_n2'] if ln else H2
        (w1, b1), (w2, b2), (w3, b3) = act.wb(0), act.wb(1), act.wb(2)
        dZ = net.buf('dZ3', (B, A))
        L.call('smi_tanh_backward', _p(dA), A, _p(out), A, B, A, _p(dZ), A, st)
        L.call('smi_linear_backward_weight', _p(dZ), A, B, A, _p(X2), h2, h2, _p(g[act.off(w3):]), h2,
               _p(g[act.off(b3):]), 0, st)
        dH2 = net.buf('dH2a', (B, h2))
        if ln:
            dN2 = net.buf('dN2a', (B, h2))
            L.call('smi_linear_backward_input', _p(dZ), A, B, A, _p(w3), h2, h2, None, 0, _p(dN2), h2,
                   st)
            net.norm_bwd(act, 1, dN2, H2, B, dH2, g, 'a_ln2')
        else:
            L.call('smi_linear_backward_input', _p(dZ), A, B, A, _p(w3), h2, h2, _p(H2), h2, _p(dH2),
                   h2, st)
        L.call('smi_linear_backward_weight', _p(dH2), h2, B, h2, _p(X1), h1, h1, _p(g[act.off(w2):]), h1,
               _p(g[act.off(b2):]), 0, st)
        dH1 = net.buf('dH1a', (B, h1))
        if ln:
            dN1 = net.buf('dN1a', (B, h1))
            L.call('smi_linear_backward_input', _p(dH2), h2, B, h2, _p(w2), h1, h1, None, 0, _p(dN1),
                   h1, st)
            net.norm_bwd(act, 0, dN1, H1, B, dH1, g, 'a_ln1')
        else:
            L.call('smi_linear_backward_input', _p(dH2), h2, B, h2, _p(w2), h1, h1, _p(H1), h1,
                   _p(dH1), h1, st)
        L.call('smi_linear_backward_weight', _p(dH1), h1, B, h1, _p(obs), obs.stride(0), D,
               _p(g[act.off(w1):]), D, _p(g[act.off(b1):]), 0, st)

    def _target_update(self):                                            # ddpg.py:403-428
        st = L.stream(self.device)
        if self.target_update_type == 'soft':
            for t, s in self._target_pairs():
                L.call('smi_soft_update', _p(t), _p(s), t.numel(), float(self.target_update_tau), st)
        else:
            self.target_update_counter += 1
            if self.target_update_counter % self.target_update_interval == 0:
                self._hard_update()

    # ------------------------------------------------------- reference API
    def learn(self, batch):                                              # ddpg.py:354-376
        self.current_iteration += 1
        self._ctx.make_current()
        if not isinstance(batch['actions'], torch.Tensor) or not batch['actions'].is_cuda:
            batch = self.preprocess(batch)
        obs, obs_next = batch['obs'], batch['obs_next']
        if not self.is_pixel_input:
            obs = obs['low_dim']['flat_inputs'] if isinstance(obs, dict) else obs
            obs_next = obs_next['low_dim']['flat_inputs'] if isinstance(obs_next, dict) else obs_next
        ins = (obs, batch['actions'], batch['rewards'], obs_next, batch['dones'])
        if self.use_graph and not self.is_pixel_input:
            self._optimize_graphed(*ins)
        else:
            self._optimize(*ins)
        self._report_metrics(self.current_iteration)                     # ddpg.py:371
        self.periodic_checkpoint(global_steps=self.current_iteration, score=None)

    def _optimize_graphed(self, obs, actions, rewards, obs_next, done):
        """One _optimize as a hipGraph replay (the step is ~40 small launches at
        batch 512, so host launch overhead, not the GPU, bounds it).  The first
        call runs eagerly (it is that call's update, and it sizes every scratch
        buffer), then captures the same launch sequence over static input
        buffers; later calls copy their inputs in (skipped when the caller
        already wrote them: graph_inputs()) and replay.  The target update stays
        on the host, where its interval counter lives (ddpg.py:403-428)."""
        ins = (obs, actions, rewards, obs_next, done)
        if self._graph is None:
            self._optimize(*ins)
            self._gin = [torch.zeros(tuple(t.shape), dtype=torch.float32, device=self.device)
                         for t in ins]
            g = torch.cuda.CUDAGraph()
            with L.gc_paused(), torch.cuda.graph(g, capture_error_mode='thread_local'):
                self._optimize(*self._gin, target_update=False)
            self._graph = g
            return
        for s, t in zip(self._gin, ins):
            if s.data_ptr() != t.data_ptr():
                s.copy_(t)
        self._graph.replay()
        self._target_update()

    def graph_inputs(self):
        """Static (obs, actions, rewards, obs_next, dones) buffers of the captured
        step (None before the first learn() in graph mode)."""
        return None if self._gin is None else dict(zip(
            ('obs', 'actions', 'rewards', 'obs_next', 'dones'), self._gin))

    def _host_scalars(self):
        return {}

    def last_stats(self):
        return self._stats_dict(self.stats_buf.cpu().numpy(), {})

    def _stats_dict(self, v, host):
        out = {'actor_loss': float(v[0]), 'critic_loss': float(v[1]), 'action_norm': float(v[2]),
               'rewards': float(v[3]), 'Q_target': float(v[4]), 'Q_policy': float(v[5])}
        if self.use_double_critic:
            out['Q_policy2'] = float(v[11])
        return out

    def module_dict(self):
        return {'ddpg': self.model}

    def checkpoint_attributes(self):                                     # ddpg.py:383-387
        """Reference list (+ the TD3 twin critics, which the reference omits);
        checkpoint_full_state adds the Adam moments / steps and the hard-update
        counter for a bit-identical continuation."""
        attrs = ['current_iteration', 'model', 'model_target']
        if self.use_double_critic:
            attrs += ['model2', 'model_target2']
        if self.checkpoint_full_state:
            attrs += ['optimizer_state_host']
        return attrs

    @property
    def optimizer_state_host(self):
        out = {name: {k: o[k].detach().cpu().clone() for k in ('m', 'v', 'step', 'lr')}
               for name, o in self.opt.items()}
        out['target_update_counter'] = getattr(self, 'target_update_counter', 0)
        return out

    @optimizer_state_host.setter
    def optimizer_state_host(self, d):
        with torch.no_grad():
            for name, o in self.opt.items():
                for k in ('m', 'v', 'step', 'lr'):
                    o[k].copy_(torch.as_tensor(d[name][k]).to(o[k].device))
        if self.target_update_type == 'hard':
            self.target_update_counter = d['target_update_counter']

    def _prefetcher_preprocess(self, batch):
        from .aggregator import FrameStackPreprocessor, SSARAggregator
        if not self.env_config.get('frame_stack_concatenate_on_env', True):
            batch = FrameStackPreprocessor(self.env_config.frame_stacks).preprocess_list(batch)
        return SSARAggregator(self.env_config.obs_spec, self.env_config.action_spec).aggregate(batch)
