"""ORACLE (test infrastructure only — see oracle/__init__.py).

fp32 CPU restatement of the reference PPO learner hot path, op by op:
  DiagGauss            surreal/model/ppo_net.py:13-91
  ZFilter              surreal/model/z_filter.py:23-79
  RewardFilter         surreal/model/reward_filter.py:5-56 (its '=' bug at :42 kept)
  actor / critic MLPs  surreal/model/model_builders/builders.py:86-175
  PPOModel forward     surreal/model/ppo_net.py:94-375 (low-dim, optional LSTM and
                       pixel CNNStemNetwork, builders.py:8-33, on obs/255)
  GAE / returns        surreal/learner/ppo.py:355-418
  clip / adapt / value losses and updates   ppo.py:194-353
  _optimize            ppo.py:487-586
  _post_publish        ppo.py:637-666
Layers are plain torch.nn (torchx is not available: SURVEY.md §8(c)); weights
are exchanged with the product through the flat MLP layout of
include/surreal_mi.h so both start from identical parameters.
"""
import math

import numpy as np
import torch
import torch.nn as nn


def cfg_get(cfg, path, default=None):
    cur = cfg
    for k in path.split('.'):
        if cur is None or k not in cur:
            return default
        cur = cur[k]
    return cur


# ---------------------------------------------------------------- DiagGauss
class DiagGaussRef:
    """ppo_net.py:13-91."""

    def __init__(self, d):
        self.d = d

    def loglikelihood(self, a, prob):                       # :29-40
        if a.dim() == 3:
            a = a.reshape(-1, self.d)
            prob = prob.reshape(-1, 2 * self.d)
        mu, sd = prob[:, :self.d], prob[:, self.d:]
        quad = ((a - mu) / sd).pow(2).sum(dim=1, keepdim=True)
        return -0.5 * quad - 0.5 * np.log(2.0 * np.pi) * self.d - sd.log().sum(dim=1, keepdim=True)

    def likelihood(self, a, prob):                          # :42-46
        return torch.clamp(self.loglikelihood(a, prob).exp(), min=1e-5)

    def kl(self, p0, p1):                                   # :48-62
        if p0.dim() == 3:
            p0 = p0.reshape(-1, 2 * self.d)
            p1 = p1.reshape(-1, 2 * self.d)
        m0, s0, m1, s1 = p0[:, :self.d], p0[:, self.d:], p1[:, :self.d], p1[:, self.d:]
        return (s1 / s0).log().sum(dim=1) + \
            ((s0.pow(2) + (m0 - m1).pow(2)) / (2.0 * s1.pow(2))).sum(dim=1) - 0.5 * self.d

    def entropy(self, prob):                                # :64-72
        if prob.dim() == 3:
            prob = prob.reshape(-1, 2 * self.d)
        return 0.5 * prob[:, self.d:].log().sum(dim=1) + .5 * np.log(2 * np.pi * np.e) * self.d


# ------------------------------------------------------------------ ZFilter
class ZFilterRef(nn.Module):
    """z_filter.py:23-79: running sum / sum of squares / count (init eps)."""

    def __init__(self, in_size, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.in_size = in_size
        self.register_buffer('running_sum', torch.zeros(in_size))
        self.register_buffer('running_sumsq', eps * torch.ones(in_size))
        self.register_buffer('count', torch.tensor([eps], dtype=torch.float32))

    def z_update(self, x):                                  # :44-57
        if x.dim() == 3:
            x = x.reshape(-1, self.in_size)
        self.running_sum += torch.sum(x, dim=0)
        self.running_sumsq += torch.sum(x * x, dim=0)
        self.count += float(len(x))

    def forward(self, inputs):                              # :59-79
        shape = inputs.size()
        x = inputs.reshape(-1, shape[-1])
        mean = self.running_sum / self.count
        std = torch.clamp((self.running_sumsq / self.count - mean.pow(2)).pow(0.5), min=self.eps)
        return torch.clamp((x - mean) / std, -5.0, 5.0).reshape(shape)

    def running_mean(self):
        return (self.running_sum / self.count).numpy()

    def running_std(self):
        return ((self.running_sumsq / self.count) - (self.running_sum / self.count).pow(2)).pow(0.5).numpy()

    def running_square(self):
        return (self.running_sumsq / self.count).numpy()


class RewardFilterRef(nn.Module):
    """reward_filter.py:5-56 (running_sumsq assigned, not accumulated: :42)."""

    def __init__(self, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.register_buffer('count', torch.tensor(eps, dtype=torch.float32))
        self.register_buffer('running_sum', torch.tensor(0.0, dtype=torch.float32))
        self.register_buffer('running_sumsq', torch.tensor(0.0, dtype=torch.float32))

    def update(self, x):
        self.count += float(np.prod(x.size()))
        self.running_sum += x.sum()
        self.running_sumsq = (x * x).sum()

    def forward(self, x):
        mean = self.running_sum / self.count
        std = torch.clamp((self.running_sumsq / self.count - mean.pow(2)).pow(0.5), min=self.eps)
        return torch.clamp((x - mean) / std, -5.0, 5.0)


# --------------------------------------------------------------------- nets
class MLP3(nn.Module):
    """Linear-ReLU-Linear-ReLU-Linear[-Tanh] (builders.py:100-110,149-157)."""

    def __init__(self, d_in, h1, h2, d_out, tanh):
        super().__init__()
        self.l1 = nn.Linear(d_in, h1)
        self.l2 = nn.Linear(h1, h2)
        self.l3 = nn.Linear(h2, d_out)
        self.tanh = tanh

    def forward(self, x):
        x = torch.relu(self.l1(x))
        x = torch.relu(self.l2(x))
        x = self.l3(x)
        return torch.tanh(x) if self.tanh else x

    def flat(self):
        return torch.cat([p.detach().reshape(-1) for p in
                          (self.l1.weight, self.l1.bias, self.l2.weight, self.l2.bias,
                           self.l3.weight, self.l3.bias)])

    def load_flat(self, f):
        o = 0
        with torch.no_grad():
            for p in (self.l1.weight, self.l1.bias, self.l2.weight, self.l2.bias,
                      self.l3.weight, self.l3.bias):
                n = p.numel()
                p.copy_(torch.as_tensor(f[o:o + n]).reshape(p.shape))
                o += n
        return o


class ActorRef(nn.Module):
    """PPO_ActorNetwork (builders.py:86-132): mean = tanh(MLP), std = exp(log_var)."""

    def __init__(self, d_in, d_act, hidden, init_log_sig):
        super().__init__()
        self.model = MLP3(d_in, hidden[0], hidden[1], d_act, tanh=True)
        self.log_var = nn.Parameter(torch.zeros(1, d_act) + init_log_sig)

    def forward(self, obs):
        shape = obs.size()
        high = obs.dim() == 3
        if high:
            obs = obs.reshape(-1, shape[2])
        mean = self.model(obs)
        std = torch.exp(self.log_var) * torch.ones_like(mean)
        out = torch.cat((mean, std), dim=1)
        if high:
            out = out.reshape(shape[0], shape[1], -1)
        return out

    def flat(self):
        return torch.cat([self.model.flat(), self.log_var.detach().reshape(-1)])

    def load_flat(self, f):
        o = self.model.load_flat(f)
        with torch.no_grad():
            self.log_var.copy_(torch.as_tensor(f[o:o + self.log_var.numel()]).reshape(self.log_var.shape))


class CriticRef(nn.Module):
    """PPO_CriticNetwork (builders.py:135-175)."""

    def __init__(self, d_in, hidden):
        super().__init__()
        self.model = MLP3(d_in, hidden[0], hidden[1], 1, tanh=False)

    def forward(self, obs):
        shape = obs.size()
        high = obs.dim() == 3
        if high:
            obs = obs.reshape(-1, shape[2])
        v = self.model(obs)
        if high:
            v = v.reshape(shape[0], shape[1], 1)
        return v

    def flat(self):
        return self.model.flat()

    def load_flat(self, f):
        self.model.load_flat(f)


def cnn_stem_ref(C, H, W, F):
    """CNNStemNetwork (builders.py:8-33) with its default conv_channels [16, 32],
    kernel_sizes [8, 4], strides [4, 2], no padding (torchx Conv2d default)."""
    H1, W1 = (H - 8) // 4 + 1, (W - 8) // 4 + 1
    H2, W2 = (H1 - 4) // 2 + 1, (W1 - 4) // 2 + 1
    return nn.Sequential(nn.Conv2d(C, 16, 8, 4), nn.ReLU(), nn.Conv2d(16, 32, 4, 2), nn.ReLU(),
                         nn.Flatten(), nn.Linear(32 * H2 * W2, F), nn.ReLU())


class PPOModelRef(nn.Module):
    """PPOModel (ppo_net.py:94-375): low-dim observations, optional LSTM stem and
    optional pixel stem.  With pixels an observation is the pair (low_dim or
    None, camera0 uint8 (..., C, H, W))."""

    def __init__(self, obs_dim, act_dim, actor_hidden, critic_hidden, init_log_sig,
                 use_z_filter, rnn=False, rnn_hidden=100, rnn_layer=1, pixel=None, cnn_feat=256):
        super().__init__()
        self.use_z_filter = use_z_filter
        self.rnn = rnn
        self.pixel = pixel
        self.cnn_stem = cnn_stem_ref(*pixel, cnn_feat) if pixel is not None else None
        d_stem = obs_dim + (cnn_feat if pixel is not None else 0)
        self.rnn_stem = nn.LSTM(d_stem, rnn_hidden, rnn_layer, batch_first=True) if rnn else None
        d_in = rnn_hidden if rnn else d_stem
        self.actor = ActorRef(d_in, act_dim, actor_hidden, init_log_sig)
        self.critic = CriticRef(d_in, critic_hidden)
        if use_z_filter:
            self.z_filter = ZFilterRef(obs_dim)

    def _features(self, x, cells):
        pix = None
        if self.pixel is not None:
            x, pix = x
        parts = []
        if x is not None:
            parts.append(self.z_filter.forward(x) if self.use_z_filter else x)
        if pix is not None:                                 # ppo_net.py:268-273, 368-375
            lead = pix.shape[:-3]
            img = pix.reshape(-1, *pix.shape[-3:])
            dt = self.actor.log_var.dtype
            img = img / 255.0 if dt == torch.float32 else img.to(dt) / 255.0
            parts.append(self.cnn_stem(img).reshape(*lead, -1))
        x = parts[0] if len(parts) == 1 else torch.cat(parts, -1)
        if self.rnn:
            x, _ = self.rnn_stem(x, cells)
            x = x.contiguous()
        return x

    def forward_actor(self, x, cells=None):                 # ppo_net.py:253-282
        return self.actor(self._features(x, cells))

    def forward_critic(self, x, cells=None):                # ppo_net.py:284-315
        return self.critic(self._features(x, cells))

    def forward_actor_expose_cells(self, x, cells=None):    # ppo_net.py:317-352
        """one agent step: x (1, D) [or a (low, pixel) pair]; with the LSTM
        the stem input is viewed (1, 1, -1) and the new (h, c) returned"""
        pix = None
        if self.pixel is not None:
            x, pix = x
        parts = []
        if x is not None:
            parts.append(self.z_filter.forward(x) if self.use_z_filter else x)
        if pix is not None:
            img = pix.reshape(-1, *pix.shape[-3:])
            dt = self.actor.log_var.dtype
            img = img / 255.0 if dt == torch.float32 else img.to(dt) / 255.0
            parts.append(self.cnn_stem(img))
        x = parts[0] if len(parts) == 1 else torch.cat(parts, -1)
        if self.rnn:
            x = x.view(1, 1, -1)
            x, cells = self.rnn_stem(x, cells)
            cells = (cells[0].detach(), cells[1].detach())
            x = x.contiguous().view(-1, self.rnn_stem.hidden_size)
        return self.actor(x), cells

    def update_target_params(self, net):                    # ppo_net.py:226-242
        self.actor.load_state_dict(net.actor.state_dict())
        self.critic.load_state_dict(net.critic.state_dict())
        if self.rnn:
            self.rnn_stem.load_state_dict(net.rnn_stem.state_dict())
        if self.pixel is not None:
            self.cnn_stem.load_state_dict(net.cnn_stem.state_dict())
        if self.use_z_filter:
            self.z_filter.load_state_dict(net.z_filter.state_dict())

    def actor_params(self):                                 # ppo_net.py:202-212
        ps = list(self.actor.parameters())
        if self.pixel is not None:
            ps += list(self.cnn_stem.parameters())
        if self.rnn:
            ps += list(self.rnn_stem.parameters())
        return ps

    def critic_params(self):                                # ppo_net.py:214-224
        ps = list(self.critic.parameters())
        if self.pixel is not None:
            ps += list(self.cnn_stem.parameters())
        if self.rnn:
            ps += list(self.rnn_stem.parameters())
        return ps


def _tmap(f, o):
    """apply f to an observation or to each non-None part of a (low, pixel) pair"""
    if isinstance(o, tuple):
        return tuple(None if p is None else f(p) for p in o)
    return f(o)


def _tmap2(f, a, b):
    if isinstance(a, tuple):
        return tuple(None if p is None else f(p, q) for p, q in zip(a, b))
    return f(a, b)


# ---------------------------------------------------------------------- GAE
def gae_and_return(values, rewards, dones, gamma, lam, n_step, horizon, rnn, norm_adv,
                   raw_out=None):
    """ppo.py:371-418 given the critic values (B, T+1).  Returns (adv, ret).
    `values` is masked in place (values[:,1:] *= 1 - dones, ppo.py:387).  The
    gamma / lambda tables are the reference's fp32 torch.pow tables whatever the
    dtype of `values` (fp64 runs of the oracle keep the reference's constants).
    raw_out: optional list that receives the advantages before normalisation."""
    idx = torch.tensor(range(n_step), dtype=torch.float32)
    g = torch.pow(gamma, idx)
    lm = torch.pow(lam, idx)
    values[:, 1:] *= 1 - dones
    if rnn:                                                  # :389-406
        tds = rewards + gamma * values[:, 1:] - values[:, :-1]
        eff_len = n_step - horizon + 1
        g, lm = g[:horizon], lm[:horizon]
        B = values.shape[0]
        ret = torch.zeros(B, eff_len, dtype=values.dtype)
        adv = torch.zeros(B, eff_len, dtype=values.dtype)
        for s in range(eff_len):
            ret[:, s] = torch.sum(g * rewards[:, s:s + horizon], 1) + values[:, s + horizon] * (gamma ** horizon)
            adv[:, s] = torch.sum(tds[:, s:s + horizon] * g * lm, 1)
        if raw_out is not None:
            raw_out.append(adv.clone())
        if norm_adv:
            std, mean = adv.std(), adv.mean()
            adv = (adv - mean) / max(std, 1e-4)
        return adv, ret
    ret = torch.sum(g * rewards, 1) + values[:, -1] * (gamma ** n_step)   # :409
    tds = rewards + gamma * values[:, 1:] - values[:, :-1]               # :410
    gae = torch.sum(tds * g * lm, 1)                                       # :411
    if raw_out is not None:
        raw_out.append(gae.clone())
    if norm_adv:                                                           # :413-416
        std, mean = gae.std(), gae.mean()
        gae = (gae - mean) / max(std, 1e-4)
    return gae.view(-1, 1), ret.view(-1, 1)


def gamma_tables(gamma, lam, n_step):
    idx = torch.tensor(range(n_step), dtype=torch.float32)
    return torch.pow(gamma, idx), torch.pow(lam, idx)


# ----------------------------------------------------------------- learner
class PPOLearnerRef:
    """PPOLearner hyper-parameters and loop (ppo.py:57-192, 194-353, 487-666).

    `lc` is a learner_config tree with the reference's keys (the product's
    surreal_amd.config.Config works).  obs are low-dim tensors (B, T, D).
    dtype=torch.float64 runs the same algorithm in double precision: the
    "truth" the parity tests measure both fp32 implementations against.
    """

    def __init__(self, lc, obs_dim, act_dim, seed=0, pixel=None, dtype=torch.float32):
        torch.manual_seed(seed)
        g = lambda p, d=None: cfg_get(lc, p, d)  # noqa: E731
        self.gamma = g('algo.gamma')
        self.lam = g('algo.advantage.lam')
        self.n_step = g('algo.n_step')
        self.use_z_filter = g('algo.use_z_filter')
        self.use_r_filter = g('algo.use_r_filter')
        self.norm_adv = g('algo.advantage.norm_adv')
        self.batch_size = g('replay.batch_size')
        self.action_dim = act_dim
        self.ppo_mode = g('algo.ppo_mode')
        self.rnn = g('algo.rnn.if_rnn_policy')
        self.horizon = g('algo.rnn.horizon')
        self.epoch_policy = g('algo.consts.epoch_policy')
        self.epoch_baseline = g('algo.consts.epoch_baseline')
        self.kl_target = g('algo.consts.kl_target')
        self.adjust_threshold = g('algo.consts.adjust_threshold')
        self.reward_scale = g('algo.advantage.reward_scale')
        self.eta = g('algo.adapt_consts.kl_cutoff_coeff')
        self.beta = g('algo.adapt_consts.beta_init')
        self.beta_range = g('algo.adapt_consts.beta_range')
        self.beta_scale = g('algo.adapt_consts.scale_constant')
        self.clip_epsilon = g('algo.clip_consts.clip_epsilon_init')
        self.clip_range = g('algo.clip_consts.clip_range')
        self.clip_scale = g('algo.clip_consts.scale_constant')
        self.clip_actor_gradient = g('algo.network.clip_actor_gradient')
        self.actor_clip = g('algo.network.actor_gradient_norm_clip')
        self.clip_critic_gradient = g('algo.network.clip_critic_gradient')
        self.critic_clip = g('algo.network.critic_gradient_norm_clip')
        self.exp_interval = g('parameter_publish.exp_interval')
        mk = lambda: PPOModelRef(  # noqa: E731
            obs_dim, act_dim, g('model.actor_fc_hidden_sizes'), g('model.critic_fc_hidden_sizes'),
            g('algo.consts.init_log_sig'), self.use_z_filter, self.rnn,
            g('algo.rnn.rnn_hidden'), g('algo.rnn.rnn_layer'), pixel, g('model.cnn_feature_dim', 256))
        self.dtype = dtype
        self.model = mk().to(dtype)
        self.ref_target_model = mk().to(dtype)
        self.ref_target_model.update_target_params(self.model)
        self.critic_optim = torch.optim.Adam(self.model.critic_params(), lr=g('algo.network.lr_critic'),
                                             weight_decay=g('algo.network.critic_regularization'))
        self.actor_optim = torch.optim.Adam(self.model.actor_params(), lr=g('algo.network.lr_actor'),
                                            weight_decay=g('algo.network.actor_regularization'))
        self.pd = DiagGaussRef(act_dim)
        self.cells = None
        self.kl_record = []
        self.exp_counter = 0
        if self.use_r_filter:
            self.reward_filter = RewardFilterRef().to(dtype)

    # -- losses -------------------------------------------------------------
    def _clip_loss(self, obs, actions, adv, behave_pol):     # ppo.py:194-225
        learn_pol = self.model.forward_actor(obs, self.cells)
        learn_prob = self.pd.likelihood(actions, learn_pol)
        behave_prob = self.pd.likelihood(actions, behave_pol)
        ratio = learn_prob / behave_prob
        clipped = torch.clamp(ratio, 1 - self.clip_epsilon, 1 + self.clip_epsilon)
        surr = -ratio * adv.view(-1, 1)
        csurr = -clipped * adv.view(-1, 1)
        loss = torch.cat([surr, csurr], 1).max(1)[0].mean()
        stats = {'_surr_loss': surr.mean().item(), '_clip_surr_loss': loss.item(),
                 '_entropy': self.pd.entropy(learn_pol).mean().item(),
                 '_clip_epsilon': self.clip_epsilon}
        return loss, stats

    def _adapt_loss(self, obs, actions, adv, behave_pol, ref_pol):   # ppo.py:250-285
        learn_pol = self.model.forward_actor(obs, self.cells)
        pb = self.pd.likelihood(actions, behave_pol)
        pl = self.pd.likelihood(actions, learn_pol)
        kl = self.pd.kl(ref_pol, learn_pol).mean()
        surr = -(adv.view(-1, 1) * (pl / torch.clamp(pb, min=1e-2))).mean()
        loss = surr + self.beta * kl
        entropy = self.pd.entropy(learn_pol).mean()
        if kl.item() - 2.0 * self.kl_target > 0:
            loss += self.eta * (kl - 2.0 * self.kl_target).pow(2)
        stats = {'_kl_loss_adapt': loss.item(), '_surr_loss': surr.item(), '_pol_kl': kl.item(),
                 '_entropy': entropy.item(), '_beta': self.beta}
        return loss, stats

    def _policy_update(self, obs, actions, adv, behave_pol, ref_pol):   # :227-248, :287-309
        if self.ppo_mode == 'clip':
            loss, stats = self._clip_loss(obs, actions, adv, behave_pol)
        else:
            loss, stats = self._adapt_loss(obs, actions, adv, behave_pol, ref_pol)
        for p in self.model.actor_params():
            p.grad = None
        loss.backward()
        if self.clip_actor_gradient:
            stats['grad_norm_actor'] = float(nn.utils.clip_grad_norm_(self.model.actor_params(),
                                                                      self.actor_clip))
        self.actor_optim.step()
        return stats

    def _value_update(self, obs, returns):                   # ppo.py:311-353
        values = self.model.forward_critic(obs, self.cells)
        if values.dim() == 3:
            values = values.squeeze(2)
        ev = 1 - torch.var(returns - values) / torch.var(returns)
        loss = (values - returns).pow(2).mean()
        stats = {'_val_loss': loss.item(), '_val_explained_var': ev.item()}
        for p in self.model.critic_params():
            p.grad = None
        loss.backward()
        if self.clip_critic_gradient:
            stats['grad_norm_critic'] = float(nn.utils.clip_grad_norm_(self.model.critic_params(),
                                                                       self.critic_clip))
        self.critic_optim.step()
        return stats

    # -- GAE through the critic (ppo.py:355-418) ------------------------------
    def gae_and_return(self, obs, obs_next, rewards, dones):
        x = _tmap2(lambda a, b: torch.cat([a, b], dim=1), obs, obs_next)
        B = rewards.shape[0]
        if not self.rnn:
            x = _tmap(lambda o: o.reshape(-1, *o.shape[2:]), x)
        values = self.model.forward_critic(x, self.cells).detach()
        values = values.view(B, self.n_step + 1)
        raw = []
        out = gae_and_return(values, rewards, dones, self.gamma, self.lam, self.n_step,
                             self.horizon, self.rnn, self.norm_adv, raw_out=raw)
        self.last_adv_raw = raw[0]
        return out

    def _as_input(self, a):
        """The reference's FloatTensor conversion of a batch array (ppo.py:420-484):
        rounded to fp32, then held in the oracle's dtype.  A torch float64 tensor
        handed to an fp64 oracle is taken as exact (the parity tests' perturbed
        executions)."""
        if isinstance(a, torch.Tensor) and a.dtype == torch.float64 and self.dtype == torch.float64:
            return a
        return torch.as_tensor(a, dtype=torch.float32).to(self.dtype)

    # -- preprocess (ppo.py:420-484, rewards part) ----------------------------
    def preprocess_rewards(self, rewards):
        rewards = self._as_input(rewards) * self.reward_scale
        if self.use_r_filter:
            normed = self.reward_filter.forward(rewards)
            self.reward_filter.update(rewards)
            rewards = normed
        return rewards

    # -- _optimize (ppo.py:487-586) ------------------------------------------
    def optimize(self, obs, actions, rewards, obs_next, pds, onetime, dones):
        if self.rnn:
            self.cells = (onetime[0].transpose(0, 1).contiguous(),
                          onetime[1].transpose(0, 1).contiguous())
        with torch.no_grad():
            adv, ret = self.gae_and_return(obs, obs_next, rewards, dones)
        self.last_adv, self.last_ret = adv.clone(), ret.clone()
        if self.rnn:
            E = self.n_step - self.horizon + 1
            behave_pol = pds[:, :E, :].contiguous()
            actions_iter = actions[:, :E, :].contiguous()
            obs_iter = _tmap(lambda o: o[:, :E].contiguous(), obs)
        else:
            behave_pol = pds[:, 0, :].contiguous()
            actions_iter = actions[:, 0, :].contiguous()
            obs_iter = _tmap(lambda o: o[:, 0].contiguous(), obs)
        with torch.no_grad():
            ref_pol = self.ref_target_model.forward_actor(obs_iter, self.cells)
        epochs_run = 0
        stats = {}
        curr_pol = None
        for _ in range(self.epoch_policy):                    # :541-557
            stats = self._policy_update(obs_iter, actions_iter, adv, behave_pol, ref_pol)
            epochs_run += 1
            with torch.no_grad():
                curr_pol = self.model.forward_actor(obs_iter, self.cells)
                kl = self.pd.kl(ref_pol, curr_pol).mean()
            stats['_pol_kl'] = kl.item()
            if kl.item() > self.kl_target * 4:
                break
        if '_pol_kl' in stats:
            self.kl_record.append(stats['_pol_kl'])               # :559
        bstats = {}
        for _ in range(self.epoch_baseline):                  # :561-562
            bstats = self._value_update(obs_iter, ret)
        stats.update(bstats)
        with torch.no_grad():
            if curr_pol is None:
                curr_pol = self.model.forward_actor(obs_iter, self.cells)
            bl = self.pd.likelihood(actions_iter, behave_pol)
            cl = self.pd.likelihood(actions_iter, curr_pol)
            stats['_avg_return_targ'] = ret.mean().item()
            stats['_avg_log_sig'] = self.model.actor.log_var.mean().item()
            stats['_avg_behave_likelihood'] = bl.mean().item()
            stats['_avg_is_weight'] = (cl / (bl + 1e-4)).mean().item()
            stats['_ref_behave_diff'] = self.pd.kl(ref_pol, behave_pol).mean().item()
            stats['epochs_run'] = epochs_run
            if self.use_z_filter:                             # :578-582
                self.model.z_filter.z_update(obs_iter[0] if isinstance(obs_iter, tuple)
                                             else obs_iter)
        return stats

    def learn(self, batch):                                   # ppo.py:588-613
        f32 = lambda a: None if a is None else self._as_input(a)  # noqa: E731
        obs = f32(batch['obs'])
        obs_next = f32(batch['obs_next'])
        if 'pixels' in batch:                 # (low_dim or None, camera0 uint8)
            obs = (obs, torch.as_tensor(batch['pixels']))
            obs_next = (obs_next, torch.as_tensor(batch['pixels_next']))
        actions = f32(batch['actions'])
        rewards = self.preprocess_rewards(batch['rewards'])
        dones = f32(batch['dones'])
        pds = f32(batch['pds'])
        onetime = None
        if batch.get('onetime') is not None:
            onetime = [f32(x) for x in batch['onetime']]
        stats = self.optimize(obs, actions, rewards, obs_next, pds, onetime, dones)
        self.exp_counter += self.batch_size
        return stats

    def post_publish(self):                                   # ppo.py:637-666
        final_kl = np.mean(self.kl_record)
        if self.ppo_mode == 'clip':
            if final_kl > self.kl_target * self.adjust_threshold[1]:
                if self.clip_range[0] < self.clip_epsilon:
                    self.clip_epsilon = self.clip_epsilon / self.clip_scale
            elif final_kl < self.kl_target * self.adjust_threshold[0]:
                if self.clip_range[1] > self.clip_epsilon:
                    self.clip_epsilon = self.clip_epsilon * self.clip_scale
        else:
            if final_kl > self.kl_target * self.adjust_threshold[1]:
                if self.beta_range[1] > self.beta:
                    self.beta = self.beta * self.beta_scale
            elif final_kl < self.kl_target * self.adjust_threshold[0]:
                if self.beta_range[0] < self.beta:
                    self.beta = self.beta / self.beta_scale
        self.ref_target_model.update_target_params(self.model)
        self.kl_record = []
        self.exp_counter = 0

    def maybe_publish(self):                                  # ppo.py:623-635
        if self.exp_counter >= self.exp_interval:
            self.post_publish()
            return True
        return False
