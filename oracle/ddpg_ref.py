"""ORACLE (test infrastructure only — see oracle/__init__.py).

fp32 CPU restatement of the DDPG learner step (low-dim observations; the
use_layernorm blocks of builders.py:41-48,65-75 — off by default,
ddpg_configs.py:21 — with torchx's L.LayerNorm(1) taken as nn.LayerNorm(n)):
  ActorNetworkX / CriticNetworkX   surreal/model/model_builders/builders.py:35-84
  DDPGModel.forward                surreal/model/ddpg_net.py:86-93; with pixel=(C, H, W) the
                                   perception CNNStemNetwork (builders.py:8-33, ddpg_net.py:
                                   40-43,69-79) on camera0 / 255, concatenated [cnn | low_dim],
                                   trained by the critic optimizer (ddpg_net.py:57-61), read
                                   detached by the actor (ddpg.py:325-328)
  DDPGLearner._optimize            surreal/learner/ddpg.py:244-352 (incl. the TD3 options:
                                   twin critic ddpg.py:280-283,312-320; target policy
                                   smoothing noise from numpy's global RNG :267-277)
  DDPGLearner._target_update       surreal/learner/ddpg.py:403-428
torchx's nnx.Module.clip_grad_value / soft_update / hard_update are not
available; they are stated here as torch.nn.utils.clip_grad_value_,
target <- tau*src + (1-tau)*target and a parameter copy.
"""
import numpy as np
import torch
import torch.nn as nn


class ActorX(nn.Module):
    """Linear-ReLU[-LN]-Linear-ReLU[-LN]-Linear-Tanh (builders.py:35-56)."""

    def __init__(self, d_in, d_act, hidden, ln=False):
        super().__init__()
        self.l1 = nn.Linear(d_in, hidden[0])
        self.l2 = nn.Linear(hidden[0], hidden[1])
        self.l3 = nn.Linear(hidden[1], d_act)
        self.ln = ln
        if ln:
            self.n1, self.n2 = nn.LayerNorm(hidden[0]), nn.LayerNorm(hidden[1])

    def forward(self, x):
        h = torch.relu(self.l1(x))
        if self.ln:
            h = self.n1(h)
        h = torch.relu(self.l2(h))
        if self.ln:
            h = self.n2(h)
        return torch.tanh(self.l3(h))

    def params(self):
        out = [self.l1.weight, self.l1.bias]
        out += [self.n1.weight, self.n1.bias] if self.ln else []
        out += [self.l2.weight, self.l2.bias]
        out += [self.n2.weight, self.n2.bias] if self.ln else []
        return out + [self.l3.weight, self.l3.bias]


class CriticX(nn.Module):
    """obs -> Linear-ReLU[-LN] ; cat(h, a) -> Linear-ReLU[-LN]-Linear (builders.py:58-84)."""

    def __init__(self, d_in, d_act, hidden, ln=False):
        super().__init__()
        self.lo = nn.Linear(d_in, hidden[0])
        self.lc = nn.Linear(hidden[0] + d_act, hidden[1])
        self.lq = nn.Linear(hidden[1], 1)
        self.ln = ln
        if ln:
            self.no, self.nc = nn.LayerNorm(hidden[0]), nn.LayerNorm(hidden[1])

    def forward(self, obs, act):
        h = torch.relu(self.lo(obs))
        if self.ln:
            h = self.no(h)
        h = torch.relu(self.lc(torch.cat((h, act), 1)))
        if self.ln:
            h = self.nc(h)
        return self.lq(h)

    def params(self):
        out = [self.lo.weight, self.lo.bias]
        out += [self.no.weight, self.no.bias] if self.ln else []
        out += [self.lc.weight, self.lc.bias]
        out += [self.nc.weight, self.nc.bias] if self.ln else []
        return out + [self.lq.weight, self.lq.bias]


def flat_of(params):
    return torch.cat([p.detach().reshape(-1) for p in params])


def load_flat(params, f):
    o = 0
    with torch.no_grad():
        for p in params:
            n = p.numel()
            p.copy_(torch.as_tensor(f[o:o + n]).reshape(p.shape))
            o += n


class DDPGLearnerRef:
    """dtype=torch.float64 runs the same step in double precision (the
    parity tests' "truth"); noise_perm (a row permutation or None) reorders
    the TD3 smoothing noise rows as the batch rows were reordered, so a
    row-permuted execution draws the same noise per transition."""

    def __init__(self, lc, obs_dim, act_dim, seed=0, dtype=torch.float32, pixel=None):
        torch.manual_seed(seed)
        self.dtype = dtype
        self.noise_perm = None
        self.pixel = pixel
        self.low_dim = obs_dim
        if pixel is not None:
            from oracle.ppo_ref import cnn_stem_ref
            F = int(lc['model'].get('conv_spec', {}).get('hidden_output_dim', 200))
            self.cnn_dim = F
            obs_dim = F + obs_dim                       # [cnn | low_dim]
            mkp = lambda: cnn_stem_ref(*pixel, F)  # noqa: E731
        net = lc['algo']['network']
        self.gamma = lc['algo']['gamma']
        self.n_step = lc['algo']['n_step']
        self.batch_size = lc['replay']['batch_size']
        ah, ch = lc['model']['actor_fc_hidden_sizes'], lc['model']['critic_fc_hidden_sizes']
        ln = bool(lc['model'].get('use_layernorm', False))
        self.actor, self.critic = ActorX(obs_dim, act_dim, ah, ln), CriticX(obs_dim, act_dim, ch, ln)
        self.actor_t, self.critic_t = ActorX(obs_dim, act_dim, ah, ln), CriticX(obs_dim, act_dim, ch, ln)
        self.double = bool(net.get('use_double_critic', False))
        self.action_reg = bool(net.get('use_action_regularization', False))
        self.act_dim = act_dim
        if self.double:
            self.critic2, self.critic2_t = CriticX(obs_dim, act_dim, ch, ln), CriticX(obs_dim, act_dim, ch, ln)
        if pixel is not None:
            self.perc, self.perc_t = mkp(), mkp()
            if self.double:
                self.perc2, self.perc2_t = mkp(), mkp()
        for m in self.nets():
            m.to(dtype)
        self.hard_update(perception=False)    # ddpg.py:174-178: actor and critic(s) only
        self.clip_actor = net['clip_actor_gradient']
        self.actor_clip_value = net['actor_gradient_value_clip']
        self.clip_critic = net['clip_critic_gradient']
        self.critic_clip_value = net['critic_gradient_value_clip']
        cp = list(self.critic.parameters()) + (list(self.perc.parameters()) if pixel is not None else [])
        self.critic_optim = torch.optim.Adam(cp, lr=net['lr_critic'],
                                             weight_decay=net['critic_regularization'])
        self.actor_optim = torch.optim.Adam(self.actor.parameters(), lr=net['lr_actor'],
                                            weight_decay=net['actor_regularization'])
        if self.double:
            cp2 = list(self.critic2.parameters()) + (list(self.perc2.parameters()) if pixel is not None else [])
            self.critic_optim2 = torch.optim.Adam(cp2, lr=net['lr_critic'],
                                                  weight_decay=net['critic_regularization'])
        tu = net['target_update']
        self.target_update_type = tu['type']
        self.tau = tu.get('tau', 1e-3)
        self.interval = tu.get('interval', 500)
        self.counter = 0

    def nets(self):
        out = [self.actor, self.critic, self.actor_t, self.critic_t]
        out += [self.critic2, self.critic2_t] if self.double else []
        if self.pixel is not None:
            out += [self.perc, self.perc_t] + ([self.perc2, self.perc2_t] if self.double else [])
        return out

    def target_pairs(self, perception=True):
        pairs = [(self.actor_t, self.actor), (self.critic_t, self.critic)]
        if self.double:
            pairs.append((self.critic2_t, self.critic2))
        if self.pixel is not None and perception:
            pairs.append((self.perc_t, self.perc))
            if self.double:
                pairs.append((self.perc2_t, self.perc2))
        return pairs

    def hard_update(self, perception=True):
        """ddpg.py:420-428 (the interval update: every target, perception
        included); perception=False is the constructor's sync (ddpg.py:174-178)"""
        for t, s in self.target_pairs(perception):
            t.load_state_dict(s.state_dict())

    def perception(self, net, obs):                                     # ddpg_net.py:69-79
        if self.pixel is None:
            return obs
        low, pix = obs
        img = torch.as_tensor(pix)
        img = img.to(self.dtype) / 255.0 if self.dtype != torch.float32 else img.float() / 255.0
        parts = [net(img)] + ([low] if low is not None and low.shape[-1] else [])
        return torch.cat(parts, 1)

    def optimize(self, obs, actions, rewards, obs_next, done):          # ddpg.py:244-352
        """obs / obs_next: (B, D) tensors, or with pixel=(C, H, W) pairs
        (low_dim (B, D) or None, camera0 uint8 (B, C, H, W))"""
        cv = lambda t: t if (isinstance(t, torch.Tensor) and t.dtype == self.dtype) \
            else torch.as_tensor(t, dtype=torch.float32).to(self.dtype)  # noqa: E731
        if self.pixel is not None:
            obs = (None if obs[0] is None else cv(obs[0]), obs[1])
            obs_next = (None if obs_next[0] is None else cv(obs_next[0]), obs_next[1])
        else:
            obs, obs_next = cv(obs), cv(obs_next)
        actions, rewards, done = (cv(t) for t in (actions, rewards, done))
        assert actions.max().item() <= 1.0 and actions.min().item() >= -1.0
        with torch.no_grad():
            pt = self.perception(self.perc_t, obs_next) if self.pixel is not None else obs_next
            pt2 = self.perception(self.perc2_t, obs_next) if self.pixel is not None and self.double \
                else pt
            a_t = self.actor_t(pt)
            q_t = self.critic_t(pt, a_t)
            if self.action_reg:
                noise = np.clip(np.random.normal(0, 0.2, size=(self.batch_size, self.act_dim)),
                                -0.5, 0.5)
                if self.noise_perm is not None:
                    noise = noise[self.noise_perm]
                a_t = (a_t + torch.tensor(noise, dtype=torch.float32).to(self.dtype)).clamp(-1, 1)
            y = rewards + pow(self.gamma, self.n_step) * q_t * (1.0 - done)
            if self.double:
                q_t2 = self.critic2_t(pt2, a_t)
                y2 = rewards + pow(self.gamma, self.n_step) * q_t2 * (1.0 - done)
                y = torch.min(y, y2)
        p_obs = self.perception(self.perc, obs) if self.pixel is not None else obs
        q = self.critic(p_obs, actions)
        self.critic.zero_grad()
        if self.pixel is not None:
            self.perc.zero_grad()
        critic_loss = nn.MSELoss()(q, y)
        critic_loss.backward()
        if self.clip_critic:
            nn.utils.clip_grad_value_(self.critic.parameters(), self.critic_clip_value)
        self.critic_optim.step()
        q2 = None
        if self.double:
            p2 = self.perception(self.perc2, obs) if self.pixel is not None else obs
            q2 = self.critic2(p2, actions)
            self.critic2.zero_grad()
            if self.pixel is not None:
                self.perc2.zero_grad()
            critic_loss = nn.MSELoss()(q2, y)
            critic_loss.backward()
            if self.clip_critic:
                nn.utils.clip_grad_value_(self.critic2.parameters(), self.critic_clip_value)
            self.critic_optim2.step()
        self.actor.zero_grad()
        pd_ = p_obs.detach()                                  # perception.detach(), ddpg.py:325-328
        actor_loss = -self.critic(pd_, self.actor(pd_)).mean()
        actor_loss.backward()
        if self.clip_actor:
            nn.utils.clip_grad_value_(self.actor.parameters(), self.actor_clip_value)
        self.actor_optim.step()
        stats = {'actor_loss': actor_loss.item(), 'critic_loss': critic_loss.item(),
                 'action_norm': actions.norm(2, 1).mean().item(), 'rewards': rewards.mean().item(),
                 'Q_target': y.mean().item(), 'Q_policy': q.mean().item()}
        if q2 is not None:
            stats['Q_policy2'] = q2.mean().item()
        self.target_update()
        return stats

    def target_update(self):                                            # ddpg.py:403-428
        if self.target_update_type == 'soft':
            with torch.no_grad():
                for tm, sm in self.target_pairs():
                    for t, s in zip(tm.parameters(), sm.parameters()):
                        t.copy_(self.tau * s + (1 - self.tau) * t)
        else:
            self.counter += 1
            if self.counter % self.interval == 0:
                self.hard_update()
