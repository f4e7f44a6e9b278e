"""ORACLE (test infrastructure only — see oracle/__init__.py).

One-agent-at-a-time restatement of the reference actors' act():
  PPOAgent.act     surreal/agent/ppo_agent.py:103-151 (cells exposed before the
                   step as onetime infos, forward_actor_expose_cells, log-sigma
                   noise, DiagGauss.sample / maxprob, clip to [-1, 1])
  PPOAgent.reset   ppo_agent.py:166-180
  DDPGAgent.act    surreal/agent/ddpg_agent.py:153-182 (actor forward, clip,
                   exploration noise, clip)
  NormalActionNoise / OrnsteinUhlenbeckActionNoise   surreal/agent/action_noise.py:9-40
Random draws come from numpy's global RNG in the reference's order.
"""
import numpy as np
import torch


class PPOAgentRef(object):
    def __init__(self, model, action_dim, rnn_hidden=None, rnn_layer=1, agent_mode='training',
                 log_sig_range=0.0):
        self.model = model
        self.action_dim = action_dim
        self.agent_mode = agent_mode
        self.rnn_hidden, self.rnn_layer = rnn_hidden, rnn_layer
        self.noise = 0 if agent_mode != 'training' else np.random.uniform(low=-log_sig_range,
                                                                          high=log_sig_range)
        self.reset()

    def reset(self):
        self.cells = None
        if self.rnn_hidden:
            dt = self.model.actor.log_var.dtype
            self.cells = (torch.zeros(self.rnn_layer, 1, self.rnn_hidden, dtype=dt),
                          torch.zeros(self.rnn_layer, 1, self.rnn_hidden, dtype=dt))

    def act(self, obs):
        """obs: (D,) low-dim observation (or a (low, pixel) pair of single frames)."""
        info = [[], []]
        if self.rnn_hidden:
            info[0].append(self.cells[0].squeeze(1).numpy())
            info[0].append(self.cells[1].squeeze(1).numpy())
        with torch.no_grad():
            if isinstance(obs, tuple):
                x = (torch.as_tensor(obs[0], dtype=torch.float32).unsqueeze(0),
                     torch.as_tensor(obs[1]).unsqueeze(0))
            else:
                x = torch.as_tensor(obs, dtype=torch.float32).unsqueeze(0)
            pd, self.cells = self.model.forward_actor_expose_cells(x, self.cells)
        pd = pd.detach().numpy()
        pd[:, self.action_dim:] *= np.exp(self.noise)
        if self.agent_mode != 'eval_deterministic':
            a = np.random.randn(pd.shape[0], self.action_dim) * pd[:, self.action_dim:] + \
                pd[:, :self.action_dim]                                   # DiagGauss.sample
        else:
            a = pd[:, :self.action_dim]                                  # DiagGauss.maxprob
        np.clip(a, -1, 1, out=a)
        info[1].append(pd.reshape((-1,)))
        return a.reshape((-1,)), info


class NormalActionNoiseRef(object):
    def __init__(self, mu, sigma):
        self.mu, self.sigma = mu, sigma

    def __call__(self):
        return np.random.normal(self.mu, self.sigma)


class OUNoiseRef(object):
    def __init__(self, mu, sigma, theta, dt):
        self.mu, self.sigma, self.theta, self.dt = mu, sigma, theta, dt
        self.x_prev = np.zeros_like(mu)

    def __call__(self):
        x = self.x_prev + self.theta * (self.mu - self.x_prev) * self.dt + \
            self.sigma * np.sqrt(self.dt) * np.random.normal(size=self.mu.shape)
        self.x_prev = x
        return x


class DDPGAgentRef(object):
    def __init__(self, actor, noise=None, agent_mode='training'):
        self.actor, self.noise, self.agent_mode = actor, noise, agent_mode

    def act(self, obs):
        with torch.no_grad():
            a = self.actor(torch.as_tensor(obs, dtype=torch.float32).unsqueeze(0))
        a = a.numpy()[0].clip(-1, 1)
        if self.agent_mode != 'eval_deterministic':
            a += self.noise()
        return a.clip(-1, 1)
