"""ORACLE (test infrastructure only — see oracle/__init__.py).

One-agent-at-a-time restatement of the reference actors' act():
  PPOAgent.act     surreal/agent/ppo_agent.py:103-151 (cells exposed before the
                   step as onetime infos, forward_actor_expose_cells, log-sigma
                   noise, DiagGauss.sample / maxprob, clip to [-1, 1])
  PPOAgent.reset   ppo_agent.py:166-180
  DDPGAgent.act    surreal/agent/ddpg_agent.py:153-182 (actor forward, clip,
                   exploration noise, clip)
  NormalActionNoise / OrnsteinUhlenbeckActionNoise   surreal/agent/action_noise.py:9-40
  NormalParameterNoise / AdaptiveNormalParameterNoise surreal/agent/param_noise.py:9-72,
                   applied on parameter fetch and (adaptive) measured in act()
                   (ddpg_agent.py:134-151, 172-173)
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


class NormalParameterNoiseRef(object):
    """param_noise.py:9-24: every array of the fetched params + N(0, sigma)"""

    def __init__(self, sigma):
        self.sigma = sigma

    def apply(self, params):
        for key in params:
            for k in params[key]:
                p = params[key][k]
                params[key][k] = p + np.random.normal(0, self.sigma, size=tuple(p.shape))
        return params


class AdaptiveNormalParameterNoiseRef(object):
    """param_noise.py:29-72.  original_actor(obs) is the unperturbed actor
    (the reference's original_model forward with calculate_value=False)"""

    def __init__(self, original_actor, load_original, target_stddev, compute_dist_interval=10,
                 alpha=1.04, sigma=0.01):
        self.sigma, self.target_stddev = sigma, target_stddev
        self.compute_dist_interval, self.alpha = compute_dist_interval, alpha
        self.original_actor, self.load_original = original_actor, load_original
        self.i = 0
        self.total_action_distance = 0.0

    def compute_action_distance(self, obs, modified_model_action):
        if self.i % self.compute_dist_interval == 0:
            with torch.no_grad():
                a0 = self.original_actor(obs)
            # assigned, not accumulated (param_noise.py:44)
            self.total_action_distance = float((((a0 - modified_model_action) ** 2).sum()) ** 0.5)
        self.i += 1

    def apply(self, params):
        if self.i > 0:
            mean_action_dist = self.total_action_distance / self.i
            if mean_action_dist > self.target_stddev:
                self.sigma /= self.alpha
            else:
                self.sigma *= self.alpha
        self.i = 0
        self.load_original({k: {kk: np.array(vv) for kk, vv in v.items()} for k, v in params.items()})
        for key in params:
            for k in params[key]:
                p = params[key][k]
                params[key][k] = p + np.random.normal(0, self.sigma, size=tuple(p.shape))
        return params


class DDPGAgentRef(object):
    def __init__(self, actor, noise=None, agent_mode='training', param_noise=None):
        self.actor, self.noise, self.agent_mode = actor, noise, agent_mode
        self.param_noise = param_noise

    def act(self, obs):
        x = torch.as_tensor(obs, dtype=torch.float32).unsqueeze(0)
        with torch.no_grad():
            a = self.actor(x)
        if isinstance(self.param_noise, AdaptiveNormalParameterNoiseRef):
            self.param_noise.compute_action_distance(x, a)
        a = a.numpy()[0].clip(-1, 1)
        if self.agent_mode != 'eval_deterministic':
            a += self.noise()
        return a.clip(-1, 1)
