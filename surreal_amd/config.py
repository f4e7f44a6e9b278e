"""Config objects and the default learner configs of the PPO / DDPG hot path.

Mirrors the reference's config surface that the learners read:
``Config`` is a nested dict with attribute access and ``extend`` (defaults
fill-in), as surreal/session/config.py:154-255; the default trees follow
surreal/main/ppo_configs.py:15-94 and surreal/main/ddpg_configs.py:16-100, plus
the learner-side keys of surreal/session/default_configs.py.  Only keys read by
the learner / replay hot path are kept.
"""
import copy


class Config(dict):
    """Nested dict with attribute access (surreal/session/config.py:154)."""

    def __init__(self, *args, **kwargs):
        super().__init__()
        data = dict(*args, **kwargs)
        for k, v in data.items():
            self[k] = v

    @staticmethod
    def _wrap(v):
        if isinstance(v, Config):
            return v
        if isinstance(v, dict):
            return Config(v)
        return v

    def __setitem__(self, k, v):
        super().__setitem__(k, self._wrap(v))

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v

    def __deepcopy__(self, memo):
        return Config(copy.deepcopy(dict(self), memo))

    def extend(self, defaults):
        """Fill keys missing here from ``defaults`` (recursively), in place."""
        for k, v in defaults.items():
            if k not in self:
                self[k] = copy.deepcopy(v)
            elif isinstance(self[k], Config) and isinstance(v, dict):
                self[k].extend(v)
        return self

    def to_dict(self):
        return {k: (v.to_dict() if isinstance(v, Config) else v) for k, v in self.items()}


class ConfigError(Exception):
    """Raised for unsupported configurations (surreal/session/config.py:7)."""


# surreal/session/default_configs.py learner keys the hot path reads
BASE_LEARNER_CONFIG = Config({
    'model': {},
    'algo': {'gamma': 0.99, 'n_step': 1},
    'replay': {'batch_size': 64, 'memory_size': 1000, 'sampling_start_size': 100,
               'replay_shards': 1},
    'parameter_publish': {'min_publish_interval': 0.3, 'exp_interval': 4096},
})

# surreal/main/ppo_configs.py:15-94
PPO_DEFAULT_LEARNER_CONFIG = Config({
    'model': {
        'convs': [],
        'actor_fc_hidden_sizes': [300, 200],
        'critic_fc_hidden_sizes': [300, 200],
        'cnn_feature_dim': 256,
        'use_layernorm': False,
    },
    'algo': {
        'use_z_filter': False,
        'use_r_filter': False,
        'gamma': .99,
        'n_step': 25,
        'stride': 20,
        'network': {
            'lr_actor': 1e-4,
            'lr_critic': 1e-4,
            'clip_actor_gradient': True,
            'actor_gradient_norm_clip': 10.,
            'clip_critic_gradient': True,
            'critic_gradient_norm_clip': 10.,
            'actor_regularization': 0.0,
            'critic_regularization': 0.0,
            'anneal': {
                'lr_scheduler': "LinearWithMinLR",
                'frames_to_anneal': 5e6,
                'lr_update_frequency': 100,
                'min_lr': 1e-4,
            },
        },
        'ppo_mode': 'adapt',
        'advantage': {'norm_adv': True, 'lam': 1.0, 'reward_scale': 1.0},
        'rnn': {'if_rnn_policy': True, 'rnn_hidden': 100, 'rnn_layer': 1, 'horizon': 5},
        'consts': {
            'init_log_sig': -1.0,
            'log_sig_range': 0,
            'epoch_policy': 10,
            'epoch_baseline': 10,
            'adjust_threshold': (0.5, 2.0),
            'kl_target': 0.02,
        },
        'adapt_consts': {
            'kl_cutoff_coeff': 500,
            'beta_init': 1.0,
            'beta_range': (1 / 35.0, 35.0),
            'scale_constant': 1.5,
        },
        'clip_consts': {
            'clip_epsilon_init': 0.2,
            'clip_range': (0.05, 0.3),
            'scale_constant': 1.2,
        },
    },
    'replay': {'batch_size': 64, 'memory_size': 96, 'sampling_start_size': 64,
               'replay_shards': 1},
    'parameter_publish': {'exp_interval': 4096},
})
PPO_DEFAULT_LEARNER_CONFIG.extend(BASE_LEARNER_CONFIG)

# surreal/main/ddpg_configs.py:16-100
DDPG_DEFAULT_LEARNER_CONFIG = Config({
    'model': {
        'convs': [],
        'actor_fc_hidden_sizes': [300, 200],
        'critic_fc_hidden_sizes': [400, 300],
        'use_layernorm': False,
        'conv_spec': {'out_channels': [16, 32], 'kernel_sizes': [8, 4], 'strides': [4, 2],
                      'hidden_output_dim': 200},
    },
    'algo': {
        'gamma': .99,
        'n_step': 3,
        'stride': 1,
        'network': {
            'lr_actor': 1e-4,
            'lr_critic': 1e-3,
            'clip_actor_gradient': True,
            'actor_gradient_value_clip': 1.,
            'clip_critic_gradient': False,
            'critic_gradient_value_clip': 5.,
            'actor_regularization': 0.0,
            'critic_regularization': 0.0,
            'use_action_regularization': False,
            'use_double_critic': False,
            'target_update': {'type': 'hard', 'interval': 500},
        },
        # agent-side exploration (ddpg_configs.py:63-86)
        'exploration': {
            'param_noise_type': None,          # None | 'normal' | 'adaptive_normal'
            'param_noise_sigma': 0.05,
            'param_noise_alpha': 1.15,
            'param_noise_target_stddev': 0.005,
            'noise_type': 'normal',
            'max_sigma': 1.0,
            'theta': 0.15,
            'dt': 1e-3,
        },
    },
    'replay': {'batch_size': 512, 'memory_size': int(1000000 / 3),
               'sampling_start_size': 3000, 'replay_shards': 3},
    'parameter_publish': {'min_publish_interval': 3},
})
DDPG_DEFAULT_LEARNER_CONFIG.extend(BASE_LEARNER_CONFIG)

# learner-side session keys (surreal/session/default_configs.py)
BASE_SESSION_CONFIG = Config({
    'folder': '/tmp/surreal_amd',
    'learner': {'num_gpus': 1},
    'checkpoint': {'restore': False, 'learner': {'periodic': 1000}},
})


def pixel_env_config(obs_dim, act_dim, camera=(3, 84, 84)):
    """env_config of a robosuite-style pixel env: obs_spec
    {'low_dim': {'flat_inputs': (D,)}, 'pixel': {'camera0': (C, H, W)}} with
    uint8 camera observations; obs_dim 0 drops the low-dim modality."""
    spec = {'pixel': {'camera0': tuple(camera)}}
    if obs_dim:
        spec['low_dim'] = {'flat_inputs': (obs_dim,)}
    return Config({
        'pixel_input': True,
        'frame_stacks': 1,
        'frame_stack_concatenate_on_env': True,
        'obs_spec': spec,
        'action_spec': {'dim': (act_dim,), 'type': 'continuous'},
    })


def gym_env_config(obs_dim, act_dim, pixel_input=False):
    """env_config with obs_spec/action_spec as make_env_config fills them
    (surreal/env/make_env.py:16-38) for a flat low-dim gym env."""
    return Config({
        'pixel_input': pixel_input,
        'frame_stacks': 1,
        'frame_stack_concatenate_on_env': True,
        'obs_spec': {'low_dim': {'flat_inputs': (obs_dim,)}},
        'action_spec': {'dim': (act_dim,), 'type': 'continuous'},
    })
