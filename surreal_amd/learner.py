"""PPOLearner / DDPGLearner mirrors (surreal/learner/ppo.py, ddpg.py) whose
learn() runs as a short sequence of HIP launches on one stream:

  PPO learn()  (ppo.py:588-613)
    1. smi_reward_filter     reward_scale [+ RewardFilter]        ppo.py:452-456
    2. smi_ppo_critic_gae    critic fwd over B(T+1) rows + GAE     ppo.py:355-418
    3. smi_ppo_update_fused  ref_pol, <=epoch_policy actor updates
                             with KL early stop, epoch_baseline
                             critic updates, statistics            ppo.py:487-576
    4. smi_zfilter_update    z_update(obs_iter)                     ppo.py:578-582
No host synchronisation happens inside learn(): statistics, the KL record and
the Adam step counters stay on the device until something asks for them
(last_stats(), _post_publish()).  The data-dependent branches of the reference
(KL early stop ppo.py:556, adapt penalty ppo.py:275) are evaluated on device.

Construction needs no tensorplex/loggerplex/ZMQ: metrics go to an injectable
`metrics` callable and parameters to an injectable `publisher` callable.
"""
import ctypes
import math
import os
import time

import numpy as np
import torch

from . import _lib as L
from .aggregator import MultistepAggregatorWithInfo, SSARAggregator, StagingArena
from .config import Config, ConfigError
from .model import DiagGauss, PPOModel, RewardFilter
from .session import LearnerHooks


def _as_config(c):
    return c if isinstance(c, Config) else Config(c or {})


class LinearWithMinLR(object):
    """Learning-rate schedule named by the reference config
    (ppo_configs.py:43-46).  torchx's implementation is not available; this is
    the build's statement of it: every `update_freq` scheduler steps the rate
    decays linearly from the initial value towards `min_lr` over `num_updates`
    steps, never below `min_lr`.  With the default min_lr == lr it is constant."""

    def __init__(self, lr, num_updates, update_freq=1, min_lr=0.0):
        self.base_lr = float(lr)
        self.num_updates = max(1, int(num_updates))
        self.update_freq = max(1, int(update_freq))
        self.min_lr = float(min_lr)
        self.steps = 0

    def step(self):
        self.steps += 1

    def get_lr(self):
        k = (self.steps // self.update_freq) * self.update_freq
        frac = min(1.0, k / self.num_updates)
        return [max(self.min_lr, self.base_lr - (self.base_lr - self.min_lr) * frac)]

    def state_dict(self):
        return {'steps': self.steps}

    def load_state_dict(self, d):
        self.steps = int(d['steps'])


class TorchDistAllReduce(object):
    """Data-parallel group over torch.distributed (backend 'nccl' = RCCL over
    xGMI on MI355X; 'gloo' for CPU tests).  all_reduce is enqueued stream-
    ordered with the learner's kernels; no host synchronisation."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self._dist = dist
        self.group = group
        self.world_size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        # optional: a list receiving (start, end, bytes) event pairs of every
        # all-reduce, recorded on the caller's stream (bench.py instrumentation)
        self.timing = None
        # RCCL collectives are enqueued on the caller's stream and can be
        # captured into a hipGraph with the learner's kernels (a PPOLearner
        # with use_graph=True then replays the whole data-parallel learn(),
        # all-reduces included); gloo's run on the host and cannot
        self.capturable = dist.get_backend(group) == 'nccl'

    def allreduce_(self, t):
        if self.timing is not None and t.is_cuda:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM, group=self.group)
            e.record()
            self.timing.append((s, e, t.numel() * t.element_size()))
            return t
        self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM, group=self.group)
        return t

    def broadcast_(self, t, src=0):
        """Rank src's tensor on every rank (replica initialisation)."""
        self._dist.broadcast(t, src=self._dist.get_global_rank(self.group, src)
                             if self.group is not None else src, group=self.group)
        return t


def replicate_from_rank0(dp, tensors):
    """Broadcast initial parameters / filter state from rank 0 so the replicas
    start identical whatever seed each rank passed ("identical
    init is broadcast at start"), then check it: an all-reduced checksum of
    every tensor must equal world_size x the local one."""
    if dp is None or getattr(dp, 'world_size', 1) <= 1 or not hasattr(dp, 'broadcast_'):
        return
    for t in tensors:
        dp.broadcast_(t)
    sums = torch.stack([t.detach().double().sum() for t in tensors])
    tot = dp.allreduce_(sums.clone())
    if not torch.allclose(tot, sums * dp.world_size, rtol=1e-12, atol=1e-30):
        raise RuntimeError('data-parallel replicas differ after the initial broadcast')


_RNN_PHASE_NAMES = {0: 'rnn_gae', 1: 'rnn_prep', 2: 'rnn_policy_fwd', 3: 'rnn_policy_bwd',
                    4: 'rnn_policy_apply', 5: 'rnn_value_grad', 6: 'rnn_value_apply',
                    7: 'rnn_zstats', 8: 'rnn_zapply', 9: 'rnn_policy_decide'}


class _GraphInputs(object):
    """The static device inputs of a captured learn(): every batch leaf in ONE
    arena (256-byte aligned slots), refreshed before each replay by ONE
    copy-gather launch on the current stream (smi_copy_gather) instead of a
    copy launch per leaf (~5 us each inside the replayed sequence); leaves that
    already are the static tensors are skipped, unaligned ones copied by torch."""

    def __init__(self, leaves, device):
        offs, lens, off = [], [], 0
        for t in leaves:
            n = t.numel() * t.element_size()
            offs.append(off)
            lens.append(n)
            off += (n + 255) // 256 * 256
        self.arena = torch.empty(max(off, 256), dtype=torch.uint8, device=device)
        self.views = [self.arena[o:o + n].view(t.dtype).view(t.shape)
                      for o, n, t in zip(offs, lens, leaves)]
        self.offs, self.lens = offs, lens

    def refresh(self, leaves):
        idx = [i for i, (v, t) in enumerate(zip(self.views, leaves)) if v.data_ptr() != t.data_ptr()]
        if not idx:
            return
        ok = [i for i in idx if leaves[i].is_contiguous() and leaves[i].data_ptr() % 16 == 0
              and self.lens[i] % 4 == 0 and self.lens[i] > 0]
        for i in idx:
            if i not in ok:
                self.views[i].copy_(leaves[i])
        for k in range(0, len(ok), 16):            # one launch per 16 segments
            part = ok[k:k + 16]
            n = len(part)
            src = (ctypes.c_void_p * n)(*[leaves[i].data_ptr() for i in part])
            off = (ctypes.c_int64 * n)(*[self.offs[i] for i in part])
            ln = (ctypes.c_int64 * n)(*[self.lens[i] for i in part])
            L.call('smi_copy_gather', ctypes.c_void_p(self.arena.data_ptr()), src, off, ln, n,
                   ctypes.c_void_p(torch.cuda.current_stream(self.arena.device).cuda_stream))


class PPOLearner(LearnerHooks):
    """ppo.py:12-682 on MI355X.  Same constructor, learn/module_dict/
    publish_parameter/checkpoint_attributes/preprocess/_prefetcher_preprocess/
    periodic_checkpoint."""

    def __init__(self, learner_config, env_config, session_config=None, metrics=None,
                 publisher=None, device=None, seed=0, dp=None, checkpoint_full_state=False,
                 use_graph=False, checkpoint=None):
        """dp: None (one GPU) or a data-parallel group exposing `world_size` and
        `allreduce_(tensor)` (in-place SUM, stream-ordered), e.g.
        TorchDistAllReduce() over RCCL.  Each rank passes its own shard of
        `replay.batch_size` segments; the update equals the reference's on the
        concatenated global batch.
        checkpoint_full_state: checkpoint_attributes() also lists the Adam
        moments / step counters and the adaptive state (beta, clip epsilon, KL
        record, experience counter), so a restored learner continues
        bit-identically.  The reference checkpoints neither (ppo.py:668-678);
        off by default, which restores exactly what the reference restores.
        use_graph (one GPU): learn() replays a hipGraph of the whole device
        sequence (preprocess, GAE, the epochs, z_update) captured after the
        first call, with the batch copied into static buffers when it lives
        elsewhere; bit-identical to eager learn() (test_ppo_graph_replay_bit_exact).
        metrics: callable(stats, global_step) called after every learn() (one
        device read each), or a throttled sink with due() (session.
        TimeThrottledMetrics, tracker.py:81-104): statistics accumulate on the
        device and are read, averaged, only when it is due.
        checkpoint: what learn() hands periodic_checkpoint(global_steps=
        current_iteration) to (ppo.py:606-609): a PeriodicCheckpoint-like
        object (the reference's own, or session.PeriodicCheckpoint) or a
        callable(global_steps=, score=)."""
        L.require_gpu()
        self.dp = dp
        self.checkpoint_full_state = bool(checkpoint_full_state)
        self.learner_config = lc = _as_config(learner_config)
        self.env_config = ec = _as_config(env_config)
        self.session_config = _as_config(session_config)
        self._init_hooks(metrics, checkpoint)
        self.publisher = publisher
        self.device = torch.device(device) if device is not None else \
            torch.device('cuda', torch.cuda.current_device())
        L.ensure_workspace(self.device)
        self._ctx = L.Context(self.device)      # this learner's own workspace (re-entrancy)

        self.current_iteration = 0
        self.global_step = 0
        algo = lc.algo
        self.gamma = algo.gamma
        self.lam = algo.advantage.lam
        self.n_step = algo.n_step
        self.use_z_filter = algo.use_z_filter
        self.use_r_filter = algo.use_r_filter
        self.norm_adv = algo.advantage.norm_adv
        self.batch_size = lc.replay.batch_size
        self.action_dim = ec.action_spec['dim'][0]
        self.obs_spec = ec.obs_spec
        self.init_log_sig = algo.consts.init_log_sig
        self.ppo_mode = algo.ppo_mode
        self.if_rnn_policy = algo.rnn.if_rnn_policy
        self.horizon = algo.rnn.horizon
        self.lr_actor = algo.network.lr_actor
        self.lr_critic = algo.network.lr_critic
        self.epoch_policy = algo.consts.epoch_policy
        self.epoch_baseline = algo.consts.epoch_baseline
        self.kl_target = algo.consts.kl_target
        self.adjust_threshold = algo.consts.adjust_threshold
        self.reward_scale = algo.advantage.reward_scale
        self.kl_cutoff_coeff = algo.adapt_consts.kl_cutoff_coeff
        self.beta_init = algo.adapt_consts.beta_init
        self.beta_range = algo.adapt_consts.beta_range
        self.clip_range = algo.clip_consts.clip_range
        self.clip_epsilon_init = algo.clip_consts.clip_epsilon_init
        if self.ppo_mode == 'adapt':
            self.beta = self.beta_init
            self.eta = self.kl_cutoff_coeff
            self.beta_upper, self.beta_lower = self.beta_range[1], self.beta_range[0]
            self.beta_adjust_threshold = self.adjust_threshold
            self.clip_epsilon = self.clip_epsilon_init
        elif self.ppo_mode == 'clip':
            self.clip_epsilon = self.clip_epsilon_init
            self.clip_adjust_threshold = self.adjust_threshold
            self.clip_upper, self.clip_lower = self.clip_range[1], self.clip_range[0]
            self.beta = self.beta_init
        else:
            raise ConfigError('ppo_mode must be clip or adapt')
        self.rnn_layer = int(algo.rnn.get('rnn_layer', 1)) if self.if_rnn_policy else 1
        if not 1 <= self.rnn_layer <= 3:
            raise NotImplementedError('surreal_amd: the LSTM policy supports rnn_layer 1..3')
        self.if_pixel_input = bool(ec.get('pixel_input', False))

        anneal = algo.network.anneal
        num_updates = int(anneal.frames_to_anneal / lc.parameter_publish.exp_interval)
        self.exp_counter = 0
        self.kl_record = []

        gen = torch.Generator().manual_seed(seed)
        mk = lambda: PPOModel(self.obs_spec, self.action_dim, lc.model, True, self.init_log_sig,  # noqa: E731
                              self.use_z_filter, self.if_pixel_input, algo.rnn, self.device, gen)
        self.model = mk()
        self.ref_target_model = mk()
        replicate_from_rank0(dp, self._replicated_state())
        self.ref_target_model.update_target_params(self.model)

        net = algo.network
        self.clip_actor_gradient = net.clip_actor_gradient
        self.actor_gradient_clip_value = net.actor_gradient_norm_clip
        self.clip_critic_gradient = net.clip_critic_gradient
        self.critic_gradient_clip_value = net.critic_gradient_norm_clip
        self.actor_regularization = net.actor_regularization
        self.critic_regularization = net.critic_regularization
        # Adam state (torch.optim.Adam defaults: betas (0.9, 0.999), eps 1e-8)
        dev = self.device
        self.adam_betas, self.adam_eps = (0.9, 0.999), 1e-8
        # Adam moments per optimizer; with the LSTM stem both optimizers own the
        # stem's parameters too (ppo.py:159-168, ppo_net.py:202-224): [head | lstm]
        n_rnn = self.model.stem_flat.numel()          # [lstm | cnn] stems (0 without)
        self.actor_m = torch.zeros(self.model.actor.flat.numel() + n_rnn, device=dev)
        self.actor_v = torch.zeros_like(self.actor_m)
        self.critic_m = torch.zeros(self.model.critic.flat.numel() + n_rnn, device=dev)
        self.critic_v = torch.zeros_like(self.critic_m)
        self.actor_step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.critic_step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.actor_lr_scheduler = LinearWithMinLR(self.lr_actor, num_updates,
                                                  anneal.lr_update_frequency, anneal.min_lr)
        self.critic_lr_scheduler = LinearWithMinLR(self.lr_critic, num_updates,
                                                   anneal.lr_update_frequency, anneal.min_lr)
        self.hyper = torch.zeros(L.HYP_COUNT, dtype=torch.float32, device=dev)
        self._write_hyper()

        self.aggregator = MultistepAggregatorWithInfo(self.obs_spec, ec.action_spec)
        self.pd = DiagGauss(self.action_dim)
        self.cells = None
        if self.use_r_filter:
            self.reward_filter = RewardFilter(device=dev)

        # device-resident learn() state
        self.stats_buf = torch.zeros(L.ST_COUNT, dtype=torch.float32, device=dev)
        self.kl_capacity = 1 << 16
        self.kl_record_buf = torch.zeros(self.kl_capacity, dtype=torch.float32, device=dev)
        self.kl_count = torch.zeros(1, dtype=torch.int32, device=dev)
        idx = torch.tensor(range(self.n_step), dtype=torch.float32)
        self.gamma_tab = torch.pow(self.gamma, idx).to(dev)        # ppo.py:372-374
        self.lam_tab = torch.pow(self.lam, idx).to(dev)
        self._bufs = {}
        self._arena = StagingArena(self.device)
        self._args = L.PPOArgs()
        # optional per-kernel HIP event timing: {kernel name: [(start, end), ...]}
        self.kernel_events = None
        # optional export of the advantages as the policy epochs use them (and
        # the RNN window returns) into self._bufs['adv_used'] / ['ret_used']
        self.export_advantages = False
        # hipGraph replay: one GPU, or data parallel over a capturable group
        # (RCCL: the all-reduces are captured with the kernels).  The data-
        # parallel RewardFilter commits host-side state between its exchange and
        # the GAE, so that combination stays eager.
        self.use_graph = bool(use_graph) and (
            dp is None or (getattr(dp, 'capturable', False) and not self.use_r_filter))
        self._graph = None
        self._gin = None
        # LSTM / pixel phases: ref_pol on a second stream beside the GAE pass
        self.prep_side_stream = os.environ.get('SMI_PREP_SIDE', '0') == '1'
        self._side = None
        self._ctx_side = None

    def _side_stream(self):
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
            self._ctx_side = L.Context(self.device)
        return self._side

    def _replicated_state(self):
        """parameters and filter buffers every data-parallel replica must share"""
        m = self.model
        out = [m.actor.flat, m.critic.flat]
        if m.stem_flat.numel():
            out.append(m.stem_flat)
        if self.use_z_filter:
            out += [m.z_filter.running_sum, m.z_filter.running_sumsq, m.z_filter.count]
        return out

    def _ev(self, name):
        """Context for recording a (start, end) event pair around one launch."""
        learner = self

        class _Ctx(object):
            def __enter__(self):
                if learner.kernel_events is not None:
                    self.s = torch.cuda.Event(enable_timing=True)
                    self.e = torch.cuda.Event(enable_timing=True)
                    self.s.record()
                return self

            def __exit__(self, *exc):
                if learner.kernel_events is not None:
                    self.e.record()
                    learner.kernel_events.setdefault(name, []).append((self.s, self.e))
                return False
        return _Ctx()

    # ------------------------------------------------------------ helpers
    def _hyper_values(self):
        lr_a = self.actor_lr_scheduler.get_lr()[0] if hasattr(self, 'actor_lr_scheduler') else self.lr_actor
        lr_c = self.critic_lr_scheduler.get_lr()[0] if hasattr(self, 'critic_lr_scheduler') else self.lr_critic
        return (self.clip_epsilon, self.beta, lr_a, lr_c)

    def _write_hyper(self):
        self._hyper_key = self._hyper_values()
        h = np.zeros(L.HYP_COUNT, dtype=np.float32)
        h[L.HYP_CLIP_EPS] = self.clip_epsilon
        h[L.HYP_BETA] = self.beta
        h[L.HYP_LR_ACTOR] = self.actor_lr_scheduler.get_lr()[0] if hasattr(self, 'actor_lr_scheduler') else self.lr_actor
        h[L.HYP_LR_CRITIC] = self.critic_lr_scheduler.get_lr()[0] if hasattr(self, 'critic_lr_scheduler') else self.lr_critic
        h[L.HYP_CLIP_LO] = np.float32(1 - self.clip_epsilon)     # torch.clamp scalar bounds
        h[L.HYP_CLIP_HI] = np.float32(1 + self.clip_epsilon)
        self.hyper.copy_(torch.from_numpy(h))

    def _buf(self, name, shape, dtype=torch.float32):
        t = self._bufs.get(name)
        if t is None or tuple(t.shape) != tuple(shape):
            t = torch.zeros(shape, dtype=dtype, device=self.device)
            self._bufs[name] = t
        return t

    def _low_dim(self, obs):
        if isinstance(obs, torch.Tensor):
            return obs
        if 'low_dim' not in obs:
            return None
        parts = [obs['low_dim'][k] for k in obs['low_dim']]
        return parts[0] if len(parts) == 1 else torch.cat(parts, -1)

    # ------------------------------------------------------- reference API
    def _preprocess_batch_ppo(self, batch, rf_sums=None):   # ppo.py:420-484
        """rf_sums (data parallel): the RewardFilter whitens with its current
        stats and writes this rank's {sum, sumsq, n} there instead of updating;
        the caller all-reduces them and commits (RewardFilter.commit_)."""
        if not isinstance(batch['actions'], torch.Tensor) or not batch['actions'].is_cuda:
            batch = self._arena.stage(batch)          # one pinned buffer, one H2D
        else:
            batch = dict(batch)
        rewards = batch['rewards'].to(torch.float32).contiguous().clone()   # filtered in place
        if self.use_r_filter and rf_sums is not None:
            self.reward_filter.scale_forward_partial_(rewards, self.reward_scale, rf_sums)
        elif self.use_r_filter:
            self.reward_filter.scale_forward_update_(rewards, self.reward_scale)
        elif self.reward_scale != 1.0:
            L.call('smi_reward_filter', L.ptr(rewards), rewards.numel(), float(self.reward_scale),
                   0, None, None, None, 0.0, L.stream(self.device))
        batch['rewards'] = rewards
        return Config(batch) if not isinstance(batch, Config) else batch

    def _optimize(self, obs, actions, rewards, obs_next, persistent_infos, onetime_infos, dones):
        """ppo.py:487-586.  The low-dim MLP model runs the single-CU epoch kernels
        when the batch and both networks fit one CU's LDS (B <= 256); an LSTM or
        CNN stem, or a larger low-dim batch (ppo.py:408-418 takes any batch), runs
        the multi-workgroup phase sequence of _optimize_rnn (one window of n_step
        per trajectory without the LSTM)."""
        c_h1, c_h2 = self.learner_config.model.critic_fc_hidden_sizes
        a_h1, a_h2 = self.learner_config.model.actor_fc_hidden_sizes
        phases = self.if_rnn_policy or self.if_pixel_input
        if not phases:
            B_, T_, D_ = self._low_dim(obs).shape
            lds = L.lib().smi_ppo_fused_lds_bytes(B_, D_, a_h1, a_h2, self.action_dim, c_h1, c_h2)
            phases = B_ > 256 or lds > 160 * 1024
        if phases:
            yield from self._optimize_rnn(obs, actions, rewards, obs_next, persistent_infos,
                                          onetime_infos, dones)
            return
        x = self._low_dim(obs).contiguous()
        xn = self._low_dim(obs_next).contiguous()
        B, T, D = x.shape
        if B != self.batch_size or T != self.n_step:
            raise ValueError(f'batch shape (B={B}, T={T}) != config (batch_size={self.batch_size}, '
                             f'n_step={self.n_step})')
        A = self.action_dim
        pds = persistent_infos[-1].contiguous()
        actions = actions.contiguous()
        dones = dones.contiguous()
        st = L.stream(self.device)
        m, rm = self.model, self.ref_target_model
        zf = m.z_filter if self.use_z_filter else None
        rzf = rm.z_filter if self.use_z_filter else None
        values = self._buf('values', (B, T + 1))
        adv_raw = self._buf('adv_raw', (B,))
        ret = self._buf('ret', (B,))
        zp = (lambda t: L.ptr(t) if zf is not None else None)
        # --- GAE over the critic (ppo.py:355-418) -- the fused path
        with self._ev('critic_gae_kernel'):
            L.call('smi_ppo_critic_gae', L.ptr(m.critic.flat), D, c_h1, c_h2, 1 if zf else 0,
                   zp(zf.running_sum if zf else None), zp(zf.running_sumsq if zf else None),
                   zp(zf.count if zf else None), float(zf.eps if zf else 1e-5),
                   L.ptr(x), L.ptr(xn), L.ptr(rewards), L.ptr(dones), B, T,
                   L.ptr(self.gamma_tab), L.ptr(self.lam_tab), float(self.gamma),
                   float(self.gamma ** self.n_step), L.ptr(values), L.ptr(adv_raw), L.ptr(ret), st)
        # --- epochs (ppo.py:505-576)
        a = self._args
        dp = self.dp
        a.B_global = B * (dp.world_size if dp is not None else 1)
        a.xbuf = a.dp_state = None
        a.B, a.obs_dim, a.h1, a.h2, a.act_dim = B, D, a_h1, a_h2, A
        a.critic_h1, a.critic_h2 = c_h1, c_h2
        a.epoch_policy, a.epoch_baseline = self.epoch_policy, self.epoch_baseline
        a.mode = 0 if self.ppo_mode == 'clip' else 1
        a.norm_adv = 1 if self.norm_adv else 0
        a.clip_actor_grad = 1 if self.clip_actor_gradient else 0
        a.clip_critic_grad = 1 if self.clip_critic_gradient else 0
        a.use_zf = 1 if zf is not None else 0
        a.obs, a.obs_stride = x.data_ptr(), T * D                     # obs[:, 0, :]
        a.actions, a.act_stride = actions.data_ptr(), T * A           # actions[:, 0, :]
        a.behave, a.beh_stride = pds.data_ptr(), T * 2 * A            # pds[:, 0, :]
        a.adv_raw, a.adv_moments, a.ret = adv_raw.data_ptr(), None, ret.data_ptr()
        if zf is not None:
            a.zf_sum, a.zf_sumsq, a.zf_count = (zf.running_sum.data_ptr(),
                                                zf.running_sumsq.data_ptr(), zf.count.data_ptr())
            a.rzf_sum, a.rzf_sumsq, a.rzf_count = (rzf.running_sum.data_ptr(),
                                                   rzf.running_sumsq.data_ptr(), rzf.count.data_ptr())
            a.zf_eps = zf.eps
        else:
            a.zf_sum = a.zf_sumsq = a.zf_count = a.rzf_sum = a.rzf_sumsq = a.rzf_count = None
            a.zf_eps = 1e-5
        a.actor, a.ref_actor, a.critic = (m.actor.flat.data_ptr(), rm.actor.flat.data_ptr(),
                                          m.critic.flat.data_ptr())
        a.actor_m, a.actor_v = self.actor_m.data_ptr(), self.actor_v.data_ptr()
        a.critic_m, a.critic_v = self.critic_m.data_ptr(), self.critic_v.data_ptr()
        a.actor_step, a.critic_step = self.actor_step.data_ptr(), self.critic_step.data_ptr()
        a.hyper = self.hyper.data_ptr()
        a.kl_target = float(self.kl_target)
        a.kl_cutoff_coeff = float(self.kl_cutoff_coeff)
        a.actor_max_norm = float(self.actor_gradient_clip_value)
        a.critic_max_norm = float(self.critic_gradient_clip_value)
        a.actor_wd, a.critic_wd = float(self.actor_regularization), float(self.critic_regularization)
        a.beta1, a.beta2, a.adam_eps = self.adam_betas[0], self.adam_betas[1], self.adam_eps
        a.stats = self.stats_buf.data_ptr()
        a.kl_record, a.kl_count, a.kl_capacity = (self.kl_record_buf.data_ptr(),
                                                  self.kl_count.data_ptr(), self.kl_capacity)
        self._last_ret = ret
        a.adv_out = self._buf('adv_used', (B,)).data_ptr() if self.export_advantages else None
        maxp = L.lib().smi_ppo_fused_max_params()
        fused = dp is None and max(L.lib().smi_mlp_param_count(D, a_h1, a_h2, A, 1),
                                   L.lib().smi_mlp_param_count(D, c_h1, c_h2, 1, 0)) <= maxp
        if fused:
            with self._ev('ppo_fused_kernel'):
                L.check(L.lib().smi_ppo_update_fused(a, st), 'smi_ppo_update_fused')
            # --- z_update(obs_iter) after the updates (ppo.py:578-582)
            if zf is not None:
                with self._ev('colstats_small_kernel'):
                    L.call('smi_zfilter_update', L.ptr(x), B, D, T * D, L.ptr(zf.running_sum),
                           L.ptr(zf.running_sumsq), L.ptr(zf.count), st)
            return
        # ---- data parallel, or one GPU with networks too large
        # for the fused kernel: global advantage moments, then max(E+1, Ev)
        # phases of [rank-local gradients -> all-reduce (dp only) -> apply]
        mom = self._buf('adv_moments', (3,), torch.float64)
        L.call('smi_moments', L.ptr(adv_raw), B, None, 0, L.ptr(mom), st)
        self._phase_tag = 'moments'
        yield mom
        a.adv_moments = mom.data_ptr()
        nx = L.lib().smi_ppo_xbuf_floats(D, a_h1, a_h2, A, c_h1, c_h2, a.mode)
        xbuf = self._buf('xbuf', (nx,))
        dp_state = self._buf('dp_state', (4,), torch.int32)
        dp_state.zero_()
        a.xbuf, a.dp_state = xbuf.data_ptr(), dp_state.data_ptr()
        for e in range(max(self.epoch_policy + 1, self.epoch_baseline)):
            with self._ev('ppo_epoch_grad_kernel'):
                L.check(L.lib().smi_ppo_epoch_grad(a, e, st), 'smi_ppo_epoch_grad')
            self._phase_tag = 'epoch_grad'          # actor AND critic gradients of epoch e
            yield xbuf
            with self._ev('ppo_epoch_apply_kernel'):
                L.check(L.lib().smi_ppo_epoch_apply(a, e, st), 'smi_ppo_epoch_apply')
        if zf is not None:                                    # global z_update
            zbuf = self._buf('zbuf', (2, D))
            L.call('smi_zfilter_colstats', L.ptr(x), B, D, T * D, L.ptr(zbuf[0]), L.ptr(zbuf[1]), st)
            self._phase_tag = 'zstats'
            yield zbuf
            L.call('smi_zfilter_accumulate', L.ptr(zbuf[0]), L.ptr(zbuf[1]), D, float(a.B_global),
                   L.ptr(zf.running_sum), L.ptr(zf.running_sumsq), L.ptr(zf.count), st)

    def _optimize_rnn(self, obs, actions, rewards, obs_next, persistent_infos, onetime_infos,
                      dones):
        """ppo.py:487-586 with if_rnn_policy: the phase sequence of
        smi_ppo_rnn_phase (include/surreal_mi.h), yielding the buffers a data-
        parallel learner all-reduces between phases."""
        x = self._low_dim(obs)
        xn = self._low_dim(obs_next)
        pix = pixn = None
        if self.if_pixel_input:
            pix = obs['pixel']['camera0']
            pixn = obs_next['pixel']['camera0']
            if pix.dtype != torch.uint8 or pixn.dtype != torch.uint8:
                raise TypeError('camera0 observations must be uint8')
            pix, pixn = pix.contiguous(), pixn.contiguous()
        if x is not None:
            x, xn = x.contiguous(), xn.contiguous()
            B, T, D = x.shape
        else:
            B, T = pix.shape[:2]
            D = 0
        if B != self.batch_size or T != self.n_step:
            raise ValueError(f'batch shape (B={B}, T={T}) != config (batch_size={self.batch_size}, '
                             f'n_step={self.n_step})')
        A = self.action_dim
        if self.if_rnn_policy:
            if onetime_infos is None or len(onetime_infos) < 2:
                raise ValueError('RNN policy: onetime_infos must hold the (h, c) LSTM cells')
            Hd = self.learner_config.algo.rnn.rnn_hidden
            # (B, L, H) -> (L, B, H), as ppo.py:508-509 transposes them
            NL = self.rnn_layer
            h0 = onetime_infos[0].reshape(B, NL, Hd).transpose(0, 1).contiguous()
            c0 = onetime_infos[1].reshape(B, NL, Hd).transpose(0, 1).contiguous()
        else:                       # MLP policy over the pixel stem (ppo.py:532-535: step 0)
            Hd, h0, c0 = 0, None, None
        pds = persistent_infos[-1].contiguous()
        actions = actions.contiguous()
        dones = dones.contiguous()
        st = L.stream(self.device)
        m, rm = self.model, self.ref_target_model
        zf = m.z_filter if self.use_z_filter else None
        rzf = rm.z_filter if self.use_z_filter else None
        a_h1, a_h2 = self.learner_config.model.actor_fc_hidden_sizes
        c_h1, c_h2 = self.learner_config.model.critic_fc_hidden_sizes
        H = self.horizon if self.if_rnn_policy else T      # non-RNN: one window of n_step
        lib = L.lib()
        pc, ph, pw = self.obs_spec['pixel']['camera0'] if pix is not None else (0, 0, 0)
        F = int(self.learner_config.model.cnn_feature_dim) if pix is not None else 0
        nbytes = lib.smi_ppo_rnn_scratch_bytes(B, T, H, D, Hd, a_h1, a_h2, A, c_h1, c_h2,
                                               pc, ph, pw, F, self.rnn_layer)
        scratch = self._buf('rnn_scratch', (nbytes // 4,))
        nx = lib.smi_ppo_rnn_xbuf_floats(D, Hd, a_h1, a_h2, A, c_h1, c_h2, pc, ph, pw, F,
                                         self.rnn_layer)
        xbuf = self._buf('rnn_xbuf', (nx,))
        moments = self._buf('rnn_moments', (3,), torch.float64)
        pstat = self._buf('rnn_pstat', (L.RNN_PSTAT,), torch.float64)
        zbuf = self._buf('rnn_zbuf', (5 + 2 * D,), torch.float64)
        nA = m.actor.flat.numel() + m.stem_flat.numel()
        nC = m.critic.flat.numel() + m.stem_flat.numel()
        a = L.RNNArgs()
        dp = self.dp
        a.B, a.T, a.horizon, a.obs_dim, a.rnn_hidden = B, T, H, D, Hd
        a.h1, a.h2, a.act_dim, a.critic_h1, a.critic_h2 = a_h1, a_h2, A, c_h1, c_h2
        a.epoch_policy, a.epoch_baseline = self.epoch_policy, self.epoch_baseline
        a.mode = 0 if self.ppo_mode == 'clip' else 1
        a.norm_adv = 1 if self.norm_adv else 0
        a.clip_actor_grad = 1 if self.clip_actor_gradient else 0
        a.clip_critic_grad = 1 if self.clip_critic_gradient else 0
        a.use_zf = 1 if zf is not None else 0
        a.B_global = B * (dp.world_size if dp is not None else 1)
        a.obs = x.data_ptr() if x is not None else None
        a.obs_next = xn.data_ptr() if xn is not None else None
        a.actions = actions.data_ptr()
        a.pix_c, a.pix_h, a.pix_w, a.cnn_feat = pc, ph, pw, F
        a.rnn_layer = self.rnn_layer
        # PREP on a second stream (below) must not depend on GAE: say so explicitly
        a.prep_independent = 1 if self.prep_side_stream else 0
        a.pixels = pix.data_ptr() if pix is not None else None
        a.pixels_next = pixn.data_ptr() if pixn is not None else None
        a.rewards, a.dones, a.behave = rewards.data_ptr(), dones.data_ptr(), pds.data_ptr()
        a.h0 = h0.data_ptr() if h0 is not None else None
        a.c0 = c0.data_ptr() if c0 is not None else None
        a.lstm, a.actor, a.critic = (m.stem_flat.data_ptr(), m.actor.flat.data_ptr(),
                                     m.critic.flat.data_ptr())
        a.ref_lstm, a.ref_actor = rm.stem_flat.data_ptr(), rm.actor.flat.data_ptr()
        if zf is not None:
            a.zf_sum, a.zf_sumsq, a.zf_count = (zf.running_sum.data_ptr(),
                                                zf.running_sumsq.data_ptr(), zf.count.data_ptr())
            a.rzf_sum, a.rzf_sumsq, a.rzf_count = (rzf.running_sum.data_ptr(),
                                                   rzf.running_sumsq.data_ptr(), rzf.count.data_ptr())
            a.zf_eps = zf.eps
        else:
            a.zf_sum = a.zf_sumsq = a.zf_count = a.rzf_sum = a.rzf_sumsq = a.rzf_count = None
            a.zf_eps = 1e-5
        a.actor_m, a.actor_v = self.actor_m.data_ptr(), self.actor_v.data_ptr()
        a.critic_m, a.critic_v = self.critic_m.data_ptr(), self.critic_v.data_ptr()
        a.actor_step, a.critic_step = self.actor_step.data_ptr(), self.critic_step.data_ptr()
        a.hyper = self.hyper.data_ptr()
        a.gamma_tab, a.lam_tab = self.gamma_tab.data_ptr(), self.lam_tab.data_ptr()
        a.gamma = float(self.gamma)
        a.gamma_H = float(self.gamma ** H)                           # ppo.py:400 (python float)
        a.kl_target = float(self.kl_target)
        a.kl_cutoff_coeff = float(self.kl_cutoff_coeff)
        a.actor_max_norm = float(self.actor_gradient_clip_value)
        a.critic_max_norm = float(self.critic_gradient_clip_value)
        a.actor_wd, a.critic_wd = float(self.actor_regularization), float(self.critic_regularization)
        a.beta1, a.beta2, a.adam_eps = self.adam_betas[0], self.adam_betas[1], self.adam_eps
        a.stats = self.stats_buf.data_ptr()
        a.kl_record, a.kl_count, a.kl_capacity = (self.kl_record_buf.data_ptr(),
                                                  self.kl_count.data_ptr(), self.kl_capacity)
        a.moments, a.pstat, a.xbuf, a.zbuf = (moments.data_ptr(), pstat.data_ptr(),
                                              xbuf.data_ptr(), zbuf.data_ptr())
        a.scratch, a.scratch_bytes = scratch.data_ptr(), nbytes
        E = T - H + 1
        a.adv_out = self._buf('adv_used', (B, E)).data_ptr() if self.export_advantages else None
        a.ret_out = self._buf('ret_used', (B, E)).data_ptr() if self.export_advantages else None
        self._rnn_args = a

        def ph(p, e=0, stream=st):
            with self._ev(_RNN_PHASE_NAMES[p]):
                L.check(lib.smi_ppo_rnn_phase(a, p, e, stream), 'smi_ppo_rnn_phase')

        # ref_pol (PREP, ppo.py:539) depends only on the batch and the reference
        # parameters: it runs on a second stream with its own workspace beside
        # the GAE phase's critic pass (two independent recurrences; at small
        # local batches each fills a fraction of the CUs), joined before the
        # first policy forward
        side = self._side_stream() if self.prep_side_stream else None
        if side is not None:
            main = torch.cuda.current_stream(self.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self._ctx_side.make_current()
                ph(L.RNN_PH_PREP, stream=L.stream(self.device))
            self._ctx.make_current()
        ph(L.RNN_PH_GAE)
        self._phase_tag = 'moments'
        yield moments
        if side is None:
            ph(L.RNN_PH_PREP)
        else:
            torch.cuda.current_stream(self.device).wait_stream(side)
        for e in range(self.epoch_policy + 1):                  # ppo.py:541-557
            ph(L.RNN_PH_POLICY_FWD, e)
            self._phase_tag = 'policy_stats'
            yield pstat
            ph(L.RNN_PH_POLICY_DECIDE, e)
            if e < self.epoch_policy:
                ph(L.RNN_PH_POLICY_BWD, e)
                self._phase_tag = 'policy_grad'
                yield xbuf[:nA]
                ph(L.RNN_PH_POLICY_APPLY, e)
        for e in range(self.epoch_baseline):                    # ppo.py:561-562
            ph(L.RNN_PH_VALUE_GRAD, e)
            self._phase_tag = 'value_grad'
            yield xbuf[nA:nA + nC]
            ph(L.RNN_PH_VALUE_APPLY, e)
        ph(L.RNN_PH_ZSTATS)                                      # ppo.py:578-582
        self._phase_tag = 'zstats'
        yield zbuf
        ph(L.RNN_PH_ZAPPLY)

    def _device_phases(self, batch, preprocessed=False):
        """the device part of learn(): preprocess + _optimize (generator)"""
        if not preprocessed:
            batch = self._preprocess_batch_ppo(batch)
        for buf in self._optimize(batch['obs'], batch['actions'], batch['rewards'],
                                  batch['obs_next'], batch['persistent_infos'],
                                  batch['onetime_infos'], batch['dones']):
            yield buf
            self._ctx.make_current()      # whatever ran on this thread meanwhile

    def _learn_phases(self, batch):
        """learn() as a generator of the buffers a data-parallel learner must
        all-reduce (SUM) between its launches (the single-CU C2 kernel yields
        nothing).  Before each yield `_phase_tag` names the buffer: 'moments',
        'policy_stats', 'policy_grad' / 'value_grad' (the parameters are still
        those the gradient was taken at), 'epoch_grad' (MLP phases: both),
        'zstats', 'reward_filter'."""
        self.current_iteration += 1
        self._ctx.make_current()
        if self._hyper_values() != self._hyper_key:       # e.g. schedulers restored from a checkpoint
            self._write_hyper()
        if self.dp is not None and self.use_r_filter:
            # global reward statistics: one 3-double all-reduce (reward_filter.py:33-42
            # over the global batch, as one learner would see it)
            rf = self._buf('rf_sums', (3,), torch.float64)
            batch = self._preprocess_batch_ppo(batch, rf_sums=rf)
            self._phase_tag = 'reward_filter'
            yield rf
            self._ctx.make_current()
            self.reward_filter.commit_(rf)
            yield from self._device_phases(batch, preprocessed=True)
        else:
            yield from self._device_phases(batch)
        self._learn_epilogue()

    def _learn_epilogue(self):                                # ppo.py:606-613
        self.periodic_checkpoint(global_steps=self.current_iteration, score=None)
        self._report_metrics(self.global_step)
        self.exp_counter += self.batch_size * (self.dp.world_size if self.dp is not None else 1)
        self.global_step += 1

    def learn(self, batch):                                   # ppo.py:588-613
        if self.use_graph and self.kernel_events is None:
            return self._learn_graphed(batch)
        for buf in self._learn_phases(batch):
            if self.dp is not None:                           # single GPU: phases, no exchange
                self.dp.allreduce_(buf)

    # ------------------------------------------------------- hipGraph replay
    @staticmethod
    def _leaves(batch):
        """the batch's tensors in a fixed order, a function rebuilding the same
        structure over another list of tensors, and the structure's signature
        (leaf paths: part of the capture key, so a batch whose nesting differs
        never replays a graph over a mismatched leaf order)"""
        out, paths = [], []

        def walk(x, path):
            if isinstance(x, dict):
                return {k: walk(v, path + (k,)) for k, v in x.items()}
            if isinstance(x, (list, tuple)):
                return [walk(v, path + (i,)) for i, v in enumerate(x)]
            if x is None:
                return None
            out.append(x)
            paths.append(path)
            return len(out) - 1
        skel = walk(batch, ())

        def build(ts):
            def mk(x):
                if isinstance(x, dict):
                    return {k: mk(v) for k, v in x.items()}
                if isinstance(x, list):
                    return [mk(v) for v in x]
                return None if x is None else ts[x]
            return mk(skel)
        return out, build, tuple(paths)

    def _learn_graphed(self, batch):
        """learn() as one hipGraph replay of the device sequence (module
        docstring: no host synchronisation happens inside learn(), so the whole
        phase sequence, the side-stream ref_pol pass included, is capturable).
        The first call (and any call whose batch shapes differ) runs eagerly —
        that call's update, sizing every scratch buffer — then captures the
        same launches over static copies of the inputs."""
        if not isinstance(batch['actions'], torch.Tensor) or not batch['actions'].is_cuda:
            batch = self._arena.stage(batch)
        leaves, build, paths = self._leaves(batch)
        # the host switches read while the launches are issued are part of
        # what a captured graph bakes in (export pointers, the side stream,
        # the epoch counts and the device the phases run on)
        key = (paths, tuple((tuple(t.shape), t.dtype) for t in leaves), bool(self.export_advantages),
               bool(self.prep_side_stream), self.epoch_policy, self.epoch_baseline)
        self.current_iteration += 1
        self._ctx.make_current()
        if self._hyper_values() != self._hyper_key:
            self._write_hyper()
        dp = self.dp
        if self._graph is None or self._graph_key != key:
            for buf in self._device_phases(batch):
                if dp is not None:
                    dp.allreduce_(buf)
            self._gin = _GraphInputs(leaves, self.device)
            self._gin.refresh(leaves)
            static = build(self._gin.views)
            # quiesce the parameter publisher (its worker thread synchronizes
            # events and launches copies on its own stream) before capturing,
            # and capture in thread-local mode so another thread's CUDA calls
            # cannot invalidate the capture
            if self.publisher is not None and hasattr(self.publisher, 'flush'):
                self.publisher.flush()
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            err = None
            try:
                with L.gc_paused(), torch.cuda.graph(g, capture_error_mode='thread_local'):
                    self._ctx.make_current()
                    for buf in self._device_phases(static):
                        if dp is not None:            # RCCL all-reduce, captured
                            dp.allreduce_(buf)
            except RuntimeError as e:
                if dp is None:
                    raise
                err = e
            # data parallel: every rank takes the same path, so no rank replays
            # a graph while another issues eager launches (one flag all-reduced
            # eagerly, once per capture)
            if dp is not None and not self._capture_agreed(err is None):
                # a collective library that refuses capture (on this rank or a
                # peer): the learners stay eager (this call's update already
                # ran above)
                import warnings
                warnings.warn('data-parallel learn() could not be captured '
                              f'({err if err is not None else "on a peer rank"}); eager launches')
                self.use_graph = False
                self._graph = None
                self._ctx.make_current()
                self._learn_epilogue()
                return
            self._ctx.make_current()
            self._graph, self._graph_key = g, key
        else:
            self._gin.refresh(leaves)
            self._graph.replay()
        self._learn_epilogue()

    def _capture_agreed(self, ok):
        """True when every rank captured its learn() (one eager all-reduce of
        a failure count)"""
        flag = torch.tensor([0.0 if ok else 1.0], dtype=torch.float32, device=self.device)
        self.dp.allreduce_(flag)
        return float(flag.item()) == 0.0

    def _host_scalars(self):
        """host-side entries of the statistics (averaged by a throttled sink)"""
        out = {'_lr': self.actor_lr_scheduler.get_lr()[0]}
        if self.ppo_mode == 'clip':
            out['_clip_epsilon'] = self.clip_epsilon
        else:
            out['_beta'] = self.beta
        return out

    def last_stats(self):
        """Statistics dict of the last learn() (ppo.py:219-224,278-284,328-331,555,571-582).
        Synchronises with the device."""
        return self._stats_dict(self.stats_buf.cpu().numpy(), self._host_scalars())

    def _stats_vector(self):
        """the statistics a throttled sink averages per call: the device vector
        and, with the z-filter, np.mean of its running mean / square / std
        (ppo.py:578-582), formed on the device (no host read per learn())"""
        if not self.use_z_filter:
            return self.stats_buf
        zf = self.model.z_filter
        m = zf.running_sum / zf.count
        sq = zf.running_sumsq / zf.count
        zv = torch.stack([m.mean(), sq.mean(), (sq - m * m).pow(0.5).mean()])
        return torch.cat([self.stats_buf, zv.to(self.stats_buf.dtype)])

    def _stats_dict(self, v, host):
        """the reference's statistics dict from a host copy of the device
        statistics vector v and the host scalars (_lr, _clip_epsilon / _beta);
        v may carry the averaged z-filter means after the L.ST_COUNT entries
        (_stats_vector)"""
        s = {}
        if self.ppo_mode == 'clip':
            for k in ('_surr_loss', '_clip_surr_loss', '_entropy'):
                s[k] = float(v[L.ST[k]])
            s['_clip_epsilon'] = host['_clip_epsilon']
        else:
            for k in ('_kl_loss_adapt', '_surr_loss', '_entropy'):
                s[k] = float(v[L.ST[k]])
            s['_beta'] = host['_beta']
        s['_pol_kl'] = float(v[L.ST['_pol_kl']])
        if self.clip_actor_gradient:
            s['grad_norm_actor'] = float(v[L.ST['grad_norm_actor']])
        for k in ('_val_loss', '_val_explained_var', '_avg_return_targ', '_avg_log_sig',
                  '_avg_behave_likelihood', '_avg_is_weight', '_ref_behave_diff'):
            s[k] = float(v[L.ST[k]])
        if self.clip_critic_gradient:
            s['grad_norm_critic'] = float(v[L.ST['grad_norm_critic']])
        s['_lr'] = host['_lr']
        er = float(v[L.ST['epochs_run']])              # (an average over a throttled window)
        s['epochs_run'] = int(er) if er == int(er) else er
        if self.use_z_filter:
            if len(v) >= L.ST_COUNT + 3:
                s['obs_running_mean'], s['obs_running_square'], s['obs_running_std'] = (
                    float(x) for x in v[L.ST_COUNT:L.ST_COUNT + 3])
            else:
                zf = self.model.z_filter
                s['obs_running_mean'] = float(np.mean(zf.running_mean()))
                s['obs_running_square'] = float(np.mean(zf.running_square()))
                s['obs_running_std'] = float(np.mean(zf.running_std()))
        if self.use_r_filter:
            s['reward_mean'] = self.reward_filter.reward_mean()
        return s

    def module_dict(self):
        return {'ppo': self.model}

    def publish_parameter(self, iteration, message=''):       # ppo.py:623-635
        """Publish once `exp_interval` experiences were learned since the last
        publish.  `publisher` may be a publish.DeviceParameterPublisher (an
        asynchronous snapshot: D2D on the learner stream, D2H on a side stream,
        serialization on a worker thread) or any callable(iteration, message,
        module_dict)."""
        if self.exp_counter >= self.learner_config.parameter_publish.exp_interval:
            deferred = False
            if self.publisher is not None:
                if hasattr(self.publisher, 'commit'):
                    self.publisher.snapshot(iteration, message, defer=True)
                    deferred = True
                elif hasattr(self.publisher, 'snapshot'):
                    self.publisher.snapshot(iteration, message)
                else:
                    self.publisher(iteration, message, self.module_dict())
            self._post_publish()
            if deferred:                  # the D2H after this thread's host reads
                self.publisher.commit()

    def _post_publish(self):                                  # ppo.py:637-666
        n = int(self.kl_count.item())
        rec = self.kl_record_buf[:min(n, self.kl_capacity)].cpu().numpy().astype(np.float64)
        self.kl_record = list(rec)
        final_kl = np.mean(self.kl_record)
        consts = self.learner_config.algo
        if self.ppo_mode == 'clip':
            if final_kl > self.kl_target * self.clip_adjust_threshold[1]:
                if self.clip_lower < self.clip_epsilon:
                    self.clip_epsilon = self.clip_epsilon / consts.clip_consts.scale_constant
            elif final_kl < self.kl_target * self.clip_adjust_threshold[0]:
                if self.clip_upper > self.clip_epsilon:
                    self.clip_epsilon = self.clip_epsilon * consts.clip_consts.scale_constant
        else:
            if final_kl > self.kl_target * self.beta_adjust_threshold[1]:
                if self.beta_upper > self.beta:
                    self.beta = self.beta * consts.adapt_consts.scale_constant
            elif final_kl < self.kl_target * self.beta_adjust_threshold[0]:
                if self.beta_lower < self.beta:
                    self.beta = self.beta / consts.adapt_consts.scale_constant
        self.ref_target_model.update_target_params(self.model)
        self.kl_record = []
        self.kl_count.zero_()
        self.exp_counter = 0
        self.actor_lr_scheduler.step()
        self.critic_lr_scheduler.step()
        self._write_hyper()

    def checkpoint_attributes(self):                          # ppo.py:668-678
        """Attribute names for the reference Checkpoint (utils/checkpoint.py:
        234-246: state_dict() of nn.Modules, the object itself otherwise).
        `model` / `ref_target_model` are nn.Modules (compact state_dicts of the
        flat device buffers), the LR schedulers plain picklable objects."""
        attrs = ['model', 'ref_target_model', 'actor_lr_scheduler', 'critic_lr_scheduler',
                 'current_iteration']
        if self.checkpoint_full_state:
            attrs += ['optimizer_state_host', 'adaptive_state']
        return attrs

    @property
    def optimizer_state_host(self):
        """Adam moments and step counters as host tensors (checkpointable)."""
        return {k: v.detach().cpu().clone() for k, v in self.optimizer_state().items()}

    @optimizer_state_host.setter
    def optimizer_state_host(self, d):
        with torch.no_grad():
            for k, v in self.optimizer_state().items():
                v.copy_(torch.as_tensor(d[k]).to(v.device))

    @property
    def adaptive_state(self):
        """Host-side adaptive hyper-parameters and the device KL record."""
        n = min(int(self.kl_count.item()), self.kl_capacity)
        out = {'beta': self.beta, 'clip_epsilon': self.clip_epsilon, 'exp_counter': self.exp_counter,
               'global_step': self.global_step, 'kl_record': self.kl_record_buf[:n].cpu().clone(),
               'kl_count': self.kl_count.cpu().clone()}
        if self.use_r_filter:
            out['reward_filter'] = {k: v.cpu().clone() for k, v in self.reward_filter.state_dict().items()}
        return out

    @adaptive_state.setter
    def adaptive_state(self, d):
        self.beta, self.clip_epsilon = d['beta'], d['clip_epsilon']
        self.exp_counter, self.global_step = d['exp_counter'], d['global_step']
        with torch.no_grad():
            rec = torch.as_tensor(d['kl_record'])
            self.kl_record_buf[:rec.numel()].copy_(rec.to(self.device))
            self.kl_count.copy_(torch.as_tensor(d['kl_count']).to(self.device))
        if self.use_r_filter and 'reward_filter' in d:
            self.reward_filter.load_state_dict(d['reward_filter'])
        self._write_hyper()

    def preprocess(self, batch):                              # learner/base.py:321-330
        return batch

    def _prefetcher_preprocess(self, batch):                  # ppo.py:680-682
        return self.aggregator.aggregate(batch)

    # extra (not in the reference API): optimizer state for tests/checkpoints
    def optimizer_state(self):
        return {'actor_m': self.actor_m, 'actor_v': self.actor_v, 'actor_step': self.actor_step,
                'critic_m': self.critic_m, 'critic_v': self.critic_v,
                'critic_step': self.critic_step}
