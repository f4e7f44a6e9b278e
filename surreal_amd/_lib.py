"""ctypes binding of libsurreal_mi.so (the C ABI of include/surreal_mi.h).

The product path has no CPU fallback: if the library is missing or no GPU is
visible, calls raise.  torch is imported first so the process holds torch's
HIP runtime before the library binds to it (same SONAME, one runtime).
"""
import contextlib
import threading
import ctypes
import gc
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
# SMI_LIB_VARIANT=prof selects the developer phase-timer build (build.py VARIANTS)
_VARIANT = os.environ.get('SMI_LIB_VARIANT')
LIB_PATH = os.path.join(HERE, 'libsurreal_mi.so' if not _VARIANT else f'libsurreal_mi_{_VARIANT}.so')

c_int, c_i64, c_f32, c_f64, c_vp = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_double, ctypes.c_void_p
P = ctypes.c_void_p

# device hyper-parameter / statistics slots (include/surreal_mi.h)
HYP_CLIP_EPS, HYP_BETA, HYP_LR_ACTOR, HYP_LR_CRITIC, HYP_CLIP_LO, HYP_CLIP_HI, HYP_COUNT = range(7)
ST_NAMES = ['_surr_loss', '_clip_surr_loss', '_kl_loss_adapt', '_entropy', '_pol_kl',
            'grad_norm_actor', '_val_loss', '_val_explained_var', 'grad_norm_critic',
            '_avg_return_targ', '_avg_log_sig', '_avg_behave_likelihood', '_avg_is_weight',
            '_ref_behave_diff', 'epochs_run', '_pol_kl_adapt']
ST_COUNT = len(ST_NAMES)
ST = {n: i for i, n in enumerate(ST_NAMES)}


class PPOArgs(ctypes.Structure):
    """struct smi_ppo_args (include/surreal_mi.h)."""
    _fields_ = [
        ('B', c_int), ('obs_dim', c_int), ('h1', c_int), ('h2', c_int), ('act_dim', c_int),
        ('critic_h1', c_int), ('critic_h2', c_int),
        ('epoch_policy', c_int), ('epoch_baseline', c_int),
        ('mode', c_int), ('norm_adv', c_int),
        ('clip_actor_grad', c_int), ('clip_critic_grad', c_int), ('use_zf', c_int),
        ('obs', P), ('obs_stride', c_i64),
        ('actions', P), ('act_stride', c_i64),
        ('behave', P), ('beh_stride', c_i64),
        ('adv_raw', P), ('adv_moments', P), ('ret', P),
        ('zf_sum', P), ('zf_sumsq', P), ('zf_count', P),
        ('rzf_sum', P), ('rzf_sumsq', P), ('rzf_count', P),
        ('zf_eps', c_f32),
        ('actor', P), ('ref_actor', P), ('critic', P),
        ('actor_m', P), ('actor_v', P), ('critic_m', P), ('critic_v', P),
        ('actor_step', P), ('critic_step', P),
        ('hyper', P),
        ('kl_target', c_f64), ('kl_cutoff_coeff', c_f32),
        ('actor_max_norm', c_f32), ('critic_max_norm', c_f32),
        ('actor_wd', c_f32), ('critic_wd', c_f32),
        ('beta1', c_f32), ('beta2', c_f32), ('adam_eps', c_f32),
        ('stats', P),
        ('kl_record', P), ('kl_count', P), ('kl_capacity', c_int),
        ('B_global', c_i64), ('xbuf', P), ('dp_state', P),
        ('adv_out', P),
    ]


class RNNArgs(ctypes.Structure):
    """struct smi_ppo_rnn_args (include/surreal_mi.h)."""
    _fields_ = [
        ('B', c_int), ('T', c_int), ('horizon', c_int), ('obs_dim', c_int), ('rnn_hidden', c_int),
        ('h1', c_int), ('h2', c_int), ('act_dim', c_int), ('critic_h1', c_int), ('critic_h2', c_int),
        ('epoch_policy', c_int), ('epoch_baseline', c_int),
        ('mode', c_int), ('norm_adv', c_int), ('clip_actor_grad', c_int), ('clip_critic_grad', c_int),
        ('use_zf', c_int),
        ('B_global', c_i64),
        ('obs', P), ('obs_next', P), ('actions', P), ('rewards', P), ('dones', P), ('behave', P),
        ('h0', P), ('c0', P),
        ('lstm', P), ('actor', P), ('critic', P), ('ref_lstm', P), ('ref_actor', P),
        ('zf_sum', P), ('zf_sumsq', P), ('zf_count', P),
        ('rzf_sum', P), ('rzf_sumsq', P), ('rzf_count', P),
        ('zf_eps', c_f32),
        ('actor_m', P), ('actor_v', P), ('critic_m', P), ('critic_v', P),
        ('actor_step', P), ('critic_step', P),
        ('hyper', P), ('gamma_tab', P), ('lam_tab', P),
        ('gamma', c_f32), ('gamma_H', c_f32),
        ('kl_target', c_f64),
        ('kl_cutoff_coeff', c_f32), ('actor_max_norm', c_f32), ('critic_max_norm', c_f32),
        ('actor_wd', c_f32), ('critic_wd', c_f32),
        ('beta1', c_f32), ('beta2', c_f32), ('adam_eps', c_f32),
        ('stats', P), ('kl_record', P), ('kl_count', P), ('kl_capacity', c_int),
        ('moments', P), ('pstat', P), ('xbuf', P), ('zbuf', P),
        ('scratch', P), ('scratch_bytes', c_i64),
        ('pix_c', c_int), ('pix_h', c_int), ('pix_w', c_int), ('cnn_feat', c_int),
        ('pixels', P), ('pixels_next', P),
        ('adv_out', P), ('ret_out', P),
        ('rnn_layer', c_int), ('prep_independent', c_int),
    ]


RNN_PH_GAE, RNN_PH_PREP, RNN_PH_POLICY_FWD, RNN_PH_POLICY_BWD, RNN_PH_POLICY_APPLY, \
    RNN_PH_VALUE_GRAD, RNN_PH_VALUE_APPLY, RNN_PH_ZSTATS, RNN_PH_ZAPPLY, RNN_PH_POLICY_DECIDE = range(10)
RNN_PSTAT = 16
KT_NAMES = ['gemm_fwd', 'gemm_dx', 'gemm_dw', 'gemm_splitk_reduce', 'lstm_fwd', 'lstm_bwd',
            'cnn_fwd', 'cnn_bwd',
            # HBM-bound streaming classes: their work unit is algorithmic BYTES
            'gae', 'policy_rows_stats', 'policy_rows_grad', 'value_rows', 'adam', 'zf_tmajor']
KT_BYTES = set(KT_NAMES[8:])


def kernel_timing(on):
    check(lib().smi_kernel_timing(1 if on else 0), 'smi_kernel_timing')


def kernel_timing_report():
    """{class: (launches, total_ms, total_flops)} of the recorded launches."""
    out = {}
    buf = (c_f64 * 4)()
    for i, n in enumerate(KT_NAMES):
        check(lib().smi_kernel_timing_report(i, ctypes.cast(buf, P)), 'smi_kernel_timing_report')
        if buf[0] > 0:
            out[n] = (int(buf[0]), float(buf[1]), float(buf[2]))
    return out

_SIGS = {
    'smi_version': (c_int, []),
    'smi_last_error': (ctypes.c_char_p, []),
    'smi_workspace_bytes': (c_i64, []),
    'smi_set_workspace': (c_int, [P, c_i64]),
    'smi_context_create': (P, [P, c_i64]),
    'smi_context_make_current': (c_int, [P]),
    'smi_context_destroy': (c_int, [P]),
    'smi_mlp_param_count': (c_i64, [c_int, c_int, c_int, c_int, c_int]),
    'smi_ppo_fused_lds_bytes': (c_i64, [c_int] * 7),
    'smi_ppo_fused_max_params': (c_i64, []),
    'smi_zfilter_apply': (c_int, [P, P, c_i64, c_int, P, P, P, c_f32, P]),
    'smi_zfilter_update': (c_int, [P, c_i64, c_int, c_i64, P, P, P, P]),
    'smi_zfilter_colstats': (c_int, [P, c_i64, c_int, c_i64, P, P, P]),
    'smi_zfilter_tmajor': (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, P, P, P, c_f32, P,
                                   c_int, c_int, P]),
    'smi_reward_filter': (c_int, [P, c_i64, c_f32, c_int, P, P, P, c_f32, P]),
    'smi_reward_filter_partial': (c_int, [P, c_i64, c_f32, c_int, P, P, P, c_f32, P, P]),
    'smi_reward_filter_commit': (c_int, [P, P, P, P, P]),
    'smi_dw_group_begin': (c_int, []),
    'smi_dw_group_flush': (c_int, [P]),
    'smi_layernorm_forward': (c_int, [P, c_i64, c_i64, c_int, P, P, c_f32, P, c_i64, P, P, P]),
    'smi_layernorm_backward': (c_int, [P, c_i64, P, c_i64, P, P, P, c_i64, c_int, c_int, P, c_i64,
                                       P, P, P]),
    'smi_diag_gauss': (c_int, [P, P, P, c_i64, c_int, P, P, P, P, P]),
    'smi_mlp_forward': (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, P, c_i64, c_i64,
                                c_int, P, P, P, c_f32, P, P]),
    'smi_ppo_critic_gae': (c_int, [P, c_int, c_int, c_int, c_int, P, P, P, c_f32, P, P, P, P,
                                   c_int, c_int, P, P, c_f32, c_f32, P, P, P, P]),
    'smi_gae_windows': (c_int, [P, P, P, P, c_i64, c_int, c_int, P, P, c_f32, c_f32, P, P, P,
                                P, P]),
    'smi_gae_windows_max_partials': (c_int, [c_i64, c_int]),
    'smi_moments': (c_int, [P, c_i64, P, c_int, P, P]),
    'smi_ppo_update_fused': (c_int, [ctypes.POINTER(PPOArgs), P]),
    'smi_ppo_xbuf_floats': (c_i64, [c_int] * 7),
    'smi_ppo_epoch_grad': (c_int, [ctypes.POINTER(PPOArgs), c_int, P]),
    'smi_ppo_epoch_apply': (c_int, [ctypes.POINTER(PPOArgs), c_int, P]),
    'smi_zfilter_accumulate': (c_int, [P, P, c_int, c_f32, P, P, P, P]),
    'smi_adam_clip': (c_int, [P, P, P, P, c_i64, P, P, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32,
                              P, P, P]),
    'smi_linear_forward': (c_int, [P, c_i64, c_int, c_int, P, c_i64, P, c_int, c_int, P, c_i64, P]),
    'smi_linear_forward_cat': (c_int, [P, c_i64, c_int, c_int, P, c_i64, P, c_int, c_int, P, c_i64,
                                       P, c_i64, c_int, P]),
    'smi_linear_backward_input': (c_int, [P, c_i64, c_int, c_int, P, c_i64, c_int, P, c_i64, P,
                                          c_i64, P]),
    'smi_linear_backward_weight': (c_int, [P, c_i64, c_int, c_int, P, c_i64, c_int, P, c_i64, P,
                                           c_int, P]),
    'smi_mse_grad': (c_int, [P, c_i64, P, c_i64, P, P, P]),
    'smi_neg_mean_grad': (c_int, [P, c_i64, c_i64, P, P, P]),
    'smi_tanh_backward': (c_int, [P, c_i64, P, c_i64, c_i64, c_int, P, c_i64, P]),
    'smi_copy_cols': (c_int, [P, c_i64, c_i64, c_int, P, c_i64, P]),
    'smi_mlp3_forward_stacked': (c_int, [P, c_i64, P, c_int, c_int, c_int, c_int, c_int, P, c_i64,
                                         c_int, P, c_i64, P]),
    'smi_copy_to_host': (c_int, [P, P, c_i64, P]),
    'smi_copy_gather': (c_int, [P, P, P, P, c_int, P]),
    'smi_head_forward': (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, c_i64, c_i64, P, P, P, P,
                                 P]),
    'smi_head_backward_input': (c_int, [P, c_int, c_int, c_int, c_int, P, P, c_i64, P, P, P, P,
                                        c_int, c_int, P, c_i64, P, c_i64, P]),
    'smi_soft_update': (c_int, [P, P, c_i64, c_f32, P]),
    'smi_ddpg_stats': (c_int, [P, c_i64, c_int, P, c_i64, P, P, c_i64, c_i64, P, P]),
    'smi_ddpg_target': (c_int, [P, P, P, P, c_i64, c_f32, P, P]),
    'smi_mt_seed': (c_int, [ctypes.c_uint64, P]),
    'smi_mt_randint_host': (c_int, [P, c_i64, c_i64, P]),
    'smi_mt_randint': (c_int, [P, c_i64, c_i64, P, P]),
    'smi_gather_rows': (c_int, [P, c_i64, P, c_i64, P, P]),
    'smi_lstm_param_count': (c_i64, [c_int, c_int]),
    'smi_kernel_timing': (c_int, [c_int]),
    'smi_kernel_timing_report': (c_int, [c_int, P]),
    'smi_calib_mfma': (c_int, [c_int, c_int, P, P, P]),
    'smi_calib_stream': (c_int, [P, P, c_i64, P]),
    'smi_clock_probe': (c_int, [P, ctypes.c_longlong, P, P]),
    'smi_clock_probe_stop': (c_int, [P, c_int, P]),
    'smi_ppo_rnn_scratch_bytes': (c_i64, [c_int] * 15),
    'smi_ppo_rnn_xbuf_floats': (c_i64, [c_int] * 12),
    'smi_cnn_param_count': (c_i64, [c_int] * 4),
    'smi_cnn_scratch_bytes': (c_i64, [c_i64] + [c_int] * 4),
    'smi_cnn_forward': (c_int, [P, P, P, c_i64, c_i64, c_i64] + [c_int] * 4 + [P, P, P, c_i64, P]),
    'smi_cnn_backward': (c_int, [P, P, P, c_i64, c_i64, c_i64] + [c_int] * 4 +
                         [P, P, P, c_i64, P, P, c_i64, P]),
    'smi_ppo_rnn_phase': (c_int, [ctypes.POINTER(RNNArgs), c_int, c_int, P]),
    'smi_lstm_forward': (c_int, [P, P, P, P, P, c_int, c_int, c_int, P, P, P, P]),
    'smi_lstm_backward': (c_int, [P, P, P, P, c_int, c_int, c_int, P, P]),
    'smi_lstm_forward_x': (c_int, [P, c_i64, c_int, P, P, P, P, P, P, c_int, c_int, c_int,
                                   P, P, P, P, P]),
}

_lib = None


def lib():
    """Load the library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError('libsurreal_mi.so not built: run `python -c "import __graft_entry__ as '
                               'g; g.build()"` (no CPU fallback exists)')
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def check(rc, name):
    if rc != 0:
        msg = lib().smi_last_error().decode(errors='replace')
        raise RuntimeError(f'{name} failed (rc={rc}): {msg}')


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    check(rc, name)
    return rc


def ptr(t):
    """Device pointer of a CUDA(HIP) tensor, or None."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError('surreal_amd kernels take device (HIP) tensors; got a CPU tensor '
                           '(there is no CPU fallback)')
    return ctypes.c_void_p(t.data_ptr())


def stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_workspaces = {}


def ensure_workspace(device):
    """Allocate and register the reduction workspace once per device."""
    dev = torch.device(device)
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _workspaces:
        nbytes = lib().smi_workspace_bytes()
        ws = torch.zeros(nbytes // 4, dtype=torch.float32, device=dev)
        _workspaces[key] = ws
        check(lib().smi_set_workspace(ctypes.c_void_p(ws.data_ptr()), nbytes), 'smi_set_workspace')
    return _workspaces[key]


_ctx_tls = threading.local()


class Context(object):
    """An smi_context (include/surreal_mi.h, re-entrancy): its own device
    workspace for the split-K / reduction partials of the launches its owner
    enqueues.  Every object that launches work (learner, agent batch) owns
    one and calls make_current() before its library calls, so objects on
    different streams or threads never share partial buffers."""

    def __init__(self, device):
        self.device = torch.device(device)
        nbytes = lib().smi_workspace_bytes()
        self.ws = torch.zeros(nbytes // 4, dtype=torch.float32, device=self.device)
        self.handle = lib().smi_context_create(ctypes.c_void_p(self.ws.data_ptr()), nbytes)
        if not self.handle:
            check(-1, 'smi_context_create')

    def make_current(self):
        check(lib().smi_context_make_current(ctypes.c_void_p(self.handle)), 'smi_context_make_current')
        # the thread keeps the context (and so its workspace) alive for as long
        # as it is this thread's current one: a launch the thread issues after
        # the owner dropped its reference still has live partial buffers
        _ctx_tls.current = self

    def __del__(self):
        # no make_current(None) here: the collector may run this on any thread
        # in the middle of another object's launches; smi_context_destroy
        # clears only this thread's current context if it is this one, and a
        # thread still holding it falls back to the default workspace
        h, self.handle = getattr(self, 'handle', None), None
        if h and _lib is not None:
            _lib.smi_context_destroy(ctypes.c_void_p(h))


@contextlib.contextmanager
def gc_paused():
    """Python's cyclic collector off while a hipGraph is captured: a
    collection inside the capture runs __del__ of unreachable objects that hold
    HIP resources from earlier work (events, graph execs), whose destroy calls
    are not allowed during stream capture and abort the process (seen once in
    the pixel graph-replay test).  torch.cuda.graph collects on entry; this
    keeps the collector from running again until the capture has ended."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError('surreal_amd requires an AMD GPU (HIP); none is visible and there is '
                           'no CPU fallback')
