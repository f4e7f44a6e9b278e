"""CPU tests of the C-ABI library surface and the host-side logic (no compute
calls on a device)."""
import os
import random
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(ROOT, 'include', 'surreal_mi.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(smi_[a-z0-9_]+)\s*\(', src)))


def test_library_exports_every_header_symbol():
    from surreal_amd import _lib
    lib = _lib.lib()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) <= set(_lib.exported_symbols()) | {'smi_version', 'smi_last_error'}


def test_struct_layout_matches_header():
    import ctypes
    from surreal_amd import _lib
    # field order of struct smi_ppo_args as declared in the header
    src = open(os.path.join(ROOT, 'include', 'surreal_mi.h')).read()
    body = src[src.index('typedef struct smi_ppo_args {'):src.index('} smi_ppo_args;')]
    body = re.sub(r'/\*.*?\*/', '', body, flags=re.S)
    names = []
    for decl in body.split(';')[:-1]:
        decl = decl.split('{')[-1]
        for part in decl.split(','):
            nm = re.findall(r'([A-Za-z_][A-Za-z0-9_]*)\s*$', part.strip())
            if nm:
                names.append(nm[0])
    assert names == [f[0] for f in _lib.PPOArgs._fields_]
    assert ctypes.sizeof(_lib.PPOArgs) % 8 == 0


def test_error_path_reports_message():
    from surreal_amd import _lib
    lib = _lib.lib()
    rc = lib.smi_gather_rows(None, 4, None, 1, None, None)
    assert rc == -1 and b'gather_rows' in lib.smi_last_error()
    with pytest.raises(RuntimeError):
        _lib.check(rc, 'smi_gather_rows')


def test_host_sampler_matches_cpython():
    from surreal_amd import _lib
    lib = _lib.lib()
    for seed, n in ((0, 333333), (7, 3), (2 ** 33 + 1, 1000)):
        st = np.zeros(625, dtype=np.uint32)
        assert lib.smi_mt_seed(seed, st.ctypes.data) == 0
        out = np.zeros(1300, dtype=np.int64)
        assert lib.smi_mt_randint_host(st.ctypes.data, n, 1300, out.ctypes.data) == 0
        random.seed(seed)
        assert out.tolist() == [random.randint(0, n - 1) for _ in range(1300)]
        assert list(st[:624]) == list(random.getstate()[1][:624])
        assert int(st[624]) == random.getstate()[1][624]


def test_layout_queries():
    from surreal_amd import _lib
    from surreal_amd.model import mlp_param_count
    lib = _lib.lib()
    assert lib.smi_mlp_param_count(17, 64, 64, 6, 1) == mlp_param_count(17, 64, 64, 6, True) == 5708
    assert lib.smi_ppo_fused_lds_bytes(64, 17, 64, 64, 6, 64, 64) <= 160 * 1024
    assert lib.smi_ppo_fused_lds_bytes(64, 100, 300, 200, 8, 300, 200) > 160 * 1024


def test_config_extend_and_attribute_access():
    from surreal_amd.config import PPO_DEFAULT_LEARNER_CONFIG, Config
    c = Config({'algo': {'gamma': 0.5}})
    c.extend(PPO_DEFAULT_LEARNER_CONFIG)
    assert c.algo.gamma == 0.5
    assert c.algo.consts.epoch_policy == 10
    assert c.replay.batch_size == 64
    c.algo.n_step = 7
    assert c['algo']['n_step'] == 7


def test_linear_with_min_lr_schedule():
    from surreal_amd.learner import LinearWithMinLR
    s = LinearWithMinLR(1e-3, 100, update_freq=10, min_lr=1e-4)
    assert s.get_lr()[0] == pytest.approx(1e-3)
    for _ in range(50):
        s.step()
    assert s.get_lr()[0] == pytest.approx(1e-3 - 0.5 * 9e-4)
    for _ in range(500):
        s.step()
    assert s.get_lr()[0] == pytest.approx(1e-4)
    c = LinearWithMinLR(1e-4, 100, 10, 1e-4)
    for _ in range(30):
        c.step()
    assert c.get_lr()[0] == pytest.approx(1e-4)


def _exp(T, D, A, rng, with_h=False):
    return {
        'obs': [{'low_dim': {'flat_inputs': rng.randn(D).astype(np.float32)}} for _ in range(T)],
        'obs_next': {'low_dim': {'flat_inputs': rng.randn(D).astype(np.float32)}},
        'actions': [rng.randn(A).astype(np.float32) for _ in range(T)],
        'rewards': list(rng.randn(T)),
        'dones': [False] * (T - 1) + [True],
        'persistent_infos': [[rng.randn(2 * A).astype(np.float32)] for _ in range(T)],
        'onetime_infos': [rng.randn(1, 5), rng.randn(1, 5)] if with_h else [],
    }


def test_multistep_aggregator_shapes():
    from surreal_amd.aggregator import MultistepAggregatorWithInfo
    rng = np.random.RandomState(0)
    spec = {'low_dim': {'flat_inputs': (4,)}}
    agg = MultistepAggregatorWithInfo(spec, {'dim': (3,), 'type': 'continuous'})
    exps = [_exp(5, 4, 3, rng, with_h=True) for _ in range(7)]
    out = agg.aggregate(exps)
    assert out['obs']['low_dim']['flat_inputs'].shape == (7, 5, 4)
    assert out['obs_next']['low_dim']['flat_inputs'].shape == (7, 1, 4)
    assert out['actions'].shape == (7, 5, 3)
    assert out['rewards'].shape == (7, 5)
    assert out['dones'].dtype == np.float32 and out['dones'][:, -1].all()
    assert out['persistent_infos'][0].shape == (7, 5, 6)
    assert out['onetime_infos'][0].shape == (7, 1, 5)
    assert np.array_equal(out['actions'][2, 3], exps[2]['actions'][3])


def test_ssar_aggregator_and_framestack():
    from surreal_amd.aggregator import FrameStackPreprocessor, SSARAggregator
    rng = np.random.RandomState(1)
    exps = []
    for _ in range(6):
        o0 = {'low_dim': {'flat_inputs': rng.randn(4)}, 'pixel': {'camera0': [rng.rand(1, 3, 3)] * 2}}
        o1 = {'low_dim': {'flat_inputs': rng.randn(4)}, 'pixel': {'camera0': [rng.rand(1, 3, 3)] * 2}}
        exps.append({'obs': [o0, o1], 'action': rng.randn(2), 'reward': 1.0, 'done': False})
    exps = FrameStackPreprocessor(2).preprocess_list(exps)
    out = SSARAggregator({}, {'dim': (2,), 'type': 'continuous'}).aggregate(exps)
    assert out['obs']['pixel']['camera0'].shape == (6, 2, 3, 3)
    assert out['rewards'].shape == (6, 1) and out['dones'].shape == (6, 1)
    assert out['actions'].dtype == np.float32


def test_fifo_replay_order():
    from surreal_amd.config import PPO_DEFAULT_LEARNER_CONFIG
    from surreal_amd.replay import FIFOReplay
    r = FIFOReplay(PPO_DEFAULT_LEARNER_CONFIG)
    for i in range(70):
        r.insert(i)
    assert r.start_sample_condition()
    assert r.sample(64) == list(range(64))
    assert len(r) == 6


def test_product_has_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU visible')
    from surreal_amd.learner import PPOLearner
    from tests.helpers import env_config, ppo_config
    with pytest.raises(RuntimeError):
        PPOLearner(ppo_config(), env_config())


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, 'surreal_amd')
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith('.py'):
                src = open(os.path.join(dp, f)).read()
                assert 'oracle' not in re.findall(r'^\s*(?:from|import)\s+(\w+)', src, re.M), f


def test_binary_hash_matches_reference_serializer():
    """surreal/utils/serializer.py:55-66: the first 16 base64 characters of
    the md5 digest, '/' kept (the replace at :65 is commented out)."""
    from surreal_amd.publish import binary_hash
    assert binary_hash(b'payload3') == '1RTGU+Gd/jOICPXV'
    assert len(binary_hash(b'')) == 16


def test_context_lifecycle_without_device_work():
    """smi_context (include/surreal_mi.h, re-entrancy): create / make current /
    destroy are host-only; bad arguments are refused with a message."""
    import ctypes
    from surreal_amd import _lib
    lib = _lib.lib()
    assert not lib.smi_context_create(None, 1024)
    assert b'context_create' in lib.smi_last_error()
    fake = ctypes.c_void_p(0x1000)            # never dereferenced: no launch is made
    h = lib.smi_context_create(fake, 1 << 20)
    assert h
    assert lib.smi_context_make_current(ctypes.c_void_p(h)) == 0
    assert lib.smi_context_make_current(None) == 0
    assert lib.smi_context_destroy(ctypes.c_void_p(h)) == 0
    assert lib.smi_context_destroy(None) == -1
    # a destroyed context cannot be made current again; one still current on
    # this thread is cleared (the thread falls back to the default workspace)
    h2 = lib.smi_context_create(fake, 1 << 20)
    assert lib.smi_context_make_current(ctypes.c_void_p(h2)) == 0
    assert lib.smi_context_destroy(ctypes.c_void_p(h2)) == 0
    assert lib.smi_context_make_current(ctypes.c_void_p(h2)) != 0
    assert b'destroyed' in lib.smi_last_error()


def test_fault_injection_only_in_the_test_build():
    """smi_fault_set (tests/negative_controls.py) exists only in the
    fault-injection variant, never in the product library"""
    import subprocess
    prod = os.path.join(ROOT, 'surreal_amd', 'libsurreal_mi.so')
    syms = subprocess.run(['nm', '-D', '--defined-only', prod], capture_output=True, text=True,
                          check=True).stdout
    assert 'smi_fault_set' not in syms and 'fault' not in syms
    var = os.path.join(ROOT, 'surreal_amd', 'libsurreal_mi_fault.so')
    if os.path.exists(var):
        syms = subprocess.run(['nm', '-D', '--defined-only', var], capture_output=True, text=True,
                              check=True).stdout
        assert 'smi_fault_set' in syms
