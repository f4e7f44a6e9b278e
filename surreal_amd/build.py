"""Builds libsurreal_mi.so (gfx950) in-tree from surreal_amd/csrc/*.hip.

Objects are compiled with hipcc for --offload-arch=gfx950 and linked against
the HIP runtime that ships inside torch (same SONAME libamdhip64.so.7), with a
RUNPATH to it, so a process that imports torch ends up with ONE HIP runtime
whichever library is loaded first.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
ROOT = os.path.dirname(HERE)
BUILD = os.path.join(ROOT, 'build', 'obj')
LIB = os.path.join(HERE, 'libsurreal_mi.so')
SOURCES = ['ppo_gae.hip', 'ppo_epochs.hip', 'ops_kernels.hip', 'sampler_kernels.hip',
           'linear_kernels.hip', 'ddpg_kernels.hip', 'lstm_kernels.hip', 'cnn_kernels.hip', 'head_kernels.hip', 'ppo_rnn.hip', 'calib_kernels.hip', 'capi.hip']
HEADERS = ['smi_device.hpp', 'smi_internal.hpp', 'lstm_cell.hpp', 'pol_rows.hpp']
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'
CXXFLAGS = ['-O3', '-fPIC', '-std=c++17', f'--offload-arch={ARCH}', '-mcode-object-version=5',
            '-Wall', '-Wno-unused-function']
# Compilation units: (object, source, extra flags).  lstm_kernels.hip is
# compiled twice: the MFMA forms + launchers, and the VALU recurrence with
# -fno-slp-vectorize (its fmaf chains stay scalar v_fmac_f32: the SLP
# vectorizer packs them into v_pk_fma_f32 + operand moves; measured at 128
# segments, one MI355X: lstm_fwd 43.0 -> 40.9 us, lstm_bwd 34.5 -> 27.0 us per
# launch, learn 3.48 -> 3.29 ms; the flag on the MFMA forms changed their
# rounding)
UNITS = [(s.replace('.hip', '.o'), s, []) for s in SOURCES if s != 'lstm_kernels.hip'] + [
    ('lstm_kernels.o', 'lstm_kernels.hip', ['-DSMI_LSTM_PART=1']),
    ('lstm_valu.o', 'lstm_kernels.hip', ['-DSMI_LSTM_PART=2', '-fno-slp-vectorize'])]


def torch_lib_dir():
    import torch
    return os.path.join(os.path.dirname(torch.__file__), 'lib')


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


# Developer variants: 'prof' adds the epoch-kernel phase timer (-DSMI_PROF,
# tools/fused_breakdown.py --phases); 'noinl' keeps the dense helpers out of line.  The product library is variant None.
VARIANTS = {None: [], 'prof': ['-DSMI_PROF'], 'noinl': ['-DSMI_DENSE_NOINLINE'],
            'noinl_prof': ['-DSMI_DENSE_NOINLINE', '-DSMI_PROF'],
            # dW-kernel experiments (tools/dwd_exp.sh)
            'p8': ['-DSMI_DWD_P=8'], 'p6': ['-DSMI_DWD_P=6'], 'occ1': ['-DSMI_DWD_OCC=1'],
            # LSTM activation A/B (the pre-round-2 cancelling tanh)
            'oldtanh': ['-DSMI_OLD_TANH'],
            # dW: the checked loop everywhere (A/B of the unchecked full-slab loop)
            'nofast': ['-DSMI_DWD_FAST=0'],
            # fused-head weight ring depth A/B (product: 2)
            'hcd3': ['-DSMI_HC_DEPTH=3'], 'hcd4': ['-DSMI_HC_DEPTH=4'],
            # grouped dW tile A/B: 64 x 128 tiles at 2 waves per SIMD (round 2)
            'dwg8': ['-DSMI_DWG_NT=8'], 'dwgocc4': ['-DSMI_DWG_OCC=4'], 'dwgocc2': ['-DSMI_DWG_OCC=2'],   # (occupancy 4: 122 us)
            # VALU recurrence: LDS reads per pipelined chunk (product: 4)
            'vc2': ['-DSMI_LSTM_VC=2'], 'vc8': ['-DSMI_LSTM_VC=8'],
            # VALU recurrence dot products on v_pk_fma_f32 (product: scalar FMAs)
            'pk': ['-DSMI_LSTM_PK=1'],
            # grouped-dW anatomy (tools/bench_dwgroup.py only; wrong results by design):
            # MFMAs without the operand stream / the stream without the MFMAs
            'dwdiag_mfma': ['-DSMI_DWD_DIAG=1'], 'dwdiag_load': ['-DSMI_DWD_DIAG=2'],
            # per-workgroup start / end clock of the grouped dW launch (product results)
            'dwtrace': ['-DSMI_DWD_DIAG=3'], 'dwtrace_mfma': ['-DSMI_DWD_DIAG=1', '-DSMI_DWD_TRACE=1'],
            # test-only fault injection (tests/negative_controls.py): the parity
            # checks must FAIL on this build's deliberate departures
            'fault': ['-DSMI_FAULT_INJECTION'],
            # round 6 A/B: the BPTT's recurrent dot product in the round-5 two
            # FMA chains (product: four; 128 segments 2.919 -> 2.908 ms)
            'ch2': ['-DSMI_BPTT_CH4=0']}


def lib_path(variant=None):
    return LIB if variant is None else LIB.replace('.so', f'_{variant}.so')


def build(verbose=False, force=False, variant=None):
    build_dir = BUILD if variant is None else f'{BUILD}_{variant}'
    lib = lib_path(variant)
    os.makedirs(build_dir, exist_ok=True)
    deps = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, 'include', 'surreal_mi.h')]
    dep_t = max(_mtime(d) for d in deps)
    objs, cmds = [], []
    for obj, src, extra in UNITS:
        sp = os.path.join(CSRC, src)
        op = os.path.join(build_dir, obj)
        objs.append(op)
        if force or _mtime(op) < max(_mtime(sp), dep_t, _mtime(__file__)):
            cmds.append([HIPCC] + CXXFLAGS + extra + VARIANTS[variant] + ['-c', sp, '-o', op])
    # one hipcc per source, run side by side (each is single-threaded)
    from concurrent.futures import ThreadPoolExecutor
    jobs = max(1, min(len(cmds), int(os.environ.get('MAX_JOBS', os.cpu_count() or 1))))

    def run(cmd):
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(run, cmds))
    if force or _mtime(lib) < max(_mtime(o) for o in objs):
        tl = torch_lib_dir()
        cmd = ['g++', '-shared', '-o', lib] + objs + [
            f'-L{tl}', '-l:libamdhip64.so', f'-Wl,-rpath,{tl}', '-Wl,--no-undefined', '-lstdc++']
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return lib


if __name__ == '__main__':
    var = next((a.split('=', 1)[1] for a in sys.argv if a.startswith('--variant=')), None)
    build(verbose=True, force='--force' in sys.argv, variant=var)
