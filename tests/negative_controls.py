"""Negative controls of the pinned parity checks (test infrastructure only).

Run as its own process with SMI_LIB_VARIANT=fault, i.e. on the test-only
build of the library (surreal_amd/build.py variant 'fault', -DSMI_FAULT_INJECTION)
whose smi_fault_set(mode) selects a deliberate departure from the reference:

  1 critic Adam skipped           (ppo.py:348-352 never applied)
  2 stems left out of the critic optimizer (ppo_net.py:202-224: the LSTM / CNN
                                   stem is in BOTH optimizers)
  3 one policy epoch fewer        (ppo.py:541-557: the last epoch's update skipped)
  4 GAE horizon off by one        (ppo.py:389-406: windows of H - 1 steps)

For every (case, fault) the fixture case is learned on the GPU and checked
exactly as tests/test_gpu_parity_pinned.py checks it (envelope, update
measures), and the checks the fault must trip are named: a control passes
when ALL of them fail.  Mode 0 on the same build is the positive control:
every check passes, so the failures come from the faults, not the build.

Usage: SMI_LIB_VARIANT=fault python tests/negative_controls.py OUT.json
Writes {case: {fault: {"failed": [...], "expected": [...], "ok": bool}}}.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FAULTS = {0: 'none', 1: 'critic_adam_skip', 2: 'critic_stem_omit', 3: 'policy_epoch_short',
          4: 'gae_horizon_off_by_one'}

# the checks each fault must fail (all of them), per case
EXPECT = {
    'c3_clip': {1: ['upd_relL2:critic@0', 'upd_1-cos:critic@0'],
                2: ['upd_relL2:lstm@0'],
                3: ['upd_relL2:actor@0'],
                4: ['adv@0', 'ret@0']},
    'c5': {1: ['upd_relL2:critic@0', 'upd_1-cos:critic@0'],
           2: ['upd_relL2:lstm@0', 'upd_relL2:cnn@0']},
}


def run_case(case, mode):
    import numpy as np
    from surreal_amd import _lib as L
    from surreal_amd import synthetic
    from tests import parity as P
    from tests.test_gpu_parity_pinned import _used, check_fixture_state, fixture_learner
    L.check(L.lib().smi_fault_set(mode), 'smi_fault_set')
    meta, fx, c, st, learner = fixture_learner(case)
    report = {}
    for it in range(len(c['batch_seeds'])):
        batch = P.case_batch(case, it)
        assert P.batch_digest(batch) == meta['batch_digest'][it]
        learner.learn(synthetic.to_device(batch, 'cuda:0'))
        m = learner.model
        fin = {'actor': m.actor.flat.cpu(), 'critic': m.critic.flat.cpu()}
        if learner.if_rnn_policy:
            fin['lstm'] = m.rnn_stem.flat.cpu()
        if learner.if_pixel_input:
            fin['cnn'] = m.cnn_stem.flat.cpu()
        zf = tuple(getattr(m.z_filter, b).cpu() for b in ('running_sum', 'running_sumsq'))
        adv, ret = _used(learner)
        check_fixture_state(meta, fx, st, it, fin, np.asarray(adv), np.asarray(ret), zf, report)
    L.check(L.lib().smi_fault_set(0), 'smi_fault_set')
    return report


def main(out):
    import ctypes
    import torch
    from surreal_amd import _lib as L
    assert os.environ.get('SMI_LIB_VARIANT') == 'fault', 'run on the fault-injection build'
    torch.cuda.set_device(0)
    L.lib().smi_fault_set.argtypes = [ctypes.c_int]
    L.lib().smi_fault_set.restype = ctypes.c_int
    res = {}
    for case, faults in EXPECT.items():
        res[case] = {}
        for mode in [0] + sorted(faults):
            rep = run_case(case, mode)
            failed = sorted(rep.get('_fail', []))
            exp = faults.get(mode, [])
            ok = (not failed) if mode == 0 else all(e in failed for e in exp)
            res[case][FAULTS[mode]] = {'failed': failed, 'expected': exp, 'ok': ok,
                                       'report': {k: rep[k] for k in exp} if mode else {}}
            print(f'{case} {FAULTS[mode]:24s} {"ok" if ok else "NOT CAUGHT"}: '
                  f'{len(failed)} checks failed {failed[:6]}', flush=True)
    with open(out, 'w') as f:
        json.dump(res, f, indent=1, sort_keys=True, default=float)


if __name__ == '__main__':
    main(sys.argv[1])
