"""Negative controls: the pinned parity checks must FAIL on deliberately faulty
learners (tests/negative_controls.py, run on the test-only fault-injection
build of the library in a child process: one library per process).

Faults: critic Adam skipped, stems left out of the critic optimizer, one
policy epoch fewer, GAE horizon off by one (c3_clip), and the first two at C5
(pixels: the CNN stem is in the critic optimizer too).  The same build with no
fault selected passes every check."""
import json
import os
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_parity_checks_catch_injected_faults():
    lib = os.path.join(ROOT, 'surreal_amd', 'libsurreal_mi_fault.so')
    if not os.path.exists(lib):
        pytest.fail('the fault-injection build is missing: python -m surreal_amd.build --variant=fault')
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, 'nc.json')
        env = dict(os.environ, SMI_LIB_VARIANT='fault')
        env.pop('SMI_PARITY_REPORT', None)
        r = subprocess.run([sys.executable, '-u', os.path.join(ROOT, 'tests', 'negative_controls.py'), out],
                           env=env, cwd=ROOT, timeout=540, capture_output=True, text=True)
        print(r.stdout[-4000:], r.stderr[-4000:])
        assert r.returncode == 0, r.stderr[-2000:]
        with open(out) as f:
            res = json.load(f)
    path = os.environ.get('SMI_PARITY_REPORT')
    if path:
        d = {}
        if os.path.exists(path):
            with open(path) as f:
                d = json.load(f)
        d['negative_controls'] = res
        with open(path, 'w') as f:
            json.dump(d, f, indent=1, sort_keys=True)
    bad = [(case, fault) for case, fs in res.items() for fault, v in fs.items() if not v['ok']]
    assert not bad, bad
    assert all(len(fs) >= 3 for fs in res.values())
