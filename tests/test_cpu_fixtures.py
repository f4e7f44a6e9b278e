"""The committed envelope fixtures (tests/golden/envelope_<case>.npz, made by
tests/golden/make_envelopes.py) match what the GPU tests regenerate: the
oracle's seeded initial weights and the seeded synthetic batches hash to the
digests recorded at generation time, every tensor has its width and scale,
and the stored truths are finite (tests/parity.py)."""
import numpy as np
import pytest

from tests import parity as P


@pytest.mark.parametrize('case', sorted(P.CASES))
def test_fixture_regenerates(case):
    meta, fx = P.load_fixture(case)
    c = P.CASES[case]
    assert meta['case'] == case
    st = P.init_state(case)
    assert P.digest([st[k] for k in sorted(st)]) == meta['init_digest']
    assert len(meta['batch_digest']) == len(c['batch_seeds']) == len(meta['epochs_run'])
    for it in range(len(c['batch_seeds'])):
        assert P.batch_digest(P.case_batch(case, it)) == meta['batch_digest'][it]
    for k, v in fx.items():
        assert k in meta['width'] and k in meta['scale'], k
        assert np.all(np.isfinite(v)), k
        assert meta['width'][k] >= 0.0 and meta['scale'][k] > 0.0, k
