import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an AMD GPU (MI355X) and libsurreal_mi.so')


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason='no GPU visible')
    for it in items:
        if 'gpu' in it.keywords:
            it.add_marker(skip)


# Heartbeat: long GPU parity tests (CPU oracles in fp64 at the benched sizes)
# can run minutes between pytest's own output; a line appended every 30 s to
# gpurun_out/pytest_heartbeat.log names the running test, so a run that is
# working is never mistaken for a hung one.
_CURRENT = {'test': None}


def pytest_sessionstart(session):
    import threading
    import time
    path = os.path.join(ROOT, 'gpurun_out', 'pytest_heartbeat.log')

    def beat():
        while True:
            time.sleep(30)
            try:
                os.makedirs(os.path.dirname(path), exist_ok=True)
                with open(path, 'a') as f:
                    f.write(f'{time.strftime("%H:%M:%S")} {_CURRENT["test"]}\n')
            except OSError:
                pass
    threading.Thread(target=beat, daemon=True).start()


def pytest_runtest_logstart(nodeid, location):
    _CURRENT['test'] = nodeid
