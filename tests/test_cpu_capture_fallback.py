"""PPOLearner._learn_graphed's capture path on the CPU (no GPU): the hipGraph
capture of a data-parallel learn() may be refused by the collective library on
one rank.  Every rank must then take the same (eager) path -- one flag is
all-reduced once per capture -- and the call's update, counters and epilogue
must still happen exactly once.  torch.cuda's graph API is replaced by fakes;
the device phases are a generator that counts the updates it runs."""
import contextlib

import pytest
import torch

from surreal_amd import learner as learner_mod
from surreal_amd.learner import PPOLearner


class FakeDP(object):
    """a 2-rank group whose peer reports `peer_fail` at the capture vote"""

    def __init__(self, peer_fail=False):
        self.world_size = 2
        self.capturable = True
        self.peer_fail = peer_fail
        self.calls = 0

    def allreduce_(self, t):
        self.calls += 1
        if t.numel() == 1:                      # the capture vote
            t.add_(1.0 if self.peer_fail else 0.0)
        else:
            t.mul_(2.0)


class FakeGraph(object):
    def __init__(self):
        self.replays = 0

    def replay(self):
        self.replays += 1


def shell(dp):
    ln = object.__new__(PPOLearner)
    ln._init_hooks(None, None)
    ln.use_graph, ln.kernel_events = True, None
    ln._graph = ln._graph_key = None
    ln.export_advantages = ln.prep_side_stream = False
    ln.epoch_policy = ln.epoch_baseline = 10
    ln.current_iteration = ln.global_step = ln.exp_counter = 0
    ln.batch_size = 8
    ln.dp = dp
    ln.publisher = None
    ln.device = torch.device('cpu')
    ln.updates = 0

    class Ctx(object):
        def make_current(self):
            pass
    ln._ctx = Ctx()
    ln._hyper_values = lambda: 1
    ln._hyper_key = 1

    def phases(batch):
        ln.updates += 1
        yield torch.zeros(4)
    ln._device_phases = phases
    return ln


@pytest.fixture
def fake_cuda(monkeypatch):
    state = {'refuse': False}

    @contextlib.contextmanager
    def graph(g, capture_error_mode=None):
        if state['refuse']:
            raise RuntimeError('capture refused by the collective library')
        yield g
    monkeypatch.setattr(torch.cuda, 'graph', graph)
    monkeypatch.setattr(torch.cuda, 'CUDAGraph', FakeGraph)
    monkeypatch.setattr(torch.cuda, 'synchronize', lambda *a, **k: None)

    def refresh(self, leaves):                   # the copy-gather launch, on the CPU
        for v, t in zip(self.views, leaves):
            if v.data_ptr() != t.data_ptr():
                v.copy_(t)
    monkeypatch.setattr(learner_mod._GraphInputs, 'refresh', refresh)
    return state


def _batch():
    # CPU tensors: _learn_graphed passes them through the arena stub below
    return {'actions': torch.zeros(8, 3), 'rewards': torch.zeros(8, 3)}


def _learn(ln):
    class Arena(object):
        def stage(self, b):
            return b
    ln._arena = Arena()
    ln._learn_graphed(_batch())


@pytest.mark.parametrize('local_refuse,peer_fail', [(True, False), (False, True), (True, True)])
def test_capture_refused_anywhere_all_ranks_eager(fake_cuda, local_refuse, peer_fail):
    fake_cuda['refuse'] = local_refuse
    dp = FakeDP(peer_fail=peer_fail)
    ln = shell(dp)
    with pytest.warns(UserWarning, match='could not be captured'):
        _learn(ln)
    # the eager pass ran once (its update kept), the capture was dropped
    assert ln.updates == 1 + (0 if local_refuse else 1)   # the capture pass runs the generator too
    assert ln.use_graph is False and ln._graph is None
    assert ln.current_iteration == 1 and ln.global_step == 1
    assert ln.exp_counter == 8 * 2
    # one eager exchange of the call, [the captured one,] then the vote
    assert dp.calls == 1 + (0 if local_refuse else 1) + 1


def test_capture_agreed_keeps_graph(fake_cuda):
    dp = FakeDP(peer_fail=False)
    ln = shell(dp)
    _learn(ln)
    assert ln.use_graph is True and isinstance(ln._graph, FakeGraph)
    assert ln.global_step == 1 and ln.exp_counter == 16
    _learn(ln)                                   # same shapes: a replay
    assert ln._graph.replays == 1 and ln.global_step == 2 and ln.exp_counter == 32
    assert ln.updates == 2                       # eager + capture pass; the replay runs no host phases


def test_single_rank_capture_error_propagates(fake_cuda):
    fake_cuda['refuse'] = True
    ln = shell(None)
    with pytest.raises(RuntimeError, match='capture refused'):
        _learn(ln)
