"""learn()'s epilogue (ppo.py:606-613, ddpg.py:371-376): periodic checkpoints and
throttled metrics, on the CPU.

PPOLearner._learn_epilogue -- the product code every learn() ends with -- runs
here on a learner shell (no GPU: the statistics vector is a host tensor), with
a fake clock.  Host reads of the statistics happen only inside _stats_dict, so
counting its calls counts the device reads a real learner would do."""
import pytest
import torch

from surreal_amd import _lib as L
from surreal_amd.learner import LinearWithMinLR, PPOLearner
from surreal_amd.session import PeriodicCheckpoint, TimeThrottledMetrics


class Clock(object):
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def shell(metrics=None, checkpoint=None, mode='adapt'):
    ln = object.__new__(PPOLearner)
    ln._init_hooks(metrics, checkpoint)
    ln.stats_buf = torch.zeros(L.ST_COUNT)
    ln.ppo_mode = mode
    ln.beta, ln.clip_epsilon = 1.0, 0.2
    ln.clip_actor_gradient = ln.clip_critic_gradient = True
    ln.use_z_filter = ln.use_r_filter = False
    ln.actor_lr_scheduler = LinearWithMinLR(3e-4, 10, 1, 3e-4)
    ln.batch_size, ln.dp = 8, None
    ln.exp_counter = ln.global_step = ln.current_iteration = 0
    reads = []
    real = PPOLearner._stats_dict

    def counted(v, host):
        reads.append(ln.current_iteration)
        return real(ln, v, host)
    ln._stats_dict = counted
    return ln, reads


def learn_once(ln, value):
    """what learn() does after its device phases: the statistics vector holds
    this call's values, then the epilogue runs"""
    ln.current_iteration += 1
    ln.stats_buf.fill_(float(value))
    PPOLearner._learn_epilogue(ln)


def test_periodic_checkpoint_every_period_calls():
    clock = Clock()
    saved = []
    ck = PeriodicCheckpoint(lambda **kw: saved.append(kw), period=3, clock=clock)
    ln, _ = shell(checkpoint=ck)
    for i in range(10):
        clock.t += 1.0
        learn_once(ln, i)
    assert [s['global_steps'] for s in saved] == [3, 6, 9]
    assert all(s['score'] is None for s in saved)
    assert ln.global_step == 10 and ln.exp_counter == 80


def test_periodic_checkpoint_min_interval():
    # utils/checkpoint.py:341-347: a period boundary saves only if min_interval
    # passed since the last save (time.time() difference)
    clock = Clock()
    saved = []
    ck = PeriodicCheckpoint(lambda **kw: saved.append(kw['global_steps']), period=2,
                            min_interval=5.0, clock=clock)
    ln, _ = shell(checkpoint=ck)
    for i in range(12):
        clock.t += 1.0
        learn_once(ln, i)
    # boundaries at 2, 4, ..., 12 (t = 1002, 1004, ...); the first save needs
    # t - 1000 >= 5 (call 6), then 5 s more each time (call 12)
    assert saved == [6, 12]


def test_checkpoint_callable_and_none():
    got = []
    ln, _ = shell(checkpoint=lambda global_steps, score: got.append(global_steps) or True)
    learn_once(ln, 0)
    learn_once(ln, 0)
    assert got == [1, 2]
    ln, _ = shell()
    assert ln.periodic_checkpoint(global_steps=1) is False


def test_throttled_metrics_read_only_when_due_and_average():
    clock = Clock()
    out = []
    sink = TimeThrottledMetrics(lambda stats, step: out.append((step, stats)), 4.0, clock=clock)
    ln, reads = shell(metrics=sink)
    for i in range(10):
        clock.t += 1.0
        learn_once(ln, i)
    # due at t = 1004 (call 4, value 3) and t = 1008 (call 8, value 7)
    assert [s for s, _ in out] == [3, 7]          # global_step before the increment
    assert reads == [4, 8], reads                  # no statistics read on the other calls
    # AverageValue (utils/common.py:606-630): the first window averages 0..3;
    # avg(clear=True) restarts from the last value with count 1, so the second
    # window averages 3..7, not 4..7
    assert out[0][1]['_surr_loss'] == pytest.approx(1.5)
    assert out[1][1]['_surr_loss'] == pytest.approx(5.0)
    assert out[0][1]['_beta'] == 1.0 and out[0][1]['_lr'] == pytest.approx(3e-4)
    assert sink.emitted == 2


def test_plain_metrics_callable_gets_every_call():
    out = []
    ln, reads = shell(metrics=lambda stats, step: out.append((step, stats['_val_loss'])),
                      mode='clip')
    for i in range(3):
        learn_once(ln, i)
    assert out == [(0, 0.0), (1, 1.0), (2, 2.0)]
    assert reads == [1, 2, 3]


def test_throttled_metrics_average_zfilter_entries():
    """obs_running_* (ppo.py:578-582) go through the same AverageValue as the
    other scalars: averaged over the window from device-side means, not read
    at the emit's current state"""
    import numpy as np
    clock = Clock()
    out = []
    sink = TimeThrottledMetrics(lambda stats, step: out.append(stats), 2.0, clock=clock)
    ln, _ = shell(metrics=sink)
    ln.use_z_filter = True

    class ZF(object):
        pass
    zf = ZF()
    zf.count = torch.tensor(1.0)
    ln.model = ZF()
    ln.model.z_filter = zf
    means = []
    for i in range(4):
        clock.t += 1.0
        zf.running_sum = torch.tensor([float(i), float(i) + 2.0])
        zf.running_sumsq = torch.tensor([float(i * i) + 1.0, (float(i) + 2.0) ** 2 + 4.0])
        means.append(np.mean([i, i + 2.0]))
        learn_once(ln, i)
    # emits at calls 2 and 4: windows {0, 1} and {1, 2, 3}
    assert out[0]['obs_running_mean'] == pytest.approx(np.mean(means[0:2]))
    assert out[1]['obs_running_mean'] == pytest.approx(np.mean(means[1:4]))
    assert out[1]['obs_running_std'] == pytest.approx(1.5)     # mean(sqrt(1), sqrt(4))
