"""The learn() epilogue of the reference learners: periodic checkpoints and
throttled metrics, without a device synchronisation on every call.

The reference's PPOLearner.learn / DDPGLearner.learn end with
  self.periodic_checkpoint(global_steps=self.current_iteration, score=None)
      (ppo.py:606-609, ddpg.py:373-376 -> learner/base.py:280-298 ->
       utils/checkpoint.py:317-347: save every `period`-th call, at most once
       per `min_interval`)
  self.tensorplex.add_scalars(stats, global_step)
      (ppo.py:611, ddpg.py:371; session/tracker.py:81-104: a TimeThrottled
       client AVERAGES every call's scalars and forwards the averages when
       `min_update_interval` seconds have passed, utils/common.py:590-648)
Its statistics are Python floats taken by .item() inside _optimize, so the
reference pays a device sync per learn() regardless.  Here the statistics
stay on the device: a throttled sink (anything with a `due()` method, e.g.
TimeThrottledMetrics) gets the device vector accumulated by a stream-ordered
add on every call and read back only when the sink is due; a plain callable
sink keeps the round-1 behaviour (every call's statistics, one read each).
"""
import time

import torch


class PeriodicCheckpoint(object):
    """utils/checkpoint.py:317-347 over a save function: save() runs
    save_fn(global_steps=..., score=..., **info) on every `period`-th call, and
    only if time.time() advanced by `min_interval` since the last save (the
    reference's docstring says minutes; its code compares the time.time()
    difference, i.e. seconds, and so does this).  Returns True when it saved.
    The reference's own PeriodicCheckpoint (which pickles
    checkpoint_attributes()) plugs into the learner the same way: anything
    with this save() signature."""

    def __init__(self, save_fn, period, min_interval=0, clock=time.time):
        if int(period) < 1:
            raise ValueError('period must be >= 1')
        self.save_fn = save_fn
        self.period = int(period)
        self.min_interval = min_interval
        self.clock = clock
        self._period_counter = 0
        self.last_update_time = clock()

    def save(self, score=None, global_steps=None, reload_metadata=False, **info):
        self._period_counter += 1
        if self._period_counter % self.period == 0:
            if self.clock() - self.last_update_time >= self.min_interval:
                self.save_fn(global_steps=global_steps, score=score, **info)
                self.last_update_time = self.clock()
                return True
        return False

    def reset_period(self):
        self._period_counter = 0


class TimeThrottledMetrics(object):
    """session/tracker.py:81-104 as a metrics sink for the learners: the
    learner asks due() once per learn(); when it is, the learner reads the
    statistics averaged over the calls since the last emit and calls
    self(stats, global_step), which forwards them to `sink(stats, step)`
    (e.g. a TensorplexClient's add_scalars).  due() follows TimedTracker
    (utils/common.py:590-602): True when `min_update_interval` seconds passed
    since the last True."""

    def __init__(self, sink, min_update_interval, clock=time.time):
        self.sink = sink
        self.min_update_interval = float(min_update_interval)
        self.clock = clock
        self.last_time = clock()
        self.emitted = 0

    def due(self):
        now = self.clock()
        if now - self.last_time >= self.min_update_interval:
            self.last_time = now
            return True
        return False

    def __call__(self, stats, global_step):
        self.emitted += 1
        if self.sink is not None:
            self.sink(stats, global_step)


class LearnerHooks(object):
    """Mixin of the learners' learn() epilogue.  The host class provides:
      stats_buf            the device statistics vector of the last learn()
      _stats_dict(vector, host_avg)  the reference's stats dict from a host
                           copy of that vector (averaged, for throttled sinks)
                           and the averaged host-side scalars
      _host_scalars()      {name: float} host-side scalars of this call
                           (schedules, adaptive coefficients) to average
    Device work per learn(): none for a plain sink beyond its read; one
    stream-ordered vector add for a throttled sink (no synchronisation)."""

    def _init_hooks(self, metrics=None, checkpoint=None):
        self.metrics = metrics
        self.checkpoint = checkpoint
        self._stats_acc = None
        self._stats_n = 0
        self._host_acc = {}

    # ---------------------------------------------------------- checkpoint
    def periodic_checkpoint(self, global_steps, score=None, **info):     # learner/base.py:280-298
        """The reference Learner's hook: the checkpoint object decides whether
        this call saves (period / min_interval).  `checkpoint` may be a
        PeriodicCheckpoint-like object (save(score=, global_steps=,
        reload_metadata=, **info)) or a callable(global_steps=, score=, **info)."""
        c = getattr(self, 'checkpoint', None)
        if c is None:
            return False
        if hasattr(c, 'save'):
            return bool(c.save(score=score, global_steps=global_steps, reload_metadata=False, **info))
        return bool(c(global_steps=global_steps, score=score, **info))

    # ------------------------------------------------------------- metrics
    def _report_metrics(self, global_step):
        m = getattr(self, 'metrics', None)
        if m is None:
            return
        if not hasattr(m, 'due'):
            m(self.last_stats(), global_step)
            return
        self._accumulate_stats()
        if m.due():
            m(self._averaged_stats(), global_step)

    def _stats_vector(self):
        """this call's device statistics to average (the host class may append
        entries computed on the device, e.g. the z-filter means)"""
        return self.stats_buf

    def _accumulate_stats(self):
        """utils/common.py:606-648 (AverageDictionary of AverageValue): every
        call adds its values; the device vector is summed stream-ordered (no
        host sync)"""
        cur = self._stats_vector().detach()
        if self._stats_acc is None or self._stats_acc.shape != cur.shape:
            self._stats_acc = torch.zeros_like(cur)
            self._stats_n = 0
            self._host_acc = {}
        self._stats_acc.add_(cur)
        self._stats_last = cur.clone()
        self._stats_n += 1
        for k, v in self._host_scalars().items():
            s, n, _ = self._host_acc.get(k, (0.0, 0, 0.0))
            self._host_acc[k] = (s + float(v), n + 1, float(v))

    def _averaged_stats(self):
        """the statistics averaged over the window (one device read), then each
        accumulator restarts from the window's LAST value with count 1, as
        AverageValue.avg(clear=True) does (utils/common.py:620-630): the next
        window's average includes the value this one ended on"""
        n = max(self._stats_n, 1)
        vec = (self._stats_acc / n).cpu().numpy()
        host = {k: s / c for k, (s, c, _) in self._host_acc.items()}
        self._stats_acc.copy_(self._stats_last)
        self._stats_n = 1
        self._host_acc = {k: (last, 1, last) for k, (_, _, last) in self._host_acc.items()}
        return self._stats_dict(vec, host)
