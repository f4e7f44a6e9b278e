"""Where does a parameter snapshot cost learner time?  C3 widths, 256
segments, publish after every learn(); times 8 x (learn + publish) for:
plain (no publisher), d2d (the snapshot's device copies only), d2h (+ the side-
stream D2H, no worker), fast (the publisher with a trivial serializer), and
the host time of snapshot() itself.
kd2h (the copy kernel issued from the learner thread), fast (the worker issues
the D2H once the snapshot's D2D ran), late (the publisher as the learner drives
it: snapshot(defer=True), then commit() after _post_publish's host reads).
Usage: python tools/diag_publish.py [--graph]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from surreal_amd import synthetic  # noqa: E402
from surreal_amd.learner import PPOLearner  # noqa: E402
from surreal_amd.publish import DeviceParameterPublisher, _Layout  # noqa: E402
from tests.helpers import env_config, ppo_config  # noqa: E402


def main():
    lc = ppo_config(B=256, T=25, mode='adapt', use_z_filter=True, hidden=(300, 200), lam=1.0,
                    rnn=True, rnn_hidden=100, horizon=5)
    lc.parameter_publish.exp_interval = lc.replay.batch_size
    D, A, Hd = 42, 8, 100
    learner = PPOLearner(lc, env_config(D, A), seed=1, use_graph='--graph' in sys.argv)
    batch = synthetic.to_device(synthetic.ppo_batch(256, 25, D, A, seed=3, rnn_hidden=Hd), 'cuda')
    lay = _Layout(learner.module_dict())
    dev_arena = torch.empty(lay.nbytes, dtype=torch.uint8, device='cuda')
    host_arena = torch.empty(lay.nbytes, dtype=torch.uint8).pin_memory()
    side = torch.cuda.Stream()
    fast = DeviceParameterPublisher(learner.module_dict(), serializer=lambda nd: b'x')
    host_t = []

    def d2d(it, msg, md):
        for view, off, nbytes in lay.storages:
            dev_arena[off:off + nbytes].copy_(view, non_blocking=True)

    def d2h(it, msg, md):
        d2d(it, msg, md)
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(side):
            side.wait_event(ev)
            host_arena.copy_(dev_arena, non_blocking=True)

    class Timed(object):
        def snapshot(self, it, msg):
            t0 = time.perf_counter()
            fast.snapshot(it, msg)
            host_t.append(time.perf_counter() - t0)

    from surreal_amd import _lib as L
    import ctypes

    def kd2h(it, msg, md):                           # the copy kernel from the learner thread
        d2d(it, msg, md)
        ev = torch.cuda.Event()
        ev.record()
        side.wait_event(ev)
        L.call('smi_copy_to_host', ctypes.c_void_p(host_arena.data_ptr()),
               ctypes.c_void_p(dev_arena.data_ptr()), lay.nbytes, ctypes.c_void_p(side.cuda_stream))

    variants = {'plain': None, 'd2d': d2d, 'd2h': d2h, 'kd2h': kd2h, 'fast': Timed(),
                'late': fast}

    def run(p, n=8):
        learner.publisher = p
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for it in range(n):
            learner.learn(batch)
            learner.publish_parameter(it)
        torch.cuda.synchronize()
        fast.flush()
        return time.perf_counter() - t0
    for p in variants.values():
        run(p, 2)
    t = {k: [] for k in variants}
    for _ in range(5):
        for k, p in variants.items():
            t[k].append(run(p))
    best = {k: round(min(v) / 8 * 1e3, 4) for k, v in t.items()}
    print(json.dumps({'graph': '--graph' in sys.argv, 'ms_per_learn_publish': best, 'snapshot_host_ms_median':
                      round(sorted(host_t)[len(host_t) // 2] * 1e3, 4), 'arena_bytes': lay.nbytes,
                      'storages': len(lay.storages)}), flush=True)
    fast.close()


if __name__ == '__main__':
    main()
