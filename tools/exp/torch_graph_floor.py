"""Per-node cost of torch.cuda.graph replays (diagnostic): 200 tiny torch
launches, then 200 tiny library launches (smi_soft_update over 64 floats),
each captured by torch.cuda.graph and replayed; microseconds per launch."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from surreal_amd import _lib as L  # noqa: E402

dev = torch.device('cuda', 0)
x = torch.zeros(64, device=dev)
y = torch.ones(64, device=dev)
N = 200


def timed(fn):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (10 * N) * 1e6


def torch_ops():
    for _ in range(N):
        x.add_(1.0)


def lib_ops():
    st = L.stream(dev)
    for _ in range(N):
        L.call('smi_soft_update', L.ptr(x), L.ptr(y), 64, 0.5, st)


print(json.dumps({'torch_add_us': round(timed(torch_ops), 2), 'lib_soft_update_us': round(timed(lib_ops), 2)}))
