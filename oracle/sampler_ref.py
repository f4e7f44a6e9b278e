"""ORACLE (test infrastructure only — see oracle/__init__.py).

Python access to the C restatement of the uniform replay index draw
(oracle/mt19937.c; reference: surreal/replay/uniform_replay.py:43-47) and the
ring-buffer insert semantics (uniform_replay.py:36-41) and FIFO order
(surreal/replay/fifo_replay.py:34-39).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    subprocess.run(['make', '-s', '-C', HERE], check=True)
    return os.path.join(HERE, '_build', 'libmt_oracle.so')


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, '_build', 'libmt_oracle.so')
        if not os.path.exists(path):
            path = build()
        lib = ctypes.CDLL(path)
        lib.oracle_randint_stream.restype = ctypes.c_int64
        lib.oracle_randint_stream.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64,
                                              ctypes.c_void_p]
        lib.oracle_seed_state.restype = None
        lib.oracle_seed_state.argtypes = [ctypes.c_uint64, ctypes.c_void_p]
        _LIB = lib
    return _LIB


def randint_stream(seed, n, batch):
    """[random.randint(0, n-1) for _ in range(batch)] after random.seed(seed)."""
    out = np.zeros(batch, dtype=np.int64)
    words = _lib().oracle_randint_stream(abs(int(seed)), int(n), int(batch), out.ctypes.data)
    return out, int(words)


def seed_state(seed):
    out = np.zeros(625, dtype=np.uint32)
    _lib().oracle_seed_state(abs(int(seed)), out.ctypes.data)
    return out


class UniformRingRef:
    """uniform_replay.py:36-41 ring insert; sample draws via the C stream."""

    def __init__(self, memory_size):
        self.memory = []
        self.memory_size = memory_size
        self.next_idx = 0

    def insert(self, exp):
        if self.next_idx >= len(self.memory):
            self.memory.append(exp)
        else:
            self.memory[self.next_idx] = exp
        self.next_idx = (self.next_idx + 1) % self.memory_size
