"""Replay buffers of the learner hot path.

UniformReplay mirrors surreal/replay/uniform_replay.py:6-74 with the memory as
a device-resident ring of fixed-width rows (obs | action | reward | obs_next |
done) in HBM and the index draw done by the CPython-exact MT19937 HIP kernel
(smi_mt_randint), so `sample()` returns exactly the rows the reference's
`[random.randint(0, len-1) for _ in range(B)]` would pick after
`random.seed(seed)`.  FIFOReplay mirrors fifo_replay.py:6-49 (host deque; the
PPO path consumes batches in insertion order).
"""
import ctypes
from collections import deque

import numpy as np
import torch

from . import _lib as L


class CPythonRandom(object):
    """Host+device MT19937 state that reproduces `random.seed(s); random.randint`."""

    def __init__(self, seed=0, device=None):
        self.device = device
        self.host = np.zeros(625, dtype=np.uint32)
        L.check(L.lib().smi_mt_seed(abs(int(seed)), self.host.ctypes.data), 'smi_mt_seed')
        self.dev = None
        if device is not None:
            self.dev = torch.from_numpy(self.host.view(np.int32).copy()).to(device)

    def randint_host(self, n, batch):
        out = np.zeros(batch, dtype=np.int64)
        L.check(L.lib().smi_mt_randint_host(self.host.ctypes.data, int(n), int(batch),
                                            out.ctypes.data), 'smi_mt_randint_host')
        return out

    def randint_device(self, n, batch, out=None):
        if out is None:
            out = torch.empty(batch, dtype=torch.int64, device=self.device)
        L.call('smi_mt_randint', L.ptr(self.dev), int(n), int(batch), L.ptr(out),
               L.stream(self.device))
        return out


class UniformReplay(object):
    """Ring buffer with CPython-exact uniform sampling (uniform_replay.py:36-47).

    Rows are fixed-width float32 records laid out [obs(D) | action(A) |
    reward(1) | obs_next(D) | done(1)] in one (memory_size, W) device tensor."""

    def __init__(self, learner_config, env_config, session_config=None, index=0, seed=0,
                 device=None):
        L.require_gpu()
        self.learner_config = learner_config
        self.memory_size = int(learner_config['replay']['memory_size'])
        self.sampling_start_size = int(learner_config['replay']['sampling_start_size'])
        self.obs_dim = int(sum(v[0] for v in env_config['obs_spec']['low_dim'].values()))
        self.act_dim = int(env_config['action_spec']['dim'][0])
        self.width = 2 * self.obs_dim + self.act_dim + 2
        self.device = torch.device(device) if device is not None else torch.device('cuda')
        self.table = torch.zeros(self.memory_size, self.width, dtype=torch.float32,
                                 device=self.device)
        self._len = 0
        self._next_idx = 0
        self.rng = CPythonRandom(seed, self.device)
        self._idx = None

    def __len__(self):
        return self._len

    def insert(self, exp_dict):
        """uniform_replay.py:36-41 for one SSAR experience dict."""
        row = self.pack([exp_dict])
        self.insert_rows(row)

    def pack(self, exps):
        D, A = self.obs_dim, self.act_dim
        out = np.zeros((len(exps), self.width), dtype=np.float32)
        for i, e in enumerate(exps):
            o0 = np.concatenate([np.ravel(v) for v in e['obs'][0]['low_dim'].values()])
            o1 = np.concatenate([np.ravel(v) for v in e['obs'][1]['low_dim'].values()])
            out[i, :D] = o0
            out[i, D:D + A] = e['action']
            out[i, D + A] = e['reward']
            out[i, D + A + 1:2 * D + A + 1] = o1
            out[i, 2 * D + A + 1] = float(e['done'])
        return out

    def insert_rows(self, rows):
        """Bulk ring insert of packed rows (same slot sequence as repeated insert)."""
        rows = torch.as_tensor(rows, dtype=torch.float32)
        n = rows.shape[0]
        # more rows than slots: only the last memory_size survive a sequence of
        # single inserts; scatter just those (no duplicate slot indices)
        skip = max(0, n - self.memory_size)
        slots = (self._next_idx + np.arange(skip, n)) % self.memory_size
        self.table[torch.as_tensor(slots, device=self.device)] = rows[skip:].to(self.device)
        self._len = min(self.memory_size, self._len + n)
        self._next_idx = int((self._next_idx + n) % self.memory_size)

    def start_sample_condition(self):
        return len(self) > self.sampling_start_size

    def sample_indices(self, batch_size):
        if self._idx is None or self._idx.numel() != batch_size:
            self._idx = torch.empty(batch_size, dtype=torch.int64, device=self.device)
        return self.rng.randint_device(len(self), batch_size, self._idx)

    def sample(self, batch_size, out=None, rank=0, world=1):
        """Returns (indices, rows[batch, W]) on device; rows gathered by kernel.

        Data parallel (world > 1, SURVEY §8(e) DDPG row): every rank holds the
        same replicated ring and the same MT19937 state (same seed, same
        inserts), so all ranks draw the SAME `batch_size` global indices -- the
        one CPython-exact stream a single learner draws
        (uniform_replay.py:43-47) -- and gather only their own slice of
        batch_size / world rows: the sampling stays bit-exact and the shards
        concatenate to the single learner's batch."""
        if world < 1 or not 0 <= rank < world or batch_size % world:
            raise ValueError(f'batch_size {batch_size} must split evenly over {world} ranks')
        idx = self.sample_indices(batch_size)
        n = batch_size // world
        mine = idx[rank * n:(rank + 1) * n]
        if out is None:
            out = torch.empty(n, self.width, dtype=torch.float32, device=self.device)
        if tuple(out.shape) != (n, self.width) or not out.is_contiguous():
            raise ValueError(f'out must be a contiguous ({n}, {self.width}) tensor')
        L.call('smi_gather_rows', L.ptr(self.table), self.width, L.ptr(mine), n, L.ptr(out),
               L.stream(self.device))
        return mine, out

    def split(self, rows):
        D, A = self.obs_dim, self.act_dim
        return {'obs': rows[:, :D], 'actions': rows[:, D:D + A],
                'rewards': rows[:, D + A:D + A + 1], 'obs_next': rows[:, D + A + 1:2 * D + A + 1],
                'dones': rows[:, 2 * D + A + 1:2 * D + A + 2]}


class FIFOReplay(object):
    """fifo_replay.py:6-49: popleft x batch in insertion order."""

    def __init__(self, learner_config, env_config=None, session_config=None, index=0):
        self.batch_size = learner_config['replay']['batch_size']
        self.memory_size = learner_config['replay']['memory_size']
        self._memory = deque(maxlen=self.memory_size + 3)

    def insert(self, exp_tuple):
        self._memory.append(exp_tuple)

    def sample(self, batch_size):
        assert batch_size <= self.memory_size
        return [self._memory.popleft() for _ in range(batch_size)]

    def start_sample_condition(self):
        return len(self._memory) >= self.batch_size

    def __len__(self):
        return len(self._memory)
