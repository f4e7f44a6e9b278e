"""Parameter publishing from the learner.

The reference publishes by `ModuleDict(module_dict).dumps()`: every module's
state_dict() moved to host numpy (`state_dict[key].cpu().numpy()`), the
{name: {key: ndarray}} dict serialized and sent with {'time', 'iteration',
'message', 'hash'} (surreal/distributed/module_dict.py:22-35,
parameter_server.py:40-55).  Agents consume it with ModuleDict.load, so the
state_dict keys and shapes are the wire format.

MI355X side: the learner's parameters live in a handful of flat device
buffers (model.py), so a snapshot is ONE gather-copy launch of those buffers
into a snapshot arena (smi_copy_gather; one ctypes call instead of a torch
copy per buffer: the learner thread's issue time is the eager learner's
critical path), enqueued on the learner's stream right after the last
learn() (stream-ordered: no host wait), followed by ONE device-to-host copy of
the arena into pinned memory on a side stream, issued by the learner thread once
its own post-publish host reads are done (commit()).  The D2H is a copy KERNEL
writing the mapped pinned buffer (smi_copy_to_host), not a runtime DMA copy:
an SDMA hipMemcpyAsync D2H held the learner thread ~0.25 ms per publish
(tools/diag_publish.py), which the GPU then spent idle.  The next learn() is
enqueued immediately and overlaps the D2H; its parameter updates cannot race
the copy because the copy reads the arena, not the parameters.  A background
thread waits for the copy and hands the numpy dict — views of the pinned
arena reshaped to the state_dict shapes — to the serializer, then frees the
slot (no host-side copies: the worker holds the GIL as briefly as possible,
since any Python it runs delays the learner thread's launches: the views of
each slot are built once, at construction).
"""
import base64
import ctypes
import hashlib
import pickle
import queue
import threading
import time

import numpy as np
import torch

from surreal_amd import _lib as L


def binary_hash(binary):
    """surreal/utils/serializer.py:55-66: the first 16 base64 characters of the
    md5 digest, returned as they are (the reference's `.replace('/', '_')` is
    commented out at :65, so '/' and '+' stay in the hash)."""
    return base64.b64encode(hashlib.md5(binary).digest())[:16].decode('utf-8')


class _Layout(object):
    """state_dict keys -> (storage index, byte offset, shape, dtype) over the
    distinct device storages the tensors live in (the flat buffers)."""

    def __init__(self, module_dict):
        self.keys = []            # (module name, key, storage idx, byte offset, shape, np dtype)
        self.storages = []        # (uint8 device view of the whole storage, arena offset, nbytes)
        index = {}
        off = 0
        for name, m in module_dict.items():
            for key, t in m.state_dict(keep_vars=True).items():
                t = t.detach()
                if not t.is_cuda or not t.is_contiguous():
                    raise ValueError(f'{name}.{key}: parameters must be contiguous device tensors')
                st = t.untyped_storage()
                sid = st.data_ptr()
                if sid not in index:
                    nbytes = st.nbytes()
                    view = torch.empty(0, dtype=torch.uint8, device=t.device).set_(st, 0, (nbytes,))
                    index[sid] = len(self.storages)
                    self.storages.append((view, off, nbytes))
                    off += (nbytes + 255) // 256 * 256
                i = index[sid]
                boff = self.storages[i][1] + t.storage_offset() * t.element_size()
                self.keys.append((name, key, boff, tuple(t.shape),
                                  torch.empty(0, dtype=t.dtype).numpy().dtype))
        self.nbytes = max(off, 256)
        # the snapshot's gather copy, as ctypes arrays built once.  The gather
        # kernel moves 16-byte aligned storages of whole 4-byte words (every
        # flat parameter buffer; arena offsets are 256-byte aligned); any other
        # storage (a bool / uint8 buffer of odd size, an unaligned view) is
        # copied by torch on the same stream instead
        def gatherable(v, nbytes):
            return nbytes % 4 == 0 and v.data_ptr() % 16 == 0
        gs = [(v, o, b) for v, o, b in self.storages if gatherable(v, b)]
        self.other = [(v, o, b) for v, o, b in self.storages if not gatherable(v, b)]
        n = len(gs)
        self.c_n = n
        self.c_src = (ctypes.c_void_p * n)(*[v.data_ptr() for v, _, _ in gs])
        self.c_off = (ctypes.c_int64 * n)(*[o for _, o, _ in gs])
        self.c_len = (ctypes.c_int64 * n)(*[b for _, _, b in gs])

    def views(self, raw):
        """{module name: {state_dict key: ndarray view}} of an arena image"""
        out = {}
        for name, key, boff, shape, dt in self.keys:
            n = int(np.prod(shape)) * dt.itemsize
            out.setdefault(name, {})[key] = raw[boff:boff + n].view(dt).reshape(shape)
        return out


class Snapshot(object):
    """One published parameter set; numpy_dict() waits for its D2H copy."""

    def __init__(self, layout, host, event, iteration, message, slot=None):
        self._layout, self._host, self._event, self._slot = layout, host, event, slot
        self.iteration, self.message = iteration, message
        self.time = time.time()

    def _commit_if_pending(self):
        """a deferred snapshot whose D2H nobody issued yet: issue it now (from
        whichever thread asks), so waiting on it cannot block forever"""
        pub = getattr(self, '_pub', None)
        if pub is not None and not self._event.is_set():
            pub._commit(self)

    def ready(self):
        self._commit_if_pending()
        return self._event.is_set()

    def numpy_dict(self, copy=True):
        """{module name: {state_dict key: ndarray}} as ModuleDict.dumps builds it.
        copy=False returns views of the pinned slot (valid until the slot is
        reused: the publisher's worker serializes from them, then frees it)."""
        self._commit_if_pending()
        self._event.wait()
        if not copy and self._slot is not None:
            return self._slot['views']
        views = self._layout.views(self._host.numpy())
        if not copy:
            return views
        return {name: {k: v.copy() for k, v in d.items()} for name, d in views.items()}


class DeviceParameterPublisher(object):
    """ParameterPublisher.publish (parameter_server.py:40-55) for the MI355X
    learner: snapshot() is asynchronous; a worker thread serializes the numpy
    dict and calls sink(binary, info) in publish order.

    module_dict: {name: nn.Module} (learner.module_dict()).
    sink: callable(binary, info) — e.g. a ZMQ socket's send; None keeps the
          last published (binary, info) in `self.last` (tests, offline use).
    serializer: the reference uses pyarrow's pa.serialize (removed from
          current pyarrow) with pickle as its commented alternative
          (utils/serializer.py:8-24); pickle is the default here.
    """

    def __init__(self, module_dict, sink=None, serializer=pickle.dumps, slots=2):
        self.layout = _Layout(module_dict)
        L.lib()
        dev = self.layout.storages[0][0].device
        self.device = dev
        self.sink = sink
        self.serializer = serializer
        self.side = torch.cuda.Stream(device=dev)
        self.slots = [{'dev': torch.empty(self.layout.nbytes, dtype=torch.uint8, device=dev),
                       'host': torch.empty(self.layout.nbytes, dtype=torch.uint8).pin_memory(),
                       'free': threading.Event()} for _ in range(slots)]
        for sl in self.slots:
            sl['free'].set()
            sl['views'] = self.layout.views(sl['host'].numpy())
        self.next = 0
        self._pending = None
        self._pending_lock = threading.Lock()
        self.last = None
        self.published = 0
        self._q = queue.Queue()
        self._err = None
        self._worker = threading.Thread(target=self._run, daemon=True)
        self._worker.start()

    def snapshot(self, iteration=0, message='', defer=False):
        """Enqueue the parameter snapshot on the current (learner) stream and its
        D2H on the side stream; returns a Snapshot without waiting.  defer=True
        leaves the D2H to the caller's commit() (the learner issues it after
        _post_publish's host reads: a D2H in flight across those reads cost the
        learner ~0.17 ms per publish whichever engine or thread ran it,
        tools/diag_publish.py)."""
        if self._err is not None:
            raise RuntimeError('parameter publisher worker failed') from self._err
        self.commit()                         # a deferred snapshot not yet committed
        slot = self.slots[self.next]
        self.next = (self.next + 1) % len(self.slots)
        slot['free'].wait()                   # the worker has copied this slot's last snapshot out
        slot['free'].clear()
        cur = torch.cuda.current_stream(self.device)
        lay = self.layout                                      # D2D, stream-ordered after learn()
        if lay.c_n:
            L.call('smi_copy_gather', ctypes.c_void_p(slot['dev'].data_ptr()), lay.c_src, lay.c_off,
                   lay.c_len, lay.c_n, ctypes.c_void_p(cur.cuda_stream))
        for v, o, b in lay.other:
            slot['dev'][o:o + b].copy_(v)
        taken = torch.cuda.Event()
        taken.record(cur)
        # the D2H is issued by the worker once the snapshot's D2D has run (it
        # then overlaps the NEXT learn(); issued here it landed in the window
        # where the learner thread syncs for the KL record and re-launches)
        snap = Snapshot(self.layout, slot['host'], threading.Event(), iteration, message, slot)
        snap._taken = taken
        snap._done = None
        snap._issued = threading.Event()
        snap._pub = self
        if defer:
            with self._pending_lock:
                self._pending = snap
        else:
            snap._issued.set()                # the worker issues the D2H
        # neither half of the slot is rewritten before the worker has serialized
        # it (slot['free'], set after the D2H completed and was read)
        self._q.put(snap)
        return snap

    def _issue(self, snap):
        """ONE D2H of the slot on the side stream, after the snapshot's D2D, as
        a kernel into the mapped pinned slot (smi_copy_to_host)"""
        slot = snap._slot
        with torch.cuda.device(self.device):
            self.side.wait_event(snap._taken)
            L.call('smi_copy_to_host', ctypes.c_void_p(slot['host'].data_ptr()),
                   ctypes.c_void_p(slot['dev'].data_ptr()), self.layout.nbytes,
                   ctypes.c_void_p(self.side.cuda_stream))
            done = torch.cuda.Event()
            done.record(self.side)
        snap._done = done

    def commit(self):
        """Issue the D2H of the last snapshot(defer=True).  The learner calls it
        after its post-publish host reads; Snapshot.numpy_dict()/ready() and
        flush() call it too, from any thread, so a deferred snapshot is never
        waited on unissued."""
        self._commit(None)

    def _commit(self, want):
        """issue the pending snapshot (if want is given: only if it is that one)"""
        with self._pending_lock:
            snap = self._pending
            if snap is None or (want is not None and snap is not want):
                return
            self._pending = None
            self._issue(snap)
            snap._issued.set()

    def _d2h(self, snap):
        """worker side: wait for the copy (issuing it unless deferred)"""
        snap._issued.wait()
        if snap._done is None:
            snap._taken.synchronize()         # issued after the D2D ran: off the learner's launches
            self._issue(snap)
        snap._done.synchronize()
        snap._event.set()

    def _run(self):
        while True:
            snap = self._q.get()
            if snap is None:
                return
            try:
                self._d2h(snap)
                nd = snap.numpy_dict(copy=False)
                binary = self.serializer(nd)
                del nd
                snap._slot['free'].set()
                info = {'time': snap.time, 'iteration': snap.iteration, 'message': snap.message,
                        'hash': binary_hash(binary)}
                if self.sink is not None:
                    self.sink(binary, info)
                self.last = (binary, info)
                self.published += 1
            except Exception as e:           # surfaced on the next snapshot() / flush()
                self._err = e
                snap._slot['free'].set()
            finally:
                self._q.task_done()

    def flush(self):
        """Wait until every snapshot taken so far has reached the sink."""
        self.commit()
        self._q.join()
        if self._err is not None:
            raise RuntimeError('parameter publisher worker failed') from self._err

    def close(self):
        self.flush()
        self._q.put(None)
        self._worker.join(timeout=10)
