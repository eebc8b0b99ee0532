"""Activation store between shards: ``--storage_location gpu | cpu | disk``.

Reference (``/root/reference/utils.py:159-213``): after the last layer of a
shard each prompt's (prefix, suffix) hidden states are kept on the GPU, moved
to host RAM with a blocking ``.cpu()``, or ``np.save``d; they are fetched back
with blocking ``.to(device)`` / ``np.load`` before the next shard.

Here the store keys whole micro-batches and reuses the copy engine:

* ``gpu``  — the device tensor stays in HBM;
* ``cpu``  — async D2H into a per-key pinned buffer on a dedicated D2H stream
  (event-fenced, ``record_stream`` keeps the source alive), and async H2D on
  the H2D stream when prefetched for the next shard;
* ``disk`` — the same D2H, then a writer thread stores an ``.npy`` file (raw
  fp16 after a standard header) with the native ``pwrite`` engine; a reader
  thread ``pread``s it back into pinned memory ahead of use.

Pinned buffers are pooled in 1 MiB size buckets so the steady state allocates
nothing; :meth:`ActivationStore.trim` (end of every call) frees the buckets the
call did not use, so the pool tracks the current shapes instead of growing with
every new batch / generation-step shape (``--num_batch`` still bounds RAM).
"""
from __future__ import annotations

import os
import threading
from collections import defaultdict
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import hostmem

_NP_DT = {torch.float16: np.float16, torch.float32: np.float32, torch.bfloat16: None}


def _npy_header(shape, dtype: torch.dtype) -> bytes:
    """Standard .npy v1.0 header (magic + dict), so spills are np.load-able."""
    import io
    npdt = _NP_DT.get(dtype)
    descr = np.lib.format.dtype_to_descr(np.dtype(npdt)) if npdt is not None else "<u2"
    bio = io.BytesIO()
    np.lib.format.write_array_header_1_0(bio, {"descr": descr, "fortran_order": False,
                                               "shape": tuple(shape)})
    return bio.getvalue()


class _Entry:
    __slots__ = ("dev", "host", "event", "shape", "dtype", "path", "write_fut")

    def __init__(self):
        self.dev = self.host = self.event = self.path = self.write_fut = None
        self.shape = None
        self.dtype = None


class ActivationStore:
    def __init__(self, mode: str, device, disk_folder: str = "./temp", tag: str = "",
                 h2d_stream=None, d2h_stream=None):
        if mode not in ("gpu", "cpu", "disk"):
            raise ValueError(f"storage_location must be gpu/cpu/disk, got {mode!r}")
        self.mode = mode
        self.dev = torch.device(device)
        self.cuda = self.dev.type == "cuda"
        self.disk_folder = disk_folder
        self.tag = tag
        if mode == "disk":
            os.makedirs(disk_folder, exist_ok=True)
        self.h2d = h2d_stream if h2d_stream is not None else (torch.cuda.Stream(self.dev) if self.cuda else None)
        self.d2h = d2h_stream if d2h_stream is not None else (torch.cuda.Stream(self.dev) if self.cuda else None)
        self._e: Dict[object, _Entry] = {}
        self._pool: Dict[int, List[torch.Tensor]] = defaultdict(list)
        self._io = ThreadPoolExecutor(2, thread_name_prefix="fls-spill") if mode == "disk" else None
        self._inflight: Dict[object, Tuple[Future, None]] = {}
        self._recycle: List[Tuple[torch.Tensor, torch.cuda.Event]] = []
        self._used_keys = set()           # pool buckets handed out since the last trim()
        # pinned buffers per size bucket (in entries, pool and recycle list) and their bound:
        # None = grow as needed; n = past n buffers of a size, a new one waits for the oldest
        # host -> device copy still reading one (the engine bounds it when host RAM is the limit)
        self._n_alloc: Dict[int, int] = defaultdict(int)
        self.max_buffers: Optional[int] = None
        self.buffer_waits = 0
        self.bytes_d2h = 0
        self.bytes_h2d = 0
        self._stall_ev: List[Tuple[torch.cuda.Event, torch.cuda.Event]] = []   # compute-stream waits on H2D
        self.lock = threading.Lock()

    # ------------------------------------------------------------- pool
    BUCKET = 1 << 20

    def _get_host(self, nbytes: int) -> torch.Tensor:
        key = (max(1, nbytes) + self.BUCKET - 1) // self.BUCKET * self.BUCKET
        wait = None
        with self.lock:
            keep = []
            for h, ev in self._recycle:
                if ev.query():
                    self._pool[h.numel()].append(h)
                else:
                    keep.append((h, ev))
            self._recycle = keep
            self._used_keys.add(key)
            lst = self._pool.get(key)
            if lst:
                return lst.pop()
            if self.max_buffers is not None and self._n_alloc[key] >= self.max_buffers:
                for i, (h, ev) in enumerate(self._recycle):
                    if h.numel() == key:
                        wait = self._recycle.pop(i)
                        break
            if wait is None:
                self._n_alloc[key] += 1
        if wait is not None:
            # the oldest pending reload of this size: its copy is already enqueued, so this wait
            # needs nothing from the host (bounds the host's run-ahead by pinned memory instead)
            wait[1].synchronize()
            self.buffer_waits += 1
            return wait[0]
        return hostmem.alloc_host(key, pinned=self.cuda)

    def pooled_bytes(self) -> int:
        with self.lock:
            return sum(k * len(v) for k, v in self._pool.items())

    def trim(self) -> None:
        """Free pooled buffers of sizes not used since the last trim (call between calls, when
        every buffer is back in the pool)."""
        with self.lock:
            for h, ev in self._recycle:
                ev.synchronize()
                self._pool[h.numel()].append(h)
            self._recycle = []
            for k in list(self._pool):
                if k not in self._used_keys:
                    self._n_alloc[k] -= len(self._pool[k])
                    del self._pool[k]
            self._used_keys = set()

    def _put_host(self, buf: torch.Tensor) -> None:
        with self.lock:
            self._pool[buf.numel()].append(buf)

    def host_buffer(self, nbytes: int) -> torch.Tensor:
        """A pooled pinned buffer (rounded up to a 1 MiB bucket) for other D2H users."""
        return self._get_host(nbytes)

    def recycle_host(self, buf: torch.Tensor) -> None:
        """Return a buffer obtained from :meth:`host_buffer` to the pool."""
        self._put_host(buf)

    def path_for(self, key) -> str:
        return os.path.join(self.disk_folder, f"act{self.tag}-{int(key):05d}.npy")

    def __len__(self):
        return len(self._e)

    def keys(self):
        return list(self._e)

    # -------------------------------------------------------------- put
    def put(self, key, t: torch.Tensor):
        """Park ``t`` under ``key`` -> the event after which ``t``'s device memory may be
        overwritten (the D2H's completion on the D2H stream; None when ``t`` itself is kept)."""
        with self.lock:
            old = self._e.pop(key, None)
        if old is not None:
            self._drop(old)
        e = _Entry()
        e.shape, e.dtype = tuple(t.shape), t.dtype
        if self.mode == "gpu":
            e.dev = t
            with self.lock:
                self._e[key] = e
            return None
        nbytes = t.numel() * t.element_size()
        if not self.cuda:
            if self.mode == "cpu":
                e.host = t
            else:
                e.path = self.path_for(key)
                self._write_npy(e.path, t.contiguous(), e.shape, e.dtype)
            with self.lock:
                self._e[key] = e
            return None
        host = self._get_host(nbytes)
        cur = torch.cuda.current_stream(self.dev)
        self.d2h.wait_stream(cur)
        with torch.cuda.stream(self.d2h):
            host[:nbytes].view(t.dtype).view(e.shape).copy_(t, non_blocking=True)
            t.record_stream(self.d2h)
            ev = torch.cuda.Event()
            ev.record(self.d2h)
        self.bytes_d2h += nbytes
        e.host, e.event = host, ev
        if self.mode == "disk":
            e.path = self.path_for(key)

            def _write(ent=e):
                ent.event.synchronize()
                self._write_npy(ent.path, ent.host.view(ent.dtype)[:int(np.prod(ent.shape))].view(ent.shape),
                                ent.shape, ent.dtype)
                self._put_host(ent.host)
                ent.host = None
            e.write_fut = self._io.submit(_write)
        with self.lock:
            self._e[key] = e
        return ev

    def _write_npy(self, path: str, t: torch.Tensor, shape, dtype) -> None:
        hdr = _npy_header(shape, dtype)
        data = t.contiguous().view(-1).view(torch.uint8)
        with open(path, "wb") as f:
            f.write(hdr)
        rt = None
        from .. import _native
        rt = _native.runtime_or_none()
        if rt is not None:
            r = rt.fls_pwrite_from(path.encode(), len(hdr), data.numel(), data.data_ptr(), 4, 0)
            if r != data.numel():
                raise IOError(f"spill write failed {path}: {r}")
        else:
            with open(path, "ab") as f:
                f.write(data.numpy().tobytes())

    def _read_npy_into(self, path: str, shape, dtype, dst: torch.Tensor) -> None:
        with open(path, "rb") as f:
            np.lib.format.read_magic(f)
            np.lib.format.read_array_header_1_0(f)
            off = f.tell()
        n = int(np.prod(shape)) * torch.empty((), dtype=dtype).element_size()
        hostmem.pread_into(path, off, n, dst)

    # -------------------------------------------------------------- get
    def prefetch(self, key) -> None:
        """Start bringing ``key`` back to the device (no-op for gpu mode)."""
        with self.lock:
            if self.mode == "gpu" or key in self._inflight or key not in self._e:
                return
            e = self._e[key]
        if not self.cuda:
            return
        if self.mode == "disk":
            def _read(ent=e):
                if ent.write_fut is not None:
                    ent.write_fut.result()
                nbytes = int(np.prod(ent.shape)) * torch.empty((), dtype=ent.dtype).element_size()
                host = self._get_host(nbytes)
                self._read_npy_into(ent.path, ent.shape, ent.dtype, host)
                return host
            self._inflight[key] = (self._io.submit(_read), None)
        else:
            self._inflight[key] = (None, None)

    def get(self, key, pop: bool = True, out: Optional[torch.Tensor] = None, wait: bool = True):
        """The state parked under ``key`` on the device: a fresh tensor, or ``out`` (a slot of the
        engine's ActRing the caller acquired for the H2D stream) when given.  ``wait=False``
        (a landing ahead of its use): -> (tensor, H2D event); the compute stream waits later, by
        :meth:`wait_landed`."""
        with self.lock:
            e = self._e.pop(key) if pop else self._e[key]
        if self.mode == "gpu":
            return e.dev
        if not self.cuda:
            if self.mode == "cpu":
                return e.host
            arr = np.load(e.path)
            t = torch.from_numpy(arr.view(np.uint16)).view(e.dtype) if e.dtype == torch.bfloat16 else torch.from_numpy(arr)
            if pop:
                os.remove(e.path)
            return t
        fut, _ = self._inflight.pop(key, (None, None))
        if self.mode == "disk":
            if fut is None:
                if e.write_fut is not None:
                    e.write_fut.result()
                host = self._get_host(int(np.prod(e.shape)) * torch.empty((), dtype=e.dtype).element_size())
                self._read_npy_into(e.path, e.shape, e.dtype, host)
            else:
                host = fut.result()
        else:
            host = e.host
        nbytes = int(np.prod(e.shape)) * torch.empty((), dtype=e.dtype).element_size()
        cur = torch.cuda.current_stream(self.dev)
        if e.event is not None:
            self.h2d.wait_event(e.event)     # D2H finished before reading the host copy back
        ring = out is not None
        with torch.cuda.stream(self.h2d):
            # Allocate ON the H2D stream: a block from the compute stream's pool may
            # still be in use by compute kernels queued before its Python-side free,
            # and this copy does not wait for them (it overlaps the previous
            # micro-batch's compute).  record_stream below keeps the block from being
            # reused until the compute stream's consumers are done.  (A ring slot's reuse is
            # ordered by its free event instead: ActRing.acquire.)
            if not ring:
                out = torch.empty(e.shape, dtype=e.dtype, device=self.dev)
            elif tuple(out.shape) != tuple(e.shape) or out.dtype != e.dtype:
                raise ValueError(f"ring slot {tuple(out.shape)} {out.dtype} != parked {e.shape} {e.dtype}")
            out.copy_(host[:nbytes].view(e.dtype).view(e.shape), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.h2d)
        self.bytes_h2d += nbytes
        if wait:
            self.wait_landed(ev)
        if not ring:
            out.record_stream(cur)
        if pop:
            # host buffer is reusable once the H2D has completed (checked lazily)
            with self.lock:
                self._recycle.append((host, ev))
            if self.mode == "disk" and e.path and os.path.exists(e.path):
                try:
                    os.remove(e.path)
                except OSError:
                    pass
        return out if wait else (out, ev)

    def wait_landed(self, ev) -> None:
        """The compute stream waits for an H2D (timed: ``act_stall_gpu_s``)."""
        cur = torch.cuda.current_stream(self.dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        cur.wait_event(ev)
        e1.record(cur)
        self._stall_ev.append((e0, e1))

    def take_stall_seconds(self) -> float:
        """GPU time the compute stream spent waiting for activation H2D since the last call
        (events must have completed: call after a synchronize)."""
        t = sum(a.elapsed_time(b) for a, b in self._stall_ev) / 1e3
        self._stall_ev = []
        return t

    def _drop(self, e: _Entry) -> None:
        if e.write_fut is not None:
            e.write_fut.result()
        if e.host is not None and self.cuda:
            if e.event is not None:
                e.event.synchronize()
            self._put_host(e.host)

    def clear(self):
        for k in list(self._e):
            self._drop(self._e.pop(k))

    def close(self):
        self.clear()
        if self._io is not None:
            self._io.shutdown(wait=True)


class ActRing:
    """Fixed HBM slots for the hidden states of a pass (single GPU / data parallel, storage cpu or
    disk): the micro-batch being computed (updated in place by the residual GEMM epilogues) and the
    next one landing from the host, or a state carried across a zigzag shard boundary.

    The caching allocator alone bounds nothing here: every H2D landing buffer allocated ahead of
    its use, and every D2H source held by ``record_stream`` until the copy drains, stays reserved
    while the host runs ahead — round 4's plan had to charge 5 live states for it, which starved
    the arena under ``--max_vram_gb``.  A slot is reused only behind its free
    event (the D2H of its last occupant, or the compute that last read it), waited for on the
    stream that fills it next, so the host never blocks and the bound is exact: ``n_slots``
    states.  Slots go least-recently-released first, so the landing of micro-batch j+1 never waits
    for the D2H of micro-batch j."""

    def __init__(self, device, dtype: torch.dtype, n_slots: int):
        self.dev, self.dtype, self.n = torch.device(device), dtype, n_slots
        self._bufs: List[Optional[torch.Tensor]] = [None] * n_slots
        self._free: List[Optional[torch.cuda.Event]] = [None] * n_slots
        self._owner: List[object] = [None] * n_slots
        self._age = [0] * n_slots
        self._tick = 0

    def resize(self, n_slots: int, elems: int) -> None:
        """At a pass start (every slot released): ``n_slots`` slots of >= ``elems`` elements."""
        if any(o is not None for o in self._owner):
            raise RuntimeError("activation ring resized with live states")
        if n_slots != self.n:
            self.n = n_slots
            self._bufs, self._free = [None] * n_slots, [None] * n_slots
            self._owner, self._age = [None] * n_slots, [0] * n_slots
        for i in range(n_slots):
            if self._bufs[i] is None or self._bufs[i].numel() < elems:
                self._bufs[i] = None
                self._bufs[i] = torch.empty(max(1, elems), dtype=self.dtype, device=self.dev)
                self._free[i] = None

    def bytes(self) -> int:
        return sum(b.numel() * b.element_size() for b in self._bufs if b is not None)

    def acquire(self, key, shape, stream) -> torch.Tensor:
        """A free slot for ``key``'s state as a ``shape`` view; ``stream`` (the one that fills it)
        waits for the slot's previous occupant to be done with it."""
        free = [i for i in range(self.n) if self._owner[i] is None]
        if not free:
            raise RuntimeError(f"activation ring: all {self.n} slots hold live states")
        i = min(free, key=lambda j: self._age[j])
        if self._free[i] is not None and stream is not None:
            stream.wait_event(self._free[i])
        self._owner[i] = key
        n = 1
        for d in shape:
            n *= d
        return self._bufs[i][:n].view(shape)

    def holds(self, t: torch.Tensor) -> int:
        """Index of the slot ``t`` lives in (-1: not a ring tensor)."""
        p = t.data_ptr()
        for i, b in enumerate(self._bufs):
            if b is not None and b.data_ptr() <= p < b.data_ptr() + b.numel() * b.element_size():
                return i
        return -1

    def release(self, key, event) -> None:
        """``key``'s slot may be refilled once ``event`` (recorded on the stream of its last use)
        has completed."""
        for i in range(self.n):
            if self._owner[i] == key:
                self._owner[i] = None
                self._free[i] = event
                self._tick += 1
                self._age[i] = self._tick
                return

    def owns(self, key) -> bool:
        return key in self._owner

    def has_free(self) -> bool:
        return any(o is None for o in self._owner)

    def reset(self) -> None:
        """After an aborted pass: every slot free, its next fill ordered after the work queued on
        the current stream so far."""
        cur = torch.cuda.current_stream(self.dev) if self.dev.type == "cuda" else None
        for i in range(self.n):
            if self._owner[i] is not None and cur is not None:
                e = torch.cuda.Event()
                e.record(cur)
                self._free[i] = e
        self._owner = [None] * self.n
