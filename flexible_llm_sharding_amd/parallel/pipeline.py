"""Model-parallel stage hand-off: a receiver thread that drains incoming activations.

Reference (``/root/reference/utils.py:159-213``): a producer stage parks each
prompt's activations in a shared dict (RAM) or, at the wrap-around boundary
(last GPU -> GPU 0) in disk mode, in ``.npy`` files; the consumer sleep-polls
``prompt2layer`` once a second and copies the entry to its device.  Producers
block while the dict holds ``max_activation_in_cpu`` entries.

Here every stage boundary is an RCCL ``isend`` / ``irecv`` pair over xGMI on a
per-edge communicator (:meth:`.comm.Comm.setup_p2p_edges`).  The receiving
side is a :class:`StageReceiver` thread that posts the stage's receives in the
sender's order, one micro-batch at a time, and drains each completed one into
an :class:`~..runtime.activations.ActivationStore` of the run's
``--storage_location``: ``gpu`` keeps it in HBM, ``cpu`` moves it to pinned RAM
on the D2H stream, ``disk`` spills it to an ``.npy`` file.  The main thread
takes micro-batches out of the store when its compute reaches them (with a
one-ahead H2D prefetch).  So a producer never waits for a busy consumer to
post a receive — the wrap-boundary queue the reference parks in RAM / on disk
lives in the same places here — and its pending ``isend`` buffers are retired
as soon as the receiver drains them (the engine prunes completed sends after
every micro-batch).
"""
from __future__ import annotations

import contextlib
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..runtime.activations import ActivationStore


def rx_key(shard: int, mb: int) -> int:
    return shard * 1_000_000 + mb


class StageReceiver:
    """Receives ``jobs`` = [(key, src_rank, shape)] in order on a thread; :meth:`get` hands them out."""

    def __init__(self, comm, device, dtype: torch.dtype, storage: str, disk_folder: str, tag: str,
                 jobs: Sequence[Tuple[int, int, Tuple[int, ...]]], timeout_s: float = 1800.0):
        self.comm, self.dev, self.dtype = comm, torch.device(device), dtype
        self.cuda = self.dev.type == "cuda"
        self.jobs = list(jobs)
        self.timeout_s = timeout_s
        self.stream = torch.cuda.Stream(self.dev) if self.cuda else None
        self.store = ActivationStore(storage, self.dev, disk_folder, tag=f"rx{tag}")
        self.cv = threading.Condition()
        self.ready: Dict[int, Optional[torch.cuda.Event]] = {}
        self.err: Optional[BaseException] = None
        self.received = 0
        self.thread = threading.Thread(target=self._run, name="fls-stage-rx", daemon=True)
        self.thread.start()

    def _run(self) -> None:
        try:
            ctx = torch.cuda.stream(self.stream) if self.cuda else contextlib.nullcontext()
            with ctx:
                for key, src, shape in self.jobs:
                    buf = torch.empty(shape, dtype=self.dtype, device=self.dev)
                    work = self.comm.irecv(buf, src)
                    work.wait()                      # GPU: the receive stream waits for RCCL; CPU: the host
                    ev = None
                    if self.cuda:
                        ev = torch.cuda.Event()
                        ev.record(self.stream)
                    self.store.put(key, buf)         # gpu: kept; cpu / disk: D2H (+ spill) off this stream
                    del buf
                    with self.cv:
                        self.ready[key] = ev
                        self.received += 1
                        self.cv.notify_all()
        except BaseException as e:  # noqa: BLE001 - re-raised in the consumer
            with self.cv:
                self.err = e
                self.cv.notify_all()

    def _wait(self, key: int) -> Optional[torch.cuda.Event]:
        with self.cv:
            ok = self.cv.wait_for(lambda: key in self.ready or self.err is not None, timeout=self.timeout_s)
            if self.err is not None:
                raise RuntimeError(f"stage receiver failed: {self.err!r}") from self.err
            if not ok:
                raise TimeoutError(f"no activation for micro-batch key {key} within {self.timeout_s:.0f}s")
            return self.ready.pop(key)

    def prefetch(self, key: int) -> None:
        """Start the H2D of ``key`` if it has already arrived (cpu / disk storage)."""
        with self.cv:
            here = key in self.ready
        if here:
            self.store.prefetch(key)

    def get(self, key: int) -> torch.Tensor:
        ev = self._wait(key)
        t = self.store.get(key)
        if self.cuda and ev is not None and self.store.mode == "gpu":
            cur = torch.cuda.current_stream(self.dev)
            cur.wait_event(ev)
            t.record_stream(cur)
        return t

    def close(self) -> None:
        self.thread.join(timeout=self.timeout_s)
        with self.cv:
            left = len(self.ready)
        self.store.close()
        if self.err is not None:
            raise RuntimeError(f"stage receiver failed: {self.err!r}") from self.err
        if left or self.received != len(self.jobs):
            raise RuntimeError(f"stage receiver: {self.received}/{len(self.jobs)} received, {left} unconsumed")
