"""Native RCCL communicator for the data-parallel weight all-gathers (``--dp_gather_comm native``).

``parallel/comm.py`` drives every collective through ``torch.distributed`` (its ``"nccl"`` backend
is RCCL on ROCm).  The weight fan-out is the one hot collective: per layer piece, an in-place byte
all-gather into an HBM slot on the prefetcher's copy stream (``parallel/data_parallel.py``).  This
communicator issues it straight from C (``csrc/comm/rccl_comm.cpp``) on the caller's current HIP
stream: the gather is ordered by the stream itself, with no ``Work`` object and no extra stream
handshake.  It is a communicator of its own (one ncclUniqueId made by rank 0 and broadcast over the
default group), like the ``dup()`` group it replaces; every other operation falls through to the
default group.  The reference has no collective layer at all: its GPUs are threads sharing a host
cache (``/root/reference/utils.py:24-75``).
"""
from __future__ import annotations

import ctypes

import torch

from .. import _native
from .comm import Comm, _DoneWork


class NativeRcclComm(Comm):
    def __init__(self, base: Comm):
        super().__init__(base.rank, base.world, base.device, base.backend, group=None)
        if self.device.type != "cuda":
            raise ValueError("the native RCCL communicator runs on a GPU")
        self.lib = _native.comm()
        n = self.lib.fls_rccl_id_bytes()
        uid = (ctypes.c_char * n)()
        if base.rank == 0 and self.lib.fls_rccl_unique_id(uid) != 0:
            raise RuntimeError("ncclGetUniqueId failed")
        if base.active:
            raw = base.broadcast_object(bytes(uid) if base.rank == 0 else None, src=0)
            ctypes.memmove(uid, raw, n)
        self._h = self.lib.fls_rccl_init(self.world, self.rank, uid, self.device.index or 0)
        if not self._h:
            raise RuntimeError(f"ncclCommInitRank failed (rank {self.rank} of {self.world})")

    def dup(self) -> "NativeRcclComm":
        return NativeRcclComm(self)

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """out = [rank 0's inp | rank 1's | ...] (bytes), enqueued on the current stream; in place when
        ``inp`` is this rank's slice of ``out``.  The returned work is already ordered."""
        nb = inp.numel() * inp.element_size()
        if (not out.is_cuda or not inp.is_cuda or not out.is_contiguous() or not inp.is_contiguous()
                or out.numel() * out.element_size() != nb * self.world):
            raise ValueError("all_gather_into: contiguous CUDA tensors, out = world x inp bytes")
        stream = torch.cuda.current_stream(self.device).cuda_stream
        if self.lib.fls_rccl_all_gather(self._h, inp.data_ptr(), out.data_ptr(), nb, stream) != 0:
            raise RuntimeError("ncclAllGather failed")
        return _DoneWork()

    def warmup(self) -> None:
        """One tiny all-gather (RCCL allocates a communicator's buffers at its first operation)."""
        t = torch.zeros(self.world * 4, dtype=torch.uint8, device=self.device)
        self.all_gather_into(t, t[self.rank * 4:(self.rank + 1) * 4])
        torch.cuda.synchronize(self.device)

    def destroy(self):
        if getattr(self, "_h", None):
            self.lib.fls_rccl_destroy(self._h)
            self._h = None
