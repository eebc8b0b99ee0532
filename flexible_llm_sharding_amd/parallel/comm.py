"""Process-per-GPU communication over ``torch.distributed``.

The reference has no collectives library: GPUs are threads of one process
that exchange activations through a shared Python dict with 1-second
sleep-polling (``/root/reference/utils.py:159-213``) and share weights through
a host-RAM cache guarded by a Condition/Lock pair (``utils.py:24-75``; ABBA
lock order).

Here each GPU is its own process.  On ROCm the ``"nccl"`` backend *is* RCCL,
so pipeline hand-offs are point-to-point ``isend``/``irecv`` over xGMI, the
data-parallel weight fan-out is ``all_gather_into_tensor`` and results are
gathered to rank 0.  On CPU (tests) the same code runs over ``gloo``.
"""
from __future__ import annotations

import datetime
import os
import pickle
from typing import Any, List, Optional

import torch
import torch.distributed as dist


class Comm:
    """Thin wrapper; ``world == 1`` works without an initialised process group."""

    def __init__(self, rank: int = 0, world: int = 1, device=None, backend: Optional[str] = None,
                 group=None):
        self.rank, self.world = rank, world
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.backend = backend
        self.group = group          # None: the default process group

    @property
    def active(self) -> bool:
        return self.world > 1

    # ------------------------------------------------------------ factory
    @classmethod
    def from_env(cls, device_type: str = "cuda", timeout_s: int = 1800) -> "Comm":
        """Initialise from RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT (torchrun)."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", str(rank)))
        if device_type == "cuda":
            dev = torch.device("cuda", local)
            torch.cuda.set_device(dev)
        else:
            dev = torch.device("cpu")
        if world <= 1:
            return cls(0, 1, dev)
        backend = "nccl" if device_type == "cuda" else "gloo"
        if not dist.is_initialized():
            kw = dict(backend=backend, rank=rank, world_size=world,
                      timeout=datetime.timedelta(seconds=timeout_s))
            if backend == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(**kw)
        return cls(rank, world, dev, backend)

    def dup(self) -> "Comm":
        """A Comm on a fresh communicator over the same ranks (collective: every rank calls it).

        The data-parallel weight all-gathers run on their own communicator, issued by the
        loader thread, so they never interleave with the main thread's collectives on the
        default group (each communicator sees the same op sequence on every rank)."""
        if not self.active:
            return Comm(self.rank, self.world, self.device, self.backend)
        return Comm(self.rank, self.world, self.device, self.backend,
                    group=dist.new_group(ranks=list(range(self.world))))

    # -------------------------------------------------------------- p2p
    def setup_p2p_edges(self, edges) -> None:
        """Create one process group per DIRECTED hand-off edge (src, dst).

        Every rank must call this with the same edge list (it is collective).
        With one communicator per direction, each NCCL/RCCL stream carries only
        sends on one side and receives on the other, so the order in which a
        receiver posts its receives can never deadlock against its own sends
        to the same peer (the G=2 pipeline has traffic both ways between the
        same two ranks).
        """
        self._edge_groups = {}
        if not self.active:
            return
        for (a, b) in sorted(set(edges)):
            self._edge_groups[(a, b)] = dist.new_group(ranks=sorted([a, b]))

    def _group(self, src: int, dst: int):
        return getattr(self, "_edge_groups", {}).get((src, dst))

    def isend(self, t: torch.Tensor, dst: int):
        return dist.isend(t, dst, group=self._group(self.rank, dst))

    def irecv(self, t: torch.Tensor, src: int):
        return dist.irecv(t, src, group=self._group(src, self.rank))

    # -------------------------------------------------------- collectives
    def barrier(self):
        if self.active:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=async_op)

    def all_reduce_max(self, x: float) -> float:
        if not self.active:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def all_reduce_min(self, x: float) -> float:
        if not self.active:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return float(t.item())

    def all_reduce_sum(self, x: float) -> float:
        if not self.active:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if not self.active:
            return obj
        lst = [obj if self.rank == src else None]
        dist.broadcast_object_list(lst, src=src, device=self.device if self.backend == "nccl" else None)
        return lst[0]

    def gather_object(self, obj: Any, dst: int = 0) -> Optional[List[Any]]:
        if not self.active:
            return [obj]
        out = [None] * self.world if self.rank == dst else None
        if self.backend == "nccl":
            # gather_object over NCCL needs device tensors; use all_gather_object for simplicity
            allv = [None] * self.world
            dist.all_gather_object(allv, obj)
            return allv if self.rank == dst else None
        dist.gather_object(obj, out, dst=dst)
        return out

    def all_gather_object(self, obj: Any) -> List[Any]:
        if not self.active:
            return [obj]
        allv = [None] * self.world
        dist.all_gather_object(allv, obj)
        return allv

    def destroy(self):
        if self.active and dist.is_initialized():
            dist.destroy_process_group()
