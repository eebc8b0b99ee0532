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
        # data-parallel weight gathers on the native RCCL communicator (--dp_gather_comm native):
        # dup() then builds a parallel/native_comm.NativeRcclComm
        self.gather_native = False

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
        if self.gather_native and self.device.type == "cuda":
            from .native_comm import NativeRcclComm
            return NativeRcclComm(self)
        if not self.active:
            return Comm(self.rank, self.world, self.device, self.backend)
        return Comm(self.rank, self.world, self.device, self.backend,
                    group=dist.new_group(ranks=list(range(self.world))))

    def warmup(self) -> None:
        """One tiny collective on this communicator (RCCL allocates its buffers at the first one),
        so memory measured afterwards includes them."""
        if not self.active:
            return
        dev = self.device if self.backend == "nccl" else torch.device("cpu")
        t = torch.zeros(1, device=dev)
        dist.all_reduce(t, group=self.group)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def warmup_gather(self, dst: int = 0) -> None:
        """The operations of :meth:`gather_scores` once, tiny: a header all-gather on the default
        group and a send / receive from every rank to ``dst`` (RCCL sets up the default group's P2P
        channels at the first one).  Run at runner construction, before a ``--max_vram_gb`` plan
        measures device memory, so the first score gather after a pass allocates nothing the plan
        did not count."""
        if not self.active:
            return
        dev = self.device if self.backend == "nccl" else torch.device("cpu")
        t = torch.zeros(1, dtype=torch.int64, device=dev)
        allh = torch.empty(self.world, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(allh, t)
        if self.rank != dst:
            dist.send(t, dst)
        else:
            for r in range(self.world):
                if r != dst:
                    dist.recv(t, r)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

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

    def warmup_p2p(self) -> None:
        """One tiny send / receive on every directed hand-off edge (RCCL allocates a P2P channel's
        buffers at its first use), so device memory measured afterwards includes them (ADVICE r2:
        a VRAM cap).  Every rank walks the edges in one global order and completes each edge it is
        on before the next (device-synchronised): the first edge not yet done always has both of
        its ranks at it, so the chain cannot deadlock."""
        if not self.active or not getattr(self, "_edge_groups", None):
            return
        dev = self.device if self.backend == "nccl" else torch.device("cpu")
        t = torch.zeros(1, device=dev)
        for (a, b) in sorted(self._edge_groups):
            if self.rank == a:
                self.isend(t, b).wait()
            elif self.rank == b:
                self.irecv(t, a).wait()
            else:
                continue
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)

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

    def gather_scores(self, outs: List[Optional["np.ndarray"]], dst: int = 0) -> Optional[List[list]]:
        """Every rank's score arrays (``[n_s, k, V]`` fp16 each; ``None`` for prompts a rank does not
        own) to ``dst`` -> per-rank lists on ``dst``, None elsewhere.

        Each rank sends ONE packed fp16 tensor plus its shapes, point-to-point to ``dst``, after a
        fixed-size header (array count, element count) all-gathered on the default communicator.
        A rank other than ``dst`` stages only its own scores (on the device for ``nccl``); ``dst``
        receives rank by rank into one staging buffer.  Nothing is pickled and nothing grows with
        the world size except ``dst``'s result (``all_gather_object`` sent every rank's pickled
        scores to every rank).  ``self.gather_stats`` records this rank's bytes."""
        import numpy as np
        if not self.active:
            return [outs]
        on_dev = self.backend == "nccl"
        dev = self.device if on_dev else torch.device("cpu")
        shapes = [(-1, -1, -1) if o is None else tuple(int(x) for x in o.shape) for o in outs]
        total = sum(int(np.prod(sh)) for sh in shapes if sh[0] >= 0)
        hdr = torch.tensor([len(outs), total], dtype=torch.int64, device=dev)
        allh = torch.empty(2 * self.world, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(allh, hdr)
        allh = allh.cpu().view(self.world, 2).tolist()
        self.gather_stats = {"sent_bytes": 0, "staged_bytes": 0, "received_bytes": 0}
        if self.rank != dst:
            if allh[self.rank][0]:
                sh = torch.tensor(shapes, dtype=torch.int64, device=dev)
                flat = (np.concatenate([o.reshape(-1) for o in outs if o is not None]) if total
                        else np.zeros(0, np.float16))
                data = torch.from_numpy(np.ascontiguousarray(flat, dtype=np.float16)).to(dev)
                dist.send(sh, dst)
                if total:
                    dist.send(data, dst)
                self.gather_stats.update(sent_bytes=total * 2, staged_bytes=total * 2)
            return None
        res: List[list] = []
        cap = max([t for r, (n, t) in enumerate(allh) if r != dst] or [0])
        stage = torch.empty(cap, dtype=torch.float16, device=dev) if cap else None
        self.gather_stats["staged_bytes"] = cap * 2
        for r, (n, t) in enumerate(allh):
            if r == dst:
                res.append(list(outs))
                continue
            if not n:
                res.append([])
                continue
            sh = torch.empty(n, 3, dtype=torch.int64, device=dev)
            dist.recv(sh, r)
            sh = sh.cpu().tolist()
            host = None
            if t:
                dist.recv(stage[:t], r)
                host = stage[:t].cpu().numpy()
                self.gather_stats["received_bytes"] += t * 2
            lst, off = [], 0
            for a, b, c in sh:
                if a < 0:
                    lst.append(None)
                    continue
                m = a * b * c
                lst.append(host[off:off + m].reshape(a, b, c).copy())
                off += m
            res.append(lst)
        return res

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


class LoopbackHub:
    """Shared state of a :class:`LoopbackComm` world: ``world`` ranks as threads of one process.

    Point-to-point messages are matched per directed edge in posting order (the RCCL / NCCL
    rule) and transferred as soon as both sides are posted, whichever posts second issuing the
    copy (CUDA: on the receive's posting stream, after the send's event — no host waits).
    Every send / receive a rank posts is appended to ``log[rank]`` as
    ``("send" | "recv", src, dst, seq)`` in submission order, which
    :func:`~.pipeline.simulate_single_queue` can replay."""

    def __init__(self, world: int, timeout_s: float = 300.0):
        import threading
        from collections import defaultdict
        self.world = world
        self.timeout_s = timeout_s
        self.cv = threading.Condition()
        self.sends = defaultdict(dict)           # (src, dst) -> seq -> _LoopOp (send side)
        self.recvs = defaultdict(dict)           # (src, dst) -> seq -> _LoopOp (receive side)
        self.n_send = defaultdict(int)
        self.n_recv = defaultdict(int)
        self.log: List[List[tuple]] = [[] for _ in range(world)]
        self._coll: dict = {}
        self._coll_round = [0] * world
        self._dup_gen = [0] * world
        self._children: dict = {}

    def child(self, rank: int) -> "LoopbackHub":
        """The hub of every rank's n-th ``dup()`` (one shared child per generation)."""
        with self.cv:
            gen = self._dup_gen[rank]
            self._dup_gen[rank] += 1
            if gen not in self._children:
                self._children[gen] = LoopbackHub(self.world, self.timeout_s)
            return self._children[gen]

    def exchange(self, rank: int, obj: Any) -> List[Any]:
        """All ranks deposit ``obj``; every rank gets the list (a blocking collective)."""
        with self.cv:
            rnd = self._coll_round[rank]
            self._coll_round[rank] += 1
            slot = self._coll.setdefault(rnd, {})
            slot[rank] = obj
            self.cv.notify_all()
            if not self.cv.wait_for(lambda: len(slot) == self.world, timeout=self.timeout_s):
                raise TimeoutError("loopback collective timed out")
            return [slot[r] for r in range(self.world)]

    def _transfer(self, snd: "_LoopOp", rcv: "_LoopOp") -> None:
        """Both sides posted: copy (caller holds ``cv``)."""
        if rcv.t.is_cuda:
            s = rcv.stream
            if snd.ev is not None:
                s.wait_event(snd.ev)
            with torch.cuda.stream(s):
                rcv.t.copy_(snd.t, non_blocking=True)
            snd.t.record_stream(s)
            ev = torch.cuda.Event()
            ev.record(s)
            snd.done_ev = rcv.done_ev = ev
        else:
            rcv.t.copy_(snd.t)
        snd.done = rcv.done = True
        self.cv.notify_all()

    def post(self, kind: str, edge, t: torch.Tensor) -> "_LoopWork":
        op = _LoopOp(t)
        with self.cv:
            if kind == "send":
                seq = self.n_send[edge]
                self.n_send[edge] += 1
                self.sends[edge][seq] = op
                self.log[edge[0]].append(("send", edge[0], edge[1], seq))
                peer = self.recvs[edge].pop(seq, None)
                if peer is not None:
                    self.sends[edge].pop(seq)
                    self._transfer(op, peer)
            else:
                seq = self.n_recv[edge]
                self.n_recv[edge] += 1
                self.recvs[edge][seq] = op
                self.log[edge[1]].append(("recv", edge[0], edge[1], seq))
                peer = self.sends[edge].pop(seq, None)
                if peer is not None:
                    self.recvs[edge].pop(seq)
                    self._transfer(peer, op)
        return _LoopWork(self, op, f"{kind} {edge}#{seq}")


class _LoopOp:
    def __init__(self, t: torch.Tensor):
        self.t = t
        self.ev = None
        self.stream = None
        if t.is_cuda:
            self.stream = torch.cuda.current_stream(t.device)
            self.ev = torch.cuda.Event()
            self.ev.record(self.stream)
        self.done = False
        self.done_ev = None


class _LoopWork:
    """Work of a loopback send / receive.  CUDA: ``wait()`` orders the CURRENT stream after the
    transfer (the host only waits until the peer has posted); CPU: blocks until copied."""

    def __init__(self, hub: LoopbackHub, op: _LoopOp, name: str):
        self.hub, self.op, self.name = hub, op, name

    def wait(self) -> bool:
        hub, op = self.hub, self.op
        with hub.cv:
            if not hub.cv.wait_for(lambda: op.done, timeout=hub.timeout_s):
                raise TimeoutError(f"loopback {self.name}: peer never posted")
        if op.done_ev is not None:
            torch.cuda.current_stream(op.t.device).wait_event(op.done_ev)
        return True

    def is_completed(self) -> bool:
        op = self.op
        if not op.done:
            return False
        return op.done_ev is None or op.done_ev.query()


class _DoneWork:
    """Work of a loopback collective: ordered on the issuing stream when it returns."""

    def wait(self) -> bool:
        return True

    def is_completed(self) -> bool:
        return True


class LoopbackComm(Comm):
    """``Comm`` for ``world`` ranks as threads of one process (tests / rehearsal): sends and
    receives are device copies ordered by events (no RCCL), collectives go through the hub."""

    def __init__(self, hub: LoopbackHub, rank: int, device=None):
        super().__init__(rank, hub.world, device, "loopback")
        self.hub = hub

    def dup(self) -> "LoopbackComm":
        """Same thread ranks, own collective sequence (the data-parallel gathers)."""
        return LoopbackComm(self.hub.child(self.rank), self.rank, self.device)

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """``all_gather_into_tensor`` by device copies: every rank's ``inp`` lands in
        ``out[r * n:(r + 1) * n]`` of every rank (``inp`` may already be this rank's place in
        ``out``).  Like RCCL's, completion on the calling stream also covers the peers' reads of
        this rank's ``inp``, so the caller may overwrite it after its stream passes this point:
        the ranks exchange (input, ready event), copy the peers' slices on their current streams,
        then exchange and wait for the copy events.  The host blocks until every rank has posted
        (as gloo does); no device wait."""
        n = inp.numel()
        flat = out.view(-1)
        cuda = inp.is_cuda
        st = torch.cuda.current_stream(inp.device) if cuda else None
        ev = None
        if cuda:
            ev = torch.cuda.Event()
            ev.record(st)
        peers = self.hub.exchange(self.rank, (inp, ev))
        for r, (t, e) in enumerate(peers):
            dst = flat[r * n:(r + 1) * n]
            if r == self.rank:
                if dst.data_ptr() != t.data_ptr():
                    dst.copy_(t, non_blocking=cuda)
                continue
            if cuda:
                st.wait_event(e)
            dst.copy_(t, non_blocking=cuda)
        done = None
        if cuda:
            done = torch.cuda.Event()
            done.record(st)
        for r, e in enumerate(self.hub.exchange(self.rank, done)):
            if cuda and r != self.rank:
                st.wait_event(e)
        return _DoneWork()

    def setup_p2p_edges(self, edges) -> None:
        self._edge_groups = {}

    def isend(self, t: torch.Tensor, dst: int):
        return self.hub.post("send", (self.rank, dst), t)

    def irecv(self, t: torch.Tensor, src: int):
        return self.hub.post("recv", (src, self.rank), t)

    def barrier(self):
        self.hub.exchange(self.rank, None)

    def warmup(self) -> None:
        pass

    def warmup_gather(self, dst: int = 0) -> None:
        pass

    def all_reduce_max(self, x: float) -> float:
        return max(self.hub.exchange(self.rank, x))

    def all_reduce_min(self, x: float) -> float:
        return min(self.hub.exchange(self.rank, x))

    def all_reduce_sum(self, x: float) -> float:
        return sum(self.hub.exchange(self.rank, x))

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        return self.hub.exchange(self.rank, obj)[src]

    def gather_object(self, obj: Any, dst: int = 0) -> Optional[List[Any]]:
        allv = self.hub.exchange(self.rank, obj)
        return allv if self.rank == dst else None

    def gather_scores(self, outs, dst: int = 0):
        """Threads share the host arrays: dst takes every rank's list as is."""
        return self.gather_object(list(outs), dst)

    def all_gather_object(self, obj: Any) -> List[Any]:
        return self.hub.exchange(self.rank, obj)

    def destroy(self):
        pass
