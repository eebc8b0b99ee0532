"""Model-parallel stage hand-off: deterministic receive program + bounded inbox.

Reference (``/root/reference/utils.py:159-213``): a producer stage parks each
prompt's activations in a shared dict (RAM) or, at the wrap-around boundary
(last GPU -> GPU 0) in disk mode, in ``.npy`` files; the consumer sleep-polls
``prompt2layer`` once a second and copies the entry to its device.  Producers
block while the dict holds ``max_activation_in_cpu`` entries
(``utils.py:178-185``).

Here every stage boundary is an RCCL ``isend`` / ``irecv`` pair over xGMI on a
per-edge communicator, issued by each rank's main thread in an order fixed
before the pass starts (:func:`build_programs`):

* **Ordering.**  All ranks' schedules (shard-major ``(shard, micro-batch)``
  items, or micro-batch-major for resident contiguous stages) are merged into
  one global topological order (a round-robin sweep that advances every rank
  whose input is ready).  A rank posts the receive of an item right before its
  first own item that comes *after the sending item* in that order.  Every
  rank therefore submits its GPU work — receives, computes, sends — in one
  global order in which each RCCL operation only waits for operations earlier
  in it.  So no receive (or send) kernel is ever queued ahead of local work it
  transitively depends on, whatever HIP streams share a hardware queue
  (``GPU_MAX_HW_QUEUES=4``: the compute, copy and RCCL streams do share).
  :func:`simulate_single_queue` checks this on the worst case (each rank's
  operations serialised in ONE in-order queue, sends and receives rendezvous)
  for every plan the tests cover.  Non-wrap edges post at the point of use
  (one item ahead in GPU time, since the host runs ahead); the wrap-around
  edge (round-robin: rank G-1 -> rank 0, consumed one round later) posts right
  after the rank's own send of the same micro-batch one round earlier — the
  rule "receive (shard j+1, b) only after send (j, b) is enqueued".
* **Bounded memory** (:class:`StageInbox`, one per runner, reused across
  calls).  Point-of-use receives land in a ring of ``window`` fixed HBM slots
  (a slot is re-posted only after its previous item's compute and send
  finished — a GPU-side wait on earlier work).  Early (wrap) receives are
  *parked*: up to ``max_parked`` entries in the ``--storage_location`` tier
  (``gpu``: the received HBM buffer itself; ``cpu``: D2H to pooled pinned RAM
  out of a ring slot), overflow in the next tier (gpu -> cpu -> disk), and
  ``disk`` spills every parked entry to ``.npy`` (the reference's wrap-boundary
  disk mode).  ``--max_activation_in_cpu`` is ``max_parked``: the reference's
  back-pressure bound, here a spill threshold instead of a blocked producer
  (blocking a producer stage cannot be made deadlock-free on shared queues).
  Parked entries come back through the runner's own H2D / D2H streams.
"""
from __future__ import annotations

import bisect
import time
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..runtime.activations import ActivationStore


def rx_key(shard: int, mb: int) -> int:
    return shard * 1_000_000 + mb


# ----------------------------------------------------------------------------- program


def rank_items(my_shards: Sequence[Tuple[int, ...]], n_batches: int, mb_major: bool = False,
               start_layer: int = 0) -> List[Tuple[int, int]]:
    """A rank's (local shard, micro-batch) execution order.  ``my_shards``: its non-empty shards;
    shards before ``start_layer`` (a resume point) are skipped."""
    ks = [k for k, sh in enumerate(my_shards) if sh and sh[0] >= start_layer]
    if mb_major:
        return [(k, b) for b in range(n_batches) for k in ks]
    return [(k, b) for k in ks for b in range(n_batches)]


@dataclass
class RankProgram:
    """One rank's hand-off program over its items (indices into ``items``)."""
    rank: int
    items: List[Tuple[int, int]]
    src: List[Optional[int]]                 # rank the item's input comes from (None: local / none)
    dst: List[Optional[int]]                 # rank the item's output goes to (None: local / final)
    posts: List[List[int]] = field(default_factory=list)   # posts[p]: items whose receive is posted before item p
    parked: frozenset = frozenset()          # items whose receive is posted before an earlier item

    def post_index(self, i: int) -> int:
        for p, lst in enumerate(self.posts):
            if i in lst:
                return p
        raise KeyError(i)


def build_programs(plans: Dict[int, object], n_batches: int, mb_major: bool = False,
                   start_layer: int = 0) -> Dict[int, RankProgram]:
    """Per-rank hand-off programs for model-parallel ``plans`` (rank -> ShardPlan, mode "mp").

    Items are merged into a global topological order by sweeping the ranks round-robin and
    advancing each one whose next item has its input (an item of the shard holding the previous
    layer, same micro-batch) already ordered.  A receive is posted before the first own item
    that follows its sending item in that order."""
    ranks = sorted(plans)
    shard_of_layer: Dict[int, Tuple[int, int]] = {}       # layer -> (owner rank, local shard index)
    items: Dict[int, List[Tuple[int, int]]] = {}
    mine: Dict[int, List[Tuple[int, ...]]] = {}
    for r in ranks:
        sh = [s for s in plans[r].my_shards if len(s)]
        mine[r] = sh
        for k, s in enumerate(sh):
            for li in s:
                shard_of_layer[li] = (r, k)
        items[r] = rank_items(sh, n_batches, mb_major, start_layer)
    index = {r: {it: i for i, it in enumerate(items[r])} for r in ranks}

    def dep(r: int, it: Tuple[int, int]) -> Optional[Tuple[int, int]]:
        k, b = it
        first = mine[r][k][0]
        if first == 0 or first == start_layer:
            return None
        r2, k2 = shard_of_layer[first - 1]
        return (r2, index[r2][(k2, b)])

    deps = {r: [dep(r, it) for it in items[r]] for r in ranks}
    order: Dict[Tuple[int, int], int] = {}
    ptr = {r: 0 for r in ranks}
    n = 0
    total = sum(len(items[r]) for r in ranks)
    while n < total:
        progressed = False
        for r in ranks:
            i = ptr[r]
            if i >= len(items[r]):
                continue
            d = deps[r][i]
            if d is None or d in order:
                order[(r, i)] = n
                n += 1
                ptr[r] += 1
                progressed = True
        if not progressed:
            raise RuntimeError("model-parallel schedule has a cyclic stage dependency")

    progs: Dict[int, RankProgram] = {}
    for r in ranks:
        its = items[r]
        src: List[Optional[int]] = []
        dst: List[Optional[int]] = [None] * len(its)
        for i, d in enumerate(deps[r]):
            src.append(d[0] if (d is not None and d[0] != r) else None)
        progs[r] = RankProgram(r, its, src, dst, [[] for _ in its], frozenset())
    for r in ranks:
        for i, d in enumerate(deps[r]):
            if d is not None and d[0] != r:
                progs[d[0]].dst[d[1]] = r
    for r in ranks:
        pos = [order[(r, i)] for i in range(len(items[r]))]      # increasing
        parked = set()
        posts: List[List[Tuple[int, int]]] = [[] for _ in items[r]]
        for i, d in enumerate(deps[r]):
            if d is None or d[0] == r:
                continue
            p = bisect.bisect_left(pos, order[d])                # own items ordered before the sender
            assert p <= i
            posts[p].append((order[d], i))
            if p < i:
                parked.add(i)
        progs[r].posts = [[i for _, i in sorted(lst)] for lst in posts]
        progs[r].parked = frozenset(parked)
    return progs


def program_ops(prog: RankProgram) -> List[Tuple]:
    """The rank's GPU operations in submission order: ("recv", src, dst, seq), ("compute", i),
    ("send", src, dst, seq); ``seq`` numbers the operations of one directed edge."""
    ops: List[Tuple] = []
    seq: Dict[Tuple[int, int], int] = defaultdict(int)
    r = prog.rank
    for p in range(len(prog.items)):
        for c in prog.posts[p]:
            e = (prog.src[c], r)
            ops.append(("recv", e[0], e[1], seq[("r",) + e]))
            seq[("r",) + e] += 1
        ops.append(("compute", p))
        if prog.dst[p] is not None:
            e = (r, prog.dst[p])
            ops.append(("send", e[0], e[1], seq[("s",) + e]))
            seq[("s",) + e] += 1
    return ops


def simulate_single_queue(ops_by_rank: Dict[int, Sequence[Tuple]]) -> Tuple[bool, Dict[int, int]]:
    """Worst-case execution model: each rank runs its operations in ONE in-order queue (every
    HIP stream of the rank mapped to the same hardware queue); a send and the receive it matches
    (same directed edge, same sequence number) complete together once both are at the head of
    their queues; anything else completes at the head.  -> (all completed, ops left per rank).

    Extra queues only remove ordering constraints, so a program that completes here cannot
    deadlock on any stream -> hardware-queue mapping."""
    head = {r: 0 for r in ops_by_rank}
    ops = {r: list(v) for r, v in ops_by_rank.items()}
    while True:
        progressed = False
        for r in ops:
            while head[r] < len(ops[r]):
                op = ops[r][head[r]]
                if op[0] == "compute" or op[0] == "other":
                    head[r] += 1
                    progressed = True
                    continue
                kind, a, b, s = op
                peer = b if kind == "send" else a
                want = ("recv" if kind == "send" else "send", a, b, s)
                if peer in ops and head[peer] < len(ops[peer]) and tuple(ops[peer][head[peer]]) == want:
                    head[r] += 1
                    head[peer] += 1
                    progressed = True
                    continue
                break
        if not progressed:
            break
    left = {r: len(ops[r]) - head[r] for r in ops}
    return all(v == 0 for v in left.values()), left


# ------------------------------------------------------------------------------- inbox


def host_wait(work, timeout_s: float = 1800.0, cuda: bool = True) -> None:
    """Block the host until a send/recv work completed.  RCCL's ``wait()`` is a stream wait, so
    poll its completion; gloo's ``is_completed()`` only turns true inside ``wait()``, which
    blocks."""
    if not cuda:
        work.wait()
        return
    t0 = time.perf_counter()
    while not work.is_completed():
        if time.perf_counter() - t0 > timeout_s:
            raise TimeoutError(f"model-parallel hand-off not completed within {timeout_s:.0f}s")
        time.sleep(5e-5)


class _Slot:
    __slots__ = ("buf", "event", "send")

    def __init__(self):
        self.buf = None            # flat tensor
        self.event = None          # cuda event: last reader on the compute / D2H stream
        self.send = None           # send work of the item that used the slot (output may alias it)


class StageInbox:
    """Receive side of the model-parallel hand-off; one per runner, reused by every call.

    ``post(key, src, shape, park)`` issues the receive (main thread, program order);
    ``get(key)`` returns the device tensor with the current stream ordered after it;
    ``release(key, send_work)`` marks the consuming item enqueued (its ring slot becomes
    reusable once that compute — and the send of its output — finished)."""

    def __init__(self, comm, device, dtype: torch.dtype, storage: str, disk_folder: str, tag: str,
                 window: int = 2, max_parked: int = 100, h2d_stream=None, d2h_stream=None,
                 timeout_s: float = 1800.0):
        if storage not in ("gpu", "cpu", "disk"):
            raise ValueError(f"storage_location must be gpu/cpu/disk, got {storage!r}")
        self.comm, self.dev, self.dtype = comm, torch.device(device), dtype
        self.cuda = self.dev.type == "cuda"
        self.storage = storage
        self.window = max(1, int(window))
        self.max_parked = max(0, int(max_parked))
        self.timeout_s = timeout_s
        self.rx_stream = torch.cuda.Stream(self.dev) if self.cuda else None
        self.h2d, self.d2h = h2d_stream, d2h_stream
        self.disk_folder, self.tag = disk_folder, tag
        self._stores: Dict[str, ActivationStore] = {}
        self.slots = [_Slot() for _ in range(self.window)]
        self.slot_bytes = 0
        self._next = 0
        self.entries: Dict[int, tuple] = {}
        self.parked_count = {"gpu": 0, "cpu": 0, "disk": 0}
        self.reset_stats()

    # ----------------------------------------------------------------- stats
    def reset_stats(self) -> None:
        self.stats = {"posted": 0, "parked": 0, "parked_gpu": 0, "parked_cpu": 0, "parked_disk": 0,
                      "max_parked_gpu": 0, "max_parked_cpu": 0, "max_parked_disk": 0,
                      "max_ring_in_use": 0, "max_parked_bytes_gpu": 0, "max_parked_bytes_cpu": 0}
        self._ring_in_use = 0
        self._parked_bytes = {"gpu": 0, "cpu": 0, "disk": 0}

    def _store(self, tier: str) -> ActivationStore:
        st = self._stores.get(tier)
        if st is None:
            st = ActivationStore(tier, self.dev, self.disk_folder, tag=f"rx{self.tag}",
                                 h2d_stream=self.h2d, d2h_stream=self.d2h)
            self._stores[tier] = st
        return st

    def pinned_pool_bytes(self) -> int:
        return sum(st.pooled_bytes() for st in self._stores.values())

    def ring_bytes(self) -> int:
        return self.slot_bytes * len(self.slots) if self.slots[0].buf is not None else 0

    # ----------------------------------------------------------------- calls
    def begin_call(self, max_bytes: int) -> None:
        """Size the ring for this call's largest received state (grown only: the previous call
        is fully synchronized when a new one starts)."""
        self.reset_stats()
        if max_bytes > self.slot_bytes or self.slots[0].buf is None:
            self.slot_bytes = max(max_bytes, self.slot_bytes, 1)
            for s in self.slots:
                s.buf = None
            for s in self.slots:
                s.buf = torch.empty(self.slot_bytes, dtype=torch.uint8, device=self.dev)
                s.event = s.send = None
        self._next = 0

    def end_call(self) -> None:
        if self.entries:
            raise RuntimeError(f"stage inbox: {len(self.entries)} received activations never consumed")
        for s in self.slots:
            s.event = s.send = None
        for st in self._stores.values():
            st.clear()
            st.trim()

    # ------------------------------------------------------------------ post
    def _tier(self) -> str:
        """Where an early (parked) receive lives: the storage tier while it holds fewer than
        ``max_parked`` entries, else the next slower one (gpu -> cpu -> disk)."""
        chain = {"gpu": ("gpu", "cpu", "disk"), "cpu": ("cpu", "disk"), "disk": ("disk",)}[self.storage]
        for t in chain[:-1]:
            if self.parked_count[t] < self.max_parked:
                return t
        return chain[-1]

    def _take_slot(self) -> Tuple[int, _Slot]:
        i = self._next
        self._next = (self._next + 1) % len(self.slots)
        s = self.slots[i]
        # the slot's previous item: its compute / D2H (event) and the send of its output
        if self.cuda:
            if s.event is not None:
                self.rx_stream.wait_event(s.event)
            if s.send is not None:
                with torch.cuda.stream(self.rx_stream):
                    s.send.wait()
        elif s.send is not None:
            s.send.wait()
        s.event = s.send = None
        return i, s

    def post(self, key: int, src: int, shape: Tuple[int, ...], park: bool) -> None:
        n = 1
        for d in shape:
            n *= int(d)
        nbytes = n * torch.empty((), dtype=self.dtype).element_size()
        self.stats["posted"] += 1
        if park:
            tier = self._tier()
            self.parked_count[tier] += 1
            self.stats["parked"] += 1
            self.stats[f"parked_{tier}"] += 1
            self.stats[f"max_parked_{tier}"] = max(self.stats[f"max_parked_{tier}"], self.parked_count[tier])
            self._parked_bytes[tier] += nbytes
            if tier != "disk":
                k = f"max_parked_bytes_{tier}"
                self.stats[k] = max(self.stats[k], self._parked_bytes[tier])
            if tier == "gpu" or not self.cuda:
                # HBM tier (or a CPU rank): the received buffer itself is the parked entry
                if self.cuda:
                    with torch.cuda.stream(self.rx_stream):
                        t = torch.empty(shape, dtype=self.dtype, device=self.dev)
                        w = self.comm.irecv(t, src)
                else:
                    t = torch.empty(shape, dtype=self.dtype, device=self.dev)
                    w = self.comm.irecv(t, src)
                    if tier == "disk":
                        w.wait()
                        self._store("disk").put(key, t)
                        self.entries[key] = ("store", "disk", None, nbytes)
                        return
                self.entries[key] = ("dev", tier, (w, t), nbytes)
                return
            # cpu / disk tier: receive into a ring slot, D2H it out (the slot is free once copied)
            i, s = self._take_slot()
            view = s.buf[:nbytes].view(self.dtype).view(shape)
            st = self._store(tier)
            with torch.cuda.stream(self.rx_stream):
                w = self.comm.irecv(view, src)
                w.wait()                                 # rx stream after the receive
                st.put(key, view)                        # D2H on the runner's D2H stream after rx
            ev = torch.cuda.Event()
            ev.record(st.d2h)
            s.event = ev
            self.entries[key] = ("store", tier, None, nbytes)
            return
        i, s = self._take_slot()
        view = s.buf[:nbytes].view(self.dtype).view(shape)
        if self.cuda:
            with torch.cuda.stream(self.rx_stream):
                w = self.comm.irecv(view, src)
        else:
            w = self.comm.irecv(view, src)
        self._ring_in_use += 1
        self.stats["max_ring_in_use"] = max(self.stats["max_ring_in_use"], self._ring_in_use)
        self.entries[key] = ("ring", i, (w, view), nbytes)

    # ------------------------------------------------------------------- get
    def prefetch(self, key: int) -> None:
        """Start the H2D of a parked cpu / disk entry ahead of its use."""
        e = self.entries.get(key)
        if e is not None and e[0] == "store":
            self._store(e[1]).prefetch(key)

    def get(self, key: int) -> torch.Tensor:
        e = self.entries.get(key)
        if e is None:
            raise KeyError(f"stage inbox: no receive posted for key {key}")
        kind = e[0]
        if kind == "store":
            del self.entries[key]
            self.parked_count[e[1]] -= 1
            self._parked_bytes[e[1]] -= e[3]
            return self._store(e[1]).get(key)
        w, t = e[2]
        w.wait()                                          # current stream after the receive
        if kind == "dev":
            self.parked_count[e[1]] -= 1
            self._parked_bytes[e[1]] -= e[3]
            del self.entries[key]
            if self.cuda:
                t.record_stream(torch.cuda.current_stream(self.dev))
        return t

    def release(self, key: int, send_work=None) -> None:
        """The consumer of ``key`` (and the send of its output, if any) is enqueued."""
        e = self.entries.pop(key, None)
        if e is None:
            return
        if e[0] == "ring":
            s = self.slots[e[1]]
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.dev))
                s.event = ev
            s.send = send_work
            self._ring_in_use -= 1

    def host_wait(self, work) -> None:
        host_wait(work, self.timeout_s, self.cuda)

    def abort(self) -> None:
        """Forget this call's receives after a failed pass (the job is going down)."""
        self.entries.clear()
        self.parked_count = {"gpu": 0, "cpu": 0, "disk": 0}
        self._parked_bytes = {"gpu": 0, "cpu": 0, "disk": 0}
        self._ring_in_use = 0
        for s in self.slots:
            s.event = s.send = None

    def close(self) -> None:
        self.entries.clear()
        for st in self._stores.values():
            st.close()
        self._stores.clear()
        for s in self.slots:
            s.buf = s.event = s.send = None
