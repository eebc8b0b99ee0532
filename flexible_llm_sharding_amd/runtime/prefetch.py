"""Shard prefetcher: host (pinned / file) -> rotating HBM weight slots.

Reference: each shard's layers are loaded synchronously before compute
(``/root/reference/utils.py:230-233``) and unloaded to ``meta`` with
``empty_cache`` afterwards (``utils.py:299-302``) — compute and weight I/O
never overlap.

Here HBM holds ``n_slots`` fixed weight slots (allocated once; no per-shard
free; the engine uses 3, or 2 = a double buffer under a VRAM cap).  The next
shards are copied into the other slots on a dedicated copy stream while shard
``k`` computes; the compute stream waits on
a per-shard *ready* event, and the copy stream waits on the slot's *free*
event recorded when the compute stream finished with its previous occupant.
File-backed sources (:class:`~.stream.FileLayerSource`) are streamed by a
loader thread through the native streamer's pinned chunk ring straight into
the slot, so disk reads, PCIe DMA and compute all overlap.

``resident=True`` gives every shard its own slot and never evicts (the whole
model stays in the 288 GB HBM — BASELINE config 5).  ``keep`` does that for a
subset (``--hbm_cache_gb``: as many shards as the budget holds, spread evenly
over the pass by :func:`choose_kept_shards`), the rest keep streaming: each
streamed load then has the kept shards' compute to hide under.

Tiny shards (the final RMSNorm of a ``layer_num_per_shard=1`` plan: 16 KB) get a
buffer of their own instead of a full slot, and the full-size shards take the
slots round-robin in their own order: the LM head then loads while the last
decoder layer computes instead of after it (a 0.5 GB copy the GPU waited for
at the end of every 70B pass, ``profiles/r2_trace``).  The round-robin runs on
across calls (``epoch``: call e's i-th full-size shard is the (e * n_big + i)-th
load), so with ``n_slots`` slots the engine can prefetch ``n_slots - 1`` shards
ahead straight across a call boundary: the slot a shard lands in was always
last used ``n_slots`` loads earlier, by a shard that is already released.
"""
from __future__ import annotations

import threading
import time
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..models.layout import ALIGN_BYTES, layer_kind
from . import hostmem
from .weights import LayerSource


def _align(n: int) -> int:
    return (n + ALIGN_BYTES - 1) // ALIGN_BYTES * ALIGN_BYTES


def choose_kept_shards(sizes: Sequence[int], budget: int) -> List[int]:
    """Shards to keep resident under ``budget`` bytes, spread evenly over the pass (a kept
    shard every ~total/budget shards), so the streamed loads between them stay evenly spaced."""
    total = sum(sizes)
    if budget <= 0 or total <= 0:
        return []
    if budget >= total:
        return list(range(len(sizes)))
    f, acc, left, keep = budget / total, 0.0, budget, []
    for k, nb in enumerate(sizes):
        acc += f
        if acc >= 1.0 and nb <= left:
            keep.append(k)
            left -= nb
            acc -= 1.0
    return keep


class ShardPrefetcher:
    # transform of a freshly loaded decoder layer (its weight views), enqueued on the copy stream
    # before the load's ready event: the engine folds the input RMSNorm into W_qkv here
    # (models.llama.fold_layer_norms), so a resident / kept shard is folded exactly once
    on_load = None

    def _loaded(self, name: str, views: Dict[str, torch.Tensor]) -> None:
        if self.on_load is not None and layer_kind(name) == "decoder":
            self.on_load(views)

    def __init__(self, source: LayerSource, layer_names: Sequence[str],
                 shards: Sequence[Tuple[int, ...]], device, n_slots: int = 2,
                 resident: bool = False, dtype=torch.float16, keep: Optional[Sequence[int]] = None):
        self.src = source
        self.names = list(layer_names)
        self.shards = [tuple(s) for s in shards]
        self.dev = torch.device(device)
        self.cuda = self.dev.type == "cuda"
        self.dtype = dtype
        self.resident = resident
        # shards that stay in HBM after their first load (all of them when resident)
        self._sticky = set(range(len(self.shards))) if resident else set(keep or ())
        sizes = [self.shard_bytes(k) for k in range(len(self.shards))]
        n_rot_slots = max(1, min(n_slots, len(self.shards) or 1))
        # shards that own a buffer instead of a rotating slot: kept (sticky) shards; with 3+ slots
        # every shard without a decoder layer (70B lnps=1: the 0.5 GB embedding and LM head; for
        # large-vocab models like Llama-3.1-8B they are the LARGEST shards), so the
        # rotation holds only decoder shards and the lookahead reaches the next call's first layer
        # while the second-to-last one still computes (the last, pruned layer is too short to hide
        # it); below 3 slots only shards under 1/32 of a decoder shard (the final norm: 16 KB)
        aux = [all(layer_kind(self.names[i]) != "decoder" for i in sh) for sh in self.shards]
        dec = [nb for k, nb in enumerate(sizes) if k not in self._sticky and not aux[k]]
        ref = max(dec) if dec else max([nb for k, nb in enumerate(sizes) if k not in self._sticky] or sizes or [0])
        many = len(self.shards) > n_rot_slots
        own = []
        for k, nb in enumerate(sizes):
            o = k in self._sticky
            if not resident and not o and many:
                o = (aux[k] and n_rot_slots >= 3) or nb <= min(ref // 32, 64 << 20)
            own.append(o)
        streamed = [nb for k, nb in enumerate(sizes) if not own[k]]
        self.slot_bytes = max(streamed or sizes) if sizes else 0
        self.n_slots = max(1, len(self.shards)) if resident else n_rot_slots
        if resident:
            self._slot_sizes = list(sizes)
            self._slot_map = list(range(len(self.shards)))
        else:
            self._slot_sizes = [self.slot_bytes] * self.n_slots
            self._slot_map, big = [], 0
            self._big_idx: List[int] = []          # index among the rotating shards, -1: own buffer
            for k, nb in enumerate(sizes):
                if own[k]:
                    self._slot_map.append(len(self._slot_sizes))
                    self._slot_sizes.append(nb)
                    self._big_idx.append(-1)
                else:
                    self._slot_map.append(big % self.n_slots)
                    self._big_idx.append(big)
                    big += 1
            self._n_big = big
        self.epoch = 0                              # calls completed (rotates the slot round-robin)
        self._slots: List[Optional[torch.Tensor]] = [None] * len(self._slot_sizes)
        self._free_ev: List[Optional[torch.cuda.Event]] = [None] * len(self._slot_sizes)
        self._pending: Dict[int, Future] = {}
        self._ready: Dict[int, Tuple[Optional[torch.cuda.Event], Dict[str, Dict[str, torch.Tensor]], int]] = {}
        self._loaded_resident = set()
        self.copy_stream = torch.cuda.Stream(self.dev) if self.cuda else None
        needs_thread = self.cuda and any(source.host_buffer(self.names[i]) is None
                                         for sh in self.shards for i in sh)
        self._pool = ThreadPoolExecutor(1, thread_name_prefix="fls-loader") if needs_thread else None
        self._staging: List[Optional[torch.Tensor]] = [None, None]
        self._staging_ev: List[Optional[torch.cuda.Event]] = [None, None]
        self._staging_i = 0
        # stats
        self.bytes_h2d = 0
        self.wait_seconds = 0.0
        self._stall_ev: List[Tuple[torch.cuda.Event, torch.cuda.Event]] = []
        self.load_seconds = 0.0
        self.lock = threading.Lock()

    # ------------------------------------------------------------ helpers
    def shard_bytes(self, k: int) -> int:
        return sum(_align(self.src.nbytes(self.names[i])) for i in self.shards[k])

    def slot_of(self, k: int, epoch: Optional[int] = None) -> int:
        if self.resident or self._big_idx[k] < 0:
            return self._slot_map[k]
        e = self.epoch if epoch is None else epoch
        return (self._big_idx[k] + e * self._n_big) % self.n_slots

    def _slot(self, s: int) -> torch.Tensor:
        if self._slots[s] is None:
            # exact-size hipMalloc outside the caching allocator: the slots live for the whole run,
            # and a slot first touched by the loader thread would otherwise sit in the copy
            # stream's private pool
            self._slots[s] = hostmem.alloc_device(max(1, self._slot_sizes[s]), self.dev) if self.cuda else \
                torch.empty(max(1, self._slot_sizes[s]), dtype=torch.uint8, device=self.dev)
        return self._slots[s]

    def planned_hbm_bytes(self) -> int:
        """Bytes of every weight slot once allocated (they are allocated on first use)."""
        return sum(self._slot_sizes)

    def hbm_bytes(self) -> int:
        return sum(t.numel() for t in self._slots if t is not None)

    def _stage_buf(self, nbytes: int) -> Tuple[torch.Tensor, int]:
        i = self._staging_i
        self._staging_i ^= 1
        if self._staging_ev[i] is not None:
            self._staging_ev[i].synchronize()          # previous DMA out of this buffer done
        b = self._staging[i]
        if b is None or b.numel() < nbytes:
            self._staging[i] = b = hostmem.alloc_host(max(nbytes, self.max_layer_bytes()), pinned=True)
        return b, i

    def max_layer_bytes(self) -> int:
        return max(self.src.nbytes(n) for n in self.names)

    # -------------------------------------------------------------- load
    def _load(self, k: int, epoch: Optional[int] = None):
        t0 = time.perf_counter()
        s = self.slot_of(k, epoch)
        views: Dict[str, Dict[str, torch.Tensor]] = {}
        if not self.cuda:
            for i in self.shards[k]:
                name = self.names[i]
                hb = self.src.host_buffer(name)
                if hb is None:
                    hb = torch.empty(self.src.nbytes(name), dtype=torch.uint8)
                    self.src.read_into(name, hb)
                views[name] = self.src.layout(name).views(hb, self.dtype)
            self.load_seconds += time.perf_counter() - t0
            return None, views, s
        slot = self._slot(s)
        ev = torch.cuda.Event()
        with torch.cuda.stream(self.copy_stream):
            if self._free_ev[s] is not None:
                self.copy_stream.wait_event(self._free_ev[s])
            off = 0
            for i in self.shards[k]:
                name = self.names[i]
                nb = self.src.nbytes(name)
                dst = slot[off:off + nb]
                hb = self.src.host_buffer(name)
                if hb is None and hasattr(self.src, "stream_into"):
                    self.src.stream_into(name, dst, self.copy_stream)
                elif hb is None:
                    stage, si = self._stage_buf(nb)
                    self.src.read_into(name, stage)
                    dst.copy_(stage[:nb], non_blocking=True)
                    e = torch.cuda.Event()
                    e.record(self.copy_stream)
                    self._staging_ev[si] = e
                else:
                    dst.copy_(hb[:nb], non_blocking=True)
                views[name] = self.src.layout(name).views(dst, self.dtype)
                self._loaded(name, views[name])
                off += _align(nb)
                self.bytes_h2d += nb
            ev.record(self.copy_stream)
        self.load_seconds += time.perf_counter() - t0
        return ev, views, s

    def prefetch(self, k: int, epoch: Optional[int] = None) -> None:
        """Start loading shard ``k`` (of call ``epoch``: default the current one; the engine
        passes ``epoch + 1`` for the next call's first shards)."""
        if k < 0 or k >= len(self.shards):
            return
        with self.lock:
            if k in self._ready or k in self._pending:
                return
            if k in self._sticky and k in self._loaded_resident:
                return
            if self._pool is not None:
                self._pending[k] = self._pool.submit(self._load, k, epoch)
                return
        r = self._load(k, epoch)
        with self.lock:
            self._ready[k] = r

    def acquire(self, k: int) -> Dict[str, Dict[str, torch.Tensor]]:
        t0 = time.perf_counter()
        self.prefetch(k)
        fut = None
        with self.lock:
            fut = self._pending.pop(k, None)
        if fut is not None:
            r = fut.result()
            with self.lock:
                self._ready[k] = r
        ev, views, _ = self._ready[k]
        if isinstance(ev, list):          # collective works (data-parallel all-gather)
            for w in ev:
                w.wait()
        elif ev is not None:
            cur = torch.cuda.current_stream(self.dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cur)
            cur.wait_event(ev)
            e1.record(cur)
            self._stall_ev.append((e0, e1))
        if k in self._sticky:
            self._loaded_resident.add(k)
        self.wait_seconds += time.perf_counter() - t0
        return views

    def discard_loaded(self) -> None:
        """Forget every loaded or loading shard that was never acquired (after an empty or aborted
        pass).  Their slots are then free for any later load: nothing computes on them, and a
        later copy into the same slot is ordered behind theirs on the copy stream.  Without this a
        shard loaded at epoch e could be overwritten by a load of the next call's round-robin
        before being used."""
        with self.lock:
            pend = list(self._pending.items())
            self._pending.clear()
        for _, f in pend:
            try:
                f.result()
            except Exception:  # noqa: BLE001 - the load is being dropped anyway
                pass
        with self.lock:
            for k in list(self._ready):
                if k not in self._sticky:
                    del self._ready[k]

    def in_rotation(self, k: int) -> bool:
        """Shard k loads into the rotating slots (not a buffer of its own)."""
        return not self.resident and self._big_idx[k] >= 0

    def is_kept_loaded(self, k: int) -> bool:
        """Shard k stays in HBM and is already there (prefetching it is a no-op)."""
        return k in self._sticky and k in self._loaded_resident

    def all_kept_loaded(self) -> bool:
        """Every shard stays in HBM and is there (resident, or an HBM cache holding the model):
        no prefetch has anything to do."""
        return len(self._loaded_resident) == len(self.shards)

    def kept_bytes(self) -> int:
        return sum(self.shard_bytes(k) for k in self._sticky)

    def take_wait_seconds(self) -> float:
        """Host time spent in :meth:`acquire` waiting for loads since the last call."""
        t, self.wait_seconds = self.wait_seconds, 0.0
        return t

    def take_stall_seconds(self) -> float:
        """GPU time the compute stream spent waiting for weight H2D since the last call
        (after a synchronize)."""
        t = sum(a.elapsed_time(b) for a, b in self._stall_ev) / 1e3
        self._stall_ev = []
        return t

    def release(self, k: int) -> None:
        if k in self._sticky:
            return
        with self.lock:
            ent = self._ready.pop(k, None)
        if ent is None:
            return
        _, _, s = ent
        if self.cuda:
            e = torch.cuda.Event()
            e.record(torch.cuda.current_stream(self.dev))
            self._free_ev[s] = e

    def close(self):
        if self._pool is not None:
            self._pool.shutdown(wait=True)
        if self.cuda:
            torch.cuda.synchronize(self.dev)
        # drop the HBM slots (and every view into them): a closed runner holds no weights
        with self.lock:
            self._pending.clear()
            self._ready.clear()
        self._loaded_resident.clear()
        self._slots = [None] * len(self._slot_sizes)
        self._free_ev = [None] * len(self._slot_sizes)


class _LayerViews(dict):
    """One decoder layer's weight views whose MLP half may still be in flight: the attention
    views are filled at acquire, the MLP views on first access (which orders the compute stream
    after the MLP piece's copy).  ``attention_done()`` (models/llama.py, after the O projection)
    hands the attention piece's HBM back to the pool when this is the layer's last use in the
    call (``final_use``, set by the engine)."""

    def __init__(self, pf: "PiecePoolPrefetcher", k: int, name: str, views: Dict[str, torch.Tensor],
                 mlp_keys):
        super().__init__(views)
        self.pf, self.k, self.name = pf, k, name
        self.mlp_keys = frozenset(mlp_keys)
        self.final_use = False

    def __missing__(self, key):
        if key not in self.mlp_keys:
            raise KeyError(key)
        self.update(self.pf._mlp_views(self.k, self.name))
        return dict.__getitem__(self, key)

    def get(self, key, default=None):
        if dict.__contains__(self, key) or key in self.mlp_keys:
            return self[key]
        return default

    def attention_done(self) -> None:
        if self.final_use:
            self.pf._release_attn(self.k)


class PiecePoolPrefetcher(ShardPrefetcher):
    """``--max_vram_gb`` weight streaming at sub-layer granularity (lnps = 1, host-resident
    layers): a decoder layer is an attention piece (ln1/ln2, QKV, O: 0.30 GB for 70B) and an
    MLP piece (gate/up, down: 1.41 GB) — the packed image puts every attention weight first
    (models/layout.py).  HBM holds ONE attention slot and TWO MLP slots (the embedding and LM
    head use the MLP slots), 3.12 GB for 70B instead of the double buffer's 3.42 GB, and loads
    are issued in one fixed order as soon as their slot is released.  The order is the pass
    order with each decoder's MLP piece moved in front of its attention piece when the previous
    shard is a decoder too (E a1 m1 m2 a2 m3 a3 ...):

    * MLP(k+1) issues as layer k starts (its slot held MLP(k-1)), so it has the whole of layer k
      to land, however many micro-batches layer k runs;
    * attention(k+1) lands while the last micro-batch of layer k runs its MLP (its slot frees
      after that micro-batch's O projection: 0.30 GB, the small piece);
    * at the call boundary the LM head, the next call's embedding and first attention piece all
      load under the last layers, and the pool continues into the next call (same weights every
      call: the reference re-streams them, ``utils.py:228-233``).

    Every load waits (copy stream) for the free event recorded when its slot's previous piece
    was released on the compute stream; a piece is only issued once that release happened."""

    def __init__(self, source: LayerSource, layer_names: Sequence[str], shards: Sequence[Tuple[int, ...]],
                 device, dtype=torch.float16):
        self.src = source
        self.names = list(layer_names)
        self.shards = [tuple(s) for s in shards]
        self.dev = torch.device(device)
        self.cuda = self.dev.type == "cuda"
        if not self.cuda or any(len(s) != 1 for s in self.shards):
            raise ValueError("piece pools stream one layer per shard on a GPU")
        self.dtype = dtype
        self.resident = False
        self._sticky = set()
        self._loaded_resident = set()
        self.epoch = 0
        self.lock = threading.Lock()
        self._pool = None
        # piece list of one pass: (kind, shard, byte lo, byte hi); kind a = attention slot,
        # m = the two alternating MLP slots, o = own small buffer
        from ..models.layout import mlp_offset
        self.pieces: List[Tuple[str, int, int, int]] = []
        self._pidx: Dict[Tuple[int, int], int] = {}     # (shard, 0 attention / 1 MLP) -> piece index
        a_max = m_max = 0
        self._own: Dict[int, int] = {}
        own_sizes: List[int] = []
        for k, sh in enumerate(self.shards):
            name = self.names[sh[0]]
            lay = source.layout(name)
            nb = source.nbytes(name)
            if lay.kind == "decoder":
                split = mlp_offset(lay)
                prev_dec = k > 0 and source.layout(self.names[self.shards[k - 1][0]]).kind == "decoder"
                pair = [("a", k, 0, split), ("m", k, split, nb)]
                self.pieces += pair[::-1] if prev_dec else pair
                a_max, m_max = max(a_max, _align(split)), max(m_max, _align(nb - split))
            elif nb <= (64 << 20):
                self._own[k] = len(own_sizes)
                own_sizes.append(_align(nb))
                self.pieces.append(("o", k, 0, nb))
            else:
                self.pieces.append(("m", k, 0, nb))
                m_max = max(m_max, _align(nb))
        for i, (kind, k, _, _) in enumerate(self.pieces):
            self._pidx[(k, 1 if kind == "m" and self._is_dec(k) else 0)] = i
        self.a_bytes, self.m_bytes = a_max, m_max
        self._own_sizes = own_sizes
        self.n_slots = 2
        self.slot_bytes = m_max
        self._slot_sizes = [a_max, m_max, m_max] + own_sizes
        self._slots: List[Optional[torch.Tensor]] = [None] * len(self._slot_sizes)
        self._slot_owner: List[Optional[int]] = [None] * len(self._slot_sizes)   # global piece id
        self._slot_free: List[Optional[torch.cuda.Event]] = [None] * len(self._slot_sizes)
        self._released = set()            # global piece ids released
        self._issued: Dict[int, Tuple[int, torch.cuda.Event]] = {}   # global piece id -> (slot, ready)
        self._next = 0                    # next global piece id to issue
        self._m_turn = 0                  # MLP slot of the next m-piece (alternates across calls)
        self._acquired = set()
        self.copy_stream = torch.cuda.Stream(self.dev)
        self.bytes_h2d = 0
        self.wait_seconds = 0.0
        self.load_seconds = 0.0
        self._stall_ev: List[Tuple[torch.cuda.Event, torch.cuda.Event]] = []
        # layers read from their files (--weight_cache stream): each piece is a byte range of the
        # layer image the native streamer reads straight into the slot; the blocking file reads
        # run on one loader thread in issue order, so the host thread never waits for the disk
        # except when a piece it needs is still being read
        self._streamed = any(source.host_buffer(self.names[s[0]]) is None for s in self.shards)
        if self._streamed and not hasattr(source, "stream_into"):
            raise ValueError("piece pools need host-resident layers or a streaming source")
        self._loader = ThreadPoolExecutor(1, thread_name_prefix="fls-piece-loader") if self._streamed else None
        self._futs: Dict[int, Future] = {}

    # ----------------------------------------------------------- bookkeeping
    def planned_hbm_bytes(self) -> int:
        return sum(self._slot_sizes)

    def in_rotation(self, k: int) -> bool:
        return k not in self._own

    def is_kept_loaded(self, k: int) -> bool:
        return False

    def _is_dec(self, k: int) -> bool:
        return self.src.layout(self.names[self.shards[k][0]]).kind == "decoder"

    def _gid(self, k: int, which: int = 0) -> int:
        """Global id of shard k's attention (0) or MLP (1) piece in the current epoch (a shard
        without a decoder layer has one piece, ``which`` 0)."""
        return self.epoch * len(self.pieces) + self._pidx[(k, which)]

    def _slot_for(self, gid: int) -> int:
        kind, k, _, _ = self.pieces[gid % len(self.pieces)]
        if kind == "a":
            return 0
        if kind == "o":
            return 3 + self._own[k]
        return 1 + self._m_turn

    # ------------------------------------------------------------------ loads
    def _try_issue(self) -> bool:
        gid = self._next
        s = self._slot_for(gid)
        owner = self._slot_owner[s]
        if owner is not None and owner not in self._released:
            return False                           # the slot's piece is still in use
        kind, k, lo, hi = self.pieces[gid % len(self.pieces)]
        name = self.names[self.shards[k][0]]
        t0 = time.perf_counter()
        slot = self._slot(s)
        ev = torch.cuda.Event()
        free = self._slot_free[s]

        def load():
            with torch.cuda.stream(self.copy_stream):
                if free is not None:
                    self.copy_stream.wait_event(free)
                if self.src.host_buffer(name) is None:
                    nbytes = self.src.stream_into(name, slot, self.copy_stream, lo, hi)
                else:
                    nbytes = self._copy_piece(slot, name, lo, hi)
                if self.on_load is not None and kind in "am" and self._is_dec(k):
                    # attention piece: ln1 into W_qkv; MLP piece (ln2 is its first tensor): ln2 into W_gate/up
                    self._loaded(name, self._piece_views(slot, name, kind == "a"))
                ev.record(self.copy_stream)
            return nbytes

        if self._loader is not None:
            self._futs[gid] = self._loader.submit(load)
            nbytes = hi - lo
        else:
            nbytes = load()
        self.load_seconds += time.perf_counter() - t0
        self.bytes_h2d += nbytes
        if owner is not None:
            self._released.discard(owner)
            self._issued.pop(owner, None)
        self._slot_owner[s] = gid
        self._released.discard(gid)
        self._issued[gid] = (s, ev)
        if kind == "m":
            self._m_turn ^= 1
        self._next += 1
        return True

    def _copy_piece(self, slot: torch.Tensor, name: str, lo: int, hi: int) -> int:
        """Enqueue image bytes [lo, hi) of ``name`` into ``slot[0:]`` on the copy stream (current
        stream) -> host bytes moved."""
        if self.emulate_fanout is not None and self.emulate_fanout[3]:
            # a data-parallel rank's own slice: 1/8 of the piece over PCIe (the rest of the slot keeps
            # stale, finite weights: a timing run)
            n = (hi - lo) // 8
            slot[:n].copy_(self.src.host_buffer(name)[lo:lo + n], non_blocking=True)
        else:
            slot[:hi - lo].copy_(self.src.host_buffer(name)[lo:hi], non_blocking=True)
        if self.emulate_fanout is not None:
            self._emulate_gather(slot, hi - lo)
        return hi - lo

    # bench.py --emulate-dp-fanout (measurement only): after each piece lands, the device traffic
    # that the data-parallel all-gather of G = 8 ranks adds on a rank -- 7/8 of the piece's bytes
    # read from HBM and written to HBM -- issued on the copy stream where AllGatherPiecePool issues
    # its gather, as (mode, blocks, scratch, slice): mode 0 / 2 on the compute units (the runtime's
    # blit kernel / a copy kernel on `blocks` workgroups, like RCCL's channels), 1 on the SDMA
    # engines; slice: only the rank's 1/8 of the piece comes over PCIe.  The writes cycle through
    # `scratch`
    emulate_fanout = None

    def _emulate_gather(self, slot: torch.Tensor, nbytes: int) -> None:
        from .. import _native
        mode, blocks, scratch, _ = self.emulate_fanout
        if mode < 0:
            return
        k = _native.kernels()
        left = nbytes * 7 // 8 // 16 * 16
        chunk = min(scratch.numel() * scratch.element_size(), nbytes) // 16 * 16
        st = torch.cuda.current_stream(self.dev).cuda_stream
        while left > 0 and chunk > 0:
            n = min(left, chunk)
            rc = k.fls_copy_d2d(scratch.data_ptr(), slot.data_ptr(), n, mode, blocks, st)
            if rc:
                raise RuntimeError(f"fls_copy_d2d failed ({rc})")
            left -= n

    def _pump(self, need: Optional[int] = None) -> None:
        """Issue loads in pass order while their slots are free (at least through ``need``)."""
        while self._try_issue():
            pass
        if need is not None and need >= self._next:
            raise RuntimeError(f"weight piece {need} cannot load: its slot is still held "
                               f"(next issuable piece {self._next})")

    def prefetch(self, k: int, epoch: Optional[int] = None) -> None:
        self._pump()

    def _wait(self, gid: int) -> Tuple[int, torch.cuda.Event]:
        self._pump(gid)
        s, ev = self._issued[gid]
        fut = self._futs.pop(gid, None)
        if fut is not None:
            fut.result()                  # the loader has enqueued the piece's DMAs and its event
        cur = torch.cuda.current_stream(self.dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        cur.wait_event(ev)
        e1.record(cur)
        self._stall_ev.append((e0, e1))
        return s, ev

    def acquire(self, k: int) -> Dict[str, Dict[str, torch.Tensor]]:
        t0 = time.perf_counter()
        name = self.names[self.shards[k][0]]
        lay = self.src.layout(name)
        s, _ = self._wait(self._gid(k, 0))
        self._acquired.add(k)
        if lay.kind == "decoder":
            from ..models.layout import mlp_offset
            split = mlp_offset(lay)
            es = torch.empty((), dtype=self.dtype).element_size()
            views = {}
            for ts in lay.slots:
                if ts.offset < split:
                    n = ts.numel * es
                    views[ts.name] = self._slots[s][ts.offset:ts.offset + n].view(self.dtype).view(ts.shape)
            out = {name: _LayerViews(self, k, name, views, [ts.name for ts in lay.slots if ts.offset >= split])}
        else:
            kind, _, lo, hi = self.pieces[self._pidx[(k, 0)]]
            out = {name: lay.views(self._slots[s][:hi - lo], self.dtype)}
        self.wait_seconds += time.perf_counter() - t0
        return out

    def _piece_views(self, slot: torch.Tensor, name: str, attention: bool) -> Dict[str, torch.Tensor]:
        """Views of the attention (or MLP) piece of decoder ``name`` held at the start of ``slot``."""
        from ..models.layout import mlp_offset
        lay = self.src.layout(name)
        split = mlp_offset(lay)
        es = torch.empty((), dtype=self.dtype).element_size()
        base = 0 if attention else split
        return {ts.name: slot[ts.offset - base:ts.offset - base + ts.numel * es].view(self.dtype).view(ts.shape)
                for ts in lay.slots if (ts.offset < split) == attention}

    def _mlp_views(self, k: int, name: str) -> Dict[str, torch.Tensor]:
        from ..models.layout import mlp_offset
        lay = self.src.layout(name)
        split = mlp_offset(lay)
        s, _ = self._wait(self._gid(k, 1))
        es = torch.empty((), dtype=self.dtype).element_size()
        views = {}
        for ts in lay.slots:
            if ts.offset >= split:
                n = ts.numel * es
                o = ts.offset - split
                views[ts.name] = self._slots[s][o:o + n].view(self.dtype).view(ts.shape)
        return views

    def _release_gid(self, gid: int) -> None:
        if gid in self._released or gid not in self._issued:
            return
        self._futs.pop(gid, None)     # (a streamed piece released unread: its load job still runs in order)
        s, _ = self._issued[gid]
        e = torch.cuda.Event()
        e.record(torch.cuda.current_stream(self.dev))
        self._slot_free[s] = e
        self._released.add(gid)

    def _release_attn(self, k: int) -> None:
        self._release_gid(self._gid(k, 0))
        self._pump()

    def release(self, k: int) -> None:
        if k not in self._acquired:
            return
        self._acquired.discard(k)
        n = 2 if (k, 1) in self._pidx else 1
        for j in range(n):
            gid = self._gid(k, j)
            if gid not in self._issued and gid not in self._released:
                # a piece never used (a data-parallel rank with no prompts acquires and releases
                # every layer): issue it now — its load / gather keeps the pass order on every
                # rank — so that its slot is freed like any other
                self._pump(gid)
            self._release_gid(gid)
        self._pump()

    def _drain_loader(self) -> None:
        for fut in list(self._futs.values()):
            try:
                fut.result()
            except Exception:       # noqa: BLE001  (a failed read surfaces where it was awaited)
                pass
        self._futs.clear()

    def discard_loaded(self) -> None:
        """After an empty or aborted pass: every issued piece is dropped (its copy stays ordered
        on the copy stream before any later load into the same slot) and the next call starts
        its pass from the first piece."""
        self._drain_loader()
        cur = torch.cuda.current_stream(self.dev)
        for gid in list(self._issued):
            if gid not in self._released:
                s, _ = self._issued[gid]
                e = torch.cuda.Event()
                e.record(cur)
                self._slot_free[s] = e
        # every slot is free now (its free event orders the next load after the dropped piece)
        self._slot_owner = [None] * len(self._slot_sizes)
        self._issued.clear()
        self._released.clear()
        self._acquired.clear()
        self._next = self.epoch * len(self.pieces)
        self._m_turn = 0

    def close(self):
        self._drain_loader()
        if self._loader is not None:
            self._loader.shutdown(wait=True)
        if self.cuda:
            torch.cuda.synchronize(self.dev)
        self._issued.clear()
        self._released.clear()
        self._slot_owner = [None] * len(self._slot_sizes)
        self._slot_free = [None] * len(self._slot_sizes)
        self._slots = [None] * len(self._slot_sizes)
