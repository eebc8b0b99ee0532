"""Prefix K/V reuse across calls (``--prefix_kv_cache``).

The reference's generation loop (``/root/reference/main.py:63-90``) re-runs
the whole model for every generated token: each step re-tokenizes
``suffix + decoded tokens`` and pushes the (unchanged) prefix through every
layer again (``utils.py:269-272``).  The prefix's hidden states never see the
suffixes (the prefix is processed alone, ``attention_mask=None``), so its
post-RoPE K/V per layer are identical in every step and in every repeated
call on the same prompts.

This cache keeps, per decoder layer, the prefix K/V rows of every prompt of a
call in HBM (``[sum Lp, 2 * n_kv * head_dim]`` fp16 per layer; 70B: 4 KB per
token per layer).  A later call whose prompts have the same prefixes (same
token ids, same order) runs only the suffix tokens: the shared-prefix
attention reads range 0 (the prefix) from the cache instead of the packed
QKV.  Results are bitwise those of the full pass on the HIP path (the cached
rows are the values the full pass computed), so the feature changes cost,
not semantics.  Entries are LRU-evicted by count; the engine only switches
to the cached path when EVERY rank holds a complete entry (model parallel
ranks must pack identical batches).

Suffix K/V reuse (``--suffix_kv_cache``, on with the prefix cache): each entry also
holds, after the prefixes, a region per (prompt, suffix) with the post-RoPE K/V of that
suffix's tokens from the last call, and their token ids.  A generation step appends
``decode(new tokens)`` to every suffix and re-tokenizes it (``main.py:87-90``): the
longest common token prefix with the cached ids has the same K/V (causal rows depend
only on the prefix and earlier suffix tokens), so only the tokens after it are packed
and computed; their attention reads the kept rows as range 2
(``csrc/kernels/attention.hip``).  At least the scored (last) token is always
recomputed.  A step then costs the new tokens instead of every suffix token; the
engine runs such calls row-exact (every row's arithmetic independent of the batch it
is packed in, ``engine.py`` "exact K/V reuse"), so a reused step's scores are bitwise
those of the full recomputation.  A suffix that outgrows its region is computed in full
and not cached.

Host mode (``PrefixKVCache(host=True)``, the ``--max_vram_gb`` runs): the per-layer
buffers live in pinned host memory and HBM holds only a staging buffer of one
layer's K/V (planned by ``runtime/memplan.py``).  A layer's attention stages its
K/V in on the compute stream (nothing the first time: a fresh layer is zeros) and, after
the attention, copies the rows it wrote back on a side stream (every row in the filling
call, the suffix regions in a reused step) while the layer's O projection and MLP run;
the other staging buffer serves the next layer.  The values are the device mode's, so
the scores are too.
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch


def prefix_fingerprint(tps: Sequence) -> str:
    h = hashlib.sha1()
    for tp in tps:
        h.update(np.asarray(tp.prefix, dtype=np.int64).tobytes())
        h.update(b"|")
    return h.hexdigest()


def common_prefix(a: Sequence[int], b: Sequence[int]) -> int:
    n = min(len(a), len(b))
    if list(a[:n]) == list(b[:n]):            # a generation step: the old suffix is a prefix of the new
        return n
    i = 0
    while i < n and a[i] == b[i]:
        i += 1
    return i


class PrefixEntry:
    REGION_ALIGN = 64      # attention key tile (csrc/kernels/attention.hip KT)

    def __init__(self, key: str, prefix_lens: Sequence[int], kv_cols: int, device, dtype,
                 suffix_caps: Optional[Sequence[Sequence[int]]] = None, stage: Optional["HostStage"] = None):
        self.key = key
        self.offsets: List[int] = []
        t = 0
        for lp in prefix_lens:
            self.offsets.append(t)
            t += lp
        self.total = t
        # suffix regions after the prefixes: rows of suffix s of prompt j, capacity, cached ids
        self.sfx_rows: List[List[int]] = []
        self.sfx_caps: List[List[int]] = []
        for caps in (suffix_caps or []):
            self.sfx_rows.append([])
            self.sfx_caps.append(list(caps))
            for c in caps:
                # every region starts on a 64-row key-tile boundary: a reused step's range-2 tiles
                # then split each suffix's keys exactly as the full computation's range-1 tiles do
                t = -(-t // self.REGION_ALIGN) * self.REGION_ALIGN
                self.sfx_rows[-1].append(t)
                t += c
        self.sfx_ids: Dict[tuple, tuple] = {}
        self.rows = t
        self.kv_cols = kv_cols
        self.dev = torch.device(device)
        self.dtype = dtype
        self.layers: Dict[str, torch.Tensor] = {}
        self.complete = False
        self.stage = stage            # host mode: the cache's staging buffers
        self._staged: Optional[tuple] = None     # (layer name, staging view) of the layer in flight

    @property
    def host(self) -> bool:
        return self.stage is not None

    def buffer(self, layer_name: str, create: bool = False) -> Optional[torch.Tensor]:
        if self.stage is not None:
            return self._stage_in(layer_name, create)
        b = self.layers.get(layer_name)
        if b is None and create:
            # zeroed: a reused step's key tiles cover the alignment gaps and unused region rows (masked,
            # P = 0 exactly, and 0 x a finite V adds nothing)
            b = torch.zeros(max(1, self.rows), self.kv_cols, dtype=self.dtype, device=self.dev)
            self.layers[layer_name] = b
        return b

    def _stage_in(self, layer_name: str, create: bool) -> Optional[torch.Tensor]:
        if self._staged is not None and self._staged[0] == layer_name:
            return self._staged[1]
        hb = self.layers.get(layer_name)
        if hb is None:
            if not create:
                return None
            hb = self.stage.alloc_host(max(1, self.rows), self.kv_cols, self.dtype)
            self.layers[layer_name] = hb
            fresh = True
        else:
            fresh = False
        buf = self.stage.acquire(hb.shape[0])
        self.stage.load(buf, hb, layer_name, fresh)
        self._staged = (layer_name, buf)
        return buf

    def write_rows(self, ops, x: torch.Tensor, src_idx, dst_idx, layer_name: str) -> bool:
        """Host mode, complete entry (a reused step): the new rows go straight into the layer's
        mapped host buffer (a row-copy kernel writing over PCIe: ~0.6 MB per layer at 160 new rows,
        instead of a write-back of every suffix region).  False when the buffer is not mapped."""
        if self.stage is None or not self.complete:
            return False
        hb = self.layers.get(layer_name)
        dp = self.stage.device_ptr(hb) if hb is not None else None
        if dp is None or not hasattr(ops, "copy_rows_to"):
            return False
        ops.copy_rows_to(x, src_idx, dp, hb.shape[1], dst_idx)
        self.stage.bytes_direct += src_idx.shape[0] * x.shape[1] * x.element_size()
        if self._staged is not None and self._staged[0] == layer_name:
            self._staged = (layer_name, self._staged[1], True)
        return True

    def flush(self, layer_name: str) -> None:
        """After a layer's attention (host mode): the rows it may have written go back to the
        host buffer — all of them while the entry fills, the suffix regions once it is complete
        (a reused step writes only its new suffix tokens; nothing when :meth:`write_rows` already
        put them there)."""
        if self._staged is None or self._staged[0] != layer_name:
            return
        buf, direct = self._staged[1], len(self._staged) > 2
        self._staged = None
        lo = self.total if self.complete else 0
        if lo < buf.shape[0] and not direct:
            self.stage.store(self.layers[layer_name], buf, lo, layer_name)

    def suffix_plan(self, tps: Sequence, reuse: bool):
        """-> (rows, keep) for :func:`runtime.batch.pack_prompts`: the cache row of every suffix
        that fits its region (-1 otherwise) and, with ``reuse``, how many of its leading tokens
        the cache already holds (the common token prefix with the last call, less the scored
        token, which is always recomputed)."""
        if not self.sfx_rows:
            return None, None
        rows, keep = [], []
        for j, tp in enumerate(tps):
            r, k = [], []
            for si, s in enumerate(tp.suffixes):
                if j >= len(self.sfx_rows) or si >= len(self.sfx_rows[j]) or len(s) > self.sfx_caps[j][si]:
                    r.append(-1)
                    k.append(0)
                    continue
                r.append(self.sfx_rows[j][si])
                old = self.sfx_ids.get((j, si))
                k.append(min(common_prefix(old, s), len(s) - 1) if (reuse and old) else 0)
            rows.append(r)
            keep.append(k)
        if any(r < 0 for rr in rows for r in rr):
            reuse = False        # reuse mode reads every suffix's K/V from its region (batch.pack_prompts)
        return rows, (keep if reuse else None)

    def commit_suffixes(self, tps: Sequence, rows) -> None:
        """After a completed call: the cache regions hold exactly these suffixes' K/V."""
        if rows is None:
            return
        for j, tp in enumerate(tps):
            for si, s in enumerate(tp.suffixes):
                if rows[j][si] >= 0:
                    self.sfx_ids[(j, si)] = tuple(s)
                else:
                    self.sfx_ids.pop((j, si), None)

    @property
    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.layers.values())


class HostStage:
    """Device staging buffer(s) for host-mode entries (one layer's K/V each) and the side stream
    their write-backs run on.  A buffer is reused only after its last write-back, and a layer's
    host rows are read back only after theirs landed (events per buffer and per layer).  One
    buffer: a layer's write-back overlaps its own O projection and MLP, which outlast it (70B,
    32 prompts: ~4 ms of D2H per layer against >= 30 ms of weight streaming per layer), so a
    second buffer would buy little for its HBM."""

    N_BUFS = 1

    def __init__(self, kv_cols: int, device, dtype, max_rows: int):
        self.dev = torch.device(device)
        self.cuda = self.dev.type == "cuda"
        self.bufs = [torch.zeros(max(1, max_rows), kv_cols, dtype=dtype, device=self.dev)
                     for _ in range(self.N_BUFS)]
        self.cur = 0
        self.stream = torch.cuda.Stream(self.dev) if self.cuda else None
        self.buf_ev: List[Optional[object]] = [None] * self.N_BUFS
        self.layer_ev: Dict[tuple, object] = {}
        self.bytes_h2d = self.bytes_d2h = 0
        self.bytes_direct = 0                 # rows kernels wrote straight into host buffers
        self._dptr: Dict[int, int] = {}       # id(host buffer) -> its device address (mapped pinned)

    @property
    def nbytes(self) -> int:
        return sum(b.numel() * b.element_size() for b in self.bufs)

    def alloc_host(self, rows: int, cols: int, dtype) -> torch.Tensor:
        if not self.cuda:
            return torch.zeros(rows, cols, dtype=dtype)
        from . import hostmem
        from .. import _native
        nbytes = rows * cols * torch.empty(0, dtype=dtype).element_size()
        t = hostmem.alloc_host(nbytes, pinned=True)
        t.zero_()
        hb = t.view(dtype).view(rows, cols)
        rt = _native.runtime_or_none()
        dp = rt.fls_host_device_ptr(t.data_ptr()) if rt is not None else None
        if dp:
            self._dptr[id(hb)] = int(dp)
        return hb

    def device_ptr(self, hb: torch.Tensor) -> Optional[int]:
        """The device address of a host buffer (kernels write its rows over PCIe), or None."""
        return self._dptr.get(id(hb))

    def acquire(self, rows: int) -> torch.Tensor:
        if rows > self.bufs[0].shape[0]:
            raise ValueError(f"prefix K/V entry of {rows} rows > the staging buffers' {self.bufs[0].shape[0]}")
        self.cur = (self.cur + 1) % self.N_BUFS
        ev = self.buf_ev[self.cur]
        if ev is not None:
            torch.cuda.current_stream(self.dev).wait_event(ev)
        return self.bufs[self.cur][:rows]

    def load(self, buf: torch.Tensor, hb: torch.Tensor, layer_name: str, fresh: bool) -> None:
        if fresh:
            buf.zero_()
            return
        ev = self.layer_ev.get((id(hb), layer_name))
        if ev is not None:
            torch.cuda.current_stream(self.dev).wait_event(ev)
        buf.copy_(hb, non_blocking=True)
        self.bytes_h2d += hb.numel() * hb.element_size()

    def store(self, hb: torch.Tensor, buf: torch.Tensor, lo: int, layer_name: str) -> None:
        self.bytes_d2h += (buf.shape[0] - lo) * buf.shape[1] * buf.element_size()
        if not self.cuda:
            hb[lo:].copy_(buf[lo:])
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev)
            hb[lo:].copy_(buf[lo:], non_blocking=True)
            done = torch.cuda.Event()
            done.record(self.stream)
        self.buf_ev[self.cur] = done
        self.layer_ev[(id(hb), layer_name)] = done

    def forget(self, e: "PrefixEntry") -> None:
        for name, hb in e.layers.items():
            self.layer_ev.pop((id(hb), name), None)
            self._dptr.pop(id(hb), None)


def suffix_growth(num_gen_token: int) -> int:
    """Rows of growth per suffix region for a generation of ``num_gen_token`` steps: each step
    appends one decoded token, which re-tokenizes to one or two tokens (4 per step + 8 spare,
    at most ``PrefixKVCache.SUFFIX_GROWTH``).  A suffix that still outgrows its region is computed
    in full (correct, not reused).  Smaller regions mean fewer key tiles per step and, in host
    mode, fewer bytes staged over PCIe."""
    return min(PrefixKVCache.SUFFIX_GROWTH, 4 * max(1, num_gen_token) + 8)


class PrefixKVCache:
    # suffix region per (prompt, suffix): its first call's length + suffix_growth tokens of growth
    # (default SUFFIX_GROWTH; generation_loop sets it from --num_gen_token)
    SUFFIX_GROWTH = 64

    def __init__(self, kv_cols: int, device, dtype=torch.float16, max_entries: int = 8,
                 suffix_reuse: bool = True, host: bool = False):
        self.suffix_reuse = suffix_reuse
        self.suffix_growth = self.SUFFIX_GROWTH
        self.host = host
        self.stage: Optional[HostStage] = None
        self.kv_cols = kv_cols
        self.dev = torch.device(device)
        self.dtype = dtype
        self.max_entries = max(1, max_entries)
        self.entries: "OrderedDict[str, PrefixEntry]" = OrderedDict()
        self.hits = 0
        self.misses = 0
        # called with an entry that leaves the cache (its K/V buffers are freed with it): graphs
        # captured on it must go first (runtime/graphs.py DecodeGraphs.forget)
        self.on_evict: List = []

    def _evict(self, e: Optional[PrefixEntry]) -> None:
        if e is not None:
            for cb in self.on_evict:
                cb(e)
            if self.stage is not None:
                self.stage.forget(e)

    def entry_rows(self, tps: Sequence) -> int:
        """Rows of the entry ``begin(tps)`` creates (prefixes + 64-aligned suffix regions)."""
        t = sum(len(tp.prefix) for tp in tps)
        if self.suffix_reuse:
            for tp in tps:
                for s in tp.suffixes:
                    t = -(-t // PrefixEntry.REGION_ALIGN) * PrefixEntry.REGION_ALIGN + len(s) + self.suffix_growth
        return t

    def ensure_stage(self, tps: Sequence) -> None:
        """Host mode: staging buffers large enough for ``tps``'s entry (grown, never shrunk)."""
        if not self.host:
            return
        rows = self.entry_rows(tps)
        if self.stage is None or self.stage.bufs[0].shape[0] < rows:
            old = self.stage
            if old is not None and old.cuda:
                # the old buffers' write-backs finish before the buffers go
                torch.cuda.current_stream(self.dev).wait_stream(old.stream)
            self.stage = HostStage(self.kv_cols, self.dev, self.dtype, rows)
            if old is not None:
                self.stage.layer_ev = old.layer_ev
            for e in self.entries.values():
                e.stage = self.stage

    def lookup(self, tps: Sequence) -> Optional[PrefixEntry]:
        e = self.entries.get(prefix_fingerprint(tps))
        if e is not None and e.complete:
            self.entries.move_to_end(e.key)
            return e
        return None

    def begin(self, tps: Sequence) -> PrefixEntry:
        """A fresh entry the coming full pass fills (replaces any partial one)."""
        key = prefix_fingerprint(tps)
        self._evict(self.entries.pop(key, None))
        while len(self.entries) >= self.max_entries:
            self._evict(self.entries.popitem(last=False)[1])
        caps = ([[len(s) + self.suffix_growth for s in tp.suffixes] for tp in tps] if self.suffix_reuse else None)
        self.ensure_stage(tps)
        e = PrefixEntry(key, [len(tp.prefix) for tp in tps], self.kv_cols, self.dev, self.dtype, caps,
                        stage=self.stage)
        self.entries[key] = e
        return e

    def drop(self, e: PrefixEntry) -> None:
        self._evict(e)
        self.entries.pop(e.key, None)

    @property
    def nbytes(self) -> int:
        return sum(e.nbytes for e in self.entries.values())
