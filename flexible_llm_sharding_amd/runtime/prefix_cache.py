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
recomputed.  A step then costs the new tokens instead of every suffix token (the
kernels see different batch shapes than a full recompute, so results agree to
rounding, not bitwise).  A suffix that outgrows its region is computed in full and
not cached.
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
                 suffix_caps: Optional[Sequence[Sequence[int]]] = None):
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

    def buffer(self, layer_name: str, create: bool = False) -> Optional[torch.Tensor]:
        b = self.layers.get(layer_name)
        if b is None and create:
            # zeroed: a reused step's key tiles cover the alignment gaps and unused region rows (masked,
            # P = 0 exactly, and 0 x a finite V adds nothing)
            b = torch.zeros(max(1, self.rows), self.kv_cols, dtype=self.dtype, device=self.dev)
            self.layers[layer_name] = b
        return b

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


class PrefixKVCache:
    # suffix region per (prompt, suffix): its first call's length + this many tokens of growth
    SUFFIX_GROWTH = 64

    def __init__(self, kv_cols: int, device, dtype=torch.float16, max_entries: int = 8,
                 suffix_reuse: bool = True):
        self.suffix_reuse = suffix_reuse
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
        caps = ([[len(s) + self.SUFFIX_GROWTH for s in tp.suffixes] for tp in tps] if self.suffix_reuse else None)
        e = PrefixEntry(key, [len(tp.prefix) for tp in tps], self.kv_cols, self.dev, self.dtype, caps)
        self.entries[key] = e
        return e

    def drop(self, e: PrefixEntry) -> None:
        self._evict(e)
        self.entries.pop(e.key, None)

    @property
    def nbytes(self) -> int:
        return sum(e.nbytes for e in self.entries.values())
