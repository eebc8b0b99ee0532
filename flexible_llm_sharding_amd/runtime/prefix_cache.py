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


class PrefixEntry:
    def __init__(self, key: str, prefix_lens: Sequence[int], kv_cols: int, device, dtype):
        self.key = key
        self.offsets: List[int] = []
        t = 0
        for lp in prefix_lens:
            self.offsets.append(t)
            t += lp
        self.total = t
        self.kv_cols = kv_cols
        self.dev = torch.device(device)
        self.dtype = dtype
        self.layers: Dict[str, torch.Tensor] = {}
        self.complete = False

    def buffer(self, layer_name: str, create: bool = False) -> Optional[torch.Tensor]:
        b = self.layers.get(layer_name)
        if b is None and create:
            b = torch.empty(max(1, self.total), self.kv_cols, dtype=self.dtype, device=self.dev)
            self.layers[layer_name] = b
        return b

    @property
    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.layers.values())


class PrefixKVCache:
    def __init__(self, kv_cols: int, device, dtype=torch.float16, max_entries: int = 8):
        self.kv_cols = kv_cols
        self.dev = torch.device(device)
        self.dtype = dtype
        self.max_entries = max(1, max_entries)
        self.entries: "OrderedDict[str, PrefixEntry]" = OrderedDict()
        self.hits = 0
        self.misses = 0

    def lookup(self, tps: Sequence) -> Optional[PrefixEntry]:
        e = self.entries.get(prefix_fingerprint(tps))
        if e is not None and e.complete:
            self.entries.move_to_end(e.key)
            return e
        return None

    def begin(self, tps: Sequence) -> PrefixEntry:
        """A fresh entry the coming full pass fills (replaces any partial one)."""
        key = prefix_fingerprint(tps)
        self.entries.pop(key, None)
        while len(self.entries) >= self.max_entries:
            self.entries.popitem(last=False)
        e = PrefixEntry(key, [len(tp.prefix) for tp in tps], self.kv_cols, self.dev, self.dtype)
        self.entries[key] = e
        return e

    def drop(self, e: PrefixEntry) -> None:
        self.entries.pop(e.key, None)

    @property
    def nbytes(self) -> int:
        return sum(e.nbytes for e in self.entries.values())
