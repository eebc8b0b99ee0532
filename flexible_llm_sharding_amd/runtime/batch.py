"""Packed micro-batches of (prefix, suffixes) prompts.

The reference runs prompts one at a time through each layer: the prefix as a
batch of 1 (``utils.py:272``) and the ``n_s`` right-padded suffixes as a batch
against the prefix K/V expanded ``n_s`` times (``utils.py:274-279``).

On MI355X we pack MANY prompts into one token matrix ``[T, H]`` so every
projection is one large MFMA GEMM, and describe the attention structure with
*work items* consumed by the shared-prefix flash-attention kernel:

* prefix segment: queries = prefix tokens; keys = the prefix
  (bidirectional — the reference's ``attention_mask=None`` on transformers
  <= 4.35, SURVEY §A.4 — or causal);
* suffix segment: queries = the suffix's real tokens at positions
  ``Lp .. Lp+len-1`` (``utils.py:275``); keys = the whole prefix (shared, read
  in place, never expanded) + the suffix itself causally (``utils.py:276``).

A prompt's suffixes are packed back to back, and their work items cover those
rows in ``q_block`` chunks regardless of suffix boundaries: an item's range 1
spans every suffix it touches and ``seg_lo`` (first row of each row's suffix)
makes it block-diagonal, so 5 suffixes of 10 tokens are one item over the
shared prefix instead of 5 mostly empty ones (the reference's one-pass
shared-prefix cascade, without a second pass to merge).

Padding tokens after a suffix's scored position are never computed: under the
causal mask they cannot influence it.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..utils.tokenizer import TokenizedPrompt

Q_BLOCK = 64            # query rows per attention work item (kernel tile)
Q_BLOCK_MHA = 128       # multi-head models: 4 waves of one query head share each staged K/V tile
WORK_ITEM_FIELDS = 8    # q_start q_len q_off r0_start r0_len r0_causal r1_start r1_len


@dataclass
class Segment:
    q_start: int
    q_len: int
    r0_start: int
    r0_len: int
    r0_causal: int
    r1_start: int
    r1_len: int          # r1 (own suffix) is always causal
    q_off: int = 0       # index of the first query inside its segment (causal compare)
    r2_start: int = 0    # suffix K/V reuse: rows of the K/V cache holding this suffix's earlier
    r2_len: int = 0      # tokens (all visible), between the prefix (r0) and the new rows (r1)


# range-2 (generation-step) attention items of <= 8 rows: the packed-GQA decode kernel
# (csrc/kernels/attention.hip attn_decode; profiles/r5_gen)
R2_Q_BLOCK = 8


@dataclass
class PackedBatch:
    prompt_ids: List[int]                 # global prompt indices in this micro-batch
    n_suffix: List[int]                   # per prompt
    ids: np.ndarray                       # [T] int32
    positions: np.ndarray                 # [T] int32
    segments: List[Segment]
    work: np.ndarray                      # [n_items, 8] int32
    seg_lo: np.ndarray                    # [T] int32: first packed row of each row's suffix (prefix rows: their own start)
    last_idx: np.ndarray                  # [S_total] int32 rows scored
    last_segments: List[Segment]          # one single-query segment per scored row (last layer)
    work_last: np.ndarray                 # [S_total, 8] their work items
    num_tokens: int
    padded_tokens: int                    # reference-equivalent token count
    max_pos: int
    kv_cached: bool = False               # prefixes come from a PrefixEntry (range 0 rows index it)
    q_block: int = Q_BLOCK                # query rows per work item
    pfx_src: Optional[np.ndarray] = None  # capture: packed rows of every prefix token ...
    pfx_dst: Optional[np.ndarray] = None  # ... and their rows in the prefix K/V cache
    prompt_rows: Optional[np.ndarray] = None    # [n_prompts, 2] packed row range of each prompt
    prompt_items: Optional[np.ndarray] = None   # [n_prompts, 2] its range of ``work`` items
    prompt_scored: Optional[np.ndarray] = None  # [n_prompts, 2] its range of ``last_idx`` / ``work_last``
    work2: Optional[np.ndarray] = None          # [n_items, 2] suffix K/V reuse: range 2 of each item
    r2win: Optional[np.ndarray] = None          # [T, 2] the cache rows [lo, hi) of range 2 each row sees
    work2_last: Optional[np.ndarray] = None     # [S_total, 2] the same for ``work_last``
    sfx_src: Optional[np.ndarray] = None        # capture: packed rows of suffix tokens ...
    sfx_dst: Optional[np.ndarray] = None        # ... and their rows in the K/V cache
    _dev: dict = field(default_factory=dict, repr=False)

    @property
    def n_scored(self) -> int:
        return int(self.last_idx.shape[0])

    @property
    def all_rows_scored(self) -> bool:
        """Every packed row is a scored row, in row order (``last_idx`` = 0..T-1: a generation
        step computing one new token per suffix), so the rows a pruned last layer keeps are all
        of them, and the full layer's output already is the scored-row state."""
        v = self._dev.get("all_rows_scored")
        if v is None:
            v = self._dev["all_rows_scored"] = bool(
                self.num_tokens == self.last_idx.shape[0] and np.array_equal(self.last_idx, np.arange(self.num_tokens)))
        return v

    @property
    def r2_q_block(self) -> int:
        """q_block for the range-2 (suffix K/V reuse) attention: 8 when every work item holds at
        most 8 rows (a generation step: one new row per suffix) — the packed-GQA decode kernel, a
        KV group's heads x rows in one MFMA column block, each K/V tile read once per group; 32 when
        every item holds at most 32 rows (one wave per query head, a whole KV group per block); the
        batch's own q_block otherwise."""
        if self.work2 is None or self.work.shape[0] == 0 or R2_Q_BLOCK not in (8, 32):
            return self.q_block
        rows = int(self.work[:, 1].max())
        if R2_Q_BLOCK == 8 and rows <= 8:
            return 8
        return 32 if rows <= 32 else self.q_block

    def attn_groups(self, max_rows: int) -> List[dict]:
        """Prompt-aligned row groups of <= ``max_rows`` packed rows (a larger prompt is a group of
        its own) with their attention work items REBASED to the group's first row, so the
        attention phase of a layer can run group by group on a [rows, qkv] buffer (every key a
        query sees belongs to its own prompt).  Each group: r0, r1 (packed rows), work, seg_lo,
        work_last (scored rows only) and last_local (scored rows, group-relative), s0, s1 (its
        range of ``last_idx``).  Rows of the prefix K/V cache (``kv_cached``) are not rebased."""
        groups, cur = [], []
        n = self.prompt_rows.shape[0]
        for j in range(n):
            rows = int(self.prompt_rows[j, 1] - self.prompt_rows[j, 0])
            if cur and (int(self.prompt_rows[j, 1] - self.prompt_rows[cur[0], 0]) > max_rows):
                groups.append(cur)
                cur = []
            cur.append(j)
            del rows
        if cur:
            groups.append(cur)
        out = []
        for g in groups:
            r0, r1 = int(self.prompt_rows[g[0], 0]), int(self.prompt_rows[g[-1], 1])
            w0, w1 = int(self.prompt_items[g[0], 0]), int(self.prompt_items[g[-1], 1])
            s0, s1 = int(self.prompt_scored[g[0], 0]), int(self.prompt_scored[g[-1], 1])
            out.append({"r0": r0, "r1": r1, "s0": s0, "s1": s1,
                        "work": self._rebase(self.work[w0:w1], r0),
                        "work_last": self._rebase(self.work_last[s0:s1], r0),
                        "seg_lo": (self.seg_lo[r0:r1] - r0).astype(np.int32),
                        "last_local": (self.last_idx[s0:s1] - r0).astype(np.int32),
                        "last_pos": self.positions[self.last_idx[s0:s1]].astype(np.int32)})
        return out

    def _rebase(self, work: np.ndarray, r0: int) -> np.ndarray:
        w = work.copy()
        w[:, 0] -= r0                                   # q_start
        if not self.kv_cached:
            w[:, 3] = np.where(w[:, 4] > 0, w[:, 3] - r0, 0)     # range 0 = packed prefix rows
        w[:, 6] = np.where(w[:, 7] > 0, w[:, 6] - r0, 0)         # range 1 = packed suffix rows
        return w

    def _rebase_seg(self, sg: Segment, r0: int) -> Segment:
        return dataclasses.replace(sg, q_start=sg.q_start - r0,
                                   r0_start=sg.r0_start if self.kv_cached else sg.r0_start - r0,
                                   r1_start=sg.r1_start - r0 if sg.r1_len else 0)

    def group_tensors(self, device, max_rows: int) -> List[dict]:
        """:meth:`attn_groups` with int32 metadata on ``device`` (cached)."""
        key = (str(device), "groups", int(max_rows))
        if key not in self._dev:
            d = torch.device(device)
            nb = d.type != "cpu"
            gs = []
            for g in self.attn_groups(max_rows):
                t = {k: (torch.from_numpy(v).to(d, non_blocking=nb) if isinstance(v, np.ndarray) else v)
                     for k, v in g.items()}
                t["segments"] = [self._rebase_seg(sg, g["r0"]) for sg in self.segments
                                 if g["r0"] <= sg.q_start < g["r1"]]
                t["last_segments"] = [self._rebase_seg(sg, g["r0"]) for sg in self.last_segments[g["s0"]:g["s1"]]]
                gs.append(t)
            self._dev[key] = gs
        return self._dev[key]

    def host_meta(self) -> dict:
        """Every int32 metadata array the layers read (the keys of :meth:`device_tensors`)."""
        m = {"ids": self.ids, "positions": self.positions, "work": self.work, "seg_lo": self.seg_lo,
             "last_idx": self.last_idx, "last_pos": self.positions[self.last_idx].astype(np.int32),
             "work_last": self.work_last}
        for name in ("pfx_src", "pfx_dst", "sfx_src", "sfx_dst", "work2", "work2_last", "r2win"):
            v = getattr(self, name)
            if v is not None:
                m[name] = v
        return m

    def device_tensors(self, device) -> dict:
        """int32 metadata on ``device`` (cached; uploaded once, reused by all layers)."""
        key = str(device)
        if key not in self._dev:
            d = torch.device(device)
            nb = d.type != "cpu"
            self._dev[key] = {k: torch.from_numpy(np.ascontiguousarray(v)).to(d, non_blocking=nb)
                              for k, v in self.host_meta().items()}
        return self._dev[key]


def pack_prompts(tps: Sequence[TokenizedPrompt], prompt_ids: Sequence[int],
                 prefix_attention: str = "bidirectional", prefix_offsets: Optional[Sequence[int]] = None,
                 kv_cached: bool = False, q_block: int = Q_BLOCK,
                 suffix_rows: Optional[Sequence[Sequence[int]]] = None,
                 suffix_keep: Optional[Sequence[Sequence[int]]] = None,
                 single_suffix_items: bool = False) -> PackedBatch:
    """Pack prompts into one token matrix + attention work items.

    ``prefix_offsets`` (rows of each prompt's prefix in a PrefixEntry) turns on
    prefix K/V reuse: with ``kv_cached`` the prefixes are NOT packed (only the
    suffix tokens are computed; range 0 of each suffix item indexes the cache),
    otherwise the batch records which packed rows to copy into the cache.

    Suffix K/V reuse (``runtime/prefix_cache.py``): ``suffix_rows[j][s]`` is the cache row of
    suffix s of prompt j (-1: not cached) — the rows computed in this call are recorded for capture
    there — and ``suffix_keep[j][s]`` (with ``kv_cached``) the number of its leading tokens whose
    K/V the cache already holds: only the tokens after them are packed and computed, at their true
    positions, and each suffix gets work items of its own whose range 2 covers the kept rows.

    ``single_suffix_items``: no work item spans two suffixes, so every key tile of range 1 starts
    at a multiple of 64 tokens from its suffix's first token, as the range-2 tiles of a reused step
    do over 64-row-aligned cache regions (generation with the prefix K/V cache: each row's attention
    then takes the same tiles, whichever step computes it; engine ``row_exact``).
    """
    if prefix_attention not in ("bidirectional", "causal"):
        raise ValueError(prefix_attention)
    if kv_cached and prefix_offsets is None:
        raise ValueError("kv_cached needs prefix_offsets")
    pcausal = 1 if prefix_attention == "causal" else 0
    # per-row arrays are gathered as numpy parts (one per prefix / suffix) and concatenated once:
    # Python lists of 43k ints cost the host ~10 ms per call (the GPU idles at the call boundary)
    ids, pos, seg_lo, segs, last, nsuf, lsegs = [], [], [], [], [], [], []
    if suffix_keep is not None and not kv_cached:
        raise ValueError("suffix K/V reuse needs the prefix K/V cache (kv_cached)")
    if suffix_keep is not None and any(r < 0 for rows in suffix_rows for r in rows):
        raise ValueError("suffix K/V reuse needs a cache region for every suffix")
    work, work2, r2win, lwork, lwork2 = [], [], [], [], []
    src, dst, sfx_src, sfx_dst = [], [], [], []
    p_rows, p_items, p_scored = [], [], []
    t = 0
    padded = 0
    max_pos = 0
    for j, tp in enumerate(tps):
        Lp = len(tp.prefix)
        row0, item0, sc0 = t, len(work), len(last)
        if kv_cached:
            p0 = prefix_offsets[j]
        else:
            p0 = t
            ids.append(np.asarray(tp.prefix, dtype=np.int32))
            pos.append(np.arange(Lp, dtype=np.int32))
            segs.append(Segment(p0, Lp, p0, Lp, pcausal, 0, 0))
            seg_lo.append(np.full(Lp, p0, dtype=np.int32))
            work.extend(_items(segs[-1], q_block))
            work2.extend([(0, 0)] * (len(work) - len(work2)))
            if prefix_offsets is not None:
                src.append(np.arange(t, t + Lp, dtype=np.int32))
                dst.append(np.arange(prefix_offsets[j], prefix_offsets[j] + Lp, dtype=np.int32))
            t += Lp
        sfx0 = t
        sfx_lo = []                    # seg_lo of this prompt's suffix rows (row - sfx0)
        keep = suffix_keep[j] if suffix_keep is not None else None
        for si, s in enumerate(tp.suffixes):
            c = keep[si] if keep is not None else 0
            c0_row = suffix_rows[j][si] if suffix_rows is not None else -1
            n = len(s) - c
            s0 = t
            ids.append(np.asarray(s[c:], dtype=np.int32))
            pos.append(np.arange(Lp + c, Lp + c + n, dtype=np.int32))
            seg_lo.append(np.full(n, s0, dtype=np.int32))
            sfx_lo.extend([s0] * n)
            r2s, r2l = (c0_row, c) if c else (0, 0)
            segs.append(Segment(s0, n, p0, Lp, 0, s0, n, r2_start=r2s, r2_len=r2l))
            last.append(s0 + n - 1)
            # the scored row alone, for a last decoder layer that computes only scored rows
            lsegs.append(Segment(s0 + n - 1, 1, p0, Lp, 0, s0, n, q_off=n - 1, r2_start=r2s, r2_len=r2l))
            if keep is not None:
                # its work item (HIP): the whole suffix from the cache through the row's window
                lwork.append((s0 + n - 1, 1, 0, p0, Lp, 0, 0, 0))
                lwork2.append((c0_row, c + n))
            if c0_row >= 0:
                sfx_src.append(np.arange(s0, s0 + n, dtype=np.int32))
                sfx_dst.append(np.arange(c0_row + c, c0_row + c + n, dtype=np.int32))
            if keep is not None:
                # the new rows' K/V are captured into the cache before the attention runs, right
                # after the kept ones: new row i sees cache rows [c0_row, c0_row + c + i] (its own
                # key included: causal by window), so the kernel needs no range 1 at all.  (With
                # keep every packed row is a suffix row: the prefixes come from the cache.)
                r2win.extend([(c0_row, c0_row + c + i + 1) for i in range(n)])
            t += n
        # the prompt's suffix rows [sfx0, t) in q_block chunks; range 1 of a chunk starts at the
        # suffix holding its first row.  Suffix K/V reuse: range 2 of every chunk spans the kept
        # rows of all the prompt's suffixes, each row seeing only its own suffix's window (r2win)
        chunks = [(c0, min(c0 + q_block, t)) for c0 in range(sfx0, t, q_block)]
        if single_suffix_items and keep is None:
            chunks = [(s0 + o, min(s0 + o + q_block, s0 + n)) for sg in segs if sg.r1_len and sg.q_start >= sfx0
                      for s0, n in [(sg.q_start, sg.q_len)] for o in range(0, n, q_block)]
        for c0, c1 in chunks:
            if keep is not None:
                w = r2win[c0:c1]
                lo, hi = min(a for a, _ in w), max(b for _, b in w)
                work.append((c0, c1 - c0, 0, p0, Lp, 0, 0, 0))
                work2.append((lo, hi - lo))
            else:
                r1 = sfx_lo[c0 - sfx0]
                work.append((c0, c1 - c0, c0 - r1, p0, Lp, 0, r1, c1 - r1))
                work2.append((0, 0))
        max_pos = max(max_pos, Lp + max([len(s) for s in tp.suffixes] or [0]))
        p_rows.append((row0, t))
        p_items.append((item0, len(work)))
        p_scored.append((sc0, len(last)))
        nsuf.append(tp.n_suffix)
        padded += tp.padded_tokens
    work = np.asarray(work, dtype=np.int32).reshape(-1, WORK_ITEM_FIELDS)
    reuse = suffix_keep is not None

    def cat(parts):
        return np.concatenate(parts) if parts else np.zeros(0, dtype=np.int32)
    return PackedBatch(
        prompt_ids=list(prompt_ids), n_suffix=nsuf,
        ids=cat(ids), positions=cat(pos),
        segments=segs, work=work, seg_lo=cat(seg_lo),
        last_idx=np.asarray(last, dtype=np.int32), last_segments=lsegs,
        work_last=(np.asarray(lwork, dtype=np.int32).reshape(-1, WORK_ITEM_FIELDS) if reuse
                   else _work_items(lsegs)), num_tokens=t, padded_tokens=padded,
        max_pos=max_pos, kv_cached=kv_cached, q_block=q_block,
        pfx_src=cat(src) if (prefix_offsets is not None and not kv_cached) else None,
        pfx_dst=cat(dst) if (prefix_offsets is not None and not kv_cached) else None,
        prompt_rows=np.asarray(p_rows, dtype=np.int64).reshape(-1, 2),
        prompt_items=np.asarray(p_items, dtype=np.int64).reshape(-1, 2),
        prompt_scored=np.asarray(p_scored, dtype=np.int64).reshape(-1, 2),
        work2=np.asarray(work2, dtype=np.int32).reshape(-1, 2) if reuse else None,
        r2win=np.asarray(r2win, dtype=np.int32).reshape(-1, 2) if reuse else None,
        work2_last=np.asarray(lwork2, dtype=np.int32).reshape(-1, 2) if reuse else None,
        sfx_src=cat(sfx_src) if sfx_src else None,
        sfx_dst=cat(sfx_dst) if sfx_dst else None)


def _items(sg: Segment, q_block: int = Q_BLOCK) -> List[tuple]:
    """One segment -> work items of at most ``q_block`` queries."""
    return [(sg.q_start + off, min(q_block, sg.q_len - off), sg.q_off + off,
             sg.r0_start, sg.r0_len, sg.r0_causal, sg.r1_start, sg.r1_len)
            for off in range(0, sg.q_len, q_block)]


def _work_items(segs: Sequence[Segment], q_block: int = Q_BLOCK) -> np.ndarray:
    """Segments -> [n_items, 8] int32 work items of at most ``q_block`` queries (one segment each)."""
    work = [it for sg in segs for it in _items(sg, q_block)]
    return np.asarray(work, dtype=np.int32).reshape(-1, WORK_ITEM_FIELDS)


def visible_keys(work: np.ndarray, seg_lo: Optional[np.ndarray], row: int,
                 work2: Optional[np.ndarray] = None, r2win: Optional[np.ndarray] = None) -> List[tuple]:
    """(range, first key row, last key row) visible to packed query ``row`` under the work items:
    the semantics of the attention kernel (csrc/kernels/attention.hip), for host-side tests."""
    for it, (q_start, q_len, q_off, r0s, r0l, r0c, r1s, r1l) in enumerate(work.tolist()):
        if q_start <= row < q_start + q_len:
            qi = q_off + row - q_start
            out = []
            if r0l > 0:
                out.append((0, r0s, r0s + (min(r0l - 1, qi) if r0c else r0l - 1)))
            if work2 is not None and work2[it, 1] > 0:
                lo, hi = int(work2[it, 0]), int(work2[it, 0] + work2[it, 1])
                if r2win is not None:
                    lo, hi = max(lo, int(r2win[row, 0])), min(hi, int(r2win[row, 1]))
                if hi > lo:
                    out.append((2, lo, hi - 1))
            if r1l > 0:
                lo = (int(seg_lo[row]) - r1s) if seg_lo is not None else 0
                out.append((1, r1s + lo, r1s + min(r1l - 1, qi)))
            return out
    return []


def split_microbatches(tps: Sequence[TokenizedPrompt], token_budget: int,
                       max_prompts: int = 0, suffix_only: bool = False) -> List[List[int]]:
    """Group consecutive prompts so each micro-batch holds <= token_budget tokens
    (a single oversized prompt still forms its own micro-batch).  ``suffix_only``
    counts only suffix tokens (prefixes served from the prefix K/V cache).

    As few micro-batches as greedy filling needs, evened out: the limit is lowered toward an equal
    share while the count stays the same (128 x 1,344-token prompts under a 24,576 budget: eight
    micro-batches of 21,504 rows instead of seven of 24,192 and one of 2,688, whose GEMMs are
    smaller than one tile round of the chip)."""
    sizes = [tp.num_tokens - (len(tp.prefix) if suffix_only else 0) for tp in tps]

    def pack(limit: int) -> List[List[int]]:
        groups, cur, cur_t = [], [], 0
        for i, n in enumerate(sizes):
            if cur and (cur_t + n > limit or (max_prompts and len(cur) >= max_prompts)):
                groups.append(cur)
                cur, cur_t = [], 0
            cur.append(i)
            cur_t += n
        if cur:
            groups.append(cur)
        return groups

    groups = pack(token_budget)
    if len(groups) > 1:
        # never above the budget: a prompt larger than it forms its own group at any limit (the
        # --max_vram_gb plan sizes the arena for token_budget rows)
        fit = max((n for n in sizes if n <= token_budget), default=0)
        lo, hi = min(max(fit, -(-sum(sizes) // len(groups))), token_budget), token_budget
        while lo < hi:                       # the smallest limit that keeps the greedy count
            mid = (lo + hi) // 2
            if len(pack(mid)) <= len(groups):
                hi = mid
            else:
                lo = mid + 1
        groups = pack(lo)
    return groups
