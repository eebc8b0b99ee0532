"""HIP-graph replay of the whole per-micro-batch forward (resident weights).

The reference dispatches every op of every layer from Python, one prompt at a
time (``/root/reference/utils.py:239-291``).  With small batches (a few short
prompts, or the ``--num_gen_token`` loop that re-runs the full model once per
generated token, ``main.py:65-90``) the GPU work per layer is a few tens of
microseconds and host-side dispatch dominates.

When every shard of this rank is resident in HBM the weight pointers never
change, so embed -> all decoder layers -> final norm -> LM head + softmax of one
micro-batch is captured ONCE as a HIP graph (``torch.cuda.CUDAGraph`` is
hipGraph on ROCm) and replayed with a single launch.  Batch shapes are
bucketed so replays are reused across calls and generation steps:

* tokens -> multiple of ``TOKEN_BUCKET`` (the GEMM M tile; padded rows compute
  garbage that no valid row ever reads: GEMM / RMSNorm rows are independent and
  no attention work item covers them),
* attention work items -> multiple of ``WORK_BUCKET`` (padding items have
  ``q_len = 0``; the kernels return before touching memory),
* scored rows -> multiple of ``SCORE_BUCKET`` (padding gathers row 0; ignored; the
  last decoder layer's single-query work items are padded with ``q_len = 0``).

The metadata of a new batch is copied into the graph's static input tensors
before the replay; the probabilities come out of its static output tensor.
All graphs share one memory pool and are replayed in order on one stream, so
intermediates are shared between them.
"""
from __future__ import annotations

import weakref
from collections import OrderedDict
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch

from .batch import WORK_ITEM_FIELDS, PackedBatch

TOKEN_BUCKET = 256
WORK_BUCKET = 32
SCORE_BUCKET = 16


def _ceil(n: int, m: int) -> int:
    return max(m, (n + m - 1) // m * m)


def bucket_key(batch: PackedBatch) -> Tuple[int, int, int]:
    return (_ceil(batch.num_tokens, TOKEN_BUCKET), _ceil(batch.work.shape[0], WORK_BUCKET),
            _ceil(batch.n_scored, SCORE_BUCKET))


def padded_meta(batch: PackedBatch, key) -> Dict[str, np.ndarray]:
    T, W, S = key
    ids = np.zeros(T, np.int32)
    ids[:batch.num_tokens] = batch.ids
    pos = np.zeros(T, np.int32)
    pos[:batch.num_tokens] = batch.positions
    work = np.zeros((W, WORK_ITEM_FIELDS), np.int32)
    work[:batch.work.shape[0]] = batch.work
    seg_lo = np.zeros(T, np.int32)                         # padding rows: never a query of any item
    seg_lo[:batch.num_tokens] = batch.seg_lo
    last = np.zeros(S, np.int32)
    last[:batch.n_scored] = batch.last_idx
    last_pos = pos[last]                                   # positions of the scored rows
    wl = np.zeros((S, WORK_ITEM_FIELDS), np.int32)        # padding items: q_len 0
    wl[:batch.work_last.shape[0]] = batch.work_last
    return {"ids": ids, "positions": pos, "work": work, "seg_lo": seg_lo, "last_idx": last, "last_pos": last_pos,
            "work_last": wl}


class _Graph:
    def __init__(self, meta: Dict[str, torch.Tensor]):
        self.meta = meta                     # static device inputs
        self.graph = torch.cuda.CUDAGraph()
        self.out: torch.Tensor = None        # static device output [S, V]
        self.replays = 0
        self.entry_ref = None                # DecodeGraphs: the cache entry whose K/V the graph baked in
        self.staging: List[Tuple[Dict[str, np.ndarray], Dict[str, torch.Tensor], Optional[torch.cuda.Event]]] = []
        self.next_stage = 0


class GraphedForward:
    """LRU cache of captured whole-model forwards, keyed by the bucketed shape.

    ``forward(meta, batch) -> probs`` must run embed..head for one micro-batch
    on the current stream using only ``meta`` (device tensors) and resident
    weights; it is called eagerly once (warm-up) and then under capture.
    """

    def __init__(self, device, forward: Callable, max_graphs: int = 8):
        self.dev = torch.device(device)
        self.forward = forward
        self.max_graphs = max_graphs
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs: "OrderedDict[tuple, _Graph]" = OrderedDict()
        self.captures = 0
        self.replays = 0

    def _capture(self, key, batch: PackedBatch) -> _Graph:
        host = padded_meta(batch, key)
        meta = {k: torch.from_numpy(v).to(self.dev) for k, v in host.items()}
        g = _Graph(meta)
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            self.forward(meta, batch)                       # warm-up (lazy inits, autotune)
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        with torch.cuda.graph(g.graph, pool=self.pool, stream=s):
            g.out = self.forward(meta, batch)
        torch.cuda.synchronize(self.dev)
        self.captures += 1
        return g

    def run(self, batch: PackedBatch) -> torch.Tensor:
        """Replay (capturing on first sight of the bucket); returns [n_scored, V] on the device."""
        key = bucket_key(batch)
        g = self.graphs.get(key)
        if g is None:
            if len(self.graphs) >= self.max_graphs:
                self.graphs.popitem(last=False)
            g = self._capture(key, batch)
            self.graphs[key] = g
        else:
            self.graphs.move_to_end(key)
            for k, v in padded_meta(batch, key).items():
                g.meta[k].copy_(torch.from_numpy(v), non_blocking=False)
        g.graph.replay()
        g.replays += 1
        self.replays += 1
        return g.out[:batch.n_scored]


class DecodeGraphs:
    """Graph replay of decode-like calls: the later steps of ``--num_gen_token`` with the prefix
    and suffix K/V caches (every prompt's prefix K/V and its suffixes' earlier tokens come from
    the cache, one new row per suffix is computed) when every weight is in HBM (resident, or the
    HBM cache holding every shard).  Such a step is ~800 launches of a few tens of microseconds
    each; one graph replays them all.

    Unlike :class:`GraphedForward` the shapes are EXACT (no bucket padding: a padded row would
    also be captured into the suffix K/V cache), keyed by the batch's array shapes and the cache
    entry, whose per-layer K/V buffers the graph reads and writes in place; consecutive steps of
    one generation have the same shapes, so one capture serves them all.  The metadata of each
    step (new token ids, positions, work items, cache rows and windows) is copied into the
    graph's static inputs before the replay."""

    def __init__(self, device, forward: Callable, max_graphs: int = 4):
        self.dev = torch.device(device)
        self.forward = forward
        self.max_graphs = max_graphs
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs: "OrderedDict[tuple, _Graph]" = OrderedDict()
        self.captures = 0
        self.replays = 0

    @staticmethod
    def key(batch: PackedBatch, entry) -> tuple:
        """The entry's identity is its fingerprint plus the device address of every per-layer K/V
        buffer the graph reads and writes (an evicted entry's id() and even its addresses can be
        reused by a new one: ``run`` also checks the graph's weak reference to the entry)."""
        ptrs = tuple((n, t.data_ptr()) for n, t in sorted(entry.layers.items()))
        return (entry.key, ptrs, batch.r2_q_block, batch.q_block) + tuple(
            (k, v.shape) for k, v in sorted(batch.host_meta().items()))

    def forget(self, entry) -> None:
        """Drop every graph captured on ``entry`` (called when the prefix cache evicts or drops it:
        its K/V buffers are about to be freed, and a replay would read / write freed HBM)."""
        for k in [k for k, g in self.graphs.items() if g.entry_ref is None or g.entry_ref() in (None, entry)]:
            del self.graphs[k]

    # pinned staging sets per graph: a replay may be enqueued while the previous one (and its
    # metadata copies) still runs, so a set is refilled only after the copies that read it ran
    STAGING_SETS = 2

    def _upload(self, g: _Graph, host: Dict[str, np.ndarray]) -> None:
        """Stream-ordered metadata copies from the graph's persistent pinned staging buffers."""
        if not g.staging:
            for _ in range(self.STAGING_SETS):
                pinned = {k: torch.empty(v.shape, dtype=torch.from_numpy(np.ascontiguousarray(v)).dtype,
                                         pin_memory=True) for k, v in host.items()}
                g.staging.append(({k: t.numpy() for k, t in pinned.items()}, pinned, None))
        views, pinned, ev = g.staging[g.next_stage]
        if ev is not None:
            ev.synchronize()                                 # the copies that last read this set ran
        for k, v in host.items():
            np.copyto(views[k], v, casting="no")
            g.meta[k].copy_(pinned[k], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        g.staging[g.next_stage] = (views, pinned, ev)
        g.next_stage = (g.next_stage + 1) % len(g.staging)

    def run(self, batch: PackedBatch, entry, ids_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Replay (capture on the first sight of the shape) -> the static [n_scored, V] output.
        ``ids_dev``: the batch's token ids as a device int32 tensor, copied over ``batch.ids`` on
        the stream (a speculative step whose new tokens are the previous step's device argmax).
        The metadata goes in by stream-ordered copies from pinned memory, so a replay can be
        enqueued while an earlier one still runs (its static inputs are overwritten after it)."""
        key = self.key(batch, entry)
        host = batch.host_meta()
        g = self.graphs.get(key)
        if g is not None and (g.entry_ref is None or g.entry_ref() is not entry):
            del self.graphs[key]                             # captured on another (dead) entry
            g = None
        if g is None:
            if len(self.graphs) >= self.max_graphs:
                self.graphs.popitem(last=False)
            meta = {k: torch.from_numpy(np.ascontiguousarray(v)).to(self.dev) for k, v in host.items()}
            if ids_dev is not None:
                meta["ids"].copy_(ids_dev)
            g = _Graph(meta)
            g.entry_ref = weakref.ref(entry)
            s = torch.cuda.Stream(self.dev)
            s.wait_stream(torch.cuda.current_stream(self.dev))
            with torch.cuda.stream(s):
                eager = self.forward(meta, batch)            # this step's result (+ lazy inits)
            torch.cuda.current_stream(self.dev).wait_stream(s)
            torch.cuda.synchronize(self.dev)
            with torch.cuda.graph(g.graph, pool=self.pool, stream=s):
                g.out = self.forward(meta, batch)            # captured, not run: the eager pass computed
            torch.cuda.synchronize(self.dev)                 # this step (its cache writes are idempotent)
            self.captures += 1
            self.graphs[key] = g
            return eager
        self.graphs.move_to_end(key)
        self._upload(g, host)
        if ids_dev is not None:
            g.meta["ids"].copy_(ids_dev, non_blocking=True)
        g.graph.replay()
        g.replays += 1
        self.replays += 1
        return g.out
