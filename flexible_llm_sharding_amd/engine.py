"""ShardedRunner — the shard-streaming executor (capability of ``ShardedLlama``).

Reference hot loop (``/root/reference/utils.py:223-305``)::

    for shard in model_shards:                 # weights: load (blocking) ... unload
        for prompt in prompts:                 # one prompt at a time
            for layer in shard: fetch | compute | store

MI355X design of the same schedule:

* weights of shard k+1 stream into the second HBM slot on a copy stream while
  shard k computes (:class:`~.runtime.prefetch.ShardPrefetcher`);
* prompts are packed into micro-batches of up to ``token_budget`` tokens so
  each projection is one large MFMA GEMM (:mod:`.runtime.batch`);
* activations between shards go through the async
  :class:`~.runtime.activations.ActivationStore` (gpu / cpu / disk), the next
  micro-batch's H2D overlapping the current one's compute;
* model parallel (reference default for >1 GPU): shard k runs on rank
  k mod G exactly like ``utils.py:151-153``; hand-offs between ranks are
  RCCL ``isend``/``irecv`` over xGMI issued in a per-rank program fixed before
  the pass (:func:`~.parallel.pipeline.build_programs`: no receive queued ahead
  of work it depends on) into a bounded, runner-lifetime
  :class:`~.parallel.pipeline.StageInbox` (no polling, no shared state).
* data parallel: each rank runs all shards on its slice of prompts; weights
  can be scatter-loaded 1/G per rank and all-gathered over xGMI
  (:mod:`.parallel.data_parallel`).
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import knobs
from .config import MAX_TOKEN_LEN, ModelConfig
from .models.layout import layer_kind
from .models.llama import ExecContext, layer_flops, rope_tables, run_layer
from .ops import get_ops
from .parallel.comm import Comm
from .parallel.pipeline import StageInbox, build_programs, host_wait, rank_items, rx_key
from .parallel.planner import ShardPlan, make_plan
from .runtime import hostmem
from .runtime.activations import ActivationStore, ActRing
from .runtime.batch import Q_BLOCK, Q_BLOCK_MHA, PackedBatch, pack_prompts, split_microbatches
from .runtime.prefetch import ShardPrefetcher
from .runtime.weights import LayerSource
from .utils import trace
from .utils.tokenizer import TokenizedPrompt, tokenize_prompts

# Default micro-batch: 48k packed tokens (the 70B bench's 43k-token pass is one micro-batch: fewer
# GEMM tails and per-layer waits, +1.0-1.2% over 16k with 2 GB less device memory in use,
# profiles/r2_budget_gen); the MLP keeps 16k-row chunks (one 43k chunk measured -1.5%).
TOKEN_BUDGET = 49152
MLP_CHUNK = 16384
MOE_MLP_CHUNK = 65536


def _parse_fault(rank: int):
    """FLS_FAULT="rank:shard" — fault injection for failure-handling tests."""
    spec = knobs.get("FLS_FAULT")
    if not spec:
        return None
    r, _, k = spec.partition(":")
    return int(k or 0) if int(r) == rank else None


class ShardedRunner:
    def __init__(self, cfg: ModelConfig, source: LayerSource, device="cpu", tokenizer=None,
                 layer_num_per_shard: int = 1, storage_location: str = "cpu",
                 disk_folder: str = "./temp", max_activation_in_cpu: int = 100,
                 prefix_attention: str = "bidirectional", token_budget: int = TOKEN_BUDGET,
                 resident: bool = False, comm: Optional[Comm] = None, data_parallel: bool = False,
                 act_dtype: Optional[torch.dtype] = None, n_slots: Optional[int] = None,
                 mlp_chunk: Optional[int] = None, prefetcher: Optional[ShardPrefetcher] = None,
                 verbose: bool = False, resume_dir: Optional[str] = None, checkpoint_every: int = 0,
                 max_token_len: int = MAX_TOKEN_LEN, hip_graphs: bool = False,
                 prefix_kv_cache: bool = False, prefix_cache_entries: int = 8, suffix_kv_cache: bool = False,
                 prune_last_layer: bool = True, pipeline_stages: str = "round_robin",
                 max_vram_gb: Optional[float] = None, hbm_cache_gb: float = 0.0, rx_window: int = 2,
                 exact_reuse: bool = True):
        self.cfg = cfg
        self.src = source
        # layers read from their files every pass (no host-resident copy): host RAM is the limit
        self._streamed_weights = hasattr(source, "stream_into") and source.host_buffer(cfg.layer_names()[0]) is None
        self.dev = torch.device(device)
        self.cuda = self.dev.type == "cuda"
        self.tok = tokenizer
        self.lnps = layer_num_per_shard
        self.storage = storage_location
        self.disk_folder = disk_folder
        # model parallel: parked (early-received) activations per tier before the next slower one
        # (utils.py:179-180's back-pressure bound, parallel/pipeline.py)
        self.max_act = max_activation_in_cpu
        self.rx_window = rx_window
        self.resident = resident
        self.prefix_attention = prefix_attention
        self.vram_plan = None
        if n_slots is None:
            # Three rotating slots (the embedding / LM head in buffers of their own), so the next
            # call's first layers stream in under this call's last ones and no pass waits for its
            # weights at the call boundary: 70B lnps=1 +0.9% (36 -> 1 ms weight wait per pass,
            # profiles/r2_slots_own), 7B lnps=8 +7.8%, 70B lnps=4 +1.6% (profiles/r2_slots7b), for
            # +2.8 GB of HBM on 70B.  The double buffer under a VRAM cap (the 6 GB mode), for
            # resident weights and for the external data-parallel prefetcher.
            n_slots = 3 if (self.cuda and not resident and not max_vram_gb and prefetcher is None) else 2
        self.comm = comm or Comm(0, 1, self.dev)
        self._vram_cap = int(max_vram_gb * 1e9) if max_vram_gb else 0
        if mlp_chunk is None:
            # MoE: the expert GEMMs see k/E of a chunk's rows per expert, and each expert's last
            # 256-row tile is half empty on average: larger chunks (a whole 43k-token micro-batch)
            # keep that waste near 1% (a VRAM cap re-plans the chunk from the MoE buffer sizes)
            mlp_chunk = MOE_MLP_CHUNK if cfg.is_moe else MLP_CHUNK
        self._plan_req = (token_budget, mlp_chunk, n_slots)
        self.names = cfg.layer_names()
        self.L = len(self.names)
        self.plan: ShardPlan = make_plan(self.L, layer_num_per_shard, self.comm.world, self.comm.rank,
                                         data_parallel, pipeline_stages)
        if self.plan.mode == "mp" and self.comm.active:
            # one communicator per directed hand-off edge, created before any memory is measured
            edges = []
            for li in range(self.L - 1):
                a, b = self.plan.owner_of_layer(li), self.plan.owner_of_layer(li + 1)
                if a != b:
                    edges.append((a, b))
            self.comm.setup_p2p_edges(edges)
        if self.comm.active:
            # RCCL creates a communicator's buffers (and, for P2P, its channels) at its first
            # operation, behind a host-blocking rendezvous.  Run one on every group this runner
            # uses now, in one global order on every rank — the default group, every directed
            # hand-off edge, the data-parallel gather group — so none is created lazily inside
            # a pass (where the single-queue schedule does not model it) and a VRAM cap measures
            # their memory
            self.comm.warmup()
            self.comm.warmup_p2p()
            self.comm.warmup_gather(0)         # the score gather to rank 0 after every call
            pcomm = getattr(prefetcher, "comm", None)
            if pcomm is not None and pcomm is not self.comm:
                pcomm.warmup()
        attn_rows = qkv_chunk = 0
        self._outside = None
        self.ops = get_ops(self.dev)
        # this runner's split-K / split-KV scratch (64 MB): the free tail of the activation arena —
        # split-K only runs for <= 512-row GEMMs, whose phase carves a sliver of an arena sized for
        # the whole micro-batch — or, when the arena is too small, a buffer of its own.  Every
        # runner gets the same 64 MB either way, so a capped and an uncapped run take the same GEMM
        # paths (bitwise-equal scores) and a cap is not charged for memory that is already there.
        self._splitk_own = None
        self._splitk_ws = self._splitk_scratch if hasattr(self.ops, "new_workspace") else None
        if max_vram_gb:
            # size the micro-batch and the QKV / MLP chunks to the HBM cap (runtime/memplan.py);
            # re-planned per call once its token count is known (_plan_call)
            from .runtime.memplan import RUNTIME_RESERVE, device_used_bytes, plan_for_vram
            if self.dev.type == "cuda":
                # device memory held outside the caching allocator before any weight slot exists:
                # context, code objects, RCCL buffers (warmed up above) — planned as measured
                self._outside = (device_used_bytes(self.dev) - torch.cuda.memory_reserved(self.dev) + (64 << 20)
                                 + RUNTIME_RESERVE + self._splitk_reserve())
            try:
                # provisional (the call's token count is unknown yet); _plan_call is authoritative
                token_budget, mlp_chunk, attn_rows, qkv_chunk, est, _ = plan_for_vram(
                    cfg, self._vram_cap, layer_num_per_shard, n_slots, token_budget, mlp_chunk,
                    overhead=self._outside, fused_norm=self._fused_norm_planned())
            except ValueError:
                token_budget, mlp_chunk, attn_rows, qkv_chunk, est = 1024, 1024, 0, 0, 0
            self.vram_plan = {"token_budget": token_budget, "mlp_chunk": mlp_chunk, "attn_rows": attn_rows,
                              "qkv_chunk": qkv_chunk, "estimated_peak_bytes": est}
        self.token_budget = token_budget
        self.mlp_chunk = mlp_chunk
        self.data_parallel = data_parallel
        self.verbose = verbose
        self.max_token_len = max_token_len
        self.resume_dir = resume_dir
        self.checkpoint_every = checkpoint_every
        if self.cuda and cfg.head_dim not in (64, 96, 128):
            raise NotImplementedError(f"head_dim={cfg.head_dim}: the HIP attention kernels serve 64, 96 and 128")
        self.act_dtype = act_dtype or (torch.float16 if self.cuda else torch.float32)
        # multi-head models (odd GQA group): 128-row attention items, 4 waves share each K/V tile
        mha = (cfg.num_attention_heads // cfg.num_key_value_heads) % 2 == 1
        self.q_block = Q_BLOCK_MHA if (self.cuda and mha) else Q_BLOCK
        cos, sin = rope_tables(cfg, max(cfg.max_position_embeddings, max_token_len),
                               torch.float16, self.dev)
        self.ctx = ExecContext(cfg, self.ops, self.dev, self.act_dtype, cos, sin, mlp_chunk, qkv_chunk=qkv_chunk,
                               attn_rows=attn_rows)
        decs = [n for n in self.names if layer_kind(n) == "decoder"]
        self.ctx.prune_last = bool(prune_last_layer and decs)
        self.ctx.last_decoder = decs[-1] if decs else ""
        my = [s for s in self.plan.my_shards if len(s)]
        self.my_shards = my
        keep = None
        if hbm_cache_gb and prefetcher is None and not resident:
            if max_vram_gb:
                raise ValueError("--hbm_cache_gb and --max_vram_gb are exclusive (a cache needs HBM, a cap limits it)")
            from .runtime.prefetch import choose_kept_shards
            sizes = [sum(source.nbytes(self.names[i]) for i in sh) for sh in my]
            keep = choose_kept_shards(sizes, int(hbm_cache_gb * 1e9))
        if prefetcher is None and self._piece_pool_ok(source, my, resident, keep, max_vram_gb, resume_dir):
            from .runtime.prefetch import PiecePoolPrefetcher
            prefetcher = PiecePoolPrefetcher(source, self.names, my, self.dev)
        self.prefetcher = prefetcher or ShardPrefetcher(source, self.names, my, self.dev,
                                                        n_slots=n_slots, resident=resident, keep=keep)
        # RMSNorm fused into the projections on the GPU: the norm weights folded into W_qkv /
        # W_gate/up — once for a whole host store (HostStore.norms_folded), or as each layer lands
        # (on the copy stream, before the layer's ready event) — and the row statistic applied in
        # the GEMM epilogue
        self.ctx.fused_norm = self._fused_norm_planned()
        prefolded = bool(getattr(source, "norms_folded", False))
        if prefolded and not self.ctx.fused_norm:
            raise ValueError("the weight source holds norm-folded weights (HostStore.fold_norms): only the "
                             "fused-norm HIP path can run them")
        if self.ctx.fused_norm and not prefolded:
            from .models.llama import fold_layer_norms
            ops = self.ops
            self.prefetcher.on_load = lambda views: fold_layer_norms(ops, views)
        self.h2d_stream = torch.cuda.Stream(self.dev) if self.cuda else None
        self.d2h_stream = torch.cuda.Stream(self.dev) if self.cuda else None
        if self.cuda:
            # the HIP runtime sets up its copy path at the first host<->device copy, holding ~0.2-0.35
            # GB of device memory for a moment (profiles/r4_vram): do it now, while nothing else is
            # allocated, on every stream this runner copies on
            from .runtime.memplan import warm_copy_paths
            warm_copy_paths(self.dev, [getattr(self.prefetcher, "copy_stream", None), self.h2d_stream,
                                       self.d2h_stream])
        if self.vram_plan is not None and self.cuda:
            # the weight slots are raw hipMalloc blocks: the allocator gets the rest of the cap
            from .runtime.memplan import RUNTIME_RESERVE, cap_allocator, device_used_bytes
            self._outside = (device_used_bytes(self.dev) - torch.cuda.memory_reserved(self.dev) + (64 << 20)
                             + RUNTIME_RESERVE + self._splitk_reserve())
            slots = self.prefetcher.planned_hbm_bytes()
            self.vram_plan["allocator_limit_bytes"] = cap_allocator(self.dev, int(max_vram_gb * 1e9), slots)
        self.stats: Dict[str, float] = {}
        self._fault = _parse_fault(self.comm.rank)
        self._store: Optional[ActivationStore] = None
        self._inbox: Optional[StageInbox] = None
        self._mp_start_layer = 0
        # whole-forward HIP graphs: only when every shard is local AND resident (fixed weight pointers)
        self.hip_graphs = bool(hip_graphs and self.cuda and resident and self.plan.mode != "mp"
                               and not resume_dir)
        self._graphs = None
        self._decode_graphs = None
        self._spec: Optional[dict] = None     # an enqueued speculative generation step
        self.last_tokens: List[Optional[np.ndarray]] = []   # last call's greedy token per suffix
        if self.cuda and not self.hip_graphs:
            from .models.llama import Workspace
            self.ctx.ws = Workspace(self.dev, self.act_dtype)   # fixed scratch buffers (VRAM plan)
        # prefix K/V reuse across calls (generation steps): runtime/prefix_cache.py
        self.prefix_cache = None
        if prefix_kv_cache and not self.hip_graphs and not resume_dir:
            from .runtime.prefix_cache import PrefixKVCache
            # under a VRAM cap the entries live in pinned host memory, staged through HBM per layer
            self.prefix_cache = PrefixKVCache(2 * cfg.num_key_value_heads * cfg.head_dim, self.dev,
                                              self.act_dtype, prefix_cache_entries, suffix_reuse=suffix_kv_cache,
                                              host=bool(max_vram_gb))
        # generation (prefix K/V cache): every call row-exact (see "exact K/V reuse" below), unless
        # exact_reuse=False trades that for the small-M kernels
        self.row_exact = self.prefix_cache is not None and exact_reuse
        self._n_decoders = sum(1 for n in self.names if layer_kind(n) == "decoder")
        self._W_all: Dict[str, Dict[str, torch.Tensor]] = {}
        self._h2d0: Optional[int] = None     # prefetcher byte count at the start of the next call
        self._ring: Optional[ActRing] = None
        self._resident_states = 0          # _plan_call: up to this many micro-batches keep a ring slot each

    # ----------------------------------------------------------- helpers
    def _fused_norm_planned(self) -> bool:
        """RMSNorm + QKV fused into one GEMM (HIP backend; FLS_QKV_FOLD=0 turns it off)."""
        return bool(self.cuda and getattr(self.ops, "fused_norm", False) and knobs.get_int("FLS_QKV_FOLD"))

    def tokenize(self, prompts) -> List[TokenizedPrompt]:
        if self.tok is None:
            raise RuntimeError("no tokenizer")
        return tokenize_prompts(self.tok, prompts, self.max_token_len)

    def _owner(self, layer_idx: int) -> int:
        return self.plan.owner_of_layer(layer_idx)

    def _state_shape(self, layer_idx: int, batch: PackedBatch):
        """Shape of the activation produced by ``layer_idx`` (utils.py:281-286)."""
        kind = layer_kind(self.names[layer_idx])
        if kind == "decoder" and self.ctx.prune_last and self.names[layer_idx] == self.ctx.last_decoder:
            return (batch.n_scored, self.cfg.hidden_size)
        if kind in ("embed", "decoder"):
            return (batch.num_tokens, self.cfg.hidden_size)
        if kind == "norm":
            return (batch.n_scored, self.cfg.hidden_size)
        return (batch.n_scored, self.cfg.vocab_size)

    # ------------------------------------------------------------- main
    def __call__(self, prompts) -> List[np.ndarray]:
        """Reference API: list of (prefix, suffixes) -> list of [n_s, 1, V] fp16 arrays."""
        if self.my_shards and prompts and not self.resume_dir and not self.hip_graphs:
            # the first shards' weights do not depend on the prompts: their H2D overlaps tokenization
            if self._h2d0 is None:
                self._h2d0 = self.prefetcher.bytes_h2d
            for k in range(min(self.prefetcher.n_slots, len(self.my_shards))):
                self.prefetcher.prefetch(k)
        t0 = time.perf_counter()
        tps = self.tokenize(prompts)
        t_tok = time.perf_counter() - t0
        out = self.run_tokenized(tps)
        self.stats["host_tokenize_s"] = t_tok
        return out

    def _splitk_reserve(self) -> int:
        """Bytes the plan keeps for this runner's split-K scratch when the arena's tail cannot hold
        it (a small-M call under a cap allocates it lazily, inside the allocator limit: ADVICE r4)."""
        from .ops.hip_backend import SPLITK_WS_BYTES
        return SPLITK_WS_BYTES if self._splitk_ws is not None else 0

    def _splitk_scratch(self):
        from .ops.hip_backend import SPLITK_WS_BYTES
        ws = self.ctx.ws.tail(SPLITK_WS_BYTES) if self.ctx.ws is not None else None
        if ws is not None:
            return ws
        if self._splitk_own is None:
            self._splitk_own = self.ops.new_workspace(self.dev)
        return self._splitk_own

    def _workspace(self):
        """This runner's split-K scratch installed for the calling thread (ops/hip_backend.py)."""
        if self._splitk_ws is None:
            import contextlib
            return contextlib.nullcontext()
        return self.ops.use_workspace(self._splitk_ws)

    def _get_inbox(self) -> StageInbox:
        if self._inbox is None:
            self._inbox = StageInbox(self.comm, self.dev, self.act_dtype, self.storage, self.disk_folder,
                                     str(self.comm.rank), window=self.rx_window, max_parked=self.max_act,
                                     h2d_stream=self.h2d_stream, d2h_stream=self.d2h_stream)
        return self._inbox

    def _mp_program(self, n_batches: int):
        """This rank's hand-off program (every rank derives all ranks' plans: same result)."""
        plans = {r: make_plan(self.L, self.lnps, self.comm.world, r, False, self.plan.stages)
                 for r in range(self.comm.world)}
        progs = build_programs(plans, n_batches, self._mb_major(), self._mp_start_layer)
        return progs[self.comm.rank]

    def _get_store(self) -> ActivationStore:
        if self._store is None:
            self._store = ActivationStore(self.storage, self.dev, self.disk_folder,
                                          tag=str(self.comm.rank) if self.comm.world > 1 else "",
                                          h2d_stream=self.h2d_stream, d2h_stream=self.d2h_stream)
        return self._store

    def _piece_pool_ok(self, source, shards, resident, keep, max_vram_gb, resume_dir) -> bool:
        """``--max_vram_gb`` on one GPU, one layer per shard, weights in pinned host RAM: stream
        each decoder layer as an attention piece + an MLP piece (runtime/prefetch.py
        PiecePoolPrefetcher: 3.12 GB of weight buffers for 70B instead of 3.42, and the next
        layer's attention weights land while this layer's MLP runs)."""
        if knobs.get_int("FLS_PIECE_POOL") == 0:
            return False
        return bool(self.cuda and max_vram_gb and not resident and not keep and not resume_dir
                    and self.plan.mode == "single" and shards and all(len(s) == 1 for s in shards)
                    and (all(source.host_buffer(self.names[s[0]]) is not None for s in shards)
                         or hasattr(source, "stream_into"))
                    and self.act_dtype == torch.float16 and getattr(source, "dtype", torch.float16) == torch.float16)

    def _mb_major(self) -> bool:
        """Model parallel with contiguous stages held resident: micro-batch-major order (a
        micro-batch runs through the whole stage and moves on), so stage r+1 starts after one
        micro-batch instead of after stage r's whole pass.  Same on every rank (a global flag)."""
        return self.plan.mode == "mp" and self.plan.stages == "contiguous" and self.resident

    def schedule(self, n_batches: int):
        """Flat (shard, micro-batch) order.

        Single-GPU / data-parallel runs visit micro-batches in zigzag order
        (0..n-1, then n-1..0, ...) so the micro-batch that ends shard k starts
        shard k+1 and its activation never leaves HBM; the model-parallel
        pipeline uses :func:`~.parallel.pipeline.rank_items` (shard-major, or
        micro-batch-major for resident contiguous stages), the order
        :func:`~.parallel.pipeline.build_programs` derives every rank's
        send / receive program from.
        """
        if self.plan.mode == "mp":
            return rank_items(self.my_shards, n_batches, self._mb_major())
        zig = True
        items = []
        for k in range(len(self.my_shards)):
            order = range(n_batches)
            if zig and k % 2 == 1:
                order = reversed(range(n_batches))
            items += [(k, b) for b in order]
        return items

    # ------------------------------------------------------- exact K/V reuse
    # With the prefix K/V cache (generation) every call runs row-exact: the GEMMs take only
    # row-independent kernels (v10 / v11 tiles: a row's result does not depend on M or on the other
    # rows of the launch), the RMSNorm statistic comes from the row itself, no work item spans two
    # suffixes and no attention is split over blocks; suffix K/V regions start on 64-row key-tile
    # boundaries and the attention's deferred rescale is decided per row.  A row's arithmetic is then
    # the same in every call that computes it: a generation step that reuses the suffixes' cached
    # K/V (--suffix_kv_cache) and computes only the new tokens gives bit for bit the scores of the
    # step that recomputes every suffix token (the exact path), so the greedy tokens are the exact
    # generation's by construction (tests/test_engine_gpu.py::test_suffix_reuse_bitwise_exact).

    def _row_exact(self, on: bool):
        """Context: row-independent kernels for this call (ops + the model's row statistics)."""
        ctx, ops = self.ctx, self.ops
        inner = ops.row_exact(on) if hasattr(ops, "row_exact") else None

        class _RowExact:
            def __enter__(self):
                self.prev = ctx.row_exact
                ctx.row_exact = bool(on)
                if inner is not None:
                    inner.__enter__()

            def __exit__(self, *exc):
                if inner is not None:
                    inner.__exit__(*exc)
                ctx.row_exact = self.prev
        return _RowExact()

    def run_tokenized(self, tps: Sequence[TokenizedPrompt]) -> List[Optional[np.ndarray]]:
        t_start = time.perf_counter()
        spec, self._spec = self._spec, None
        if spec is not None:
            if self._spec_matches(spec, tps):
                return self._finish_spec(spec, tps, t_start)
            self._drop_spec(spec)
        n = len(tps)
        sw = self.cfg.sliding_window
        if sw:
            # windowed attention equals full attention while every sequence fits the window
            # (HF: query i sees keys i - sw + 1 .. i); longer ones would need the band mask
            longest = max((len(tp.prefix) + max((len(s) for s in tp.suffixes), default=0) for tp in tps),
                          default=0)
            if longest > sw:
                raise ValueError(f"a prompt spans {longest} tokens > sliding_window={sw}: "
                                 "sliding-window attention is not implemented")
        entry, cached = self._prefix_entry(tps)
        if self._vram_cap:
            self._plan_call(tps, cached)
        groups = split_microbatches(tps, self.micro_budget(tps, cached), suffix_only=cached)
        # suffix K/V reuse (runtime/prefix_cache.py): rows of every suffix in the entry, and with a
        # cached entry the leading tokens each suffix shares with the last call's (not recomputed)
        sfx_rows, sfx_keep = (entry.suffix_plan(tps, reuse=cached and not self.hip_graphs)
                              if entry is not None else (None, None))
        if sfx_keep is not None and not any(k for ks in sfx_keep for k in ks):
            sfx_keep = None          # nothing to reuse: keep the multi-suffix work items
        kept = sum(k for ks in sfx_keep for k in ks) if sfx_keep is not None else 0
        batches = [pack_prompts([tps[i] for i in g], g, self.prefix_attention,
                                prefix_offsets=[entry.offsets[i] for i in g] if entry is not None else None,
                                kv_cached=cached, q_block=self.q_block,
                                suffix_rows=[sfx_rows[i] for i in g] if sfx_rows is not None else None,
                                suffix_keep=[sfx_keep[i] for i in g] if sfx_keep is not None else None,
                                single_suffix_items=self.row_exact)
                   for g in groups]
        t_pack = time.perf_counter() - t_start
        if self.hip_graphs:
            with self._workspace():
                return self._run_graphed(tps, batches, t_start)
        self.ctx.prefix_entry = entry
        try:
            with self._workspace(), self._row_exact(self.row_exact):
                if self._decode_graphable(batches, cached) and not entry.host:    # (graphs: K/V in HBM)
                    outputs = self._run_graphed(tps, batches, t_start, entry=entry)
                else:
                    outputs = self._run_batches(tps, batches, t_start)
        except BaseException:
            if entry is not None and not cached:
                self.prefix_cache.drop(entry)
            elif entry is not None:
                entry.sfx_ids.clear()        # suffix regions may hold part of this call's rows
            raise
        finally:
            self.ctx.prefix_entry = None
        if entry is not None:
            entry.complete = True
            entry.commit_suffixes(tps, sfx_rows)
            if cached:
                self.prefix_cache.hits += 1
            else:
                self.prefix_cache.misses += 1
        self.stats["prefix_cached"] = float(cached)
        self.stats["suffix_tokens_reused"] = float(kept)
        self.stats["host_pack_s"] = t_pack
        return outputs

    def _plan_call(self, tps, cached: bool) -> None:
        """--max_vram_gb: re-plan micro-batch and chunk sizes for this call's token count (one
        micro-batch whenever the cap allows it: the hidden state then never leaves HBM)."""
        from .runtime.memplan import plan_for_vram
        rows = [tp.num_tokens - (len(tp.prefix) if cached else 0) for tp in tps]
        total = sum(rows)
        tb, mc, n_slots = self._plan_req
        # host-mode prefix K/V cache: its staging buffer; the attention phase then runs over the
        # whole micro-batch (the cache's row copies index it), never in prompt-aligned groups
        pc = self.prefix_cache
        stage = pc.stage.nbytes if (pc is not None and pc.stage is not None) else 0
        tb, mc, ar, qc, est, res = plan_for_vram(self.cfg, self._vram_cap, self.lnps, self.prefetcher.n_slots, tb, mc,
                                        total_tokens=max(1, total), max_prompt_rows=max(rows or [0]),
                                        overhead=self._outside,
                                        weight_bytes=self.prefetcher.planned_hbm_bytes() if self.cuda else None,
                                        fused_norm=self.ctx.fused_norm, extra_bytes=stage,
                                        grouped=self.prefix_cache is None)
        self.token_budget, self.mlp_chunk = tb, mc
        self.ctx.mlp_chunk, self.ctx.attn_rows, self.ctx.qkv_chunk = mc, ar, qc
        # (the plan charged ceil(total / tb) states; a split that needs more micro-batches — whole
        # prompts per micro-batch — parks through the two-slot ring instead)
        self._resident_states = -(-max(1, total) // tb) if res else 0
        self.vram_plan.update({"token_budget": tb, "mlp_chunk": mc, "attn_rows": ar, "qkv_chunk": qc,
                               "estimated_peak_bytes": est, "resident_states": res,
                               "call_tokens": total})

    # model parallel: micro-batches per pipeline stage wanted before the budget may shrink, and the
    # smallest budget it shrinks to (GEMM efficiency falls off below ~8k rows)
    MP_MICRO_PER_STAGE = 2
    MP_MIN_BUDGET = 8192

    def micro_budget(self, tps, cached: bool = False) -> int:
        """Token budget of this call's micro-batches.  Model parallel: a rank computes its next
        layer only when the previous stage hands over a micro-batch, so with fewer micro-batches
        than stages every rank idles part of each round (utilisation ~ micro-batches / stages);
        the budget then shrinks so that there are >= MP_MICRO_PER_STAGE x stages micro-batches
        (not below MP_MIN_BUDGET tokens).  Every rank tokenizes the same prompts, so all ranks
        derive the same split."""
        b = self.token_budget
        if self.plan.mode == "mp" and self.comm.world > 1:
            total = sum(tp.num_tokens - (len(tp.prefix) if cached else 0) for tp in tps)
            want = -(-total // (self.MP_MICRO_PER_STAGE * self.comm.world))
            b = min(b, max(self.MP_MIN_BUDGET, want))
        return b

    def _prefix_entry(self, tps):
        """-> (PrefixEntry or None, cached?).  Model-parallel ranks agree (identical packing)."""
        pc = self.prefix_cache
        if pc is None:
            return None, False
        e = pc.lookup(tps)
        have = 1.0 if e is not None else 0.0
        if self.plan.mode == "mp" and self.comm.active:
            have = self.comm.all_reduce_min(have)
        if have >= 1.0:
            return e, True
        return pc.begin(tps), False

    # ------------------------------------------------------------------ one pass
    # A pass is a list of (shard, micro-batch) items (``schedule``) run by one of two executors —
    # ``_exec_local`` (single GPU, data parallel) and ``_exec_pipeline`` (model parallel, a fixed
    # send / receive program) — over shared per-item routines.  Each lifetime rule lives in one
    # routine: weight slots in ``_enter_shard`` / ``_close_weights`` (acquire, release, prefetch,
    # discard on abort), activation ownership in ``_emit`` (output copy, send, carry, store; a
    # received state leaves its ring slot), receive-ring slots in ``_exec_pipeline`` (release after
    # the item's send), checkpoints in ``_enter_shard`` / the executors.

    class _Pass:
        """Mutable state of one ``_run_batches`` call."""

        def __init__(self, tps, batches, metas, store, items):
            self.tps, self.batches, self.metas, self.store, self.items = tps, batches, metas, store, items
            self.pos = {it: i for i, it in enumerate(items)}
            self.outputs: List[Optional[np.ndarray]] = [None] * len(tps)
            self.out_pending = []      # (batch, host tensor, event, pool buffer)
            self.carry = {}            # micro-batch -> device activation kept across a shard boundary
            self.sends = []            # (tensor, work) of outputs in flight to another rank
            self.shard_ev: List = []   # end-of-shard events on the compute stream (host run-ahead bound)
            self.allocs0, self.alloc_s0 = hostmem.alloc_calls, hostmem.alloc_seconds
            self.flops = 0.0
            self.flops_of = {}              # (micro-batch, pruned layer) -> FLOPs of one decoder layer
            self.compute_s = 0.0
            self.cur_k = -1
            self.W = None
            self.dst_rank = 0
            self.prefetch_due = -1
            self.ck = None
            self.prog = self.inbox = None
            self.pbar = None
            self.ring: Optional[ActRing] = None      # hidden-state slots (storage cpu / disk, local passes)
            self.landed = {}           # micro-batch -> (ring-slot state, H2D event) landed ahead of its use

    def _run_batches(self, tps, batches, t_start: float) -> List[Optional[np.ndarray]]:
        metas = [b.device_tensors(self.dev) for b in batches]   # all uploads before any compute
        store = self._get_store()
        store.bytes_d2h = store.bytes_h2d = store.buffer_waits = 0
        # weights read from the layer files (the small-host-RAM mode): at most one pinned state
        # buffer per micro-batch + ACT_BUFFER_SLACK, the host's run-ahead then waits for a reload
        # to free one instead of growing the pool by its depth (128 prompts of 70B: 12 x 352 MB
        # buffers for 8 micro-batches)
        store.max_buffers = len(batches) + self.ACT_BUFFER_SLACK if self._streamed_weights else None
        pf = self.prefetcher
        # weight bytes of this call: counted from its early prefetch (or the previous call's
        # speculative one), not from the first acquire
        h2d0 = pf.bytes_h2d if self._h2d0 is None else self._h2d0
        self._h2d0 = None
        px = self._Pass(tps, batches, metas, store, self.schedule(len(batches)))
        collective = getattr(pf, "collective", False)
        # the resume point first: ranks agree on it with a collective on the default group, which
        # every rank must reach before any weight gather (a rank without prompts included)
        px.ck, k0, ck_loaded = self._open_checkpoint(tps)
        if not px.items and self.my_shards and collective:
            # a data-parallel rank with no prompts in this call still joins every shard's weight
            # all-gather from the resume point on, so all ranks issue the same collective sequence
            for k in range(k0, len(self.my_shards)):
                pf.acquire(k)
                pf.prefetch(k + 1)
                pf.release(k)
                if px.ck is not None and self._ckpt_due(k):
                    # an empty checkpoint, so the ranks' common resume point still advances
                    px.ck.commit(self._ckpt_key(k), [], self.act_dtype)
        if k0 > 0 or ck_loaded:
            for b, t in ck_loaded.items():
                store.put(b, t.to(self.dev))
            px.items = [it for it in px.items if it[0] >= k0]
            px.pos = {it: i for i, it in enumerate(px.items)}
        if self.plan.mode == "mp" and self.comm.active and px.items:
            px.prog = self._mp_program(len(batches))
            if list(px.prog.items) != list(px.items):
                raise RuntimeError("model-parallel program does not match this rank's schedule")
            px.inbox = self._get_inbox()
            px.inbox.begin_call(max([self._rx_bytes(k, batches[b]) for (k, b), src in zip(px.items, px.prog.src)
                                     if src is not None] or [0]))
        if px.prog is None and self.cuda and self.storage != "gpu" and px.items:
            # hidden states in fixed HBM slots: 1 (the call is one micro-batch: it never leaves HBM),
            # one per micro-batch (the VRAM plan found room for every state: none is parked) or 2
            # (computing + landing; the zigzag carries fit) — exactly the plan's live states
            if self._ring is None:
                self._ring = ActRing(self.dev, self.act_dtype, 1)
            n_ring = 1 if len(batches) == 1 else len(batches) if len(batches) <= self._resident_states else 2
            self._ring.resize(n_ring, max(b.num_tokens for b in batches) * self.cfg.hidden_size)
            px.ring = self._ring
        if self.my_shards and px.items:
            pf.prefetch(px.items[0][0])
        px.pbar = self._progress(len(px.items))
        ok = False
        try:
            if px.prog is not None:
                self._exec_pipeline(px)
            else:
                self._exec_local(px)
            ok = True
        finally:
            self._close_weights(px, ok)
        return self._finish_pass(px, t_start, h2d0, k0)

    def _exec_local(self, px: "_Pass") -> None:
        """Single GPU / data parallel: every shard on every micro-batch, activations through the
        carry window or the store."""
        collective = getattr(self.prefetcher, "collective", False)
        for idx, (k, b) in enumerate(px.items):
            self._enter_shard(px, k)
            state = self._take_state(px, k, b)
            self._prefetch_activation(px, idx)
            state = self._compute(px, k, b, state)
            if collective and px.prefetch_due == k:
                # data parallel: the next shard's all-gather is enqueued after this shard's first
                # compute (a collective kernel sharing a hardware queue with compute then sits
                # behind it, never ahead of it)
                px.prefetch_due = -1
                with trace.range(f"shard{k + 1}:prefetch"):
                    self._prefetch_ahead(k)
            if px.ck is not None and self._ckpt_due(k):
                px.ck.save_state(self._ckpt_key(k), b, state)     # a shard's outputs
            self._emit(px, k, b, state, from_rx=False)

    def _exec_pipeline(self, px: "_Pass") -> None:
        """Model parallel: this rank's items in program order; inputs from the previous stage
        arrive in the StageInbox (receives posted per the program, never ahead of work they depend
        on); a received slot is released once the item's output no longer needs it."""
        prog, inbox = px.prog, px.inbox
        for idx, (k, b) in enumerate(px.items):
            self._enter_shard(px, k)
            for c in prog.posts[idx]:                  # receives due before this item
                kc, bc = px.items[c]
                inbox.post(rx_key(kc, bc), prog.src[c],
                           self._state_shape(self.my_shards[kc][0] - 1, px.batches[bc]), park=c in prog.parked)
            from_rx = prog.src[idx] is not None
            state = inbox.get(rx_key(k, b)) if from_rx else self._take_state(px, k, b)
            if px.ck is not None and self._ckpt_due(k) and state is not None:
                px.ck.save_state(self._ckpt_key(k), b, state)     # a stage's inputs
            self._prefetch_activation(px, idx)
            state = self._compute(px, k, b, state)
            send_w = self._emit(px, k, b, state, from_rx)
            del state
            if from_rx:
                inbox.release(rx_key(k, b), send_w)
            # pending sends are retired per micro-batch (the consumer posts its receive at the
            # point of use); at most SEND_WINDOW outputs stay alive waiting for their consumer
            px.sends = [(t, w) for (t, w) in px.sends if not w.is_completed()]
            while len(px.sends) > self.SEND_WINDOW:
                host_wait(px.sends.pop(0)[1], cuda=self.cuda)
        if px.ck is not None and px.cur_k >= 0 and self._ckpt_due(px.cur_k):
            px.ck.commit(self._ckpt_key(px.cur_k), range(len(px.batches)), self.act_dtype)

    def _enter_shard(self, px: "_Pass", k: int) -> None:
        """Weights of shard k in HBM (the previous shard's released, the next ones prefetched)."""
        if k == px.cur_k:
            return
        pf = self.prefetcher
        if px.ck is not None and px.cur_k >= 0 and self._ckpt_due(px.cur_k):
            px.ck.commit(self._ckpt_key(px.cur_k), range(len(px.batches)), self.act_dtype)
        if self._fault is not None and k == self._fault:
            raise RuntimeError(f"FLS_FAULT injected on rank {self.comm.rank} at shard {k}")
        if px.cur_k >= 0:
            pf.release(px.cur_k)
            self._throttle(px.shard_ev)
        with trace.range(f"shard{k}:acquire"):
            px.W = pf.acquire(k)
        px.cur_k = k
        if getattr(pf, "collective", False):
            px.prefetch_due = k                    # _exec_local: after this shard's first compute
        else:
            with trace.range(f"shard{k + 1}:prefetch"):
                self._prefetch_ahead(k)
        last = self.my_shards[k][-1]
        mp = self.plan.mode == "mp"
        px.dst_rank = self._owner(last + 1) if (mp and last + 1 < self.L) else self.comm.rank

    def _take_state(self, px: "_Pass", k: int, b: int):
        """Input activation of (shard k, micro-batch b) held on this rank (with the activation
        ring: in a slot acquired for it — the embedding writes into it, or the H2D lands in it)."""
        ring, batch = px.ring, px.batches[b]
        if self.my_shards[k][0] == 0:
            if ring is not None:
                self.ctx.embed_out = ring.acquire(b, (batch.num_tokens, self.cfg.hidden_size),
                                                  torch.cuda.current_stream(self.dev))
            return None
        if b in px.carry:
            return px.carry.pop(b)
        if b in px.landed:
            t, ev = px.landed.pop(b)
            px.store.wait_landed(ev)
            return t
        shape = self._state_shape(self.my_shards[k][0] - 1, batch)
        if ring is not None and shape[0] == batch.num_tokens:
            return px.store.get(b, out=ring.acquire(b, shape, px.store.h2d))
        return px.store.get(b)

    def _prefetch_activation(self, px: "_Pass", idx: int) -> None:
        """One-ahead activation prefetch (crosses shard boundaries; parked receives too)."""
        if idx + 1 >= len(px.items):
            return
        k, _ = px.items[idx]
        k2, b2 = px.items[idx + 1]
        if px.prog is not None and px.prog.src[idx + 1] is not None:
            if idx + 1 in px.prog.parked:
                px.inbox.prefetch(rx_key(k2, b2))
        elif self.my_shards[k2][0] > 0 and k2 == k:
            px.store.prefetch(b2)
            self._land(px, k2, b2)
        elif k2 != k and idx + 2 < len(px.items):
            px.store.prefetch(px.items[idx + 2][1])

    def _land(self, px: "_Pass", k: int, b: int) -> None:
        """Bring the next item's parked state into a free ring slot now, ahead of this item's
        compute and of its output's D2H: its H2D then waits only for the D2H of the slot's last
        occupant (two items back), never behind the D2H of the item computing now (with the
        copies of a pass issued only at the point of use, a 16k-budget pass measured ~18 ms of
        H2D wait in front of most micro-batches, profiles/r5_spill)."""
        ring, batch = px.ring, px.batches[b]
        if (ring is None or px.prog is not None or b in px.carry or b in px.landed
                or not ring.has_free() or b not in px.store.keys()):
            return
        shape = self._state_shape(self.my_shards[k][0] - 1, batch)
        if shape[0] != batch.num_tokens:
            return
        px.landed[b] = px.store.get(b, out=ring.acquire(b, shape, px.store.h2d), wait=False)

    def _compute(self, px: "_Pass", k: int, b: int, state):
        """Every layer of shard k on micro-batch b."""
        batch, meta = px.batches[b], px.metas[b]
        idx = px.pos[(k, b)]
        last_use = idx + 1 >= len(px.items) or px.items[idx + 1][0] != k
        tc = time.perf_counter()
        with trace.range(f"shard{k}:mb{b}:compute"):
            for li in self.my_shards[k]:
                name = self.names[li]
                if hasattr(px.W[name], "final_use"):
                    px.W[name].final_use = last_use
                state = run_layer(self.ctx, name, px.W[name], state, batch, meta)
                if layer_kind(name) == "decoder":
                    key = (b, self._pruned(name))        # same FLOPs for every layer of a batch
                    if key not in px.flops_of:
                        px.flops_of[key] = layer_flops(self.cfg, batch, key[1])
                    px.flops += px.flops_of[key]
        px.compute_s += time.perf_counter() - tc
        if px.pbar is not None:
            px.pbar.update(1)
        return state

    def _emit(self, px: "_Pass", k: int, b: int, state, from_rx: bool):
        """Where the output of (shard k, micro-batch b) goes -> the send's work handle, if sent."""
        last = self.my_shards[k][-1]
        ring = px.ring
        if ring is not None and ring.owns(b) and ring.holds(state) < 0:
            # the layer's output left the slot (the pruned last decoder layer, norm, head): the
            # slot's last reader is the compute just enqueued
            ring.release(b, self._event())
        if from_rx and last < self.L - 1 and px.dst_rank == self.comm.rank:
            # the residual GEMMs update the received state in place, so it may still BE the
            # receive-ring slot that inbox.release() hands to the next receive: a state that
            # stays on this rank (contiguous stages) leaves the slot first
            state = state.clone()
        if last == self.L - 1:
            px.out_pending.append(self._start_output_copy(px.batches[b], state))
        elif px.dst_rank != self.comm.rank:
            st = state.contiguous()
            w = self.comm.isend(st, px.dst_rank)
            px.sends.append((st, w))
            return w
        elif self.storage != "gpu" and ((ring is not None and ring.n >= len(px.batches))
                                        or px.pos.get((k + 1, b), len(px.items)) - px.pos[(k, b)]
                                        <= (self.CARRY_WINDOW if ring is None or ring.n >= 2 else 1)):
            # a slot per micro-batch (resident plan): the state stays in its slot for the next
            # shard.  Else re-used within CARRY_WINDOW micro-batch computes (the zigzag boundary
            # micro-batch and its neighbour): a PCIe round trip would only add traffic, keep it in
            # HBM (with two ring slots both carries of a zigzag boundary fit: the neighbour is
            # consumed before anything else needs a slot)
            px.carry[b] = state
        else:
            ev = px.store.put(b, state)
            if ring is not None and ring.owns(b):
                ring.release(b, ev if ev is not None else self._event())
        return None

    def _event(self):
        e = torch.cuda.Event()
        e.record(torch.cuda.current_stream(self.dev))
        return e

    def _close_weights(self, px: "_Pass", ok: bool) -> None:
        """End of a pass: release the held shard; after an aborted one forget every loaded-but-
        unused shard (so a later call's loads never land on weights still waiting to be used)
        and abort the receive ring; after an empty one drop the early prefetch."""
        pf = self.prefetcher
        collective = getattr(pf, "collective", False)
        if px.cur_k >= 0:
            pf.release(px.cur_k)
            px.cur_k = -1
        if not ok:
            if not collective:
                pf.discard_loaded()
            if px.inbox is not None:
                px.inbox.abort()
            if px.ring is not None:
                px.ring.reset()
                self.ctx.embed_out = None
            return
        if px.items or (collective and self.my_shards):
            # the next call's loads continue the slot round-robin (a data-parallel rank with no
            # prompts also went through every shard: its piece / slot numbering must advance with
            # the other ranks', whose gathers it joins)
            pf.epoch += 1
        elif not collective:
            pf.discard_loaded()

    def _finish_pass(self, px: "_Pass", t_start: float, h2d0: int, k0: int) -> List[Optional[np.ndarray]]:
        """Wait for sends and copies, assemble the scores, record the pass statistics."""
        pf, store = self.prefetcher, px.store
        h2d_end = pf.bytes_h2d         # after the last release: loads it triggers count to this call
        for t, w in px.sends:
            w.wait()
        if self.cuda:
            # the compute and activation streams, not the whole device: the weight copy stream
            # may already be streaming the next call's first shards (speculative prefetch)
            torch.cuda.current_stream(self.dev).synchronize()
            self.h2d_stream.synchronize()
            self.d2h_stream.synchronize()
        rx_stats = {}
        if px.inbox is not None:
            px.inbox.end_call()
            rx_stats = {f"rx_{k}": float(v) for k, v in px.inbox.stats.items()}
        self.last_tokens = [None] * len(px.tps)
        for batch, host, ev, pool_buf, am in px.out_pending:
            self._collect(batch, host.numpy(), am, px.outputs)
            if pool_buf is not None:
                store.recycle_host(pool_buf)
        store.clear()
        store.trim()                   # pinned pool follows this call's shapes
        wait_s = pf.take_wait_seconds()
        if px.pbar is not None:
            px.pbar.close()
        if px.ck is not None:
            px.ck.clear()              # run complete: nothing to resume
        wall = time.perf_counter() - t_start
        batches = px.batches
        self.stats = {
            "wall_s": wall, "compute_launch_s": px.compute_s,
            "tokens": float(sum(b.num_tokens for b in batches)),
            "padded_tokens": float(sum(b.padded_tokens for b in batches)),
            "decoder_flops": px.flops, "micro_batches": float(len(batches)),
            "weight_wait_s": wait_s, "weight_h2d_bytes": float(h2d_end - h2d0),
            "act_d2h_bytes": float(store.bytes_d2h), "act_h2d_bytes": float(store.bytes_h2d),
            "resumed_from_shard": float(k0),
            # GPU-side: compute stream stalled on the weight / activation copy streams
            "weight_stall_gpu_s": pf.take_stall_seconds() if self.cuda else 0.0,
            "act_stall_gpu_s": store.take_stall_seconds() if self.cuda else 0.0,
            "pinned_allocs": float(hostmem.alloc_calls - px.allocs0),
            "pinned_alloc_s": hostmem.alloc_seconds - px.alloc_s0,
            "act_buffer_waits": float(store.buffer_waits),
        }
        self.stats.update(rx_stats)
        if self.verbose:
            # utils.py:304 prints "loaded N layers in Ts" per device
            n_layers = sum(len(s) for s in self.my_shards[k0:])
            print(f"{self.dev} rank{self.comm.rank}: loaded {n_layers} layers in {wait_s:.2f}s "
                  f"(exposed weight wait); {len(self.my_shards)} shards, {len(batches)} micro-batches, "
                  f"{self.stats['tokens']:.0f} tokens in {wall:.2f}s")
        return px.outputs

    # model parallel: outputs waiting for their consumer before the host waits for the oldest
    SEND_WINDOW = 3

    def _rx_bytes(self, k: int, batch: PackedBatch) -> int:
        shape = self._state_shape(self.my_shards[k][0] - 1, batch)
        return int(np.prod(shape)) * torch.empty((), dtype=self.act_dtype).element_size()

    def _pruned(self, name: str) -> bool:
        return self.ctx.prune_last and name == self.ctx.last_decoder

    def _speculative_prefetch(self) -> bool:
        """Cached :meth:`_speculative_prefetch_policy` (static for a runner; asked per scanned shard)."""
        v = getattr(self, "_spec_cached", None)
        if v is None:
            v = self._spec_cached = self._speculative_prefetch_policy()
        return v

    def _speculative_prefetch_policy(self) -> bool:
        """Let the prefetch run on into the next call's first shards (same weights every call)?
        On with 3+ slots (the default): the next call's embedding and first layer then load under
        this call's last layers (profiles/r2_slots_own, profiles/r2_slots7b).  With 2 slots the
        only free slot at the end of a call is the last layer's; measured neutral
        (profiles/r1_host_path, profiles/r2_chunk_spec), off.
        Never when resuming (the next call may start
        elsewhere), resident (nothing to load), model parallel, or with the data-parallel
        all-gather prefetcher (no collectives left in flight after a call)."""
        from .parallel.data_parallel import AllGatherPrefetcher
        pf = self.prefetcher
        if pf.n_slots < 3:
            return False
        return (self.cuda and not self.resume_dir and not pf.resident and not self.hip_graphs
                and not (self.plan.mode == "mp" and self.comm.active)
                and not isinstance(pf, AllGatherPrefetcher))

    def _prefetch_ahead(self, k: int) -> None:
        """After acquiring shard k: start loads up to the ``n_slots - 1``-th next shard that uses the
        rotating slots (each lands in the slot of a shard already released; shards with a buffer of
        their own on the way load too); past the last shard, the next call's first shards."""
        pf = self.prefetcher
        if getattr(pf, "all_kept_loaded", None) is not None and pf.all_kept_loaded():
            return                            # (the scan below would walk every shard for nothing)
        n = len(self.my_shards)
        depth = 1 if pf.resident else max(1, pf.n_slots - 1)
        issued, j = 0, k + 1
        while issued < depth and j < k + 1 + n:
            if j < n:
                kk, ep = j, None
            elif j - n < n and self._speculative_prefetch():
                kk, ep = j - n, pf.epoch + 1
            else:
                break
            if not pf.is_kept_loaded(kk):     # kept shards already in HBM load nothing
                pf.prefetch(kk, epoch=ep)
                # with 3+ slots own-buffer shards do not use up the lookahead (the double buffer
                # keeps its one-shard lookahead: data-parallel ranks issue gathers in that order)
                if pf.n_slots < 3 or pf.in_rotation(kk):
                    issued += 1
            j += 1

    def _throttle(self, shard_ev: List, bound: int = 0) -> None:
        """Bound how far the host runs ahead of the GPU to ``RUNAHEAD_SHARDS`` shards.

        Nothing else stops Python from queueing the whole pass: every activation
        buffer that crosses streams (H2D landing buffers, D2H sources) is then
        held by the caching allocator until the GPU catches up, which costs a
        hipMalloc per micro-batch and tens of GB of reserved HBM.  Two shards of
        queued work are far more than the copy streams need to overlap."""
        if not self.cuda:
            return
        e = torch.cuda.Event()
        e.record(torch.cuda.current_stream(self.dev))
        shard_ev.append(e)
        while len(shard_ev) > (bound or self.RUNAHEAD_SHARDS):
            shard_ev.pop(0).synchronize()

    RUNAHEAD_SHARDS = 2
    # an activation consumed again within this many micro-batch computes stays in HBM
    # (zigzag: the boundary micro-batch is next, its neighbour 3 computes later)
    CARRY_WINDOW = 3
    # --weight_cache stream: pinned hidden-state buffers allowed beyond one per micro-batch before
    # the host waits for a reload to free one (profiles/r5_envelope)
    ACT_BUFFER_SLACK = 1

    # ------------------------------------------------------ HIP graphs
    def _forward_all(self, meta: dict, batch: PackedBatch) -> torch.Tensor:
        """embed -> every layer -> norm -> head on resident weights (captured by GraphedForward)."""
        state = None
        for name in self.names:
            state = run_layer(self.ctx, name, self._W_all[name], state, batch, meta)
        return state

    def _decode_graphable(self, batches, cached: bool) -> bool:
        """A decode-like call (suffix K/V reuse: prefixes and kept suffix tokens from the cache)
        on weights that stay at fixed HBM addresses (resident, or an HBM cache holding every
        shard), on one rank: the whole call replays as captured HIP graphs (``DecodeGraphs``)."""
        pf = self.prefetcher
        return bool(cached and self.cuda and self.plan.mode == "single" and not self.resume_dir
                    and knobs.get_int("FLS_DECODE_GRAPHS") and batches
                    and all(b.work2 is not None for b in batches)
                    and (pf.resident or (getattr(pf, "all_kept_loaded", None) is not None and pf.all_kept_loaded())))

    def _run_graphed(self, tps, batches, t_start: float, entry=None) -> List[Optional[np.ndarray]]:
        """Static-weights path: one graph replay per micro-batch (runtime/graphs.py): resident
        full forwards (``--hip_graphs``), or decode-like calls on the prefix / suffix K/V cache
        ``entry`` (exact shapes; the graph reads and writes the entry's per-layer K/V in place).

        Activations never leave HBM (there is no shard boundary inside the
        graph), so ``storage_location`` has nothing to park.
        """
        from .runtime.graphs import DecodeGraphs, GraphedForward
        pf = self.prefetcher
        if not self._W_all:
            for k in range(len(self.my_shards)):
                self._W_all.update(pf.acquire(k))
        if entry is not None:
            if getattr(self, "_decode_graphs", None) is None:
                self._decode_graphs = DecodeGraphs(self.dev, self._forward_all)
                if self.prefix_cache is not None:
                    self.prefix_cache.on_evict.append(self._decode_graphs.forget)
            graphs = self._decode_graphs
            run = lambda b: graphs.run(b, entry)          # noqa: E731
        else:
            if self._graphs is None:
                self._graphs = GraphedForward(self.dev, self._forward_all)
            graphs = self._graphs
            run = graphs.run
        outputs: List[Optional[np.ndarray]] = [None] * len(tps)
        ws, self.ctx.ws = self.ctx.ws, None           # the graph's own memory pool, not the arena
        try:
            pending, ams, flops = self._enqueue_graphed(batches, lambda b, i: run(b))
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream(self.dev))
            if entry is not None and self.spec_steps > 0:
                # the next generation step, enqueued behind this one (see _launch_spec)
                self._spec = self._launch_spec(tps, entry, batches, ams)
        finally:
            self.ctx.ws = ws
        done.synchronize()                            # this step's scores (not the speculative one)
        self._collect_graphed(pending, outputs, len(tps))
        if self._spec is not None:
            self._spec["prev_tokens"] = list(self.last_tokens)
        wall = time.perf_counter() - t_start
        self.stats = {
            "wall_s": wall, "compute_launch_s": wall,
            "tokens": float(sum(b.num_tokens for b in batches)),
            "padded_tokens": float(sum(b.padded_tokens for b in batches)),
            "decoder_flops": flops, "micro_batches": float(len(batches)),
            "weight_wait_s": pf.take_wait_seconds(), "weight_h2d_bytes": 0.0,
            "act_d2h_bytes": 0.0, "act_h2d_bytes": 0.0, "resumed_from_shard": 0.0,
            "graph_captures": float(graphs.captures), "graph_replays": float(graphs.replays),
            "speculative": 0.0,
        }
        return outputs

    def _enqueue_graphed(self, batches, run):
        """Replay every micro-batch (``run(batch, index) -> probs``), its row argmax and the D2H
        of both into pooled pinned buffers, all on the current stream -> (pending, argmax tensors,
        decoder FLOPs)."""
        store = self._get_store()
        pending, ams, flops = [], [], 0.0
        for i, batch in enumerate(batches):
            probs = run(batch, i)
            am = self.ops.argmax_rows(probs)
            nbytes = probs.numel() * probs.element_size()
            pool_buf = store.host_buffer(nbytes + 4 * probs.shape[0])
            host = pool_buf[:nbytes].view(probs.dtype).view(probs.shape)
            host_am = pool_buf[nbytes:nbytes + 4 * probs.shape[0]].view(torch.int32)
            host.copy_(probs, non_blocking=True)     # same stream: ordered before the next replay
            host_am.copy_(am, non_blocking=True)
            pending.append((batch, host, pool_buf, host_am))
            ams.append(am)
            # every unpruned decoder layer has the same count: one evaluation each way (80 per step
            # cost 3.4 ms of host time, on the path that must stay under a generation step's GPU time)
            pruned = [self._pruned(n) for n in self.names if layer_kind(n) == "decoder"]
            n_pruned = sum(pruned)
            flops += (len(pruned) - n_pruned) * layer_flops(self.cfg, batch, False)
            if n_pruned:
                flops += n_pruned * layer_flops(self.cfg, batch, True)
        return pending, ams, flops

    def _collect_graphed(self, pending, outputs, n_prompts: int) -> None:
        store = self._get_store()
        self.last_tokens = [None] * n_prompts
        for batch, host, pool_buf, host_am in pending:
            self._collect(batch, host.numpy(), host_am, outputs)
            store.recycle_host(pool_buf)

    # ------------------------------------------------- speculative generation steps
    # A greedy generation step re-tokenizes ``suffix + decode(tokens)`` (main.py:86-88), which
    # almost always gives the last step's ids plus the new token.  With ``spec_steps`` > 0 (set by
    # api.generation_loop: steps still to come) a decode-graphed call enqueues the NEXT step right
    # behind itself on that assumption, its new-token ids copied on the device from this step's
    # argmax, so the GPU computes it while the host collects, decodes, re-tokenizes and packs.  The
    # next call compares its real tokenization with the assumption: equal -> that step was computed
    # from exactly the inputs the call would pack (same graph, same metadata: bitwise the same
    # scores) and only its copies are waited for; different -> it is dropped and the call runs
    # normally (the suffix regions' committed ids are the last step's, so the normal step
    # recomputes every row from the first differing token, overwriting the speculative rows).
    spec_steps = 0

    def _launch_spec(self, tps, entry, batches, ams) -> Optional[dict]:
        if not (knobs.get_int("FLS_SPEC_DECODE") and self._decode_graphs is not None
                and all(b.work2 is not None and b.num_tokens == b.n_scored for b in batches)):
            return None
        try:
            spec_tps = [TokenizedPrompt(list(tp.prefix), [list(s) + [0] for s in tp.suffixes], tp.padded_len + 1,
                                        [len(s) for s in tp.suffixes]) for tp in tps]
            groups = split_microbatches(spec_tps, self.micro_budget(spec_tps, True), suffix_only=True)
            if groups != [list(b.prompt_ids) for b in batches]:
                return None
            rows, keep = [], []
            for j, tp in enumerate(spec_tps):
                if j >= len(entry.sfx_rows) or len(tp.suffixes) != len(entry.sfx_rows[j]):
                    return None
                if any(len(s) > cap for s, cap in zip(tp.suffixes, entry.sfx_caps[j])):
                    return None                       # a suffix outgrew its cache region
                rows.append(list(entry.sfx_rows[j]))
                keep.append([len(s) - 1 for s in tp.suffixes])
            sb = [pack_prompts([spec_tps[i] for i in g], g, self.prefix_attention,
                               prefix_offsets=[entry.offsets[i] for i in g], kv_cached=True, q_block=self.q_block,
                               suffix_rows=[rows[i] for i in g], suffix_keep=[keep[i] for i in g]) for g in groups]
            if not self._decode_graphable(sb, True) or any(x.num_tokens != b.n_scored for x, b in zip(sb, batches)):
                return None
            graphs = self._decode_graphs
            pe, self.ctx.prefix_entry = self.ctx.prefix_entry, entry     # (a capture's eager forward reads it)
            try:
                pending, ams2, flops = self._enqueue_graphed(sb, lambda b, i: graphs.run(b, entry, ids_dev=ams[i]))
            finally:
                self.ctx.prefix_entry = pe
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream(self.dev))
            return {"tps": spec_tps, "entry": entry, "rows": rows, "batches": sb, "pending": pending, "ams": ams2,
                    "flops": flops, "done": done, "prev_tokens": None, "t0": time.perf_counter()}
        except Exception:
            return None

    def _spec_matches(self, spec: dict, tps) -> bool:
        """Is ``tps`` (this call's tokenization) what the speculative step assumed: the same
        prefixes, every suffix the last step's ids plus that step's greedy token?"""
        prev = spec["prev_tokens"]
        exp = spec["tps"]
        if prev is None or len(tps) != len(exp) or any(t is None for t in prev):
            return False
        for j, (tp, e) in enumerate(zip(tps, exp)):
            if tp.prefix != e.prefix or len(tp.suffixes) != len(e.suffixes):
                return False
            for si, (s, es) in enumerate(zip(tp.suffixes, e.suffixes)):
                if len(s) != len(es) or s[:-1] != es[:-1] or s[-1] != int(prev[j][si, 0]):
                    return False
        return True

    def _finish_spec(self, spec: dict, tps, t_start: float) -> List[Optional[np.ndarray]]:
        entry = spec["entry"]
        if self.spec_steps > 0:
            ws, self.ctx.ws = self.ctx.ws, None
            try:
                self._spec = self._launch_spec(tps, entry, spec["batches"], spec["ams"])
            finally:
                self.ctx.ws = ws
        spec["done"].synchronize()
        outputs: List[Optional[np.ndarray]] = [None] * len(tps)
        self._collect_graphed(spec["pending"], outputs, len(tps))
        if self._spec is not None:
            self._spec["prev_tokens"] = list(self.last_tokens)
        entry.complete = True
        entry.commit_suffixes(tps, spec["rows"])
        self.prefix_cache.hits += 1
        wall = time.perf_counter() - t_start
        graphs = self._decode_graphs
        batches = spec["batches"]
        self.stats = {
            "wall_s": wall, "compute_launch_s": wall,
            "tokens": float(sum(b.num_tokens for b in batches)),
            "padded_tokens": float(sum(b.padded_tokens for b in batches)),
            "decoder_flops": spec["flops"], "micro_batches": float(len(batches)),
            "weight_wait_s": 0.0, "weight_h2d_bytes": 0.0, "act_d2h_bytes": 0.0, "act_h2d_bytes": 0.0,
            "resumed_from_shard": 0.0, "graph_captures": float(graphs.captures),
            "graph_replays": float(graphs.replays), "speculative": 1.0, "prefix_cached": 1.0,
            "suffix_tokens_reused": float(sum(len(s) - 1 for tp in tps for s in tp.suffixes)), "host_pack_s": 0.0,
        }
        return outputs

    def _drop_spec(self, spec: dict) -> None:
        spec["done"].synchronize()
        store = self._get_store()
        for _, _, pool_buf, _ in spec["pending"]:
            store.recycle_host(pool_buf)
        self.spec_dropped += 1

    spec_dropped = 0

    # ------------------------------------------------- progress / resume
    def _progress(self, total: int):
        """tqdm bar on rank 0 when verbose (the reference's tqdm over shards, utils.py:226-238)."""
        if not (self.verbose and self.comm.rank == 0):
            return None
        try:
            from tqdm import tqdm
        except ImportError:
            return None
        return tqdm(total=total, desc=f"{self.dev} shard x micro-batch", unit="step")

    def _ckpt_due(self, k: int) -> bool:
        """Checkpoint at shard k (index into my_shards)?

        Single / data parallel: after shard k, its outputs (never after the lm_head shard).
        Model parallel: the inputs of shard k, every ``every`` global shards (a stage boundary
        the consumer holds, so a restart needs no in-flight pipeline state)."""
        e = self.checkpoint_every
        if e <= 0:
            return False
        if self.plan.mode == "mp":
            g = self.plan.all_shards.index(self.my_shards[k])
            return g > 0 and g % e == 0 and self.my_shards[k][0] > 0
        return ((k + 1) % e == 0 and k + 1 < len(self.my_shards)
                and self.my_shards[k][-1] < self.L - 1)

    def _ckpt_key(self, k: int) -> int:
        """Checkpoint key: next local shard (single / DP) or the stage's first layer (MP)."""
        return self.my_shards[k][0] if self.plan.mode == "mp" else k + 1

    def _open_checkpoint(self, tps):
        """-> (RunCheckpoint or None, first local shard to run, states to start from).

        Data-parallel ranks agree on a shard they all hold.  Model-parallel ranks agree on the
        latest stage boundary whose consumer holds its inputs: every rank skips the shards
        before it, the consumer restarts from the checkpointed inputs, the others as usual."""
        self._mp_start_layer = 0
        if not self.resume_dir or not self.my_shards:
            return None, 0, {}
        from .runtime.checkpoint import RunCheckpoint, run_fingerprint
        fp = run_fingerprint(self.cfg, [tp.prefix + [t for s in tp.suffixes for t in s] + [-1] for tp in tps],
                             lnps=self.lnps, budget=self.token_budget, attn=self.prefix_attention,
                             world=self.comm.world, rank=self.comm.rank, dp=self.data_parallel,
                             dtype=str(self.act_dtype), every=self.checkpoint_every,
                             prune=self.ctx.prune_last, stages=self.plan.stages)
        ck = RunCheckpoint(self.resume_dir, fp, self.comm.rank)
        have = set(ck.available())
        if self.plan.mode == "mp":
            allsets = self.comm.all_gather_object(sorted(have)) if self.comm.world > 1 else [sorted(have)]
            usable = [L for r, keys in enumerate(allsets) for L in keys if self.plan.owner_of_layer(L) == r]
            Lc = max(usable) if usable else 0
            if Lc == 0:
                return ck, 0, {}
            self._mp_start_layer = Lc
            k0 = next((k for k, sh in enumerate(self.my_shards) if sh[0] >= Lc), len(self.my_shards))
            loaded = ck.load(Lc) if k0 < len(self.my_shards) and self.my_shards[k0][0] == Lc else {}
            if self.verbose:
                print(f"rank{self.comm.rank}: resuming at layer {Lc} (local shard {k0}) from {ck.dir}")
            return ck, k0, loaded
        if self.comm.world > 1:
            for other in self.comm.all_gather_object(sorted(have)):
                have &= set(other)
        k0 = max(have) if have else 0
        if k0 and self.verbose:
            print(f"rank{self.comm.rank}: resuming at shard {k0} from {ck.dir}")
        return ck, k0, (ck.load(k0) if k0 else {})

    def _collect(self, batch: PackedBatch, probs: np.ndarray, am, outputs) -> None:
        """Host scores of a finished micro-batch into ``outputs`` (prompt order) and its greedy
        tokens into ``self.last_tokens`` (``am``: the rows' argmax, computed on the device)."""
        am = am.numpy() if am is not None else None
        r = 0
        for j, pid in enumerate(batch.prompt_ids):
            ns = batch.n_suffix[j]
            outputs[pid] = np.expand_dims(probs[r:r + ns].astype(np.float16, copy=True), axis=1)
            if am is not None:
                self.last_tokens[pid] = am[r:r + ns].astype(np.int64).reshape(ns, 1)
            r += ns

    def _start_output_copy(self, batch: PackedBatch, probs: torch.Tensor):
        """D2H of a micro-batch's probabilities and of their row argmax (the greedy token of
        each suffix: api.generation_loop needs no host pass over the [n_s, V] scores)."""
        am = self.ops.argmax_rows(probs) if hasattr(self.ops, "argmax_rows") else None
        if not self.cuda:
            return batch, probs.detach().to(torch.float16).cpu(), None, None, am
        store = self._get_store()
        nbytes = probs.numel() * probs.element_size()
        pool_buf = store.host_buffer(nbytes + 4 * probs.shape[0])
        host = pool_buf[:nbytes].view(probs.dtype).view(probs.shape)
        host_am = pool_buf[nbytes:nbytes + 4 * probs.shape[0]].view(torch.int32)
        self.d2h_stream.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(self.d2h_stream):
            host.copy_(probs, non_blocking=True)
            probs.record_stream(self.d2h_stream)
            if am is not None:
                host_am.copy_(am, non_blocking=True)
                am.record_stream(self.d2h_stream)
            ev = torch.cuda.Event()
            ev.record(self.d2h_stream)
        return batch, host, ev, pool_buf, (host_am if am is not None else None)

    def close(self):
        if self._spec is not None:             # an enqueued speculative step finishes first
            self._spec["done"].synchronize()
            self._spec = None
        # captured graphs and per-layer weight views hold the weight slots (resident: the whole
        # model) and the K/V caches: drop them with the runner
        self._graphs = self._decode_graphs = None
        self._W_all = {}
        self.prefix_cache = None
        self.ctx.prefix_entry = None
        if self._inbox is not None:
            self._inbox.close()
            self._inbox = None
        self.prefetcher.close()
        if hasattr(self.src, "close"):
            self.src.close()           # the streaming source's pinned ring
        if self._store is not None:
            self._store.close()
            self._store = None
        self._splitk_ws = self._splitk_own = None
