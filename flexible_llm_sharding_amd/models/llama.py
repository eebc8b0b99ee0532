"""Llama layer execution on packed weights and packed token batches.

Equivalent of the per-layer dispatch in the reference hot loop
(``/root/reference/utils.py:266-291``):

* ``model.embed_tokens``  -> embedding gather of the packed token ids;
* ``model.layers.i``      -> pre-norm decoder block; the prefix and all its
  suffixes are processed in one pass (shared-prefix attention work items);
* ``model.norm``          -> gather of each suffix's scored token + RMSNorm
  (``utils.py:281-286``);
* ``lm_head``             -> logits + vocab softmax, fp16 probabilities
  (``utils.py:287-290``).

The op implementations come from an ``ops`` backend (HIP kernels on MI355X,
PyTorch on CPU).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from ..config import ModelConfig, MAX_TOKEN_LEN
from .layout import layer_kind


def rope_inv_freq(cfg: ModelConfig):
    """-> (inverse frequencies [hd/2] fp32, cos/sin scale) for the config's RoPE.

    Static scalings only change the tables, so the fused RoPE epilogue of the
    QKV GEMM serves all of them: ``linear`` (positions / factor), ``llama3``
    (Llama-3.1: long wavelengths / factor, a smooth ramp between) and ``yarn``
    (NTK-by-parts ramp between interpolated and extrapolated frequencies, cos/sin
    scaled by the attention factor) — the formulas of HF ``modeling_rope_utils``.
    """
    hd = cfg.head_dim
    base = float(cfg.rope_theta)
    inv = 1.0 / (base ** (torch.arange(0, hd, 2, dtype=torch.int64).float() / hd))
    rs = cfg.rope_scaling
    if not rs:
        return inv, 1.0
    kind = rs.get("rope_type", rs.get("type"))
    factor = float(rs.get("factor") or 1.0)
    if kind == "linear":
        return inv / factor, 1.0
    orig = float(rs.get("original_max_position_embeddings") or cfg.max_position_embeddings)
    if kind == "llama3":
        lo_f, hi_f = float(rs.get("low_freq_factor", 1.0)), float(rs.get("high_freq_factor", 4.0))
        wavelen = 2 * math.pi / inv
        out = torch.where(wavelen > orig / lo_f, inv / factor, inv)
        smooth = (orig / wavelen - lo_f) / (hi_f - lo_f)
        smoothed = (1 - smooth) * out / factor + smooth * out
        medium = (wavelen >= orig / hi_f) & (wavelen <= orig / lo_f)
        return torch.where(medium, smoothed, out), 1.0
    if kind == "yarn":
        if rs.get("factor") is None:
            factor = cfg.max_position_embeddings / orig

        def mscale(scale, m=1.0):
            return 1.0 if scale <= 1 else 0.1 * m * math.log(scale) + 1.0
        att = rs.get("attention_factor")
        if att is None:
            m, m_all = rs.get("mscale"), rs.get("mscale_all_dim")
            att = (mscale(factor, m) / mscale(factor, m_all)) if (m and m_all) else mscale(factor)
        beta_fast, beta_slow = float(rs.get("beta_fast") or 32), float(rs.get("beta_slow") or 1)

        def corr_dim(n_rot):
            return (hd * math.log(orig / (n_rot * 2 * math.pi))) / (2 * math.log(base))
        lo, hi = corr_dim(beta_fast), corr_dim(beta_slow)
        if rs.get("truncate", True):
            lo, hi = math.floor(lo), math.ceil(hi)
        lo, hi = max(lo, 0), min(hi, hd - 1)
        if lo == hi:
            hi += 0.001
        ramp = ((torch.arange(hd // 2, dtype=torch.float32) - lo) / (hi - lo)).clamp(0, 1)
        extrap = 1 - ramp
        return (inv / factor) * (1 - extrap) + inv * extrap, float(att)
    if kind == "longrope":
        # Phi-3 LongRoPE: per-frequency divisors; short_factor while the sequence stays within
        # the pretraining context (always, under the token cap: ModelConfig.validate), and the
        # attention factor from max_position_embeddings / original when ``factor`` is unset
        if rs.get("factor") is None:
            factor = cfg.max_position_embeddings / orig
        att = rs.get("attention_factor")
        if att is None:
            att = 1.0 if factor <= 1.0 else math.sqrt(1 + math.log(factor) / math.log(orig))
        ext = torch.tensor(rs["short_factor"], dtype=torch.float32)
        shape = torch.arange(0, hd, 2, dtype=torch.int64).float() / hd
        return 1.0 / (ext * base ** shape), float(att)
    raise NotImplementedError(f"rope_scaling {rs}")


def rope_tables(cfg: ModelConfig, max_pos: int = MAX_TOKEN_LEN, table_dtype=torch.float16,
                device="cpu"):
    """cos/sin [max_pos, hd/2] in fp32 holding ``table_dtype``-rounded values.

    HF (4.31-4.35) builds ``cos_cached``/``sin_cached`` in fp32 and the reference
    casts every buffer to fp16 (``utils.py:118-119``); rotate-half uses
    ``emb = cat(freqs, freqs)`` so only hd/2 distinct frequencies exist.
    """
    inv_freq, att = rope_inv_freq(cfg)
    t = torch.arange(max(max_pos, 1), dtype=torch.float32)
    freqs = torch.outer(t, inv_freq)
    cos, sin = freqs.cos() * att, freqs.sin() * att
    if table_dtype is not None and table_dtype != torch.float32:
        cos, sin = cos.to(table_dtype).float(), sin.to(table_dtype).float()
    return cos.contiguous().to(device), sin.contiguous().to(device)


class Workspace:
    """One scratch arena reused by every decoder layer: the attention phase carves
    [normed input | QKV | attention output] out of it, the MLP phase (where those are dead)
    [normed chunk | SwiGLU chunk].  It is sized once, at the largest micro-batch seen, so the
    caching allocator sees one fixed block instead of four fresh, differently sized
    allocations per layer and micro-batch, and the two phases share the same bytes
    (profiles/r2_vram).  Every user runs on the compute stream, so carving the same bytes in
    the next phase / layer is ordered after their last reader."""

    def __init__(self, device, dtype):
        self.device, self.dtype = device, dtype
        self.buf: Optional[torch.Tensor] = None
        self.pos = 0

    def reset(self) -> None:
        self.pos = 0

    def take(self, rows: int, cols: int) -> torch.Tensor:
        n = rows * cols
        n_al = (n + 127) // 128 * 128            # 256-byte aligned views
        if self.buf is None or self.pos + n_al > self.buf.numel():
            if self.pos:
                raise RuntimeError("workspace phase outgrew its arena; reserve() the phase first")
            self.buf = None
            self.buf = torch.empty(n_al, dtype=self.dtype, device=self.device)
        v = self.buf[self.pos:self.pos + n].view(rows, cols)
        self.pos += n_al
        return v

    def reserve(self, *shapes) -> None:
        """Grow the arena (between phases) to hold ``shapes`` = [(rows, cols), ...] at once."""
        need = sum((r * c + 127) // 128 * 128 for r, c in shapes)
        if self.buf is None or self.buf.numel() < need:
            self.buf = None
            self.buf = torch.empty(need, dtype=self.dtype, device=self.device)
        self.pos = 0

    def tail(self, nbytes: int) -> Optional[torch.Tensor]:
        """The arena's free bytes after the current phase's carvings, as a uint8 view of exactly
        ``nbytes`` (None if fewer are free): scratch for a kernel that runs between this phase's
        carvings and the next (the small-M split-K GEMM partials; the compute stream orders it)."""
        if self.buf is None:
            return None
        es = self.buf.element_size()
        start = (self.pos * es + 255) // 256 * 256
        if start + nbytes > self.buf.numel() * es:
            return None
        return self.buf.view(torch.uint8)[start:start + nbytes]

    def nbytes(self) -> int:
        return 0 if self.buf is None else self.buf.numel() * self.buf.element_size()


@dataclass
class ExecContext:
    cfg: ModelConfig
    ops: object
    device: torch.device
    act_dtype: torch.dtype
    cos: torch.Tensor
    sin: torch.Tensor
    mlp_chunk: int = 16384       # rows per gate/up + down chunk (bounds the [T, I] buffer)
    qkv_chunk: int = 0           # rows per RMSNorm + QKV chunk (0: all rows; bounds the normed-input buffer)
    attn_rows: int = 0           # attention phase in prompt-aligned groups of <= this many rows (0: one group)
    prefix_entry: Optional[object] = None   # runtime.prefix_cache.PrefixEntry of the current call
    # the last decoder layer computes only the scored rows (its K/V still cover every token):
    # nothing downstream reads the other rows (final norm gathers the scored rows, utils.py:284-286)
    prune_last: bool = True
    last_decoder: str = ""
    ws: Optional[Workspace] = None          # scratch arena (None: fresh allocations, e.g. graph capture)
    # RMSNorm + QKV projection fused (HIP): every decoder layer's ln1 is folded into its W_qkv when
    # the weights land (fold_layer_norms, called by the prefetcher on its copy stream) and the QKV
    # GEMM reads the raw hidden state, scaling each row by its rsqrt(mean(x^2) + eps) in the epilogue
    fused_norm: bool = False
    embed_out: Optional[torch.Tensor] = None   # destination of the next embedding gather (engine's ring)
    # Fused norm: the residual GEMMs also write each row's partial sums of squares (fp32 per 128
    # columns, Epi::ss) into ss_buf, and the next norm-folded projection of the SAME rows takes its
    # statistic from them (a [rows, H/128] read) instead of a pass over the hidden state (row_rstd).
    # ss_key names what ss_buf holds: (id(batch), decoder index, "attn" | "mlp", rows) -- valid for
    # the projection right after that residual GEMM on this rank (any state parked and reloaded in
    # between keeps its values); anything else (another micro-batch, the first layer, a grouped
    # attention phase, MoE) misses and computes the same partials from the hidden state (row_stat:
    # bitwise the epilogue's).  Reset at every call's embedding.
    # generation with the K/V caches (engine "exact K/V reuse"): every row's arithmetic independent
    # of the other rows of the call (row-exact GEMM paths, the row statistic from the row itself)
    row_exact: bool = False
    ss_buf: Optional[torch.Tensor] = None      # the arena-backed buffer (grown, reused)
    ss_cur: Optional[torch.Tensor] = None      # the buffer the last residual GEMM wrote
    ss_key: Optional[tuple] = None

    def phase(self, *shapes) -> None:
        """Start a workspace phase that will carve ``shapes`` (rows, cols) in order."""
        if self.ws is not None:
            self.ws.reserve(*shapes)

    def scratch(self, rows: int, cols: int) -> Optional[torch.Tensor]:
        return self.ws.take(rows, cols) if self.ws is not None else None

    def scratch_f32(self, n: int) -> Optional[torch.Tensor]:
        """n fp32 values from the current phase (2 fp16 columns each); reserve (1, 2 n)."""
        t = self.scratch(1, 2 * n)
        return t.view(torch.float32).view(n) if t is not None else None

    def ss_take(self, rows: int, key: Optional[tuple] = None) -> Optional[torch.Tensor]:
        """The [rows, H/128] partial-sums buffer the next residual GEMM writes (None when the path
        is off: unfused norm, MoE, or a hidden size the 128-column partials do not divide).  With
        ``key`` holding (the partials about to be read), that same buffer.  Eagerly, one buffer
        grown to the largest micro-batch (like the workspace); without a workspace (graph capture)
        a fresh one per forward from the graph's own pool, never a buffer that eager code frees."""
        H = self.cfg.hidden_size
        if not self.fused_norm or self.cfg.is_moe or H % 128 or self.row_exact:
            return None
        if key is not None and self.ss_key == key and self.ss_cur is not None:
            return self.ss_cur[:rows]
        if self.ws is None:
            self.ss_cur = torch.empty(rows, H // 128, dtype=torch.float32, device=self.device)
            return self.ss_cur
        if self.ss_buf is None or self.ss_buf.shape[0] < rows:
            self.ss_buf = None
            self.ss_buf = torch.empty(rows, H // 128, dtype=torch.float32, device=self.device)
        self.ss_cur = self.ss_buf[:rows]
        return self.ss_cur

    def rstd(self, x: torch.Tensor, key: Optional[tuple], out=None, rows: Optional[slice] = None) -> torch.Tensor:
        """Row statistic rsqrt(mean(x^2) + eps) of x: from the partial sums the residual GEMM named
        ``key`` left (rows ``rows`` of them) when they are there, else from a pass over x."""
        eps = self.cfg.rms_norm_eps
        if key is not None and self.ss_key == key and self.ss_cur is not None:
            ss = self.ss_cur[:key[3]]
            return self.ops.rstd_from_ss(ss[rows] if rows is not None else ss, self.cfg.hidden_size, eps, out=out)
        return self.row_stat(x, out=out)

    def row_stat(self, x: torch.Tensor, out=None) -> torch.Tensor:
        """The statistic from a pass over x.  With 128-column partials it is computed exactly as the
        residual GEMM epilogue's partials + rstd_from_ss would give it, so a row's statistic (and the
        scores) do not depend on whether its partials survived: a state received from another
        pipeline rank, parked in host memory, after grouped attention or in the pruned last layer
        gets the same bits as one straight from the residual GEMM."""
        H, eps = self.cfg.hidden_size, self.cfg.rms_norm_eps
        if H % 128 == 0 and H <= 16384 and hasattr(self.ops, "row_stat"):
            return self.ops.row_stat(x, eps, out=out)
        return self.ops.row_rstd(x, eps, out=out)


def _decoder_index(layer_name: str) -> int:
    try:
        return int(layer_name.rsplit(".", 1)[1])
    except (IndexError, ValueError):
        return -10


def run_embed(ctx: ExecContext, W: Dict[str, torch.Tensor], meta: dict) -> torch.Tensor:
    """Embedding gather (Granite: scaled by embedding_multiplier in the same kernel), into the
    engine's activation buffer when it set one."""
    out, ctx.embed_out = ctx.embed_out, None
    ctx.ss_key, ctx.ss_cur = None, None       # a new call / micro-batch: no partials carry over
    return ctx.ops.embed(meta["ids"], W["embed"], ctx.act_dtype, scale=ctx.cfg.embedding_multiplier, out=out)


def _resid(ctx: ExecContext, a: torch.Tensor, w: torch.Tensor, x: torch.Tensor, bias=None, ss=None) -> torch.Tensor:
    """x + r * (a @ w^T (+ bias)): the fused residual GEMM, in place on x (r: Granite's
    residual_multiplier, scaled in the epilogue; 1 otherwise); ``ss``: the rows' partial sums of
    squares too (ExecContext.ss_buf)."""
    kw = {"ss": ss} if ss is not None else {}
    return ctx.ops.linear_residual(a, w, x, bias=bias, alpha=ctx.cfg.residual_multiplier, **kw)


def fold_layer_norms(ops, views: Dict[str, torch.Tensor]) -> None:
    """Fold a decoder layer's RMSNorm weights into the projections that read the normalised rows,
    in place (W_qkv[n, k] *= ln1[k]; dense MLPs: W_gate/up[n, k] *= ln2[k]): the fused path then
    needs no normalised copy of the hidden state (ExecContext.fused_norm).  ``views`` may hold one
    piece of the layer (attention or MLP); each pair present is folded.  Called once per load, on
    the stream that loaded the weights, or once for a whole host store (HostStore.fold_norms)."""
    if "wqkv" in views and "ln1" in views:
        ops.fold_norm(views["wqkv"], views["ln1"])
    if "wgu" in views and "ln2" in views and views["wgu"].dim() == 2:
        ops.fold_norm(views["wgu"], views["ln2"])


CHUNK_ALIGN = 3072     # row multiple of the QKV / MLP chunks: 8 v11 tiles (profiles/r4_gemm)


def balanced_step(rows: int, limit: int, align: int = 0) -> int:
    """Rows per chunk when ``rows`` are cut into the fewest chunks of <= ``limit`` rows, sized
    evenly (43,008 rows under a 16,384 limit -> 15,360 + 15,360 + 12,288, not 16k+16k+10k).
    Chunks are multiples of 3,072 = 8 of v11's 384-row GEMM tiles (csrc/kernels/gemm_v11.hip):
    with 32 or 224 column tiles (the 70B O / down and gate/up projections) every launch is then a
    whole number of 256-CU tile rounds, no tail round; else of 768 = lcm(256, 384) (no chunk pads
    a v10 or v11 tile), else of 256."""
    if limit <= 0 or rows <= limit:
        return max(rows, 1)
    n = -(-rows // limit)
    step = -(-rows // n)
    for a in (align or CHUNK_ALIGN, 768, 256):
        s = -(-step // a) * a
        if s <= limit:
            return s
    return limit


def _proj(ctx: ExecContext, W: Dict[str, torch.Tensor], h, wr, p, n_q, n_k, bias, out=None, rscale=None):
    """QKV-shaped projection of ``h`` by ``wr`` with RoPE on the first n_q + n_k heads (Qwen3:
    per-head q / k RMSNorm first); ``rscale``: per-row scale of the fused RMSNorm (HIP only)."""
    cfg = ctx.cfg
    kw = {"rscale": rscale} if rscale is not None else {}
    if cfg.qk_norm:
        return ctx.ops.qkv_norm_rope(h, wr, p, ctx.cos, ctx.sin, n_q, n_k, cfg.head_dim, W["qn"], W["kn"],
                                     cfg.rms_norm_eps, bias=bias, out=out, **kw)
    return ctx.ops.qkv_rope(h, wr, p, ctx.cos, ctx.sin, n_q, n_k, cfg.head_dim, bias=bias, out=out, **kw)


def _scored_q(ctx: ExecContext, W: Dict[str, torch.Tensor], x: torch.Tensor, last_idx: torch.Tensor,
              last_pos: torch.Tensor) -> torch.Tensor:
    """Q (+ RoPE) of the scored rows of the pruned last layer: [n_scored, q_size] — their raw rows
    gathered and scaled by their own RMSNorm statistic (fused) or normalised explicitly."""
    cfg, ops = ctx.cfg, ctx.ops
    qs, eps = cfg.q_size, cfg.rms_norm_eps
    w, b = W["wqkv"], W.get("bqkv")
    bq = b[:qs] if b is not None else None
    xq = ops.gather_rows(x, last_idx)
    if ctx.fused_norm:
        return _proj(ctx, W, xq, w[:qs], last_pos, cfg.num_attention_heads, 0, bq, rscale=ctx.row_stat(xq))
    return _proj(ctx, W, ops.rmsnorm(xq, W["ln1"], eps), w[:qs], last_pos, cfg.num_attention_heads, 0, bq)


def _attn_inputs(ctx: ExecContext, W: Dict[str, torch.Tensor], x: torch.Tensor, pos: torch.Tensor,
                 last_idx: Optional[torch.Tensor], prune: bool, last_pos: Optional[torch.Tensor] = None,
                 q_scored: Optional[torch.Tensor] = None, ss_key: Optional[tuple] = None) -> torch.Tensor:
    """RMSNorm + QKV projection (+ RoPE, + bias) of every row into one [T, qkv] buffer.
    ``prune`` (the last decoder layer): K/V (+ RoPE on K) for every row, Q only for the scored rows,
    scattered into the Q columns of those rows — the other rows' Q columns stay unwritten, the last
    layer's attention work items (``work_last``) query only scored rows (Q is q_size / qkv_size of
    the projection: 80% for Llama-2-70B).  ``q_scored``: that Q, already projected (the grouped
    attention phase projects every group's scored rows in one GEMM, as the whole-batch path does).
    ``ss_key``: the previous layer's residual GEMM whose partial sums give the row statistic.

    Fused (``ctx.fused_norm``, HIP): one GEMM over the raw hidden state with ln1 folded into W_qkv
    and each row scaled by its rsqrt(mean(x^2) + eps) in the epilogue — the workspace holds only
    [QKV | row statistics], so every row goes through one launch.  Otherwise an explicit RMSNorm
    per row chunk of ``ctx.qkv_chunk`` (the workspace holds [normed chunk | QKV])."""
    cfg, ops = ctx.cfg, ctx.ops
    H, Qn, qs = cfg.hidden_size, cfg.qkv_size, cfg.q_size
    nq, nkv = cfg.num_attention_heads, cfg.num_key_value_heads
    eps = cfg.rms_norm_eps
    T0 = x.shape[0]
    w, b = W["wqkv"], W.get("bqkv")

    def proj(h, wr, p, n_q, n_k, bias, out=None, rscale=None):
        return _proj(ctx, W, h, wr, p, n_q, n_k, bias, out=out, rscale=rscale)

    def put(r, dst):
        if r.data_ptr() != dst.data_ptr():
            dst.copy_(r)

    def scored_q():
        q = q_scored if q_scored is not None else _scored_q(ctx, W, x, last_idx, last_pos)
        ops.scatter_rows(q, last_idx, qkv[:, :qs])

    if ctx.fused_norm:
        ctx.phase((T0, Qn), (1, 2 * T0))
        qkv = ctx.scratch(T0, Qn)
        if qkv is None:
            qkv = torch.empty(T0, Qn, dtype=x.dtype, device=x.device)
        rstd = ctx.rstd(x, ss_key, out=ctx.scratch_f32(T0))
        if not prune:
            put(proj(x, w, pos, nq, nkv, b, out=qkv, rscale=rstd), qkv)
            return qkv
        put(proj(x, w[qs:], pos, 0, nkv, b[qs:] if b is not None else None, out=qkv[:, qs:], rscale=rstd),
            qkv[:, qs:])
        scored_q()
        return qkv

    step = balanced_step(T0, ctx.qkv_chunk) if ctx.qkv_chunk else T0
    ctx.phase((step, H), (T0, Qn))
    hbuf = ctx.scratch(step, H)
    qkv = ctx.scratch(T0, Qn)
    if qkv is None:
        qkv = torch.empty(T0, Qn, dtype=x.dtype, device=x.device)
    for s in range(0, T0, step):
        e = min(T0, s + step)
        h = ops.rmsnorm(x[s:e], W["ln1"], eps, out=hbuf[:e - s] if hbuf is not None else None)
        if prune:
            put(proj(h, w[qs:], pos[s:e], 0, nkv, b[qs:] if b is not None else None, out=qkv[s:e, qs:]),
                qkv[s:e, qs:])
        else:
            put(proj(h, w, pos[s:e], nq, nkv, b, out=qkv[s:e]), qkv[s:e])
        del h
    if prune:
        scored_q()
    return qkv


def _attention_whole(ctx: ExecContext, W: Dict[str, torch.Tensor], x: torch.Tensor, batch, meta: dict,
                     prune: bool, layer_name: str) -> torch.Tensor:
    """Attention phase over the whole micro-batch: QKV of every row, one attention launch, O
    projection + residual (in place on x; the pruned last layer returns its scored rows)."""
    cfg, ops = ctx.cfg, ctx.ops
    li = _decoder_index(layer_name)
    qkv = _attn_inputs(ctx, W, x, meta["positions"], meta["last_idx"], prune, meta["last_pos"],
                       ss_key=(id(batch), li - 1, "mlp", x.shape[0]))
    kv0 = None
    pe = ctx.prefix_entry
    if pe is not None:
        qs, kv = cfg.q_size, 2 * cfg.num_key_value_heads * cfg.head_dim
        if batch.kv_cached:                  # prefix K/V of every prompt from the cache
            kv0 = pe.buffer(layer_name)
        elif "pfx_src" in meta:              # full pass: keep the prefix rows' post-RoPE K/V
            ops.copy_rows(qkv[:, qs:qs + kv], meta["pfx_src"], pe.buffer(layer_name, create=True), meta["pfx_dst"])
        if "sfx_src" in meta:                # the suffix rows computed now (suffix K/V reuse)
            if kv0 is None:
                kv0 = pe.buffer(layer_name, create=True)
            ops.copy_rows(qkv[:, qs:qs + kv], meta["sfx_src"], kv0, meta["sfx_dst"])
            if pe.host:                      # host-mode entry: the new rows into its host buffer too
                pe.write_rows(ops, qkv[:, qs:qs + kv], meta["sfx_src"], meta["sfx_dst"], layer_name)
    work_items = getattr(ops, "uses_work_items", False)
    if prune:
        attn_arg = meta["work_last"] if work_items else batch.last_segments
    else:
        attn_arg = meta["work"] if work_items else batch.segments
    # work items span several suffixes of a prompt: seg_lo makes their range 1 block-diagonal
    kw = {"seg_lo": meta["seg_lo"]} if work_items else {}
    if work_items and "work2" in meta:       # suffix K/V reuse: range 2 = the suffixes' kept rows
        kw["work2"] = meta["work2_last"] if prune else meta["work2"]
        kw["r2win"] = meta["r2win"]
    qb = batch.r2_q_block if "work2" in kw else batch.q_block     # (work_last items: one row each)
    a = ops.attention(qkv, attn_arg, cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim,
                      kv0=kv0 if batch.kv_cached else None, q_block=qb, out=qkv[:, :cfg.q_size],
                      scale=cfg.attn_scale, **kw)
    if pe is not None and pe.host:
        pe.flush(layer_name)                 # host-mode entry: the rows written go back to the host
    del qkv
    if prune:
        idx = meta["last_idx"]
        a = ops.gather_rows(a, idx)
        x = ops.gather_rows(x, idx)
    ss = ctx.ss_take(x.shape[0])
    y = _resid(ctx, a, W["wo"], x, bias=W.get("bo"), ss=ss)
    ctx.ss_key = (id(batch), li, "attn", x.shape[0]) if ss is not None else None
    return y


def _attention_grouped(ctx: ExecContext, W: Dict[str, torch.Tensor], x: torch.Tensor, batch,
                       prune: bool) -> torch.Tensor:
    """Attention phase in prompt-aligned row groups (``--max_vram_gb``): per group RMSNorm, QKV
    (+ RoPE), attention with group-relative work items (every key a query sees is in its own
    prompt), O projection + residual into x's rows — the workspace holds one group's
    [normed | QKV] instead of the whole micro-batch's.  Same kernels per row as the whole-batch
    path, so the scores are bitwise the same: the pruned last layer projects Q of every scored
    row before the groups and O of every scored row after them, one GEMM each as in the
    whole-batch path (a GEMM of a few hundred rows takes a skinny / split-K path chosen by its row
    count; per-group launches changed the scores' last bits, scripts/bits_probe.py)."""
    cfg, ops = ctx.cfg, ctx.ops
    nq, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    work_items = getattr(ops, "uses_work_items", False)
    meta = batch.device_tensors(x.device)
    pos = meta["positions"]
    if prune:
        q_all = _scored_q(ctx, W, x, meta["last_idx"], meta["last_pos"])
        a_all = torch.empty_like(q_all)
    for g in batch.group_tensors(x.device, ctx.attn_rows):
        r0, r1 = g["r0"], g["r1"]
        s0, s1 = g["s0"], g["s1"]
        qkv = _attn_inputs(ctx, W, x[r0:r1], pos[r0:r1], g["last_local"], prune, g["last_pos"],
                           q_scored=q_all[s0:s1] if prune else None)
        if prune:
            arg = g["work_last"] if work_items else g["last_segments"]
        else:
            arg = g["work"] if work_items else g["segments"]
        kw = {"seg_lo": g["seg_lo"]} if work_items else {}
        a = ops.attention(qkv, arg, nq, nkv, hd, q_block=batch.q_block, out=qkv[:, :cfg.q_size],
                          scale=cfg.attn_scale, **kw)
        if prune:
            if s1 > s0:
                a_all[s0:s1].copy_(ops.gather_rows(a, g["last_local"]))
        else:
            xr = x[r0:r1]
            y = _resid(ctx, a, W["wo"], xr, bias=W.get("bo"))
            if y.data_ptr() != xr.data_ptr():
                xr.copy_(y)
        del a, qkv
    if prune:
        return _resid(ctx, a_all, W["wo"], ops.gather_rows(x, meta["last_idx"]), bias=W.get("bo"))
    return x


def run_decoder(ctx: ExecContext, W: Dict[str, torch.Tensor], x: torch.Tensor, batch,
                meta: dict, layer_name: str = "") -> torch.Tensor:
    """One pre-norm decoder block on the packed rows.  With ``prune`` (the last decoder
    layer) Q/attention/O/MLP run only for the scored rows and the result is
    [n_scored, H]: K/V are still projected for every token (the scored rows attend to
    the whole prefix and their own suffix).

    Activation memory per micro-batch of T rows: the hidden state x (updated in place by the
    residual epilogues) plus one workspace arena holding [normed chunk | QKV] in the attention
    phase — the attention output overwrites the Q columns it was computed from (each (row,
    head) is read and written by one work item) and feeds the O projection as a strided view
    — and [normed chunk | SwiGLU chunk] in the MLP phase."""
    cfg, ops = ctx.cfg, ctx.ops
    # (every row scored, in row order — a generation step's new tokens: pruning selects them all,
    # so the plain path runs instead, its single QKV GEMM and the item-per-prompt attention)
    prune = ctx.prune_last and layer_name == ctx.last_decoder and not getattr(batch, "all_rows_scored", False)
    eps = cfg.rms_norm_eps
    if ctx.attn_rows and x.shape[0] > ctx.attn_rows and ctx.prefix_entry is None:
        x = _attention_grouped(ctx, W, x, batch, prune)
        ctx.ss_key = None                      # (per-group residual GEMMs: no partials)
    else:
        x = _attention_whole(ctx, W, x, batch, meta, prune, layer_name)
    done = getattr(W, "attention_done", None)
    if done is not None:
        done()             # sub-layer weight streaming: the attention piece's HBM can be refilled
    T = x.shape[0]
    I, H = cfg.intermediate_size, cfg.hidden_size
    step = balanced_step(T, max(1, ctx.mlp_chunk))
    if cfg.is_moe:
        ctx.ss_key = None
        return _moe_mlp(ctx, W, x, step)
    if ctx.fused_norm:
        # ln2 folded into W_gate/up: the SwiGLU GEMM reads the raw rows, scaled by their statistic
        # in the epilogue (from the O projection's partial sums when it left them); the arena holds
        # [SwiGLU chunk | row statistics].  Each chunk's down projection overwrites only its own rows'
        # partials, which its gate/up has already read.
        li = _decoder_index(layer_name)
        key = (id(batch), li, "attn", T)
        ss_all = ctx.ss_take(T, key)          # (the O projection's buffer when the key matches)
        for s in range(0, T, step):
            xs = x[s:s + step]
            n = xs.shape[0]
            ctx.phase((n, I), (1, 2 * n))
            m = ctx.scratch(n, I)
            rstd = ctx.rstd(xs, key, out=ctx.scratch_f32(n), rows=slice(s, s + n))
            m = ops.swiglu_up(xs, W["wgu"], out=m, rscale=rstd)
            y = _resid(ctx, m, W["wdown"], xs, ss=ss_all[s:s + n] if ss_all is not None else None)
            if y.data_ptr() != xs.data_ptr():
                xs.copy_(y)
        ctx.ss_key = (id(batch), li, "mlp", T) if ss_all is not None else None
        return x
    if T <= step:
        ctx.phase((T, H), (T, I))               # the attention-phase bytes are dead: reuse them
        h = ops.rmsnorm(x, W["ln2"], eps, out=ctx.scratch(T, H))
        m = ops.swiglu_up(h, W["wgu"], out=ctx.scratch(T, I))
        del h
        x = _resid(ctx, m, W["wdown"], x)
    else:
        for s in range(0, T, step):
            xs = x[s:s + step]
            n = xs.shape[0]
            ctx.phase((n, H), (n, I))
            h = ops.rmsnorm(xs, W["ln2"], eps, out=ctx.scratch(n, H))
            m = ops.swiglu_up(h, W["wgu"], out=ctx.scratch(n, I))
            del h
            x[s:s + step] = _resid(ctx, m, W["wdown"], xs)
    return x


def _moe_mlp(ctx: ExecContext, W: Dict[str, torch.Tensor], x: torch.Tensor, step: int) -> torch.Tensor:
    """Sparse-MoE MLP phase in token chunks of ``step`` rows, in place on x: per chunk the
    workspace holds [normed chunk | expert SwiGLU rows (k per token) | expert outputs]."""
    cfg, ops = ctx.cfg, ctx.ops
    H, Ie, k = cfg.hidden_size, cfg.expert_intermediate, cfg.num_experts_per_tok
    for s in range(0, x.shape[0], step):
        xs = x[s:s + step]
        n = xs.shape[0]
        ctx.phase((n, H), (n * k, Ie), (n * k, H))
        h = ops.rmsnorm(xs, W["ln2"], cfg.rms_norm_eps, out=ctx.scratch(n, H))
        shared = _shared_expert(ctx, W, h) if cfg.shared_expert_intermediate_size else None
        ops.moe_ffn(h, xs, W["wrouter"], W["wgu"], W["wdown"], k, cfg.norm_topk_prob,
                    round_w16=cfg.model_type in ("qwen3_moe", "qwen2_moe"), m_out=ctx.scratch(n * k, Ie),
                    y_out=ctx.scratch(n * k, H), shared=shared)
        del shared
        del h
    return x


def _shared_expert(ctx: ExecContext, W: Dict[str, torch.Tensor], h: torch.Tensor) -> torch.Tensor:
    """Qwen2-MoE's shared expert on the normed rows h, in HF's fp16 roundings
    (Qwen2MoeSparseMoeBlock): sigmoid(h . w_gate) * down(silu(gate(h)) * up(h))."""
    ops = ctx.ops
    s = ops.linear(ops.swiglu_up(h, W["wsgu"]), W["wsdown"])
    g = torch.sigmoid(ops.linear(h, W["wsg"]))
    return s * g


def run_norm(ctx: ExecContext, W: Dict[str, torch.Tensor], x: torch.Tensor, meta: dict) -> torch.Tensor:
    if ctx.prune_last and ctx.last_decoder:
        return ctx.ops.rmsnorm(x, W["norm"], ctx.cfg.rms_norm_eps)    # rows already gathered
    return ctx.ops.gather_rmsnorm(x, meta["last_idx"], W["norm"], ctx.cfg.rms_norm_eps)


def run_head(ctx: ExecContext, W: Dict[str, torch.Tensor], h: torch.Tensor) -> torch.Tensor:
    return ctx.ops.lm_head_softmax(h, W["head"], logits_scaling=ctx.cfg.logits_scaling)


def run_layer(ctx: ExecContext, layer_name: str, W: Dict[str, torch.Tensor],
              state: Optional[torch.Tensor], batch, meta: dict) -> torch.Tensor:
    kind = layer_kind(layer_name)
    if kind == "embed":
        return run_embed(ctx, W, meta)
    if kind == "decoder":
        return run_decoder(ctx, W, state, batch, meta, layer_name)
    if kind == "norm":
        return run_norm(ctx, W, state, meta)
    return run_head(ctx, W, state)


def layer_flops(cfg: ModelConfig, batch, pruned: bool = False) -> float:
    """Approximate forward FLOPs of one decoder layer on ``batch`` (GEMMs + attention);
    ``pruned``: the last decoder layer (K/V for every token, the rest for scored rows)."""
    T = batch.num_tokens
    if pruned:
        S = batch.n_scored
        kv = 2 * cfg.kv_size * cfg.hidden_size
        gemm = 2.0 * (T * kv + S * (cfg.decoder_active_params() - kv))
        segs = batch.last_segments
    else:
        gemm = 2.0 * T * cfg.decoder_active_params()
        segs = batch.segments
    att = 0.0
    for sg in segs:
        keys = sg.r0_len if not sg.r0_causal else (sg.q_len + 1) / 2.0
        keys += sg.q_off + (sg.q_len + 1) / 2.0 if sg.r1_len else 0.0
        att += 4.0 * sg.q_len * keys * cfg.q_size
    return gemm + att
