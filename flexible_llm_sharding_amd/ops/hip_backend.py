"""HIP backend: every op is a hand-written gfx950 kernel in ``libfls_kernels.so``.

Kernels run on the caller's current HIP stream (``torch.cuda.current_stream``)
so they compose with the copy/comm streams of the runtime; outputs are
allocated through PyTorch's caching allocator.  There is deliberately no
fallback and no second GEMM backend: a missing library raises (see
``_native.kernels``).

Projection GEMMs are the fused MFMA kernels of ``csrc/kernels/gemm.hip``:
RoPE / SwiGLU / residual / bias epilogues in registers, on the checkpoint's
own weight layout (``wqkv = [q; k; v]``, ``wgu = [gate; up]``).
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass

import torch

from .. import _native, knobs
from .torch_backend import fill_params

EPI_NONE, EPI_RESID, EPI_SWIGLU, EPI_ROPE = 0, 1, 2, 3
ROW_EXACT = 0x100                  # csrc/include/fls.h: the row-exact epi flag
SPLITK_MAX_M = 512                 # csrc/kernels/gemm.hip SPLITK_MAX_M
SPLITK_WS_BYTES = 64 << 20        # fp32 partial slabs: e.g. 8 slices x 160 rows x 10240 columns
CAST_BF16, CAST_F32 = 1, 2


def _stream():
    # the raw current stream of the current device, without torch.cuda.current_stream()'s Python
    # device bookkeeping: every op calls this, ~800 times per 70B generation step
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def _chk(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")


def _f16(t: torch.Tensor, name: str):
    if t.dtype != torch.float16 or not t.is_cuda:
        raise TypeError(f"{name}: expected fp16 CUDA tensor, got {t.dtype} on {t.device}")
    if t.stride(-1) != 1:
        raise ValueError(f"{name}: last dim must be contiguous")


@dataclass
class MoeRoute:
    """Device-side routing of one MoE call (csrc/kernels/moe.hip): per (token, slot) entry the
    expert id and weight; per expert its permuted-row offsets and 256-row tile prefix; permuted
    row -> token (``rows``) and entry -> permuted row (``dest``)."""
    ids: torch.Tensor
    w: torch.Tensor
    offs: torch.Tensor
    tiles: torch.Tensor
    rows: torch.Tensor
    dest: torch.Tensor
    k: int


class HipOps:
    name = "hip"
    uses_work_items = True
    # RMSNorm + projection as one GEMM on the raw hidden state: row statistics (row_rstd), the norm
    # weight folded into the projection weight once per load (fold_norm), the statistic applied in
    # the GEMM epilogue (gemm(rscale=...)); models/llama.py _attn_inputs
    fused_norm = True

    def __init__(self):
        self.k = _native.kernels()
        self._ws = {}
        self._tl = threading.local()
        # A/B switches (knobs.py); the kernels' defaults are the measured winners
        if knobs.get_int("FLS_SPLITK") == 0:
            self.k.fls_gemm_set_splitk(0)

    # ---------------------------------------------------------------- GEMM
    def gemm(self, x: torch.Tensor, w: torch.Tensor, epi: int = EPI_NONE, out: torch.Tensor = None,
             resid: torch.Tensor = None, positions=None, cos=None, sin=None, rope_cols: int = 0,
             head_dim: int = 0, bias: torch.Tensor = None, rscale: torch.Tensor = None,
             alpha: float = 1.0, ss: torch.Tensor = None) -> torch.Tensor:
        """rscale ([M] fp32): per-row scale of the raw product (before bias / epilogue); alpha:
        RESID's C = alpha * (product + bias) + R; ss ([>= M, N / 128] fp32, RESID): each output
        row's partial sums of squares per 128 columns (:meth:`rstd_from_ss`)."""
        _f16(x, "x")
        _f16(w, "w")
        if rscale is not None and (rscale.dtype != torch.float32 or not rscale.is_cuda
                                   or rscale.numel() < x.shape[0] or not rscale.is_contiguous()):
            raise TypeError("rscale must be a contiguous fp32 CUDA vector with one entry per row")
        M, K = x.shape
        N, K2 = w.shape
        if K != K2:
            raise ValueError(f"gemm K mismatch {x.shape} x {w.shape}")
        ncols = N // 2 if epi == EPI_SWIGLU else N
        code = epi | (ROW_EXACT if getattr(self._tl, "row_exact", False) else 0)
        if out is None:
            out = torch.empty(M, ncols, dtype=torch.float16, device=x.device)
        R = resid if resid is not None else out
        ws = self._splitk_ws(x.device, M, N) if M <= SPLITK_MAX_M else None
        if bias is not None:
            _f16(bias, "bias")
            if bias.numel() != N or not bias.is_contiguous():
                raise ValueError(f"bias must be a contiguous [{N}] vector")
        if ss is not None and (ss.dtype != torch.float32 or not ss.is_cuda or ss.dim() != 2 or ss.shape[0] < M
                               or ss.shape[1] < N // 128 or ss.stride(1) != 1):
            raise TypeError(f"ss must be an fp32 CUDA [>= {M}, >= {N // 128}] matrix with unit column stride")
        rc = self.k.fls_gemm(x.data_ptr(), w.data_ptr(), out.data_ptr(), R.data_ptr(), M, N, K,
                             x.stride(0), w.stride(0), out.stride(0), R.stride(0), code,
                             positions.data_ptr() if positions is not None else None,
                             cos.data_ptr() if cos is not None else None,
                             sin.data_ptr() if sin is not None else None,
                             rope_cols, head_dim, bias.data_ptr() if bias is not None else None,
                             rscale.data_ptr() if rscale is not None else None, float(alpha),
                             ss.data_ptr() if ss is not None else None, ss.stride(0) if ss is not None else 0,
                             ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0, _stream())
        _chk(rc, "fls_gemm")
        return out

    @staticmethod
    def new_workspace(device) -> torch.Tensor:
        """A split-K / split-KV scratch buffer (``SPLITK_WS_BYTES``).  Each ShardedRunner owns one,
        allocated before it plans its memory (so a ``--max_vram_gb`` plan charges it) and installed
        for its calls with :meth:`use_workspace`: which GEMM path a shape takes, and its rounding,
        then never depends on what the allocator could give or on which thread ran before."""
        return torch.empty(SPLITK_WS_BYTES, dtype=torch.uint8, device=device)

    def use_workspace(self, ws):
        """Context manager: GEMMs / attention issued by this host thread use ``ws`` (a buffer of
        ``SPLITK_WS_BYTES``, or a callable returning one at each use) as their fp32 partial scratch.  A runner's kernels run on one stream in order, so its GEMMs and attention
        share it; runners driven from different threads (ranks as threads on one GPU) each install
        their own, since their multi-kernel sequences (partials, then reduce) can interleave."""
        ops = self

        class _Use:
            def __enter__(self):
                self.prev = getattr(ops._tl, "ws", None)
                ops._tl.ws = ws

            def __exit__(self, *exc):
                ops._tl.ws = self.prev
        return _Use()

    def _splitk_ws(self, device, M: int, N: int):
        """The scratch of the calling thread's runner (:meth:`use_workspace`: a buffer, or a callable
        returning one); outside a runner (kernel tests, tools) one buffer per (device, thread),
        reserved at first use."""
        ws = getattr(self._tl, "ws", None)
        if callable(ws):
            ws = ws()
        if ws is not None:
            return ws
        key = (torch.device(device), threading.get_ident())
        if key not in self._ws:
            self._ws[key] = self.new_workspace(key[0])
        return self._ws[key]

    def gemv_skinny(self, x, w):
        """Weight-streaming GEMV for M <= 16 rows (skinny LM head)."""
        _f16(x, "x")
        _f16(w, "w")
        M, K = x.shape
        N = w.shape[0]
        out = torch.empty(M, N, dtype=torch.float16, device=x.device)
        _chk(self.k.fls_gemv_skinny(x.data_ptr(), w.data_ptr(), out.data_ptr(), M, N, K, x.stride(0), w.stride(0),
                                    out.stride(0), _stream()), "fls_gemv_skinny")
        return out

    def linear(self, x, w):
        if x.shape[0] <= 16 and x.shape[1] % 32 == 0 and not getattr(self._tl, "row_exact", False):
            return self.gemv_skinny(x, w)
        return self.gemm(x, w)

    def row_exact(self, on: bool = True):
        """Context manager: GEMMs issued by this host thread take only row-independent paths
        (fls.h GEMM_ROW_EXACT; no GEMV / skinny / split-K), so each row's result is the same
        whatever other rows share the launch (engine.ShardedRunner: exact K/V reuse)."""
        ops = self

        class _Exact:
            def __enter__(self):
                self.prev = getattr(ops._tl, "row_exact", False)
                ops._tl.row_exact = bool(on)

            def __exit__(self, *exc):
                ops._tl.row_exact = self.prev
        return _Exact()

    def linear_residual(self, x, w, resid, bias=None, alpha: float = 1.0, ss=None):
        """resid += alpha * (x @ w^T (+ bias)), in place (alpha: Granite's residual_multiplier);
        ``ss``: also each updated row's partial sums of squares (the next fused norm's statistic)."""
        _f16(resid, "resid")
        return self.gemm(x, w, EPI_RESID, out=resid, resid=resid, bias=bias, alpha=alpha, ss=ss)

    def rstd_from_ss(self, ss, H: int, eps, out=None):
        """[rows] fp32 rsqrt(sum of the row's ss partials / H + eps): the RMSNorm statistic of the rows
        a residual GEMM just wrote (:meth:`linear_residual` ``ss``), without reading them again."""
        rows = ss.shape[0]
        r = out if out is not None else torch.empty(rows, dtype=torch.float32, device=ss.device)
        _chk(self.k.fls_rstd_from_ss(ss.data_ptr(), ss.stride(0), -(-H // 128), rows, int(H), float(eps), r.data_ptr(),
                                     _stream()), "fls_rstd_from_ss")
        return r

    def swiglu_up(self, x, wgu, out=None, rscale=None):
        """silu(x @ gate^T) * (x @ up^T) with wgu = [gate; up]."""
        return self.gemm(x, wgu, EPI_SWIGLU, out=out, rscale=rscale)

    def row_ss(self, x, out=None):
        """[rows, H/128] fp32 partial sums of squares of x's rows (H % 128 == 0), bitwise the ones a
        residual GEMM epilogue writes for the same fp16 values (:meth:`linear_residual` ``ss``)."""
        _f16(x, "x")
        rows, H = x.shape
        ss = out if out is not None else torch.empty(rows, H // 128, dtype=torch.float32, device=x.device)
        _chk(self.k.fls_row_ss(x.data_ptr(), x.stride(0), rows, H, ss.data_ptr(), ss.stride(0), _stream()),
             "fls_row_ss")
        return ss

    def row_stat(self, x, eps, out=None):
        """[rows] fp32 rsqrt(mean(x[row]^2) + eps) computed as :meth:`row_ss` + :meth:`rstd_from_ss`
        would (bitwise), in one launch (H % 128 == 0; rows 16-byte aligned, else those two launches)."""
        _f16(x, "x")
        rows, H = x.shape
        if x.stride(0) % 8 or x.data_ptr() % 16:
            return self.rstd_from_ss(self.row_ss(x), H, eps, out=out)
        r = out if out is not None else torch.empty(rows, dtype=torch.float32, device=x.device)
        _chk(self.k.fls_row_stat(x.data_ptr(), x.stride(0), rows, H, float(eps), r.data_ptr(), _stream()),
             "fls_row_stat")
        return r

    def row_rstd(self, x, eps, row_idx=None, out=None):
        """[rows] fp32 rsqrt(mean(x[row]^2) + eps) (rows = row_idx or every row of x)."""
        _f16(x, "x")
        rows = row_idx.shape[0] if row_idx is not None else x.shape[0]
        r = out if out is not None else torch.empty(rows, dtype=torch.float32, device=x.device)
        if row_idx is not None and (row_idx.dtype != torch.int32 or not row_idx.is_cuda):
            raise TypeError("row_idx must be int32 CUDA")
        _chk(self.k.fls_row_rstd(x.data_ptr(), x.stride(0), row_idx.data_ptr() if row_idx is not None else None,
                                 rows, x.shape[1], float(eps), r.data_ptr(), _stream()), "fls_row_rstd")
        return r

    def fold_norm(self, w, gamma):
        """w[n, k] *= gamma[k] in place (fp16): the RMSNorm weight folded into its projection."""
        _f16(w, "w")
        _f16(gamma, "gamma")
        if gamma.numel() != w.shape[-1] or not gamma.is_contiguous():
            raise ValueError(f"gamma must be a contiguous [{w.shape[-1]}] vector")
        _chk(self.k.fls_fold_norm(w.data_ptr(), w.stride(0), w.shape[0], w.shape[1], gamma.data_ptr(), _stream()),
             "fls_fold_norm")

    def copy_rows(self, x, src_idx, y, dst_idx):
        """y[dst_idx[r]] = x[src_idx[r]] (int32 CUDA indices; None = identity; rows of x.shape[1])."""
        _f16(x, "x")
        _f16(y, "y")
        idx = src_idx if src_idx is not None else dst_idx
        for t in (src_idx, dst_idx):
            if t is not None and (t.dtype != torch.int32 or not t.is_cuda):
                raise TypeError("row indices must be int32 CUDA")
        if x.shape[1] != y.shape[1]:
            raise ValueError(f"row width mismatch {tuple(x.shape)} -> {tuple(y.shape)}")
        rows = idx.shape[0] if idx is not None else x.shape[0]
        _chk(self.k.fls_copy_rows(x.data_ptr(), x.stride(0), src_idx.data_ptr() if src_idx is not None else None,
                                  y.data_ptr(), y.stride(0), dst_idx.data_ptr() if dst_idx is not None else None,
                                  rows, x.shape[1], _stream()), "fls_copy_rows")
        return y

    def copy_rows_to(self, x, src_idx, y_ptr: int, y_ld: int, dst_idx):
        """copy_rows into raw device-addressable memory (``y_ptr``: e.g. the device address of a
        mapped pinned host buffer, row stride ``y_ld`` fp16 elements, rows of x.shape[1])."""
        _f16(x, "x")
        for t in (src_idx, dst_idx):
            if t is None or t.dtype != torch.int32 or not t.is_cuda:
                raise TypeError("row indices must be int32 CUDA")
        if y_ld < x.shape[1]:
            raise ValueError("destination rows narrower than the source rows")
        _chk(self.k.fls_copy_rows(x.data_ptr(), x.stride(0), src_idx.data_ptr(), y_ptr, y_ld, dst_idx.data_ptr(),
                                  src_idx.shape[0], x.shape[1], _stream()), "fls_copy_rows")

    def gather_rows(self, x, idx, out=None):
        """x[idx] into a new (or ``out``) [len(idx), H] tensor."""
        y = out if out is not None else torch.empty(idx.shape[0], x.shape[1], dtype=x.dtype, device=x.device)
        return self.copy_rows(x, idx, y, None)

    def scatter_rows(self, x, idx, y):
        """y[idx] = x in place (distinct indices)."""
        return self.copy_rows(x, None, y, idx)

    def qkv_rope(self, x, wqkv, positions, cos, sin, n_q_heads, n_kv_heads, head_dim, bias=None, out=None,
                 rscale=None):
        if positions.dtype != torch.int32:
            raise TypeError("positions must be int32")
        rope_cols = (n_q_heads + n_kv_heads) * head_dim
        if head_dim not in (64, 128):
            # the fused epilogue finds a column's rotate-half partner 2 or 4 subtiles away inside
            # the GEMM tile; other head sizes (Phi-3-mini: 96) rotate in a second pass
            y = self.gemm(x, wqkv, EPI_NONE, out=out, bias=bias, rscale=rscale)
            rc = self.k.fls_headnorm_rope(y.data_ptr(), y.stride(0), y.shape[0], n_q_heads, n_kv_heads, None, None,
                                          positions.data_ptr(), cos.data_ptr(), sin.data_ptr(), head_dim, 0.0,
                                          _stream())
            _chk(rc, "fls_headnorm_rope")
            return y
        return self.gemm(x, wqkv, EPI_ROPE, out=out, positions=positions, cos=cos, sin=sin,
                         rope_cols=rope_cols, head_dim=head_dim, bias=bias, rscale=rscale)

    def qkv_norm_rope(self, x, wqkv, positions, cos, sin, n_q_heads, n_kv_heads, head_dim, qn, kn, eps,
                      bias=None, out=None, rscale=None):
        """Qwen3: projection (+ bias), then RMSNorm over head_dim on every q / k head (q_norm /
        k_norm weights) and RoPE, in place (``headnorm_rope_kernel``); V columns untouched."""
        if positions.dtype != torch.int32:
            raise TypeError("positions must be int32")
        y = self.gemm(x, wqkv, EPI_NONE, out=out, bias=bias, rscale=rscale)
        _f16(qn, "q_norm")
        _f16(kn, "k_norm")
        rc = self.k.fls_headnorm_rope(y.data_ptr(), y.stride(0), y.shape[0], n_q_heads, n_kv_heads, qn.data_ptr(),
                                      kn.data_ptr(), positions.data_ptr(), cos.data_ptr(), sin.data_ptr(), head_dim,
                                      float(eps), _stream())
        _chk(rc, "fls_headnorm_rope")
        return y

    # ------------------------------------------------------ mixture of experts
    def moe_ffn(self, h, x, wrouter, wgu, wdown, top_k: int, norm_topk: bool, round_w16: bool = False,
                m_out=None, y_out=None, shared=None):
        """x += sparse-MoE FFN of h, in place (csrc/kernels/moe.hip): router GEMM, top-k routing,
        stable expert sort, grouped SwiGLU GEMM gathering h's rows, grouped down GEMM, ordered
        combine.  wgu [E, 2I, H] ([gate; up] per expert), wdown [E, H, I].  No host sync: the
        grouped GEMMs read the per-expert row counts on the device.  m_out [T*k, I] / y_out
        [T*k, H]: optional scratch for the expert intermediates.  shared ([T, H] fp16): the gated
        shared-expert output (Qwen2-MoE), added to the experts' sum before the residual."""
        route = self.moe_route(h, wrouter, top_k, norm_topk, round_w16)
        return self.moe_experts(h, x, wgu, wdown, route, m_out=m_out, y_out=y_out, shared=shared)

    def moe_route(self, h, wrouter, top_k: int, norm_topk: bool, round_w16: bool = False) -> "MoeRoute":
        _f16(h, "h")
        _f16(wrouter, "router")
        T, H = h.shape
        E = wrouter.shape[0]
        k = int(top_k)
        if E > 64:                                # logits by the mid-M GEMM (N = E), then routing
            return self.moe_route_logits(self.gemm(h, wrouter), k, norm_topk, round_w16)
        # few experts: router logits fused into the routing kernel (an N = E GEMM would be padding)
        ids = torch.empty(T * k, dtype=torch.int32, device=h.device)
        w = torch.empty(T * k, dtype=torch.float32, device=h.device)
        _chk(self.k.fls_moe_router_route(h.data_ptr(), h.stride(0), wrouter.data_ptr(), wrouter.stride(0), T, H, E,
                                         k, int(bool(norm_topk)), int(bool(round_w16)), ids.data_ptr(),
                                         w.data_ptr(), _stream()), "fls_moe_router_route")
        return self._moe_plan(ids, w, E, k)

    def moe_route_logits(self, logits, top_k: int, norm_topk: bool, round_w16: bool = False) -> "MoeRoute":
        """Routing from fp16 router logits [T, E]: top-k ids / weights per token and the stable
        expert sort (offsets, 256-row tile prefix, permuted row -> token, entry -> permuted row)."""
        _f16(logits, "logits")
        T, E = logits.shape
        k, n, dev = int(top_k), T * int(top_k), logits.device
        ids = torch.empty(n, dtype=torch.int32, device=dev)
        w = torch.empty(n, dtype=torch.float32, device=dev)
        st = _stream()
        _chk(self.k.fls_moe_route(logits.data_ptr(), logits.stride(0), T, E, k, int(bool(norm_topk)),
                                  int(bool(round_w16)), ids.data_ptr(), w.data_ptr(), st), "fls_moe_route")
        return self._moe_plan(ids, w, E, k)

    def _moe_plan(self, ids, w, E: int, k: int) -> "MoeRoute":
        n, dev = ids.numel(), ids.device
        scratch = self.k.fls_moe_plan_scratch(n, E)
        meta = torch.empty(2 * (E + 1) + 2 * n + scratch, dtype=torch.int32, device=dev)
        o = 2 * (E + 1)
        r = MoeRoute(ids, w, meta[:E + 1], meta[E + 1:o], meta[o:o + n], meta[o + n:o + 2 * n], k)
        _chk(self.k.fls_moe_plan(ids.data_ptr(), n, k, E, r.offs.data_ptr(), r.tiles.data_ptr(), r.rows.data_ptr(),
                                 r.dest.data_ptr(), meta[o + 2 * n:].data_ptr(), _stream()), "fls_moe_plan")
        return r

    def moe_experts(self, h, x, wgu, wdown, route: "MoeRoute", m_out=None, y_out=None, shared=None):
        """x += sum over each token's routed experts of w * down(swiglu(h)), in place."""
        for t, nm in ((h, "h"), (x, "x"), (wgu, "wgu"), (wdown, "wdown")):
            _f16(t, nm)
        T, H = h.shape
        E, I2, _ = wgu.shape
        I, k = I2 // 2, route.k
        n = T * k
        dev, st = h.device, _stream()
        m = m_out if m_out is not None else torch.empty(n, I, dtype=torch.float16, device=dev)
        y = y_out if y_out is not None else torch.empty(n, H, dtype=torch.float16, device=dev)
        bound = n + 255 * E                       # >= sum over experts of their rows rounded up to 256
        rc = self.k.fls_moe_gemm(h.data_ptr(), wgu.data_ptr(), m.data_ptr(), bound, I2, H, h.stride(0),
                                 wgu.stride(1), m.stride(0), EPI_SWIGLU, route.tiles.data_ptr(),
                                 route.offs.data_ptr(), route.rows.data_ptr(), E, wgu.stride(0), T, st)
        if rc == -5:                              # shape outside the grouped kernel: per-expert GEMMs
            self._moe_per_expert(h, wgu, wdown, route, m, y)
        else:
            _chk(rc, "fls_moe_gemm(gate/up)")
            _chk(self.k.fls_moe_gemm(m.data_ptr(), wdown.data_ptr(), y.data_ptr(), bound, H, I, m.stride(0),
                                     wdown.stride(1), y.stride(0), EPI_NONE, route.tiles.data_ptr(),
                                     route.offs.data_ptr(), None, E, wdown.stride(0), n, st), "fls_moe_gemm(down)")
        if shared is not None:
            _f16(shared, "shared")
            if tuple(shared.shape) != (T, H) or shared.stride(1) != 1:
                raise ValueError(f"shared must be a row-major [{T}, {H}] tensor, got {tuple(shared.shape)}")
        _chk(self.k.fls_moe_combine(y.data_ptr(), y.stride(0), route.ids.data_ptr(), route.dest.data_ptr(),
                                    route.w.data_ptr(), x.data_ptr(), x.stride(0), T, k, H,
                                    shared.data_ptr() if shared is not None else None,
                                    shared.stride(0) if shared is not None else 0, st), "fls_moe_combine")
        return x

    def _moe_per_expert(self, h, wgu, wdown, route, m, y):
        """Fallback for shapes outside the grouped kernel's contract: one host read of the
        per-expert row counts, then the dense fused GEMMs expert by expert."""
        o = route.offs.cpu().tolist()
        for e in range(wgu.shape[0]):
            a, b = o[e], o[e + 1]
            if a == b:
                continue
            self.gemm(h.index_select(0, route.rows[a:b]), wgu[e], EPI_SWIGLU, out=m[a:b])
            self.gemm(m[a:b], wdown[e], out=y[a:b])

    # ----------------------------------------------------------- attention
    def attention(self, qkv, work, n_q_heads, n_kv_heads, head_dim, kv0=None, q_block: int = 64, out=None,
                  seg_lo=None, work2=None, r2win=None, scale=None):
        """kv0 ([P, 2 * n_kv * hd], K then V): range 0 of every work item reads these rows (prefix cache).
        seg_lo ([T] int32, first row of each row's suffix): work items may span several suffixes.
        work2 ([n_items, 2] int32: r2_start, r2_len) + r2win ([T, 2] int32: kv0 rows [lo, hi) per row):
        range 2 = the kv0 rows of the item's suffixes cached by an earlier call (suffix K/V reuse),
        walked between the prefix and the new rows, each row seeing its own suffix's window."""
        _f16(qkv, "qkv")
        if work.dtype != torch.int32 or not work.is_cuda:
            raise TypeError("work items must be an int32 CUDA tensor")
        if kv0 is not None:
            _f16(kv0, "kv0")
            if kv0.shape[1] != 2 * n_kv_heads * head_dim:
                raise ValueError(f"kv0 must be [P, {2 * n_kv_heads * head_dim}], got {tuple(kv0.shape)}")
        T = qkv.shape[0]
        # work items from runtime/batch.py span suffix boundaries: without seg_lo a query would see the
        # other suffixes of its item, so it is required here (the C ABI's null form is one-suffix items)
        if seg_lo is None or seg_lo.dtype != torch.int32 or not seg_lo.is_cuda or seg_lo.shape[0] < T:
            raise TypeError("seg_lo (PackedBatch.seg_lo: int32 CUDA, one row per packed token) is required")
        if work2 is not None and (kv0 is None or work2.dtype != torch.int32 or not work2.is_cuda
                                  or tuple(work2.shape) != (work.shape[0], 2) or r2win is None
                                  or r2win.dtype != torch.int32 or r2win.shape[0] < T):
            raise TypeError("work2 must be int32 CUDA [n_items, 2] with r2win [T, 2] and kv0")
        if out is None:
            out = torch.empty(T, n_q_heads * head_dim, dtype=torch.float16, device=qkv.device)
        # the range-2 (decode-like) kernel splits its key tiles over blocks when the grid is small;
        # its fp32 partials live in the split-K GEMM scratch (same stream: never in use by both)
        # (row-exact calls: no split, whose merge would round differently from the unsplit kernel)
        ws = self._splitk_ws(qkv.device, 0, 0) if work2 is not None and not getattr(self._tl, "row_exact", False) \
            else None
        rc = self.k.fls_attention(qkv.data_ptr(), out.data_ptr(), work.data_ptr(), work.shape[0],
                                  n_q_heads, n_kv_heads, head_dim, qkv.stride(0), out.stride(0),
                                  head_dim ** -0.5 if scale is None else float(scale),
                                  kv0.data_ptr() if kv0 is not None else None,
                                  kv0.stride(0) if kv0 is not None else 0,
                                  seg_lo.data_ptr() if seg_lo is not None else None, q_block,
                                  work2.data_ptr() if work2 is not None else None,
                                  r2win.data_ptr() if work2 is not None else None,
                                  ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0,
                                  T, _stream())
        _chk(rc, "fls_attention")
        return out

    # ------------------------------------------------------- elementwise
    def rmsnorm(self, x, w, eps, row_idx=None, out=None):
        _f16(x, "x")
        _f16(w, "w")
        rows = row_idx.shape[0] if row_idx is not None else x.shape[0]
        H = x.shape[1]
        y = out if out is not None else torch.empty(rows, H, dtype=torch.float16, device=x.device)
        rc = self.k.fls_rmsnorm(x.data_ptr(), w.data_ptr(), y.data_ptr(),
                                row_idx.data_ptr() if row_idx is not None else None,
                                rows, H, x.stride(0), y.stride(0), float(eps), _stream())
        _chk(rc, "fls_rmsnorm")
        return y

    def gather_rmsnorm(self, x, idx, w, eps):
        if idx.dtype != torch.int32:
            raise TypeError("row indices must be int32")
        return self.rmsnorm(x, w, eps, row_idx=idx)

    def embed(self, ids, table, out_dtype, scale: float = 1.0, out=None):
        """table[ids] (scale != 1: fp16(e * scale), Granite's embedding_multiplier)."""
        _f16(table, "table")
        if out_dtype != torch.float16:
            raise TypeError("HIP path runs fp16 activations")
        T = ids.shape[0]
        V, H = table.shape
        if out is None:
            out = torch.empty(T, H, dtype=torch.float16, device=table.device)
        elif tuple(out.shape) != (T, H) or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous [{T}, {H}] tensor")
        _chk(self.k.fls_embed(ids.data_ptr(), table.data_ptr(), out.data_ptr(), T, H, V, float(scale), _stream()),
             "fls_embed")
        return out

    def softmax(self, logits, logits_scaling: float = 1.0):
        """Row softmax of fp16 logits (logits_scaling != 1: of fp16(logits / logits_scaling))."""
        _f16(logits, "logits")
        rows, V = logits.shape
        probs = torch.empty_like(logits)
        _chk(self.k.fls_softmax_rows(logits.data_ptr(), probs.data_ptr(), rows, V, 1.0 / float(logits_scaling),
                                     _stream()), "fls_softmax")
        return probs

    def argmax_rows(self, probs):
        """[rows] int32: the first index of each row's maximum (non-negative fp16 probabilities)."""
        _f16(probs, "probs")
        out = torch.empty(probs.shape[0], dtype=torch.int32, device=probs.device)
        _chk(self.k.fls_argmax_rows(probs.data_ptr(), probs.stride(0), probs.shape[0], probs.shape[1],
                                    out.data_ptr(), _stream()), "fls_argmax_rows")
        return out

    def lm_head_softmax(self, h, w, logits_scaling: float = 1.0):
        return self.softmax(self.linear(h, w), logits_scaling)

    def cast_f16(self, dst: torch.Tensor, src: torch.Tensor, src_code: int) -> None:
        """dst (fp16 bytes) = fp16(src bytes of bf16 (code 1; may be in place) or fp32 (code 2))."""
        n = dst.numel() * dst.element_size() // 2
        _chk(self.k.fls_cast_f16(dst.data_ptr(), src.data_ptr(), src_code, n, _stream()), "fls_cast_f16")

    def fill_layer_random(self, buf: torch.Tensor, layout, seed: int, std: float = 0.02) -> None:
        views = layout.views(buf, torch.float16)
        for i, (name, v) in enumerate(views.items()):
            mean, sd = fill_params(name, std)
            _chk(self.k.fls_fill_random(v.data_ptr(), v.numel(), int(seed) * 131 + i, float(mean),
                                        float(sd), _stream()), "fls_fill_random")

    def synchronize(self):
        torch.cuda.synchronize()
