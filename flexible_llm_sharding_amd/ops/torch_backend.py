"""Plain-PyTorch implementation of every op (CPU path + numerics oracle).

Semantics follow the HF Llama block the reference drives
(``/root/reference/utils.py:266-290``): RMSNorm with fp32
statistics, RoPE rotate-half with fp16-rounded cos/sin tables, softmax in
fp32, SwiGLU MLP.  Weights are the packed images of :mod:`..models.layout`
(checkpoint row order: ``wqkv = [q; k; v]``, ``wgu = [gate; up]``), exactly
what the HIP kernels consume, so this backend is a drop-in oracle for them.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


class TorchOps:
    name = "torch"
    fused_norm = False          # explicit RMSNorm (the oracle keeps HF's cast points)

    def __init__(self, compute_dtype: torch.dtype = torch.float32):
        self.cdt = compute_dtype

    # ---------------------------------------------------------------- helpers
    def _c(self, t: torch.Tensor) -> torch.Tensor:
        return t if t.dtype == self.cdt else t.to(self.cdt)

    # ------------------------------------------------------------------- ops
    def embed(self, ids: torch.Tensor, table: torch.Tensor, out_dtype, scale: float = 1.0, out=None) -> torch.Tensor:
        e = table.index_select(0, ids.long())
        if scale != 1.0:                       # Granite: GraniteModel scales the embeddings
            e = (self._c(e) * scale).to(table.dtype)
        e = e.to(out_dtype)
        if out is not None:
            out.copy_(e)
            return out
        return e

    def copy_rows(self, x, src_idx, y, dst_idx):
        rows = x.index_select(0, src_idx.long()) if src_idx is not None else x
        if dst_idx is not None:
            y.index_copy_(0, dst_idx.long(), rows.to(y.dtype))
        else:
            y.copy_(rows)
        return y

    def gather_rows(self, x, idx, out=None):
        return x.index_select(0, idx.long()) if out is None else self.copy_rows(x, idx, out, None)

    def scatter_rows(self, x, idx, y):
        return self.copy_rows(x, None, y, idx)

    def rmsnorm(self, x: torch.Tensor, w: torch.Tensor, eps: float, out=None) -> torch.Tensor:
        # LlamaRMSNorm: fp32 variance, normalise, cast back, scale by weight.
        xf = x.float()
        var = xf.pow(2).mean(-1, keepdim=True)
        y = (xf * torch.rsqrt(var + eps)).to(x.dtype)
        return (self._c(w) * self._c(y)).to(x.dtype)

    def linear(self, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        return (self._c(x) @ self._c(w).t()).to(x.dtype)

    def linear_residual(self, x: torch.Tensor, w: torch.Tensor, resid: torch.Tensor,
                        bias: torch.Tensor = None, alpha: float = 1.0) -> torch.Tensor:
        y = self._c(x) @ self._c(w).t()
        if bias is not None:
            y = y + self._c(bias)
        if alpha != 1.0:
            # Granite's residual_multiplier in HF GraniteDecoderLayer's roundings: x + fp16(fp16(y) * r)
            y = (self._c(y.to(resid.dtype)) * alpha).to(resid.dtype)
        return (self._c(resid) + self._c(y)).to(resid.dtype)

    def swiglu_up(self, x: torch.Tensor, wgu: torch.Tensor, out=None) -> torch.Tensor:
        y = self._c(x) @ self._c(wgu).t()                     # [T, 2I] = [gate | up]
        I = y.shape[1] // 2
        return (F.silu(y[:, :I]) * y[:, I:]).to(x.dtype)

    def qkv_rope(self, x: torch.Tensor, wqkv: torch.Tensor, positions: torch.Tensor,
                 cos: torch.Tensor, sin: torch.Tensor, n_q_heads: int, n_kv_heads: int,
                 head_dim: int, bias: torch.Tensor = None, out=None) -> torch.Tensor:
        y = self._c(x) @ self._c(wqkv).t()
        if bias is not None:
            y = y + self._c(bias)
        qk_cols = (n_q_heads + n_kv_heads) * head_dim
        T = y.shape[0]
        half = head_dim // 2
        qk = y[:, :qk_cols].reshape(T, n_q_heads + n_kv_heads, 2, half)   # HF rotate_half halves
        c = cos.index_select(0, positions.long()).to(self.cdt).reshape(T, 1, half)   # [T, 1, hd/2]
        s = sin.index_select(0, positions.long()).to(self.cdt).reshape(T, 1, half)
        x1, x2 = qk[:, :, 0, :], qk[:, :, 1, :]
        o1 = x1 * c - x2 * s
        o2 = x2 * c + x1 * s
        qk_out = torch.stack([o1, o2], dim=2).reshape(T, qk_cols)
        return torch.cat([qk_out, y[:, qk_cols:]], dim=1).to(x.dtype)

    def qkv_norm_rope(self, x: torch.Tensor, wqkv: torch.Tensor, positions: torch.Tensor, cos: torch.Tensor,
                      sin: torch.Tensor, n_q_heads: int, n_kv_heads: int, head_dim: int, qn: torch.Tensor,
                      kn: torch.Tensor, eps: float, bias: torch.Tensor = None, out=None) -> torch.Tensor:
        """Qwen3 projection: RMSNorm over head_dim on the q (q_norm) and k (k_norm) heads, then RoPE."""
        y = self._c(x) @ self._c(wqkv).t()
        if bias is not None:
            y = y + self._c(bias)
        y = y.to(x.dtype)
        T = y.shape[0]
        nqk = n_q_heads + n_kv_heads
        heads = y[:, :nqk * head_dim].reshape(T, nqk, head_dim).float()
        var = heads.pow(2).mean(-1, keepdim=True)
        normed = (heads * torch.rsqrt(var + eps)).to(x.dtype)
        w = torch.cat([qn.reshape(1, -1).expand(n_q_heads, -1), kn.reshape(1, -1).expand(n_kv_heads, -1)])
        normed = (self._c(w)[None] * self._c(normed)).to(x.dtype)
        half = head_dim // 2
        qk = self._c(normed).reshape(T, nqk, 2, half)
        c = cos.index_select(0, positions.long()).to(self.cdt).reshape(T, 1, half)
        s = sin.index_select(0, positions.long()).to(self.cdt).reshape(T, 1, half)
        x1, x2 = qk[:, :, 0, :], qk[:, :, 1, :]
        qk_out = torch.stack([x1 * c - x2 * s, x2 * c + x1 * s], dim=2).reshape(T, nqk * head_dim)
        return torch.cat([qk_out.to(x.dtype), y[:, nqk * head_dim:]], dim=1)

    def moe_ffn(self, h: torch.Tensor, x: torch.Tensor, wrouter: torch.Tensor, wgu: torch.Tensor,
                wdown: torch.Tensor, top_k: int, norm_topk: bool, round_w16: bool = False, m_out=None,
                y_out=None, shared=None) -> torch.Tensor:
        """x += sparse-MoE FFN of h, in place, in the order and rounding of HF's expert loop
        (transformers MixtralExperts / Qwen3MoeExperts): router Linear in the activation dtype,
        fp32 softmax, top-k, optional renormalisation (Qwen3-MoE rounds the weights to the
        activation dtype), each expert's weighted output rounded to the activation dtype and
        accumulated in expert order, plus the gated shared-expert output (Qwen2-MoE) in one more
        rounding, then added to the residual."""
        logits = self.linear(h, wrouter)
        w, idx = torch.topk(torch.softmax(logits.float(), dim=-1), top_k, dim=-1)
        if norm_topk:
            w = w / w.sum(-1, keepdim=True)
        if round_w16:
            w = w.to(h.dtype).float()
        acc = torch.zeros_like(x)
        for e in range(wgu.shape[0]):
            tok, slot = torch.where(idx == e)
            if tok.numel() == 0:
                continue
            y = self.linear(self.swiglu_up(h.index_select(0, tok), wgu[e]), wdown[e])
            acc.index_add_(0, tok, (y.float() * w[tok, slot, None]).to(x.dtype))
        if shared is not None:
            acc = (acc.float() + shared.float()).to(x.dtype)
        x.copy_((x.float() + acc.float()).to(x.dtype))
        return x

    def attention(self, qkv: torch.Tensor, segments, n_q_heads: int, n_kv_heads: int,
                  head_dim: int, kv0: torch.Tensor = None, q_block: int = 64, out=None,
                  scale: float = None) -> torch.Tensor:
        """Shared-prefix attention over packed segments (see runtime.batch).

        ``kv0`` ([P, 2 * n_kv * hd], K then V): range 0 of every segment indexes
        these rows instead of the packed QKV (prefix K/V cache)."""
        T = qkv.shape[0]
        qs = n_q_heads * head_dim
        ks = n_kv_heads * head_dim
        q_all = qkv[:, :qs].view(T, n_q_heads, head_dim)
        k_all = qkv[:, qs:qs + ks].view(T, n_kv_heads, head_dim)
        v_all = qkv[:, qs + ks:qs + 2 * ks].view(T, n_kv_heads, head_dim)
        if kv0 is not None:
            k0_all = kv0[:, :ks].reshape(-1, n_kv_heads, head_dim)
            v0_all = kv0[:, ks:2 * ks].reshape(-1, n_kv_heads, head_dim)
        else:
            k0_all, v0_all = k_all, v_all
        out = torch.empty(T, qs, dtype=qkv.dtype, device=qkv.device)
        rep = n_q_heads // n_kv_heads
        scale = head_dim ** -0.5 if scale is None else scale
        dev = qkv.device
        for sg in segments:
            q = self._c(q_all[sg.q_start:sg.q_start + sg.q_len])                # [q, nh, d]
            kr = [(sg.r0_start, sg.r0_len, sg.r0_causal, k0_all, v0_all)]
            if getattr(sg, "r2_len", 0):        # suffix K/V reuse: the suffix's kept rows, all visible
                kr.append((sg.r2_start, sg.r2_len, 0, k0_all, v0_all))
            if sg.r1_len:
                kr.append((sg.r1_start, sg.r1_len, 1, k_all, v_all))
            ks_, vs_, masks = [], [], []
            qi = torch.arange(sg.q_len, device=dev) + sg.q_off
            for st, ln, causal, kk, vv in kr:
                ks_.append(kk[st:st + ln])
                vs_.append(vv[st:st + ln])
                kj = torch.arange(ln, device=dev)
                m = torch.ones(sg.q_len, ln, dtype=torch.bool, device=dev)
                if causal:
                    m = kj[None, :] <= qi[:, None]
                masks.append(m)
            k = self._c(torch.cat(ks_, 0)).repeat_interleave(rep, dim=1)        # [k, nh, d]
            v = self._c(torch.cat(vs_, 0)).repeat_interleave(rep, dim=1)
            mask = torch.cat(masks, 1)                                          # [q, k]
            s = torch.einsum("qhd,khd->hqk", q.float(), k.float()) * scale
            s = s.masked_fill(~mask[None], float("-inf"))
            p = torch.softmax(s, dim=-1)
            o = torch.einsum("hqk,khd->qhd", p, v.float())
            out[sg.q_start:sg.q_start + sg.q_len] = o.reshape(sg.q_len, qs).to(qkv.dtype)
        return out

    def gather_rmsnorm(self, x: torch.Tensor, idx: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
        return self.rmsnorm(x.index_select(0, idx.long()), w, eps)

    def lm_head_softmax(self, h: torch.Tensor, w: torch.Tensor, logits_scaling: float = 1.0) -> torch.Tensor:
        logits = (self._c(h) @ self._c(w).t()).to(h.dtype)   # fp16 logits like nn.Linear in fp16
        return self.softmax(logits, logits_scaling)

    def row_exact(self, on: bool = True):
        """HipOps.row_exact: nothing to select here (one matmul path)."""
        import contextlib
        return contextlib.nullcontext()

    def argmax_rows(self, probs: torch.Tensor) -> torch.Tensor:
        return probs.float().argmax(-1).to(torch.int32)

    def softmax(self, logits: torch.Tensor, logits_scaling: float = 1.0) -> torch.Tensor:
        if logits_scaling != 1.0:                            # Granite: logits / logits_scaling
            logits = logits / logits_scaling
        return torch.softmax(logits.float(), dim=-1).to(torch.float16)

    def synchronize(self):
        pass

    # ------------------------------------------------------- synthetic init
    def fill_layer_random(self, buf: torch.Tensor, layout, seed: int, std: float = 0.02) -> None:
        """Random-init one packed layer in place (norm weights ~ 1, embeddings ~ N(0,1))."""
        g = torch.Generator(device=buf.device).manual_seed(int(seed))
        views = layout.views(buf, torch.float16)
        for name, v in views.items():
            mean, sd = fill_params(name, std)
            v.copy_(torch.randn(v.shape, generator=g, device=buf.device) * sd + mean)


def fill_params(slot_name: str, std: float):
    """(mean, std) of the synthetic distribution of a packed slot."""
    if slot_name in ("ln1", "ln2", "norm", "qn", "kn"):
        return 1.0, 0.1
    if slot_name == "embed":
        return 0.0, 1.0
    if slot_name in ("bqkv", "bo"):
        return 0.0, 10 * std
    return 0.0, std
