"""Independent fp32 oracle of the reference's forward semantics.

Operates per prompt on HF-layout weights (no packing, no permutations), with
the reference's padded suffix batch, its ``suffix_eos`` gather and its
prefix-KV expansion — written directly from ``/root/reference/utils.py:246-290``
so the packed engine and the HIP kernels can be checked against it.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from ..config import ModelConfig


def _rms(x, w, eps):
    v = x.pow(2).mean(-1, keepdim=True)
    return w * (x * torch.rsqrt(v + eps))


def _rotate_half(x):
    h = x.shape[-1] // 2
    return torch.cat([-x[..., h:], x[..., :h]], -1)


def _rope(x, pos, cos, sin):
    # x [B, nh, T, d]; cos/sin [maxpos, d/2]
    c = torch.cat([cos, cos], -1)[pos][:, None]      # [B,1,T,d]
    s = torch.cat([sin, sin], -1)[pos][:, None]
    return x * c + _rotate_half(x) * s


def _block(x, sd, p, cfg, pos, cos, sin, mask, past_kv=None):
    """HF LlamaDecoderLayer (eager) in fp32. x [B,T,H]; mask [B,1,T,K] additive or None."""
    B, T, H = x.shape
    nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    g = lambda n: sd[f"{p}.{n}"].float()
    b = lambda n: sd[f"{p}.{n}"].float() if f"{p}.{n}" in sd else 0.0    # Qwen2 / attention_bias
    h = _rms(x, g("input_layernorm.weight"), cfg.rms_norm_eps)
    q = (h @ g("self_attn.q_proj.weight").t() + b("self_attn.q_proj.bias")).view(B, T, nh, hd).transpose(1, 2)
    k = (h @ g("self_attn.k_proj.weight").t() + b("self_attn.k_proj.bias")).view(B, T, nkv, hd).transpose(1, 2)
    v = (h @ g("self_attn.v_proj.weight").t() + b("self_attn.v_proj.bias")).view(B, T, nkv, hd).transpose(1, 2)
    if cfg.qk_norm:                   # HF Qwen3Attention: RMSNorm over head_dim before RoPE
        q = _rms(q, g("self_attn.q_norm.weight"), cfg.rms_norm_eps)
        k = _rms(k, g("self_attn.k_norm.weight"), cfg.rms_norm_eps)
    q, k = _rope(q, pos, cos, sin), _rope(k, pos, cos, sin)
    if past_kv is not None:
        k = torch.cat([past_kv[0], k], 2)
        v = torch.cat([past_kv[1], v], 2)
    present = (k, v)
    rep = nh // nkv
    kk = k.repeat_interleave(rep, 1)
    vv = v.repeat_interleave(rep, 1)
    s = q @ kk.transpose(2, 3) * cfg.attn_scale
    if mask is not None:
        s = s + mask
    a = torch.softmax(s, -1) @ vv
    a = a.transpose(1, 2).reshape(B, T, nh * hd)
    r = cfg.residual_multiplier                       # Granite; 1 elsewhere
    x = x + (a @ g("self_attn.o_proj.weight").t() + b("self_attn.o_proj.bias")) * r
    h = _rms(x, g("post_attention_layernorm.weight"), cfg.rms_norm_eps)
    if cfg.is_moe:
        return x + _moe(h, sd, p, cfg) * r, present
    m = F.silu(h @ g("mlp.gate_proj.weight").t()) * (h @ g("mlp.up_proj.weight").t())
    x = x + (m @ g("mlp.down_proj.weight").t()) * r
    return x, present


def _moe(h, sd, p, cfg):
    """HF MixtralSparseMoeBlock / Qwen3MoeSparseMoeBlock / Qwen2MoeSparseMoeBlock in fp32: router
    softmax, top-k, optional renormalisation, weighted sum of the chosen experts' SwiGLU outputs
    (+ the sigmoid-gated shared expert)."""
    from .layout import expert_names, router_name
    shape = h.shape
    h = h.reshape(-1, shape[-1])
    probs = torch.softmax(h @ sd[router_name(cfg, p)].float().t(), -1)
    w, idx = torch.topk(probs, cfg.num_experts_per_tok, dim=-1)
    if cfg.norm_topk_prob:
        w = w / w.sum(-1, keepdim=True)
    out = torch.zeros_like(h)
    for e in range(cfg.num_local_experts):
        tok, slot = torch.where(idx == e)
        if tok.numel() == 0:
            continue
        gn, un, dn = expert_names(cfg, p, e)
        he = h[tok]
        y = (F.silu(he @ sd[gn].float().t()) * (he @ sd[un].float().t())) @ sd[dn].float().t()
        out.index_add_(0, tok, y * w[tok, slot, None])
    if cfg.shared_expert_intermediate_size:   # HF Qwen2MoeSparseMoeBlock: gated shared expert
        b = f"{p}.mlp.shared_expert"
        s = (F.silu(h @ sd[f"{b}.gate_proj.weight"].float().t()) * (h @ sd[f"{b}.up_proj.weight"].float().t())) \
            @ sd[f"{b}.down_proj.weight"].float().t()
        out = out + torch.sigmoid(h @ sd[f"{p}.mlp.shared_expert_gate.weight"].float().t()) * s
    return out.reshape(shape)


def reference_scores(cfg: ModelConfig, sd: Dict[str, torch.Tensor], tok, prompts: Sequence,
                     prefix_attention: str = "bidirectional", max_len: int = 4096,
                     cos=None, sin=None) -> List[np.ndarray]:
    """list of [n_s, 1, V] float32 probabilities, one per prompt."""
    from .llama import rope_tables
    from ..utils.synthetic import split_projections
    sd = split_projections(cfg, sd)          # Phi-3 fused qkv_proj / gate_up_proj -> split names
    if cos is None:
        cos, sin = rope_tables(cfg, max_len)
    outs = []
    neg = torch.finfo(torch.float32).min
    for prefix, suffixes in prompts:
        pids = torch.tensor(tok(prefix, truncation=True, max_length=max_len)["input_ids"])[None]
        sids = torch.tensor(tok(list(suffixes), truncation=True, max_length=max_len,
                                padding=True)["input_ids"])[:, 1:]
        eos = (sids != tok.pad_token_id).sum(1) - 1
        Lp, Ls, ns = pids.shape[1], sids.shape[1], sids.shape[0]
        P = sd["model.embed_tokens.weight"].float()[pids] * cfg.embedding_multiplier
        S = sd["model.embed_tokens.weight"].float()[sids] * cfg.embedding_multiplier
        ppos = torch.arange(Lp)[None]
        spos = torch.arange(Lp, Lp + Ls)[None].expand(ns, -1)
        pmask = None
        if prefix_attention == "causal":
            pmask = torch.full((Lp, Lp), neg).triu(1)[None, None]
        full = torch.full((Lp + Ls, Lp + Ls), neg).triu(1)
        smask = full[-Ls:, -(Lp + Ls):][None, None].expand(ns, 1, Ls, Lp + Ls)   # utils.py:276
        for i in range(cfg.num_hidden_layers):
            p = f"model.layers.{i}"
            P, (kc, vc) = _block(P, sd, p, cfg, ppos, cos, sin, pmask)
            kv = (kc.expand(ns, -1, -1, -1), vc.expand(ns, -1, -1, -1))
            S, _ = _block(S, sd, p, cfg, spos, cos, sin, smask, past_kv=kv)
        last = S[torch.arange(ns), eos][:, None]                             # utils.py:286
        h = _rms(last, sd["model.norm.weight"].float(), cfg.rms_norm_eps)
        head = sd.get("lm_head.weight", sd["model.embed_tokens.weight"]).float()
        logits = (h @ head.t())[:, 0] / cfg.logits_scaling
        outs.append(torch.softmax(logits, -1)[:, None].numpy())
    return outs
