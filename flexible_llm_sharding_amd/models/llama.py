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


def rope_tables(cfg: ModelConfig, max_pos: int = MAX_TOKEN_LEN, table_dtype=torch.float16,
                device="cpu"):
    """cos/sin [max_pos, hd/2] in fp32 holding ``table_dtype``-rounded values.

    HF (4.31-4.35) builds ``cos_cached``/``sin_cached`` in fp32 and the reference
    casts every buffer to fp16 (``utils.py:118-119``); rotate-half uses
    ``emb = cat(freqs, freqs)`` so only hd/2 distinct frequencies exist.
    """
    hd = cfg.head_dim
    inv_freq = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd, 2, dtype=torch.int64).float() / hd))
    t = torch.arange(max(max_pos, 1), dtype=torch.float32)
    freqs = torch.outer(t, inv_freq)
    cos, sin = freqs.cos(), freqs.sin()
    if table_dtype is not None and table_dtype != torch.float32:
        cos, sin = cos.to(table_dtype).float(), sin.to(table_dtype).float()
    return cos.contiguous().to(device), sin.contiguous().to(device)


@dataclass
class ExecContext:
    cfg: ModelConfig
    ops: object
    device: torch.device
    act_dtype: torch.dtype
    cos: torch.Tensor
    sin: torch.Tensor
    mlp_chunk: int = 16384       # rows per gate/up + down chunk (bounds the [T, I] buffer)
    prefix_entry: Optional[object] = None   # runtime.prefix_cache.PrefixEntry of the current call


def run_embed(ctx: ExecContext, W: Dict[str, torch.Tensor], meta: dict) -> torch.Tensor:
    return ctx.ops.embed(meta["ids"], W["embed"], ctx.act_dtype)


def run_decoder(ctx: ExecContext, W: Dict[str, torch.Tensor], x: torch.Tensor, batch,
                meta: dict, layer_name: str = "") -> torch.Tensor:
    cfg, ops = ctx.cfg, ctx.ops
    eps = cfg.rms_norm_eps
    h = ops.rmsnorm(x, W["ln1"], eps)
    qkv = ops.qkv_rope(h, W["wqkv"], meta["positions"], ctx.cos, ctx.sin,
                       cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim, bias=W.get("bqkv"))
    del h
    kv0 = None
    pe = ctx.prefix_entry
    if pe is not None:
        qs, kv = cfg.q_size, 2 * cfg.num_key_value_heads * cfg.head_dim
        if batch.kv_cached:                  # prefix K/V of every prompt from the cache
            kv0 = pe.buffer(layer_name)
        elif "pfx_src" in meta:              # full pass: keep the prefix rows' post-RoPE K/V
            pe.buffer(layer_name, create=True).index_copy_(
                0, meta["pfx_dst"], qkv[:, qs:qs + kv].index_select(0, meta["pfx_src"]))
    attn_arg = meta["work"] if getattr(ops, "uses_work_items", False) else batch.segments
    a = ops.attention(qkv, attn_arg, cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim, kv0=kv0)
    del qkv
    x = ops.linear_residual(a, W["wo"], x, bias=W.get("bo"))
    del a
    T = x.shape[0]
    step = max(1, ctx.mlp_chunk)
    if T <= step:
        h = ops.rmsnorm(x, W["ln2"], eps)
        m = ops.swiglu_up(h, W["wgu"])
        del h
        x = ops.linear_residual(m, W["wdown"], x)
    else:
        for s in range(0, T, step):
            xs = x[s:s + step]
            h = ops.rmsnorm(xs, W["ln2"], eps)
            m = ops.swiglu_up(h, W["wgu"])
            del h
            x[s:s + step] = ops.linear_residual(m, W["wdown"], xs)
    return x


def run_norm(ctx: ExecContext, W: Dict[str, torch.Tensor], x: torch.Tensor, meta: dict) -> torch.Tensor:
    return ctx.ops.gather_rmsnorm(x, meta["last_idx"], W["norm"], ctx.cfg.rms_norm_eps)


def run_head(ctx: ExecContext, W: Dict[str, torch.Tensor], h: torch.Tensor) -> torch.Tensor:
    return ctx.ops.lm_head_softmax(h, W["head"])


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


def layer_flops(cfg: ModelConfig, batch) -> float:
    """Approximate forward FLOPs of one decoder layer on ``batch`` (GEMMs + attention)."""
    T = batch.num_tokens
    gemm = 2.0 * T * cfg.decoder_layer_params()
    att = 0.0
    for sg in batch.segments:
        keys = sg.r0_len if not sg.r0_causal else (sg.q_len + 1) / 2.0
        keys += (sg.r1_len + 1) / 2.0 if sg.r1_len else 0.0
        att += 4.0 * sg.q_len * keys * cfg.q_size
    return gemm + att
