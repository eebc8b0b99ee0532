"""Packed per-layer weight layout — the HBM-native format the kernels consume.

The reference keeps HF modules and installs each parameter separately with
``set_module_tensor_to_device`` (``/root/reference/utils.py:128-130``).  We
instead pack each layer into ONE contiguous buffer so that a shard moves
host->HBM as a single large ``hipMemcpyAsync`` and every kernel gets raw
pointers at fixed offsets.

Decoder layer packing (fp16, every tensor 256-byte aligned)::

    ln1   [H]              input_layernorm.weight
    ln2   [H]              post_attention_layernorm.weight
    wqkv  [Hq+2Hkv, H]     q|k|v projections, q and k rows RoPE-pair permuted
    wo    [H, Hq]          o_proj
    wgu   [2I, H]          gate/up interleaved in blocks of 16 rows
    wdown [H, I]           down_proj
    bqkv  [Hq+2Hkv]        q|k|v biases, permuted like wqkv rows (Qwen2 / attention_bias only)
    bo    [H]              o_proj bias (Llama attention_bias only)

*RoPE pair permutation* — HF Llama rotates (d, d + hd/2) pairs
(``rotate_half``).  Per head we reorder rows as ``[0:16], [hd/2:hd/2+16],
[16:32], [hd/2+16:hd/2+32], ...`` so the MFMA GEMM epilogue finds each
rotation partner in the neighbouring 16-column subtile of the same lane and
can apply RoPE in registers.  Q and K stay in this permuted head-dim order all
the way into attention (QK^T is invariant to a common permutation of d).

*Gate/up interleave* — rows ``[g0:16], [u0:16], [g16:32], [u16:32] ...`` so
the SwiGLU epilogue reads gate and up of the same intermediate column from two
accumulator subtiles held by the same lane.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch

from ..config import ModelConfig

ALIGN_BYTES = 256
PAIR_BLOCK = 16


def _align(n_bytes: int) -> int:
    return (n_bytes + ALIGN_BYTES - 1) // ALIGN_BYTES * ALIGN_BYTES


@dataclass(frozen=True)
class TensorSlot:
    name: str
    shape: Tuple[int, ...]
    offset: int  # bytes from layer base

    @property
    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n


@dataclass(frozen=True)
class LayerLayout:
    kind: str                       # embed | decoder | norm | head
    slots: Tuple[TensorSlot, ...]
    nbytes: int                     # total (aligned)
    elem_size: int = 2

    def slot(self, name: str) -> TensorSlot:
        for s in self.slots:
            if s.name == name:
                return s
        raise KeyError(name)

    def views(self, buf: torch.Tensor, dtype: torch.dtype) -> Dict[str, torch.Tensor]:
        """Typed views into a flat uint8 (or any) buffer holding one packed layer."""
        b = buf.view(torch.uint8) if buf.dtype != torch.uint8 else buf
        es = torch.empty((), dtype=dtype).element_size()
        out = {}
        for s in self.slots:
            n = s.numel * es
            out[s.name] = b[s.offset:s.offset + n].view(dtype).view(s.shape)
        return out


def layer_kind(name: str) -> str:
    if name == "model.embed_tokens":
        return "embed"
    if name.startswith("model.layers."):
        return "decoder"
    if name == "model.norm":
        return "norm"
    if name == "lm_head":
        return "head"
    raise ValueError(f"unknown layer {name}")


def layer_layout(cfg: ModelConfig, kind: str, elem_size: int = 2) -> LayerLayout:
    H, V, I = cfg.hidden_size, cfg.vocab_size, cfg.intermediate_size
    if kind == "embed":
        specs = [("embed", (V, H))]
    elif kind == "head":
        specs = [("head", (V, H))]
    elif kind == "norm":
        specs = [("norm", (H,))]
    elif kind == "decoder":
        specs = [("ln1", (H,)), ("ln2", (H,)), ("wqkv", (cfg.qkv_size, H)),
                 ("wo", (H, cfg.q_size)), ("wgu", (2 * I, H)), ("wdown", (H, I))]
        if cfg.attention_bias:
            specs.append(("bqkv", (cfg.qkv_size,)))
        if cfg.o_proj_bias:
            specs.append(("bo", (H,)))
    else:
        raise ValueError(kind)
    slots, off = [], 0
    for name, shape in specs:
        n = 1
        for s in shape:
            n *= s
        slots.append(TensorSlot(name, tuple(shape), off))
        off += _align(n * elem_size)
    return LayerLayout(kind, tuple(slots), off, elem_size)


# ----------------------------------------------------------------- permutations
def rope_row_perm(head_dim: int) -> List[int]:
    """Row order inside one head: packed row i takes HF row perm[i]."""
    half = head_dim // 2
    assert half % PAIR_BLOCK == 0, "head_dim/2 must be a multiple of 16"
    perm = []
    for j in range(half // PAIR_BLOCK):
        perm += list(range(PAIR_BLOCK * j, PAIR_BLOCK * (j + 1)))
        perm += list(range(half + PAIR_BLOCK * j, half + PAIR_BLOCK * (j + 1)))
    return perm


def permute_heads_rows(w: torch.Tensor, n_heads: int, head_dim: int) -> torch.Tensor:
    perm = torch.tensor(rope_row_perm(head_dim), dtype=torch.long)
    w3 = w.reshape(n_heads, head_dim, -1)
    return w3[:, perm, :].reshape(w.shape)


def unpermute_heads_rows(w: torch.Tensor, n_heads: int, head_dim: int) -> torch.Tensor:
    perm = torch.tensor(rope_row_perm(head_dim), dtype=torch.long)
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())
    w3 = w.reshape(n_heads, head_dim, -1)
    return w3[:, inv, :].reshape(w.shape)


def permute_head_cols(x: torch.Tensor, n_heads: int, head_dim: int) -> torch.Tensor:
    """Apply the rope head-dim permutation to activations [..., n_heads*head_dim]."""
    perm = torch.tensor(rope_row_perm(head_dim), dtype=torch.long, device=x.device)
    shp = x.shape
    return x.reshape(*shp[:-1], n_heads, head_dim)[..., perm].reshape(shp)


def unpermute_head_cols(x: torch.Tensor, n_heads: int, head_dim: int) -> torch.Tensor:
    perm = torch.tensor(rope_row_perm(head_dim), dtype=torch.long)
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())
    inv = inv.to(x.device)
    shp = x.shape
    return x.reshape(*shp[:-1], n_heads, head_dim)[..., inv].reshape(shp)


def interleave_gate_up(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    I, H = gate.shape
    assert I % PAIR_BLOCK == 0, "intermediate_size must be a multiple of 16"
    g = gate.reshape(I // PAIR_BLOCK, PAIR_BLOCK, H)
    u = up.reshape(I // PAIR_BLOCK, PAIR_BLOCK, H)
    return torch.stack([g, u], dim=1).reshape(2 * I, H)


def deinterleave_gate_up(wgu: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    I2, H = wgu.shape
    w = wgu.reshape(I2 // (2 * PAIR_BLOCK), 2, PAIR_BLOCK, H)
    return w[:, 0].reshape(I2 // 2, H), w[:, 1].reshape(I2 // 2, H)


# ------------------------------------------------------------------- packing
def hf_param_names(cfg: ModelConfig, layer_name: str) -> List[str]:
    kind = layer_kind(layer_name)
    if kind == "embed":
        return ["model.embed_tokens.weight"]
    if kind == "norm":
        return ["model.norm.weight"]
    if kind == "head":
        return ["lm_head.weight"]
    p = layer_name
    names = [f"{p}.self_attn.q_proj.weight", f"{p}.self_attn.k_proj.weight",
             f"{p}.self_attn.v_proj.weight", f"{p}.self_attn.o_proj.weight",
             f"{p}.mlp.gate_proj.weight", f"{p}.mlp.up_proj.weight",
             f"{p}.mlp.down_proj.weight", f"{p}.input_layernorm.weight",
             f"{p}.post_attention_layernorm.weight"]
    if cfg.attention_bias:
        names += [f"{p}.self_attn.{n}_proj.bias" for n in ("q", "k", "v")]
    if cfg.o_proj_bias:
        names.append(f"{p}.self_attn.o_proj.bias")
    return names


def pack_layer(cfg: ModelConfig, layer_name: str, sd: Dict[str, torch.Tensor],
               dtype: torch.dtype = torch.float16, out: torch.Tensor = None) -> torch.Tensor:
    """HF-named state dict of one layer -> flat packed uint8 buffer (CPU).

    ``sd`` keys are full HF names (the per-layer file format of
    ``prepare_weights.py:40-43``).  ``int8`` is rejected like the reference
    (``utils.py:129``).  Other float dtypes are cast to ``dtype`` (``utils.py:130``).
    """
    kind = layer_kind(layer_name)
    es = torch.empty((), dtype=dtype).element_size()
    lay = layer_layout(cfg, kind, es)
    for k, v in sd.items():
        if v.dtype == torch.int8:
            raise AssertionError("int8 not supported (need to add fp16_statistics)")
    if out is None:
        out = torch.zeros(lay.nbytes, dtype=torch.uint8)
    views = lay.views(out, dtype)

    def get(name):
        if name not in sd:
            raise KeyError(f"{layer_name}: missing tensor {name}")
        return sd[name].to(dtype)

    if kind == "embed":
        views["embed"].copy_(get("model.embed_tokens.weight"))
    elif kind == "norm":
        views["norm"].copy_(get("model.norm.weight"))
    elif kind == "head":
        key = "lm_head.weight"
        if key not in sd and cfg.tie_word_embeddings and "model.embed_tokens.weight" in sd:
            key = "model.embed_tokens.weight"
        views["head"].copy_(sd[key].to(dtype))
    else:
        p = layer_name
        hd = cfg.head_dim
        q = permute_heads_rows(get(f"{p}.self_attn.q_proj.weight"), cfg.num_attention_heads, hd)
        k = permute_heads_rows(get(f"{p}.self_attn.k_proj.weight"), cfg.num_key_value_heads, hd)
        v = get(f"{p}.self_attn.v_proj.weight")
        views["wqkv"].copy_(torch.cat([q, k, v], 0))
        views["wo"].copy_(get(f"{p}.self_attn.o_proj.weight"))
        views["wgu"].copy_(interleave_gate_up(get(f"{p}.mlp.gate_proj.weight"),
                                              get(f"{p}.mlp.up_proj.weight")))
        views["wdown"].copy_(get(f"{p}.mlp.down_proj.weight"))
        views["ln1"].copy_(get(f"{p}.input_layernorm.weight"))
        views["ln2"].copy_(get(f"{p}.post_attention_layernorm.weight"))
        if cfg.attention_bias:
            bq = permute_heads_rows(get(f"{p}.self_attn.q_proj.bias")[:, None], cfg.num_attention_heads, hd)
            bk = permute_heads_rows(get(f"{p}.self_attn.k_proj.bias")[:, None], cfg.num_key_value_heads, hd)
            views["bqkv"].copy_(torch.cat([bq[:, 0], bk[:, 0], get(f"{p}.self_attn.v_proj.bias")], 0))
        if cfg.o_proj_bias:
            views["bo"].copy_(get(f"{p}.self_attn.o_proj.bias"))
    return out


def unpack_layer(cfg: ModelConfig, layer_name: str, buf: torch.Tensor,
                 dtype: torch.dtype = torch.float16) -> Dict[str, torch.Tensor]:
    """Inverse of :func:`pack_layer` (HF names, HF row order)."""
    kind = layer_kind(layer_name)
    es = torch.empty((), dtype=dtype).element_size()
    v = layer_layout(cfg, kind, es).views(buf, dtype)
    if kind == "embed":
        return {"model.embed_tokens.weight": v["embed"].clone()}
    if kind == "norm":
        return {"model.norm.weight": v["norm"].clone()}
    if kind == "head":
        return {"lm_head.weight": v["head"].clone()}
    p = layer_name
    hd = cfg.head_dim
    qs, ks = cfg.q_size, cfg.kv_size
    wqkv = v["wqkv"]
    g, u = deinterleave_gate_up(v["wgu"])
    out = {}
    if cfg.attention_bias:
        b = v["bqkv"][:, None]
        out[f"{p}.self_attn.q_proj.bias"] = unpermute_heads_rows(b[:qs], cfg.num_attention_heads, hd)[:, 0].clone()
        out[f"{p}.self_attn.k_proj.bias"] = unpermute_heads_rows(b[qs:qs + ks], cfg.num_key_value_heads,
                                                                  hd)[:, 0].clone()
        out[f"{p}.self_attn.v_proj.bias"] = v["bqkv"][qs + ks:].clone()
    if cfg.o_proj_bias:
        out[f"{p}.self_attn.o_proj.bias"] = v["bo"].clone()
    return {
        **out,
        f"{p}.self_attn.q_proj.weight": unpermute_heads_rows(wqkv[:qs], cfg.num_attention_heads, hd).clone(),
        f"{p}.self_attn.k_proj.weight": unpermute_heads_rows(wqkv[qs:qs + ks], cfg.num_key_value_heads, hd).clone(),
        f"{p}.self_attn.v_proj.weight": wqkv[qs + ks:].clone(),
        f"{p}.self_attn.o_proj.weight": v["wo"].clone(),
        f"{p}.mlp.gate_proj.weight": g.clone(),
        f"{p}.mlp.up_proj.weight": u.clone(),
        f"{p}.mlp.down_proj.weight": v["wdown"].clone(),
        f"{p}.input_layernorm.weight": v["ln1"].clone(),
        f"{p}.post_attention_layernorm.weight": v["ln2"].clone(),
    }


def max_layer_bytes(cfg: ModelConfig, elem_size: int = 2) -> int:
    return max(layer_layout(cfg, k, elem_size).nbytes for k in ("embed", "decoder", "norm", "head"))
