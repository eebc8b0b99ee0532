"""Packed per-layer weight layout — the HBM image the kernels consume.

The reference keeps HF modules and installs each parameter separately with
``set_module_tensor_to_device`` (``/root/reference/utils.py:128-130``).  Here
each layer is ONE contiguous buffer (a weight slot), so a shard moves to HBM
as large DMAs and every kernel gets raw pointers at fixed offsets.

Decoder layer image (fp16, every slot 256-byte aligned)::

    ln1   [H]              input_layernorm.weight
    wqkv  [Hq+2Hkv, H]     q_proj | k_proj | v_proj   (rows concatenated)
    bqkv  [Hq+2Hkv]        q|k|v biases (Qwen2 / attention_bias only)
    qn    [hd]             q_norm.weight (Qwen3 only)
    kn    [hd]             k_norm.weight (Qwen3 only)
    wo    [H, Hq]          o_proj
    bo    [H]              o_proj bias (Llama attention_bias only)
    ln2   [H]              post_attention_layernorm.weight
    wgu   [2I, H]          gate_proj | up_proj        (rows concatenated)
    wdown [H, I]           down_proj

MoE decoder (Mixtral / Qwen3-MoE / Qwen2-MoE) — the MLP piece is the router and every expert, each
expert's tensors whole and in checkpoint row order::

    ln2     [H]            post_attention_layernorm.weight
    wrouter [E, H]         router (Mixtral block_sparse_moe.gate / Qwen3-MoE mlp.gate)
    wgu     [E, 2I', H]    per expert: gate (w1 / gate_proj) | up (w3 / up_proj)
    wdown   [E, H, I']     per expert: down (w2 / down_proj)
    wsgu    [2Is, H]       Qwen2-MoE shared expert: gate_proj | up_proj
    wsdown  [H, Is]        shared expert down_proj
    wsg     [1, H]         shared_expert_gate

so expert e's [gate; up] block is the same stacked operand as the dense wgu, at a fixed stride:
the grouped GEMM (csrc/kernels/moe.hip) indexes experts by that stride.

Everything the attention phase reads comes before ``ln2`` and nothing after it: the image
splits into an attention piece and an MLP piece (:func:`mlp_offset`) that the
``--max_vram_gb`` prefetcher streams into separate HBM pools and frees separately
(runtime/prefetch.py ``PiecePoolPrefetcher``).

Every checkpoint tensor keeps its own row order and byte image: a slot is a
plain concatenation of whole tensors.  The two places where the fused kernels
need partners side by side are handled inside the GEMM, not by permuting
weights: the RoPE epilogue finds the rotate-half partner ``d + hd/2`` of a
head's column ``d`` in the same lane (``csrc/kernels/gemm.hip``), and the
SwiGLU GEMM's W-tile loader reads gate and up rows interleaved per 16 from the
two stacked blocks.  So a layer file streams to HBM as raw DMA of its tensors
(:mod:`..runtime.stream`), with at most an in-place dtype cast on the GPU.

:func:`placements` is the single description of where each checkpoint tensor
lands; the host cache, the streamer, data-parallel slices, ``pack_layer`` and
``unpack_layer`` all derive from it.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch

from ..config import ModelConfig

ALIGN_BYTES = 256


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
        specs = [("ln1", (H,)), ("wqkv", (cfg.qkv_size, H))]
        if cfg.attention_bias:
            specs.append(("bqkv", (cfg.qkv_size,)))
        if cfg.qk_norm:
            specs += [("qn", (cfg.head_dim,)), ("kn", (cfg.head_dim,))]
        specs.append(("wo", (H, cfg.q_size)))
        if cfg.o_proj_bias:
            specs.append(("bo", (H,)))
        if cfg.is_moe:
            E, Ie = cfg.num_local_experts, cfg.expert_intermediate
            specs += [("ln2", (H,)), ("wrouter", (E, H)), ("wgu", (E, 2 * Ie, H)), ("wdown", (E, H, Ie))]
            Is = cfg.shared_expert_intermediate_size
            if Is:
                specs += [("wsgu", (2 * Is, H)), ("wsdown", (H, Is)), ("wsg", (1, H))]
        else:
            specs += [("ln2", (H,)), ("wgu", (2 * I, H)), ("wdown", (H, I))]
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


def mlp_offset(lay: LayerLayout) -> int:
    """Byte offset of a decoder image's MLP piece (``ln2``, ``wgu``, ``wdown``); 0 for other kinds."""
    return lay.slot("ln2").offset if lay.kind == "decoder" else 0


@dataclass(frozen=True)
class Placement:
    """Checkpoint tensor ``hf_name`` occupies ``numel`` elements of ``elem_size`` bytes at byte
    ``offset`` of the image."""
    hf_name: str
    offset: int
    numel: int
    shape: Tuple[int, ...]
    elem_size: int = 2

    @property
    def nbytes(self) -> int:
        return self.elem_size * self.numel


def placements(cfg: ModelConfig, layer_name: str, elem_size: int = 2) -> List[Placement]:
    """Where every checkpoint tensor of ``layer_name`` lands in the packed image."""
    kind = layer_kind(layer_name)
    lay = layer_layout(cfg, kind, elem_size)
    es = elem_size
    H, I = cfg.hidden_size, cfg.intermediate_size
    if kind == "embed":
        return [Placement("model.embed_tokens.weight", 0, cfg.vocab_size * H, (cfg.vocab_size, H), es)]
    if kind == "head":
        return [Placement("lm_head.weight", 0, cfg.vocab_size * H, (cfg.vocab_size, H), es)]
    if kind == "norm":
        return [Placement("model.norm.weight", 0, H, (H,), es)]
    p = layer_name
    qs, ks = cfg.q_size, cfg.kv_size
    o = {s.name: s.offset for s in lay.slots}
    out = [
        Placement(f"{p}.input_layernorm.weight", o["ln1"], H, (H,), es),
        Placement(f"{p}.post_attention_layernorm.weight", o["ln2"], H, (H,), es),
        Placement(f"{p}.self_attn.o_proj.weight", o["wo"], H * qs, (H, qs), es),
    ]
    if cfg.is_moe:
        out += _expert_placements(cfg, p, o, es)
    else:
        out.append(Placement(f"{p}.mlp.down_proj.weight", o["wdown"], H * I, (H, I), es))
    if cfg.fused_projections:
        # Phi-3: one tensor each, already in slot row order
        qkv = qs + 2 * ks
        out += [Placement(f"{p}.self_attn.qkv_proj.weight", o["wqkv"], qkv * H, (qkv, H), es),
                Placement(f"{p}.mlp.gate_up_proj.weight", o["wgu"], 2 * I * H, (2 * I, H), es)]
    else:
        out += [
            Placement(f"{p}.self_attn.q_proj.weight", o["wqkv"], qs * H, (qs, H), es),
            Placement(f"{p}.self_attn.k_proj.weight", o["wqkv"] + es * qs * H, ks * H, (ks, H), es),
            Placement(f"{p}.self_attn.v_proj.weight", o["wqkv"] + es * (qs + ks) * H, ks * H, (ks, H), es),
        ]
        if not cfg.is_moe:
            out += [Placement(f"{p}.mlp.gate_proj.weight", o["wgu"], I * H, (I, H), es),
                    Placement(f"{p}.mlp.up_proj.weight", o["wgu"] + es * I * H, I * H, (I, H), es)]
    if cfg.attention_bias:
        out += [Placement(f"{p}.self_attn.q_proj.bias", o["bqkv"], qs, (qs,), es),
                Placement(f"{p}.self_attn.k_proj.bias", o["bqkv"] + es * qs, ks, (ks,), es),
                Placement(f"{p}.self_attn.v_proj.bias", o["bqkv"] + es * (qs + ks), ks, (ks,), es)]
    if cfg.o_proj_bias:
        out.append(Placement(f"{p}.self_attn.o_proj.bias", o["bo"], H, (H,), es))
    if cfg.qk_norm:
        hd = cfg.head_dim
        out += [Placement(f"{p}.self_attn.q_norm.weight", o["qn"], hd, (hd,), es),
                Placement(f"{p}.self_attn.k_norm.weight", o["kn"], hd, (hd,), es)]
    return out


def expert_names(cfg: ModelConfig, p: str, e: int) -> Tuple[str, str, str]:
    """Checkpoint names of expert ``e``'s (gate, up, down) weights in decoder layer ``p``: the
    per-expert tensors of the released checkpoints (Mixtral ``block_sparse_moe.experts.e.w1/w3/w2``,
    Qwen3-MoE ``mlp.experts.e.gate_proj/up_proj/down_proj``)."""
    if cfg.model_type == "mixtral":
        b = f"{p}.block_sparse_moe.experts.{e}"
        return f"{b}.w1.weight", f"{b}.w3.weight", f"{b}.w2.weight"
    b = f"{p}.mlp.experts.{e}"
    return f"{b}.gate_proj.weight", f"{b}.up_proj.weight", f"{b}.down_proj.weight"


def router_name(cfg: ModelConfig, p: str) -> str:
    return f"{p}.block_sparse_moe.gate.weight" if cfg.model_type == "mixtral" else f"{p}.mlp.gate.weight"


def _expert_placements(cfg: ModelConfig, p: str, o: Dict[str, int], es: int) -> List[Placement]:
    H, E, Ie = cfg.hidden_size, cfg.num_local_experts, cfg.expert_intermediate
    out = [Placement(router_name(cfg, p), o["wrouter"], E * H, (E, H), es)]
    for e in range(E):
        g, u, d = expert_names(cfg, p, e)
        gu = o["wgu"] + es * e * 2 * Ie * H
        out += [Placement(g, gu, Ie * H, (Ie, H), es),
                Placement(u, gu + es * Ie * H, Ie * H, (Ie, H), es),
                Placement(d, o["wdown"] + es * e * H * Ie, H * Ie, (H, Ie), es)]
    Is = cfg.shared_expert_intermediate_size
    if Is:
        b = f"{p}.mlp.shared_expert"
        out += [Placement(f"{b}.gate_proj.weight", o["wsgu"], Is * H, (Is, H), es),
                Placement(f"{b}.up_proj.weight", o["wsgu"] + es * Is * H, Is * H, (Is, H), es),
                Placement(f"{b}.down_proj.weight", o["wsdown"], H * Is, (H, Is), es),
                Placement(f"{p}.mlp.shared_expert_gate.weight", o["wsg"], H, (1, H), es)]
    return out


def source_key(cfg: ModelConfig, layer_name: str, hf_name: str, available) -> str:
    """Checkpoint key that feeds ``hf_name`` (tied LM head: the embedding table)."""
    if hf_name in available:
        return hf_name
    if hf_name == "lm_head.weight" and cfg.tie_word_embeddings and "model.embed_tokens.weight" in available:
        return "model.embed_tokens.weight"
    raise KeyError(f"{layer_name}: missing tensor {hf_name}")


def check_layer_tensors(cfg: ModelConfig, layer_name: str, available) -> None:
    """A config of an unlisted family runs as Llama (config.llama_like_rejection): its layer files
    must hold exactly the tensors a Llama layer reads — an extra one (a q/k norm, a post-MLP norm, a
    bias) means a different block, which is refused rather than run without it."""
    from ..config import SUPPORTED_MODEL_TYPES
    if cfg.model_type in SUPPORTED_MODEL_TYPES:
        return
    want = {pl.hf_name for pl in placements(cfg, layer_name)}
    extra = sorted(k for k in available if k not in want and not k.endswith("rotary_emb.inv_freq"))
    if extra:
        raise NotImplementedError(f"model_type={cfg.model_type!r} runs as Llama, but {layer_name} holds tensors a "
                                  f"Llama layer does not have: {extra[:4]}")


# ------------------------------------------------------------------- packing
def hf_param_names(cfg: ModelConfig, layer_name: str) -> List[str]:
    return [pl.hf_name for pl in placements(cfg, layer_name)]


def pack_layer(cfg: ModelConfig, layer_name: str, sd: Dict[str, torch.Tensor],
               dtype: torch.dtype = torch.float16, out: torch.Tensor = None) -> torch.Tensor:
    """HF-named state dict of one layer -> flat packed uint8 buffer (CPU).

    ``sd`` keys are full HF names (the per-layer file format of
    ``prepare_weights.py:40-43``).  ``int8`` is rejected like the reference
    (``utils.py:129``); other float dtypes are cast to ``dtype`` (``utils.py:130``).
    """
    kind = layer_kind(layer_name)
    es = torch.empty((), dtype=dtype).element_size()
    lay = layer_layout(cfg, kind, es)
    for v in sd.values():
        if v.dtype == torch.int8:
            raise AssertionError("int8 not supported (need to add fp16_statistics)")
    check_layer_tensors(cfg, layer_name, sd)
    if out is None:
        out = torch.zeros(lay.nbytes, dtype=torch.uint8)
    b = out.view(torch.uint8)
    for pl in placements(cfg, layer_name, es):
        key = source_key(cfg, layer_name, pl.hf_name, sd)
        t = sd[key]
        if tuple(t.shape) != pl.shape:
            raise ValueError(f"{layer_name}: {key} has shape {tuple(t.shape)}, config expects {pl.shape}")
        b[pl.offset:pl.offset + pl.nbytes].view(dtype).copy_(t.reshape(-1).to(dtype))
    return out


def unpack_layer(cfg: ModelConfig, layer_name: str, buf: torch.Tensor,
                 dtype: torch.dtype = torch.float16) -> Dict[str, torch.Tensor]:
    """Inverse of :func:`pack_layer` (HF names and shapes)."""
    es = torch.empty((), dtype=dtype).element_size()
    b = buf.view(torch.uint8)
    out = {}
    for pl in placements(cfg, layer_name, es):
        out[pl.hf_name] = b[pl.offset:pl.offset + pl.nbytes].view(dtype).view(pl.shape).clone()
    return out


def max_layer_bytes(cfg: ModelConfig, elem_size: int = 2) -> int:
    return max(layer_layout(cfg, k, elem_size).nbytes for k in ("embed", "decoder", "norm", "head"))
