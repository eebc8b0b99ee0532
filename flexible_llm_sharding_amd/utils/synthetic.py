"""Synthetic (no-network) checkpoints and prompts.

* :func:`write_synthetic_checkpoint` writes a complete per-layer model
  directory (``config.json``, tokenizer, ``{layer}.safetensors`` with full HF
  names) with random-init weights of a given architecture — the same format
  ``prepare_weights.py`` produces from a real HF checkpoint.
* :func:`synthetic_prompts` builds ``(prefix, suffixes)`` prompts with exact
  token counts under the synthetic tokenizer (Kaggle LLM-science-exam shape:
  one context, several answer options).
"""
from __future__ import annotations

import os
import random
from typing import Dict, List, Tuple

import torch

from ..config import ModelConfig
from .layer_format import layer_file
from .safetensors_io import save_file
from .tokenizer import synthetic_word, write_synthetic_tokenizer


def synthetic_layer_state_dict(cfg: ModelConfig, layer_name: str, seed: int = 0,
                               std: float = 0.02, dtype=torch.float16, device="cpu") -> Dict[str, torch.Tensor]:
    idx = cfg.layer_names().index(layer_name)
    g = torch.Generator(device=device).manual_seed(seed * 1000003 + idx)
    H, I, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size

    def rnd(*shape):
        return (torch.randn(*shape, generator=g, device=device) * std).to(dtype)

    def norm_w(n):
        return (1.0 + 0.1 * torch.randn(n, generator=g, device=device)).to(dtype)

    if layer_name == "model.embed_tokens":
        return {"model.embed_tokens.weight": (torch.randn(V, H, generator=g, device=device) * 1.0).to(dtype)}
    if layer_name == "model.norm":
        return {"model.norm.weight": norm_w(H)}
    if layer_name == "lm_head":
        return {"lm_head.weight": rnd(V, H)}
    p = layer_name
    bias = {}
    if cfg.attention_bias:
        bias.update({f"{p}.self_attn.q_proj.bias": rnd(cfg.q_size) * 10,
                     f"{p}.self_attn.k_proj.bias": rnd(cfg.kv_size) * 10,
                     f"{p}.self_attn.v_proj.bias": rnd(cfg.kv_size) * 10})
    if cfg.o_proj_bias:
        bias[f"{p}.self_attn.o_proj.bias"] = rnd(H) * 10
    if cfg.qk_norm:
        bias[f"{p}.self_attn.q_norm.weight"] = norm_w(cfg.head_dim)
        bias[f"{p}.self_attn.k_norm.weight"] = norm_w(cfg.head_dim)
    sd = {
        **bias,
        f"{p}.self_attn.q_proj.weight": rnd(cfg.q_size, H),
        f"{p}.self_attn.k_proj.weight": rnd(cfg.kv_size, H),
        f"{p}.self_attn.v_proj.weight": rnd(cfg.kv_size, H),
        f"{p}.self_attn.o_proj.weight": rnd(H, cfg.q_size),
        f"{p}.input_layernorm.weight": norm_w(H),
        f"{p}.post_attention_layernorm.weight": norm_w(H),
    }
    if cfg.is_moe:
        from ..models.layout import expert_names, router_name
        Ie = cfg.expert_intermediate
        # router rows ~ N(0, 1/H): logits of unit-RMS inputs ~ N(0, 1), so tokens spread over experts
        sd[router_name(cfg, p)] = (torch.randn(cfg.num_local_experts, H, generator=g, device=device)
                                   * H ** -0.5).to(dtype)
        for e in range(cfg.num_local_experts):
            gn, un, dn = expert_names(cfg, p, e)
            sd[gn], sd[un], sd[dn] = rnd(Ie, H), rnd(Ie, H), rnd(H, Ie)
        Is = cfg.shared_expert_intermediate_size
        if Is:
            b = f"{p}.mlp.shared_expert"
            sd[f"{b}.gate_proj.weight"], sd[f"{b}.up_proj.weight"] = rnd(Is, H), rnd(Is, H)
            sd[f"{b}.down_proj.weight"] = rnd(H, Is)
            sd[f"{p}.mlp.shared_expert_gate.weight"] = rnd(1, H) * 10
    else:
        sd.update({f"{p}.mlp.gate_proj.weight": rnd(I, H), f"{p}.mlp.up_proj.weight": rnd(I, H),
                   f"{p}.mlp.down_proj.weight": rnd(H, I)})
    return fuse_projections(cfg, p, sd) if cfg.fused_projections else sd


def fuse_projections(cfg: ModelConfig, p: str, sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Split q/k/v and gate/up tensors of layer ``p`` -> Phi-3's ``qkv_proj`` / ``gate_up_proj``."""
    sd = dict(sd)
    sd[f"{p}.self_attn.qkv_proj.weight"] = torch.cat(
        [sd.pop(f"{p}.self_attn.{n}_proj.weight") for n in "qkv"], 0)
    sd[f"{p}.mlp.gate_up_proj.weight"] = torch.cat(
        [sd.pop(f"{p}.mlp.{n}_proj.weight") for n in ("gate", "up")], 0)
    return sd


def split_projections(cfg: ModelConfig, sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Inverse of :func:`fuse_projections` over a whole state dict (HF Phi-3 chunk order)."""
    out = {}
    for k, v in sd.items():
        if k.endswith(".self_attn.qkv_proj.weight"):
            p = k[:-len("qkv_proj.weight")]
            q, kk, vv = torch.split(v, [cfg.q_size, cfg.kv_size, cfg.kv_size], 0)
            out.update({p + "q_proj.weight": q, p + "k_proj.weight": kk, p + "v_proj.weight": vv})
        elif k.endswith(".mlp.gate_up_proj.weight"):
            p = k[:-len("gate_up_proj.weight")]
            g, u = v.chunk(2, 0)
            out.update({p + "gate_proj.weight": g, p + "up_proj.weight": u})
        else:
            out[k] = v
    return out


def write_synthetic_checkpoint(cfg: ModelConfig, out_dir: str, seed: int = 0,
                               std: float = 0.02, dtype=torch.float16, unique_layers: int = 0,
                               device="cpu", progress=None) -> None:
    """``unique_layers`` > 0: only the first K decoder layers get their own random weights;
    decoder layer i >= K is a hard link to layer i % K (a 138 GB 70B checkpoint in ~K x 1.7 GB of
    disk for streaming benchmarks — the reads are per file, as for a real checkpoint)."""
    os.makedirs(out_dir, exist_ok=True)
    cfg.save(out_dir)
    write_synthetic_tokenizer(out_dir, cfg.vocab_size)
    names = cfg.layer_names()
    for li, name in enumerate(names):
        if progress is not None:
            progress(li, len(names))
        path = layer_file(out_dir, name)
        if unique_layers and name.startswith("model.layers."):
            i = int(name.split(".")[2])
            if i >= unique_layers:
                src = layer_file(out_dir, f"model.layers.{i % unique_layers}")
                if os.path.exists(path):
                    os.remove(path)
                os.link(src, path)
                continue
        sd = synthetic_layer_state_dict(cfg, name, seed, std, dtype, device)
        save_file(sd, path)


def load_full_state_dict(cfg: ModelConfig, model_path: str) -> Dict[str, torch.Tensor]:
    from .safetensors_io import load_file
    sd = {}
    for name in cfg.layer_names():
        sd.update(load_file(layer_file(model_path, name)))
    return sd


def _words(rng: random.Random, n: int, vocab_size: int) -> str:
    return " ".join(synthetic_word(rng.randrange(3, vocab_size)) for _ in range(n))


def synthetic_prompts(n_prompts: int, prefix_len: int, n_suffix: int, suffix_len: int,
                      vocab_size: int = 32000, seed: int = 0,
                      vary: bool = False) -> List[Tuple[str, Tuple[str, ...]]]:
    """Prompts whose tokenization gives Lp = prefix_len (BOS incl.) and, per
    suffix, suffix_len tokens after the BOS drop (``vary`` randomises lengths)."""
    rng = random.Random(seed)
    out = []
    for _ in range(n_prompts):
        lp = prefix_len if not vary else rng.randint(max(2, prefix_len // 2), prefix_len)
        pre = _words(rng, lp - 1, vocab_size)
        sufs = []
        for _ in range(n_suffix):
            ls = suffix_len if not vary else rng.randint(1, suffix_len)
            sufs.append(_words(rng, ls, vocab_size))
        out.append((pre, tuple(sufs)))
    return out
