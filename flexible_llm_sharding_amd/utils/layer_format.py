"""Per-layer checkpoint conversion (``prepare_weights.py``) and layer-file paths.

Reference: ``/root/reference/prepare_weights.py:12-49``.  Each parameter maps
to the layer ``'.'.join(name.replace('.weight','').split('.')[:3])``
(``prepare_weights.py:21``); every non-``.bin`` file (config, tokenizer) is
copied; each layer is written to ``{out}/{layer}.safetensors`` keeping full HF
names and dtype.

Fixes over the reference: ``model.safetensors.index.json`` and
single-file checkpoints are supported besides ``pytorch_model.bin.index.json``;
layers are processed in source-shard order and source tensors are evicted as
soon as their layer is written.  ``.bin`` shards are read with
``torch.load(weights_only=True)`` (never unpickling arbitrary objects).
"""
from __future__ import annotations

import glob
import json
import os
import shutil
from collections import OrderedDict, defaultdict
from typing import Dict, List

import torch

from .safetensors_io import load_file, save_file


def layer_of_param(name: str) -> str:
    """prepare_weights.py:21 — first three dotted components after stripping '.weight'."""
    return ".".join(name.replace(".weight", "").split(".")[:3])


def normalize_expert_names(model_type: str, sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """MoE state dicts in transformers-v5 form (``mlp.experts.gate_up_proj`` [E, 2I, H] /
    ``mlp.experts.down_proj`` [E, H, I], Mixtral's router as ``mlp.gate``) -> the per-expert tensors
    of the released checkpoints (Mixtral ``block_sparse_moe.experts.e.w1/w3/w2``, Qwen3-MoE
    ``mlp.experts.e.gate_proj/up_proj/down_proj``), the one form the per-layer files hold
    (``models.layout.placements``).  Other keys pass through."""
    if model_type not in ("mixtral", "qwen3_moe", "qwen2_moe"):
        return sd
    out = {}
    for k, v in sd.items():
        if k.endswith(".mlp.experts.gate_up_proj") or k.endswith(".mlp.experts.down_proj"):
            p = k[:-len(".mlp.experts.gate_up_proj")] if k.endswith("gate_up_proj") else k[:-len(".mlp.experts.down_proj")]
            for e in range(v.shape[0]):
                if model_type == "mixtral":
                    b = f"{p}.block_sparse_moe.experts.{e}"
                    names = (f"{b}.w1.weight", f"{b}.w3.weight", f"{b}.w2.weight")
                else:
                    b = f"{p}.mlp.experts.{e}"
                    names = (f"{b}.gate_proj.weight", f"{b}.up_proj.weight", f"{b}.down_proj.weight")
                if k.endswith("gate_up_proj"):
                    g, u = v[e].chunk(2, 0)
                    out[names[0]], out[names[1]] = g.contiguous(), u.contiguous()
                else:
                    out[names[2]] = v[e].contiguous()
        elif model_type == "mixtral" and k.endswith(".mlp.gate.weight"):
            out[k[:-len(".mlp.gate.weight")] + ".block_sparse_moe.gate.weight"] = v
        else:
            out[k] = v
    return out


def layer_file(model_path: str, layer_name: str) -> str:
    return os.path.join(model_path, f"{layer_name}.safetensors")


def _weight_map(src: str) -> Dict[str, str]:
    for idx in ("pytorch_model.bin.index.json", "model.safetensors.index.json"):
        p = os.path.join(src, idx)
        if os.path.exists(p):
            with open(p) as f:
                return json.load(f)["weight_map"]
    for single in ("model.safetensors", "pytorch_model.bin"):
        p = os.path.join(src, single)
        if os.path.exists(p):
            if single.endswith(".safetensors"):
                from .safetensors_io import read_header
                names = read_header(p)[0].keys()
            else:
                names = torch.load(p, map_location="cpu", weights_only=True).keys()
            return {n: single for n in names}
    raise FileNotFoundError(f"{src}: no weight index / checkpoint found")


def _load_shard(path: str) -> Dict[str, torch.Tensor]:
    if path.endswith(".safetensors"):
        return load_file(path)
    return torch.load(path, map_location="cpu", weights_only=True)


def split_into_layers(src_dir: str, out_dir: str, verbose: bool = True) -> List[str]:
    """Convert an HF checkpoint directory into per-layer safetensors files."""
    os.makedirs(out_dir, exist_ok=True)
    for fn in glob.glob(os.path.join(src_dir, "*")):
        base = os.path.basename(fn)
        if os.path.isdir(fn):
            continue
        if ".bin" in base or base.endswith(".safetensors") or base.endswith(".index.json"):
            continue
        shutil.copy(fn, os.path.join(out_dir, base))

    wmap = _weight_map(src_dir)
    layer_params: Dict[str, List[str]] = defaultdict(list)
    for p in wmap:
        layer_params[layer_of_param(p)].append(p)
    tied = "lm_head" not in layer_params and "model.embed_tokens.weight" in wmap and _tied(src_dir)
    model_type = _config(src_dir).get("model_type", "llama")
    # deterministic order: by the (sorted) source shards each layer needs
    shard_order = {s: i for i, s in enumerate(sorted(set(wmap.values())))}
    layers = sorted(layer_params, key=lambda l: (max(shard_order[wmap[p]] for p in layer_params[l]), l))
    # last layer that needs each shard -> evict after it
    last_use = {}
    for l in layers:
        for p in layer_params[l]:
            last_use[wmap[p]] = l

    cache: "OrderedDict[str, Dict[str, torch.Tensor]]" = OrderedDict()
    written = []
    it = layers
    if verbose:
        try:
            from tqdm import tqdm
            it = tqdm(layers, desc="split_into_layers")
        except Exception:  # pragma: no cover
            pass
    for l in it:
        need = sorted({wmap[p] for p in layer_params[l]})
        for s in need:
            if s not in cache:
                cache[s] = _load_shard(os.path.join(src_dir, s))
        sd = {}
        for p in layer_params[l]:
            sd[p] = cache[wmap[p]][p]
        assert len(sd) == len(layer_params[l]), f"Should have {len(layer_params[l])} keys for {l}"
        save_file(normalize_expert_names(model_type, sd), layer_file(out_dir, l))
        written.append(l)
        if tied and l == "model.embed_tokens":
            # tie_word_embeddings checkpoints store no lm_head: give the head its own layer file so
            # the per-layer format stays complete (the reference would fail to open lm_head here)
            save_file({"lm_head.weight": sd["model.embed_tokens.weight"].clone()}, layer_file(out_dir, "lm_head"))
            written.append("lm_head")
        for s in need:
            if last_use.get(s) == l:
                cache.pop(s, None)
    return written


def _config(src_dir: str) -> dict:
    try:
        with open(os.path.join(src_dir, "config.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _tied(src_dir: str) -> bool:
    return bool(_config(src_dir).get("tie_word_embeddings", False))
