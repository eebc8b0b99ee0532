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
        save_file(sd, layer_file(out_dir, l))
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


def _tied(src_dir: str) -> bool:
    try:
        with open(os.path.join(src_dir, "config.json")) as f:
            return bool(json.load(f).get("tie_word_embeddings", False))
    except (OSError, ValueError):
        return False
