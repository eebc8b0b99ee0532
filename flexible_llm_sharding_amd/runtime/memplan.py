"""HBM budget planning (``--max_vram_gb``).

The reference's headline claim is a 70B model on a GPU with >= 6 GB of VRAM
at ``layer_num_per_shard=1`` (``/root/reference/README.md:2,31``).  Here the
HBM in use is

    weight slots (2 x the largest shard: 2 x 1.71 GB for 70B, lnps=1)
  + activations of one packed micro-batch (``token_budget`` tokens)
  + the MLP chunk intermediate (``mlp_chunk`` rows x intermediate_size)
  + states kept across shard boundaries / in flight on the copy streams
  + the HIP context, code objects and allocator slack,

so a VRAM cap is met by sizing ``token_budget`` and ``mlp_chunk``:
:func:`plan_for_vram` picks the largest (most MFMA-efficient) pair whose
estimated peak fits.  The estimate is deliberately simple and conservative;
``bench.py --max-vram-gb`` reports the measured ``hipMemGetInfo`` peak next
to it (``profiles/r2_vram``).
"""
from __future__ import annotations

from typing import Tuple

from ..config import ModelConfig
from ..models.layout import layer_kind, layer_layout

# HIP context + code objects + allocator slack (measured on MI355X: device use before the first
# allocation ~0.3 GB; caching-allocator rounding / fragmentation of a few hundred MB)
DEVICE_OVERHEAD = int(0.9e9)
# hidden states alive besides the one being computed: carry window (3) + one H2D landing buffer
EXTRA_STATES = 4


def activation_bytes(cfg: ModelConfig, tokens: int, mlp_chunk: int, elem: int = 2) -> int:
    """Peak activation bytes of one micro-batch of ``tokens`` rows through a decoder layer."""
    H, I = cfg.hidden_size, cfg.intermediate_size
    chunk = min(tokens, mlp_chunk)
    attn = tokens * (H + cfg.qkv_size + cfg.q_size)               # x, qkv, attention output
    mlp = tokens * H + chunk * (H + I)                             # x, normed chunk, SwiGLU chunk
    return elem * (max(attn, mlp) + EXTRA_STATES * tokens * H)


def weight_slot_bytes(cfg: ModelConfig, lnps: int, n_slots: int = 2) -> int:
    dec = layer_layout(cfg, "decoder").nbytes
    emb = layer_layout(cfg, layer_kind("model.embed_tokens")).nbytes
    return n_slots * max(lnps * dec, emb + (lnps - 1) * dec)


def plan_for_vram(cfg: ModelConfig, max_vram_bytes: int, lnps: int = 1, n_slots: int = 2,
                  token_budget: int = 16384, mlp_chunk: int = 16384) -> Tuple[int, int, int]:
    """-> (token_budget, mlp_chunk, estimated peak bytes), the largest pair <= the requested one
    that fits ``max_vram_bytes``; raises if even the smallest does not."""
    weights = weight_slot_bytes(cfg, lnps, n_slots)
    best = None
    for tb in sorted({token_budget, 16384, 12288, 8192, 6144, 4096, 3072, 2048, 1024}, reverse=True):
        if tb > token_budget:
            continue
        for mc in sorted({mlp_chunk, 16384, 8192, 4096, 2048, 1024}, reverse=True):
            if mc > mlp_chunk or mc > tb:
                continue
            est = weights + activation_bytes(cfg, tb, mc) + DEVICE_OVERHEAD
            if est <= max_vram_bytes:
                best = (tb, mc, est)
                break
        if best:
            break
    if best is None:
        raise ValueError(f"--max_vram_gb {max_vram_bytes / 1e9:.1f}: the weight slots alone need "
                         f"{(weights + DEVICE_OVERHEAD) / 1e9:.1f} GB")
    return best
