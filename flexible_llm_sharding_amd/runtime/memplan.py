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

# HIP context + code objects (measured on MI355X: 0.665 GB of device memory in use right after
# context creation, profiles/r2_vram/ctx.log) + events / small buffers
DEVICE_OVERHEAD = int(0.75e9)
# hidden states alive at once: the one being computed, the carry window (3, engine.CARRY_WINDOW)
# and one H2D landing buffer
STATES = 5
# caching-allocator slack on the (few, reused) activation blocks
SLACK = 1.10


def activation_bytes(cfg: ModelConfig, tokens: int, mlp_chunk: int, elem: int = 2) -> int:
    """Peak activation bytes of one micro-batch of ``tokens`` rows: the fixed scratch buffers
    (models.llama.Workspace: normed input, QKV, attention output, SwiGLU chunk) + live states."""
    H, I = cfg.hidden_size, cfg.intermediate_size
    chunk = min(tokens, mlp_chunk)
    scratch = max(tokens * (H + cfg.qkv_size + cfg.q_size), chunk * (H + I))   # one arena, two phases
    return int(SLACK * elem * (scratch + STATES * tokens * H))


def cap_allocator(device, max_vram_bytes: int, other_device_bytes: int) -> int:
    """Bound the caching allocator so that, with ``other_device_bytes`` held outside it (the
    raw weight slots), the device's memory in use stays <= ``max_vram_bytes``; when a request
    would pass the bound the allocator returns its unused cached blocks and retries.  Returns
    the allocator byte limit."""
    import torch
    free, total = torch.cuda.mem_get_info(device)
    outside = (total - free) - torch.cuda.memory_reserved(device)     # context, code objects, raw blocks
    limit = max_vram_bytes - outside - other_device_bytes - (64 << 20)
    if limit <= 0:
        raise ValueError(f"--max_vram_gb {max_vram_bytes / 1e9:.2f}: context + weight slots alone need "
                         f"{(outside + other_device_bytes) / 1e9:.2f} GB")
    torch.cuda.set_per_process_memory_fraction(min(1.0, limit / total), device)
    return limit


def weight_slot_bytes(cfg: ModelConfig, lnps: int, n_slots: int = 2) -> int:
    dec = layer_layout(cfg, "decoder").nbytes
    emb = layer_layout(cfg, layer_kind("model.embed_tokens")).nbytes
    return n_slots * max(lnps * dec, emb + (lnps - 1) * dec)


def plan_for_vram(cfg: ModelConfig, max_vram_bytes: int, lnps: int = 1, n_slots: int = 2,
                  token_budget: int = 49152, mlp_chunk: int = 16384) -> Tuple[int, int, int]:
    """-> (token_budget, mlp_chunk, estimated peak bytes), the largest pair <= the requested one
    that fits ``max_vram_bytes``; raises if even the smallest does not."""
    weights = weight_slot_bytes(cfg, lnps, n_slots)
    best = None
    # every GEMM wants a large M: prefer the pair with the largest smaller side, then the largest sum
    for tb in (t for t in sorted({token_budget, 49152, 32768, 24576, 16384, 12288, 8192, 6144, 4096, 3072, 2048, 1024}) if t <= token_budget):
        for mc in (m for m in sorted({mlp_chunk, 16384, 8192, 4096, 2048, 1024}) if m <= min(mlp_chunk, tb)):
            est = weights + activation_bytes(cfg, tb, mc) + DEVICE_OVERHEAD
            key = (min(tb, mc), tb + mc)
            if est <= max_vram_bytes and (best is None or key > best[3]):
                best = (tb, mc, est, key)
    if best is None:
        raise ValueError(f"--max_vram_gb {max_vram_bytes / 1e9:.1f}: the weight slots alone need "
                         f"{(weights + DEVICE_OVERHEAD) / 1e9:.1f} GB")
    return best[:3]
