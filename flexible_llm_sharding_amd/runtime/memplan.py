"""HBM budget planning (``--max_vram_gb``).

The reference's headline claim is a 70B model on a GPU with >= 6 GB of VRAM
at ``layer_num_per_shard=1`` (``/root/reference/README.md:2,31``).  Here the
HBM in use is

    weight slots (2 x the largest shard: 2 x 1.71 GB for 70B, lnps=1)
  + one workspace arena (models/llama.py): [QKV of the micro-batch | row statistics] in the
    attention phase with the fused RMSNorm + QKV GEMM ([normed chunk (``qkv_chunk`` rows) | QKV]
    without it) — the attention output overwrites Q in place — and [normed chunk | SwiGLU chunk]
    (``mlp_chunk`` rows) in the MLP phase
  + the hidden states alive: the engine's activation ring (engine.ActRing): 1 slot when the whole
    call is one micro-batch (it never leaves HBM), one per micro-batch when a token budget splits
    a call whose states all fit (resident: none is parked), else 2 — the micro-batch being
    computed and the next one landing (the zigzag order's carries fit in the same two slots)
  + the HIP context, code objects and allocator slack,

so a VRAM cap is met by sizing ``token_budget``, ``qkv_chunk`` and ``mlp_chunk``:
:func:`plan_for_vram` picks, for the call's token count, the fewest micro-batches (one means
no activation traffic over PCIe at all) and then the largest chunks whose estimated peak
fits.  ``bench.py --max-vram-gb`` reports the measured ``hipMemGetInfo`` peak next to it.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

from .. import knobs
from ..config import ModelConfig
from ..models.layout import layer_kind, layer_layout

# HIP context + code objects (measured on MI355X: 0.665 GB of device memory in use right after
# context creation, profiles/r2_vram/ctx.log) + events / small buffers
DEVICE_OVERHEAD = int(0.75e9)
# hidden states alive at once with several micro-batches per call: the activation ring's slots
# (engine.ActRing: the state being computed + the next one landing, or a zigzag carry)
RING_SLOTS = 2
STATES = RING_SLOTS
# caching-allocator slack on the few fixed activation blocks (ring slots + arena), 2 MB rounded;
# the small per-call tensors (metadata, pruned rows, logits) are in the 64 MB margin
SLACK = 1.02
SLACK_ONE = 1.02
# the multi-micro-batch plan prefers MLP chunks of at least this many rows before fewer
# micro-batches (round 4's capped plan fell to 2,048-row chunks with 5 live states: -31%, VERDICT
# r4 #2); chunks are multiples of 3,072 rows = whole 256-CU rounds of the 70B MLP GEMMs, so
# 9,216 and 12,288 differ only in per-launch ramps, while each extra micro-batch adds a round of
# small per-layer launches (r5: 15 micro-batches of 12,288 rows ran 94.8% of the headline rate)
MLP_CHUNK_TARGET = 9216
# the plan aims this far below the cap (the estimate is a model; hipMemGetInfo is the judge: the
# 70B headline's plan estimates 5.92 GB against a 2 ms-sampled peak of 5.77-5.78, profiles/r6_head)
CAP_MARGIN = 0.012
# device memory the HIP runtime takes outside any allocator for a moment while a pass runs: up to
# ~185 MB above the steady context for <= 2 ms around some host -> device weight copies, sampled
# every 2 ms on the 70B headline (profiles/r4_vram); kept free under a cap, by the allocator limit
# and by the plan
RUNTIME_RESERVE = knobs.get_int("FLS_RUNTIME_RESERVE_MB") << 20
# one activation-ring slot per micro-batch when they all fit (A/B knob)


def activation_bytes(cfg: ModelConfig, tokens: int, mlp_chunk: int, elem: int = 2, qkv_chunk: int = 0,
                     states: int = STATES, attn_rows: int = 0, fused_norm: bool = False) -> int:
    """Peak activation bytes of one micro-batch of ``tokens`` rows: the workspace arena
    (models.llama: [QKV | row statistics] with ``fused_norm``, else [normed chunk | QKV] — of the
    whole micro-batch, or of one prompt-aligned group of <= ``attn_rows`` rows — then [normed
    chunk | SwiGLU chunk]) + live states."""
    from ..models.llama import balanced_step
    H, I, Q = cfg.hidden_size, cfg.intermediate_size, cfg.qkv_size
    chunk = balanced_step(tokens, mlp_chunk)
    rows = attn_rows if (attn_rows and attn_rows < tokens) else tokens
    if fused_norm:
        attn = rows * (Q + 2)                  # QKV + the fp32 row statistic (2 fp16 columns)
    elif attn_rows and attn_rows < tokens:
        attn = attn_rows * (H + Q)
    else:
        qc = balanced_step(tokens, qkv_chunk) if qkv_chunk else tokens
        attn = qc * H + tokens * Q
    # MLP phase: [normed chunk | SwiGLU chunk] ([SwiGLU chunk | row statistics] fused); MoE: k
    # SwiGLU rows and k expert outputs per token
    if fused_norm and not cfg.is_moe:
        mlp = chunk * (I + 2)
    else:
        mlp = chunk * (H + (cfg.num_experts_per_tok * (cfg.expert_intermediate + H) if cfg.is_moe else I))
    # Qwen2-MoE shared expert: its SwiGLU rows, output and gated output per chunk (allocator)
    mlp += chunk * (cfg.shared_expert_intermediate_size + 2 * H) if cfg.shared_expert_intermediate_size else 0
    scratch = max(attn, mlp)                             # one arena, two phases
    # fused norm: the residual GEMMs' per-row partial sums of squares (fp32 per 128 columns), kept
    # from one residual GEMM to the next norm-folded projection (models.llama ExecContext.ss_buf)
    ss = tokens * 2 * -(-H // 128) if (fused_norm and not cfg.is_moe) else 0
    slack = SLACK_ONE if states == 1 else SLACK
    return int(slack * elem * (scratch + ss + states * tokens * H))


def shared_device_bytes() -> int:
    """Device memory held by OTHER processes on the same GPU (``FLS_VRAM_SHARED_GB``, default 0),
    left out of this process's ``--max_vram_gb`` budget: hipMemGetInfo counts the whole device,
    so a co-tenant (e.g. the pytest process that launched a capped worker) would otherwise be
    charged to the cap."""
    return int(float(knobs.get("FLS_VRAM_SHARED_GB") or 0) * 1e9)


def device_used_bytes(device) -> int:
    """This process's share of the device memory in use: hipMemGetInfo minus other tenants."""
    import torch
    free, total = torch.cuda.mem_get_info(device)
    return (total - free) - shared_device_bytes()


def warm_copy_paths(device, streams, nbytes: int = 8 << 20) -> None:
    """One host -> device and one device -> host copy on each stream (and the current one).  The
    first copy of a process makes the HIP runtime set up its copy path, which holds ~0.2-0.35 GB
    of device memory outside any allocator for a moment (scripts/copy_probe.py: +340 MB and a
    150 ms enqueue on the first 1.4 GB copy, nothing on later ones); under ``--max_vram_gb`` that
    belongs before the plan measures the context, not inside the first pass."""
    import torch
    from . import hostmem
    host = hostmem.alloc_host(nbytes, pinned=True)
    dev = torch.empty(nbytes, dtype=torch.uint8, device=device)
    for st in [s for s in streams if s is not None] + [torch.cuda.current_stream(device)]:
        with torch.cuda.stream(st):
            dev.copy_(host, non_blocking=True)
            host.copy_(dev, non_blocking=True)
        st.synchronize()
    del dev, host


def cap_allocator(device, max_vram_bytes: int, other_device_bytes: int) -> int:
    """Bound the caching allocator so that, with ``other_device_bytes`` held outside it (the
    raw weight slots), the device's memory in use stays <= ``max_vram_bytes``; when a request
    would pass the bound the allocator returns its unused cached blocks and retries.  Returns
    the allocator byte limit."""
    import torch
    total = torch.cuda.mem_get_info(device)[1]
    outside = device_used_bytes(device) - torch.cuda.memory_reserved(device)   # context, code objects, raw blocks
    limit = max_vram_bytes - outside - other_device_bytes - (64 << 20) - RUNTIME_RESERVE
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
                  token_budget: int = 49152, mlp_chunk: int = 16384,
                  total_tokens: Optional[int] = None, max_prompt_rows: int = 0,
                  overhead: Optional[int] = None, weight_bytes: Optional[int] = None,
                  fused_norm: bool = False, extra_bytes: int = 0,
                  grouped: bool = True) -> Tuple[int, int, int, int, int, bool]:
    """-> (token_budget, mlp_chunk, attn_rows, qkv_chunk, estimated peak bytes, resident) for a
    call of ``total_tokens`` packed tokens (None: unknown, assume several micro-batches) whose
    largest prompt has ``max_prompt_rows`` rows.  ``overhead``: device memory held outside the plan
    (measured context + code objects; default DEVICE_OVERHEAD); ``weight_bytes``: the weight
    buffers actually planned (default ``n_slots`` full-shard slots); ``extra_bytes``: other fixed
    device buffers (the host-mode prefix K/V cache's staging); ``grouped=False``: no prompt-aligned
    attention groups (the prefix K/V cache runs the whole micro-batch).  ``resident``: every
    micro-batch's hidden state keeps an activation-ring slot of its own for the whole pass (no
    state is parked in host memory); else the ring has ``STATES`` slots.

    Preference, by measured cost on the 70B pass (one box, ``profiles/r3_vram``): one micro-batch
    when it fits with MLP chunks of ``MLP_CHUNK_TARGET`` rows (the hidden state never leaves HBM:
    no activation traffic over PCIe); else MLP chunks up to that size first (14,336 vs 10,752
    rows: 2.1% of a pass, GEMM tile-round tails), then every state resident (a call split by a
    token budget whose states together fit: no PCIe round trip per micro-batch and layer, which
    the piece pool's weight loads share; profiles/r5_spill), then the fewest micro-batches (each
    parks its state over PCIe in the copy engine's shadow); then the largest MLP chunk, then the
    whole micro-batch in one attention phase (prompt-aligned groups: ~1%) with the QKV projection
    in the largest row chunks that fit, then the largest groups; raises if nothing fits."""
    from ..models.llama import balanced_step
    weights = weight_slot_bytes(cfg, lnps, n_slots) if weight_bytes is None else weight_bytes
    target = int(max_vram_bytes * (1.0 - CAP_MARGIN))
    over = (DEVICE_OVERHEAD if overhead is None else overhead) + extra_bytes
    best = None
    budgets = sorted({token_budget, 49152, 32768, 24576, 16384, 12288, 8192, 6144, 4096, 3072, 2048, 1024})
    # multiples of 3072 rows give whole 256-CU rounds of the 384-row GEMM tile (models/llama.py)
    chunks = sorted({mlp_chunk, 16384, 15360, 12288, 9216, 8192, 6144, 4096, 3072, 2048, 1024})
    for tb in (t for t in budgets if t <= token_budget):
        rows = min(tb, total_tokens) if total_tokens else tb
        n_mb = -(-total_tokens // tb) if total_tokens else 2
        # live states: 1 (one micro-batch), every micro-batch's own (resident; known call only)
        # or the ring's two
        state_opts = (1,) if n_mb == 1 else ((n_mb, STATES) if total_tokens and n_mb > STATES
                                                   else (STATES,))
        for states in state_opts:
            resident = states == n_mb
            for mc in (m for m in chunks if m <= min(mlp_chunk, tb)):
                mce = balanced_step(rows, mc)
                for ar in (sorted({0, 32768, 24576, 16384, 12288, 8192, 4096}) if grouped else (0,)):
                    if ar and (ar >= rows or ar < max_prompt_rows):
                        continue
                    qcs = (0, 16384, 12288, 9216, 8192, 6144, 4096, 3072, 2048) if ar == 0 and not fused_norm else (0,)
                    for qc in qcs:
                        if qc and qc >= rows:
                            continue
                        est = weights + over + activation_bytes(cfg, rows, mc, qkv_chunk=qc, states=states,
                                                                attn_rows=ar, fused_norm=fused_norm)
                        good = min(mce, MLP_CHUNK_TARGET, rows)
                        key = (n_mb == 1 and mce >= min(MLP_CHUNK_TARGET, rows), good, resident, -n_mb, mce,
                               ar == 0, balanced_step(rows, qc) if qc else rows, ar)
                        if est <= target and (best is None or key > best[6]):
                            best = (tb, mc, ar, qc, est, resident, key)
    if best is None:
        raise ValueError(f"--max_vram_gb {max_vram_bytes / 1e9:.1f}: the weight slots alone need "
                         f"{(weights + over) / 1e9:.1f} GB")
    return best[:6]
