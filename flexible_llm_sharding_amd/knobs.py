"""Every ``FLS_*`` environment variable the framework reads, in one documented list.

The CLI flags (``utils/cli.py``) are the interface; these are test hooks, A/B switches of
measured design choices and deployment settings.  Code reads them only through :func:`get` /
:func:`get_int`, which refuse a name that is not registered here, so this table is complete by
construction (``tests/test_cli.py::test_every_env_knob_is_registered`` greps the sources).
"""
from __future__ import annotations

import os
from typing import Dict, Tuple

# name -> (default, what it does)
KNOBS: Dict[str, Tuple[str, str]] = {
    # ---- deployment
    "FLS_OFFLOAD_ARCH": ("gfx950", "hipcc --offload-arch of the kernel build (_native/build.py)"),
    "FLS_IO_THREADS": ("8", "threads of the native pread / pwrite pool (weights and activation spills)"),
    "FLS_STREAM_CHUNK_MB": ("64", "--weight_cache stream: pinned chunk size of the streamer ring (MB)"),
    "FLS_STREAM_CHUNKS": ("6", "--weight_cache stream: chunks in the pinned ring (6 x 64 MB holds a whole 70B "
                               "attention piece read ahead of its busy slot: profiles/r5_envelope)"),
    "FLS_O_DIRECT": ("0", "--weight_cache stream: read layer files with O_DIRECT (same as --o_direct)"),
    "FLS_RUNTIME_RESERVE_MB": ("192", "--max_vram_gb: device memory kept free for HIP-runtime transients "
                                      "(profiles/r4_vram)"),
    "FLS_VRAM_SHARED_GB": ("0", "--max_vram_gb: device memory held by other processes on the same GPU, "
                                "left out of this process's budget"),
    # ---- observability
    "FLS_TRACE": ("0", "roctx ranges around load / compute / store / comm (same as --profile)"),
    "FLS_PROFILE_GEN_STEPS": ("", "comma-separated generation steps to run under cProfile"),
    # ---- tests / fault injection
    "FLS_FAULT": ("", "'rank:shard': raise on that rank when it enters that local shard"),
    "FLS_PIECE_POOL": ("1", "0: whole-layer weight slots under --max_vram_gb instead of the "
                            "attention / MLP piece pool (tests: both must give the same scores)"),
    # ---- A/B switches of measured choices (defaults are the measured winners)
    "FLS_SPLITK": ("1", "0: no split-K path for <= 512-row GEMMs"),
    "FLS_DECODE_GRAPHS": ("1", "0: no HIP-graph replay of decode-like calls (generation steps with the "
                               "prefix + suffix K/V caches and every weight in HBM)"),
    "FLS_SPEC_DECODE": ("1", "0: no speculative generation steps (the next decode-graphed step enqueued behind the "
                             "current one, assuming re-tokenization appends exactly the greedy token; checked)"),
    "FLS_QKV_FOLD": ("1", "0: RMSNorm + QKV as two kernels instead of the row-scaled GEMM on the "
                          "raw hidden state with the norm weight folded into W_qkv"),
}


def get(name: str) -> str:
    """The knob's value (its registered default when unset)."""
    if name not in KNOBS:
        raise KeyError(f"{name} is not a registered FLS_* knob (flexible_llm_sharding_amd/knobs.py)")
    return os.environ.get(name, KNOBS[name][0])


def get_int(name: str) -> int:
    v = get(name)
    return int(v) if v.strip() else 0


def is_set(name: str) -> bool:
    if name not in KNOBS:
        raise KeyError(f"{name} is not a registered FLS_* knob (flexible_llm_sharding_amd/knobs.py)")
    return name in os.environ


def table() -> str:
    """Markdown table of every knob (README)."""
    rows = ["| variable | default | effect |", "|---|---|---|"]
    rows += [f"| `{k}` | `{d}` | {doc} |" for k, (d, doc) in KNOBS.items()]
    return "\n".join(rows)
