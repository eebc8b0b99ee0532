"""Command-line interface — the reference flags verbatim plus additive ones.

Reference: ``/root/reference/main.py:30-49``.  Deliberate fix:
``--data_parallel`` is parsed as a real boolean (the reference uses
``type=bool``, so ``--data_parallel False`` silently meant True); a bare
``--data_parallel`` also enables it.
"""
from __future__ import annotations

import argparse


def str2bool(v) -> bool:
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y", "on"):
        return True
    if s in ("0", "false", "f", "no", "n", "off", ""):
        return False
    raise argparse.ArgumentTypeError(f"boolean expected, got {v!r}")


def bool_or_auto(v):
    return "auto" if str(v).strip().lower() == "auto" else str2bool(v)


def gb_or_auto(v):
    return "auto" if str(v).strip().lower() == "auto" else float(v)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X-native layer-sharded Llama scoring / generation")
    # ---- reference flags (main.py:31-46)
    p.add_argument("--model_path", type=str, default="./")
    p.add_argument("--prompt_pickle", type=str, required=True, help="Path to the input prompt pickle file")
    p.add_argument("--output_file", type=str, required=True, help="Path to the LLM output scores file")
    p.add_argument("--num_batch", type=int, default=1)
    p.add_argument("--layer_num_per_shard", type=int, default=1,
                   help="upper bound on layers per shard (balanced split)")
    p.add_argument("--storage_location", type=str, default="cpu", choices=["gpu", "cpu", "disk"],
                   help="'gpu': keep intermediate activations in HBM, 'cpu': pinned host RAM, 'disk': spill files")
    p.add_argument("--max_activation_in_cpu", type=int, default=100)
    p.add_argument("--data_parallel", type=str2bool, nargs="?", const=True, default=False,
                   help="multi-GPU: data parallel if true, model (pipeline) parallel otherwise")
    p.add_argument("--disk_folder", type=str, default="./temp",
                   help="folder for intermediate activation files in 'disk' mode")
    p.add_argument("--num_gen_token", type=int, default=1, help="how many new tokens to be generated")
    # ---- additive flags
    p.add_argument("--num_gpus", type=int, default=None, help="GPUs to use (default: all visible; 0 = CPU)")
    p.add_argument("--prefix_attention", choices=["bidirectional", "causal"], default="bidirectional",
                   help="prefix self-attention: reference-compatible bidirectional (default) or causal")
    p.add_argument("--hip_graphs", type=str2bool, nargs="?", const=True, default=False,
                   help="with --resident: capture each micro-batch's whole forward as one HIP graph and "
                        "replay it (shape-bucketed; removes per-op host dispatch for small batches)")
    p.add_argument("--prefix_kv_cache", type=bool_or_auto, nargs="?", const=True, default="auto",
                   help="keep every prompt's prefix K/V per layer in HBM and reuse it in later calls on the same "
                        "prefixes (each --num_gen_token step then computes only the suffix tokens; exact). "
                        "auto (default): on when --num_gen_token > 1")
    p.add_argument("--suffix_kv_cache", type=bool_or_auto, nargs="?", const=True, default="auto",
                   help="with the prefix K/V cache: also keep every suffix's K/V and, in the next call (generation "
                        "step), compute only the tokens after the longest common token prefix with the last call's "
                        "suffix (each step then costs its new tokens).  Exact: with the prefix cache every call runs "
                        "row-independent kernels, so a reused step's scores are bit for bit those of recomputing "
                        "every suffix token (PARITY.md C21).  auto (default): on with the prefix K/V cache on one GPU "
                        "without --max_vram_gb (capped steps are PCIe-bound: staging the suffix regions costs more "
                        "than recomputing the suffix tokens)")
    p.add_argument("--exact_reuse", type=str2bool, nargs="?", const=True, default=True,
                   help="with the K/V caches: run every call row-exact (default), so reused steps are bit for "
                        "bit the full recomputation; false: the faster small-M kernels (skinny / split-K GEMMs, "
                        "multi-suffix attention items), scores equal to rounding and tokens not guaranteed")
    p.add_argument("--prefix_cache_entries", type=int, default=8,
                   help="prefix K/V cache: calls (prompt batches) kept, LRU")
    p.add_argument("--resident", type=str2bool, nargs="?", const=True, default=False,
                   help="keep every shard resident in HBM after first load (288 GB fits 70B)")
    p.add_argument("--hbm_cache_gb", type=gb_or_auto, default="auto",
                   help="keep this many GB of shards resident in HBM after their first load, spread evenly "
                        "over the pass; the others stream every pass (generation steps with a partly "
                        "cached model move fewer bytes over PCIe).  auto (default): with repeated passes "
                        "over the same weights (--num_gen_token > 1 or --num_batch > 1) the free HBM minus "
                        "the activation plan (the whole 70B model on one 288 GB MI355X; data parallel: "
                        "resident all-gathered layers when they fit), else 0")
    p.add_argument("--weight_cache", choices=["auto", "host", "stream", "disk"], default="auto",
                   help="host: read every layer once into pinned host RAM (needs ~model-size RAM); "
                        "stream (alias disk, the reference behaviour): re-read the per-layer safetensors every "
                        "pass through a small pinned chunk ring (~256 MB of RAM) straight into HBM; "
                        "auto: host if it fits --host_mem_gb, else stream")
    p.add_argument("--host_mem_gb", type=float, default=None,
                   help="host RAM budget for --weight_cache auto / host (default: 80%% of MemAvailable)")
    p.add_argument("--o_direct", type=str2bool, nargs="?", const=True, default=False,
                   help="stream layer files with O_DIRECT (bypass the page cache)")
    p.add_argument("--dp_gather_comm", choices=["torch", "native"], default="torch",
                   help="data parallel: the weight all-gathers on a torch.distributed group (default) or on the "
                        "native RCCL communicator (csrc/comm/rccl_comm.cpp), issued from C on the copy stream")
    p.add_argument("--dp_weight_shard", type=str2bool, nargs="?", const=True, default=True,
                   help="data parallel: scatter-load 1/G of each layer per GPU + RCCL all-gather")
    p.add_argument("--rx_window", type=int, default=2,
                   help="model parallel: HBM receive-ring slots per rank (receives in flight at the point of use)")
    p.add_argument("--pipeline_stages", choices=["round_robin", "contiguous"], default="round_robin",
                   help="model parallel: shard k on GPU k mod G (reference) or one contiguous stage per GPU")
    p.add_argument("--token_budget", type=int, default=49152,
                   help="max tokens per packed micro-batch (MLP still runs in 16k-row chunks)")
    p.add_argument("--max_vram_gb", type=float, default=None,
                   help="HBM cap per GPU: sizes --token_budget and the MLP chunk to fit (reference: 70B in 6 GB)")
    p.add_argument("--dtype", choices=["float16", "float32"], default=None,
                   help="activation dtype (default fp16 on GPU, fp32 on CPU)")
    p.add_argument("--verbose", type=str2bool, nargs="?", const=True, default=False)
    p.add_argument("--metrics_json", type=str, default=None, help="write run metrics here (rank 0)")
    p.add_argument("--max_token_len", type=int, default=None,
                   help="token cap per prefix / suffix (reference: 4096, utils.py:14); also sizes the RoPE tables")
    p.add_argument("--synthetic", type=str, default=None, metavar="PRESET",
                   help="random-init weights of a preset architecture (tiny|small|llama2-7b|llama2-13b|llama2-70b) "
                        "generated in pinned host RAM, plus a synthetic tokenizer; --model_path is not read")
    p.add_argument("--resume_dir", type=str, default=None,
                   help="checkpoint inter-shard activations here and resume a crashed run from them "
                        "(single-GPU, data-parallel and model-parallel)")
    p.add_argument("--checkpoint_every", type=int, default=8, help="shards between checkpoints (with --resume_dir)")
    p.add_argument("--profile", type=str2bool, nargs="?", const=True, default=False,
                   help="emit roctx ranges (shard load / micro-batch compute) for rocprofv3 --marker-trace")
    return p


def parse_args(argv=None):
    return build_parser().parse_args(argv)
