"""End-to-end driver: ``main.py`` semantics on one process per GPU.

Reference (``/root/reference/main.py:52-98``): load the prompt pickle, split
it into ``--num_batch`` contiguous batches, run every batch through the
sharded model on all GPUs (threads; DP = ``np.array_split`` of prompts, MP =
the same list on every GPU), then ``--num_gen_token`` times extend every
suffix with the greedy argmax token (re-running the whole model each time),
and finally dump ``<prompts>_updated.pkl`` and the score list.

Here >1 GPU means >1 process (spawned by :func:`main` or launched by
``torchrun``), RCCL between them, and every rank runs the same loop; rank 0
owns the file I/O.
"""
from __future__ import annotations

import copy
import json
import os
import pickle
import socket
import sys
import tempfile
import time
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import knobs
from .config import MAX_TOKEN_LEN, ModelConfig
from .engine import ShardedRunner
from .parallel.comm import Comm
from .parallel.planner import make_plan
from .runtime.stream import FileLayerSource
from .runtime.weights import HostStore
from .utils.cli import parse_args
from .utils.tokenizer import load_tokenizer


def batch_ranges(n: int, num_batch: int):
    """main.py:19-20 (contiguous batches; the last one takes the remainder)."""
    ends = [n // num_batch * i for i in range(1, num_batch)] + [n]
    return list(zip([0] + ends[:-1], ends))


def resolve_weight_cache(args, cfg: ModelConfig, comm: Comm, names: Sequence[str], sliced: bool) -> str:
    """``--weight_cache`` -> ``host`` or ``stream``.

    ``auto`` pins the packed layers in host RAM only when they fit the host budget
    (``--host_mem_gb``, default 80% of MemAvailable shared by this node's ranks), and
    otherwise streams them from the layer files every pass — the reference's small-RAM mode
    (README: 70B with >= 8 GB RAM).  ``disk`` is the reference-named alias of ``stream``.
    An explicit ``host`` that cannot fit is rejected instead of being OOM-killed mid-load
    (e.g. ``--dp_weight_shard false`` would pin the whole model once per rank)."""
    from .models.layout import layer_kind, layer_layout
    from .runtime.stream import host_ram_available
    from .runtime.weights import piece_slices
    mode = getattr(args, "weight_cache", "auto")
    if getattr(args, "synthetic", None):
        return "host"                  # generated in host RAM; there are no files to stream
    if mode in ("disk", "stream"):
        return "stream"
    need = 0
    for n in names:
        lay = layer_layout(cfg, layer_kind(n))
        need += sum(p.chunk for p in piece_slices(lay, comm.world)) if sliced else lay.nbytes
    local = int(os.environ.get("LOCAL_WORLD_SIZE", comm.world))
    if getattr(args, "host_mem_gb", None):
        budget = int(args.host_mem_gb * 1e9) // max(1, local)
    else:
        budget = int(0.8 * host_ram_available()) // max(1, local)
    fits = budget <= 0 or need <= budget            # unknown RAM size: trust the user
    if mode == "host":
        if not fits:
            raise SystemExit(f"--weight_cache host needs {need / 1e9:.1f} GB of pinned RAM per rank, the budget "
                             f"is {budget / 1e9:.1f} GB: use --weight_cache stream (or auto)")
        return "host"
    return "host" if fits else "stream"


def build_source(args, cfg: ModelConfig, comm: Comm, device: torch.device):
    names = cfg.layer_names()
    plan = make_plan(len(names), args.layer_num_per_shard, comm.world, comm.rank, args.data_parallel,
                     getattr(args, "pipeline_stages", "round_robin"))
    mine = [names[i] for i in sorted({i for sh in plan.my_shards for i in sh})]
    # GPU: host-cached weights are kept with their RMSNorms folded into the projections (once, on
    # the device), which the fused-norm GEMMs read as they are (HostStore.fold_norms)
    fold = device.type == "cuda" and knobs.get_int("FLS_QKV_FOLD") == 1
    if getattr(args, "synthetic", None):
        return HostStore.synthetic(cfg, device, seed=0, pinned=device.type == "cuda", names=mine, fold_norms=fold)
    src = FileLayerSource(cfg, args.model_path, names=mine, direct=getattr(args, "o_direct", False))
    if resolve_weight_cache(args, cfg, comm, mine, sliced=False) == "stream":
        return src
    st = HostStore.from_source(src, pinned=device.type == "cuda", names=mine)
    return st.fold_norms(device) if fold else st


def repeated_passes(args) -> bool:
    """The same weights stream more than once per run (reference: every generation step and every
    batch re-streams the whole model, ``main.py:19-23,65-76``)."""
    return getattr(args, "num_gen_token", 1) > 1 or getattr(args, "num_batch", 1) > 1


def resolve_prefix_kv_cache(args) -> bool:
    """``--prefix_kv_cache auto``: on for greedy generation (exact: later steps re-score the same
    prefixes, runtime/prefix_cache.py).  Under ``--max_vram_gb`` the cache lives in pinned host
    memory (host mode: a staging buffer of one layer's K/V in HBM, planned by runtime/memplan.py);
    ``build_runner`` turns an auto cache off when the host lacks the memory for it."""
    v = getattr(args, "prefix_kv_cache", False)
    if v == "auto":
        return getattr(args, "num_gen_token", 1) > 1 and not getattr(args, "resume_dir", None)
    return bool(v)


# host mode may take at most this share of the host's available memory
HOST_KV_SHARE = 0.5


def host_kv_fits(nbytes: int) -> bool:
    import psutil
    return nbytes <= HOST_KV_SHARE * psutil.virtual_memory().available


def resolve_suffix_kv_cache(args, world: int = 1) -> bool:
    """``--suffix_kv_cache auto``: on whenever the prefix K/V cache is, on one rank, without a VRAM
    cap.  Under ``--max_vram_gb`` the caches live in host memory and a step is PCIe-bound (weights +
    staged K/V): the suffix regions add more bytes per step than recomputing the suffix tokens costs
    (70B, 32 prompts: 2.93 s per step with reuse against 2.84 s prefix-only, same tokens,
    profiles/r6_decode), so auto keeps the prefix cache only."""
    v = getattr(args, "suffix_kv_cache", False)
    if v == "auto":
        return resolve_prefix_kv_cache(args) and world == 1 and not getattr(args, "max_vram_gb", None)
    return bool(v)


def prefix_kv_bytes(cfg: ModelConfig, tok, prompts, n_decoders: int, elem: int = 2,
                    suffix_kv_cache: bool = False, growth: Optional[int] = None) -> int:
    """HBM the prefix K/V cache needs for ``prompts``: post-RoPE K and V of every prefix token, and
    with ``suffix_kv_cache`` every suffix's region too (its tokens + ``growth`` rows, default
    ``PrefixKVCache.SUFFIX_GROWTH``, as ``PrefixKVCache.begin`` sizes them), for every decoder layer
    this rank runs."""
    if tok is None or not prompts:
        return 0
    from .runtime.prefix_cache import PrefixKVCache
    n = sum(len(tok(p[0]).input_ids) for p in prompts)
    if suffix_kv_cache:
        for p in prompts:
            sfx = list(p[1])
            if sfx:
                g = PrefixKVCache.SUFFIX_GROWTH if growth is None else growth
                n += sum(len(ids) + g for ids in tok(sfx).input_ids)
    return n * 2 * cfg.num_key_value_heads * cfg.head_dim * elem * n_decoders


def auto_hbm_cache_bytes(args, cfg: ModelConfig, device: torch.device, reserve: int = 0,
                         n_slots: int = 3) -> int:
    """Free HBM minus this run's activation plan (weight slots, one micro-batch's activations and
    workspace, ``reserve`` — e.g. the prefix K/V cache — and a 4 GB margin)."""
    if device.type != "cuda":
        return 0
    from .runtime.memplan import DEVICE_OVERHEAD, activation_bytes, weight_slot_bytes
    free, _ = torch.cuda.mem_get_info(device)
    need = (weight_slot_bytes(cfg, args.layer_num_per_shard, n_slots)
            + activation_bytes(cfg, getattr(args, "token_budget", 49152), 16384)
            + DEVICE_OVERHEAD + reserve + int(4e9))
    return max(0, free - need)


def resolve_hbm_cache_gb(args, cfg: ModelConfig, device: torch.device, reserve: int = 0) -> float:
    """``--hbm_cache_gb auto``: repeated passes keep as many shards in HBM as fit (the 70B model
    in full on one MI355X, so only the first pass crosses PCIe); a single pass caches nothing."""
    v = getattr(args, "hbm_cache_gb", 0.0)
    if v != "auto":
        return float(v or 0.0)
    if (device.type != "cuda" or not repeated_passes(args) or getattr(args, "resident", False)
            or getattr(args, "max_vram_gb", None) or getattr(args, "resume_dir", None)):
        return 0.0
    return auto_hbm_cache_bytes(args, cfg, device, reserve) / 1e9


def build_runner(args, cfg: ModelConfig, device, comm: Comm, tok, prompts=None) -> ShardedRunner:
    device = torch.device(device)
    from .models.layout import layer_kind
    pkv = resolve_prefix_kv_cache(args)
    skv = resolve_suffix_kv_cache(args, comm.world) and pkv
    n_dec = sum(1 for n in cfg.layer_names() if layer_kind(n) == "decoder")
    if not args.data_parallel and comm.world > 1:
        n_dec = -(-n_dec // comm.world)
    from .runtime.prefix_cache import suffix_growth
    growth = suffix_growth(getattr(args, "num_gen_token", 1))
    reserve = prefix_kv_bytes(cfg, tok, prompts, n_dec, suffix_kv_cache=skv, growth=growth) if pkv else 0
    if pkv and getattr(args, "max_vram_gb", None) and not host_kv_fits(reserve):
        # host mode (a VRAM cap): the cache's pinned host buffers
        msg = (f"the prefix K/V cache needs {reserve / 1e9:.1f} GB of pinned host memory (--max_vram_gb "
               f"keeps it on the host): more than {HOST_KV_SHARE:.0%} of the available memory")
        if getattr(args, "prefix_kv_cache", False) != "auto":
            raise ValueError(msg)
        print(msg + "; running without it", file=sys.stderr)
        pkv = skv = False
        reserve = 0
    if args.data_parallel and comm.world > 1 and args.dp_weight_shard:
        from .parallel.data_parallel import build_dp_sharded_runner
        hv = getattr(args, "hbm_cache_gb", 0.0)
        if hv not in ("auto", 0, 0.0, None):
            print("--hbm_cache_gb is not used with the data-parallel all-gather weight path", file=sys.stderr)
        if hv == "auto" and not args.resident and device.type == "cuda" and repeated_passes(args):
            # repeated passes: gather every layer once and keep it (resident) when the model fits
            from .models.layout import layer_layout
            model = sum(layer_layout(cfg, layer_kind(n)).nbytes for n in cfg.layer_names())
            if model <= auto_hbm_cache_bytes(args, cfg, device, reserve, n_slots=0):
                args = copy.copy(args)
                args.resident = True
        wc = resolve_weight_cache(args, cfg, comm, cfg.layer_names(), sliced=True)
        return build_dp_sharded_runner(args, cfg, device, comm, tok, weight_cache=wc, prefix_kv_cache=pkv)
    src = build_source(args, cfg, comm, device)
    act = None
    if args.dtype:
        act = torch.float16 if args.dtype == "float16" else torch.float32
    return ShardedRunner(cfg, src, device, tok, layer_num_per_shard=args.layer_num_per_shard,
                         storage_location=args.storage_location, disk_folder=args.disk_folder,
                         max_activation_in_cpu=args.max_activation_in_cpu,
                         prefix_attention=args.prefix_attention, token_budget=args.token_budget,
                         resident=args.resident, comm=comm, data_parallel=args.data_parallel,
                         act_dtype=act, verbose=args.verbose,
                         resume_dir=getattr(args, "resume_dir", None),
                         checkpoint_every=getattr(args, "checkpoint_every", 0),
                         max_token_len=getattr(args, "max_token_len", None) or MAX_TOKEN_LEN,
                         hip_graphs=getattr(args, "hip_graphs", False),
                         hbm_cache_gb=resolve_hbm_cache_gb(args, cfg, device, reserve),
                         prefix_kv_cache=pkv,
                         prefix_cache_entries=getattr(args, "prefix_cache_entries", 8),
                         suffix_kv_cache=skv, exact_reuse=getattr(args, "exact_reuse", True),
                         pipeline_stages=getattr(args, "pipeline_stages", "round_robin"),
                         rx_window=getattr(args, "rx_window", 2),
                         max_vram_gb=getattr(args, "max_vram_gb", None))


def load_model_meta(args):
    """(config, tokenizer) from --model_path, or a preset + synthetic tokenizer for --synthetic."""
    if getattr(args, "synthetic", None):
        from .config import preset
        from .utils.tokenizer import write_synthetic_tokenizer
        cfg = preset(args.synthetic)
        tok_dir = os.path.join(tempfile.gettempdir(), f"fls_synth_tok_{cfg.vocab_size}_{os.getpid()}")
        write_synthetic_tokenizer(tok_dir, cfg.vocab_size)
        return cfg, load_tokenizer(tok_dir)
    return ModelConfig.from_pretrained(args.model_path), load_tokenizer(args.model_path)


def run_all(args, runner: ShardedRunner, comm: Comm, prompts: Sequence) -> List[np.ndarray]:
    """One full pass over ``prompts`` on every rank; returns the ordered score list on rank 0."""
    if args.data_parallel and comm.world > 1:
        idx = np.array_split(np.arange(len(prompts)), comm.world)[comm.rank]
        mine = [prompts[i] for i in idx]
    else:
        mine = list(prompts)
    if not prompts:
        return []
    # data parallel with all-gathered weights: every rank runs num_batch passes, even over an
    # empty slice, so the weight collectives line up across ranks
    collective = getattr(runner.prefetcher, "collective", False)
    outs: List[np.ndarray] = []
    for b0, b1 in batch_ranges(len(mine), args.num_batch):
        if b1 > b0 or collective:
            outs += runner(mine[b0:b1])
    if comm.world == 1:
        return outs
    allv = comm.gather_scores(outs, dst=0)
    if comm.rank != 0:
        return []
    if args.data_parallel:
        return sum(allv, [])
    # model parallel: the rank owning lm_head holds every score
    for v in allv:
        if v and all(x is not None for x in v):
            return v
    raise RuntimeError("no rank produced scores")


def generation_loop(args, runner, comm: Comm, tok, original_prompts: Sequence, step_times: Optional[list] = None):
    """main.py:63-90 — greedy extension of every suffix, one full pass per step (the prefix K/V
    cache and the HBM weight cache, on by default for repeated passes, make the later passes
    cheaper; the scores are the same).  ``step_times`` collects each step's wall time."""
    input_prompts = copy.deepcopy(list(original_prompts))
    # per prompt: every step's [n_s, 1, V] scores and argmax tokens.  The reference concatenates the
    # scores each step and takes the argmax over all of them (main.py:83-88); the argmax of the
    # earlier steps cannot change, so each step's is taken once, and the scores are concatenated
    # once at the end — same tokens, same output
    step_scores: List[List[np.ndarray]] = []
    step_tokens: List[List[np.ndarray]] = []
    # host-side profile of chosen steps (FLS_PROFILE_GEN_STEPS="2,3" -> cProfile stats in
    # gen_profile.<step>): where a generation step's host time goes
    prof_steps = {int(s) for s in knobs.get("FLS_PROFILE_GEN_STEPS").split(",") if s.strip()}
    # one runner call per step on one rank: each decode-graphed step may enqueue the next one behind
    # itself (ShardedRunner._launch_spec) while the host decodes and re-tokenizes
    spec = comm.world == 1 and len(batch_ranges(len(input_prompts), args.num_batch)) == 1
    pc = getattr(runner, "prefix_cache", None)
    if pc is not None:
        from .runtime.prefix_cache import suffix_growth
        pc.suffix_growth = suffix_growth(args.num_gen_token)      # suffix regions sized for this run
    for i_new in range(args.num_gen_token):
        t_step = time.perf_counter()
        if hasattr(runner, "spec_steps"):
            runner.spec_steps = (args.num_gen_token - 1 - i_new) if spec else 0
        prof = None
        if i_new in prof_steps:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        outputs = run_all(args, runner, comm, input_prompts)
        # the greedy tokens the runner took on the device (one rank holding every prompt), else a
        # host argmax over the gathered scores
        dev_tok = getattr(runner, "last_tokens", None) if comm.world == 1 else None
        if not dev_tok or len(dev_tok) != len(outputs) or any(t is None for t in dev_tok):
            dev_tok = None
        if prof is not None:
            prof.disable()
            prof.dump_stats(f"gen_profile.{i_new}")
        if comm.rank == 0:
            toks = dev_tok if dev_tok is not None else [greedy_tokens(o) for o in outputs]
            if i_new == 0:
                step_scores = [[o] for o in outputs]
                step_tokens = [[t] for t in toks]
            else:
                for pi, o in enumerate(outputs):
                    step_scores[pi].append(o)
                    step_tokens[pi].append(toks[pi])
            # s + tok.decode(t) for every suffix (main.py:86-88), the decodes in one batched call
            news = [np.concatenate(step_tokens[pi], axis=1) for pi in range(len(input_prompts))]
            flat = [t for nt in news for t in nt]
            texts = iter(tok.batch_decode(flat) if hasattr(tok, "batch_decode") else [tok.decode(t) for t in flat])
            for pi in range(len(input_prompts)):
                prefix, suffix = original_prompts[pi]
                input_prompts[pi] = (prefix, tuple(s + next(texts) for s in suffix))
        if comm.world > 1:
            input_prompts = comm.broadcast_object(input_prompts, src=0)
        if step_times is not None:
            step_times.append(time.perf_counter() - t_step)
        if getattr(args, "verbose", False) and comm.rank == 0:
            print(f"step {i_new}: {time.perf_counter() - t_step:.3f}s", flush=True)
    output_scores = [ss[0] if len(ss) == 1 else np.concatenate(ss, axis=1) for ss in step_scores]
    return output_scores, input_prompts


def greedy_tokens(scores: np.ndarray) -> np.ndarray:
    """np.argmax(scores, axis=-1) (first index on ties).  fp16 probabilities are >= 0, whose bit
    patterns order like their values: the argmax runs on the uint16 view (numpy has no fast fp16
    compare: ~30x faster at [160, 1, 32000])."""
    if scores.dtype == np.float16:
        bits = scores.view(np.uint16)
        if not (bits >= 0x8000).any():
            return np.argmax(bits, axis=-1)
    return np.argmax(scores, axis=-1)


def _device_for(args, comm: Comm) -> torch.device:
    if comm.world > 1:
        return comm.device
    n = torch.cuda.device_count() if args.num_gpus is None else args.num_gpus
    return torch.device("cuda", 0) if n > 0 and torch.cuda.is_available() else torch.device("cpu")


def run_rank(args, comm: Comm) -> Optional[dict]:
    if getattr(args, "profile", False):
        from .utils import trace
        trace.enable(True)
    device = _device_for(args, comm)
    if args.storage_location == "disk":
        os.makedirs(args.disk_folder, exist_ok=True)
    with open(args.prompt_pickle, "rb") as f:
        original = pickle.load(f)      # the user's own prompt file (reference format)
    cfg, tok = load_model_meta(args)
    t0 = time.perf_counter()
    runner = build_runner(args, cfg, device, comm, tok, original)
    t_build = time.perf_counter() - t0
    t1 = time.perf_counter()
    step_times: List[float] = []
    scores, updated = generation_loop(args, runner, comm, tok, original, step_times)
    t_run = time.perf_counter() - t1
    tokens = comm.all_reduce_sum(runner.stats.get("tokens", 0.0)) if not (
        comm.world > 1 and not args.data_parallel) else runner.stats.get("tokens", 0.0)
    metrics = {"device": str(device), "world": comm.world, "build_s": t_build, "run_s": t_run,
               "step_s": step_times, "tokens_last_pass": tokens, "stats": runner.stats,
               "hbm_cache_kept_shards": len(getattr(runner.prefetcher, "_sticky", ())),
               "prefix_kv_cache": runner.prefix_cache is not None}
    if device.type == "cuda":
        metrics["peak_hbm_bytes"] = torch.cuda.max_memory_allocated(device)
    if comm.rank == 0:
        if args.data_parallel and comm.world > 1:
            updated = np.array(updated, dtype=object)   # reference quirk: main.py:69 makes it an ndarray
        with open(args.prompt_pickle.replace(".pkl", "_updated.pkl"), "wb") as f:
            pickle.dump(updated, f)
        with open(args.output_file, "wb") as f:
            pickle.dump(scores, f)
        if args.verbose:
            print(json.dumps(metrics, default=float))
        if args.metrics_json:
            with open(args.metrics_json, "w") as f:
                json.dump(metrics, f, default=float, indent=1)
    runner.close()
    return metrics


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn_worker(local_rank: int, world: int, port: int, argv: List[str]):
    os.environ.update({"RANK": str(local_rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    args = parse_args(argv)
    comm = Comm.from_env("cuda")
    try:
        run_rank(args, comm)
    finally:
        comm.destroy()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    print(args)
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        comm = Comm.from_env("cuda" if torch.cuda.device_count() > 0 else "cpu")
        try:
            run_rank(args, comm)
        finally:
            comm.destroy()
        return 0
    n = torch.cuda.device_count() if args.num_gpus is None else args.num_gpus
    if n > 1:
        import torch.multiprocessing as mp
        port = _free_port()
        mp.start_processes(_spawn_worker, args=(n, port, argv), nprocs=n, start_method="spawn", join=True)
        return 0
    run_rank(args, Comm(0, 1))
    return 0
