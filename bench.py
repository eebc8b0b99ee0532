"""Benchmark: tokens/s + peak GPU memory of sharded Llama-2-70B scoring (lnps=1).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
launched by ``torch.distributed.run`` (one rank per GPU, RCCL), or, without a
launcher, this script starts the N rank processes itself (before touching any
GPU) and waits for them.  One *step* is one full pass of the sharded model
over a batch of synthetic (prefix, 5 suffixes) prompts — the reference's
``ShardedLlama.__call__`` (``/root/reference/utils.py:133-305``): every
layer's weights streamed into HBM (layer_num_per_shard=1, double-buffered),
every prompt scored, fp16 probabilities copied back to the host.  Prompts are
synthetic text tokenized inside the timed step by a synthetic tokenizer;
weights are random-init Llama-2-70B (no network, no checkpoint):

* ``--weights host`` (default): generated on the GPU and parked in pinned host
  RAM before timing (138 GB for 70B);
* ``--weights stream``: written once as per-layer safetensors files
  (``--ckpt-dir``; ``--unique-layers K`` hard-links decoder layers >= K to the
  first K so 70B fits a small disk) and re-read from the files on every pass
  through the native streamer's pinned chunk ring (~256 MB of pinned RAM) —
  the reference's small-RAM mode.  ``--o-direct`` bypasses the page cache.

Scaling is weak: each GPU adds ``--prompts-per-gpu`` prompts.  N>1 runs the
data-parallel schedule (each GPU scores its own prompts; every layer is
scatter-loaded 1/N per GPU over its own PCIe link and re-assembled in HBM by
an RCCL all-gather over xGMI), or with ``--mode mp`` the reference's default
model-parallel schedule (shard k on GPU k mod N, RCCL send/recv of
activations; each GPU streams only its own shards).

Memory is reported as measured: ``peak_gpu_mem_gb`` (allocator high-water),
``peak_device_used_gb`` (``hipMemGetInfo`` total - free sampled every 10 ms by a thread during every
step: context, code objects, RCCL buffers and allocator slack included),
``host_pinned_gb`` and ``host_peak_rss_gb``.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

METRIC = "tokens/sec + peak GPU mem, Llama-2-70B layer_num_per_shard=1 at 1/2/4/8 MI355X"


class DeviceSampler:
    """hipMemGetInfo (total - free) sampled every ``period_s`` (2 ms) by a thread for the whole run —
    warmup and timed steps, inside the passes, not only at step boundaries."""

    def __init__(self, dev, period_s: float = 0.002):
        import threading

        import torch
        self.dev, self.period, self.peak, self.n = dev, period_s, 0.0, 0
        self.peak_outside = 0.0           # device memory in use outside the caching allocator
        self.rss_peak = 0.0               # this process's resident host memory (warmup + timed steps)
        self._stop = threading.Event()
        page = os.sysconf("SC_PAGE_SIZE")

        def rss():
            try:
                with open("/proc/self/statm") as f:
                    return int(f.read().split()[1]) * page
            except (OSError, ValueError, IndexError):
                return 0

        def run():
            torch.cuda.set_device(dev)
            while not self._stop.is_set():
                free, total = torch.cuda.mem_get_info(dev)
                used = float(total - free)
                self.peak = max(self.peak, used)
                self.peak_outside = max(self.peak_outside, used - torch.cuda.memory_reserved(dev))
                if self.n % 16 == 0:
                    self.rss_peak = max(self.rss_peak, float(rss()))
                self.n += 1
                self._stop.wait(self.period)

        self._t = threading.Thread(target=run, daemon=True)
        self._t.start()

    def stop(self):
        self._stop.set()
        self._t.join()
        return self.peak, self.n, self.peak_outside


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama2-70b")
    ap.add_argument("--num-layers", type=int, default=None, help="override (debug only; result not comparable)")
    ap.add_argument("--prompts-per-gpu", type=int, default=32)
    ap.add_argument("--prefix-len", type=int, default=1024)
    ap.add_argument("--n-suffix", type=int, default=5)
    ap.add_argument("--suffix-len", type=int, default=64)
    ap.add_argument("--lnps", type=int, default=1)
    ap.add_argument("--storage", default="cpu", choices=["gpu", "cpu", "disk"])
    ap.add_argument("--mode", default="auto", choices=["auto", "mp", "dp"])
    ap.add_argument("--stages", default="round_robin", choices=["round_robin", "contiguous"],
                    help="--mode mp: shard k on GPU k mod N (reference) or one contiguous stage per GPU")
    ap.add_argument("--token-budget", type=int, default=49152)
    ap.add_argument("--mlp-chunk", type=int, default=None,
                    help="rows per SwiGLU MLP chunk (default: 16384, MoE models 65536)")
    ap.add_argument("--attn-rows", type=int, default=0,
                    help="attention phase in prompt-aligned groups of <= this many rows (A/B of the --max-vram-gb layout)")
    ap.add_argument("--slots", type=int, default=None, help="HBM weight slots (default 3, 2 under --max-vram-gb; 3 prefetches across call boundaries)")
    ap.add_argument("--max-vram-gb", type=float, default=None,
                    help="HBM cap per GPU (sizes micro-batch / chunks, sub-layer weight streaming). Default: 6 for "
                         "the 70B lnps=1 headline on one GPU (the reference's 70B-in-6-GB envelope, README.md:2; "
                         "BASELINE config 3), none otherwise (e.g. N > 1 data parallel); 0 = no cap")
    ap.add_argument("--resident", action="store_true")
    ap.add_argument("--hbm-cache-gb", type=float, default=0.0,
                    help="keep this many GB of layers resident in HBM, stream the rest (not the headline config)")
    ap.add_argument("--hip-graphs", action="store_true", help="with --resident: whole-forward HIP graph replay")
    ap.add_argument("--no-prune-last", action="store_true",
                    help="compute every row in the last decoder layer (A/B of the scored-rows-only layer)")
    ap.add_argument("--norm-fold", default="prefolded", choices=["on_landing", "prefolded"],
                    help="--weights host: the RMSNorm weights folded into W_qkv / W_gate-up once, into the pinned "
                         "host image, when it is built before timing (default: a load-time transform of the "
                         "host cache, like the dtype cast), or as each layer lands in HBM on every pass (on the "
                         "copy stream, from the checkpoint's own bytes; -1.0%%: profiles/r6_head).  --weights "
                         "stream always folds on landing")
    ap.add_argument("--emulate-dp-fanout", default="none", choices=["none", "blit", "sdma", "cu32"],
                    help="measurement only (1 GPU, piece pool): after each weight piece lands, copy 7/8 of its bytes "
                         "HBM -> HBM on the copy stream, the per-rank traffic of the 8-GPU data-parallel all-gather: "
                         "blit = the HIP runtime's copy kernel, cu32 = a 32-workgroup copy kernel (RCCL-like "
                         "channels), sdma = hipMemcpyDeviceToDeviceNoCU (copy engines, no compute unit)")
    ap.add_argument("--emulate-dp-slice", action="store_true",
                    help="with --emulate-dp-fanout: H2D only a rank's 1/8 of each piece (timing only: stale weights)")
    ap.add_argument("--prefix-attention", default="bidirectional")
    ap.add_argument("--weights", default="host", choices=["host", "stream"])
    ap.add_argument("--ckpt-dir", default=None, help="--weights stream: layer-file directory (written if absent)")
    ap.add_argument("--ckpt-dtype", default="float16", choices=["float16", "bfloat16"])
    ap.add_argument("--unique-layers", type=int, default=8)
    ap.add_argument("--o-direct", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--cpu", action="store_true", help="CPU/gloo rehearsal of the same code path (tests only)")
    ap.add_argument("--loopback-ranks", type=int, default=0,
                    help="model-parallel rehearsal on ONE device: R pipeline ranks as threads over the loopback "
                         "comm (device copies instead of RCCL), the real StageInbox / program; not a scaling number")
    return ap.parse_args(argv)


def spawn_ranks(a, argv) -> int:
    """--gpus N without a launcher: start N rank processes (children, no exec) and wait."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    try:
        for p in procs:
            rc = max(rc, p.wait())
            if rc:
                break                     # one rank failed: stop the others (no hung collectives)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def loopback_main(a) -> int:
    """--loopback-ranks R: the model-parallel pipeline (round-robin or contiguous stages, the
    per-rank hand-off program, StageInbox ring and parking) with R ranks as threads of this process
    on one device, exchanging activations by device copies (parallel/comm.py LoopbackComm).  Every
    rank computes its own layers on the same GPU, so the rate is the single-GPU rate minus the
    pipeline's overheads: it measures those overheads at full scale, not scaling."""
    import threading

    import torch

    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.parallel.comm import LoopbackComm, LoopbackHub
    from flexible_llm_sharding_amd.parallel.pipeline import simulate_single_queue
    from flexible_llm_sharding_amd.runtime.weights import HostStore
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, write_synthetic_tokenizer
    R = a.loopback_ranks
    dev = torch.device("cpu") if a.cpu else torch.device("cuda", 0)
    if not a.cpu:
        torch.cuda.set_device(dev)
    kw = {} if a.num_layers is None else {"num_hidden_layers": a.num_layers}
    cfg = preset(a.model, **kw)
    t0 = time.perf_counter()
    from flexible_llm_sharding_amd import knobs
    store = HostStore.synthetic(cfg, dev, seed=a.seed, pinned=not a.cpu,
                                fold_norms=not a.cpu and knobs.get_int("FLS_QKV_FOLD") == 1)
    log(0, f"[bench] loopback x{R}: host store {store.total_bytes / 1e9:.1f} GB in {time.perf_counter() - t0:.1f}s")
    if not a.cpu:
        torch.cuda.empty_cache()
    tok_dir = f"/tmp/fls_bench_tok_{os.getpid()}"
    write_synthetic_tokenizer(tok_dir, cfg.vocab_size)
    tok = load_tokenizer(tok_dir)
    prompts = synthetic_prompts(a.prompts_per_gpu, a.prefix_len, a.n_suffix, a.suffix_len, cfg.vocab_size,
                                seed=a.seed)
    hub = LoopbackHub(R, timeout_s=1800)
    res, err = {}, []

    def rank(r):
        try:
            if not a.cpu:
                torch.cuda.set_device(dev)
            comm = LoopbackComm(hub, r, dev)
            run = ShardedRunner(cfg, store, dev, tok, layer_num_per_shard=a.lnps, storage_location=a.storage,
                                disk_folder=f"/tmp/fls_bench_spill_lb{r}", prefix_attention=a.prefix_attention,
                                token_budget=a.token_budget, mlp_chunk=a.mlp_chunk, comm=comm,
                                pipeline_stages=a.stages, max_activation_in_cpu=4)
            for _ in range(a.warmup):
                run(prompts)
            comm.barrier()
            if not a.cpu:
                torch.cuda.synchronize(dev)
            ts = time.perf_counter()
            for _ in range(a.steps):
                out = run(prompts)
            if not a.cpu:
                torch.cuda.synchronize(dev)
            res[r] = (time.perf_counter() - ts, dict(run.stats), out)
            comm.barrier()
            run.close()
        except BaseException as e:  # noqa: BLE001
            err.append(e)
            raise

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(R)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if err:
        raise err[0]
    elapsed = max(v[0] for v in res.values())
    tokens = res[0][1]["tokens"]
    owner = [v[2] for v in res.values() if v[2] and v[2][0] is not None]
    finite = bool(owner) and all(np.isfinite(o.astype(np.float32)).all() for o in owner[0])
    rx = {r: {k: v for k, v in res[r][1].items() if k.startswith("rx_")} for r in range(R)}
    ok, _ = simulate_single_queue({r: hub.log[r] for r in range(R)})
    out = {"metric": "model-parallel rehearsal on one device (loopback ranks; not a scaling number)",
           "value": round(tokens * a.steps / elapsed, 2), "unit": "tokens/s", "n_gpus": 1, "loopback_ranks": R,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1000.0, 2),
           "higher_is_better": True, "scores_finite": finite, "single_queue_replay_ok": ok,
           "micro_batches": res[0][1]["micro_batches"], "rx_stats": rx,
           "config": {"model": a.model, "stages": a.stages, "storage_location": a.storage, "lnps": a.lnps,
                      "tokens_per_step": tokens}}
    print(json.dumps(out), flush=True)
    return 0


def ensure_checkpoint(cfg, d: str, dtype: str, unique: int, rank: int, comm, progress) -> None:
    """Write the synthetic per-layer checkpoint once (rank 0; a marker file makes it reusable)."""
    import torch
    from flexible_llm_sharding_amd.utils.synthetic import write_synthetic_checkpoint
    import hashlib
    tag = hashlib.sha1(json.dumps([cfg.to_dict(), dtype, unique], sort_keys=True, default=str).encode()).hexdigest()[:12]
    marker = os.path.join(d, f".fls_bench_complete_{tag}")
    if rank == 0 and not os.path.exists(marker):
        dev = "cpu" if not torch.cuda.is_available() else torch.device("cuda", torch.cuda.current_device())
        write_synthetic_checkpoint(cfg, d, seed=0, dtype=getattr(torch, dtype), unique_layers=unique,
                                   device=dev, progress=progress)
        open(marker, "w").close()
    comm.barrier()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse(argv)
    if a.loopback_ranks:
        return loopback_main(a)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(a, argv)
    if a.max_vram_gb is None:
        # the headline (70B, lnps=1) runs in the reference's 6 GB envelope at every GPU count: one
        # GPU and data parallel (sub-layer piece pool, all-gathered per piece) alike, so a scaling
        # curve compares one memory configuration
        headline = a.model == "llama2-70b" and a.lnps == 1 and a.num_layers is None
        a.max_vram_gb = 6.0 if (headline and (a.gpus == 1 or a.mode in ("auto", "dp")) and not a.cpu
                                and not a.resident and a.hbm_cache_gb == 0) else 0.0
    a.max_vram_gb = a.max_vram_gb or None
    if a.max_vram_gb and not a.cpu:
        # a VRAM cap: let the caching allocator grow segments in place instead of keeping one
        # rounded block per size class and stream (set before the first HIP allocation)
        for k in ("PYTORCH_HIP_ALLOC_CONF", "PYTORCH_CUDA_ALLOC_CONF"):
            os.environ.setdefault(k, "expandable_segments:True")

    import resource

    import numpy as np
    import torch

    from flexible_llm_sharding_amd.config import preset
    from flexible_llm_sharding_amd.engine import ShardedRunner
    from flexible_llm_sharding_amd.parallel.comm import Comm
    from flexible_llm_sharding_amd.parallel.data_parallel import (AllGatherPiecePool, AllGatherPrefetcher,
                                                                  SlicedHostStore)
    from flexible_llm_sharding_amd.parallel.planner import make_plan
    from flexible_llm_sharding_amd.runtime import hostmem
    from flexible_llm_sharding_amd.runtime.stream import FileLayerSource
    from flexible_llm_sharding_amd.runtime.weights import HostStore
    from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import clear_prefix_ids, load_tokenizer, write_synthetic_tokenizer

    from flexible_llm_sharding_amd import knobs
    # the fused-norm GEMMs read W_qkv / W_gate-up with the RMSNorm weights folded in: once into the
    # pinned host image as it is built, before timing (--norm-fold prefolded, the default:
    # HostStore.fold_norms), or as each layer lands in HBM on every pass, on the copy stream, from the
    # checkpoint's own bytes (--norm-fold on_landing; the layer-file path always does this).  The JSON
    # config says which ("norm_fold")
    fused = not a.cpu and knobs.get_int("FLS_QKV_FOLD") == 1
    fold = fused and a.norm_fold == "prefolded" and a.weights == "host"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    comm = Comm.from_env("cpu" if a.cpu else "cuda")
    rank = comm.rank
    if a.cpu:
        dev = torch.device("cpu")
    else:
        dev = comm.device if world > 1 else torch.device("cuda", 0)
        torch.cuda.set_device(dev)
    sync = (lambda: None) if a.cpu else (lambda: torch.cuda.synchronize(dev))
    mode = a.mode if a.mode != "auto" else ("dp" if world > 1 else "single")
    dp = mode == "dp"

    kw = {} if a.num_layers is None else {"num_hidden_layers": a.num_layers}
    cfg = preset(a.model, **kw)
    names = cfg.layer_names()
    plan = make_plan(len(names), a.lnps, world, rank, dp, a.stages)
    mine = sorted({i for sh in plan.my_shards for i in sh})
    t0 = time.perf_counter()
    prog = lambda i, n: log(rank, f"[bench]   layer {i}/{n} ({time.perf_counter() - t0:.0f}s)") if i % 10 == 0 else None  # noqa: E731
    if a.weights == "stream":
        ckpt = a.ckpt_dir or f"/tmp/fls_bench_ckpt_{a.model}{'' if a.num_layers is None else f'-L{a.num_layers}'}_{a.ckpt_dtype}_u{a.unique_layers}"
        log(rank, f"[bench] per-layer checkpoint {ckpt} (unique decoder layers: {a.unique_layers}) ...")
        ensure_checkpoint(cfg, ckpt, a.ckpt_dtype, a.unique_layers, rank, comm, prog)
        # writing the checkpoint freed GBs of host tensors into glibc's heap; hand them back so the
        # run's resident set (the small-RAM envelope's measure) is the engine's own
        try:
            import ctypes
            ctypes.CDLL("libc.so.6").malloc_trim(0)
        except (OSError, AttributeError):
            pass
        store = FileLayerSource(cfg, ckpt, names=[names[i] for i in mine], direct=a.o_direct)
        data_w = (f"random-init {a.model} weights as per-layer {a.ckpt_dtype} safetensors files "
                  f"({a.unique_layers} distinct decoder layers, the rest hard links), streamed from the files "
                  f"every pass ({'O_DIRECT' if a.o_direct else 'page cache'})")
    else:
        log(rank, f"[bench] generating {len(mine)} random-init {a.model} layers on {dev} -> pinned host ...")
        if dp:
            # scatter-load: this rank keeps 1/G of every layer; layers re-assembled by RCCL all-gather
            store = SlicedHostStore.synthetic(cfg, dev, rank, world, seed=a.seed, names=[names[i] for i in mine],
                                              progress=prog, fold_norms=fold)
        else:
            store = HostStore.synthetic(cfg, dev, seed=a.seed, names=[names[i] for i in mine], progress=prog,
                                        fold_norms=fold)
        log(rank, f"[bench] host store {store.total_bytes / 1e9:.1f} GB in {time.perf_counter() - t0:.1f}s")
        data_w = f"random-init {a.model} weights in {'HBM (resident)' if a.resident else 'pinned host RAM'}"

    if not a.cpu:
        torch.cuda.empty_cache()     # set-up only: the weight generator's staging blocks are not part of a pass
    tok_dir = f"/tmp/fls_bench_tok_{os.getpid()}"
    write_synthetic_tokenizer(tok_dir, cfg.vocab_size)
    tok = load_tokenizer(tok_dir)
    n_prompts = a.prompts_per_gpu * (world if mode == "mp" else 1)
    prompts = synthetic_prompts(n_prompts, a.prefix_len, a.n_suffix, a.suffix_len, cfg.vocab_size,
                                seed=a.seed + (rank if dp else 0))
    def build(cap):
        pf = None
        if dp:
            my = [s for s in plan.my_shards if len(s)]
            if cap and a.lnps == 1 and not a.resident and isinstance(store, SlicedHostStore) and not a.cpu:
                pf = AllGatherPiecePool(store, names, my, dev, comm)       # the 1-GPU memory envelope
            else:
                pf = AllGatherPrefetcher(store, names, my, dev, comm, resident=a.resident)
        return ShardedRunner(cfg, store, dev, tok, layer_num_per_shard=a.lnps, storage_location=a.storage,
                             disk_folder=f"/tmp/fls_bench_spill_{rank}", prefix_attention=a.prefix_attention,
                             token_budget=a.token_budget, mlp_chunk=a.mlp_chunk, resident=a.resident, comm=comm,
                             data_parallel=dp, n_slots=a.slots, hbm_cache_gb=a.hbm_cache_gb,
                             prefetcher=pf, hip_graphs=a.hip_graphs, prune_last_layer=not a.no_prune_last,
                             pipeline_stages=a.stages, max_vram_gb=cap)

    runner, cap_note = None, None
    try:
        runner = build(a.max_vram_gb)
        if a.max_vram_gb:
            runner._plan_call(runner.tokenize(prompts), False)    # the cap must hold this call's plan
        ok = 1.0
    except ValueError as e:
        ok, cap_note = 0.0, str(e)
    if world > 1:
        # every rank takes the same path (the rebuild creates communicators collectively); the
        # capped plan can fail only on multi-GPU boxes, where RCCL's buffers are counted
        ok = comm.all_reduce_min(ok)
    if not ok:
        log(rank, f"[bench] --max-vram-gb {a.max_vram_gb} cannot hold this run ({cap_note or 'another rank'}): "
                  "running uncapped")
        if runner is not None:
            runner.close()
        if not a.cpu:
            torch.cuda.set_per_process_memory_fraction(1.0, dev)
        cap_note = f"--max-vram-gb {a.max_vram_gb} infeasible: {cap_note or 'on another rank'}"
        a.max_vram_gb = None
        runner = build(None)
    if a.attn_rows:
        runner.ctx.attn_rows = a.attn_rows
    if runner.vram_plan:
        log(rank, f"[bench] --max-vram-gb {a.max_vram_gb}: {runner.vram_plan}")
    sampler = DeviceSampler(dev) if not a.cpu else None
    if not a.cpu:
        torch.cuda.reset_peak_memory_stats(dev)

    for i in range(a.warmup):
        tw = time.perf_counter()
        clear_prefix_ids()
        runner(prompts)
        log(rank, f"[bench] warmup {i}: {time.perf_counter() - tw:.2f}s")
        if i == 0 and (a.emulate_dp_fanout != "none" or a.emulate_dp_slice):
            # (after one full pass: every weight slot holds real weights, so a slice-only run computes
            # on stale random weights, not on the zeros of fresh slots -- MFMA power depends on the data)
            # 256 MB of write target (outside the plan: run with --max-vram-gb 6.3)
            mode = {"none": -1, "blit": 0, "sdma": 1, "cu32": 2}[a.emulate_dp_fanout]
            runner.prefetcher.emulate_fanout = (mode, 32, torch.empty(256 << 20, dtype=torch.uint8, device=dev),
                                                a.emulate_dp_slice)
    comm.barrier()
    sync()
    t_start = time.perf_counter()
    outs = None
    for i in range(a.steps):
        ts = time.perf_counter()
        clear_prefix_ids()       # every timed call tokenizes its prompts in full
        outs = runner(prompts)
        log(rank, f"[bench] step {i}: {time.perf_counter() - ts:.2f}s  stats={json.dumps({k: round(v, 3) for k, v in runner.stats.items()})}")
        if i == 0 and runner.vram_plan:
            log(rank, f"[bench] call plan: {runner.vram_plan}")
    sync()
    comm.barrier()
    elapsed = time.perf_counter() - t_start
    dev_used_peak, n_samples, outside_peak = sampler.stop() if sampler is not None else (0.0, 0, 0.0)
    rss_run = sampler.rss_peak if sampler is not None else 0.0
    if not a.cpu:
        ms_ = torch.cuda.memory_stats(dev)
        log(rank, f"[bench] allocator: device mallocs {ms_.get('num_device_alloc')}, "
                  f"retries {ms_.get('num_alloc_retries')}, reserved {ms_.get('reserved_bytes.all.peak', 0) / 1e9:.2f} GB")
    if a.weights == "stream":
        log(rank, f"[bench] streamer: {json.dumps({k: round(v, 3) for k, v in store.stats().items()})}")
    elapsed = comm.all_reduce_max(elapsed)

    tok_step = runner.stats["tokens"]
    padded_step = runner.stats["padded_tokens"]
    if dp:
        tok_step = comm.all_reduce_sum(tok_step)
        padded_step = comm.all_reduce_sum(padded_step)
    # weight slots are exact-size hipMalloc blocks outside the caching allocator: add them back
    slots = 0.0 if a.cpu else float(runner.prefetcher.hbm_bytes())
    peak = comm.all_reduce_max(0.0 if a.cpu else float(torch.cuda.max_memory_allocated(dev)) + slots)
    peak_res = comm.all_reduce_max(0.0 if a.cpu else float(torch.cuda.max_memory_reserved(dev)) + slots)
    dev_used_peak = comm.all_reduce_max(dev_used_peak)
    pinned = hostmem.pinned_peak + (store.pinned_bytes() if a.weights == "stream" else 0)
    pinned = comm.all_reduce_max(float(pinned))
    rss = comm.all_reduce_max(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024.0)
    # every score this rank produced must be a finite probability (guards the timed path's numerics)
    finite = all(np.isfinite(o.astype(np.float32)).all() for o in (outs or []) if o is not None)
    finite = comm.all_reduce_min(1.0 if finite else 0.0) >= 1.0
    # digest of the last step's scores (this rank's, in prompt order): runs of one config under
    # different plans (capped / uncapped, piece pool / slots) must print the same value
    h = hashlib.sha1()
    for o in (outs or []):
        if o is not None:
            h.update(np.ascontiguousarray(o).tobytes())
    digests = comm.all_gather_object(h.hexdigest()[:16])
    # which ranks / devices took part (the process group the collectives actually ran on)
    import torch.distributed as dist
    pg_world = dist.get_world_size() if dist.is_initialized() else 1
    devices = comm.all_gather_object(str(dev) if a.cpu else f"{dev}:{torch.cuda.get_device_properties(dev).name}")
    ms = elapsed / a.steps * 1000.0
    value = tok_step * a.steps / elapsed
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "tokens/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32-cpu-rehearsal" if a.cpu else "fp16",
        "data": f"synthetic prompts (synthetic tokenizer) + {data_w}",
        "peak_gpu_mem_gb": round(peak / 1e9, 3), "peak_gpu_reserved_gb": round(peak_res / 1e9, 3),
        "peak_device_used_gb": round(dev_used_peak / 1e9, 3), "device_mem_samples": n_samples,
        "peak_outside_allocator_gb": round(comm.all_reduce_max(outside_peak) / 1e9, 3),
        "host_pinned_gb": round(pinned / 1e9, 3), "host_peak_rss_gb": round(rss / 1e9, 3),
        # resident memory sampled every ~32 ms through warmup and timed steps (host_peak_rss_gb is
        # the lifetime maximum: it includes building the host store / writing the checkpoint)
        "host_rss_run_peak_gb": round(comm.all_reduce_max(rss_run) / 1e9, 3),
        "scores_finite": finite, "scores_sha1": digests,
        "world": world, "process_group_ranks": pg_world,
        "backend": comm.backend or ("none" if world == 1 else "?"), "rank_devices": devices,
        "config": {"model": a.model if a.num_layers is None else f"{a.model}-L{a.num_layers}",
                   "global_batch": n_prompts * (world if dp else 1),
                   "seq_len": a.prefix_len + a.suffix_len,
                   "prefix_len": a.prefix_len, "n_suffix": a.n_suffix, "suffix_len": a.suffix_len,
                   "tokens_per_step": tok_step, "padded_tokens_per_step": padded_step,
                   "layer_num_per_shard": a.lnps, "storage_location": a.storage,
                   "parallelism": (f"pp{world}-{a.stages.replace('_', '')}" if mode == "mp" else
                                   (f"dp{world}-allgather-weights" if dp else "single")),
                   "weights": a.weights, "resident": a.resident, "hip_graphs": bool(runner.hip_graphs),
                   "token_budget": runner.token_budget, "mlp_chunk": runner.mlp_chunk,
                   "weight_slots": runner.prefetcher.n_slots, "hbm_cache_gb": a.hbm_cache_gb,
                   # where the RMSNorm weights meet W_qkv / W_gate-up ("none": the unfused CPU path)
                   "norm_fold": ("prefolded" if fold else "on_landing") if fused else "none",
                   # the last decoder layer computes only the scored rows (K/V for every token);
                   # tokens/s counts every token either way (--no-prune-last: A/B)
                   "prune_last_layer": not a.no_prune_last,
                   "emulate_dp_fanout": a.emulate_dp_fanout, "emulate_dp_slice": a.emulate_dp_slice,
                   "max_vram_gb": a.max_vram_gb, "cap_fallback": cap_note},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                json.dump(out, f, indent=1)
    runner.close()
    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
