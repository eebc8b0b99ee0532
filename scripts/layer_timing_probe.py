"""Per-layer GPU timeline of one capped 70B pass (no profiler): CUDA events around every
``run_layer`` call on the compute stream, so the time of each (layer, micro-batch) compute — any
stream waits inside it included — and the gaps between consecutive computes (weight acquire,
activation reloads, host) can be compared between runner configurations without rocprofv3's copy
substitutions.

    python scripts/layer_timing_probe.py --token-budget 16384 [--max-vram-gb 6] [--steps 2]
    FLS_PIECE_POOL=0 python scripts/layer_timing_probe.py --token-budget 16384
"""
import argparse
import os
import sys
import time
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import flexible_llm_sharding_amd.engine as eng  # noqa: E402
from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.runtime.weights import HostStore  # noqa: E402
from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, write_synthetic_tokenizer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--token-budget", type=int, default=49152)
    ap.add_argument("--max-vram-gb", type=float, default=6.0)
    ap.add_argument("--prompts", type=int, default=32)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = preset("llama2-70b")
    store = HostStore.synthetic(cfg, dev, seed=0, pinned=True, fold_norms=True)
    torch.cuda.empty_cache()
    write_synthetic_tokenizer("/tmp/fls_probe_tok", cfg.vocab_size)
    tok = load_tokenizer("/tmp/fls_probe_tok")
    prompts = synthetic_prompts(a.prompts, 1024, 5, 64, cfg.vocab_size, seed=0)
    r = eng.ShardedRunner(cfg, store, dev, tok, layer_num_per_shard=1, storage_location="cpu",
                          token_budget=a.token_budget, max_vram_gb=a.max_vram_gb or None)
    rec = []
    orig = eng.run_layer

    def timed(ctx, name, W, state, batch, meta):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = orig(ctx, name, W, state, batch, meta)
        e1.record()
        rec.append((name, batch.num_tokens, e0, e1))
        return out

    eng.run_layer = timed
    # host time in the calls that may block: prefetcher issue / wait, activation store, event syncs
    host = defaultdict(float)

    def wrap(obj, attr, tag):
        f = getattr(obj, attr)

        def g(*a_, **k_):
            t = time.perf_counter()
            try:
                return f(*a_, **k_)
            finally:
                host[tag] += time.perf_counter() - t
        setattr(obj, attr, g)
    from flexible_llm_sharding_amd.runtime import activations, prefetch
    for cls in (prefetch.PiecePoolPrefetcher, prefetch.ShardPrefetcher):
        for name in ("_try_issue", "_wait", "acquire", "release", "prefetch"):
            if name in cls.__dict__:
                wrap(cls, name, f"{cls.__name__}.{name}")
    for name in ("get", "put", "prefetch"):
        wrap(activations.ActivationStore, name, f"ActivationStore.{name}")
    wrap(activations.ActRing, "acquire", "ActRing.acquire")
    wrap(torch.cuda.Event, "synchronize", "Event.synchronize")
    wrap(eng.ShardedRunner, "_throttle", "_throttle")
    host_in_layer = defaultdict(float)
    orig2 = eng.run_layer

    def timed2(ctx, name, W, state, batch, meta):
        t = time.perf_counter()
        try:
            return orig2(ctx, name, W, state, batch, meta)
        finally:
            host_in_layer[batch.num_tokens] += time.perf_counter() - t
    eng.run_layer = timed2
    r(prompts)                                     # warmup
    for step in range(a.steps):
        rec.clear()
        host.clear()
        host_in_layer.clear()
        t0 = time.perf_counter()
        r(prompts)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        comp = [e0.elapsed_time(e1) for _, _, e0, e1 in rec]
        gaps = [rec[i][3].elapsed_time(rec[i + 1][2]) for i in range(len(rec) - 1)]
        by_rows = defaultdict(list)
        for (name, rows, _, _), c in zip(rec, comp):
            if name.startswith("model.layers."):
                by_rows[rows].append(c)
        print(f"step {step}: wall {wall * 1e3:.1f} ms, layer computes {sum(comp):.1f} ms, gaps {sum(gaps):.1f} ms "
              f"({len(rec)} computes), plan {r.vram_plan}")
        for rows, cs in sorted(by_rows.items()):
            cs = np.array(cs)
            print(f"    decoder computes of {rows:6d} rows: n {len(cs):3d}  median {np.median(cs):7.2f} ms  "
                  f"p90 {np.percentile(cs, 90):7.2f}  max {cs.max():7.2f}  sum {cs.sum():8.1f}")
        big = [g for g in gaps if g > 1.0]
        print(f"    gaps > 1 ms: {len(big)}, sum {sum(big):.1f} ms; position of each in its layer's item order: "
              + str(sorted({(i + 1 - 1) % max(1, int(r.stats.get('micro_batches', 1))) for i, g in enumerate(gaps) if g > 1.0})))
        top = sorted(range(len(gaps)), key=lambda i: -gaps[i])[:12]
        print("    largest gaps (ms) after -> before:")
        for i in top:
            print(f"      {gaps[i]:7.2f}  #{i} {rec[i][0]}[{rec[i][1]}] -> #{i + 1} {rec[i + 1][0]}[{rec[i + 1][1]}]")
        st = {k: round(v, 3) for k, v in r.stats.items() if "stall" in k or "wait" in k}
        print(f"    stats {st}", flush=True)
        print("    host seconds in: " + ", ".join(f"{k} {v:.3f}" for k, v in sorted(host.items(), key=lambda kv: -kv[1])))
        print("    host seconds enqueuing layers, by micro-batch rows: " +
              ", ".join(f"{k}: {v:.3f}" for k, v in sorted(host_in_layer.items())))
        slow = [(c, rec[i][0], rec[i][1], i) for i, c in enumerate(comp) if rec[i][0].startswith("model.layers.")]
        slow.sort(reverse=True)
        print("    slowest decoder computes (ms, layer, rows, index in pass): " +
              "; ".join(f"{c:.1f} {n}[{rw}] #{i}" for c, n, rw, i in slow[:10]))
    r.close()


if __name__ == "__main__":
    main()
