"""Generation with suffix K/V reuse (the default) against the exact generation (--suffix_kv_cache
false), both greedy over the same synthetic prompts, weights resident in HBM: are the scores bitwise
equal at every step (ShardedRunner "exact K/V reuse"), and what does a step cost?

    python scripts/gen_exact_probe.py [--model llama2-70b] [--prompts 64] [--gen 8] [--json out.json]
        [--max-vram-gb 6]     # weights streamed through the piece pool, K/V caches in host memory
"""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.api import generation_loop  # noqa: E402
from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.engine import ShardedRunner  # noqa: E402
from flexible_llm_sharding_amd.parallel.comm import Comm  # noqa: E402
from flexible_llm_sharding_amd.runtime.weights import HostStore  # noqa: E402
from flexible_llm_sharding_amd.utils.synthetic import synthetic_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import load_tokenizer, write_synthetic_tokenizer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-70b")
    ap.add_argument("--gen", type=int, default=8)
    ap.add_argument("--prompts", type=int, default=64)
    ap.add_argument("--prefix-len", type=int, default=1024)
    ap.add_argument("--suffix-len", type=int, default=64)
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None, choices=["exact", "reuse", "fast"], help="one run (a kernel trace)")
    ap.add_argument("--fast", action="store_true",
                    help="also the --exact_reuse false arm (small-M kernels; tokens compared, not guaranteed)")
    ap.add_argument("--max-vram-gb", type=float, default=None)
    ap.add_argument("--mid-bn", type=int, default=0, help="force the mid-M kernel's block columns (64 / 128; A/B)")
    ap.add_argument("--mid-waves", type=int, default=0, help="force the 128-column mid blocks' waves (4 / 8; A/B)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    if a.mid_bn or a.mid_waves:
        from flexible_llm_sharding_amd import _native
        _native.kernels().fls_gemm_set_mid_bn(a.mid_bn)
        _native.kernels().fls_gemm_set_mid_waves(a.mid_waves)
    cfg = preset(a.model)
    store = HostStore.synthetic(cfg, dev, seed=0, fold_norms=True)
    tok_dir = f"/tmp/fls_probe_tok_{os.getpid()}"
    write_synthetic_tokenizer(tok_dir, cfg.vocab_size)
    tok = load_tokenizer(tok_dir)
    prompts = synthetic_prompts(a.prompts, a.prefix_len, 5, a.suffix_len, cfg.vocab_size, seed=0)
    args = argparse.Namespace(num_gen_token=a.gen, data_parallel=False, num_batch=1)
    res = {"model": a.model, "prompts": a.prompts, "prefix_len": a.prefix_len, "suffix_len": a.suffix_len,
           "mid_bn": a.mid_bn or "auto", "mid_waves": a.mid_waves or "auto",
           "num_gen_token": a.gen,
           "weights": f"streamed, --max_vram_gb {a.max_vram_gb}" if a.max_vram_gb else "resident in HBM"}
    runs = {}
    arms = [("exact", False, True), ("reuse", True, True)] + ([("fast", True, False)] if a.fast or a.only == "fast" else [])
    for name, sfx, exact_reuse in arms:
        if a.only and name != a.only:
            continue
        kw = {"max_vram_gb": a.max_vram_gb} if a.max_vram_gb else {"resident": True}
        r = ShardedRunner(cfg, store, dev, tok, layer_num_per_shard=1, prefix_kv_cache=True, suffix_kv_cache=sfx,
                          exact_reuse=exact_reuse, **kw)
        step_s = []
        sampler = None
        if a.max_vram_gb:
            from bench import DeviceSampler          # hipMemGetInfo sampled every 2 ms
            sampler = DeviceSampler(dev)
        t = time.perf_counter()
        s, u = generation_loop(args, r, Comm(0, 1, dev), tok, prompts, step_s)
        runs[name] = (s, u)
        res[name] = {"total_s": round(time.perf_counter() - t, 3), "step_s": [round(x, 4) for x in step_s],
                     "later_step_s_median": round(float(np.median(step_s[1:])), 4) if len(step_s) > 1 else None}
        if sfx:
            res[name]["speculative_dropped"] = r.spec_dropped
            res[name]["last_step_stats"] = {k: r.stats.get(k) for k in ("tokens", "suffix_tokens_reused",
                                                                         "speculative", "graph_replays")}
        pc = r.prefix_cache
        if pc.host:
            res[name]["host_kv"] = {"host_gb": round(pc.nbytes / 1e9, 2), "staging_gb": round(pc.stage.nbytes / 1e9, 3),
                                    "h2d_gb": round(pc.stage.bytes_h2d / 1e9, 2),
                                    "d2h_gb": round(pc.stage.bytes_d2h / 1e9, 2),
                                    "direct_gb": round(pc.stage.bytes_direct / 1e9, 3)}
        if a.max_vram_gb:
            from flexible_llm_sharding_amd.runtime.memplan import device_used_bytes
            res[name]["device_used_gb_end"] = round(device_used_bytes(dev) / 1e9, 3)
            res[name]["peak_device_used_gb"] = round(sampler.stop()[0] / 1e9, 3)
            res[name]["max_reserved_gb"] = round(torch.cuda.max_memory_reserved(dev) / 1e9, 3)
            res[name]["vram_plan"] = r.vram_plan
        print(json.dumps({name: res[name]}), flush=True)
        r.close()
        del r
        gc.collect()
        torch.cuda.empty_cache()
    if a.only:
        return
    (s0, u0), (s1, u1) = runs["exact"], runs["reuse"]
    res["tokens_equal"] = bool(u0 == u1)
    res["scores_bitwise_equal"] = bool(all(np.array_equal(x, y) for x, y in zip(s0, s1)))
    res["max_abs_diff_scores"] = float(max(np.abs(x.astype(np.float32) - y.astype(np.float32)).max()
                                           for x, y in zip(s0, s1)))
    res["steps_speedup_later"] = round(res["exact"]["later_step_s_median"] / res["reuse"]["later_step_s_median"], 2)
    keys = ["tokens_equal", "scores_bitwise_equal", "max_abs_diff_scores", "steps_speedup_later"]
    if "fast" in runs:
        s2, u2 = runs["fast"]
        res["fast_tokens_equal"] = bool(u0 == u2)
        res["fast_max_abs_diff_scores"] = float(max(np.abs(x.astype(np.float32) - y.astype(np.float32)).max()
                                                    for x, y in zip(s0, s2)))
        keys += ["fast_tokens_equal", "fast_max_abs_diff_scores"]
    print(json.dumps({k: res[k] for k in keys}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
