"""Greedy generation (--num_gen_token) with and without the prefix K/V cache.

The reference re-runs the whole model for every generated token
(``/root/reference/main.py:63-90``).  With ``--prefix_kv_cache`` every step
after the first computes only the suffix tokens.  Same synthetic setup as
bench.py (random-init weights in pinned host RAM, lnps=1 streaming).

    python scripts/gen_bench.py [--model llama2-70b] [--gen 4] [--prompts 32] [--json out.json]
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


class _TimedRunner:
    def __init__(self, r):
        self.r, self.times, self.tokens = r, [], []

    def __call__(self, prompts):
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = self.r(prompts)
        torch.cuda.synchronize()
        self.times.append(time.perf_counter() - t)
        self.tokens.append(self.r.stats["tokens"])
        return out

    def __getattr__(self, name):          # run_all reads the runner's prefetcher / plan
        return getattr(self.r, name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-70b")
    ap.add_argument("--gen", type=int, default=4)
    ap.add_argument("--prompts", type=int, default=32)
    ap.add_argument("--prefix-len", type=int, default=1024)
    ap.add_argument("--suffix-len", type=int, default=64)
    ap.add_argument("--resident", action="store_true", help="weights resident in HBM (288 GB holds 70B)")
    ap.add_argument("--token-budget", type=int, default=49152)
    ap.add_argument("--hbm-cache-gb", type=float, default=0.0, help="layers kept resident in HBM, the rest streamed")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = preset(a.model)
    store = HostStore.synthetic(cfg, dev, seed=0, fold_norms=True)
    tok_dir = f"/tmp/fls_gen_tok_{os.getpid()}"
    write_synthetic_tokenizer(tok_dir, cfg.vocab_size)
    tok = load_tokenizer(tok_dir)
    prompts = synthetic_prompts(a.prompts, a.prefix_len, 5, a.suffix_len, cfg.vocab_size, seed=0)
    args = argparse.Namespace(num_gen_token=a.gen, data_parallel=False, num_batch=1)
    res = {"model": a.model, "prompts": a.prompts, "prefix_len": a.prefix_len, "suffix_len": a.suffix_len,
           "num_gen_token": a.gen, "layer_num_per_shard": 1, "storage_location": "cpu",
           "resident": a.resident, "token_budget": a.token_budget, "hbm_cache_gb": a.hbm_cache_gb}
    scores = {}
    for name, pkv in (("rerun", False), ("prefix_kv_cache", True)):
        r = ShardedRunner(cfg, store, dev, tok, layer_num_per_shard=1, storage_location="cpu",
                          prefix_kv_cache=pkv, resident=a.resident, token_budget=a.token_budget,
                          hbm_cache_gb=a.hbm_cache_gb)
        tr = _TimedRunner(r)
        t = time.perf_counter()
        s, _ = generation_loop(args, tr, Comm(0, 1, dev), tok, prompts)
        total = time.perf_counter() - t
        scores[name] = s
        res.setdefault("non_finite", {})[name] = [int((~np.isfinite(x.astype(np.float32))).sum()) for x in s]
        res[name] = {"total_s": round(total, 3), "step_s": [round(x, 3) for x in tr.times],
                     "computed_tokens": tr.tokens, "peak_hbm_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)}
        if pkv:
            res[name]["cache_gb"] = round(r.prefix_cache.nbytes / 1e9, 2)
        print(json.dumps({name: res[name]}), flush=True)
        r.close()
        del r, tr
        gc.collect()
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats(dev)
    res["max_abs_diff"] = float(max(np.abs(x.astype(np.float32) - y.astype(np.float32)).max()
                                    for x, y in zip(scores["rerun"], scores["prefix_kv_cache"])))
    res["speedup"] = round(res["rerun"]["total_s"] / res["prefix_kv_cache"]["total_s"], 3)
    print(json.dumps({"max_abs_diff": res["max_abs_diff"], "speedup": res["speedup"],
                      "non_finite": res["non_finite"]}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
