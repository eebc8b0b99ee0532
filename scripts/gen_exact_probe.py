"""Generation with suffix K/V reuse (the default) against the exact generation (--suffix_kv_cache
false), both greedy over the same synthetic prompts, weights resident in HBM: are the scores bitwise
equal at every step (ShardedRunner "exact K/V reuse"), and what does a step cost?

    python scripts/gen_exact_probe.py [--model llama2-70b] [--prompts 64] [--gen 8] [--json out.json]
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
    ap.add_argument("--only", default=None, choices=["exact", "reuse"], help="one run (a kernel trace)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = preset(a.model)
    store = HostStore.synthetic(cfg, dev, seed=0, fold_norms=True)
    tok_dir = f"/tmp/fls_probe_tok_{os.getpid()}"
    write_synthetic_tokenizer(tok_dir, cfg.vocab_size)
    tok = load_tokenizer(tok_dir)
    prompts = synthetic_prompts(a.prompts, a.prefix_len, 5, a.suffix_len, cfg.vocab_size, seed=0)
    args = argparse.Namespace(num_gen_token=a.gen, data_parallel=False, num_batch=1)
    res = {"model": a.model, "prompts": a.prompts, "prefix_len": a.prefix_len, "suffix_len": a.suffix_len,
           "num_gen_token": a.gen, "weights": "resident in HBM"}
    runs = {}
    for name, sfx in (("exact", False), ("reuse", True)):
        if a.only and name != a.only:
            continue
        r = ShardedRunner(cfg, store, dev, tok, layer_num_per_shard=1, prefix_kv_cache=True, suffix_kv_cache=sfx,
                          resident=True)
        step_s = []
        t = time.perf_counter()
        s, u = generation_loop(args, r, Comm(0, 1, dev), tok, prompts, step_s)
        runs[name] = (s, u)
        res[name] = {"total_s": round(time.perf_counter() - t, 3), "step_s": [round(x, 4) for x in step_s],
                     "later_step_s_median": round(float(np.median(step_s[1:])), 4) if len(step_s) > 1 else None}
        if sfx:
            res[name]["speculative_dropped"] = r.spec_dropped
            res[name]["last_step_stats"] = {k: r.stats.get(k) for k in ("tokens", "suffix_tokens_reused",
                                                                         "speculative", "graph_replays")}
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
    print(json.dumps({k: res[k] for k in ("tokens_equal", "scores_bitwise_equal", "max_abs_diff_scores",
                                          "steps_speedup_later")}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
