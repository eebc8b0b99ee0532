"""Generation with suffix K/V reuse + tie guard (the default) against the exact generation
(--suffix_kv_cache false), both greedy over the same synthetic prompts: are the tokens equal, what
does a step cost, and how far do the reused steps' probabilities deviate from the exact ones (the
measurement behind ShardedRunner.TIE_REL).

For each reused step (before the guard replaces anything) and each suffix: the relative deviation
of the reused probabilities of the exact run's top-2 tokens, and whether the reused argmax differs;
the count of suffixes / prompts the guard re-ran at several TIE_REL values.

    python scripts/tie_guard_probe.py [--model llama2-70b] [--prompts 64] [--gen 8] [--json out.json]
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
           "num_gen_token": a.gen, "weights": "resident in HBM", "tie_rel": ShardedRunner.TIE_REL}
    runs = {}
    reused = []                          # per reused step: the outputs before the guard
    for name, sfx in (("exact", False), ("reuse_guard", True)):
        r = ShardedRunner(cfg, store, dev, tok, layer_num_per_shard=1, prefix_kv_cache=True, suffix_kv_cache=sfx,
                          resident=True)
        step_s, guard = [], []
        if sfx:
            orig = r._tie_guard

            def spy(tps, outputs, orig=orig, r=r):
                reused.append([None if o is None else o.copy() for o in outputs])
                out = orig(tps, outputs)
                guard.append((r.stats["tie_guard_prompts"], round(r.stats["tie_guard_s"], 4)))
                return out
            r._tie_guard = spy
        t = time.perf_counter()
        s, u = generation_loop(args, r, Comm(0, 1, dev), tok, prompts, step_s)
        runs[name] = (s, u)
        res[name] = {"total_s": round(time.perf_counter() - t, 3), "step_s": [round(x, 4) for x in step_s],
                     "later_step_s_median": round(float(np.median(step_s[1:])), 4) if len(step_s) > 1 else None}
        if sfx:
            res[name]["guard_reruns_per_step"] = [g[0] for g in guard]
            res[name]["guard_s_per_step"] = [g[1] for g in guard]
            res[name]["speculative_dropped"] = r.spec_dropped
        print(json.dumps({name: res[name]}), flush=True)
        r.close()
        del r
        gc.collect()
        torch.cuda.empty_cache()
    (s0, u0), (s1, u1) = runs["exact"], runs["reuse_guard"]
    res["tokens_equal"] = bool(u0 == u1)
    res["prompts_with_equal_tokens"] = int(sum(x == y for x, y in zip(u0, u1)))
    res["max_abs_diff_scores"] = float(max(np.abs(x.astype(np.float32) - y.astype(np.float32)).max()
                                           for x, y in zip(s0, s1)))
    # deviation of the reused (pre-guard) steps from the exact run, step by step
    dev_rel, flips, flagged = [], 0, {}
    rels = (2.0 ** -4, 2.0 ** -5, 2.0 ** -6, 2.0 ** -7, 2.0 ** -8)
    for st, outs in enumerate(reused, start=1):
        n_flag = {x: 0 for x in rels}
        for j, o in enumerate(outs):
            e = s0[j][:, st].astype(np.float32)            # [n_s, V] exact step st
            o = o[:, 0].astype(np.float32)
            top = np.argsort(e, axis=-1)[:, -2:]
            for si in range(e.shape[0]):
                for t in top[si]:
                    dev_rel.append(abs(o[si, t] - e[si, t]) / max(e[si, t], 1e-30))
            flips += int((np.argmax(o, -1) != np.argmax(e, -1)).sum())
            p = np.sort(o, -1)[:, -2:]
            for x in rels:
                n_flag[x] += int((p[:, 0] >= p[:, 1] * (1 - x)).sum())
        for x in rels:
            flagged.setdefault(f"{x:.6f}", []).append(n_flag[x])
    res["reused_vs_exact_top2_rel_dev"] = {"max": float(max(dev_rel)) if dev_rel else None,
                                           "p99": float(np.percentile(dev_rel, 99)) if dev_rel else None,
                                           "median": float(np.median(dev_rel)) if dev_rel else None}
    res["reused_argmax_flips"] = flips
    res["suffixes_flagged_per_step_by_tie_rel"] = flagged
    print(json.dumps({k: res[k] for k in ("tokens_equal", "prompts_with_equal_tokens", "max_abs_diff_scores",
                                          "reused_vs_exact_top2_rel_dev", "reused_argmax_flips",
                                          "suffixes_flagged_per_step_by_tie_rel")}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
