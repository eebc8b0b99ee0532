"""The 70B generation-step attention on its own (range-2 kernel, suffix K/V reuse): 32 prompts x
(1024-token prefix + 5 suffixes), one new row per suffix after its kept rows, K/V read from a
prefix + suffix cache.  The cache rotates over enough copies (> 600 MB) that no launch finds its
K/V in the 256 MB Infinity Cache, as in a real step where 80 layers' caches stream by.  Prints
microseconds per launch and the K/V read rate; used for rocprofv3 --pmc passes.

    python scripts/attn_gen_one.py [--iters 20] [--suffix-len 66]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.ops.hip_backend import HipOps  # noqa: E402
from flexible_llm_sharding_amd.runtime.batch import pack_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--prompts", type=int, default=32)
    ap.add_argument("--prefix-len", type=int, default=1024)
    ap.add_argument("--suffix-len", type=int, default=66)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    nh, nkv, hd = 64, 8, 128
    lp, ls = a.prefix_len, [a.suffix_len] * 5
    tps = [TokenizedPrompt(list(range(lp)), [list(range(l)) for l in ls], max(ls), [l - 1 for l in ls])
           for _ in range(a.prompts)]
    offs, t = [], 0
    for _ in tps:
        offs.append(t)
        t += lp
    rows = []
    for _ in tps:
        rows.append([])
        for l in ls:
            rows[-1].append(t)
            t += l
    keep = [[l - 1 for l in ls] for _ in tps]
    b = pack_prompts(tps, list(range(len(tps))), "bidirectional", prefix_offsets=offs, kv_cached=True,
                     suffix_rows=rows, suffix_keep=keep)
    m = b.device_tensors(dev)
    kv = 2 * nkv * hd
    ncopy = max(1, -(-600_000_000 // (t * kv * 2)))
    caches = [(torch.randn(t, kv, device=dev) * 0.5).half() for _ in range(ncopy)]
    qkv = (torch.randn(b.num_tokens, (nh + 2 * nkv) * hd, device=dev) * 0.5).half()
    out = torch.empty(b.num_tokens, nh * hd, dtype=torch.float16, device=dev)

    def run(c):
        ops.attention(qkv, m["work"], nh, nkv, hd, kv0=c, seg_lo=m["seg_lo"], work2=m["work2"],
                      r2win=m["r2win"], q_block=b.r2_q_block, out=out)
    for i in range(3):
        run(caches[i % ncopy])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(a.iters):
        run(caches[i % ncopy])
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / a.iters * 1e3
    kv_bytes = a.prompts * (lp + sum(ls)) * kv * 2          # every cached K/V row read once per launch
    print(json.dumps({"rows": b.num_tokens, "items": int(m["work"].shape[0]), "q_block": b.r2_q_block,
                      "us": round(us, 1), "kv_MB": round(kv_bytes / 1e6, 1),
                      "kv_TBps": round(kv_bytes / (us * 1e-6) / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
