"""Attention at the 70B headline shape (32 prompts x (1k-token bidirectional prefix + 5 x 64-token
causal suffixes), 64 q / 8 kv heads, hd 128, 64-row work items): the persistent full-pass kernel
vs one block per (work item, head group), interleaved in one process; useful TFLOP/s (masked work
not counted) and whether the outputs are bitwise equal.

    python scripts/attn_head_bench.py [--iters 20] [--prefix 1024] [--prompts 32]
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
from attn_bench import timeit, useful_flops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--prefix", type=int, default=1024)
    ap.add_argument("--prompts", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sweep", action="store_true",
                    help="also the persistent kernel's heads-per-block (4 / 2 / 1) and 128-row items (4 waves per head)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    nh, nkv, hd = 64, 8, 128
    tps = [TokenizedPrompt(list(range(a.prefix)), [list(range(64))] * 5, 64, [63] * 5) for _ in range(a.prompts)]
    b = pack_prompts(tps, list(range(a.prompts)), "bidirectional", q_block=64)
    qkv = torch.randn(b.num_tokens, (nh + 2 * nkv) * hd, device=dev).half()
    meta = b.device_tensors(dev)
    fl = useful_flops(b.segments, nh, hd)
    outs, best = {}, {}
    for _ in range(a.rounds):
        for pers in (1, 0):
            ops.k.fls_attention_set_persistent(pers)
            out = torch.empty(b.num_tokens, nh * hd, device=dev).half()
            t = timeit(lambda: ops.attention(qkv, meta["work"], nh, nkv, hd, q_block=64, out=out,
                                             seg_lo=meta["seg_lo"]), a.iters)
            best[pers] = min(best.get(pers, 1e9), t)
            outs[pers] = out
    ops.k.fls_attention_set_persistent(1)
    for pers in (1, 0):
        print(json.dumps({"kernel": ["per_unit", "persistent"][pers], "prefix": a.prefix, "prompts": a.prompts,
                          "items": int(b.work.shape[0]), "us": round(best[pers] * 1e6, 1),
                          "tflops": round(fl / best[pers] / 1e12, 1)}), flush=True)
    print(json.dumps({"bitwise_equal": bool(torch.equal(outs[0], outs[1]))}), flush=True)
    if not a.sweep:
        return
    for qb in (64, 128):
        bq = pack_prompts(tps, list(range(a.prompts)), "bidirectional", q_block=qb)
        mq = bq.device_tensors(dev)
        for hpb in (4, 2, 1):
            if qb == 128 and hpb == 4:
                continue                      # (4 waves per head x 4 heads: beyond 8 waves per block)
            old = ops.k.fls_attention_set_hpb(hpb)
            try:
                out = torch.empty(bq.num_tokens, nh * hd, device=dev).half()
                t = min(timeit(lambda: ops.attention(qkv, mq["work"], nh, nkv, hd, q_block=qb, out=out,
                                                     seg_lo=mq["seg_lo"]), a.iters) for _ in range(a.rounds))
            finally:
                ops.k.fls_attention_set_hpb(old)
            print(json.dumps({"kernel": "persistent", "q_block": qb, "hpb": hpb, "us": round(t * 1e6, 1),
                              "tflops": round(fl / t / 1e12, 1),
                              "bitwise_equal_default": bool(torch.equal(out, outs[1]))}), flush=True)


if __name__ == "__main__":
    main()
