"""Attention study on MI355X (profiles/r2_attn): the shared-prefix flash attention over the bench's
work items for the Llama-2-70B (64 q / 8 kv heads, 64-row items) and Llama-2-7B (32 / 32, 128-row
items) head layouts, prefix 1k and 4k, five suffixes of 64 tokens (the bench) or of 10 tokens.

* prefix items vs suffix items: a suffix item re-reads the prompt's prefix K/V that every other
  suffix item of the prompt reads too; if that costs, suffix items run at a lower TFLOP/s;
* one suffix per item (round-1 packing, runtime.batch._work_items) vs items over all of a prompt's
  suffix rows with a block-diagonal range 1 (seg_lo): the one-pass shared-prefix form.

    python scripts/attn_bench.py [--iters 20] [--json out.json]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.ops.hip_backend import HipOps  # noqa: E402
from flexible_llm_sharding_amd.runtime.batch import _work_items, pack_prompts  # noqa: E402
from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def useful_flops(segs, nh: int, hd: int) -> float:
    """2 matmuls x 2 FLOP x visible (query, key) pairs x heads x head_dim (masked work not counted)."""
    pairs = 0
    for sg in segs:
        for i in range(sg.q_len):
            qi = sg.q_off + i
            pairs += (min(sg.r0_len, qi + 1) if sg.r0_causal else sg.r0_len) + (i + 1 if sg.r1_len else 0)
    return 4.0 * pairs * nh * hd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    hd = 128
    res = []
    for model, nh, nkv in (("70b", 64, 8), ("7b", 32, 32)):
        q_block = 128 if (nh // nkv) % 2 == 1 else 64
        for lp, n_prompts, ls in ((1024, 12, 64), (4096, 3, 64), (1024, 12, 10)):
            tps = [TokenizedPrompt(list(range(lp)), [list(range(ls))] * 5, ls, [ls - 1] * 5) for _ in range(n_prompts)]
            b = pack_prompts(tps, list(range(n_prompts)), "bidirectional", q_block=q_block)
            qkv = torch.randn(b.num_tokens, (nh + 2 * nkv) * hd, device=dev).half()
            out = torch.empty(b.num_tokens, nh * hd, device=dev).half()
            seg_lo = torch.from_numpy(b.seg_lo).to(dev)
            single = _work_items(b.segments, q_block)
            pfx = [sg for sg in b.segments if not sg.r1_len]
            sfx = [sg for sg in b.segments if sg.r1_len]
            sets = {"prefix_items": (b.work[b.work[:, 7] == 0], pfx),
                    "suffix_items_multi": (b.work[b.work[:, 7] > 0], sfx),
                    "suffix_items_single": (single[single[:, 7] > 0], sfx),
                    "all_multi": (b.work, b.segments), "all_single": (single, b.segments)}
            base = {"model": model, "prefix": lp, "suffix_len": ls, "prompts": n_prompts}
            times = {}
            for _ in range(5):                   # interleaved rounds
                for name, (w, _) in sets.items():
                    wd = torch.from_numpy(np.ascontiguousarray(w)).to(dev)
                    t = timeit(lambda: ops.attention(qkv, wd, nh, nkv, hd, q_block=q_block, out=out, seg_lo=seg_lo),
                               a.iters)
                    times[name] = min(times.get(name, 1e9), t)
            for name, (w, segs) in sets.items():
                fl = useful_flops(segs, nh, hd)
                row = dict(base, items=name, n_items=int(w.shape[0]), us=round(times[name] * 1e6, 1),
                           tflops=round(fl / times[name] / 1e12, 1))
                res.append(row)
                print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
