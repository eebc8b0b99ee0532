"""Decode-step attention microbenchmark at the 70B generation shape (32 prompts x 5 suffixes, one
new row per suffix, 1,024-token prefixes and ~67 cached rows per suffix in the K/V cache).

Times the range-2 attention launch (q_block 8: packed-GQA decode kernel; 32: one wave per head)
on two cache layouts holding the same bytes:
  * production: one cache row = K and V of all 8 KV heads (4 KB), 8 blocks per prompt each read
    512 B of every row;
  * grouped: the same K/V re-laid out per KV group (each block reads one contiguous region),
    run as 256 one-group items.
and reports the effective K/V read bandwidth.  Each launch reads a different one of --layers
caches (2.9 GB at 16: the 256 MB Infinity Cache holds none of them across launches, like the
80 layers of a real step).

    python scripts/attn_decode_bench.py [--iters 50] [--prefix 1024] [--kept 67]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.ops.hip_backend import HipOps  # noqa: E402


def items(n_prompts, n_suffix, prefix, kept, groups=1):
    """Work items / range-2 windows of a decode step: item j = prompt j (x group), q rows = one new
    row per suffix; the cache holds per prompt the prefix, then every suffix's kept rows + its new
    row.  ``groups`` > 1: one item per (prompt, group) over a cache laid out per group."""
    per = prefix + n_suffix * (kept + 1)            # cache rows per prompt
    work, work2, win = [], [], []
    t = 0
    for gi in range(groups):
        for j in range(n_prompts):
            base = (gi * n_prompts + j) * per
            work.append((t, n_suffix, 0, base, prefix, 0, 0, 0))
            s0 = base + prefix
            work2.append((s0, n_suffix * (kept + 1)))
            for s in range(n_suffix):
                c0 = s0 + s * (kept + 1)
                win.append((c0, c0 + kept + 1))
            t += n_suffix
    return (np.asarray(work, np.int32), np.asarray(work2, np.int32), np.asarray(win, np.int32), t,
            n_prompts * per * groups)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--prompts", type=int, default=32)
    ap.add_argument("--suffixes", type=int, default=5)
    ap.add_argument("--prefix", type=int, default=1024)
    ap.add_argument("--kept", type=int, default=67)
    ap.add_argument("--layers", type=int, default=16)
    a = ap.parse_args()
    ops = HipOps()
    dev = torch.device("cuda", 0)
    nh, nkv, hd = 64, 8, 128
    hpg = nh // nkv
    for layout in ("production", "grouped"):
        G = 1 if layout == "production" else nkv
        w, w2, win, T, rows = items(a.prompts, a.suffixes, a.prefix, a.kept, groups=G)
        h, k = (nh, nkv) if G == 1 else (hpg, 1)
        caches = [(torch.randn(rows, 2 * k * hd, device=dev) * 0.5).half() for _ in range(a.layers)]
        qkv = (torch.randn(T, (h + 2 * k) * hd, device=dev) * 0.5).half()
        wt, w2t, wint = (torch.from_numpy(x).to(dev) for x in (w, w2, win))
        seg = torch.zeros(T, dtype=torch.int32, device=dev)
        kv_bytes = int(sum(int(x[4]) for x in w) + sum(int(x[1]) for x in w2)) * 2 * hd * 2 * (nkv if G == 1 else 1)
        for qb, ns in ((8, 0), (8, 2), (8, 4), (8, 6), (8, 8), (32, 0)):
            ops.k.fls_attention_set_split(ns)
            li = [0]

            def run():
                li[0] = (li[0] + 1) % a.layers
                ops.attention(qkv, wt, h, k, hd, kv0=caches[li[0]], q_block=qb, seg_lo=seg, work2=w2t, r2win=wint)
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            # captured in a graph: GPU time (a launch loop from Python measures the host at few prompts)
            g = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                with torch.cuda.graph(g, stream=st):
                    for _ in range(a.iters):
                        run()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000 / a.iters
            ops.k.fls_attention_set_split(0)
            print(f"{layout:10s} q_block {qb:2d} split {ns or 'auto'}: {us:7.1f} us/launch  K/V {kv_bytes / 1e6:.0f} MB  "
                  f"{kv_bytes / us / 1e6:.2f} TB/s  (x80 layers: {us * 80 / 1000:.2f} ms/step)", flush=True)
        del caches


if __name__ == "__main__":
    main()
