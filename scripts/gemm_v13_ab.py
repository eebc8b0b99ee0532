"""A/B of the persistent GEMM v13 against v10 on the Llama-2-7B and -70B projection shapes
(all four epilogues as the engine uses them), alternating the two kernels 5 times per shape.

    python scripts/gemm_v13_ab.py [--m 16128] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.ops.hip_backend import HipOps, EPI_NONE, EPI_RESID, EPI_SWIGLU, EPI_ROPE  # noqa


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16128)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    M = a.m
    pos = torch.randint(0, 4096, (M,), dtype=torch.int32, device=dev)
    cos = torch.rand(4096, 64, device=dev)
    sin = torch.rand(4096, 64, device=dev)
    shapes = []
    for model, H, I, nh, nkv in (("7b", 4096, 11008, 32, 32), ("70b", 8192, 28672, 64, 8)):
        shapes += [(model, "qkv_rope", (nh + 2 * nkv) * 128, H, EPI_ROPE, (nh + nkv) * 128),
                   (model, "o_resid", H, H, EPI_RESID, 0), (model, "gateup_swiglu", 2 * I, H, EPI_SWIGLU, 0),
                   (model, "down_resid", H, I, EPI_RESID, 0)]
    ops.k.fls_gemm_set_rope_persistent(0)
    for model, name, N, K, epi, rc in shapes:
        x = (torch.rand(M, K, device=dev) * 2 - 1).half()
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
        r = torch.randn(M, N, device=dev).half()
        kw = {}
        if epi == EPI_RESID:
            kw = dict(out=r, resid=r)
        if epi == EPI_ROPE:
            kw = dict(positions=pos, cos=cos, sin=sin, rope_cols=rc, head_dim=128)
        t = {10: [], 13: []}
        for _ in range(5):
            for var in (10, 13):
                ops.k.fls_gemm_set_variant(var)
                t[var].append(timeit(lambda: ops.gemm(x, w, epi, **kw), a.iters))
        ops.k.fls_gemm_set_variant(10)
        fl = 2.0 * M * N * K
        m10, m13 = min(t[10]), min(t[13])
        print(json.dumps({"model": model, "op": name, "M": M, "N": N, "K": K, "v10_ms": round(m10, 4),
                          "v13_ms": round(m13, 4), "v13_gain_pct": round(100 * (m10 / m13 - 1), 2),
                          "v10_tflops": round(fl / m10 / 1e9, 1)}), flush=True)
        del x, w, r
    ops.k.fls_gemm_set_rope_persistent(1)


if __name__ == "__main__":
    main()
