"""A/B of v10 tile orders on the 70B projection GEMMs with their fused epilogues
(interleaved rounds, median of 3).   python scripts/gemm_order_ab.py [--m 14336] [--orders 0,-8,8,-4]

order 0 = the launcher's default (each XCD owns 1/8 of the smaller tile dimension);
g > 0 = groups of g M tiles, g < 0 = groups of -g N tiles."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from flexible_llm_sharding_amd.ops.hip_backend import HipOps, EPI_RESID, EPI_SWIGLU, EPI_ROPE  # noqa: E402
from kernel_bench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=14336)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--orders", default="0,-8,8,-4")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    M = a.m
    orders = [int(x) for x in a.orders.split(",")]
    H, I, nh, nkv, hd = 8192, 28672, 64, 8, 128
    pos = torch.randint(0, 4096, (M,), dtype=torch.int32, device=dev)
    cos = torch.rand(4096, hd // 2, device=dev)
    sin = torch.rand(4096, hd // 2, device=dev)
    for name, N, K, epi in [("qkv_rope", (nh + 2 * nkv) * hd, H, EPI_ROPE), ("o_resid", H, H, EPI_RESID),
                            ("gateup_swiglu", 2 * I, H, EPI_SWIGLU), ("down_resid", H, I, EPI_RESID)]:
        x = (torch.rand(M, K, device=dev) * 2 - 1).half()
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
        r = torch.randn(M, N, device=dev).half()
        kw = {}
        if epi == EPI_RESID:
            kw = dict(out=r, resid=r)
        if epi == EPI_ROPE:
            kw = dict(positions=pos, cos=cos, sin=sin, rope_cols=(nh + nkv) * hd, head_dim=hd)
        fl = 2.0 * M * N * K
        ts = {o: [] for o in orders}
        ts["hipblaslt"] = []
        for _ in range(3):
            for o in orders:
                ops.k.fls_gemm_set_order(o)
                ts[o].append(timeit(lambda: ops.gemm(x, w, epi, **kw), a.iters))
            ts["hipblaslt"].append(timeit(lambda: torch.matmul(x, w.t()), a.iters))
        ops.k.fls_gemm_set_order(0)
        row = {"op": name, "M": M, "N": N, "K": K}
        for k, v in ts.items():
            row[f"tflops_{k}"] = round(fl / sorted(v)[1] / 1e12, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
