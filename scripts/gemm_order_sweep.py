"""Tile-order sweep of the fused v10 GEMMs on the production shapes of the 70B headline pass
(interleaved rounds in one process; order 0 = the shipped ``auto_order``).

    python scripts/gemm_order_sweep.py [--orders 0,-4,-8,4,8] [--rounds 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.ops.hip_backend import EPI_RESID, EPI_ROPE, EPI_SWIGLU, HipOps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--orders", default="0,-2,-4,-7,-8,-14,4,7,8")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    H, I, nh, nkv, hd = 8192, 28672, 64, 8, 128
    shapes = [("qkv_rope", 14336, (nh + 2 * nkv) * hd, H, EPI_ROPE), ("o_resid", 43008, H, H, EPI_RESID),
              ("gateup_swiglu", 14336, 2 * I, H, EPI_SWIGLU), ("down_resid", 14336, H, I, EPI_RESID)]
    orders = [int(o) for o in a.orders.split(",")]
    pos = torch.randint(0, 4096, (43008,), dtype=torch.int32, device=dev)
    cos = torch.rand(4096, hd // 2, device=dev)
    sin = torch.rand(4096, hd // 2, device=dev)
    for name, M, N, K, epi in shapes:
        x = (torch.rand(M, K, device=dev) * 2 - 1).half()
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
        r = torch.randn(M, N, device=dev).half()
        kw = {}
        if epi == EPI_RESID:
            kw = dict(out=r, resid=r)
        if epi == EPI_ROPE:
            kw = dict(positions=pos[:M], cos=cos, sin=sin, rope_cols=(nh + nkv) * hd, head_dim=hd)
        fl = 2.0 * M * N * K
        times = {o: [] for o in orders}
        for _ in range(a.rounds):
            for o in orders:
                ops.k.fls_gemm_set_order(o)
                for _ in range(2):
                    ops.gemm(x, w, epi, **kw)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    ops.gemm(x, w, epi, **kw)
                e.record()
                torch.cuda.synchronize()
                times[o].append(s.elapsed_time(e) / a.iters / 1e3)
        ops.k.fls_gemm_set_order(0)
        tl = []
        for _ in range(a.rounds):
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                torch.matmul(x, w.t())
            e.record()
            torch.cuda.synchronize()
            tl.append(s.elapsed_time(e) / a.iters / 1e3)
        row = {"op": name, "M": M, "N": N, "K": K,
               "tflops": {str(o): round(fl / sorted(t)[len(t) // 2] / 1e12, 1) for o, t in times.items()},
               "hipblaslt_plain_tflops": round(fl / sorted(tl)[len(tl) // 2] / 1e12, 1)}
        print(json.dumps(row), flush=True)
        del x, w, r
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
