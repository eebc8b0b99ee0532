"""A/B of the GEMM main kernels on the 70B production shapes: v10 (256 x 256 tile), v11 (384 x 256,
gemm_v11.hip) and hipBLASLt (torch.matmul, plain epilogue), interleaved rounds in one process,
random fp16 data; first checks v11 == v10 bitwise on every shape.

    python scripts/gemm_v11_ab.py [--rounds 3] [--orders 0] [--rows 0]
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--orders", default="0", help="v11 tile orders to sweep (0 = auto)")
    ap.add_argument("--rows", default="0", help="v11 rows per launch to sweep (0 = all)")
    ap.add_argument("--mchunk", type=int, default=14592, help="rows of the chunked QKV / MLP GEMMs")
    ap.add_argument("--only", default="")
    ap.add_argument("--plain", action="store_true", help="no epilogue (EPI_NONE) on every shape")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    k = ops.k
    H, I, nh, nkv, hd = 8192, 28672, 64, 8, 128
    mc = a.mchunk
    shapes = [("qkv_rope", mc, (nh + 2 * nkv) * hd, H, EPI_ROPE), ("o_resid", 43008, H, H, EPI_RESID),
              ("gateup_swiglu", mc, 2 * I, H, EPI_SWIGLU), ("down_resid", mc, H, I, EPI_RESID)]
    if a.only:
        shapes = [s for s in shapes if s[0] in a.only.split(",")]
    if a.plain:
        shapes = [(n + "_plain", M, N, K, 0) for n, M, N, K, _ in shapes]
    pos = torch.randint(0, 4096, (43008,), dtype=torch.int32, device=dev)
    cos = torch.rand(4096, hd // 2, device=dev)
    sin = torch.rand(4096, hd // 2, device=dev)
    variants = [("v10", 0, 0, 0)]
    for o in [int(v) for v in a.orders.split(",")]:
        for r in [int(v) for v in a.rows.split(",")]:
            variants.append((f"v11_o{o}_r{r}", 2, o, r))
    for name, M, N, K, epi in shapes:
        x = (torch.rand(M, K, device=dev) * 2 - 1).half()
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
        r = torch.randn(M, N, device=dev).half()
        kw = {}
        if epi == EPI_RESID:
            kw = dict(out=r, resid=r)
        if epi == EPI_ROPE:
            kw = dict(positions=pos[:M], cos=cos, sin=sin, rope_cols=(nh + nkv) * hd, head_dim=hd)
        # bitwise check (non-resid: outputs independent of r)
        chk = {}
        for vn, mode, o, rr in variants[:2]:
            k.fls_gemm_set_v11(mode)
            k.fls_gemm_v11_tune(o, rr)
            if epi == EPI_RESID:
                rc = r.clone()
                chk[vn] = ops.gemm(x, w, epi, out=rc, resid=rc)
            else:
                chk[vn] = ops.gemm(x, w, epi, **kw)
        torch.cuda.synchronize()
        same = bool(torch.equal(*chk.values()))
        del chk
        fl = 2.0 * M * N * K
        times = {v[0]: [] for v in variants}
        times["hipblaslt"] = []
        for _ in range(a.rounds):
            for vn, mode, o, rr in variants:
                k.fls_gemm_set_v11(mode)
                k.fls_gemm_v11_tune(o, rr)
                for _ in range(2):
                    ops.gemm(x, w, epi, **kw)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    ops.gemm(x, w, epi, **kw)
                e.record()
                torch.cuda.synchronize()
                times[vn].append(s.elapsed_time(e) / a.iters / 1e3)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                torch.matmul(x, w.t())
            e.record()
            torch.cuda.synchronize()
            times["hipblaslt"].append(s.elapsed_time(e) / a.iters / 1e3)
        k.fls_gemm_set_v11(1)
        k.fls_gemm_v11_tune(0, 0)
        row = {"op": name, "M": M, "N": N, "K": K, "v11_bitwise_v10": same,
               "tflops": {v: round(fl / sorted(t)[len(t) // 2] / 1e12, 1) for v, t in times.items()}}
        print(json.dumps(row), flush=True)
        del x, w, r
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
