"""Generation-step GEMMs at the 70B shapes: the row-exact path (mid-M kernel, 64- or 128-column
blocks) against the non-exact skinny / split-K paths.

    python scripts/decode_gemm_bench.py [--rows 64,160,320] [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.ops.hip_backend import EPI_NONE, EPI_RESID, EPI_ROPE, EPI_SWIGLU, HipOps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="64,160,320")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    H, I, nh, nkv, hd = 8192, 28672, 64, 8, 128
    g = torch.Generator(device=dev).manual_seed(0)
    w = {"qkv": torch.randn((nh + 2 * nkv) * hd, H, device=dev, generator=g).half() * 0.02,
         "o": torch.randn(H, H, device=dev, generator=g).half() * 0.02,
         "gate_up": torch.randn(2 * I, H, device=dev, generator=g).half() * 0.02,
         "down": torch.randn(H, I, device=dev, generator=g).half() * 0.02}
    cos = torch.rand(8192, hd // 2, device=dev)
    sin = torch.rand(8192, hd // 2, device=dev)
    # arm -> (row-exact, fls_gemm_set_mid_bn, fls_gemm_set_mid_waves, fls_gemm_set_mid_rows): exact
    # default (mid-M kernel), exact with 128-column blocks of 4 / 8 waves only (8: 64- or 128-row
    # blocks), with 64-column blocks of 4 / 8 waves only, with 32-column blocks (O / down; the others
    # fall back), the non-exact default (skinny / split-K)
    arms = {"exact": (True, 0, 0, 0), "exact_w4": (True, 128, 4, 0), "exact_w8": (True, 128, 8, 64),
            "exact_w8r128": (True, 128, 8, 128), "exact_bn64w4": (True, 64, 4, 0),
            "exact_bn64w8": (True, 64, 8, 0), "exact_bn32": (True, 32, 8, 0), "fast": (False, 0, 0, 0)}
    for M in [int(r) for r in a.rows.split(",")]:
        x = torch.randn(M, H, device=dev, generator=g).half()
        xi = torch.randn(M, I, device=dev, generator=g).half()
        r0 = torch.randn(M, H, device=dev, generator=g).half()
        pos = torch.randint(0, 8000, (M,), dtype=torch.int32, device=dev)
        rs = torch.rand(M, device=dev) + 0.5
        calls = {
            "qkv": lambda: ops.gemm(x, w["qkv"], EPI_ROPE, positions=pos, cos=cos, sin=sin,
                                    rope_cols=(nh + nkv) * hd, head_dim=hd, rscale=rs),
            "o": lambda: ops.gemm(x, w["o"], EPI_RESID, out=r0, resid=r0),
            "gate_up": lambda: ops.gemm(x, w["gate_up"], EPI_SWIGLU, rscale=rs),
            "down": lambda: ops.gemm(xi, w["down"], EPI_RESID, out=r0, resid=r0),
        }
        res = {"M": M}
        outs = {}
        for _ in range(4 * a.iters):       # clocks up before the first arm is timed
            calls["gate_up"]()
        for arm, (exact, bn, waves, rows) in arms.items():
            old_bn, old_w = ops.k.fls_gemm_set_mid_bn(bn), ops.k.fls_gemm_set_mid_waves(waves)
            old_r = ops.k.fls_gemm_set_mid_rows(rows)
            try:
                with ops.row_exact(exact):
                    tot = 0.0
                    for name, f in calls.items():
                        f()
                        torch.cuda.synchronize()
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for _ in range(a.iters):
                            f()
                        e1.record()
                        torch.cuda.synchronize()
                        us = e0.elapsed_time(e1) * 1000 / a.iters
                        tbs = w[name].numel() * 2 / (us * 1e-6) / 1e12
                        res[f"{arm}.{name}_us"] = round(us, 1)
                        res[f"{arm}.{name}_TBps"] = round(tbs, 2)
                        tot += us
                        if name == "gate_up":
                            outs[arm] = f().clone()
                    res[f"{arm}.layer_us"] = round(tot, 1)
            finally:
                ops.k.fls_gemm_set_mid_bn(old_bn)
                ops.k.fls_gemm_set_mid_waves(old_w)
                ops.k.fls_gemm_set_mid_rows(old_r)
        res["exact_arms_bitwise_equal"] = all(torch.equal(outs["exact"], v) for k, v in outs.items()
                                              if k.startswith("exact_"))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
