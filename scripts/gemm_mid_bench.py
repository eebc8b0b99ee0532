"""Small/medium-M GEMM: 64x128-tile mid kernel vs the 256x256 main kernel vs hipBLASLt.

    python scripts/gemm_mid_bench.py [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.ops.hip_backend import HipOps  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    ops.backend = "hip"
    shapes = [("7b_qkv", 12288, 4096), ("7b_o", 4096, 4096), ("7b_gateup", 22016, 4096), ("7b_down", 4096, 11008),
              ("70b_gateup", 57344, 8192), ("70b_down", 8192, 28672), ("lm_head", 32000, 4096)]
    rows = []
    for M in (64, 160, 416, 1024, 2048):
        for name, N, K in shapes:
            x = (torch.rand(M, K, device=dev) * 2 - 1).half()
            w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
            fl = 2.0 * M * N * K
            row = {"shape": name, "M": M, "N": N, "K": K}
            for mid in (1, 0):
                ops.k.fls_gemm_set_mid(mid)
                t = timeit(lambda: ops.gemm(x, w))
                row["mid_us" if mid else "main_us"] = round(t * 1e6, 1)
            ops.k.fls_gemm_set_mid(1)
            t = timeit(lambda: torch.matmul(x, w.t()))
            row["hipblaslt_us"] = round(t * 1e6, 1)
            row["weight_GBps_mid"] = round(N * K * 2 / (row["mid_us"] * 1e-6) / 1e9)
            row["tflops_mid"] = round(fl / (row["mid_us"] * 1e-6) / 1e12)
            rows.append(row)
            print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
