"""A/B of the fused gate/up + SwiGLU GEMM as one launch vs P launches over the intermediate columns
(70B shapes; interleaved rounds in one process, random data; fls_gemm_set_gu_split).

    python scripts/gemm_gu_split.py [--ps 1,2,4] [--ms 14336,43008]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.ops.hip_backend import EPI_SWIGLU, HipOps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ps", default="1,2,4")
    ap.add_argument("--ms", default="14336,43008")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    H, I = 8192, 28672
    w = ((torch.rand(2 * I, H, device=dev) * 2 - 1) * 0.02).half()
    ps = [int(p) for p in a.ps.split(",")]
    for M in (int(m) for m in a.ms.split(",")):
        x = (torch.rand(M, H, device=dev) * 2 - 1).half()
        out = torch.empty(M, I, dtype=torch.float16, device=dev)
        ref = None
        times = {p: [] for p in ps}
        for _ in range(a.rounds):
            for p in ps:
                ops.k.fls_gemm_set_gu_split(p)
                ops.gemm(x, w, EPI_SWIGLU, out=out)
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                else:
                    assert torch.equal(out, ref), p
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    ops.gemm(x, w, EPI_SWIGLU, out=out)
                e.record()
                torch.cuda.synchronize()
                times[p].append(s.elapsed_time(e) / 5 / 1e3)
        ops.k.fls_gemm_set_gu_split(1)
        fl = 2.0 * M * 2 * I * H
        print(json.dumps({"M": M, "tflops": {str(p): round(fl / sorted(t)[len(t) // 2] / 1e12, 1)
                                             for p, t in times.items()},
                          "min_ms": {str(p): round(min(t) * 1e3, 3) for p, t in times.items()}}), flush=True)
        del x, out, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
