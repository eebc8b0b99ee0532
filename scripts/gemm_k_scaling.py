"""Per-tile overhead of the v10 GEMM: TFLOP/s of the same output tiles at growing K (one process,
interleaved rounds).  If the gap to hipBLASLt on the short-K shapes (gate/up, O, QKV: K = 8192) is
the per-tile prologue / epilogue, TFLOP/s rise with K.

    python scripts/gemm_k_scaling.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.ops.hip_backend import EPI_NONE, EPI_SWIGLU, HipOps  # noqa: E402


def tflops(fn, fl, iters=6, rounds=3):
    ts = []
    for _ in range(rounds):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / iters / 1e3)
    return fl / sorted(ts)[len(ts) // 2] / 1e12


def main():
    dev = torch.device("cuda", 0)
    ops = HipOps()
    M, N = 14336, 28672
    for epi, name in ((EPI_SWIGLU, "swiglu"), (EPI_NONE, "plain")):
        for K in (4096, 8192, 16384, 32768):
            x = (torch.rand(M, K, device=dev) * 2 - 1).half()
            w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
            fl = 2.0 * M * N * K
            ours = tflops(lambda: ops.gemm(x, w, epi), fl)
            lib = tflops(lambda: torch.matmul(x, w.t()), fl)
            print(json.dumps({"epi": name, "M": M, "N": N, "K": K, "ours_tflops": round(ours, 1),
                              "hipblaslt_plain_tflops": round(lib, 1)}), flush=True)
            del x, w
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
