"""Is the LDS-DMA stream channel-bound by the power-of-two row stride?

Times the gate/up GEMM (v10 fused path and hipBLASLt) with X and W stored at
row strides K + pad (elements), pad in {0, 64, 128, 256}.  Interleaved rounds,
median of 5.
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.ops.hip_backend import HipOps, EPI_NONE  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ops = HipOps()
    M, N, K = 16128, 57344, 8192
    shapes = [(M, N, K), (M, 8192, 28672)]
    res = {}
    for (m, n, k) in shapes:
        cases = {}
        for pad in (0, 64, 128, 256):
            xb = (torch.rand(m, k + pad, device=dev) * 2 - 1).half()
            wb = ((torch.rand(n, k + pad, device=dev) * 2 - 1) * 0.02).half()
            cases[pad] = (xb[:, :k], wb[:, :k], torch.empty(m, n, dtype=torch.float16, device=dev))
        times = {}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for rnd in range(6):
            for pad, (x, w, c) in cases.items():
                for name, fn in (("v10", lambda: ops.gemm(x, w, EPI_NONE, out=c)),
                                 ("hipblaslt", lambda: torch.matmul(x, w.t(), out=c))):
                    ev[0].record()
                    for _ in range(2):
                        fn()
                    ev[1].record()
                    torch.cuda.synchronize()
                    times.setdefault(f"{name}_pad{pad}", []).append(ev[0].elapsed_time(ev[1]) / 2)
        fl = 2.0 * m * n * k
        res[f"{m}x{n}x{k}"] = {key: round(fl / statistics.median(v[1:]) / 1e9, 1) for key, v in times.items()}
        print(json.dumps({f"{m}x{n}x{k}": res[f"{m}x{n}x{k}"]}), flush=True)
        del cases


if __name__ == "__main__":
    main()
