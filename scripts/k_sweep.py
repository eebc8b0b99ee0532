"""Per-tile fixed cost vs per-K cost: time C = X W^T at fixed (M, N) over K and
fit T(K) = a + b K for our kernel and hipBLASLt (interleaved rounds, medians).
A large `a` (prologue + epilogue + wave quantisation) argues for a persistent
kernel that overlaps one tile's epilogue with the next tile's prologue."""
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.ops.hip_backend import HipOps, EPI_NONE  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ops = HipOps()
    out = {}
    for M, N in ((16128, 8192), (16128, 57344)):
        Ks = (1024, 2048, 4096, 8192)
        xs = {k: (torch.rand(M, k, device=dev) * 2 - 1).half() for k in Ks}
        ws = {k: ((torch.rand(N, k, device=dev) * 2 - 1) * 0.02).half() for k in Ks}
        c = torch.empty(M, N, dtype=torch.float16, device=dev)
        t = {}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for rnd in range(6):
            for k in Ks:
                for name, fn in (("ours", lambda: ops.gemm(xs[k], ws[k], EPI_NONE, out=c)),
                                 ("hipblaslt", lambda: torch.matmul(xs[k], ws[k].t(), out=c))):
                    ev[0].record()
                    for _ in range(3):
                        fn()
                    ev[1].record()
                    torch.cuda.synchronize()
                    t.setdefault((name, k), []).append(ev[0].elapsed_time(ev[1]) / 3)
        row = {}
        for name in ("ours", "hipblaslt"):
            ms = [statistics.median(t[(name, k)][1:]) for k in Ks]
            b, a = np.polyfit(np.array(Ks, dtype=float), np.array(ms), 1)
            row[name] = {"ms": [round(m, 3) for m in ms], "fixed_ms": round(float(a), 3),
                         "ms_per_1k_K": round(float(b) * 1024, 3),
                         "tflops_at_8k": round(2 * M * N * 8192 / ms[-1] / 1e9, 1)}
        out[f"{M}x{N}"] = row
        print(json.dumps({f"{M}x{N}": row}), flush=True)
        del xs, ws, c


if __name__ == "__main__":
    main()
