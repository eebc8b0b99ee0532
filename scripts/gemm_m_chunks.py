"""One fused GEMM over all rows vs the same rows in chunks (70B O-projection + residual, gate/up +
SwiGLU), interleaved rounds in one process: does the 256x256-tile kernel prefer smaller grids?

    python scripts/gemm_m_chunks.py [--rows 43008] [--chunks 1,2,3,4]

A chunk count ``0`` is one call with the launcher's own row chunking turned off
(``fls_gemm_set_row_chunk(0)``); ``1`` is one call with the launcher's default (<= 16384 rows a launch).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.ops.hip_backend import EPI_RESID, EPI_SWIGLU, HipOps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=43008)
    ap.add_argument("--chunks", default="1,2,3,4")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    H, I, M = 8192, 28672, a.rows
    x = (torch.rand(M, H, device=dev) * 2 - 1).half()
    for name, N, epi in (("o_resid", H, EPI_RESID), ("gateup_swiglu", 2 * I, EPI_SWIGLU)):
        w = ((torch.rand(N, H, device=dev) * 2 - 1) * 0.02).half()
        out = torch.randn(M, N if epi == EPI_RESID else I, device=dev).half()
        cs = [int(c) for c in a.chunks.split(",")]
        default_chunk = ops.k.fls_gemm_set_row_chunk(0)
        ops.k.fls_gemm_set_row_chunk(default_chunk)
        times = {c: [] for c in cs}
        for _ in range(a.rounds):
            for c in cs:
                ops.k.fls_gemm_set_row_chunk(0 if c == 0 else default_chunk)
                step = -(-M // max(c, 1))
                step = -(-step // 256) * 256

                def run():
                    for s in range(0, M, step):
                        if epi == EPI_RESID:
                            ops.gemm(x[s:s + step], w, epi, out=out[s:s + step], resid=out[s:s + step])
                        else:
                            ops.gemm(x[s:s + step], w, epi, out=out[s:s + step])
                run()
                torch.cuda.synchronize()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                for _ in range(3):
                    run()
                ev[1].record()
                torch.cuda.synchronize()
                times[c].append(ev[0].elapsed_time(ev[1]) / 3 / 1e3)
        fl = 2.0 * M * N * H
        print(json.dumps({"op": name, "M": M, "tflops_by_chunks": {str(c): round(fl / sorted(t)[len(t) // 2] / 1e12, 1)
                                                                    for c, t in times.items()}}), flush=True)
        del w, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
