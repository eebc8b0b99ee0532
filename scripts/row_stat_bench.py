"""Time the fused norm's row statistic (ops.row_stat: fls_row_stat) at generation-step row counts.

    python scripts/row_stat_bench.py [--rows 40,160,320] [--hidden 8192]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.ops.hip_backend import HipOps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="40,160,320")
    ap.add_argument("--hidden", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    ops = HipOps()
    for m in [int(r) for r in a.rows.split(",")]:
        x = torch.randn(m, a.hidden, device="cuda").half()
        out = torch.empty(m, device="cuda")
        for _ in range(20):
            ops.row_stat(x, 1e-5, out=out)
        torch.cuda.synchronize()
        # captured in a graph, so the time is the GPU's (a Python launch loop measures the host)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(a.iters):
                    ops.row_stat(x, 1e-5, out=out)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / a.iters
        ref = torch.rsqrt(x.float().pow(2).mean(-1) + 1e-5)
        print(json.dumps({"rows": m, "hidden": a.hidden, "us": round(us, 2),
                          "max_rel_err": float(((out - ref).abs() / ref).max())}), flush=True)


if __name__ == "__main__":
    main()
