"""v10 (256 x 256 tile) against v11 (384 x 256 tile) on the 70B projections at row counts that
are not whole tile rounds (micro-batches of a token-budget split: 11 / 10 prompts of 1,344 rows),
interleaved in one process, plus what the launcher's automatic choice takes (``FLS_GEMM_V11=1``: no
more whole 256-CU tile rounds, a v11 tile priced at 1.45 v10 tiles).  (profiles/r5_resident/gemm_m.log
was measured while the round rule was mode 3 and "auto" was the older "no more padded rows than
v10" rule, since removed.)

    python scripts/gemm_v10_v11_m.py [--rows 14784,13440,...]

One JSON line per (shape, rows): median ms of v10, v11, auto, and the tile rounds of each
(tiles / 256 CUs, rounded up).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.ops.hip_backend import EPI_NONE, EPI_RESID, EPI_SWIGLU, HipOps  # noqa: E402

ROWS = "4096,6144,8064,10752,12288,13440,14784,15360,16128,43008"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default=ROWS)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    H, I = 8192, 28672
    Ms = [int(m) for m in a.rows.split(",")]
    Mmax = max(Ms)
    shapes = (("qkv", 10240, H, EPI_NONE), ("o_resid", H, H, EPI_RESID),
              ("gateup_swiglu", 2 * I, H, EPI_SWIGLU), ("down_resid", H, I, EPI_RESID))
    for name, N, K, epi in shapes:
        x = ((torch.rand(Mmax, K, device=dev) * 2 - 1) * 0.5).half()
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
        out = torch.randn(Mmax, N // 2 if epi == EPI_SWIGLU else N, device=dev).half()
        for M in Ms:
            def run():
                if epi == EPI_RESID:
                    ops.gemm(x[:M], w, epi, out=out[:M], resid=out[:M])
                else:
                    ops.gemm(x[:M], w, epi, out=out[:M])
            times = {"v10": [], "v11": [], "auto": []}
            for _ in range(a.reps):
                for tag, mode in (("v10", 0), ("v11", 2), ("auto", 1)):
                    ops.k.fls_gemm_set_v11(mode)
                    run()
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                    ev[0].record()
                    for _ in range(3):
                        run()
                    ev[1].record()
                    torch.cuda.synchronize()
                    times[tag].append(ev[0].elapsed_time(ev[1]) / 3)
            ops.k.fls_gemm_set_v11(1)
            med = {k: round(sorted(v)[len(v) // 2], 3) for k, v in times.items()}
            r10 = -(-(-(-M // 256) * (N // 256)) // 256)
            r11 = -(-(-(-M // 384) * (N // 256)) // 256)
            print(json.dumps({"op": name, "M": M, "ms": med, "rounds_v10": r10, "rounds_v11": r11,
                              "v11_over_v10": round(med["v11"] / med["v10"], 3)}), flush=True)
        del x, w, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
