"""Small-M projection GEMMs (generation steps, small calls): our kernels vs hipBLASLt at the 70B
shapes, reported as TB/s of weight reads (each weight byte is read once per GEMM; at M <= a few
hundred rows these GEMMs are bound by streaming the weights).  The skinny-M kernel forced
(``fls_gemm_set_skinny(2)``) with each weight-block height is reported next to the automatic
choice.

    python scripts/skinny_bench.py [--ms 16,64,160,256,512]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.ops.hip_backend import EPI_NONE, EPI_RESID, EPI_SWIGLU, HipOps  # noqa: E402


def timed(fn, iters=20, rounds=3):
    ts = []
    for _ in range(rounds):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / iters / 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="16,64,160,256,512")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    H, I, Q = 8192, 28672, 10240
    shapes = [("qkv", Q, H, EPI_NONE), ("o_resid", H, H, EPI_RESID), ("gateup_swiglu", 2 * I, H, EPI_SWIGLU),
              ("down_resid", H, I, EPI_RESID)]
    for name, N, K, epi in shapes:
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
        for M in (int(m) for m in a.ms.split(",")):
            x = (torch.rand(M, K, device=dev) * 2 - 1).half()
            r = torch.randn(M, N, device=dev).half()
            kw = dict(out=r, resid=r) if epi == EPI_RESID else {}
            t_ours = timed(lambda: ops.gemm(x, w, epi, **kw))
            old = ops.k.fls_gemm_set_splitk(0)
            t_nosplit = timed(lambda: ops.gemm(x, w, epi, **kw))
            ops.k.fls_gemm_set_splitk(old)
            forced = {}
            for tag, bn in (("skinny", 0), ("skinny_bn128", 128), ("skinny_bn256", 256)):
                old_m = ops.k.fls_gemm_set_skinny(2, 0)
                old_bn = ops.k.fls_gemm_set_skinny_bn(bn)
                forced[tag + "_us"] = round(timed(lambda: ops.gemm(x, w, epi, **kw)) * 1e6, 1)
                ops.k.fls_gemm_set_skinny_bn(old_bn)
                ops.k.fls_gemm_set_skinny(old_m, 0)
            t_lib = timed(lambda: torch.matmul(x, w.t()))
            wb = N * K * 2
            print(json.dumps({"op": name, "M": M, "N": N, "K": K, "ours_us": round(t_ours * 1e6, 1),
                              "ours_TBps": round(wb / t_ours / 1e12, 2),
                              "no_splitk_TBps": round(wb / t_nosplit / 1e12, 2), "hipblaslt_us": round(t_lib * 1e6, 1),
                              "hipblaslt_TBps": round(wb / t_lib / 1e12, 2), **forced}), flush=True)
        del w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
