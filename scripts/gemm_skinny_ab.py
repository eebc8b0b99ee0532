"""A/B of the small-M GEMM paths on the 70B projections at generation-step row counts: skinny
kernel (gemm_skinny.h) vs the previous small-M paths (split-K 256 x 256 / mid-M / main) vs
hipBLASLt (torch.matmul, plain epilogue).  Weights rotate over enough copies (> 600 MB) that no
launch finds its weights in the 256 MB Infinity Cache, as in a real step where 80 layers stream
by.  Prints one JSON line per (shape, M): microseconds and the effective weight-read rate.

    python scripts/gemm_skinny_ab.py [--ms 32,64,128,160,256] [--rounds 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.ops.hip_backend import EPI_RESID, EPI_ROPE, EPI_SWIGLU, HipOps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="32,64,128,160,256")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--blocks", default="", help="skinny K-split block targets to sweep besides the default rule")
    ap.add_argument("--blocks256", default="", help="the same for the 256-row weight block")
    ap.add_argument("--only", default="")
    ap.add_argument("--variants", default="", help="kernel-library variants (build.py --variant) to add")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    k = ops.k
    from flexible_llm_sharding_amd import _native
    vops = {}
    for v in [x for x in a.variants.split(",") if x]:
        o = HipOps()
        o.k = _native._load_kernels(os.path.join(os.path.dirname(_native.__file__), "variants",
                                                 f"libfls_kernels_{v}.so"))
        vops[v] = o
    H, I, nh, nkv, hd = 8192, 28672, 64, 8, 128
    shapes = [("qkv_rope", (nh + 2 * nkv) * hd, H, EPI_ROPE), ("o_resid", H, H, EPI_RESID),
              ("gateup_swiglu", 2 * I, H, EPI_SWIGLU), ("down_resid", H, I, EPI_RESID)]
    if a.only:
        shapes = [s for s in shapes if s[0] in a.only.split(",")]
    pos = torch.randint(0, 4096, (256,), dtype=torch.int32, device=dev)
    cos = torch.rand(4096, hd // 2, device=dev)
    sin = torch.rand(4096, hd // 2, device=dev)
    variants = ([("before", 0, 0, 0), ("skinny", 2, 0, 128), ("skinny256", 2, 0, 256)]
                + [(f"skinny_b{b}", 2, int(b), 128) for b in a.blocks.split(",") if b]
                + [(f"skinny256_b{b}", 2, int(b), 256) for b in a.blocks256.split(",") if b])
    for name, N, K, epi in shapes:
        wbytes = N * K * 2
        ncopy = max(1, -(-600_000_000 // wbytes))
        ws = [((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half() for _ in range(ncopy)]
        for M in [int(m) for m in a.ms.split(",")]:
            x = (torch.rand(M, K, device=dev) * 2 - 1).half()
            r = torch.randn(M, N, device=dev).half()
            kw = {}
            if epi == EPI_RESID:
                kw = dict(out=r, resid=r)
            if epi == EPI_ROPE:
                kw = dict(positions=pos[:M], cos=cos, sin=sin, rope_cols=(nh + nkv) * hd, head_dim=hd)
            outs = {}
            for vn, mode, b, bn in variants:
                k.fls_gemm_set_skinny(mode, b)
                k.fls_gemm_set_skinny_bn(bn)
                outs[vn] = ops.gemm(x, ws[0], epi, **({} if epi == EPI_RESID else kw)).float()
            torch.cuda.synchronize()
            ref = outs["before"]
            err = {vn: round(((o - ref).norm() / ref.norm()).item(), 6) for vn, o in outs.items()}
            del outs
            times = {v[0]: [] for v in variants}
            times["hipblaslt"] = []

            def timed(fn):
                for i in range(2):
                    fn(ws[i % ncopy])
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for i in range(a.iters):
                    fn(ws[i % ncopy])
                e.record()
                torch.cuda.synchronize()
                return s.elapsed_time(e) / a.iters * 1e3       # us
            for v in vops:
                times[v] = []
            for _ in range(a.rounds):
                for vn, mode, b, bn in variants:
                    k.fls_gemm_set_skinny(mode, b)
                    k.fls_gemm_set_skinny_bn(bn)
                    times[vn].append(timed(lambda w: ops.gemm(x, w, epi, **kw)))
                for v, o in vops.items():
                    o.k.fls_gemm_set_skinny(2, 0)
                    times[v].append(timed(lambda w: o.gemm(x, w, epi, **kw)))
                times["hipblaslt"].append(timed(lambda w: torch.matmul(x, w.t())))
            k.fls_gemm_set_skinny(1, 0)
            k.fls_gemm_set_skinny_bn(0)
            med = {v: sorted(t)[len(t) // 2] for v, t in times.items()}
            print(json.dumps({"op": name, "M": M, "N": N, "K": K, "rel_err_vs_before": err,
                              "us": {v: round(t, 1) for v, t in med.items()},
                              "weight_TBps": {v: round(wbytes / (t * 1e-6) / 1e12, 2) for v, t in med.items()}}),
                  flush=True)
            del x, r
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
