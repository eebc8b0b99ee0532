"""A/B of GEMM kernel-library variants (``build.py --variant NAME --define ...``) against the in-tree
build on the 70B production shapes, interleaved rounds in ONE process (guide §5.4 rule 24):
v10 (in-tree, v11 off), v11 (in-tree), v11 of every variant library, hipBLASLt (plain epilogue).

    python scripts/gemm_variant_ab.py --variants s2 [--rounds 3] [--mchunk 12288]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd import _native  # noqa: E402
from flexible_llm_sharding_amd.ops.hip_backend import EPI_RESID, EPI_ROPE, EPI_SWIGLU, HipOps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--mchunk", type=int, default=12288)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    main_ops = HipOps()
    arms = [("v10", main_ops, 0), ("v11", main_ops, 2)]
    for v in [x for x in a.variants.split(",") if x]:
        o = HipOps()
        o.k = _native._load_kernels(os.path.join(os.path.dirname(_native.__file__), "variants",
                                                 f"libfls_kernels_{v}.so"))
        arms.append((f"v11_{v}", o, 2))
    H, I, nh, nkv, hd = 8192, 28672, 64, 8, 128
    mc = a.mchunk
    shapes = [("qkv_rope", mc, (nh + 2 * nkv) * hd, H, EPI_ROPE), ("o_resid", 43008, H, H, EPI_RESID),
              ("gateup_swiglu", mc, 2 * I, H, EPI_SWIGLU), ("down_resid", mc, H, I, EPI_RESID)]
    if a.only:
        shapes = [s for s in shapes if s[0] in a.only.split(",")]
    pos = torch.randint(0, 4096, (43008,), dtype=torch.int32, device=dev)
    cos = torch.rand(4096, hd // 2, device=dev)
    sin = torch.rand(4096, hd // 2, device=dev)
    for name, M, N, K, epi in shapes:
        x = (torch.rand(M, K, device=dev) * 2 - 1).half()
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
        r = torch.randn(M, N, device=dev).half()
        kw = {}
        if epi == EPI_RESID:
            kw = dict(out=r, resid=r)
        if epi == EPI_ROPE:
            kw = dict(positions=pos[:M], cos=cos, sin=sin, rope_cols=(nh + nkv) * hd, head_dim=hd)
        # every arm's output equals v10's (bitwise; RoPE within 1 ulp is not checked here)
        same = {}
        if epi != EPI_ROPE:
            ref = None
            for an, ops, mode in arms:
                ops.k.fls_gemm_set_v11(mode)
                if epi == EPI_RESID:
                    rc = r.clone()
                    y = ops.gemm(x, w, epi, out=rc, resid=rc)
                else:
                    y = ops.gemm(x, w, epi)
                torch.cuda.synchronize()
                if ref is None:
                    ref = y
                same[an] = bool(torch.equal(y, ref))
                del y
            del ref
        fl = 2.0 * M * N * K
        times = {an: [] for an, _, _ in arms}
        times["hipblaslt"] = []
        for _ in range(a.rounds):
            for an, ops, mode in arms:
                ops.k.fls_gemm_set_v11(mode)
                for _ in range(2):
                    ops.gemm(x, w, epi, **kw)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    ops.gemm(x, w, epi, **kw)
                e.record()
                torch.cuda.synchronize()
                times[an].append(s.elapsed_time(e) / a.iters / 1e3)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                torch.matmul(x, w.t())
            e.record()
            torch.cuda.synchronize()
            times["hipblaslt"].append(s.elapsed_time(e) / a.iters / 1e3)
        for _, ops, _ in arms:
            ops.k.fls_gemm_set_v11(1)
        row = {"op": name, "M": M, "N": N, "K": K, "bitwise_v10": same,
               "tflops": {v: round(fl / sorted(t)[len(t) // 2] / 1e12, 1) for v, t in times.items()}}
        print(json.dumps(row), flush=True)
        del x, w, r
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
