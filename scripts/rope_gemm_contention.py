"""Persistent (v13) vs non-persistent (v10) QKV+RoPE GEMM while other kernels hold a few CUs.

Under world > 1 the RCCL all-gather / send-recv kernels co-run with the projection GEMMs. This stands
them in with `torch.cuda._sleep` spin kernels on side streams (one block each, each pinning one CU's
SIMD for the whole GEMM), and times the 70B QKV+RoPE GEMM with each variant.

    python scripts/rope_gemm_contention.py [--m 16128] [--spinners 0 1 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.ops.hip_backend import HipOps, EPI_ROPE  # noqa


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16128)
    ap.add_argument("--spinners", type=int, nargs="+", default=[0, 1, 3])
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    M, H, nh, nkv = a.m, 8192, 64, 8
    N, rc = (nh + 2 * nkv) * 128, (nh + nkv) * 128
    pos = torch.randint(0, 4096, (M,), dtype=torch.int32, device=dev)
    cos, sin = torch.rand(4096, 64, device=dev), torch.rand(4096, 64, device=dev)
    x = (torch.rand(M, H, device=dev) * 2 - 1).half()
    w = ((torch.rand(N, H, device=dev) * 2 - 1) * 0.02).half()
    kw = dict(positions=pos, cos=cos, sin=sin, rope_cols=rc, head_dim=128)
    side = [torch.cuda.Stream(dev) for _ in range(max(a.spinners))] if max(a.spinners) else []
    ops.k.fls_gemm_set_variant(10)
    for persist in (0, 1, 0, 1):
        ops.k.fls_gemm_set_rope_persistent(persist)
        for ns in a.spinners:
            ops.gemm(x, w, EPI_ROPE, **kw)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for st in side[:ns]:
                with torch.cuda.stream(st):
                    torch.cuda._sleep(int(3e8))        # ~100+ ms spin, longer than the timed loop
            s.record()
            for _ in range(a.iters):
                ops.gemm(x, w, EPI_ROPE, **kw)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / a.iters
            print(json.dumps({"variant": "v13" if persist else "v10", "spinners": ns, "ms": round(ms, 4),
                              "tflops": round(2.0 * M * N * H / ms / 1e9, 1)}), flush=True)
    ops.k.fls_gemm_set_rope_persistent(1)


if __name__ == "__main__":
    main()
