"""Run one GEMM shape for profiling (rocprofv3 --pmc): python scripts/gemm_one.py WHICH [M N K] [iters]

WHICH 0: the hand-written v10 kernel (256 x 256 tile); 11: v11 (384 x 256 tile, gemm_v11.hip);
< 0: hipBLASLt (torch.matmul) for comparison.  EPI (optional 6th arg): 0 plain, 1 residual, 2 SwiGLU."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.ops.hip_backend import HipOps, EPI_NONE  # noqa: E402


def main():
    var = int(sys.argv[1])
    M, N, K = (int(x) for x in sys.argv[2:5]) if len(sys.argv) >= 5 else (16128, 57344, 8192)
    iters = int(sys.argv[5]) if len(sys.argv) >= 6 else 10
    epi = int(sys.argv[6]) if len(sys.argv) >= 7 else 0
    dev = torch.device("cuda", 0)
    ops = HipOps()
    x = (torch.rand(M, K, device=dev) * 2 - 1).half()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
    out = torch.empty(M, N // 2 if epi == 2 else N, dtype=torch.float16, device=dev)
    if var >= 0:
        ops.k.fls_gemm_set_v11(2 if var == 11 else 0)
        kw = dict(resid=out) if epi == 1 else {}
        for _ in range(iters):
            ops.gemm(x, w, epi, out=out, **kw)
        torch.cuda.synchronize()
    if var < 0:
        full = torch.empty(M, N, dtype=torch.float16, device=dev)
        for _ in range(iters):
            torch.matmul(x, w.t(), out=full)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
