"""GEMM main-loop ablation (guide §7 'The diagnostic loop', step 2): interleaved
rounds of the full v1 loop vs. builds with LDS-DMA / ds_reads / MFMAs removed."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd import _native  # noqa: E402

NAMES = {0: "full", 1: "no_dma", 2: "no_lds_read", 3: "mfma_only", 4: "no_mfma", 5: "lds_read_only",
         6: "dma_only", 10: "v4_full", 11: "v4_no_dma", 14: "v4_no_mfma",
         20: "v1_groupN_full", 26: "v1_groupN_dma_only",
         40: "v10_full", 41: "v10_no_dma", 42: "v10_no_lds_read", 43: "v10_mfma_only",
         45: "v10_no_dma_no_sync", 47: "v10_mfma_only_no_sync", 50: "v11_full",
         60: "v10_sched0", 61: "v10_sched1_dma_first", 62: "v10_sched2_spread", 63: "v10_sched3_front",
         70: "v12_full", 71: "v12_no_dma"}
if os.environ.get("ABL_ONLY"):
    NAMES = {k: v for k, v in NAMES.items() if k >= int(os.environ["ABL_ONLY"])}


def main():
    M, N, K = 16128, 57344, 8192
    dev = torch.device("cuda", 0)
    k = _native.kernels()
    x = (torch.rand(M, K, device=dev) * 2 - 1).half()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
    c = torch.empty(M, N, dtype=torch.float16, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    times = {a: [] for a in NAMES}
    tl = []
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for rnd in range(6):
        for a in NAMES:
            ev[0].record()
            for _ in range(3):
                assert k.fls_gemm_ablate(a, x.data_ptr(), w.data_ptr(), c.data_ptr(), M, N, K, s) == 0
            ev[1].record()
            torch.cuda.synchronize()
            times[a].append(ev[0].elapsed_time(ev[1]) / 3)
        ev[0].record()
        for _ in range(3):
            torch.matmul(x, w.t(), out=c)
        ev[1].record()
        torch.cuda.synchronize()
        tl.append(ev[0].elapsed_time(ev[1]) / 3)
    fl = 2.0 * M * N * K
    res = {}
    for a, nm in NAMES.items():
        med = statistics.median(times[a][1:])
        res[nm] = {"ms": round(med, 3), "tflops_equiv": round(fl / med / 1e9, 1)}
    med = statistics.median(tl[1:])
    res["hipblaslt"] = {"ms": round(med, 3), "tflops_equiv": round(fl / med / 1e9, 1)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
