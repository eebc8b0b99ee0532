"""GEMM v10 tile-order sweep on the 70B projection shapes at one micro-batch (M = 14336):
GM M-tiles grouped per N-tile (default 8) vs other group sizes and N-grouped orders.
Interleaved rounds, median; EPI none (fls_gemm_ablate entries 80-86)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd import _native  # noqa: E402

ORDERS = {80: "gm2", 81: "gm4", 82: "gm8 (default)", 83: "gm16", 84: "gn4", 85: "gn8", 86: "gn16",
          87: "gn2", 88: "gm1", 89: "gm8 (repeat)"}
SHAPES = {"gateup": (14336, 57344, 8192), "down": (14336, 8192, 28672), "o": (14336, 8192, 8192),
          "qkv": (14336, 10240, 8192)}


def main():
    dev = torch.device("cuda", 0)
    k = _native.kernels()
    s = torch.cuda.current_stream().cuda_stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    out = {}
    for name, (M, N, K) in SHAPES.items():
        x = (torch.rand(M, K, device=dev) * 2 - 1).half()
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
        c = torch.empty(M, N, dtype=torch.float16, device=dev)
        times = {a: [] for a in ORDERS}
        for rnd in range(int(os.environ.get("ROUNDS", "9"))):
            for a in ORDERS:
                ev[0].record()
                for _ in range(3):
                    assert k.fls_gemm_ablate(a, x.data_ptr(), w.data_ptr(), c.data_ptr(), M, N, K, s) == 0
                ev[1].record()
                torch.cuda.synchronize()
                times[a].append(ev[0].elapsed_time(ev[1]) / 3)
        fl = 2.0 * M * N * K
        out[name] = {nm: round(fl / statistics.median(times[a][1:]) / 1e9, 1) for a, nm in ORDERS.items()}
        print(json.dumps({name: out[name]}), flush=True)
        del x, w, c


if __name__ == "__main__":
    main()
