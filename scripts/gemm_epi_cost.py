"""Cost of each fused epilogue: the same GEMM shape with EPI none vs RoPE / residual / SwiGLU
(70B and 7B projection shapes at M = 14336).  Interleaved rounds, median, TFLOP/s."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.config import preset  # noqa: E402
from flexible_llm_sharding_amd.models.llama import rope_tables  # noqa: E402
from flexible_llm_sharding_amd.ops.hip_backend import EPI_NONE, EPI_RESID, EPI_ROPE, EPI_SWIGLU, HipOps  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ops = HipOps()
    M = 14336
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for model in ("llama2-70b", "llama2-7b"):
        cfg = preset(model)
        H, I, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
        cos, sin = (t.to(dev) for t in rope_tables(cfg, 4096))
        pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=dev)
        x = (torch.rand(M, H, device=dev) * 2 - 1).half()
        xi = (torch.rand(M, I, device=dev) * 2 - 1).half()
        shapes = {
            "qkv": (x, ((torch.rand(cfg.qkv_size, H, device=dev) * 2 - 1) * 0.02).half(), EPI_ROPE),
            "o": (x, ((torch.rand(H, H, device=dev) * 2 - 1) * 0.02).half(), EPI_RESID),
            "gateup": (x, ((torch.rand(2 * I, H, device=dev) * 2 - 1) * 0.02).half(), EPI_SWIGLU),
            "down": (xi, ((torch.rand(H, I, device=dev) * 2 - 1) * 0.02).half(), EPI_RESID),
        }
        r = torch.randn(M, H, device=dev).half()
        for name, (a, w, epi) in shapes.items():
            N, K = w.shape
            kw = {}
            if epi == EPI_ROPE:
                kw = dict(positions=pos, cos=cos, sin=sin,
                          rope_cols=(cfg.num_attention_heads + cfg.num_key_value_heads) * hd, head_dim=hd)
            out_none = torch.empty(M, N, dtype=torch.float16, device=dev)
            out_epi = r.clone() if epi == EPI_RESID else None
            fns = {"none": lambda: ops.gemm(a, w, EPI_NONE, out=out_none),
                   "epi": (lambda: ops.gemm(a, w, epi, out=out_epi, resid=out_epi)) if epi == EPI_RESID else
                          (lambda: ops.gemm(a, w, epi, **kw))}
            ts = {k: [] for k in fns}
            for rnd in range(7):
                for k, f in fns.items():
                    f()
                    ev[0].record()
                    for _ in range(3):
                        f()
                    ev[1].record()
                    torch.cuda.synchronize()
                    ts[k].append(ev[0].elapsed_time(ev[1]) / 3)
            fl = 2.0 * M * N * K
            row = {k: round(fl / statistics.median(v[1:]) / 1e9, 1) for k, v in ts.items()}
            print(json.dumps({"model": model, "shape": name, "N": N, "K": K, "tflops": row}), flush=True)
        del shapes, x, xi


if __name__ == "__main__":
    main()
