"""A/B at generation-step row counts: the wide 70B gate/up + SwiGLU GEMM on the default path
(main / skinny rules) vs the 64 x 128 mid kernel forced (fls_gemm_set_mid(2)) vs hipBLASLt (plain).
Weights rotate over > 600 MB so none stay in the Infinity Cache."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.ops.hip_backend import EPI_RESID, EPI_SWIGLU, HipOps  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ops = HipOps()
    H, I = 8192, 28672
    for name, N, K, epi in (("gateup_swiglu", 2 * I, H, EPI_SWIGLU), ("down_resid", H, I, EPI_RESID)):
        ncopy = max(1, -(-600_000_000 // (N * K * 2)))
        ws = [((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half() for _ in range(ncopy)]
        for M in (64, 128, 160, 192, 256):
            x = (torch.rand(M, K, device=dev) * 2 - 1).half()
            r = torch.randn(M, N, device=dev).half()

            def timed(fn, iters=8):
                for i in range(2):
                    fn(ws[i % ncopy])
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for i in range(iters):
                    fn(ws[i % ncopy])
                e.record()
                torch.cuda.synchronize()
                return s.elapsed_time(e) / iters * 1e3
            kw = dict(out=r, resid=r) if epi == EPI_RESID else {}
            res = {"default": [], "mid": [], "hipblaslt": []}
            outs = {}
            for mode, key in ((1, "default"), (2, "mid")):
                ops.k.fls_gemm_set_mid(mode)
                outs[key] = ops.gemm(x, ws[0], epi).float() if epi != EPI_RESID else None
            for _ in range(3):
                for mode, key in ((1, "default"), (2, "mid")):
                    ops.k.fls_gemm_set_mid(mode)
                    res[key].append(timed(lambda w: ops.gemm(x, w, epi, **kw)))
                res["hipblaslt"].append(timed(lambda w: torch.matmul(x, w.t())))
            ops.k.fls_gemm_set_mid(1)
            err = None
            if outs["default"] is not None:
                err = round(((outs["mid"] - outs["default"]).norm() / outs["default"].norm()).item(), 6)
            med = {k: round(sorted(v)[1], 1) for k, v in res.items()}
            print(json.dumps({"op": name, "M": M, "us": med, "rel_err_mid": err}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
