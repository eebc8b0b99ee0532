"""Microbenchmarks of the hot HIP kernels on Llama-2-70B shapes (random data),
with hipBLASLt (torch.matmul) as the library reference point.

    python scripts/kernel_bench.py [--m 16384] [--iters 20] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd.ops.hip_backend import HipOps, EPI_NONE, EPI_RESID, EPI_SWIGLU, EPI_ROPE  # noqa


def timeit(fn, iters, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = HipOps()
    H, I, nh, nkv, hd = 8192, 28672, 64, 8, 128
    M = a.m
    res = []
    shapes = [("qkv_rope", (nh + 2 * nkv) * hd, H, EPI_ROPE), ("o_resid", H, H, EPI_RESID),
              ("gateup_swiglu", 2 * I, H, EPI_SWIGLU), ("down_resid", H, I, EPI_RESID),
              ("lm_head_m160", 32000, H, EPI_NONE)]
    pos = torch.randint(0, 4096, (M,), dtype=torch.int32, device=dev)
    cos = torch.rand(4096, hd // 2, device=dev)
    sin = torch.rand(4096, hd // 2, device=dev)
    for name, N, K, epi in shapes:
        m = 160 if name.startswith("lm_head") else M
        x = (torch.rand(m, K, device=dev) * 2 - 1).half()
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
        r = torch.randn(m, N, device=dev).half()
        kw = {}
        if epi == EPI_RESID:
            kw = dict(out=r, resid=r)
        if epi == EPI_ROPE:
            kw = dict(positions=pos, cos=cos, sin=sin, rope_cols=(nh + nkv) * hd, head_dim=hd)
        fl = 2.0 * m * N * K
        row = {"op": name, "M": m, "N": N, "K": K}
        # correctness of each variant vs hipBLASLt (plain epilogue)
        ref = torch.matmul(x, w.t()).float()
        y = ops.gemm(x, w)
        err = ((y.float() - ref).norm() / ref.norm()).item()
        t = timeit(lambda: ops.gemm(x, w, epi, **kw), a.iters)
        row.update({"v10_ms": t * 1e3, "v10_tflops": fl / t / 1e12, "v10_relerr": err})
        tl = timeit(lambda: torch.matmul(x, w.t()), a.iters)
        row.update({"hipblaslt_ms": tl * 1e3, "hipblaslt_tflops": fl / tl / 1e12})
        res.append(row)
        print(json.dumps(row), flush=True)
    # skinny LM head (one prompt x 5 suffixes): weight-streaming GEMV vs hipBLASLt
    xs = (torch.rand(5, H, device=dev) * 2 - 1).half()
    wl = ((torch.rand(32000, H, device=dev) * 2 - 1) * 0.02).half()
    tg = timeit(lambda: ops.gemv_skinny(xs, wl), a.iters)
    tb = timeit(lambda: torch.matmul(xs, wl.t()), a.iters)
    row = {"op": "lm_head_m5_gemv", "ours_ms": tg * 1e3, "ours_GBps": wl.numel() * 2 / tg / 1e9,
           "hipblaslt_ms": tb * 1e3}
    res.append(row)
    print(json.dumps(row), flush=True)
    # attention: 12 prompts of prefix 1024 + 5 x 64 suffixes
    from flexible_llm_sharding_amd.runtime.batch import pack_prompts
    from flexible_llm_sharding_amd.utils.tokenizer import TokenizedPrompt
    tps = [TokenizedPrompt(list(range(1024)), [list(range(64))] * 5, 64, [63] * 5) for _ in range(12)]
    b = pack_prompts(tps, list(range(12)), "bidirectional")
    meta = b.device_tensors(dev)
    qkv = torch.randn(b.num_tokens, (nh + 2 * nkv) * hd, device=dev).half()
    from flexible_llm_sharding_amd.models.llama import layer_flops
    from flexible_llm_sharding_amd.config import preset
    cfg = preset("llama2-70b")
    cases = [("p1024_s5x64", b, meta, qkv)]
    tps4 = [TokenizedPrompt(list(range(4096)), [list(range(64))] * 5, 64, [63] * 5) for _ in range(3)]
    b4 = pack_prompts(tps4, list(range(3)), "bidirectional")
    cases.append(("p4096_s5x64", b4, b4.device_tensors(dev),
                  torch.randn(b4.num_tokens, (nh + 2 * nkv) * hd, device=dev).half()))
    for cname, bb, mm, qq in cases:
        att_fl = layer_flops(cfg, bb) - 2.0 * bb.num_tokens * cfg.decoder_layer_params()
        row = {"op": "attention_shared_prefix", "case": cname, "tokens": bb.num_tokens}
        t = timeit(lambda: ops.attention(qq, mm["work"], nh, nkv, hd, seg_lo=mm["seg_lo"]), a.iters)
        row.update({"ours_ms": t * 1e3, "ours_tflops": att_fl / t / 1e12})
        res.append(row)
        print(json.dumps(row), flush=True)
    x = torch.randn(M, H, device=dev).half()
    wln = torch.randn(H, device=dev).half()
    t = timeit(lambda: ops.rmsnorm(x, wln, 1e-5), a.iters)
    row = {"op": "rmsnorm", "rows": M, "H": H, "ours_ms": t * 1e3, "GBps": 2 * M * H * 2 / t / 1e9}
    res.append(row)
    print(json.dumps(row), flush=True)
    # host<->device copy bandwidth (pinned), the streaming bound
    from flexible_llm_sharding_amd.runtime.hostmem import alloc_host
    nb = 1 << 30
    h = alloc_host(nb)
    d = torch.empty(nb, dtype=torch.uint8, device=dev)
    t = timeit(lambda: d.copy_(h, non_blocking=True), 5, 1)
    t2 = timeit(lambda: h.copy_(d, non_blocking=True), 5, 1)
    row = {"op": "pinned_copy_1GiB", "h2d_GBps": nb / t / 1e9, "d2h_GBps": nb / t2 / 1e9}
    res.append(row)
    print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
