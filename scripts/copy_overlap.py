"""Does the weight stream (pinned H2D) slow the GEMMs it overlaps with?

hipMemcpyAsync of a 1.7 GB layer from pinned memory shows up in rocprof as a
256-workgroup ``__amd_rocclr_copyBuffer`` shader.  A one-wave-per-SIMD GEMM
(v9, hipBLASLt's MT256x256) needs a whole SIMD register file, so resident blit
waves can keep GEMM blocks off CUs.  This runs, per runtime setting (each in a
fresh child process, since the env must be set before HIP initialises):

  gemm alone | copy alone | gemm + concurrent copy (two streams)

    python scripts/copy_overlap.py            # parent: loops over settings
"""
import json
import os
import subprocess
import sys
import time

SETTINGS = {
    "default": {},
    "limit_blit_wg16": {"DEBUG_CLR_LIMIT_BLIT_WG": "16"},
    "limit_blit_wg4": {"DEBUG_CLR_LIMIT_BLIT_WG": "4"},
    "sdma_on": {"HSA_ENABLE_SDMA": "1"},
    "sdma_off": {"HSA_ENABLE_SDMA": "0"},
}


def child():
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from flexible_llm_sharding_amd.ops.hip_backend import HipOps, EPI_SWIGLU
    from flexible_llm_sharding_amd.runtime.hostmem import alloc_host
    dev = torch.device("cuda", 0)
    ops = HipOps()
    ops.backend = os.environ.get("CO_BACKEND", "hip")
    M, N, K = 16128, 57344, 8192
    x = (torch.rand(M, K, device=dev) * 2 - 1).half()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.02).half()
    nb = 1_711_276_032
    h = alloc_host(nb)
    d = torch.empty(nb, dtype=torch.uint8, device=dev)
    side = torch.cuda.Stream(dev)
    gemm_iters = 3

    def gemms():
        for _ in range(gemm_iters):
            ops.swiglu_up(x, w)

    def copy():
        with torch.cuda.stream(side):
            d.copy_(h, non_blocking=True)

    # warm
    gemms(); copy(); torch.cuda.synchronize()
    res = {}
    for rep in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); gemms(); e1.record(); torch.cuda.synchronize()
        res.setdefault("gemm_alone_ms", []).append(e0.elapsed_time(e1) / gemm_iters)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record(side); copy(); c1.record(side); torch.cuda.synchronize()
        res.setdefault("copy_alone_ms", []).append(c0.elapsed_time(c1))
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record(side); copy(); c1.record(side)
        e0.record(); gemms(); e1.record()
        torch.cuda.synchronize()
        res.setdefault("gemm_with_copy_ms", []).append(e0.elapsed_time(e1) / gemm_iters)
        res.setdefault("copy_with_gemm_ms", []).append(c0.elapsed_time(c1))
    # bandwidth-bound kernel next to the streams: rmsnorm over [16128, 8192]
    xr = torch.randn(16128, 8192, device=dev).half()
    wn = torch.randn(8192, device=dev).half()
    hd = alloc_host(nb)

    def norms():
        for _ in range(20):
            ops.rmsnorm(xr, wn, 1e-5)

    norms(); torch.cuda.synchronize()
    for rep in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); norms(); e1.record(); torch.cuda.synchronize()
        res.setdefault("rmsnorm_alone_ms", []).append(e0.elapsed_time(e1) / 20)
        copy()
        e0.record(); norms(); e1.record(); torch.cuda.synchronize()
        res.setdefault("rmsnorm_with_h2d_ms", []).append(e0.elapsed_time(e1) / 20)
        with torch.cuda.stream(side):
            hd.copy_(d, non_blocking=True)
        e0.record(); norms(); e1.record(); torch.cuda.synchronize()
        res.setdefault("rmsnorm_with_d2h_ms", []).append(e0.elapsed_time(e1) / 20)
    out = {k: round(min(v), 3) for k, v in res.items()}
    out["copy_GBps_alone"] = round(nb / out["copy_alone_ms"] / 1e6, 1)
    print("RESULT " + json.dumps(out), flush=True)


def main():
    rows = {}
    names = sys.argv[1:] or list(SETTINGS)
    for backend in ("hip", "hipblaslt"):
        for name in names:
            env = dict(os.environ, **SETTINGS[name], CO_BACKEND=backend)
            t0 = time.time()
            p = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                               timeout=300)
            line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")]
            rows[f"{backend}/{name}"] = json.loads(line[0][7:]) if line else {"rc": p.returncode,
                                                                               "err": p.stderr[-400:]}
            print(f"{backend}/{name}", rows[f"{backend}/{name}"], f"{time.time() - t0:.0f}s", flush=True)
            if p.returncode != 0:
                sys.exit(p.returncode)
    out = os.environ.get("CO_JSON")
    if out:
        with open(out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    if "--child" in sys.argv:
        child()
    else:
        main()
