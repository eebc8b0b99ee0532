"""Do host-to-device copies on two streams overlap, or does the second wait for the first?

A 1.41 GB copy (a 70B MLP weight piece) is enqueued on stream 1, then a 176 MB copy (an activation
reload) on stream 2 right behind it; the probe reports when the small copy finishes, measured from
the moment both were enqueued.  ~3.5 ms: the copies run side by side (the small one shares PCIe);
~30 ms: the small copy waited behind the large one.  Also: the large copy cut into 64 MB pieces,
a device-to-host copy next to the large host-to-device one, and each direction next to a
long compute kernel that fills every CU (a copy done by a blit kernel has to wait for CUs).

    python scripts/copy_concurrency_probe.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexible_llm_sharding_amd.runtime.hostmem import alloc_host  # noqa: E402


def ms(a, b):
    return a.elapsed_time(b)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    big, small = 1409 << 20, 176 << 20
    hA, hB = alloc_host(big), alloc_host(small)
    dA = torch.empty(big, dtype=torch.uint8, device=dev)
    dB = torch.empty(small, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def ev(s):
        e = torch.cuda.Event(enable_timing=True)
        e.record(s)
        return e

    def run(case):
        torch.cuda.synchronize()
        t0 = ev(torch.cuda.current_stream())
        s1.wait_event(t0)
        s2.wait_event(t0)
        with torch.cuda.stream(s1):
            if case == "chunked":
                for o in range(0, big, 64 << 20):
                    dA[o:o + (64 << 20)].copy_(hA[o:o + (64 << 20)], non_blocking=True)
            else:
                dA.copy_(hA, non_blocking=True)
            eA = ev(s1)
        with torch.cuda.stream(s2):
            if case == "d2h":
                hB.copy_(dB, non_blocking=True)
            else:
                dB.copy_(hB, non_blocking=True)
            eB = ev(s2)
        torch.cuda.synchronize()
        return ms(t0, eA), ms(t0, eB)

    for case in ("h2d", "chunked", "d2h"):
        for rep in range(3):
            a, b = run(case)
            print(f"{case:8s} rep {rep}: large copy done at {a:6.2f} ms, small copy done at {b:6.2f} ms", flush=True)
    # copies next to a long compute kernel that fills every CU: an SDMA copy finishes in its own
    # time, a copy done by a blit kernel waits for CUs
    x = torch.randn(16384, 8192, device=dev, dtype=torch.float16)
    w = torch.randn(16384, 8192, device=dev, dtype=torch.float16)
    for case in ("gemm+d2h", "gemm+h2d"):
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = ev(torch.cuda.current_stream())
            s1.wait_event(t0)
            s2.wait_event(t0)
            with torch.cuda.stream(s1):
                for _ in range(3):
                    y = x @ w.t()
                eG = ev(s1)
            with torch.cuda.stream(s2):
                if case == "gemm+d2h":
                    hB.copy_(dB, non_blocking=True)
                else:
                    dB.copy_(hB, non_blocking=True)
                eB = ev(s2)
            torch.cuda.synchronize()
            print(f"{case:9s} rep {rep}: compute done at {ms(t0, eG):6.2f} ms, copy done at {ms(t0, eB):6.2f} ms",
                  flush=True)
            del y
    # control: the small copy alone
    torch.cuda.synchronize()
    t0 = ev(torch.cuda.current_stream())
    dB.copy_(hB, non_blocking=True)
    t1 = ev(torch.cuda.current_stream())
    torch.cuda.synchronize()
    print(f"small copy alone: {ms(t0, t1):.2f} ms")
    time.sleep(0.1)


if __name__ == "__main__":
    main()
