"""Does a host -> device weight copy hold device memory outside the caching allocator while it
runs?  1.41 GB (one 70B MLP piece) from an exact-size hipHostMalloc block (runtime/hostmem.py)
into a raw hipMalloc slot, by (a) torch ``copy_(non_blocking=True)`` (the piece pool's path),
(b) hipMemcpyAsync through the native runtime, (c) torch from a torch-pinned tensor.  A thread
samples hipMemGetInfo every 1 ms; prints the peak rise over the idle baseline and the enqueue time.

    python scripts/copy_probe.py
"""
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flexible_llm_sharding_amd import _native  # noqa: E402
from flexible_llm_sharding_amd.runtime import hostmem  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
N = 1_409_286_144
slot = hostmem.alloc_device(N, dev)
host = hostmem.alloc_host(N, pinned=True)
host_t = torch.empty(N, dtype=torch.uint8, pin_memory=True)
rt = _native.runtime_or_none()
stream = torch.cuda.Stream(dev)
torch.cuda.synchronize()


def used():
    free, total = torch.cuda.mem_get_info(dev)
    return total - free


peak = [0]
stop = threading.Event()


def sample():
    torch.cuda.set_device(dev)
    while not stop.is_set():
        peak[0] = max(peak[0], used())
        stop.wait(0.001)


th = threading.Thread(target=sample, daemon=True)
th.start()
print(f"host.is_pinned() = {host.is_pinned()}, torch-pinned source is_pinned() = {host_t.is_pinned()}", flush=True)


def run(name, fn, reps=4):
    torch.cuda.synchronize()
    time.sleep(0.05)
    base = used()
    peak[0] = base
    enq = []
    t0 = time.perf_counter()
    for _ in range(reps):
        a = time.perf_counter()
        with torch.cuda.stream(stream):
            fn()
        enq.append(time.perf_counter() - a)
    stream.synchronize()
    dt = time.perf_counter() - t0
    time.sleep(0.05)
    print(f"{name:34s} peak rise {(peak[0] - base) / 1e6:8.1f} MB   enqueue {max(enq) * 1e3:7.2f} ms max   "
          f"{reps * N / dt / 1e9:6.1f} GB/s", flush=True)


for _ in range(2):
    run("torch copy_ from hipHostMalloc", lambda: slot.copy_(host, non_blocking=True))
    run("hipMemcpyAsync from hipHostMalloc",
        lambda: rt.fls_memcpy_async(slot.data_ptr(), host.data_ptr(), N, 1, torch.cuda.current_stream().cuda_stream))
    run("torch copy_ from torch-pinned", lambda: slot.copy_(host_t, non_blocking=True))
    run("torch copy_ 256 MB pieces", lambda: [slot[o:o + (256 << 20)].copy_(host[o:o + (256 << 20)], non_blocking=True)
                                           for o in range(0, N - (256 << 20), 256 << 20)])
stop.set()
th.join()
