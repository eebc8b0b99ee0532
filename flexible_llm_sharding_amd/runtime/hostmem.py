"""Host memory + file I/O helpers on top of the native runtime.

* :func:`alloc_host` — exact-size pinned buffers from ``hipHostMalloc``
  (PyTorch's caching host allocator rounds to powers of two: a 1.71 GB 70B
  layer would take 2 GB), wrapped as uint8 CPU tensors; falls back to
  pageable memory when no GPU is present.
* :func:`read_safetensors` — header via the native index, tensor bytes with
  the multi-threaded ``pread`` engine into one host buffer, zero-copy views.
"""
from __future__ import annotations

import ctypes
import os
import time
from typing import Dict

import torch

from .. import _native, knobs
from ..utils import safetensors_io

_IO_THREADS = knobs.get_int("FLS_IO_THREADS")

# pinned bytes currently held / high-water mark (alloc_host blocks; the streamer's ring is
# reported by runtime.stream separately)
pinned_live = 0
pinned_peak = 0
# alloc_host calls and their host seconds (hipHostMalloc is slow: a pass should reuse pooled
# buffers, not allocate; engine stats report the per-call counts)
alloc_calls = 0
alloc_seconds = 0.0


def _count(n: int) -> None:
    global pinned_live, pinned_peak
    pinned_live += n
    pinned_peak = max(pinned_peak, pinned_live)


class _PinnedOwner:
    __slots__ = ("ptr", "lib", "n", "__weakref__")

    def __init__(self, ptr, lib, n):
        self.ptr, self.lib, self.n = ptr, lib, n
        _count(n)

    def __del__(self):
        try:
            if self.ptr:
                self.lib.fls_pinned_free(self.ptr)
                self.ptr = None
                _count(-self.n)
        except Exception:
            pass


def _gpu_present() -> bool:
    try:
        return torch.cuda.is_available()
    except Exception:
        return False


def alloc_host(nbytes: int, pinned: bool = True) -> torch.Tensor:
    """uint8 CPU tensor of exactly ``nbytes`` (pinned when a GPU is present).

    The pinned block is owned by a ctypes array object that every tensor view
    keeps alive (``torch.frombuffer`` holds a reference), so the memory is
    ``hipHostFree``d exactly when the last view dies.
    """
    if pinned and _gpu_present():
        global alloc_calls, alloc_seconds
        rt = _native.runtime_or_none()
        if rt is not None:
            n = max(1, nbytes)
            t0 = time.perf_counter()
            ptr = rt.fls_pinned_alloc(n)
            alloc_calls += 1
            alloc_seconds += time.perf_counter() - t0
            if ptr:
                arr_t = type("PinnedBlock", (ctypes.c_uint8 * n,), {})
                arr = arr_t.from_address(ptr)
                arr.owner = _PinnedOwner(ptr, rt, n)
                return torch.frombuffer(arr, dtype=torch.uint8)[:nbytes]
        return torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    return torch.empty(nbytes, dtype=torch.uint8)


class _DeviceBlock:
    """A raw hipMalloc block exposed to torch through ``__cuda_array_interface__`` (zero copy;
    the tensor keeps this object alive, ``hipFree`` when the last view dies)."""

    def __init__(self, ptr: int, nbytes: int, device: int, lib):
        self.ptr, self.nbytes, self.device, self.lib = ptr, nbytes, device, lib
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}

    def __del__(self):
        try:
            if self.ptr:
                self.lib.fls_device_free(self.device, self.ptr)
                self.ptr = None
        except Exception:
            pass


def alloc_device(nbytes: int, device: torch.device) -> torch.Tensor:
    """uint8 device tensor of exactly ``nbytes`` allocated outside PyTorch's caching allocator
    (weight slots: one allocation per run, so they never fragment the per-stream pools the
    activations use).  Falls back to ``torch.empty`` if the native runtime is unavailable."""
    dev = torch.device(device)
    rt = _native.runtime_or_none()
    if rt is not None and dev.type == "cuda":
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        ptr = rt.fls_device_alloc(idx, max(1, nbytes))
        if not ptr:
            raise torch.cuda.OutOfMemoryError(f"hipMalloc of {nbytes / 1e9:.2f} GB failed on {dev}")
        t = torch.as_tensor(_DeviceBlock(ptr, max(1, nbytes), idx, rt), device=dev)
        return t[:nbytes]
    return torch.empty(nbytes, dtype=torch.uint8, device=dev)


def pread_into(path: str, offset: int, nbytes: int, dst: torch.Tensor) -> None:
    """Read ``nbytes`` at ``offset`` of ``path`` into a contiguous CPU tensor."""
    assert dst.device.type == "cpu" and dst.is_contiguous()
    assert dst.numel() * dst.element_size() >= nbytes
    if nbytes == 0:
        return
    rt = _native.runtime_or_none()
    if rt is not None:
        r = rt.fls_pread_into(path.encode(), offset, nbytes, dst.data_ptr(), _IO_THREADS)
        if r != nbytes:
            raise IOError(f"pread {path} @{offset}+{nbytes} failed: {r}")
        return
    with open(path, "rb") as f:
        f.seek(offset)
        mv = memoryview(dst.view(-1).view(torch.uint8).numpy())[:nbytes]
        if f.readinto(mv) != nbytes:
            raise IOError(f"short read {path}")


def pwrite_from(path: str, src: torch.Tensor, nbytes: int = None) -> None:
    n = src.numel() * src.element_size() if nbytes is None else nbytes
    rt = _native.runtime_or_none()
    if rt is not None:
        r = rt.fls_pwrite_from(path.encode(), 0, n, src.data_ptr(), _IO_THREADS, 1)
        if r != n:
            raise IOError(f"pwrite {path} failed: {r}")
        return
    with open(path, "wb") as f:
        f.write(memoryview(src.contiguous().view(-1).view(torch.uint8).numpy())[:n])


def read_header_native(path: str):
    rt = _native.runtime_or_none()
    if rt is None:
        return None
    h = rt.fls_st_open(path.encode())
    if not h:
        raise ValueError(f"{path}: cannot parse safetensors header")
    try:
        out = {}
        name = ctypes.create_string_buffer(1024)
        dt = ctypes.create_string_buffer(16)
        shape = (ctypes.c_int64 * 8)()
        nd = ctypes.c_int()
        b, e = ctypes.c_uint64(), ctypes.c_uint64()
        for i in range(rt.fls_st_count(h)):
            rc = rt.fls_st_info(h, i, name, 1024, dt, 16, ctypes.addressof(shape), ctypes.byref(nd),
                                ctypes.byref(b), ctypes.byref(e))
            if rc != 0:
                raise ValueError(f"{path}: bad entry {i} ({rc})")
            nm = name.value.decode()
            out[nm] = safetensors_io.TensorInfo(nm, safetensors_io.DTYPES[dt.value.decode()],
                                                tuple(shape[:nd.value]), b.value, e.value)
        return out
    finally:
        rt.fls_st_close(h)


def read_safetensors(path: str) -> Dict[str, torch.Tensor]:
    infos = read_header_native(path)
    if infos is None:
        return safetensors_io.load_file(path)
    if not infos:
        return {}
    lo = min(t.begin for t in infos.values())
    hi = max(t.end for t in infos.values())
    buf = torch.empty(hi - lo, dtype=torch.uint8)
    pread_into(path, lo, hi - lo, buf)
    out = {}
    for n, t in infos.items():
        if not t.nbytes:
            out[n] = torch.empty(t.shape, dtype=t.dtype)
            continue
        v = buf[t.begin - lo:t.end - lo]
        es = torch.empty((), dtype=t.dtype).element_size()
        if (t.begin - lo) % es:
            v = v.clone()          # misaligned tensor start: realign before the dtype view
        out[n] = v.view(t.dtype).view(t.shape)
    return out
