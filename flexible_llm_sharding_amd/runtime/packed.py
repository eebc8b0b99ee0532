"""Packed-layer disk cache (`--weight_cache packed`).

The reference re-reads every layer file from disk on every pass and
deserialises it on the CPU (``/root/reference/utils.py:72-73,126-130``).
Our per-layer safetensors files are in HF layout, and turning one into the
HBM-native packed layout (RoPE-pair row permutation, gate/up interleave,
bias packing: ``models/layout.py``) is CPU work of the order of a second per
70B layer.  That is fine once (``weight_cache=host`` packs into pinned RAM at
start-up) but too slow per pass when host RAM is small (``weight_cache=disk``).

This cache stores each layer ONCE in its packed byte image:

    <dir>/<layer>.fls   = 4 KiB header (magic, version, fingerprint, nbytes) + packed bytes

so a pass reads exactly the bytes that go to HBM with the native multi-threaded
``pread`` straight into the pinned staging buffer: no per-pass CPU transform.
Data-parallel ranks read only their 1/G byte slice of each file.  The
fingerprint covers the model config, dtype and packing version, so a cache
written for another config is rebuilt instead of silently misread.
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import time
from typing import Optional, Sequence

import torch

from ..config import ModelConfig
from . import hostmem
from .weights import LayerSource

MAGIC = b"FLSPACK1"
HEADER_BYTES = 4096
PACK_VERSION = 2            # bump when models/layout.py changes the packed image


def fingerprint(cfg: ModelConfig, dtype: torch.dtype) -> str:
    d = json.dumps({"cfg": cfg.to_dict(), "dtype": str(dtype), "v": PACK_VERSION}, sort_keys=True, default=str)
    return hashlib.sha256(d.encode()).hexdigest()


def packed_path(cache_dir: str, name: str) -> str:
    return os.path.join(cache_dir, f"{name}.fls")


def _header(fp: str, nbytes: int) -> bytes:
    h = MAGIC + struct.pack("<Q", nbytes) + fp.encode()
    return h + b"\0" * (HEADER_BYTES - len(h))


def _read_header(path: str):
    with open(path, "rb") as f:
        h = f.read(HEADER_BYTES)
    if len(h) != HEADER_BYTES or h[:8] != MAGIC:
        return None, None
    nbytes = struct.unpack("<Q", h[8:16])[0]
    return h[16:16 + 64].decode(errors="replace"), nbytes


class PackedFileSource(LayerSource):
    """Layers as packed images on disk; ``read_into`` is a raw pread."""

    def __init__(self, cfg: ModelConfig, cache_dir: str, dtype=torch.float16,
                 names: Optional[Sequence[str]] = None):
        self.cfg, self.cache_dir, self.dtype = cfg, cache_dir, dtype
        self.fp = fingerprint(cfg, dtype)
        stale = [n for n in (names or cfg.layer_names()) if not self._valid(n)]
        if stale:
            raise FileNotFoundError(f"{cache_dir}: missing or stale packed layers {stale[:4]}...")
        self.read_seconds = 0.0
        self.read_bytes = 0

    def _valid(self, name: str) -> bool:
        p = packed_path(self.cache_dir, name)
        if not os.path.exists(p):
            return False
        fp, nb = _read_header(p)
        return fp == self.fp and nb == self.nbytes(name) and os.path.getsize(p) >= HEADER_BYTES + nb

    def read_into(self, name: str, dst: torch.Tensor) -> None:
        self.read_range_into(name, dst, 0, self.nbytes(name))

    def read_range_into(self, name: str, dst: torch.Tensor, lo: int, hi: int) -> None:
        """Bytes [lo, hi) of the packed image into ``dst[:hi-lo]`` (data-parallel slices)."""
        t0 = time.perf_counter()
        hostmem.pread_into(packed_path(self.cache_dir, name), HEADER_BYTES + lo, hi - lo, dst)
        self.read_bytes += hi - lo
        self.read_seconds += time.perf_counter() - t0


def build_packed_cache(src: LayerSource, cache_dir: str, names: Optional[Sequence[str]] = None,
                       verbose: bool = False) -> int:
    """Write packed images of ``names`` (default: all layers) that are missing or stale.
    Returns the number of layers written.  Writes go to a temp name and are renamed."""
    os.makedirs(cache_dir, exist_ok=True)
    fp = fingerprint(src.cfg, src.dtype)
    names = list(names or src.cfg.layer_names())
    buf = None
    written = 0
    t0 = time.perf_counter()
    for i, n in enumerate(names):
        p = packed_path(cache_dir, n)
        if os.path.exists(p):
            hfp, hnb = _read_header(p)
            if hfp == fp and hnb == src.nbytes(n):
                continue
        nb = src.nbytes(n)
        if buf is None or buf.numel() < HEADER_BYTES + nb:
            buf = hostmem.alloc_host(HEADER_BYTES + max(nb, max(src.nbytes(x) for x in names)), pinned=False)
        buf[:HEADER_BYTES].copy_(torch.frombuffer(bytearray(_header(fp, nb)), dtype=torch.uint8))
        src.read_into(n, buf[HEADER_BYTES:HEADER_BYTES + nb])
        tmp = f"{p}.tmp{os.getpid()}"
        hostmem.pwrite_from(tmp, buf, HEADER_BYTES + nb)
        os.replace(tmp, p)
        written += 1
        if verbose and (written % 10 == 1 or i == len(names) - 1):
            print(f"[packed cache] {i + 1}/{len(names)} layers ({time.perf_counter() - t0:.0f}s)", flush=True)
    return written
