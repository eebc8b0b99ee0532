"""Minimal safetensors reader/writer for the per-layer checkpoint format.

Layout: ``u64 little-endian header length N`` | ``N bytes JSON header`` | raw
tensor bytes; header entries ``{"name": {"dtype", "shape", "data_offsets":
[begin, end]}}`` relative to the byte after the header.

The reference reads each layer file whole (``f.read()``) and deserializes it
through the Rust ``safetensors`` core into CPU tensors (``utils.py:126-127``),
i.e. two host copies per layer.  Here the header is parsed once and tensor
bytes are read straight into their destination (a pinned slot) with the
native multi-threaded ``pread`` engine when it is available
(``csrc/runtime/file_io.cpp``).
"""
from __future__ import annotations

import json
import os
import struct
from dataclasses import dataclass
from typing import Dict, Iterable, Optional, Tuple

import torch

DTYPES = {
    "F16": torch.float16, "BF16": torch.bfloat16, "F32": torch.float32, "F64": torch.float64,
    "I8": torch.int8, "U8": torch.uint8, "I16": torch.int16, "I32": torch.int32, "I64": torch.int64,
    "BOOL": torch.bool,
}
DTYPE_NAMES = {v: k for k, v in DTYPES.items()}


@dataclass(frozen=True)
class TensorInfo:
    name: str
    dtype: torch.dtype
    shape: Tuple[int, ...]
    begin: int   # absolute file offset
    end: int

    @property
    def nbytes(self) -> int:
        return self.end - self.begin


def read_header(path: str) -> Tuple[Dict[str, TensorInfo], dict]:
    with open(path, "rb") as f:
        raw = f.read(8)
        if len(raw) != 8:
            raise ValueError(f"{path}: not a safetensors file")
        (n,) = struct.unpack("<Q", raw)
        if n > 100 * 1024 * 1024:
            raise ValueError(f"{path}: header too large ({n})")
        hdr = json.loads(f.read(n))
    base = 8 + n
    meta = hdr.pop("__metadata__", {}) or {}
    infos = {}
    for name, e in hdr.items():
        b, en = e["data_offsets"]
        infos[name] = TensorInfo(name, DTYPES[e["dtype"]], tuple(e["shape"]), base + b, base + en)
    return infos, meta


def load_file(path: str, names: Optional[Iterable[str]] = None) -> Dict[str, torch.Tensor]:
    """Read tensors into fresh CPU tensors (test / conversion path)."""
    infos, _ = read_header(path)
    out = {}
    with open(path, "rb") as f:
        for name, ti in infos.items():
            if names is not None and name not in names:
                continue
            t = torch.empty(ti.shape, dtype=ti.dtype)
            if ti.nbytes:
                f.seek(ti.begin)
                mv = memoryview(t.view(-1).view(torch.uint8).numpy())
                got = f.readinto(mv)
                if got != ti.nbytes:
                    raise IOError(f"{path}:{name}: short read {got}/{ti.nbytes}")
            out[name] = t
    return out


def save_file(tensors: Dict[str, torch.Tensor], path: str, metadata: Optional[dict] = None) -> None:
    """Write a safetensors file (same byte format as ``safetensors.torch.save_file``)."""
    hdr, off, items = {}, 0, []
    for name in sorted(tensors):
        t = tensors[name].detach().contiguous().cpu()
        n = t.numel() * t.element_size()
        hdr[name] = {"dtype": DTYPE_NAMES[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + n]}
        items.append(t)
        off += n
    if metadata:
        hdr["__metadata__"] = {str(k): str(v) for k, v in metadata.items()}
    hb = json.dumps(hdr, separators=(",", ":")).encode()
    hb += b" " * ((8 - len(hb) % 8) % 8)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(struct.pack("<Q", len(hb)))
        f.write(hb)
        for t in items:
            if t.numel():
                f.write(t.view(-1).view(torch.uint8).numpy().tobytes())
    os.replace(tmp, path)
