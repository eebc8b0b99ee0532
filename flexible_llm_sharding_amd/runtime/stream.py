"""Weight streaming from per-layer safetensors files (``--weight_cache stream``).

Reference (``/root/reference/utils.py:121-131``; DP ``utils.py:72-73``): every
time a layer is needed its file is read whole into a Python ``bytes`` object,
deserialised on the CPU, and each tensor is copied to the GPU (pageable,
synchronous) with a cast to fp16.  Host RAM needed: about one layer; the model
itself never has to fit in RAM (README: 70B with >= 8 GB of RAM).

Here the same small-RAM envelope costs no CPU work per pass:

* the packed HBM image of a layer is the checkpoint's own tensors concatenated
  (:mod:`..models.layout`), so a layer is a set of *file byte ranges* with a
  destination offset each (:class:`LayerPlan`);
* the native streamer (``fls_streamer_*`` in ``csrc/runtime/runtime.cpp``)
  reads those ranges with a persistent ``pread`` pool (optionally
  ``O_DIRECT``) into a small ring of pinned chunks (default 6 x 64 MiB) and
  DMAs every piece straight to its place in the HBM weight slot on the copy
  stream, so disk reads, PCIe DMA and compute of the previous shard overlap;
* bf16 tensors are converted to fp16 in place in HBM by a HIP kernel on the
  copy stream (``fls_cast_f16``); fp32 tensors (norm weights of mixed
  checkpoints) are converted on the host while they sit in the pinned chunk.

Data-parallel ranks stream only their 1/G byte range of the packed image
(:meth:`LayerPlan.pieces`) and complete the layer with an RCCL all-gather
(:mod:`..parallel.data_parallel`): each layer file is read from disk once per
pass for all GPUs, like the reference's shared host cache.
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from .. import _native, knobs
from ..config import ModelConfig
from ..models.layout import check_layer_tensors, layer_kind, layer_layout, placements, source_key
from ..utils.layer_format import layer_file
from ..utils.safetensors_io import TensorInfo, read_header
from . import hostmem
from .weights import LayerSource

KIND_RAW, KIND_F32 = 0, 1
_SRC_ES = {torch.float16: 2, torch.bfloat16: 2, torch.float32: 4}


@dataclass(frozen=True)
class TensorRun:
    """One checkpoint tensor: file bytes [file_off, file_off + numel * src_es) -> image bytes
    [img_off, img_off + 2 * numel)."""
    hf_name: str
    file_off: int
    img_off: int
    numel: int
    src_dtype: torch.dtype

    @property
    def src_es(self) -> int:
        return _SRC_ES[self.src_dtype]


class LayerPlan:
    """Byte-level plan of one layer file -> packed fp16 image."""

    def __init__(self, cfg: ModelConfig, layer_name: str, path: str):
        self.name, self.path = layer_name, path
        infos = hostmem.read_header_native(path)
        if infos is None:
            infos, _ = read_header(path)
        infos = _relabel_layer(infos, layer_name)
        check_layer_tensors(cfg, layer_name, infos)
        runs = []
        for pl in placements(cfg, layer_name):
            key = source_key(cfg, layer_name, pl.hf_name, infos)
            ti: TensorInfo = infos[key]
            if ti.dtype == torch.int8:
                raise AssertionError("int8 not supported (need to add fp16_statistics)")   # utils.py:129
            if ti.dtype not in _SRC_ES:
                raise TypeError(f"{path}: {key} has dtype {ti.dtype}; fp16 / bf16 / fp32 supported")
            if tuple(ti.shape) != pl.shape:
                raise ValueError(f"{path}: {key} has shape {tuple(ti.shape)}, config expects {pl.shape}")
            if ti.nbytes != pl.numel * _SRC_ES[ti.dtype]:
                raise ValueError(f"{path}: {key} byte size {ti.nbytes} does not match its shape")
            runs.append(TensorRun(key, ti.begin, pl.offset, pl.numel, ti.dtype))
        self.runs = sorted(runs, key=lambda r: r.file_off)
        self.nbytes = layer_layout(cfg, layer_kind(layer_name)).nbytes
        self.file_bytes = sum(r.numel * r.src_es for r in self.runs)

    def pieces(self, lo: int = 0, hi: Optional[int] = None) -> List[Tuple[int, int, int, int]]:
        """(file_off, file_bytes, dst_off, kind) covering image bytes [lo, hi); dst_off relative to lo.
        lo / hi must be even (whole fp16 elements)."""
        hi = self.nbytes if hi is None else hi
        if lo % 2 or hi % 2:
            raise ValueError("image ranges must cover whole fp16 elements")
        out = []
        for r in self.runs:
            a, b = max(lo, r.img_off), min(hi, r.img_off + 2 * r.numel)
            if a >= b:
                continue
            e0, e1 = (a - r.img_off) // 2, (b - r.img_off) // 2
            out.append((r.file_off + e0 * r.src_es, (e1 - e0) * r.src_es, a - lo,
                        KIND_F32 if r.src_dtype == torch.float32 else KIND_RAW))
        return out

    def bf16_runs(self, lo: int = 0, hi: Optional[int] = None) -> List[Tuple[int, int]]:
        """(image offset, bytes) of bf16 tensors within [lo, hi) (offsets relative to lo): these
        are converted to fp16 in place after landing."""
        hi = self.nbytes if hi is None else hi
        out = []
        for r in self.runs:
            if r.src_dtype != torch.bfloat16:
                continue
            a, b = max(lo, r.img_off), min(hi, r.img_off + 2 * r.numel)
            if a < b:
                out.append((a - lo, b - a))
        return out


def _relabel_layer(infos: Dict[str, TensorInfo], layer_name: str) -> Dict[str, TensorInfo]:
    """A decoder-layer file whose tensors all carry another layer index (a copied / hard-linked
    layer file, e.g. ``prepare_weights.py --synthetic --unique_layers K``) is read as this layer:
    tensors are identified by their name inside the layer."""
    if not layer_name.startswith("model.layers.") or any(k.startswith(layer_name + ".") for k in infos):
        return infos
    prefixes = {".".join(k.split(".")[:3]) for k in infos if k.startswith("model.layers.")}
    if len(prefixes) != 1:
        return infos
    (p,) = prefixes
    return {(layer_name + k[len(p):]) if k.startswith(p + ".") else k: v for k, v in infos.items()}


def _piece_array(pieces) -> ctypes.Array:
    arr = (_native.Piece * max(1, len(pieces)))()
    for i, (fo, nb, do, kind) in enumerate(pieces):
        arr[i].file_off, arr[i].nbytes, arr[i].dst_off, arr[i].kind = fo, nb, do, kind
    return arr


class FileLayerSource(LayerSource):
    """Per-layer safetensors files streamed to HBM on every pass (``--weight_cache stream``).

    ``chunk_mb`` x ``n_chunks`` is the whole pinned host footprint of the weight path.
    ``direct`` reads with ``O_DIRECT`` (bypassing the page cache; falls back to buffered
    reads where the file system refuses it).
    """

    def __init__(self, cfg: ModelConfig, model_path: str, names: Optional[Sequence[str]] = None,
                 dtype=torch.float16, chunk_mb: Optional[int] = None, n_chunks: Optional[int] = None,
                 io_threads: Optional[int] = None, direct: Optional[bool] = None):
        if dtype != torch.float16:
            raise ValueError("the packed weight image is fp16")
        self.cfg, self.model_path, self.dtype = cfg, model_path, dtype
        self.names = list(names) if names is not None else cfg.layer_names()
        missing = [n for n in self.names if not os.path.exists(layer_file(model_path, n))]
        if missing:
            raise FileNotFoundError(f"{model_path}: missing layer files {missing[:4]}...")
        self.chunk_bytes = (chunk_mb or knobs.get_int("FLS_STREAM_CHUNK_MB")) << 20
        self.n_chunks = n_chunks or knobs.get_int("FLS_STREAM_CHUNKS")
        self.io_threads = io_threads or knobs.get_int("FLS_IO_THREADS")
        self.direct = bool(knobs.get_int("FLS_O_DIRECT")) if direct is None else bool(direct)
        self._plans: Dict[str, LayerPlan] = {}
        self._lock = threading.Lock()
        self._streamer = None
        self._streamer_dev = None
        self.read_seconds = 0.0
        self.read_bytes = 0

    # ---------------------------------------------------------------- plans
    def plan(self, name: str) -> LayerPlan:
        with self._lock:
            p = self._plans.get(name)
            if p is None:
                p = self._plans[name] = LayerPlan(self.cfg, name, layer_file(self.model_path, name))
            return p

    # ------------------------------------------------------------ host path
    def read_into(self, name: str, dst: torch.Tensor) -> None:
        """The whole packed image into a CPU byte buffer (host cache build, CPU runs)."""
        self.read_range_into(name, dst, 0, self.nbytes(name))

    def read_range_into(self, name: str, dst: torch.Tensor, lo: int, hi: int) -> None:
        """Image bytes [lo, hi) into ``dst[:hi - lo]`` (CPU); bf16 converted on the host."""
        t0 = time.perf_counter()
        pl = self.plan(name)
        pieces = pl.pieces(lo, hi)
        b = dst.view(torch.uint8)
        rt = _native.runtime_or_none()
        if rt is not None and pieces:
            arr = _piece_array(pieces)
            r = rt.fls_stream_read_host(pl.path.encode(), ctypes.addressof(arr), len(pieces), b.data_ptr(),
                                        self.io_threads)
            if r < 0:
                raise IOError(f"{pl.path}: read failed ({r})")
        else:
            self._read_pieces_py(pl.path, pieces, b)
        for off, nb in pl.bf16_runs(lo, hi):
            v = b[off:off + nb]
            v.view(torch.float16).copy_(v.view(torch.bfloat16).clone())
        self.read_bytes += sum(p[1] for p in pieces)
        self.read_seconds += time.perf_counter() - t0

    @staticmethod
    def _read_pieces_py(path: str, pieces, b: torch.Tensor) -> None:
        with open(path, "rb") as f:
            for fo, nb, do, kind in pieces:
                f.seek(fo)
                raw = f.read(nb)
                if len(raw) != nb:
                    raise IOError(f"{path}: short read")
                t = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
                if kind == KIND_F32:
                    t = t.view(torch.float32).to(torch.float16).view(torch.uint8)
                b[do:do + t.numel()].copy_(t)

    # ------------------------------------------------------------- GPU path
    def _get_streamer(self, device: torch.device):
        if self._streamer is None:
            rt = _native.runtime()
            h = rt.fls_streamer_create(device.index or 0, self.chunk_bytes, self.n_chunks, self.io_threads,
                                       int(self.direct))
            if not h:
                raise RuntimeError("fls_streamer_create failed (pinned chunk ring)")
            self._streamer, self._streamer_dev = h, device
        elif self._streamer_dev != device:
            raise RuntimeError("one streaming source serves one device")
        return self._streamer

    def pinned_bytes(self) -> int:
        if self._streamer is None:
            return self.chunk_bytes * self.n_chunks
        return int(_native.runtime().fls_streamer_pinned_bytes(self._streamer))

    def stream_into(self, name: str, dst: torch.Tensor, stream, lo: int = 0, hi: Optional[int] = None,
                    cast: bool = True) -> int:
        """Enqueue image bytes [lo, hi) of ``name`` into the HBM byte tensor ``dst`` on ``stream``
        (a ``torch.cuda.Stream``).  Returns once every DMA is enqueued; the caller records its
        completion event.  ``cast`` also enqueues the in-place bf16 -> fp16 conversions (the
        data-parallel path casts after its all-gather instead).  Returns file bytes read."""
        pl = self.plan(name)
        hi = pl.nbytes if hi is None else hi
        pieces = pl.pieces(lo, hi)
        if not pieces:
            return 0
        h = self._get_streamer(dst.device)
        arr = _piece_array(pieces)
        t0 = time.perf_counter()
        r = _native.runtime().fls_streamer_load(h, pl.path.encode(), ctypes.addressof(arr), len(pieces),
                                                dst.data_ptr(), stream.cuda_stream)
        if r < 0:
            raise IOError(f"{pl.path}: streaming failed ({r})")
        self.read_seconds += time.perf_counter() - t0
        self.read_bytes += int(r)
        if cast:
            self.cast_on_gpu(name, dst, lo, hi)
        return int(r)

    def cast_on_gpu(self, name: str, dst: torch.Tensor, lo: int = 0, hi: Optional[int] = None) -> None:
        """In-place bf16 -> fp16 of the bf16 tensors in image bytes [lo, hi) of ``dst``, whose byte 0
        is image byte ``lo`` (current stream)."""
        runs = self.plan(name).bf16_runs(lo, hi)
        if not runs:
            return
        from ..ops import get_ops
        ops = get_ops(dst.device)
        for off, nb in runs:
            v = dst[off:off + nb]
            ops.cast_f16(v, v, 1)

    def stats(self) -> Dict[str, float]:
        out = {"read_s": self.read_seconds, "read_bytes": float(self.read_bytes)}
        if self._streamer is not None:
            rs, ws = ctypes.c_double(), ctypes.c_double()
            rb, hb = ctypes.c_uint64(), ctypes.c_uint64()
            fb = ctypes.c_int()
            _native.runtime().fls_streamer_stats(self._streamer, ctypes.byref(rs), ctypes.byref(ws),
                                                 ctypes.byref(rb), ctypes.byref(hb), ctypes.byref(fb))
            out.update({"pread_s": rs.value, "ring_wait_s": ws.value, "h2d_bytes": float(hb.value),
                        "direct_fallbacks": float(fb.value)})
        return out

    def close(self) -> None:
        if self._streamer is not None:
            _native.runtime().fls_streamer_destroy(self._streamer)
            self._streamer = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def host_ram_available() -> int:
    """MemAvailable from /proc/meminfo (bytes), 0 if unknown."""
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 0
