"""Weight sources: where packed layer bytes come from before they reach HBM.

Reference behaviour (``/root/reference/utils.py:121-131``, DP cache
``utils.py:24-75``): every time a layer is needed its safetensors file is read
whole from disk, deserialized to CPU tensors and copied parameter by parameter
(pageable, synchronous) to the GPU; the whole thing repeats for every batch,
generation step and GPU.

Here a source yields the *packed* layer image (see :mod:`..models.layout`):

* :class:`~.stream.FileLayerSource` — per-layer safetensors files streamed
  every pass (file byte ranges -> pinned chunk ring -> HBM DMA, no CPU work);
  the reference's small-RAM mode (``--weight_cache stream``).
* :class:`HostStore` — every packed layer resident in pinned host memory
  (read once), so each shard H2D is one DMA at PCIe line rate
  (``--weight_cache host``).  Also built directly from synthetic random-init
  weights (generated on the GPU and copied down) for the 70B benchmark.
* data-parallel scatter-load (:func:`piece_slices`): a rank keeps only its
  1/G byte-slice of every layer piece; the layer (or one piece of it) is
  re-assembled in HBM with an RCCL all-gather over xGMI
  (:mod:`..parallel.data_parallel`).
"""
from __future__ import annotations

import threading
from typing import Dict, List, NamedTuple, Optional, Sequence, Tuple

import torch

from ..config import ModelConfig
from ..models.layout import LayerLayout, layer_kind, layer_layout
from . import hostmem


class LayerSource:
    cfg: ModelConfig
    dtype: torch.dtype = torch.float16

    def layout(self, name: str) -> LayerLayout:
        return layer_layout(self.cfg, layer_kind(name), torch.empty((), dtype=self.dtype).element_size())

    def nbytes(self, name: str) -> int:
        return self.layout(name).nbytes

    def host_buffer(self, name: str) -> Optional[torch.Tensor]:
        """Pinned uint8 buffer holding the packed layer, if resident on the host."""
        return None

    def read_into(self, name: str, dst: torch.Tensor) -> None:
        raise NotImplementedError


class HostStore(LayerSource):
    """All packed layers resident in (pinned) host memory.

    ``norms_folded``: every decoder layer's RMSNorm weights are already folded into the
    projections that consume the normalised rows (:meth:`fold_norms`, done once on the GPU), so
    the fused-norm engine streams them as they are — no per-load fold on the copy stream."""

    norms_folded = False

    def __init__(self, cfg: ModelConfig, dtype=torch.float16, pinned: bool = True,
                 names: Optional[Sequence[str]] = None):
        self.cfg, self.dtype, self.pinned = cfg, dtype, pinned
        self.names = list(names) if names is not None else cfg.layer_names()
        self.buffers: Dict[str, torch.Tensor] = {}

    def fold_norms(self, device) -> "HostStore":
        """Fold the RMSNorm weights into the projections (models.llama.fold_layer_norms) for
        every decoder layer, on ``device``: each layer goes H2D, is folded, and comes back.  Once
        per store, in place; a full 70B store takes a few seconds at PCIe rate."""
        from ..models.llama import fold_layer_norms
        from ..ops import get_ops
        if self.norms_folded:
            return self
        dev = torch.device(device)
        ops = get_ops(dev)
        dec = [n for n in self.names if layer_kind(n) == "decoder" and n in self.buffers]
        if dec:
            stage = torch.empty(max(self.nbytes(n) for n in dec), dtype=torch.uint8, device=dev)
            for n in dec:
                buf = self.buffers[n]
                full = stage[:buf.numel()]
                full.copy_(buf)
                fold_layer_norms(ops, self.layout(n).views(full, self.dtype))
                buf.copy_(full)
            del stage
        self.norms_folded = True
        return self

    @property
    def total_bytes(self) -> int:
        return sum(b.numel() for b in self.buffers.values())

    def host_buffer(self, name: str) -> Optional[torch.Tensor]:
        return self.buffers.get(name)

    def read_into(self, name: str, dst: torch.Tensor) -> None:
        src = self.buffers[name]
        dst[:src.numel()].copy_(src)

    def alloc(self, name: str) -> torch.Tensor:
        buf = hostmem.alloc_host(self.nbytes(name), pinned=self.pinned)
        self.buffers[name] = buf
        return buf

    @classmethod
    def from_source(cls, src: LayerSource, pinned: bool = True, threads: int = 4,
                    names: Optional[Sequence[str]] = None) -> "HostStore":
        st = cls(src.cfg, src.dtype, pinned, names)
        for n in st.names:
            st.alloc(n)
        errs: List[BaseException] = []
        todo = list(st.names)
        lock = threading.Lock()

        def worker():
            while True:
                with lock:
                    if not todo or errs:
                        return
                    n = todo.pop(0)
                try:
                    src.read_into(n, st.buffers[n])
                except BaseException as e:  # noqa: BLE001
                    errs.append(e)
                    return

        ts = [threading.Thread(target=worker, daemon=True) for _ in range(max(1, threads))]
        [t.start() for t in ts]
        [t.join() for t in ts]
        if errs:
            raise errs[0]
        return st

    @classmethod
    def from_model_path(cls, cfg: ModelConfig, model_path: str, dtype=torch.float16,
                        pinned: bool = True, threads: int = 4) -> "HostStore":
        from .stream import FileLayerSource
        return cls.from_source(FileLayerSource(cfg, model_path, dtype=dtype), pinned, threads)

    @classmethod
    def synthetic(cls, cfg: ModelConfig, device: torch.device, seed: int = 0, std: float = 0.02,
                  pinned: bool = True, names: Optional[Sequence[str]] = None,
                  byte_range=None, progress=None, fold_norms: bool = False) -> "HostStore":
        """Random-init packed layers generated on ``device`` and copied to pinned host memory.

        ``byte_range=(r, G)`` keeps only slice r of G equal byte slices of every
        layer (data-parallel scatter-load).  Generation is deterministic in
        (seed, layer index, byte offset) so every rank's slices tile one model.
        ``fold_norms``: the RMSNorm weights are folded into the projections on the device before
        the copy (see :meth:`fold_norms`).
        """
        from ..models.llama import fold_layer_norms
        from ..ops import get_ops
        st = cls(cfg, torch.float16, pinned, names)
        dev = torch.device(device)
        ops = get_ops(dev)
        maxb = max((st.nbytes(n) for n in st.names), default=0)   # an MP rank may own no layers
        stage = torch.empty(maxb, dtype=torch.uint8, device=dev)
        for li, n in enumerate(st.names):
            if progress is not None and li % 10 == 0:
                progress(li, len(st.names))
            lay = st.layout(n)
            full = stage[:lay.nbytes]
            ops.fill_layer_random(full, lay, seed=seed * 7919 + cfg.layer_names().index(n), std=std)
            if fold_norms and lay.kind == "decoder":
                fold_layer_norms(ops, lay.views(full, torch.float16))
            if byte_range is None:
                buf = st.alloc(n)
                buf.copy_(full, non_blocking=False)
            else:
                r, G = byte_range
                sl = piece_slices(lay, G)
                buf = hostmem.alloc_host(sum(p.chunk for p in sl), pinned=pinned)
                for p in sl:
                    a, b = p.rank_range(r)
                    if b > a:
                        buf[p.buf_off:p.buf_off + b - a].copy_(full[a:b])
                st.buffers[n] = buf
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        del stage
        st.norms_folded = bool(fold_norms)
        return st


def shard_chunk_bytes(nbytes: int, world: int, align: int = 4096) -> int:
    c = (nbytes + world - 1) // world
    return (c + align - 1) // align * align


def layer_pieces(lay: LayerLayout) -> List[Tuple[int, int]]:
    """Byte ranges of a packed layer image that load as one unit: a decoder layer's attention
    piece and MLP piece (``models.layout.mlp_offset``; the sub-layer piece pool streams them
    separately), one range for every other kind."""
    from ..models.layout import mlp_offset
    if lay.kind == "decoder":
        s = mlp_offset(lay)
        return [(0, s), (s, lay.nbytes)]
    return [(0, lay.nbytes)]


class PieceSlice(NamedTuple):
    """Data-parallel scatter-load of one piece ``[lo, hi)`` of a layer image over G ranks: rank r
    holds bytes ``[lo + r * chunk, min(hi, lo + (r + 1) * chunk))`` at ``buf_off`` of its host
    buffer, and the all-gather rebuilds the piece in a ``chunk * G``-byte HBM region."""
    lo: int
    hi: int
    chunk: int
    buf_off: int

    def rank_range(self, r: int) -> Tuple[int, int]:
        a = self.lo + r * self.chunk
        return a, max(a, min(self.hi, a + self.chunk))


def piece_slices(lay: LayerLayout, world: int) -> List[PieceSlice]:
    """Every rank's slices of ``lay``, piece by piece (:func:`layer_pieces`): each piece is split
    on its own, so a rank's slices serve the whole-layer all-gather and the per-piece one alike."""
    out, off = [], 0
    for lo, hi in layer_pieces(lay):
        c = shard_chunk_bytes(hi - lo, world)
        out.append(PieceSlice(lo, hi, c, off))
        off += c
    return out


def piece_views(lay: LayerLayout, regions: Sequence[Tuple[int, torch.Tensor]], dtype) -> Dict[str, torch.Tensor]:
    """Typed tensor views of a layer whose pieces sit in separate byte regions: ``regions`` =
    [(image offset of the piece, uint8 region holding it)] in image order."""
    es = torch.empty((), dtype=dtype).element_size()
    out = {}
    for ts in lay.slots:
        lo, reg = [(lo, reg) for lo, reg in regions if lo <= ts.offset][-1]
        o = ts.offset - lo
        out[ts.name] = reg[o:o + ts.numel * es].view(dtype).view(ts.shape)
    return out
