"""Op backends.

* ``HipOps`` (``hip_backend``) — hand-written CDNA4 kernels from
  ``libfls_kernels.so``; the only backend on a GPU (it raises if the library
  is missing rather than silently falling back).
* ``TorchOps`` (``torch_backend``) — plain PyTorch: the CPU path (BASELINE
  config 1) and the numerics oracle for the kernels.
"""
from __future__ import annotations

import torch

from .torch_backend import TorchOps

_cache = {}


def get_ops(device, compute_dtype=None):
    dev = torch.device(device)
    key = (dev.type, compute_dtype)
    if key in _cache:
        return _cache[key]
    if dev.type == "cuda":
        from .hip_backend import HipOps
        ops = HipOps()
    else:
        ops = TorchOps(compute_dtype or torch.float32)
    _cache[key] = ops
    return ops
