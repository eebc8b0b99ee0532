"""Op backends.

* ``HipOps`` (``hip_backend``) — hand-written CDNA4 kernels from
  ``libfls_kernels.so``; the only backend used on a GPU (it raises if the
  library is missing rather than silently falling back).
* ``TorchOps`` (``torch_backend``) — plain PyTorch: the CPU path and the
  numerics oracle for the kernels.
"""
from __future__ import annotations

import os

import torch

from .torch_backend import TorchOps

_cache = {}


def get_ops(device, compute_dtype=None):
    dev = torch.device(device)
    backend = os.environ.get("FLS_OPS", "")
    key = (dev.type, backend, compute_dtype)
    if key in _cache:
        return _cache[key]
    if dev.type == "cuda" and backend != "torch":
        from .hip_backend import HipOps
        ops = HipOps()
    else:
        ops = TorchOps(compute_dtype or (torch.float32 if dev.type == "cpu" else torch.float16))
    _cache[key] = ops
    return ops
