"""Tracing: roctx ranges (visible in ``rocprofv3 --marker-trace``) + host timers.

The reference's only instrumentation is a wall-clock accumulator of weight
load time printed per device (``/root/reference/utils.py:223-233, 304``).
Here every shard load / micro-batch compute / activation store / collective
can be bracketed by roctx ranges when ``FLS_TRACE=1`` (or ``--profile``), and
:class:`Timers` accumulates host-side durations that end up in the run's
metrics JSON.  Disabled tracing costs one attribute lookup per range.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import defaultdict

from .. import knobs

_roctx = None
_enabled = knobs.get("FLS_TRACE") not in ("0", "", "false")


def _load():
    global _roctx
    if _roctx is not None:
        return _roctx
    for name in ("librocprofiler-sdk-roctx.so", "librocprofiler-sdk-roctx.so.1", "libroctx64.so"):
        for base in (os.environ.get("ROCM_PATH", "/opt/rocm") + "/lib/", ""):
            try:
                lib = ctypes.CDLL(base + name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _roctx = lib
                return lib
            except (OSError, AttributeError):
                continue
    _roctx = False
    return _roctx


def enable(flag: bool = True) -> None:
    global _enabled
    _enabled = flag


def enabled() -> bool:
    return _enabled and bool(_load())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    if not _enabled:
        yield
        return
    lib = _load()
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


def mark(name: str) -> None:
    if _enabled and _load():
        _roctx.roctxMarkA(name.encode())


class Timers:
    """Accumulating host timers: ``with timers("load"): ...``."""

    def __init__(self):
        self.total = defaultdict(float)
        self.count = defaultdict(int)

    @contextlib.contextmanager
    def __call__(self, key: str):
        t0 = time.perf_counter()
        try:
            with range(key):
                yield
        finally:
            self.total[key] += time.perf_counter() - t0
            self.count[key] += 1

    def as_dict(self):
        return {k: {"s": round(v, 6), "n": self.count[k]} for k, v in self.total.items()}
