"""roctx ranges for rocprofv3 / omnitrace timelines (SURVEY §5.1 plan: "Add roctx ranges").

``GAI_ROCTX=1`` loads the ROCm marker library (``librocprofiler-sdk-roctx`` for rocprofv3, else
``libroctx64``) and the engine, embedder, index and reranker wrap their phases in named ranges
(``prefill``/``decode`` steps, ``embed``, ``index_search``, ``rerank``); capture them with
``rocprofv3 --marker-trace`` (a marker trace is a trace domain: keep ``--pmc`` counters in a separate run).
Disabled (the default), a range is one attribute check.
"""
from __future__ import annotations

import ctypes
import os
from contextlib import contextmanager

ENABLED = os.environ.get("GAI_ROCTX") == "1"
_lib = None


def _load():
    global _lib, ENABLED
    if _lib is not None or not ENABLED:
        return _lib
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so"):
        for d in ("", "/opt/rocm/lib/"):
            try:
                lib = ctypes.CDLL(d + name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                return _lib
            except OSError:
                continue
    ENABLED = False
    return None


@contextmanager
def roctx_range(name: str):
    if not ENABLED or _load() is None:
        yield
        return
    _lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        _lib.roctxRangePop()


def roctx_mark(name: str):
    if ENABLED and _load() is not None:
        _lib.roctxMarkA(name.encode())
