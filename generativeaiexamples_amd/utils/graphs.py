"""HIP graph capture helper shared by the engine's decode graphs and the embedder's query graphs."""
from __future__ import annotations

import contextlib
import gc

import torch


@contextlib.contextmanager
def hip_graph_capture(g: "torch.cuda.CUDAGraph", stream):
    """``torch.cuda.graph`` (thread-local capture mode) with Python's cyclic garbage collector held off until the
    capture ends. A collection that fires inside the capture runs finalizers of unrelated objects - an event or a
    pinned staging buffer from an earlier step - whose HIP release calls a capturing stream forbids; raised inside
    a destructor, that error aborts the process (seen once in the GPU suite, test_guided_gpu, round 4)."""
    enabled = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
            yield
    finally:
        if enabled:
            gc.enable()
