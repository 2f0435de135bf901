"""HIP graph capture helper shared by the engine's decode graphs and the embedder's query graphs."""
from __future__ import annotations

import contextlib
import gc

import torch

# per device: a graph captured outside inference mode, kept alive for the life of the process (see _rng_graph_state)
_RNG_STATE_GRAPHS: dict = {}


def _rng_graph_state(stream) -> None:
    """Make the first graph registration of this device's CUDA generator happen outside inference mode.

    The generator creates its graph-safe seed / offset tensors at the first graph capture and fills them in place at
    every later one. The engine captures lazily inside ``LLMEngine.step()`` (``torch.inference_mode``): if that is the
    process's first capture, those tensors are inference tensors and any later capture outside inference mode (a model
    or embedder capturing its own graphs, a test) fails with "Inplace update to inference tensor outside
    InferenceMode". One tiny capture with inference mode off, before any other, creates them as normal tensors (fine
    to update in either mode); the graph is kept so the registration stays."""
    dev = getattr(stream, "device", None)
    dev = torch.device("cuda", torch.cuda.current_device()) if dev is None else torch.device(dev)
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key in _RNG_STATE_GRAPHS:
        return
    try:
        with torch.inference_mode(False):
            x = torch.zeros(1, device=dev)
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                x.add_(1)
            torch.cuda.current_stream(dev).wait_stream(s)
        _RNG_STATE_GRAPHS[key] = (g, x)
    except RuntimeError:
        # a direct torch.cuda.graph capture inside inference mode registered the state first: nothing to fix from
        # here (captures in inference mode keep working); do not retry on every capture
        _RNG_STATE_GRAPHS[key] = None


@contextlib.contextmanager
def hip_graph_capture(g: "torch.cuda.CUDAGraph", stream):
    """``torch.cuda.graph`` (thread-local capture mode) with Python's cyclic garbage collector held off until the
    capture ends. A collection that fires inside the capture runs finalizers of unrelated objects - an event or a
    pinned staging buffer from an earlier step - whose HIP release calls a capturing stream forbids; raised inside
    a destructor, that error aborts the process (seen once in the GPU suite, test_guided_gpu, round 4)."""
    _rng_graph_state(stream)
    enabled = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
            yield
    finally:
        if enabled:
            gc.enable()
