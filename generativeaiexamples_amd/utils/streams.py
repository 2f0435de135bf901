"""HIP streams of the serving process.

The generator engine thread replays its decode graphs on the default stream. The query path (embedding
micro-batches and exact index scans, issued from retrieval threads) runs on a separate HIGH-priority
stream per device, so a new query's embed + scan kernels are scheduled beside a running decode graph
instead of queueing behind it (a K-step decode run is ~65 ms at batch 64). Work on this stream is
self-contained: its inputs are host data or persistent index buffers, and its results are read back
(``.cpu()``) on the same stream before any other thread uses them.
"""
from __future__ import annotations

import contextlib
import threading

import torch

_streams: dict = {}
_lock = threading.Lock()


def retrieval_stream(device) -> "torch.cuda.Stream | None":
    device = torch.device(device)
    if device.type != "cuda":
        return None
    key = device.index if device.index is not None else torch.cuda.current_device()
    with _lock:
        s = _streams.get(key)
        if s is None:
            lo, hi = torch.cuda.Stream.priority_range()  # hi is the numerically smallest = highest priority
            s = _streams[key] = torch.cuda.Stream(device=torch.device("cuda", key), priority=hi)
        return s


@contextlib.contextmanager
def on_retrieval_stream(device):
    """Run the enclosed GPU work on the retrieval stream (no-op on CPU); the stream is synchronised on exit so
    results are complete for any consumer thread or stream."""
    s = retrieval_stream(device)
    if s is None:
        yield
        return
    with torch.cuda.stream(s):
        yield
    s.synchronize()


class RetrievalGate:
    """Count of query-path requests (embed + scan) submitted and not yet answered, process-wide. The
    generator's serving loop consults it before it starts a prefill with nothing else to run: a burst of
    concurrent queries then joins ONE prefill instead of the first query's prefill occupying every CU
    (persistent GEMM kernels hold the whole chip for milliseconds) while the others' embeds queue behind it
    (served p50 TTFT 1.8 s vs 0.93 s in-process before this gate, profiles/r3/README.md)."""

    def __init__(self):
        self.n = 0
        self.cv = threading.Condition()

    def enter(self):
        with self.cv:
            self.n += 1

    def exit(self):
        with self.cv:
            self.n -= 1
            if self.n <= 0:
                self.n = 0
                self.cv.notify_all()

    def busy(self) -> bool:
        return self.n > 0

    def wait_idle(self, timeout: float) -> bool:
        """Block until no retrieval is pending or ``timeout`` seconds passed; True when idle."""
        with self.cv:
            return self.cv.wait_for(lambda: self.n <= 0, timeout)


RETRIEVAL_GATE = RetrievalGate()
