"""Failure detection and fault injection for the collectives.

Detection: every collective issued through :class:`~.dist.DistContext` runs under ``guard``, which
turns a backend error (peer process died, RCCL/gloo connection closed, collective timeout from the
process-group timeout ``GAI_DIST_TIMEOUT_S``) into :class:`RankFailure` naming the collective and
the rank, so serving code can mark itself unhealthy and fail in-flight requests instead of hanging.
``TORCH_NCCL_ASYNC_ERROR_HANDLING=1`` is set before RCCL init so a hung collective aborts the
communicator rather than blocking forever.

Injection (used by the distributed tests, no effect unless set):
  FI_KILL_RANK=r  FI_KILL_AT_CALL=n   rank r exits (code 17) at its n-th collective
  FI_DELAY_ALLREDUCE_MS=ms [FI_DELAY_RANK=r]   sleep before every collective (on rank r, default all)
"""
from __future__ import annotations

import os
import time
from contextlib import contextmanager


class RankFailure(RuntimeError):
    pass


class _Injector:
    def __init__(self):
        self.calls = 0
        self.reload()

    def reload(self):
        g = os.environ.get
        self.kill_rank = int(g("FI_KILL_RANK", "-1"))
        self.kill_at = int(g("FI_KILL_AT_CALL", "1"))
        self.delay_s = float(g("FI_DELAY_ALLREDUCE_MS", "0")) / 1000.0
        self.delay_rank = int(g("FI_DELAY_RANK", "-1"))

    def before(self, rank: int):
        self.calls += 1
        if rank == self.kill_rank and self.calls >= self.kill_at:
            os._exit(17)  # simulated process crash (no cleanup, like a lost GPU / OOM kill)
        if self.delay_s and (self.delay_rank < 0 or self.delay_rank == rank):
            time.sleep(self.delay_s)


INJECTOR = _Injector()


@contextmanager
def guard(name: str, rank: int):
    INJECTOR.before(rank)
    try:
        yield
    except RankFailure:
        raise
    except (RuntimeError, ConnectionError, TimeoutError) as e:  # DistBackendError subclasses RuntimeError
        raise RankFailure(f"collective '{name}' failed on rank {rank}: {e}") from e
