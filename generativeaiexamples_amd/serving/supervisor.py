"""Replica supervisor: starts R model-server replicas (each a TP group of T ranks, one process per GPU) and
restarts a replica whose group died, with back-off (SURVEY §5.3 TP-group restart).

A TP group fails as a unit: when any rank dies (lost GPU, OOM kill, a hung collective the watchdog turned
into an error), ``parallel/launch.spawn_ranks`` - the group's parent process - stops the other ranks and
exits with the failing code. The supervisor sees that exit and starts the whole group again on the same
GPUs and port, so it rejoins the router's rotation (serving/router.py) once its ``/v1/health/ready``
passes; requests it was serving have meanwhile been re-queued by the router.

Each replica runs in its own process group (``start_new_session``) so stopping it signals exactly the
processes this supervisor started. ``HIP_VISIBLE_DEVICES`` gives replica i the GPUs [i*T, (i+1)*T).
"""
from __future__ import annotations

import logging
import os
import signal
import subprocess
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

log = logging.getLogger(__name__)


@dataclass
class ReplicaProc:
    index: int
    port: int
    gpus: Optional[str]
    proc: Optional[subprocess.Popen] = None
    generation: int = 0
    restarts: List[float] = field(default_factory=list)
    exit_codes: List[int] = field(default_factory=list)
    given_up: bool = False


class ReplicaSupervisor:
    """``server_args``: arguments of ``python -m generativeaiexamples_amd.serving`` (model, weights, ...);
    ``--port`` / ``--tp`` are added per replica. ``first_env``: extra environment for the first generation
    of replica i only (tests inject faults with it)."""

    def __init__(self, server_args: List[str], replicas: int = 1, tp: int = 1, base_port: int = 8001,
                 host: str = "127.0.0.1", assign_gpus: bool = True, max_restarts: int = 5, window_s: float = 600.0,
                 backoff_s: float = 1.0, env: Optional[Dict[str, str]] = None,
                 first_env: Optional[Dict[int, Dict[str, str]]] = None, log_dir: Optional[str] = None):
        self.server_args, self.tp, self.host = list(server_args), tp, host
        self.max_restarts, self.window_s, self.backoff_s = max_restarts, window_s, backoff_s
        self.env = dict(env or {})
        self.first_env = first_env or {}
        self.log_dir = log_dir
        self.reps = [ReplicaProc(i, base_port + i,
                                 ",".join(str(g) for g in range(i * tp, (i + 1) * tp)) if assign_gpus else None)
                     for i in range(replicas)]
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self._thread: Optional[threading.Thread] = None

    @property
    def urls(self) -> List[str]:
        return [f"http://{self.host}:{r.port}" for r in self.reps]

    def _launch(self, r: ReplicaProc):
        env = dict(os.environ, **self.env)
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
            env.pop(k, None)  # the replica spawns its own ranks
        if r.gpus is not None:
            env["HIP_VISIBLE_DEVICES"] = r.gpus
        if r.generation == 0:
            env.update(self.first_env.get(r.index, {}))
        env["GAI_REPLICA"] = str(r.index)
        env["GAI_REPLICA_GENERATION"] = str(r.generation)
        cmd = [sys.executable, "-m", "generativeaiexamples_amd.serving", *self.server_args,
               "--host", self.host, "--port", str(r.port), "--tp", str(self.tp)]
        out = None
        if self.log_dir:
            os.makedirs(self.log_dir, exist_ok=True)
            out = open(os.path.join(self.log_dir, f"replica{r.index}.gen{r.generation}.log"), "wb")
        r.proc = subprocess.Popen(cmd, env=env, stdout=out, stderr=subprocess.STDOUT if out else None,
                                  start_new_session=True)
        if out is not None:
            out.close()
        log.info("replica %d generation %d: pid %d port %d gpus %s", r.index, r.generation, r.proc.pid, r.port,
                 r.gpus)

    def start(self):
        for r in self.reps:
            self._launch(r)
        self._thread = threading.Thread(target=self._monitor, daemon=True, name="replica-supervisor")
        self._thread.start()

    def _monitor(self):
        while not self._stop.wait(0.2):
            for r in self.reps:
                with self._lock:
                    if self._stop.is_set() or r.given_up or r.proc is None:
                        continue
                    code = r.proc.poll()
                    if code is None:
                        continue
                    r.exit_codes.append(code)
                    now = time.time()
                    r.restarts = [t for t in r.restarts if now - t < self.window_s]
                    if len(r.restarts) >= self.max_restarts:
                        r.given_up = True
                        log.error("replica %d exited %d; %d restarts in %.0fs, giving up", r.index, code,
                                  len(r.restarts), self.window_s)
                        continue
                    log.warning("replica %d exited with %d; restarting the TP group", r.index, code)
                    r.restarts.append(now)
                    r.generation += 1
                time.sleep(self.backoff_s * len(r.restarts))
                with self._lock:
                    if not self._stop.is_set():
                        self._launch(r)

    def kill_replica(self, index: int, sig: int = signal.SIGKILL):
        """Fault injection: signal every process of replica ``index``'s group."""
        r = self.reps[index]
        if r.proc is not None and r.proc.poll() is None:
            os.killpg(r.proc.pid, sig)

    def stop(self, timeout: float = 20.0):
        self._stop.set()
        with self._lock:
            live = [r.proc for r in self.reps if r.proc is not None and r.proc.poll() is None]
            for p in live:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.time() + timeout
        for p in live:
            try:
                p.wait(max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait(5)
        if self._thread is not None:
            self._thread.join(timeout=5)
