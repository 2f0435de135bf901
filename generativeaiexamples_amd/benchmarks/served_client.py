"""Load-generator process of ``bench.py --served``.

The clients of the served benchmark must not share the server's Python interpreter: 64 client threads
parsing SSE in the server process would compete with the engine and event-loop threads for the GIL, which
no real deployment does. ``start()`` spawns this process BEFORE the parent initialises the GPU (it never
touches the GPU itself); it runs every stream of a wave concurrently on one asyncio loop (httpx.AsyncClient)
and measures client-side TTFT (send -> first non-empty ``data:`` frame) exactly like
``evaluation/load_generator.py``.
"""
from __future__ import annotations

import asyncio
import json
import time
from typing import Dict, List


async def _one(client, url: str, question: str, max_tokens: int, delay: float = 0.0) -> Dict:
    if delay > 0:
        await asyncio.sleep(delay)
    body = {"messages": [{"role": "user", "content": question}], "use_knowledge_base": True,
            "temperature": 0.2, "top_p": 0.7, "max_tokens": max_tokens}
    t0 = time.perf_counter()
    first, n = None, 0
    async with client.stream("POST", url + "/generate", json=body) as r:
        if r.status_code != 200:
            raise RuntimeError(f"/generate returned {r.status_code}")
        async for ln in r.aiter_lines():
            if not ln.startswith("data: "):
                continue
            ch = json.loads(ln[6:])["choices"][0]
            if ch["message"]["content"]:
                n += 1
                if first is None:
                    first = time.perf_counter()
            if ch.get("finish_reason") == "[DONE]":
                break
    t1 = time.perf_counter()
    return {"ttft": (first or t1) - t0, "e2e": t1 - t0, "chunks": n, "t0": t0, "t_first": first}


async def _wave(url: str, questions: List[str], max_tokens: int, delays: List[float]) -> Dict:
    import httpx

    limits = httpx.Limits(max_connections=len(questions) + 8, max_keepalive_connections=len(questions) + 8)
    async with httpx.AsyncClient(timeout=600, limits=limits) as client:
        t0 = time.perf_counter()
        res = await asyncio.gather(*[_one(client, url, q, max_tokens, d) for q, d in zip(questions, delays)])
        return {"wall": time.perf_counter() - t0, "results": res}


def client_main(conn) -> None:
    """Command loop: ('wave', url, questions, max_tokens, delays) -> {'wall', 'results'}; ('stop',)."""
    while True:
        msg = conn.recv()
        if msg[0] == "stop":
            return
        try:
            _, url, qs, mt, delays = msg
            conn.send(asyncio.run(_wave(url, qs, mt, delays or [0.0] * len(qs))))
        except Exception as e:  # noqa: BLE001 - reported to the parent
            conn.send({"error": repr(e)})


class ClientProcess:
    def __init__(self):
        import multiprocessing as mp

        ctx = mp.get_context("spawn")
        self.conn, child = ctx.Pipe()
        self.proc = ctx.Process(target=client_main, args=(child,), daemon=True, name="served-bench-client")
        self.proc.start()

    def wave(self, url: str, questions: List[str], max_tokens: int, delays: List[float] | None = None) -> Dict:
        self.conn.send(("wave", url, list(questions), int(max_tokens), list(delays or [])))
        out = self.conn.recv()
        if "error" in out:
            raise RuntimeError(f"served-bench client: {out['error']}")
        return out

    def close(self) -> None:
        try:
            self.conn.send(("stop",))
        except Exception:  # noqa: BLE001
            pass
        self.proc.join(10)


_CLIENT: "ClientProcess | None" = None


def start() -> ClientProcess:
    """Spawn the client process (call before any GPU initialisation in this process)."""
    global _CLIENT
    if _CLIENT is None:
        _CLIENT = ClientProcess()
    return _CLIENT
