"""Parallel guardrails (reference nemo/NeMo-Guardrails/Parallel_Rails_Tutorial: content-safety
and topic-control 8B models run as input rails in parallel, output rails on the stream with chunk
200 / context 50).

* input rails run concurrently (thread pool: each rail is an independent LLM call - on one MI355X the
  engine batches them into the same decode steps); the request is blocked when any rail says unsafe;
* output rails check the streamed answer in windows of ``chunk`` characters with ``context`` characters
  of overlap, stopping the stream with the refusal message at the first unsafe window.
A rail is any callable ``(text) -> bool`` (True = allowed); ``llm_rail`` builds one from a chat model
and a yes/no policy prompt, so the rail models can be served by this framework's /v1 endpoints.
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterator, List, Optional

Rail = Callable[[str], bool]
REFUSAL = "I'm sorry, I can't respond to that."

CONTENT_SAFETY_POLICY = ("You are a content safety classifier. Reply 'unsafe' if the text requests or contains "
                         "violence, self-harm, hate, sexual content involving minors, or instructions for crimes; "
                         "otherwise reply 'safe'. Reply with one word.")
TOPIC_POLICY = ("You check whether a message is on-topic for a technical documentation assistant. Reply 'on-topic' "
                "or 'off-topic'. Reply with one word.")


def llm_rail(llm, policy: str, allowed_words=("safe", "on-topic", "yes")) -> Rail:
    def rail(text: str) -> bool:
        out = llm.invoke([{"role": "system", "content": policy}, {"role": "user", "content": text}])
        return out.strip().lower().split()[0].strip(".,!") in allowed_words if out.strip() else False
    return rail


@dataclass
class Guardrails:
    input_rails: Dict[str, Rail] = field(default_factory=dict)
    output_rails: Dict[str, Rail] = field(default_factory=dict)
    chunk: int = 200
    context: int = 50
    refusal: str = REFUSAL
    parallel: bool = True

    def check_input(self, text: str) -> Optional[str]:
        """-> name of the first failing rail, or None when every rail allows the text."""
        if not self.input_rails:
            return None
        names = list(self.input_rails)
        if self.parallel and len(names) > 1:
            with ThreadPoolExecutor(len(names)) as ex:
                ok = list(ex.map(lambda n: self.input_rails[n](text), names))
        else:
            ok = [self.input_rails[n](text) for n in names]
        for n, o in zip(names, ok):
            if not o:
                return n
        return None

    def _output_ok(self, window: str) -> bool:
        if not self.output_rails:
            return True
        rails = list(self.output_rails.values())
        if self.parallel and len(rails) > 1:
            with ThreadPoolExecutor(len(rails)) as ex:
                return all(ex.map(lambda r: r(window), rails))
        return all(r(window) for r in rails)

    def guard_stream(self, stream: Iterator[str]) -> Iterator[str]:
        """Holds back at most ``chunk`` characters: each full window (with ``context`` chars of the previous
        one) is checked before it is released."""
        pending, prev_tail = "", ""
        for piece in stream:
            pending += piece
            while len(pending) >= self.chunk:
                window, pending = pending[: self.chunk], pending[self.chunk:]
                if not self._output_ok(prev_tail + window):
                    yield "\n" + self.refusal
                    return
                prev_tail = window[-self.context:]
                yield window
        if pending:
            if not self._output_ok(prev_tail + pending):
                yield "\n" + self.refusal
                return
            yield pending

    def generate(self, query: str, answer_stream_fn: Callable[[], Iterator[str]]) -> Iterator[str]:
        failed = self.check_input(query)
        if failed:
            yield self.refusal
            return
        yield from self.guard_stream(answer_stream_fn())
