"""Question answering over the live transcript stream (reference: /root/reference/community/fm-asr-streaming-rag/
chain-server/chains.py:33-199, utils.py:126-164). The model first classifies the question's intent:

* ``RecentSummary`` ("what was said in the last five minutes?") - the chunks stored since then, by time;
* ``TimeWindow`` ("what were they talking about an hour ago?") - the chunks within +/- ``window`` seconds of then;
* ``SpecificTopic`` / ``Unknown`` - similarity search (+ rerank, outlier drop) over the stream's vector index.

For the two time intents a second classification extracts (number, unit). When more chunks come back than
``max_docs``, they are either reduced by recursive summarization (``allow_summary``) or cut to the most recent /
the closest in time. Structured outputs are parsed leniently (the first JSON object in the reply, common unit
spellings), and any failure falls back to similarity retrieval like the reference.
"""
from __future__ import annotations

import datetime as _dt
import json
import logging
import re
from dataclasses import dataclass
from typing import Callable, Dict, Generator, Iterable, List, Optional

from ...index.hbm_index import Document
from ...rag.text_splitter import RecursiveCharacterTextSplitter
from .stream_store import StreamRetriever, TextAccumulator

log = logging.getLogger(__name__)
MAX_SUMMARIZATION_ATTEMPTS = 3
INTENTS = ("SpecificTopic", "RecentSummary", "TimeWindow", "Unknown")

INTENT_PROMPT = (
    "You sort questions about a live radio transcript into one of four kinds and answer ONLY with JSON of the form "
    '{"intentType": "<kind>"}. Kinds: "RecentSummary" - the user wants a summary or recap of what was said over a '
    'recent stretch of time ("what happened in the last 10 minutes?"); "TimeWindow" - the user asks about what was '
    'said at some point in the past ("what were they discussing an hour ago?"); "SpecificTopic" - the user asks '
    'about a subject, person or event without a time reference; "Unknown" - none of these.')
RECENCY_PROMPT = (
    "Extract the amount of time a question refers to. Answer ONLY with JSON of the form "
    '{"timeNum": <number>, "timeUnit": "<seconds|minutes|hours|days|weeks>"}. "the last half hour" -> '
    '{"timeNum": 30, "timeUnit": "minutes"}; "two hours ago" -> {"timeNum": 2, "timeUnit": "hours"}.')
SUMMARIZATION_PROMPT = (
    "Summarize the following radio transcript excerpt in a few sentences, keeping names, numbers and events.")
RAG_SYSTEM = (
    "You answer questions about a live radio broadcast using its transcript. Use only the transcript; if it does not "
    "contain the answer, say so. Be concise.")

_UNITS = {"s": "seconds", "sec": "seconds", "secs": "seconds", "second": "seconds", "seconds": "seconds",
          "m": "minutes", "min": "minutes", "mins": "minutes", "minute": "minutes", "minutes": "minutes",
          "h": "hours", "hr": "hours", "hrs": "hours", "hour": "hours", "hours": "hours",
          "d": "days", "day": "days", "days": "days", "w": "weeks", "wk": "weeks", "week": "weeks", "weeks": "weeks"}


@dataclass
class TimeResponse:
    timeNum: float
    timeUnit: str

    def to_seconds(self) -> float:
        unit = _UNITS.get(str(self.timeUnit).strip().lower().rstrip("."))
        if unit is None:
            raise ValueError(f"unknown time unit {self.timeUnit!r}")
        return _dt.timedelta(**{unit: float(self.timeNum)}).total_seconds()


def first_json_object(text: str) -> Optional[dict]:
    """The first parseable {...} object in a model reply (after normalising curly quotes)."""
    for t in (text, text.replace("\u201c", '"').replace("\u201d", '"').replace("'", '"')):
        for m in re.finditer(r"\{[^{}]*\}", t):
            try:
                obj = json.loads(m.group(0))
            except ValueError:
                continue
            if isinstance(obj, dict):
                return obj
    return None


@dataclass
class StreamQuery:
    """GET / POST /generate body of the reference (common.py LLMConfig)."""
    question: str
    use_knowledge_base: bool = True
    allow_summary: bool = False
    temperature: float = 0.2
    max_docs: int = 8
    num_tokens: int = 512
    context: Optional[str] = None


class StreamRagChain:
    def __init__(self, llm, accumulator: TextAccumulator, retriever: StreamRetriever,
                 clock: Callable[[], _dt.datetime] = _dt.datetime.now):
        self.llm, self.acc, self.ret, self.clock = llm, accumulator, retriever, clock
        self.db = accumulator.timestamp_db

    # ---- model calls
    def _ask(self, system: str, user: str, **kw) -> str:
        return self.llm.invoke([{"role": "system", "content": system}, {"role": "user", "content": user}], **kw)

    def classify_intent(self, question: str) -> Optional[str]:
        obj = first_json_object(self._ask(INTENT_PROMPT, question, temperature=0.0, max_tokens=32))
        intent = obj.get("intentType") if obj else None
        return intent if intent in INTENTS else None

    def classify_time(self, question: str) -> Optional[TimeResponse]:
        obj = first_json_object(self._ask(RECENCY_PROMPT, question, temperature=0.0, max_tokens=48))
        if not obj or "timeNum" not in obj or "timeUnit" not in obj:
            return None
        try:
            return TimeResponse(float(obj["timeNum"]), str(obj["timeUnit"]))
        except (TypeError, ValueError):
            return None

    def _generate(self, docs: Iterable[Document], q: StreamQuery) -> Generator[str, None, None]:
        context = "\n".join(d.page_content for d in docs)
        if q.context:
            context = f"{q.context}\n{context}"
        msgs = [{"role": "system", "content": RAG_SYSTEM},
                {"role": "user", "content": f"Transcript: '{context}'\nUser: '{q.question}'\nAI:"}]
        yield from self.llm.stream(msgs, temperature=q.temperature, max_tokens=q.num_tokens)

    def summarize(self, docs: List[Document], max_docs: int) -> List[Document]:
        """One reduction round: every ``max_docs`` chunks summarized, the summaries re-split (no overlap)."""
        splitter = RecursiveCharacterTextSplitter(self.acc.chunk_size, 0)
        summary = ""
        for i in range(0, len(docs), max_docs):
            text = " ".join(d.page_content for d in docs[i:i + max_docs])
            summary = f"{summary} {self._ask(SUMMARIZATION_PROMPT, text, temperature=0.2, max_tokens=256)}"
        return [Document(c, {}) for c in splitter.split_text(summary.strip())]

    # ---- answers
    def answer(self, q: StreamQuery) -> Generator[str, None, None]:
        if not q.use_knowledge_base:
            yield from self.llm.stream([{"role": "user", "content": q.question}], temperature=q.temperature,
                                       max_tokens=q.num_tokens)
            return
        intent = self.classify_intent(q.question)
        if intent in ("RecentSummary", "TimeWindow"):
            recency = self.classify_time(q.question)
            try:
                if recency is None:
                    raise ValueError("no time reference parsed")
                seconds = recency.to_seconds()
                if intent == "RecentSummary":
                    yield from self.answer_by_recent(q, seconds)
                else:
                    yield from self.answer_by_past(q, seconds)
                return
            except ValueError as e:
                log.warning("time-based answer failed (%s); falling back to similarity retrieval", e)
        yield from self.answer_by_relevance(q)

    def answer_by_relevance(self, q: StreamQuery) -> Generator[str, None, None]:
        docs = self.ret.search(q.question, max_entries=q.max_docs)
        if not docs:
            yield "*Found no documents related to the query*"
            return
        yield f"*Returned {len(docs)} related entries*\n\n"
        yield from self._generate(docs, q)

    def _reduce(self, docs: List[Document], q: StreamQuery, keep) -> Generator[str, None, List[Document]]:
        if len(docs) <= q.max_docs:
            return docs
        if q.allow_summary:
            yield "*Using summarization to reduce context*\n"
            for attempt in range(MAX_SUMMARIZATION_ATTEMPTS):
                docs = self.summarize(docs, q.max_docs)
                yield f"*Reduced to {len(docs)} entries on attempt {attempt + 1}*\n"
                if len(docs) <= q.max_docs:
                    break
            return docs[-q.max_docs:]
        docs = keep(docs)
        yield f"*Reduced to {len(docs)} entries*\n"
        return docs

    def answer_by_recent(self, q: StreamQuery, seconds: float) -> Generator[str, None, None]:
        docs = self.db.recent(self.clock() - _dt.timedelta(seconds=seconds))
        yield f"*Found {len(docs)} entries from the last {seconds:.0f}s*\n"
        docs = yield from self._reduce(docs, q, lambda ds: ds[-q.max_docs:])
        if docs:
            yield "\n"
            yield from self._generate(docs, q)

    def answer_by_past(self, q: StreamQuery, seconds: float, window: float = 90.0) -> Generator[str, None, None]:
        when = self.clock() - _dt.timedelta(seconds=seconds)
        docs = self.db.past(when, window=window)
        yield f"*Found {len(docs)} entries from {seconds:.0f}s ago (+/- {window:.0f}s)*\n"
        closest = lambda ds: sorted(ds, key=lambda d: abs((d.metadata["tstamp"] - when).total_seconds()))[:q.max_docs]  # noqa: E731
        docs = yield from self._reduce(docs, q, closest)
        if docs:
            yield "\n"
            yield from self._generate(docs, q)


def query_from_dict(d: Dict) -> StreamQuery:
    keys = StreamQuery.__dataclass_fields__.keys()
    return StreamQuery(**{k: v for k, v in d.items() if k in keys})
