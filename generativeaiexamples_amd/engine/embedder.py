"""Embedding and reranking engines (replace the embedding NIM and the reranking NIM).

* :class:`Embedder` - E5-style asymmetric encoding (``"query: "`` / ``"passage: "`` prefixes selected
  by the NIM ``input_type`` field), ``truncate`` = END | START | NONE like ``NVIDIAEmbeddings``,
  length-sorted packing into varlen micro-batches under a token budget (no padding FLOPs).
* :class:`Reranker` - cross-encoder scoring of (query, passage) pairs (``/v1/ranking``; the
  multi-turn example reranks 40 candidates down to 4, multi_turn_rag/chains.py:147,177-191).
* :class:`DynamicBatcher` - coalesces concurrent requests (<= max_batch, <= max_delay) onto one
  engine call, the Triton ``dynamic_batching`` behaviour of the reference's MiniLM service
  (all-MiniLM-L6-v2_config.pbtxt: preferred sizes up to 256, max_queue_delay 50 ms).
"""
from __future__ import annotations

import os
import threading
import time
from concurrent.futures import Future
from typing import List, Sequence, Tuple

import torch

from ..models.bert import BertModel
from .tokenizer import Tokenizer
from ..utils.graphs import hip_graph_capture
from ..utils.profiling import roctx_range


class TruncationError(ValueError):
    pass


def _truncate(ids: List[int], max_len: int, mode: str) -> List[int]:
    if len(ids) <= max_len:
        return ids
    mode = (mode or "END").upper()
    if mode == "NONE":
        raise TruncationError(f"input has {len(ids)} tokens > max {max_len} and truncate=NONE")
    return ids[:max_len] if mode == "END" else ids[-max_len:]


class Embedder:
    def __init__(self, model: BertModel, tokenizer: Tokenizer, max_len: int | None = None,
                 max_batch_tokens: int = 65536, query_prefix: str = "query: ", passage_prefix: str = "passage: ",
                 model_name: str | None = None):
        self.model, self.tok = model, tokenizer
        self.max_len = min(max_len or model.cfg.max_position, model.cfg.max_position)
        self.max_batch_tokens = max_batch_tokens
        self.prefix = {"query": query_prefix, "passage": passage_prefix}
        self.dim = model.cfg.hidden_size
        self.name = model_name or model.cfg.name
        self.cls_id = tokenizer.token_id("[CLS]") if tokenizer.token_id("[CLS]") is not None else tokenizer.bos_id
        self.sep_id = tokenizer.token_id("[SEP]") if tokenizer.token_id("[SEP]") is not None else (
            tokenizer.eos_ids[0] if tokenizer.eos_ids else None)
        self.lock = threading.Lock()
        # query-sized batches (<= 64 sequences of <= 128 tokens) replay a captured HIP graph per (B, L) bucket:
        # the 24-layer e5-large forward of one query is ~250 launches, launch-bound without the graph
        self.use_graphs = model.device.type == "cuda" and os.environ.get("GAI_EMBED_GRAPHS", "1") == "1"
        self._graphs: dict = {}

    GRAPH_B = (1, 2, 4, 8, 16, 32, 64)
    GRAPH_L = (32, 48, 64, 96, 128)  # the bench's 78-88-token queries pad to 96, not 128

    def _graph_for(self, B: int, L: int):
        key = (B, L)
        if key not in self._graphs:
            from ..models.common import PackedAttention

            m, dev = self.model, self.model.device
            c = m.cfg
            ids = torch.zeros(B * L, dtype=torch.int32, device=dev)
            lens = torch.full((B,), L, dtype=torch.int32, device=dev)
            attn = PackedAttention([L] * B, c.num_heads, c.head_dim_padded, dev, m.dtype)
            attn.ctx = lens  # the key count per sequence IS the real length (keys past it are masked)
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                m.embed_padded(ids, lens, attn, B, L)  # warm-up (allocator, kernel attributes)
            torch.cuda.current_stream(dev).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with hip_graph_capture(g, s):
                out = m.embed_padded(ids, lens, attn, B, L)
            # the graph reads and writes attn's buffers (KV scratch, index tensors) by address: keep them alive
            self._graphs[key] = (g, ids, lens, out, attn)
        return self._graphs[key]

    def capture_graphs(self, max_batch: int = 64, max_len: int = 128) -> int:
        """Capture every (batch, length) bucket up front (service start-up): a capture while the engine thread
        runs would otherwise happen on the first query of each new shape. Returns the number captured."""
        if not self.use_graphs:
            return 0
        with self.lock:
            for B in self.GRAPH_B:
                for L in self.GRAPH_L:
                    if B <= max_batch and L <= max_len:
                        self._graph_for(B, L)
        return len(self._graphs)

    def _embed_graphed(self, seqs: List[List[int]]) -> "torch.Tensor | None":
        n, longest = len(seqs), max(len(x) for x in seqs)
        B = next((b for b in self.GRAPH_B if b >= n), None)
        L = next((x for x in self.GRAPH_L if x >= longest), None)
        if B is None or L is None:
            return None
        g, ids, lens, out, _ = self._graph_for(B, L)
        flat = torch.zeros(B, L, dtype=torch.int32)
        ln = torch.ones(B, dtype=torch.int32)
        for i, x in enumerate(seqs):
            flat[i, :len(x)] = torch.tensor(x, dtype=torch.int32)
            ln[i] = len(x)
        ids.copy_(flat.view(-1), non_blocking=True)
        lens.copy_(ln, non_blocking=True)
        g.replay()
        return out[:n].clone()

    def tokenize(self, text: str, input_type: str = "passage", truncate: str = "END") -> List[int]:
        body = self.tok.encode(self.prefix.get(input_type, "") + text)
        n_special = (self.cls_id is not None) + (self.sep_id is not None)
        body = _truncate(body, self.max_len - n_special, truncate)
        ids = ([self.cls_id] if self.cls_id is not None else []) + body + ([self.sep_id] if self.sep_id is not None else [])
        return ids

    def count_tokens(self, texts: Sequence[str]) -> int:
        return sum(len(self.tok.encode(t)) for t in texts)

    @torch.inference_mode()
    def embed_ids(self, seqs: List[List[int]]) -> torch.Tensor:
        """Token id lists -> fp32 [B, D] on the model device (input order preserved)."""
        dev = self.model.device
        if self.use_graphs and seqs:
            with self.lock:
                o = self._embed_graphed(seqs)
            if o is not None:
                return o
        order = sorted(range(len(seqs)), key=lambda i: len(seqs[i]))
        out = torch.empty(len(seqs), self.dim, dtype=torch.float32, device=dev)
        i = 0
        with self.lock:
            while i < len(order):
                j, tot = i, 0
                while j < len(order) and (tot + len(seqs[order[j]]) <= self.max_batch_tokens or j == i):
                    tot += len(seqs[order[j]])
                    j += 1
                idx = order[i:j]
                lens = [len(seqs[k]) for k in idx]
                flat = torch.tensor([t for k in idx for t in seqs[k]], dtype=torch.int32)
                cu = torch.zeros(len(idx) + 1, dtype=torch.int32)
                cu[1:] = torch.tensor(lens).cumsum(0)
                if dev.type == "cuda":
                    flat, cu = flat.pin_memory().to(dev, non_blocking=True), cu.pin_memory().to(dev, non_blocking=True)
                e = self.model.embed(flat, cu, lens)
                out[torch.tensor(idx, device=dev)] = e
                i = j
        return out

    def embed(self, texts: Sequence[str], input_type: str = "passage", truncate: str = "END") -> torch.Tensor:
        with roctx_range("embed"):
            return self.embed_ids([self.tokenize(t, input_type, truncate) for t in texts])

    # ---- coalesced serving path (/v1/embeddings, chain-server queries)
    @property
    def batcher(self) -> DynamicBatcher:
        """Concurrent embed requests -> one encoder call per batch, on the high-priority retrieval stream."""
        if getattr(self, "_batcher", None) is None:
            with self.lock:
                if getattr(self, "_batcher", None) is None:
                    from ..utils.streams import RETRIEVAL_GATE

                    self._batcher = DynamicBatcher(self._embed_requests, max_batch=256, name="embed-batcher",
                                                   gate=RETRIEVAL_GATE)
        return self._batcher

    def _embed_requests(self, reqs: List[Tuple[Tuple[str, ...], str, str]]) -> List[torch.Tensor]:
        from ..utils.streams import on_retrieval_stream

        out: List = [None] * len(reqs)
        groups: dict = {}
        for i, (texts, itype, trunc) in enumerate(reqs):
            groups.setdefault((itype, trunc), []).append(i)
        with on_retrieval_stream(self.model.device):
            for (itype, trunc), idx in groups.items():
                seqs, spans = [], []
                for i in idx:
                    try:
                        ids = [self.tokenize(t, itype, trunc) for t in reqs[i][0]]
                    except TruncationError as e:  # this request fails alone
                        out[i] = e
                        continue
                    spans.append((i, len(seqs), len(seqs) + len(ids)))
                    seqs += ids
                if not seqs:
                    continue
                e = self.embed_ids(seqs)
                for i, a, b in spans:
                    out[i] = e[a:b]
        return out

    def embed_coalesced(self, texts: Sequence[str], input_type: str = "passage", truncate: str = "END") -> torch.Tensor:
        r = self.batcher.submit((tuple(texts), input_type, truncate)).result()
        if isinstance(r, Exception):
            raise r
        return r


class ClipEmbedder:
    """NV-CLIP-style multimodal embedder over :class:`~..models.clip.ClipModel` (BASELINE config 4,
    SURVEY W14 "NV-CLIP search"): each ``/v1/embeddings`` input is either text or an image given as a
    ``data:image/...;base64,`` URI, and both land in the same normalised projection space. Images are
    batched through the vision tower (patchify kernel + MFMA GEMMs + packed bidirectional attention),
    texts through the causal text tower."""

    accepts_images = True

    def __init__(self, model, tokenizer: Tokenizer, model_name: str | None = None, max_batch_images: int = 64):
        self.model, self.tok = model, tokenizer
        self.name = model_name or model.cfg.name
        self.dim = model.cfg.projection_dim
        self.max_len = model.cfg.max_text_len
        self.max_batch_images = max_batch_images
        self.lock = threading.Lock()

    @staticmethod
    def is_image(x) -> bool:
        return not isinstance(x, str) or x.startswith("data:image")

    def tokenize(self, text, input_type: str = "query", truncate: str = "END") -> List[int]:
        if self.is_image(text):
            return [0] * (self.model.cfg.num_patches + 1)  # usage accounting: one token per patch + CLS
        body = self.tok.encode(text)
        bos = [self.tok.bos_id] if self.tok.bos_id is not None else []
        eos = [self.tok.eos_ids[0]] if self.tok.eos_ids else []
        body = _truncate(body, self.max_len - len(bos) - len(eos), truncate)
        return bos + body + eos

    @torch.inference_mode()
    def embed(self, inputs: Sequence, input_type: str = "query", truncate: str = "END") -> torch.Tensor:
        dev = self.model.device
        out = torch.empty(len(inputs), self.dim, dtype=torch.float32, device=dev)
        img_idx = [i for i, x in enumerate(inputs) if self.is_image(x)]
        txt_idx = [i for i, x in enumerate(inputs) if not self.is_image(x)]
        with self.lock:
            for s in range(0, len(img_idx), self.max_batch_images):
                idx = img_idx[s:s + self.max_batch_images]
                px = self.model.preprocess([inputs[i] for i in idx])
                out[torch.tensor(idx, device=dev)] = self.model.encode_image(px)
            if txt_idx:
                toks = [self.tokenize(inputs[i], input_type, truncate) for i in txt_idx]
                out[torch.tensor(txt_idx, device=dev)] = self.model.encode_text(toks)
        return out


class Reranker:
    def __init__(self, model: BertModel, tokenizer: Tokenizer, max_len: int | None = None,
                 max_batch_tokens: int = 65536, model_name: str | None = None):
        assert model.cfg.num_labels > 0, "reranker needs a cross-encoder head (num_labels > 0)"
        self.model, self.tok = model, tokenizer
        self.max_len = min(max_len or model.cfg.max_position, model.cfg.max_position)
        self.max_batch_tokens = max_batch_tokens
        self.name = model_name or model.cfg.name
        self.cls_id = tokenizer.token_id("[CLS]") if tokenizer.token_id("[CLS]") is not None else tokenizer.bos_id
        self.sep_id = tokenizer.token_id("[SEP]") if tokenizer.token_id("[SEP]") is not None else (
            tokenizer.eos_ids[0] if tokenizer.eos_ids else 0)
        self.lock = threading.Lock()

    def pair_ids(self, query: str, passage: str, truncate: str = "END") -> Tuple[List[int], List[int]]:
        q = self.tok.encode(query)[: self.max_len // 2]
        p = self.tok.encode(passage)
        budget = self.max_len - len(q) - 3
        p = _truncate(p, max(budget, 1), truncate)
        ids = [self.cls_id] + q + [self.sep_id] + p + [self.sep_id]
        types = [0] * (len(q) + 2) + [1] * (len(p) + 1)
        return ids, types

    def score_many(self, items: Sequence[Tuple[str, Sequence[str]]], truncate: str = "END") -> List[List[float]]:
        return [self.score(q, ps, truncate) for q, ps in items]

    @torch.inference_mode()
    def score(self, query: str, passages: Sequence[str], truncate: str = "END") -> List[float]:
        if not passages:
            return []
        pairs = [self.pair_ids(query, p, truncate) for p in passages]
        dev = self.model.device
        scores = [0.0] * len(pairs)
        order = sorted(range(len(pairs)), key=lambda i: len(pairs[i][0]))
        i = 0
        with self.lock:
            while i < len(order):
                j, tot = i, 0
                while j < len(order) and (tot + len(pairs[order[j]][0]) <= self.max_batch_tokens or j == i):
                    tot += len(pairs[order[j]][0])
                    j += 1
                idx = order[i:j]
                lens = [len(pairs[k][0]) for k in idx]
                flat = torch.tensor([t for k in idx for t in pairs[k][0]], dtype=torch.int32, device=dev)
                typ = torch.tensor([t for k in idx for t in pairs[k][1]], dtype=torch.int32, device=dev)
                cu = torch.zeros(len(idx) + 1, dtype=torch.int32)
                cu[1:] = torch.tensor(lens).cumsum(0)
                s = self.model.score(flat, cu.to(dev), lens, typ).float().cpu().tolist()
                for k, v in zip(idx, s):
                    scores[k] = v
                i = j
        return scores

    def rank(self, query: str, passages: Sequence[str], top_n: int | None = None, truncate: str = "END"):
        """-> [(index, logit)] sorted by relevance (the NIM ``rankings`` list)."""
        s = self.score(query, passages, truncate)
        r = sorted(enumerate(s), key=lambda x: -x[1])
        return r[:top_n] if top_n else r


class DynamicBatcher:
    """Thread-safe request coalescer in front of a batch function ``fn(list[item]) -> list[result]``
    (Triton ``dynamic_batching`` semantics of the reference's embedding service,
    all-MiniLM-L6-v2_config.pbtxt:19-29: preferred batch sizes up to 256, bounded queue delay).

    One worker thread runs ``fn``. When it is free it takes everything queued (up to ``max_batch``) at
    once, so an idle service adds no latency; while ``fn`` runs, new requests queue and form the next
    batch. ``max_delay_ms`` > 0 additionally holds a batch that is not yet a preferred size for up to that
    long to collect more. ``batch_sizes`` keeps the recent batch sizes (tests / metrics)."""

    def __init__(self, fn, max_batch: int = 256, max_delay_ms: float = 0.0, preferred=None, name="dynamic-batcher",
                 gate=None):
        self.fn, self.max_batch, self.max_delay = fn, max_batch, max_delay_ms / 1000.0
        self.gate = gate  # utils.streams.RetrievalGate: a request counts as pending from submit to result
        self.preferred = set(preferred or [1 << i for i in range(9) if (1 << i) <= max_batch])
        self.q: List[Tuple[object, Future]] = []
        self.cv = threading.Condition()
        self.stop = False
        self.batch_sizes: List[int] = []
        self.t = threading.Thread(target=self._loop, daemon=True, name=name)
        self.t.start()

    def submit(self, item) -> Future:
        f: Future = Future()
        with self.cv:
            if self.stop:
                raise RuntimeError("batcher closed")
            if self.gate is not None:
                self.gate.enter()
                f.add_done_callback(lambda _f: self.gate.exit())
            self.q.append((item, f))
            self.cv.notify()
        return f

    def submit_many(self, items) -> List[Future]:
        """Enqueue several items atomically: an idle worker takes them as ONE batch (e.g. the augmented queries of one
        multi-query retrieval)."""
        futs: List[Future] = []
        with self.cv:
            if self.stop:
                raise RuntimeError("batcher closed")
            for item in items:
                f: Future = Future()
                if self.gate is not None:
                    self.gate.enter()
                    f.add_done_callback(lambda _f: self.gate.exit())
                self.q.append((item, f))
                futs.append(f)
            self.cv.notify()
        return futs

    def __call__(self, item):
        return self.submit(item).result()

    def _loop(self):
        while True:
            with self.cv:
                while not self.q and not self.stop:
                    self.cv.wait()
                if self.stop and not self.q:
                    return
                if self.max_delay > 0 and len(self.q) not in self.preferred:
                    deadline = time.perf_counter() + self.max_delay
                    while len(self.q) < self.max_batch and len(self.q) not in self.preferred and not self.stop:
                        rem = deadline - time.perf_counter()
                        if rem <= 0:
                            break
                        self.cv.wait(rem)
                batch, self.q = self.q[: self.max_batch], self.q[self.max_batch:]
            self.batch_sizes.append(len(batch))
            del self.batch_sizes[:-1024]
            try:
                res = self.fn([b[0] for b in batch])
                for (_, f), r in zip(batch, res):
                    f.set_result(r)
            except Exception as e:  # propagate to every waiter
                for _, f in batch:
                    if not f.done():
                        f.set_exception(e)

    def close(self):
        with self.cv:
            self.stop = True
            self.cv.notify_all()


class DecoderReranker:
    """Service over :class:`~..models.decoder_reranker.DecoderRerankerModel` (NV-RerankQA-Mistral-4B class):
    pairs are formatted ``"question:{q} \\n \\n passage:{p}"`` (BOS first), passages truncated to fit
    ``max_length``, and every pair of one or many queries is packed into varlen micro-batches under a
    token budget (one bidirectional encoder pass per micro-batch, no padding)."""

    def __init__(self, model, tokenizer: Tokenizer, model_name: str | None = None, max_batch_tokens: int = 65536):
        self.model, self.tok = model, tokenizer
        self.name = model_name or model.cfg.name
        self.max_len = model.cfg.max_length
        self.max_batch_tokens = max_batch_tokens
        self.lock = threading.Lock()

    def pair_ids(self, query: str, passage: str, truncate: str = "END") -> List[int]:
        bos = [self.tok.bos_id] if self.tok.bos_id is not None else []
        q = self.tok.encode(f"question:{query} \n \n passage:")[: self.max_len // 2]
        p = _truncate(self.tok.encode(passage), max(1, self.max_len - len(q) - len(bos)), truncate)
        return bos + q + p

    @torch.inference_mode()
    def score_many(self, items: Sequence[Tuple[str, Sequence[str]]], truncate: str = "END") -> List[List[float]]:
        pairs = [(qi, self.pair_ids(q, p, truncate)) for qi, (q, ps) in enumerate(items) for p in ps]
        flat_scores = [0.0] * len(pairs)
        dev = self.model.device
        order = sorted(range(len(pairs)), key=lambda i: len(pairs[i][1]))
        i = 0
        with self.lock:
            while i < len(order):
                j, tot = i, 0
                while j < len(order) and (tot + len(pairs[order[j]][1]) <= self.max_batch_tokens or j == i):
                    tot += len(pairs[order[j]][1])
                    j += 1
                idx = order[i:j]
                lens = [len(pairs[k][1]) for k in idx]
                flat = torch.tensor([t for k in idx for t in pairs[k][1]], dtype=torch.int32).to(dev)
                cu = torch.zeros(len(idx) + 1, dtype=torch.int32)
                cu[1:] = torch.tensor(lens).cumsum(0)
                sc = self.model.score(flat, cu.to(dev), lens).float().cpu().tolist()
                for k, v in zip(idx, sc):
                    flat_scores[k] = v
                i = j
        out: List[List[float]] = [[] for _ in items]
        for (qi, _), v in zip(pairs, flat_scores):
            out[qi].append(v)
        return out

    def score(self, query: str, passages: Sequence[str], truncate: str = "END") -> List[float]:
        return self.score_many([(query, passages)], truncate)[0] if passages else []
