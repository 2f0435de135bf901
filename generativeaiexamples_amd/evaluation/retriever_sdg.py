"""Retriever synthetic-data generation and evaluation (reference
nemo/retriever-synthetic-data-generation: ``nemo_retriever_sdg/{dataset,qa_generator,filter,evaluator}.py``,
``scripts/run_pipeline.py``, ``scripts/conf/config.yaml``).

Pipeline, all in-process against this framework's engines or any OpenAI-compatible ``/v1`` server:

  corpus (SQuAD JSON or raw-doc JSONL)
    -> QA generation: an instruction LLM writes ``Question: / Answer: / Explanation:`` blocks per passage
    -> filters, each annotating every QA with ``<prefix>__keep``:
         * easiness: cosine(passage, question) from the embedder; questions whose similarity is ABOVE the
           threshold (fixed, or the ``percentile``-th percentile of the batch) are too easy and dropped,
         * answerability: LLM judge answering N Y/N criteria as JSON; any "N" drops the question
    -> SQuAD JSON (all / filtered) + BEIR folders (corpus.jsonl, queries.jsonl, qrels/test.tsv)
    -> retrieval evaluation of embedder(s) on the BEIR data: exact cosine top-k (HBM index kernel on GPU,
       torch on CPU) scored with trec-style NDCG@k, MAP@k, Recall@k, P@k, plus the per-query
       "a relevant doc in the top 5" flags.

Differences from the reference: the embedder and retrieval run in-process (no SentenceBERT/BEIR packages,
no NIM round trip); the metric code is this module's own (pytrec_eval is not available offline), with
binary-relevance formulas documented on :func:`ir_metrics`.
"""
from __future__ import annotations

import argparse
import copy
import csv
import json
import logging
import math
import os
import re
import uuid
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from .llm import LLMFn

log = logging.getLogger(__name__)

EmbedFn = Callable[[List[str], str], np.ndarray]  # (texts, "query" | "passage") -> L2-normalised [n, d]

QA_SYSTEM_PROMPT = (
    "You are a data annotator trying to generate questions and corresponding answers based on an input document.\n"
    "- Generate questions that could be answered by a specific piece of information in the document, asked by "
    "someone who is not looking at the document.\n"
    "- Avoid vague questions (what is the purpose of the document, what does it refer to).\n"
    "- Vary phrasing and difficulty; do not copy sentences from the document.\n"
    "- Start every question with 'Question:', every answer with 'Answer:' and every justification with "
    "'Explanation:'.")

JUDGE_SYSTEM_PROMPT = (
    "You are an evaluator who is rating questions to given context passages. For each criterion answer Y or N.\n"
    "Criterion 1 - Is the question self-contained (answerable without references not given in the question)?\n"
    "Criterion 2 - Is it clear what type of answer the question seeks?\n"
    "Criterion 3 - Does the context contain information that answers the question or part of it?\n"
    "Criterion 4 - Does the context completely answer the question?\n"
    "Reply with only a JSON object {\"criterion_1\": \"Y|N\", ..., \"criterion_4\": \"Y|N\"} (explanations "
    "optional as criterion_<i>_explanation).")
JUDGE_USER_TEMPLATE = "Context Passage:\n{context}\nQuestion:\n{question}\n"


# ------------------------------------------------------------------------------------------------ corpus
class Corpus:
    """SQuAD-v2-shaped container: ``{"data": [{"paragraphs": [{"context", "document_id", "qas": [...]}]}]}``."""

    def __init__(self, data: dict):
        self.data = data

    @classmethod
    def load(cls, path: str, fmt: str) -> "Corpus":
        if fmt == "squad":
            with open(path, encoding="utf-8") as f:
                data = json.load(f)
        elif fmt == "rawdoc":
            ex = []
            with open(path, encoding="utf-8") as f:
                for i, line in enumerate(f):
                    if not line.strip():
                        continue
                    d = json.loads(line)
                    ex.append({"paragraphs": [{"context": d["text"], "document_id": d.get("_id", f"doc{i}"),
                                               "title": d.get("title", ""), "qas": []}]})
            data = {"data": ex, "version": "2.0"}
        else:
            raise ValueError(f"unknown input format {fmt!r} (squad | rawdoc)")
        for i, ex in enumerate(data["data"]):  # every paragraph gets a stable id
            p = ex["paragraphs"][0]
            p.setdefault("document_id", f"doc{i}")
            p.setdefault("qas", [])
        return cls(data)

    def paragraphs(self) -> Iterable[dict]:
        for ex in self.data["data"]:
            yield ex["paragraphs"][0]

    def qas(self) -> Iterable[Tuple[dict, dict]]:
        for p in self.paragraphs():
            for qa in p.get("qas") or []:
                yield p, qa

    def num_questions(self) -> int:
        return sum(1 for _ in self.qas())

    def copy(self) -> "Corpus":
        return Corpus(copy.deepcopy(self.data))

    def to_json(self, path: str):
        with open(path, "w", encoding="utf-8") as f:
            json.dump(self.data, f, indent=1)

    def to_csv(self, path: str):
        with open(path, "w", newline="", encoding="utf-8") as f:
            w = csv.writer(f)
            w.writerow(["doc_id", "context", "question", "answer", "synthetic"])
            for p, qa in self.qas():
                ans = (qa.get("answers") or [{"text": ""}])[0]["text"]
                w.writerow([p["document_id"], p["context"], qa["question"], ans, bool(qa.get("synthetic"))])

    def to_beir(self, out_dir: str, create_original: bool = False):
        """Writes ``synthetic/`` (and ``original/`` for non-synthetic questions) BEIR folders."""
        kinds = [("synthetic", True)] + ([("original", False)] if create_original else [])
        for kind, synthetic in kinds:
            d = os.path.join(out_dir, kind)
            os.makedirs(os.path.join(d, "qrels"), exist_ok=True)
            with open(os.path.join(d, "corpus.jsonl"), "w", encoding="utf-8") as f:
                for p in self.paragraphs():
                    f.write(json.dumps({"_id": p["document_id"], "title": p.get("title", ""), "text": p["context"],
                                        "metadata": {}}) + "\n")
            with open(os.path.join(d, "queries.jsonl"), "w", encoding="utf-8") as fq, \
                    open(os.path.join(d, "qrels", "test.tsv"), "w", encoding="utf-8") as fr:
                fr.write("query-id\tcorpus-id\tscore\n")
                for p, qa in self.qas():
                    if bool(qa.get("synthetic")) != synthetic:
                        continue
                    fq.write(json.dumps({"_id": qa["id"], "text": qa["question"], "metadata": {}}) + "\n")
                    fr.write(f"{qa['id']}\t{p['document_id']}\t1\n")


def load_beir(folder: str) -> Tuple[Dict[str, dict], Dict[str, str], Dict[str, Dict[str, int]]]:
    corpus, queries, qrels = {}, {}, {}
    with open(os.path.join(folder, "corpus.jsonl"), encoding="utf-8") as f:
        for line in f:
            d = json.loads(line)
            corpus[d["_id"]] = {"title": d.get("title", ""), "text": d["text"]}
    with open(os.path.join(folder, "queries.jsonl"), encoding="utf-8") as f:
        for line in f:
            d = json.loads(line)
            queries[d["_id"]] = d["text"]
    with open(os.path.join(folder, "qrels", "test.tsv"), encoding="utf-8") as f:
        next(f)
        for line in f:
            q, c, s = line.rstrip("\n").split("\t")
            qrels.setdefault(q, {})[c] = int(s)
    return corpus, queries, qrels


# ------------------------------------------------------------------------------------------------ generation
_BLOCK = re.compile(r"Question\s*\d*\s*:(.*?)Answer\s*\d*\s*:(.*?)(?:Explanation\s*\d*\s*:(.*?))?(?=Question\s*\d*\s*:|\Z)",
                    re.S | re.I)


def parse_qa_blocks(reply: str) -> List[dict]:
    """``Question: ... Answer: ... [Explanation: ...]`` blocks -> SQuAD qas entries (synthetic)."""
    out = []
    for q, a, _expl in _BLOCK.findall(reply):
        q, a = q.strip(), a.strip()
        if q and a:
            out.append({"question": q, "id": uuid.uuid4().hex[:16], "synthetic": True,
                        "answers": [{"text": a, "answer_start": -1, "synthetic": True}]})
    return out


class QAGenerator:
    def __init__(self, llm: LLMFn, num_questions: int = 5, max_examples: Optional[int] = None,
                 system_prompt: str = QA_SYSTEM_PROMPT, cache_file: Optional[str] = None):
        self.llm, self.num_questions, self.max_examples = llm, num_questions, max_examples
        self.system_prompt, self.cache_file = system_prompt, cache_file

    def generate(self, corpus: Corpus) -> Corpus:
        """Adds synthetic qas to the first ``max_examples`` paragraphs (cached line per paragraph when a
        cache file is given, so an interrupted run resumes)."""
        out = corpus.copy()
        cached = []
        if self.cache_file and os.path.isfile(self.cache_file):
            with open(self.cache_file, encoding="utf-8") as f:
                cached = [json.loads(line) for line in f if line.strip()]
        n = 0
        for i, ex in enumerate(out.data["data"]):
            if self.max_examples is not None and n >= self.max_examples:
                break
            p = ex["paragraphs"][0]
            if i < len(cached):
                if cached[i]["paragraphs"][0]["context"] != p["context"]:
                    raise ValueError("QA cache does not match the corpus")
                out.data["data"][i] = cached[i]
                n += 1
                continue
            reply = self.llm([{"role": "system", "content": self.system_prompt},
                              {"role": "user", "content": f"Input document:\n{p['context']}\n\nGenerate "
                                                          f"{self.num_questions} questions.\nGenerated Questions:"}])
            p["qas"] = list(p.get("qas") or []) + parse_qa_blocks(reply)[: self.num_questions]
            if self.cache_file:
                with open(self.cache_file, "a", encoding="utf-8") as f:
                    f.write(json.dumps(ex) + "\n")
            n += 1
        return out


# ------------------------------------------------------------------------------------------------ filters
class EasinessFilter:
    """Drops questions that are too easy for the embedder: cosine(passage, question) above a threshold
    (``threshold``, or the ``percentile``-th percentile over all synthetic questions)."""

    prefix = "easiness"

    def __init__(self, embed: EmbedFn, percentile: Optional[float] = 70.0, threshold: Optional[float] = None,
                 batch_size: int = 64):
        if (percentile is None) == (threshold is None):
            raise ValueError("give exactly one of percentile / threshold")
        self.embed, self.percentile, self.threshold, self.batch_size = embed, percentile, threshold, batch_size

    def apply(self, corpus: Corpus) -> Corpus:
        out = corpus.copy()
        pairs = list(out.qas())
        sims: List[float] = []
        for s in range(0, len(pairs), self.batch_size):
            chunk = pairs[s:s + self.batch_size]
            dp = self.embed([p["context"] for p, _ in chunk], "passage")
            dq = self.embed([qa["question"] for _, qa in chunk], "query")
            sims += np.einsum("nd,nd->n", np.asarray(dp, np.float32), np.asarray(dq, np.float32)).tolist()
        if not sims:
            return out
        thr = self.threshold if self.threshold is not None else float(np.percentile(sims, self.percentile))
        for (_, qa), s in zip(pairs, sims):
            qa[f"{self.prefix}__cossim"] = float(s)
            qa[f"{self.prefix}__keep"] = bool(s <= thr)
        return out


class AnswerabilityFilter:
    """LLM judge over ``num_criteria`` Y/N criteria (JSON reply); any N drops the question, an unparseable
    reply marks it ``None`` (kept, like the reference)."""

    prefix = "answerability"

    def __init__(self, llm: LLMFn, num_criteria: int = 4, system_prompt: str = JUDGE_SYSTEM_PROMPT,
                 user_template: str = JUDGE_USER_TEMPLATE):
        self.llm, self.num_criteria = llm, num_criteria
        self.system_prompt, self.user_template = system_prompt, user_template

    def judge(self, context: str, question: str) -> Tuple[Optional[bool], str]:
        reply = self.llm([{"role": "user", "content": self.system_prompt + "\n\n" +
                           self.user_template.format(context=context, question=question)}])
        m = re.search(r"\{.*\}", reply, re.S)
        try:
            obj = json.loads(m.group(0) if m else reply)
            keep = all(str(obj[f"criterion_{i + 1}"]).strip().upper().startswith("Y") for i in range(self.num_criteria))
        except (ValueError, KeyError, TypeError):
            keep = None
        return keep, reply

    def apply(self, corpus: Corpus) -> Corpus:
        out = corpus.copy()
        for p, qa in out.qas():
            keep, reply = self.judge(p["context"], qa["question"])
            qa[f"{self.prefix}__keep"] = keep
            qa[f"{self.prefix}__llm_as_judge_score"] = reply
        return out


def apply_filters(corpus: Corpus, filters: Sequence) -> Tuple[Corpus, Corpus]:
    """Runs every filter on every QA (consistent annotations), then returns (all, kept-only)."""
    for f in filters:
        corpus = f.apply(corpus)
    kept = corpus.copy()
    for p in kept.paragraphs():
        qas = []
        for qa in p.get("qas") or []:
            qa["is_keep"] = all(qa.get(f"{f.prefix}__keep", True) is not False for f in filters)
            if qa["is_keep"]:
                qas.append(qa)
        p["qas"] = qas
    return corpus, kept


# ------------------------------------------------------------------------------------------------ evaluation
K_VALUES = (1, 3, 5, 10, 100)


def ir_metrics(results: Dict[str, Dict[str, float]], qrels: Dict[str, Dict[str, int]],
               k_values: Sequence[int] = K_VALUES) -> Dict[str, Dict[str, float]]:
    """Mean over queries (trec_eval conventions, graded relevance allowed):
    NDCG@k = sum_{r<=k} rel_r / log2(r + 1) / IDCG@k;  MAP@k = sum_{r<=k, rel_r>0} P@r / |relevant|;
    Recall@k = |relevant in top k| / |relevant|;  P@k = |relevant in top k| / k."""
    agg = {m: {f"{m}@{k}": 0.0 for k in k_values} for m in ("NDCG", "MAP", "Recall", "P")}
    n = 0
    for qid, rel in qrels.items():
        relevant = {d: g for d, g in rel.items() if g > 0}
        if not relevant:
            continue
        n += 1
        ranked = sorted((results.get(qid) or {}).items(), key=lambda kv: (-kv[1], kv[0]))
        ideal = sorted(relevant.values(), reverse=True)
        for k in k_values:
            top = [d for d, _ in ranked[:k]]
            gains = [relevant.get(d, 0) for d in top]
            dcg = sum(g / math.log2(r + 2) for r, g in enumerate(gains))
            idcg = sum(g / math.log2(r + 2) for r, g in enumerate(ideal[:k]))
            hits, ap = 0, 0.0
            for r, g in enumerate(gains):
                if g > 0:
                    hits += 1
                    ap += hits / (r + 1)
            agg["NDCG"][f"NDCG@{k}"] += dcg / idcg if idcg > 0 else 0.0
            agg["MAP"][f"MAP@{k}"] += ap / len(relevant)
            agg["Recall"][f"Recall@{k}"] += hits / len(relevant)
            agg["P"][f"P@{k}"] += hits / k
    for m in agg.values():
        for key in m:
            m[key] = round(m[key] / max(n, 1), 5)
    return agg


def retrieve(embed: EmbedFn, corpus: Dict[str, dict], queries: Dict[str, str], top_k: int = 100,
             batch_size: int = 128, device=None) -> Dict[str, Dict[str, float]]:
    """Exact cosine top-k of every query over the corpus (GPU: the fused similarity top-k kernel of the
    HBM index; CPU: torch)."""
    import torch

    from .. import ops

    doc_ids = list(corpus)
    texts = [(corpus[d].get("title", "") + " " + corpus[d]["text"]).strip() for d in doc_ids]
    D = np.concatenate([np.asarray(embed(texts[s:s + batch_size], "passage"), np.float32)
                        for s in range(0, len(texts), batch_size)]) if texts else np.zeros((0, 1), np.float32)
    qids = list(queries)
    Q = np.concatenate([np.asarray(embed([queries[q] for q in qids[s:s + batch_size]], "query"), np.float32)
                        for s in range(0, len(qids), batch_size)]) if qids else np.zeros((0, D.shape[1]), np.float32)
    k = min(top_k, len(doc_ids))
    dev = torch.device(device) if device is not None else torch.device("cpu")
    Xt = torch.from_numpy(D).to(dev, torch.bfloat16 if dev.type == "cuda" else torch.float32)
    Qt = torch.from_numpy(Q).to(dev, Xt.dtype)
    if dev.type == "cuda" and k <= 64:
        scores, idx = ops.sim_topk(Qt, Xt, torch.zeros(len(doc_ids), device=dev), len(doc_ids), k)
    else:
        scores, idx = torch.topk(Qt.float() @ Xt.float().t(), k, dim=1)
    scores, idx = scores.cpu().numpy(), idx.cpu().numpy()
    return {q: {doc_ids[int(i)]: float(s) for s, i in zip(scores[r], idx[r]) if i >= 0} for r, q in enumerate(qids)}


def evaluate_beir(folder: str, embedders: Dict[str, EmbedFn], out_dir: str, top_k: int = 100,
                  device=None) -> Dict[str, Dict[str, Dict[str, float]]]:
    """Writes ``beir_evaluator__type_model_eval_dict.json``, ``beir_evaluator__recall5.csv`` and the
    per-query top-5 relevance flags; returns {model: metrics}."""
    corpus, queries, qrels = load_beir(folder)
    os.makedirs(out_dir, exist_ok=True)
    evals, flags = {}, {}
    for name, fn in embedders.items():
        res = retrieve(fn, corpus, queries, top_k=top_k, device=device)
        evals[name] = {k.lower(): v for k, v in ir_metrics(res, qrels).items()}
        flags[name] = {q: bool(set(sorted(res.get(q, {}), key=lambda d: -res[q][d])[:5]) & set(qrels[q]))
                       for q in qrels}
    with open(os.path.join(out_dir, "beir_evaluator__type_model_eval_dict.json"), "w") as f:
        json.dump({"synthetic": evals}, f, indent=2)
    with open(os.path.join(out_dir, "beir_evaluator__recall5.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["model_name", "synthetic"])
        for name, ev in evals.items():
            w.writerow([name, ev["recall"]["Recall@5"]])
    with open(os.path.join(out_dir, "beir_evaluator__synthetic_topk_rel_doc_flags.csv"), "w", newline="") as f:
        w = csv.writer(f)
        names = list(flags)
        w.writerow(["query_id"] + names)
        for q in qrels:
            w.writerow([q] + [flags[n][q] for n in names])
    return evals


# ------------------------------------------------------------------------------------------------ pipeline
def run_pipeline(corpus: Corpus, out_dir: str, generator: Optional[QAGenerator], filters: Sequence,
                 embedders: Dict[str, EmbedFn], input_format: str = "rawdoc", device=None) -> dict:
    """scripts/run_pipeline.py: generate -> filter -> SQuAD + BEIR outputs -> evaluate (all / filtered)."""
    if os.path.exists(out_dir) and os.listdir(out_dir):
        raise ValueError(f"output directory {out_dir} already exists")
    squad_dir = os.path.join(out_dir, "squad")
    os.makedirs(squad_dir, exist_ok=True)
    if generator is not None:
        corpus = generator.generate(corpus)
    c_all, c_kept = apply_filters(corpus, filters)
    c_all.to_json(os.path.join(squad_dir, "synthetic_data__all.json"))
    c_kept.to_json(os.path.join(squad_dir, "synthetic_data__filtered.json"))
    report = {}
    for name, c in (("all", c_all), ("filtered", c_kept)):
        beir_dir = os.path.join(out_dir, "beir", name)
        c.to_beir(beir_dir, create_original=input_format == "squad")
        report[name] = {"questions": c.num_questions(), "documents": sum(1 for _ in c.paragraphs())}
        if embedders and c.num_questions():
            report[name]["eval"] = evaluate_beir(os.path.join(beir_dir, "synthetic"), embedders,
                                                 os.path.join(out_dir, "eval", name), device=device)
    with open(os.path.join(out_dir, "report.json"), "w") as f:
        json.dump(report, f, indent=2)
    return report


def engine_embed_fn(embedder) -> EmbedFn:
    """Adapter from :class:`~..engine.embedder.Embedder` to ``EmbedFn``."""
    def fn(texts: List[str], input_type: str) -> np.ndarray:
        return embedder.embed(texts, input_type).float().cpu().numpy()
    return fn


def http_embed_fn(base_url: str, model: str, truncate: str = "END") -> EmbedFn:
    """``/v1/embeddings`` client (this framework's server or a NIM) with ``input_type``/``truncate``."""
    import httpx

    url = base_url.rstrip("/") + ("" if base_url.rstrip("/").endswith("/v1") else "/v1") + "/embeddings"
    cli = httpx.Client(timeout=600.0)

    def fn(texts: List[str], input_type: str) -> np.ndarray:
        r = cli.post(url, json={"input": texts, "model": model, "input_type": input_type, "truncate": truncate,
                                "encoding_format": "float"})
        r.raise_for_status()
        e = np.asarray([d["embedding"] for d in r.json()["data"]], np.float32)
        return e / np.maximum(np.linalg.norm(e, axis=1, keepdims=True), 1e-12)
    return fn


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--input-file", required=True)
    ap.add_argument("--input-format", choices=["squad", "rawdoc"], default="rawdoc")
    ap.add_argument("--output-dir", required=True)
    ap.add_argument("--max-examples", type=int, default=20)
    ap.add_argument("--num-questions", type=int, default=5)
    ap.add_argument("--llm-base-url", default="http://localhost:8000/v1", help="/v1 server for generation + judge")
    ap.add_argument("--llm-model", default="mistralai/mixtral-8x7b-instruct-v0.1")
    ap.add_argument("--judge-model", default="meta/llama3-70b-instruct")
    ap.add_argument("--embed-base-url", default=None, help="/v1/embeddings server (default: in-process embedder)")
    ap.add_argument("--embedder", default="e5-large-v2", help="in-process encoder preset (or HF dir via --weights)")
    ap.add_argument("--weights", default=None)
    ap.add_argument("--percentile", type=float, default=70.0)
    ap.add_argument("--no-generate", action="store_true", help="evaluate the questions already in the input")
    ap.add_argument("--no-answerability", action="store_true")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    from .llm import ChatFn

    corpus = Corpus.load(a.input_file, a.input_format)
    if a.embed_base_url:
        embed = http_embed_fn(a.embed_base_url, a.embedder)
        device = None
    else:
        import torch

        from ..engine.embedder import Embedder
        from ..models.registry import build_encoder
        device = "cuda" if torch.cuda.is_available() else "cpu"
        enc, tok, _ = build_encoder(a.embedder, a.weights, device=device)
        embed = engine_embed_fn(Embedder(enc, tok))
    gen = None if a.no_generate else QAGenerator(ChatFn(a.llm_base_url, a.llm_model, temperature=0.6, max_tokens=2048),
                                                a.num_questions, a.max_examples)
    filters = [EasinessFilter(embed, percentile=a.percentile)]
    if not a.no_answerability:
        filters.append(AnswerabilityFilter(ChatFn(a.llm_base_url, a.judge_model, temperature=0.5, max_tokens=1024)))
    rep = run_pipeline(corpus, a.output_dir, gen, filters, {a.embedder: embed}, a.input_format, device=device)
    print(json.dumps(rep, indent=2))


if __name__ == "__main__":
    main()
