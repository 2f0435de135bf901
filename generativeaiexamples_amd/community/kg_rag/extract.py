"""Document -> knowledge-graph ingestion (reference: /root/reference/community/knowledge_graph_rag/backend/utils/
preprocessor.py:31-129 - the triple-extraction prompt, ``ast.literal_eval`` of a Python list of 5-tuples, the QA-pair
generator and the LLM-as-judge prompt; utils/lc_graph.py:27-112 - directory load, recursive split (chunk 500 /
overlap 100), a thread pool of extraction calls with a progress callback).

The model is asked for a Python-literal list of ``(head, head_type, relation, tail, tail_type)`` tuples with typed,
disambiguated entities and a closed relation vocabulary. ``parse_triples`` accepts what models actually return: the
list in a fenced block or after prose, JSON arrays, lists instead of tuples, dict rows, and drops rows with a missing /
NaN / single-letter entity. Relations outside the vocabulary are kept but normalised to ``Title_Case`` (``strict``
rejects them instead). The LLM is anything with ``invoke(messages, **kw) -> str`` (the framework's chain-server LLM).
"""
from __future__ import annotations

import ast
import json
import logging
import os
import re
from concurrent.futures import ThreadPoolExecutor, as_completed
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from ...index.hbm_index import Document
from ...rag.text_splitter import RecursiveCharacterTextSplitter
from .graph import KnowledgeGraph

log = logging.getLogger(__name__)

ENTITY_TYPES = {
    "ORG": "a company or organisation that is neither a government nor a regulator",
    "ORG/GOV": "a government body",
    "ORG/REG": "a regulatory body",
    "PERSON": "a named individual",
    "GPE": "a country, state, city or other geopolitical entity",
    "INSTITUTION": "a university, lab or research institute",
    "PRODUCT": "a product, service or technology",
    "EVENT": "a specific, material event",
    "FIELD": "an academic field or discipline",
    "METRIC": "a named measure or indicator (not a bare number)",
    "TOOL": "a research tool or method",
    "CONCEPT": "an abstract idea or theme",
}
RELATIONS = ("Has", "Announce", "Operate_In", "Introduce", "Produce", "Control", "Participates_In", "Impact",
             "Positive_Impact_On", "Negative_Impact_On", "Relate_To", "Is_Member_Of", "Invests_In", "Raise",
             "Decrease")

TRIPLE_PROMPT = (
    "You build a knowledge graph from text. List the factual relationships the text states as a Python list of "
    "5-tuples (head, head_type, relation, tail, tail_type), all strings, and output nothing but that list.\n"
    "Entity types:\n" + "\n".join(f"  {k}: {v}" for k, v in ENTITY_TYPES.items()) + "\n"
    "Relations (use exactly one of): " + ", ".join(RELATIONS) + ".\n"
    "Rules: entities are specific names of at most four words - never dates, numbers, percentages, pronouns or "
    "generic nouns; merge aliases and acronyms of one entity under one name; omit a relationship rather than leave an "
    "element empty or NaN.\n"
    "Example - text: 'Contoso Labs released the Falcon sensor in Norway; regulators at the Norwegian Energy Agency "
    "expect it to cut grid losses.'\n"
    "Output: [('Contoso Labs', 'ORG', 'Introduce', 'Falcon sensor', 'PRODUCT'), "
    "('Contoso Labs', 'ORG', 'Operate_In', 'Norway', 'GPE'), "
    "('Falcon sensor', 'PRODUCT', 'Positive_Impact_On', 'Grid Losses', 'METRIC')]")

QA_PROMPT = (
    "Write one hard question about the passage that needs most of it and several reasoning steps to answer, and a "
    "thorough answer drawn only from the passage. Reply with JSON only: {\"question\": \"...\", \"answer\": \"...\"}.")

JUDGE_PROMPT = (
    "Rate how well the answer addresses the question on a 1-4 scale: 1 irrelevant or very partial, 2 misses key "
    "aspects, 3 mostly helpful, 4 relevant, direct, detailed and complete. Reply in the form\n"
    "Evaluation: <your reasoning>\nTotal rating: <1-4>")

_BAD = {"", "nan", "none", "null", "n/a", "unknown"}


def _norm_relation(r: str) -> str:
    r = re.sub(r"[\s\-]+", "_", str(r).strip())
    for v in RELATIONS:
        if v.lower() == r.lower():
            return v
    return "_".join(p[:1].upper() + p[1:] for p in r.split("_") if p)


def _literal(text: str):
    for parse in (ast.literal_eval, json.loads):
        try:
            return parse(text)
        except (ValueError, SyntaxError, TypeError, MemoryError, RecursionError):
            continue
    return None


def parse_triples(text: str, strict: bool = False) -> List[Dict[str, str]]:
    """Model reply -> [{subject, subject_type, relation, object, object_type}] (never raises)."""
    if not isinstance(text, str):
        return []
    body = text
    m = re.search(r"```(?:python|json)?\s*(.*?)```", body, re.S)
    if m:
        body = m.group(1)
    start, end = body.find("["), body.rfind("]")
    rows = _literal(body[start:end + 1]) if 0 <= start < end else None
    if rows is None:  # one tuple per line, or a list cut off mid-way: take every complete (...) group
        rows = [r for r in (_literal(g) for g in re.findall(r"\((?:[^()'\"]|'[^']*'|\"[^\"]*\")*\)", body))
                if r is not None]
    out = []
    for r in rows if isinstance(rows, (list, tuple)) else []:
        if isinstance(r, dict):
            r = (r.get("subject", r.get("h")), r.get("subject_type"), r.get("relation", r.get("r")),
                 r.get("object", r.get("o")), r.get("object_type"))
        if not isinstance(r, (list, tuple)) or len(r) != 5:
            continue
        s, st, rel, o, ot = (str(x).strip() if x is not None else "" for x in r)
        if s.lower() in _BAD or o.lower() in _BAD or len(s) < 2 or len(o) < 2 or not rel:
            continue
        rel_n = _norm_relation(rel)
        if strict and rel_n not in RELATIONS:
            continue
        out.append({"subject": s, "subject_type": st or "Unknown", "relation": rel_n, "object": o,
                    "object_type": ot or "Unknown"})
    return out


def _ask(llm, system: str, user: str, **kw) -> str:
    r = llm.invoke([{"role": "system", "content": system}, {"role": "user", "content": user}], **kw)
    return getattr(r, "content", r)


def extract_triples(text: str, llm, strict: bool = False) -> List[Dict[str, str]]:
    return parse_triples(_ask(llm, TRIPLE_PROMPT, text, temperature=0.0, max_tokens=1024), strict=strict)


def load_directory(directory: str) -> List[Document]:
    """Every loadable file under ``directory`` (the framework's PDF / DOCX / PPTX / HTML / text loaders)."""
    from ...rag.loaders import load

    docs = []
    for root, _, files in os.walk(directory):
        for f in sorted(files):
            try:
                docs += load(os.path.join(root, f), f)
            except Exception as e:  # noqa: BLE001 - one unreadable file does not stop the ingest
                log.warning("skipping %s: %s", f, e)
    return docs


def process_documents(source, llm, graph: Optional[KnowledgeGraph] = None, chunk_size: int = 500,
                      chunk_overlap: int = 100, max_workers: int = 8, triplets: bool = True,
                      update_progress: Optional[Callable[[int, int], None]] = None
                      ) -> Tuple[List[Document], KnowledgeGraph]:
    """Split ``source`` (a directory, or a list of Documents / strings) and extract triples from every chunk
    concurrently into ``graph``. Returns (chunks, graph); each chunk's triples are also kept in its metadata."""
    if isinstance(source, str):
        docs = load_directory(source)
    else:
        docs = [d if isinstance(d, Document) else Document(str(d), {}) for d in source]
    chunks = RecursiveCharacterTextSplitter(chunk_size, chunk_overlap).split_documents(docs)
    graph = graph if graph is not None else KnowledgeGraph()
    if not triplets or not chunks:
        return chunks, graph
    done = 0
    with ThreadPoolExecutor(max_workers=max(1, max_workers)) as ex:
        futs = {ex.submit(extract_triples, c.page_content, llm): c for c in chunks}
        for f in as_completed(futs):
            try:
                tr = f.result()
            except Exception as e:  # noqa: BLE001 - a failed call loses that chunk's triples only
                log.warning("triple extraction failed: %s", e)
                tr = []
            futs[f].metadata["triples"] = tr
            graph.add_triples(tr)
            done += 1
            if update_progress is not None:
                update_progress(done, len(chunks))
    return chunks, graph


def generate_qa_pair(text: str, llm) -> Optional[Dict[str, str]]:
    from ..fm_asr.chains import first_json_object

    reply = _ask(llm, QA_PROMPT, text, temperature=0.2, max_tokens=512)
    try:
        obj = json.loads(reply)
    except (ValueError, TypeError):
        obj = first_json_object(reply or "")
    if not isinstance(obj, dict) or not obj.get("question") or not obj.get("answer"):
        return None
    return {"question": str(obj["question"]), "answer": str(obj["answer"])}


def parse_judgement(reply: str) -> Dict[str, object]:
    ev = re.search(r"Evaluation:(.*?)Total rating:", reply or "", re.S)
    sc = re.search(r"Total rating:\s*(\d+(?:\.\d+)?)", reply or "")
    return {"llm_judge_evaluation": ev.group(1).strip() if ev else "no match found",
            "llm_judge_score": float(sc.group(1)) if sc else 0.0}


def judge_answer(question: str, answer: str, llm) -> Dict[str, object]:
    return parse_judgement(_ask(llm, JUDGE_PROMPT, f"Question: {question}\nAnswer: {answer}", temperature=0.2,
                                max_tokens=300))


def sample_documents(docs: Sequence[Document], n: int, seed: int = 0) -> List[Document]:
    import random

    return random.Random(seed).sample(list(docs), min(n, len(docs)))
