"""Synthetic QA-pair generation (T1; reference synthetic_data_generator/data_generator.py: 3000/100 chunks,
two QA pairs per chunk from an instruction-tuned LLM, regex parse of the JSON-ish reply)."""
from __future__ import annotations

import json
import logging
import os
import re
from typing import List

from ..rag.loaders import load
from ..rag.text_splitter import RecursiveCharacterTextSplitter
from .llm import LLMFn

log = logging.getLogger(__name__)

SYS_PROMPT = ("Given the context paragraph, create two very good question answer pairs. Your output should be "
              "strictly in a json format of individual question answer pairs with keys from [\"question\",\"answer\"]. "
              "Restrict the question to the context information provided.")

_Q = re.compile(r'"question"\s*:\s*"((?:[^"\\]|\\.)*)"', re.S)
_A = re.compile(r'"answer"\s*:\s*"((?:[^"\\]|\\.)*)"', re.S)


def parse_pairs(reply: str) -> List[dict]:
    """Extract (question, answer) pairs from a model reply: strict JSON first, then the regex fallback."""
    try:
        obj = json.loads(reply)
        items = obj if isinstance(obj, list) else obj.get("pairs", [obj]) if isinstance(obj, dict) else []
        pairs = [{"question": str(i["question"]), "answer": str(i["answer"])} for i in items
                 if isinstance(i, dict) and "question" in i and "answer" in i]
        if pairs:
            return pairs
    except (ValueError, AttributeError, TypeError):
        pass
    qs, ans = _Q.findall(reply), _A.findall(reply)
    return [{"question": json.loads(f'"{q}"'), "answer": json.loads(f'"{a}"')} for q, a in zip(qs, ans)]


def generate_synthetic_data(dataset_folder: str, out_file: str, llm: LLMFn, chunk_size: int = 3000,
                            chunk_overlap: int = 100, max_chunks: int | None = None) -> List[dict]:
    splitter = RecursiveCharacterTextSplitter(chunk_size=chunk_size, chunk_overlap=chunk_overlap)
    out: List[dict] = []
    n = 0
    for fn in sorted(os.listdir(dataset_folder)):
        path = os.path.join(dataset_folder, fn)
        if not os.path.isfile(path):
            continue
        try:
            docs = load(path, fn)
        except ValueError as e:
            log.warning("skip %s: %s", fn, e)
            continue
        for chunk in splitter.split_documents(docs):
            if max_chunks is not None and n >= max_chunks:
                break
            n += 1
            reply = llm([{"role": "system", "content": SYS_PROMPT},
                         {"role": "user", "content": f"[The Start of the Reference Context]{chunk.page_content}"
                                                     f"[The End of Reference Context]"}])
            for p in parse_pairs(reply):
                out.append({"question": p["question"], "gt_answer": p["answer"], "gt_context": chunk.page_content,
                            "document": fn})
    with open(out_file, "w", encoding="utf-8") as f:
        json.dump(out, f, indent=2)
    log.info("wrote %d QA pairs from %d chunks to %s", len(out), n, out_file)
    return out
