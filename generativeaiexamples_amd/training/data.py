"""Instruction-tuning data: JSONL rows ``{"prompt", "response"}`` or Dolly-style
``{"instruction", "context", "response"}`` (the reference's Gemma SFT notebook uses databricks-dolly-15k;
the LoRA notebook PubMedQA). Each row becomes chat-templated prompt tokens + response tokens + EOS;
labels are -100 on the prompt. Rows are packed greedily into [micro_batch, seq_len] tensors."""
from __future__ import annotations

import json
import random
from typing import Iterator, List, Tuple

import torch

from ..engine.tokenizer import apply_chat_template
from ..rag import synthetic


def load_jsonl(path: str) -> List[dict]:
    with open(path, encoding="utf-8") as f:
        return [json.loads(line) for line in f if line.strip()]


def synthetic_rows(n: int, seed: int = 0) -> List[dict]:
    """Deterministic toy SFT set (question -> templated answer) for tests and benchmarks."""
    rows = []
    for i in range(n):
        q = synthetic.question(seed * 100000 + i)
        rows.append({"prompt": q, "response": f"Section {i % 97} reports that the answer is {i % 13}."})
    return rows


def encode(row: dict, tok, max_len: int) -> Tuple[List[int], List[int]]:
    if "prompt" in row:
        user = row["prompt"]
    else:
        user = row.get("instruction", "") + (("\n\nContext: " + row["context"]) if row.get("context") else "")
    p = apply_chat_template([{"role": "user", "content": user}], tok)
    r = tok.encode(row.get("response", row.get("output", ""))) + ([tok.eos_ids[0]] if tok.eos_ids else [])
    r = r[: max(1, max_len // 2)] if len(p) + len(r) > max_len else r
    if len(p) + len(r) > max_len:  # keep the response: drop the oldest prompt tokens
        p = p[len(p) + len(r) - max_len:]
    return p + r, [-100] * len(p) + r


def batches(rows: List[dict], tok, seq_len: int, micro_batch: int, seed: int = 0, pad_id: int = 0,
            epochs: int = 10 ** 9) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
    rng = random.Random(seed)
    enc = [encode(r, tok, seq_len) for r in rows]
    for _ in range(epochs):
        order = list(range(len(enc)))
        rng.shuffle(order)
        buf_i, buf_l = [], []
        for j in order:
            ids, lab = enc[j]
            buf_i.append(ids + [pad_id] * (seq_len - len(ids)))
            buf_l.append(lab + [-100] * (seq_len - len(lab)))
            if len(buf_i) == micro_batch:
                yield torch.tensor(buf_i), torch.tensor(buf_l)
                buf_i, buf_l = [], []
