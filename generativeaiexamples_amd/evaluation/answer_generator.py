"""Fill RAG answers for a QA set through a running chain server (T2; reference
rag_evaluator/llm_answer_generator.py: upload docs, stream /generate with the knowledge base at
temperature 0.2 / top_p 0.7 / max_tokens 256, and /search top_k=1 for the retrieved contexts)."""
from __future__ import annotations

import json
import logging
import os
from typing import List, Optional

from ..playground.chat_client import ChatClient

log = logging.getLogger(__name__)


def generate_answers(base_url: str, dataset_folder: Optional[str], qa_file: str, out_file: str,
                     client: Optional[ChatClient] = None, temperature: float = 0.2, top_p: float = 0.7,
                     max_tokens: int = 256, num_docs: int = 1) -> List[dict]:
    cc = client or ChatClient(base_url)
    if dataset_folder:
        files = [os.path.join(dataset_folder, f) for f in sorted(os.listdir(dataset_folder))
                 if os.path.isfile(os.path.join(dataset_folder, f))]
        cc.upload_documents(files)
    with open(qa_file, encoding="utf-8") as f:
        data = json.load(f)
    out = []
    for i, d in enumerate(data):
        q = d["question"]
        answer = "".join(cc.predict(q, True, max_tokens, temperature=temperature, top_p=top_p))
        ctx = [c["content"] for c in cc.search(q, num_docs)]
        out.append({"question": q, "gt_answer": d.get("gt_answer", d.get("ground_truth_answer", "")),
                    "gt_context": d.get("gt_context", d.get("ground_truth_context", "")), "answer": answer,
                    "contexts": ctx})
        if (i + 1) % 10 == 0:
            log.info("answers: %d/%d", i + 1, len(data))
    with open(out_file, "w", encoding="utf-8") as f:
        json.dump(out, f, indent=2)
    return out
