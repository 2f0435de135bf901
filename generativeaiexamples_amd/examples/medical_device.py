"""industries/healthcare/medical-device-training-assistant (E7; reference
industries/healthcare/medical-device-training-assistant/app_chain/chains.py:61-369, a MultiTurnChatbot
fork for instructions-for-use (IFU) manuals of medical devices).

Behaviour: multi-turn RAG over the ingested device manuals with per-conversation memory; with a
ranker, 40 document candidates and 40 memory candidates are each reranked to top_k; the answer is
grounded in the retrieved manual excerpts with the "document chatbot" prompt (``app_chain_template``:
``{input}``, ``{history}``, ``{context}``) and every answer lists the manual sections it used, which
is what a training assistant for clinical staff needs to verify a procedure against the IFU.
``parse_gt_qa_txt`` reads the example's ground-truth file format ("Example n: / Question: / Answer:")
for the evaluation tool.
"""
from __future__ import annotations

import re
from typing import Dict, Generator, List, Optional

from ..chain_server.utils import get_llm
from ..index.hbm_index import Document
from .basic_rag import NO_CONTEXT
from .multi_turn import MultiTurnRAG, conversation_key

DEFAULT_TEMPLATE = (
    "You are a training assistant for clinical staff learning to use medical devices. Help the user as they ask "
    "questions about the device's instructions for use.\nUser message just asked: {input}\n\n"
    "For this, we have retrieved the following potentially-useful info:\nConversation History Retrieved:\n{history}\n\n"
    "Document Retrieved:\n{context}\n\nAnswer only from retrieved data; if the manual does not cover the question, "
    "say so and advise consulting the manufacturer. Make your response conversational.")


class MedicalDeviceAssistant(MultiTurnRAG):
    def rag_chain(self, query: str, chat_history: List[Dict[str, str]], session_id: Optional[str] = None,
                  **kwargs) -> Generator[str, None, None]:
        conv_id = conversation_key(chat_history, query, session_id)
        docs = self._fetch(self.store, query)
        memory = self._fetch(self.conv_store, query, conv_id) if len(self.conv_store) else []
        if not docs and not memory:
            yield NO_CONTEXT
            return
        template = self.prompts.get("app_chain_template") or DEFAULT_TEMPLATE
        context = "\n\n".join(f"[{d.metadata.get('filename', 'manual')} p.{d.metadata.get('page', '?')}] {d.page_content}"
                              for d in docs)
        prompt = template.format(input=query, history="\n".join(d.page_content for d in memory), context=context)
        msgs = [{"role": "system", "content": self.prompts.get("chat_template", "")},
                {"role": "user", "content": prompt}]
        answer = []
        for chunk in get_llm(**kwargs).stream(msgs):
            answer.append(chunk)
            yield chunk
        sources = sorted({d.metadata.get("filename", "") for d in docs if d.metadata.get("filename")})
        if sources:
            tail = "\n\nSources: " + ", ".join(sources)
            answer.append(tail)
            yield tail
        turn = f"User: {query}\nAssistant: {''.join(answer)}"
        self.conv_store.add_documents([Document(turn, {"conversation": conv_id, "filename": f"conversation-{conv_id}"})])


_EX = re.compile(r"^\s*Example\s+\d+\s*:\s*$", re.M | re.I)


def parse_gt_qa_txt(text: str) -> List[Dict[str, str]]:
    """'Example n:' blocks with 'Question:' and a multi-line 'Answer:' -> [{question, gt_answer}]."""
    out = []
    for block in _EX.split(text):
        q = re.search(r"Question\s*:\s*(.+)", block)
        a = re.search(r"Answer\s*:\s*(.*)", block, re.S)
        if q and a:
            out.append({"question": q.group(1).strip(), "gt_answer": a.group(1).strip()})
    return out
