"""Plugin contract of the example pipelines (parity with RAG/src/chain_server/base.py:22-68).

An example implements ``ingest_docs``, ``llm_chain`` and ``rag_chain``; ``document_search``,
``get_documents`` and ``delete_documents`` are optional (the /search and /documents routes report
an error when absent). ``llm_chain`` / ``rag_chain`` return an iterator of text chunks that the
server streams as SSE frames.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Dict, Generator, List


class BaseExample(ABC):
    @abstractmethod
    def llm_chain(self, query: str, chat_history: List[Dict[str, str]], **kwargs) -> Generator[str, None, None]:
        ...

    @abstractmethod
    def rag_chain(self, query: str, chat_history: List[Dict[str, str]], **kwargs) -> Generator[str, None, None]:
        ...

    @abstractmethod
    def ingest_docs(self, data_dir: str, filename: str) -> None:
        ...

    def document_search(self, content: str, num_docs: int) -> List[Dict[str, Any]]:
        raise NotImplementedError

    def get_documents(self) -> List[str]:
        raise NotImplementedError

    def delete_documents(self, filenames: List[str]) -> bool:
        raise NotImplementedError
