"""advanced_rag/multimodal_rag (E6; reference chains.py:66-193 + vectorstore/custom_*_parser.py).

Ingest: PDF (text per page), PPTX (slide text + speaker notes), images (PNG/JPG: caption from the
vision model served in-process when one is configured, else an image placeholder with its
filename and size), plus everything basic_rag accepts; chunks of 1000 characters / 100 overlap
(vectorstore_updater.py:56-66). Query path as basic_rag with the "Relevant documents" framing.
"""
from __future__ import annotations

import logging
import os
import struct
from typing import Dict, Generator, List

from ..chain_server.utils import get_hub, get_llm
from ..index.hbm_index import Document
from ..rag import loaders
from ..rag.text_splitter import RecursiveCharacterTextSplitter
from .basic_rag import NO_CONTEXT, BasicRAG

log = logging.getLogger(__name__)
IMAGE_EXT = {".png", ".jpg", ".jpeg"}


def image_size(data: bytes):
    if data[:8] == b"\x89PNG\r\n\x1a\n":
        w, h = struct.unpack(">II", data[16:24])
        return w, h
    if data[:2] == b"\xff\xd8":
        i = 2
        while i < len(data) - 9:
            if data[i] != 0xFF:
                i += 1
                continue
            marker = data[i + 1]
            if marker in (0xC0, 0xC1, 0xC2):
                h, w = struct.unpack(">HH", data[i + 5:i + 9])
                return w, h
            seg = struct.unpack(">H", data[i + 2:i + 4])[0]
            i += 2 + seg
    return None


class MultimodalRAG(BasicRAG):
    def __init__(self):
        super().__init__()
        self.char_splitter = RecursiveCharacterTextSplitter(1000, 100)

    def describe_image(self, path: str, filename: str) -> str:
        hub = get_hub()
        vlm = getattr(hub, "vlm", None)
        if vlm is not None:
            try:
                return vlm.caption(path)
            except Exception as e:  # fall back to metadata
                log.warning("captioning failed for %s: %s", filename, e)
        with open(path, "rb") as f:
            sz = image_size(f.read(1 << 16))
        return f"Image {filename}" + (f" ({sz[0]}x{sz[1]} pixels)" if sz else "")

    def ingest_docs(self, filepath: str, filename: str) -> None:
        ext = os.path.splitext(filename)[1].lower()
        if ext in IMAGE_EXT:
            docs = [Document(self.describe_image(filepath, filename), {"filename": filename, "type": "image"})]
        elif ext in loaders.SUPPORTED:
            docs = loaders.load(filepath, filename)
        else:
            raise ValueError(f"{filename}: unsupported file type")
        chunks = self.char_splitter.split_documents(docs)
        if not chunks:
            raise ValueError(f"no content extracted from {filename}")
        self.store.add_documents(chunks)

    def rag_chain(self, query: str, chat_history: List[Dict[str, str]], **kwargs) -> Generator[str, None, None]:
        hits = self.retrieve(query)
        if not hits:
            return iter([NO_CONTEXT])
        docs = "\n\n".join(d.page_content for d, _ in hits)
        msgs = [{"role": "system", "content": self.prompts["rag_template"]},
                {"role": "user", "content": f"Relevant documents:\n{docs}\n\n[[QUESTION]]\n{query}"}]
        return get_llm(**kwargs).stream(msgs)
