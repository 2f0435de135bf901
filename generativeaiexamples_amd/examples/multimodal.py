"""advanced_rag/multimodal_rag (E6; reference chains.py:66-193 + vectorstore/custom_*_parser.py).

Ingest (rag/multimodal_ingest.py): PDF - text blocks (header / footer cropped, CID / ToUnicode fonts
decoded), ruled tables and embedded images; PPTX - slide text, speaker notes, tables and pictures;
standalone PNG / JPG images. Every image is described by the vision model served in-process
(Llama-3.2-Vision, asked to linearise charts - the reference's NeVA + DePlot path), with the text
around it; without a vision model it is a searchable placeholder. Chunks of 1000 characters / 100
overlap (vectorstore_updater.py:56-66). Query path as basic_rag with the "Relevant documents" framing.
"""
from __future__ import annotations

import logging
import os
import struct
from typing import Dict, Generator, List

from ..chain_server.utils import get_hub, get_llm
from ..index.hbm_index import Document
from ..rag import loaders, multimodal_ingest
from ..rag.text_splitter import RecursiveCharacterTextSplitter
from .basic_rag import NO_CONTEXT, BasicRAG

log = logging.getLogger(__name__)
IMAGE_EXT = {".png", ".jpg", ".jpeg"}
# extracted page images / slide pictures (the reference keeps them under /tmp-data/vectorstore/*_references)
IMAGE_DIR = os.environ.get("APP_VECTORSTORE_IMAGEDIR", os.path.join(os.environ.get("TMPDIR", "/tmp"),
                                                                    "gai_vectorstore_images"))
DESCRIBE_PROMPT = ("Describe this image in detail. If it is a chart, graph or plot, say so, then list the "
                   "data it shows as a table (one row per data point).")


def vlm_describer(hub):
    """describe(path, context) on the hub's generator when it accepts images (Llama-3.2-Vision), else None."""
    llm = hub.llm() if hub is not None else None
    if llm is None or not hasattr(llm.engine.model, "register_request"):
        return None
    import base64

    from ..engine import SamplingParams
    from ..engine.tokenizer import apply_chat_template, image_token_of

    def describe(path: str, context: str) -> str:
        with open(path, "rb") as f:
            uri = "data:image;base64," + base64.b64encode(f.read()).decode()
        ask = DESCRIBE_PROMPT + (f" Text around the image: {context}" if context else "")
        ids = apply_chat_template([{"role": "user", "content": [{"type": "image"}, {"type": "text", "text": ask}]}],
                                  llm.tokenizer, image_token_id=image_token_of(llm.engine.model))
        out = llm.generate_sync(ids, SamplingParams(temperature=0.0, max_tokens=256), images=[uri])
        return "".join(it.delta for it in out).strip()

    return describe


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
        d = vlm_describer(get_hub())
        if d is not None:
            try:
                return d(path, "")
            except Exception as e:  # fall back to metadata
                log.warning("captioning failed for %s: %s", filename, e)
        with open(path, "rb") as f:
            sz = image_size(f.read(1 << 16))
        return f"Image {filename}" + (f" ({sz[0]}x{sz[1]} pixels)" if sz else "")

    def ingest_docs(self, filepath: str, filename: str) -> None:
        ext = os.path.splitext(filename)[1].lower()
        if ext in IMAGE_EXT:
            docs = [Document(self.describe_image(filepath, filename), {"filename": filename, "type": "image"})]
        elif ext in (".pdf", ".pptx"):
            with open(filepath, "rb") as f:
                data = f.read()
            fn = multimodal_ingest.pdf_documents if ext == ".pdf" else multimodal_ingest.pptx_documents
            docs = fn(data, filename, describe=vlm_describer(get_hub()), image_dir=IMAGE_DIR)
            if not docs:
                docs = loaders.load(filepath, filename)
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
