"""Document loaders with no third-party parsers (unstructured / pdfplumber / LibreOffice are not
available offline): plain text, Markdown, HTML, CSV, JSON, PDF (text operators of Flate-compressed
or raw content streams), DOCX and PPTX (Office Open XML, incl. slide notes).

Replaces ``UnstructuredFileLoader`` (basic_rag/langchain/chains.py:54-88), the LlamaIndex
PDFReader / UnstructuredReader (basic_rag/llamaindex/chains.py:59-108) and the multimodal
PDF / PPTX text paths (multimodal_rag/vectorstore/custom_pdf_parser.py,
custom_powerpoint_parser.py).
"""
from __future__ import annotations

import csv
import html
import io
import json
import os
import re
import zipfile
import zlib
from typing import List

from ..index.hbm_index import Document

SUPPORTED = {".txt", ".md", ".pdf", ".html", ".htm", ".csv", ".json", ".docx", ".pptx", ".xml", ".rst", ".py"}


def load(path: str, filename: str | None = None) -> List[Document]:
    filename = filename or os.path.basename(path)
    ext = os.path.splitext(filename)[1].lower()
    meta = {"source": path, "filename": filename}
    with open(path, "rb") as f:
        data = f.read()
    if ext in (".pdf", ".pptx"):
        # structured parse (rag/pdf.py: ToUnicode / CID fonts, ruled tables, layout); images need a vision
        # model and are handled by the multimodal example
        from .multimodal_ingest import pdf_documents, pptx_documents

        try:
            docs = (pdf_documents if ext == ".pdf" else pptx_documents)(data, filename)
        except Exception:  # a file the structured parser cannot read: fall back to the stream scan
            docs = []
        docs = [Document(d.page_content, dict(meta, **{k: v for k, v in d.metadata.items() if k != "source"}))
                for d in docs if d.metadata.get("type") != "image" and d.page_content.strip()]
        if docs:
            return docs
        pages = pdf_pages(data) if ext == ".pdf" else pptx_slides(data)
        return [Document(t, dict(meta, page=i + 1)) for i, t in enumerate(pages) if t.strip()]
    if ext == ".docx":
        return [Document(docx_text(data), meta)]
    if ext in (".html", ".htm", ".xml"):
        return [Document(html_text(data.decode("utf-8", "replace")), meta)]
    if ext == ".csv":
        rows = list(csv.reader(io.StringIO(data.decode("utf-8", "replace"))))
        if not rows:
            return []
        head = rows[0]
        text = "\n".join(", ".join(f"{h}: {v}" for h, v in zip(head, r)) for r in rows[1:])
        return [Document(text, meta)]
    if ext == ".json":
        try:
            return [Document(json.dumps(json.loads(data), indent=1), meta)]
        except json.JSONDecodeError:
            pass
    return [Document(data.decode("utf-8", "replace"), meta)]


# ------------------------------------------------------------------------------------------- PDF
_STREAM = re.compile(rb"<<(.*?)>>\s*stream\r?\n(.*?)\r?\nendstream", re.S)
_TEXT_OP = re.compile(rb"\[(.*?)\]\s*TJ|\((.*?)(?<!\\)\)\s*Tj|\((.*?)(?<!\\)\)\s*'|(T\*|Td|TD|Tm|ET)", re.S)
_STR_IN_ARRAY = re.compile(rb"\((.*?)(?<!\\)\)", re.S)


def _pdf_unescape(b: bytes) -> str:
    out = bytearray()
    i = 0
    while i < len(b):
        c = b[i]
        if c == 0x5C and i + 1 < len(b):  # backslash
            n = b[i + 1]
            m = {ord("n"): 10, ord("r"): 13, ord("t"): 9, ord("b"): 8, ord("f"): 12}
            if n in m:
                out.append(m[n])
                i += 2
            elif 48 <= n <= 55:
                j = i + 1
                oct_digits = b""
                while j < len(b) and len(oct_digits) < 3 and 48 <= b[j] <= 55:
                    oct_digits += bytes([b[j]])
                    j += 1
                out.append(int(oct_digits, 8) & 255)
                i = j
            else:
                out.append(n)
                i += 2
        else:
            out.append(c)
            i += 1
    return out.decode("latin-1")


def _content_text(stream: bytes) -> str:
    parts: List[str] = []
    for m in _TEXT_OP.finditer(stream):
        if m.group(1) is not None:
            parts.append("".join(_pdf_unescape(s) for s in _STR_IN_ARRAY.findall(m.group(1))))
        elif m.group(2) is not None:
            parts.append(_pdf_unescape(m.group(2)))
        elif m.group(3) is not None:
            parts.append("\n" + _pdf_unescape(m.group(3)))
        elif m.group(4) in (b"T*", b"Td", b"TD", b"ET"):
            parts.append("\n")
        else:
            parts.append(" ")
    txt = "".join(parts)
    return re.sub(r"[ \t]+", " ", re.sub(r"\n\s*\n+", "\n", txt)).strip()


def pdf_pages(data: bytes) -> List[str]:
    """Best-effort text per content stream (page order as stored)."""
    pages = []
    for m in _STREAM.finditer(data):
        dic, body = m.group(1), m.group(2)
        if b"/Subtype/Image" in dic.replace(b" ", b"") or b"/XObject" in dic and b"/Image" in dic:
            continue
        if b"/FlateDecode" in dic:
            try:
                body = zlib.decompress(body)
            except zlib.error:
                try:
                    body = zlib.decompressobj().decompress(body)
                except zlib.error:
                    continue
        elif b"/Filter" in dic:
            continue  # other filters (DCT, LZW, ...) carry no extractable text here
        if b"Tj" in body or b"TJ" in body:
            t = _content_text(body)
            if t:
                pages.append(t)
    return pages


# ------------------------------------------------------------------------------------------- OOXML
_XML_TEXT = re.compile(r"<a:t>(.*?)</a:t>|<w:t(?: [^>]*)?>(.*?)</w:t>|<w:p[ >]|<a:p>", re.S)


def _xml_text(x: str) -> str:
    out = []
    for m in _XML_TEXT.finditer(x):
        if m.group(1) is not None:
            out.append(html.unescape(m.group(1)))
        elif m.group(2) is not None:
            out.append(html.unescape(m.group(2)))
        else:
            out.append("\n")
    return re.sub(r"\n+", "\n", "".join(out)).strip()


def pptx_slides(data: bytes) -> List[str]:
    z = zipfile.ZipFile(io.BytesIO(data))
    names = sorted((n for n in z.namelist() if re.match(r"ppt/slides/slide\d+\.xml$", n)),
                   key=lambda n: int(re.findall(r"\d+", n)[-1]))
    out = []
    for n in names:
        t = _xml_text(z.read(n).decode("utf-8", "replace"))
        note = n.replace("slides/slide", "notesSlides/notesSlide")
        if note in z.namelist():
            nt = _xml_text(z.read(note).decode("utf-8", "replace"))
            if nt:
                t += "\nNotes: " + nt
        out.append(t)
    return out


def docx_text(data: bytes) -> str:
    z = zipfile.ZipFile(io.BytesIO(data))
    return _xml_text(z.read("word/document.xml").decode("utf-8", "replace"))


def html_text(s: str) -> str:
    s = re.sub(r"(?is)<(script|style).*?</\1>", " ", s)
    s = re.sub(r"(?i)<br\s*/?>|</p>|</div>|</li>|</h\d>", "\n", s)
    s = re.sub(r"<[^>]+>", " ", s)
    return re.sub(r"[ \t]+", " ", html.unescape(s)).strip()


def make_pdf(pages: List[str]) -> bytes:
    """Minimal valid PDF writer (tests / synthetic corpora)."""
    objs = []
    kids = []
    for i, text in enumerate(pages):
        lines = text.split("\n")
        ops = "BT /F1 12 Tf 72 720 Td " + " T* ".join(
            "(" + ln.replace("\\", "\\\\").replace("(", "\\(").replace(")", "\\)") + ") Tj" for ln in lines) + " ET"
        stream = zlib.compress(ops.encode("latin-1", "replace"))
        objs.append(("stream", stream))
        kids.append(i)
    out = io.BytesIO()
    out.write(b"%PDF-1.4\n")
    offsets = []
    n_pages = len(pages)
    # 1: catalog, 2: pages, 3: font, then per page: page obj + content obj
    def obj(num, body: bytes):
        offsets.append((num, out.tell()))
        out.write(f"{num} 0 obj\n".encode() + body + b"\nendobj\n")

    obj(1, b"<< /Type /Catalog /Pages 2 0 R >>")
    kid_refs = " ".join(f"{4 + 2 * i} 0 R" for i in range(n_pages))
    obj(2, f"<< /Type /Pages /Kids [{kid_refs}] /Count {n_pages} >>".encode())
    obj(3, b"<< /Type /Font /Subtype /Type1 /BaseFont /Helvetica >>")
    for i, (_, stream) in enumerate(objs):
        obj(4 + 2 * i, f"<< /Type /Page /Parent 2 0 R /Resources << /Font << /F1 3 0 R >> >> "
                       f"/MediaBox [0 0 612 792] /Contents {5 + 2 * i} 0 R >>".encode())
        obj(5 + 2 * i, f"<< /Length {len(stream)} /Filter /FlateDecode >>\nstream\n".encode() + stream + b"\nendstream")
    xref = out.tell()
    offsets.sort()
    out.write(f"xref\n0 {len(offsets) + 1}\n0000000000 65535 f \n".encode())
    for _, off in offsets:
        out.write(f"{off:010d} 00000 n \n".encode())
    out.write(f"trailer << /Size {len(offsets) + 1} /Root 1 0 R >>\nstartxref\n{xref}\n%%EOF\n".encode())
    return out.getvalue()
