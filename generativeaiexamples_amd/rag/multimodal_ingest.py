"""Multimodal document ingest: PDF / PPTX -> text, table and image documents.

Mirrors the reference's multimodal vector-store updater (RAG/examples/advanced_rag/multimodal_rag/
vectorstore/custom_pdf_parser.py get_pdf_documents:312-370, custom_powerpoint_parser.py:26-122,
custom_img_parser.py:35-60) on the in-process stack:

* PDF (rag/pdf.py): header / footer bands dropped, text grouped into heading + paragraph blocks, ruled
  tables extracted cell by cell ("This is a table with the following rows: ..."), embedded images written
  out and described by the served vision model (Llama-3.2-Vision) - asked whether the image is a chart and,
  if so, to linearise its data (the reference's NeVA is-graph check + DePlot + summarisation) - with the
  text right above / below the image as context (extract_text_around_item);
* PPTX: per slide the title, body text, speaker notes, tables (a:tbl) and pictures (ppt/media via the
  slide relationships), each picture described the same way.

``describe(path, context) -> str`` is injected (examples/multimodal.py binds it to the hub's VLM); without
one, images become placeholders carrying their size and surrounding text, so they stay searchable.
"""
from __future__ import annotations

import html
import io
import os
import re
import zipfile
from typing import Callable, List, Optional

from ..index.hbm_index import Document
from . import pdf as pdfmod

Describe = Callable[[str, str], str]


def stringify_table(rows: List[List[str]]) -> str:
    return "\n".join(" | ".join(c for c in r) for r in rows if any(c for c in r))


def _save(image_dir: Optional[str], stem: str, data: bytes, ext: str) -> Optional[str]:
    if not image_dir:
        return None
    os.makedirs(image_dir, exist_ok=True)
    path = os.path.join(image_dir, stem + ext)
    with open(path, "wb") as f:
        f.write(data)
    return path


def _image_doc(describe: Optional[Describe], path: Optional[str], w: int, h: int, before: str, after: str,
               meta: dict) -> Optional[Document]:
    ctx = " ".join(t for t in (before, after) if t)
    desc = ""
    if describe is not None and path is not None:
        try:
            desc = describe(path, ctx) or ""
        except Exception:  # a failing VLM must not lose the document
            desc = ""
    if not desc:
        desc = f"an embedded image ({w}x{h} pixels)"
    caption = " ".join(t for t in (before.replace("\n", " "), desc, after.replace("\n", " ")) if t).strip()
    if not caption:
        return None
    return Document("This is an image with the caption: " + caption, dict(meta, type="image", caption=caption,
                                                                          image=path or ""))


def pdf_documents(data: bytes, filename: str, describe: Optional[Describe] = None,
                  image_dir: Optional[str] = None, crop: float = 0.1) -> List[Document]:
    docs: List[Document] = []
    stem0 = re.sub(r"[^A-Za-z0-9_.-]", "_", os.path.splitext(os.path.basename(filename))[0])
    for pg in pdfmod.parse_pdf(data):
        meta = {"source": filename, "filename": filename, "page": pg.number, "page_num": pg.number - 1}
        lo, hi = pg.height * crop, pg.height * (1 - crop)
        body_runs = [r for r in pg.runs if lo <= r.y <= hi]
        lines_all = pdfmod.page_lines(pg, body_runs)
        # tables
        for ti, t in enumerate(pg.tables, 1):
            before, after = pdfmod.around(lines_all, t.bbox, pg.height)
            txt = stringify_table(t.rows)
            if txt:
                head = f"{before}\n" if before else ""
                docs.append(Document(f"{head}This is a table with the following rows:\n{txt}",
                                     dict(meta, type="table", table=ti, bbox=list(t.bbox))))
        # text outside tables
        free = [r for r in body_runs if not any(pdfmod._inside(r, t.bbox) for t in pg.tables)]
        for heading, body in pdfmod.text_blocks(pdfmod.page_lines(pg, free)):
            text = f"{heading}\n{body}".strip()
            if text:
                docs.append(Document(text, dict(meta, type="text")))
        # images
        for ii, im in enumerate(pg.images, 1):
            if im.width * im.height < 64:  # decorations
                continue
            before, after = pdfmod.around(lines_all, im.bbox, pg.height)
            path = _save(image_dir, f"{stem0}-page{pg.number}-image{ii}", im.data, im.ext)
            d = _image_doc(describe, path, im.width, im.height, before, after, dict(meta, bbox=list(im.bbox)))
            if d:
                docs.append(d)
    return docs


# ------------------------------------------------------------------------------------------------ PPTX
_A_T = re.compile(r"<a:t>(.*?)</a:t>", re.S)


def _paras(xml: str) -> List[str]:
    out = []
    for p in re.findall(r"<a:p>(.*?)</a:p>|<a:p .*?>(.*?)</a:p>", xml, re.S):
        body = p[0] or p[1]
        t = "".join(html.unescape(x) for x in _A_T.findall(body)).strip()
        if t:
            out.append(t)
    return out


def _tables(xml: str) -> List[List[List[str]]]:
    tabs = []
    for tb in re.findall(r"<a:tbl>(.*?)</a:tbl>", xml, re.S):
        rows = []
        for tr in re.findall(r"<a:tr[ >](.*?)</a:tr>", tb, re.S):
            rows.append([" ".join(_paras(tc)) for tc in re.findall(r"<a:tc[ >](.*?)</a:tc>", tr, re.S)])
        tabs.append(rows)
    return tabs


def pptx_documents(data: bytes, filename: str, describe: Optional[Describe] = None,
                   image_dir: Optional[str] = None) -> List[Document]:
    z = zipfile.ZipFile(io.BytesIO(data))
    names = set(z.namelist())
    slides = sorted((n for n in names if re.match(r"ppt/slides/slide\d+\.xml$", n)),
                    key=lambda n: int(re.findall(r"\d+", n)[-1]))
    stem0 = re.sub(r"[^A-Za-z0-9_.-]", "_", os.path.splitext(os.path.basename(filename))[0])
    docs: List[Document] = []
    for si, n in enumerate(slides, 1):
        xml = z.read(n).decode("utf-8", "replace")
        meta = {"source": filename, "filename": filename, "page": si, "page_num": si - 1}
        tabs = _tables(xml)
        no_tab = re.sub(r"<a:tbl>.*?</a:tbl>", "", xml, flags=re.S)
        paras = _paras(no_tab)
        title = paras[0] if paras else ""
        text = "\n".join(paras)
        note = n.replace("slides/slide", "notesSlides/notesSlide")
        notes = ""
        if note in names:
            notes = "\n".join(p for p in _paras(z.read(note).decode("utf-8", "replace"))
                              if not re.fullmatch(r"\d+", p))
        if text or notes:
            docs.append(Document(text + (f"\nNotes: {notes}" if notes else ""), dict(meta, type="text")))
        for ti, rows in enumerate(tabs, 1):
            txt = stringify_table(rows)
            if txt:
                docs.append(Document(f"{title}\nThis is a table with the following rows:\n{txt}".strip(),
                                     dict(meta, type="table", table=ti)))
        rel = n.replace("slides/slide", "slides/_rels/slide") + ".rels"
        if rel in names:
            rels = dict(re.findall(r'Id="([^"]+)"[^>]*Target="([^"]+)"', z.read(rel).decode("utf-8", "replace")))
            rels.update({k: v for v, k in re.findall(r'Target="([^"]+)"[^>]*Id="([^"]+)"',
                                                     z.read(rel).decode("utf-8", "replace"))})
            for ii, rid in enumerate(re.findall(r'<a:blip [^>]*r:embed="([^"]+)"', xml), 1):
                target = rels.get(rid)
                if not target:
                    continue
                media = os.path.normpath(os.path.join("ppt/slides", target)).replace("\\", "/")
                if media not in names:
                    continue
                img = z.read(media)
                ext = os.path.splitext(media)[1].lower() or ".png"
                path = _save(image_dir, f"{stem0}-slide{si}-image{ii}", img, ext)
                from ..examples.multimodal import image_size  # local: avoids an import cycle

                sz = image_size(img) or (0, 0)
                d = _image_doc(describe, path, sz[0], sz[1], title, notes[:200], meta)
                if d:
                    docs.append(d)
    return docs
