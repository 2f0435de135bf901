"""Structured PDF / PPTX ingest (rag/pdf.py, rag/multimodal_ingest.py): CID fonts through ToUnicode CMaps,
object streams, ruled tables, embedded images handed to the vision model, header/footer crop, PPTX
slides with notes, tables and pictures; plus the multimodal example end to end on a tiny stack."""
import io
import struct
import zipfile
import zlib

import pytest

from generativeaiexamples_amd.rag import pdf as pdfmod
from generativeaiexamples_amd.rag.multimodal_ingest import pdf_documents, pptx_documents

# ------------------------------------------------------------------------------------------ fixtures


def _cid_hex(text):
    # glyph ids: 'A'..'Z' -> 0x0011.., ' ' -> 0x0003, digits -> 0x0040 + d
    out = []
    for ch in text.upper():
        if ch == " ":
            out.append(0x0003)
        elif ch.isdigit():
            out.append(0x0040 + int(ch))
        else:
            out.append(0x0011 + ord(ch) - ord("A"))
    return "<" + "".join(f"{c:04X}" for c in out) + ">"


TOUNICODE = b"""/CIDInit /ProcSet findresource begin 12 dict begin begincmap
1 begincodespacerange <0000> <FFFF> endcodespacerange
1 beginbfchar <0003> <0020> endbfchar
2 beginbfrange <0011> <002A> <0041> <0040> <0049> [<0030> <0031> <0032> <0033> <0034> <0035> <0036> <0037> <0038> <0039>] endbfrange
endcmap CMapName currentdict /CMap defineresource pop end end"""


def make_rich_pdf() -> bytes:
    w, h = 12, 8
    pix = b"".join(bytes([x * 20 % 256, y * 30 % 256, 128]) for y in range(h) for x in range(w))
    content = "\n".join([
        "BT /F1 9 Tf 72 770 Td (ACME CONFIDENTIAL HEADER) Tj ET",
        f"BT /F2 18 Tf 72 700 Td {_cid_hex('QUARTERLY RESULTS')} Tj ET",
        "BT /F1 11 Tf 72 680 Td (Revenue grew strongly in the third quarter.) Tj 0 -14 Td "
        "[(Costs were ) -300 (flat.)] TJ ET",
        # a ruled 3 x 2 table
        "0.5 w 72 600 m 372 600 l S 72 580 m 372 580 l S 72 560 m 372 560 l S 72 540 m 372 540 l S",
        "72 540 m 72 600 l S 222 540 m 222 600 l S 372 540 m 372 600 l S",
        "BT /F1 10 Tf 80 586 Td (Region) Tj 150 0 Td (Sales) Tj ET",
        "BT /F1 10 Tf 80 566 Td (North) Tj 150 0 Td (120) Tj ET",
        "BT /F1 10 Tf 80 546 Td (South) Tj 150 0 Td (95) Tj ET",
        "BT /F1 10 Tf 72 470 Td (Figure 1: revenue by month) Tj ET",
        "q 120 0 0 80 72 380 cm /Im1 Do Q",
        "BT /F1 10 Tf 72 360 Td (Source: internal ledger) Tj ET",
        f"BT /F2 10 Tf 72 300 Td {_cid_hex('TOTAL 215 UNITS')} Tj ET",
        "BT /F1 9 Tf 72 20 Td (Page 1 footer) Tj ET",
    ]).encode()
    objs = {
        1: b"<< /Type /Catalog /Pages 2 0 R >>",
        2: b"<< /Type /Pages /Kids [3 0 R] /Count 1 >>",
        3: b"<< /Type /Page /Parent 2 0 R /MediaBox [0 0 612 792] /Contents 4 0 R "
           b"/Resources << /Font << /F1 5 0 R /F2 6 0 R >> /XObject << /Im1 9 0 R >> >> >>",
        5: b"<< /Type /Font /Subtype /Type1 /BaseFont /Helvetica /Encoding /WinAnsiEncoding >>",
        7: b"<< /Type /Font /Subtype /CIDFontType2 /BaseFont /Noto /CIDSystemInfo << /Registry (Adobe) "
           b"/Ordering (Identity) /Supplement 0 >> >>",
    }
    streams = {
        4: (b"<< /Filter /FlateDecode", zlib.compress(content)),
        8: (b"<< /Filter /FlateDecode", zlib.compress(TOUNICODE)),
        9: (b"<< /Type /XObject /Subtype /Image /Width %d /Height %d /ColorSpace /DeviceRGB "
            b"/BitsPerComponent 8 /Filter /FlateDecode" % (w, h), zlib.compress(pix)),
    }
    # the Type0 font dict lives in an object stream (PDF 1.5)
    f6 = b"<< /Type /Font /Subtype /Type0 /BaseFont /Noto /Encoding /Identity-H /DescendantFonts [7 0 R] " \
         b"/ToUnicode 8 0 R >>"
    hdr = b"6 0 "
    objstm = hdr + f6
    streams[10] = (b"<< /Type /ObjStm /N 1 /First %d /Filter /FlateDecode" % len(hdr), zlib.compress(objstm))
    out = io.BytesIO()
    out.write(b"%PDF-1.5\n")
    for n in sorted(set(objs) | set(streams)):
        if n in objs:
            out.write(b"%d 0 obj\n" % n + objs[n] + b"\nendobj\n")
        else:
            d, body = streams[n]
            out.write(b"%d 0 obj\n" % n + d + b" /Length %d >>\nstream\n" % len(body) + body + b"\nendstream\nendobj\n")
    out.write(b"trailer << /Root 1 0 R >>\n%%EOF\n")
    return out.getvalue()


def make_pptx() -> bytes:
    png = pdfmod.encode_png(bytes(range(48)) * 4, 8, 8, 3)
    slide = ('<p:sld xmlns:a="a" xmlns:p="p" xmlns:r="r"><p:cSld><p:spTree>'
             '<p:sp><p:txBody><a:p><a:r><a:t>Roadmap 2025</a:t></a:r></a:p></p:txBody></p:sp>'
             '<p:sp><p:txBody><a:p><a:r><a:t>Ship the MI355X engine</a:t></a:r></a:p></p:txBody></p:sp>'
             '<p:graphicFrame><a:graphic><a:graphicData><a:tbl>'
             '<a:tr h="1"><a:tc><a:txBody><a:p><a:r><a:t>Quarter</a:t></a:r></a:p></a:txBody></a:tc>'
             '<a:tc><a:txBody><a:p><a:r><a:t>Goal</a:t></a:r></a:p></a:txBody></a:tc></a:tr>'
             '<a:tr h="1"><a:tc><a:txBody><a:p><a:r><a:t>Q1</a:t></a:r></a:p></a:txBody></a:tc>'
             '<a:tc><a:txBody><a:p><a:r><a:t>TP serving</a:t></a:r></a:p></a:txBody></a:tc></a:tr>'
             '</a:tbl></a:graphicData></a:graphic></p:graphicFrame>'
             '<p:pic><p:blipFill><a:blip r:embed="rId2"/></p:blipFill></p:pic>'
             '</p:spTree></p:cSld></p:sld>')
    rels = ('<Relationships><Relationship Id="rId2" Type="image" Target="../media/image1.png"/>'
            '</Relationships>')
    notes = ('<p:notes xmlns:a="a" xmlns:p="p"><p:cSld><p:spTree><p:sp><p:txBody><a:p><a:r>'
             '<a:t>Mention the xGMI all-reduce</a:t></a:r></a:p></p:txBody></p:sp></p:spTree></p:cSld></p:notes>')
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as z:
        z.writestr("ppt/slides/slide1.xml", slide)
        z.writestr("ppt/slides/_rels/slide1.xml.rels", rels)
        z.writestr("ppt/notesSlides/notesSlide1.xml", notes)
        z.writestr("ppt/media/image1.png", png)
    return buf.getvalue()


# ------------------------------------------------------------------------------------------ tests
def test_cmap_parsing():
    m, w = pdfmod.parse_cmap(TOUNICODE)
    assert w == 2 and m[0x0011] == "A" and m[0x002A] == "Z" and m[0x0003] == " " and m[0x0043] == "3"


def test_pdf_text_tables_images():
    seen = []

    def describe(path, ctx):
        from PIL import Image

        im = Image.open(path)  # a real PNG of the embedded raster
        seen.append((im.size, ctx))
        return "a bar chart of monthly revenue"

    docs = pdf_documents(make_rich_pdf(), "report.pdf", describe=describe, image_dir=None)
    # no image_dir: the describer is not called, a placeholder is kept
    img = [d for d in docs if d.metadata["type"] == "image"]
    assert len(img) == 1 and "12x8" in img[0].page_content and "Figure 1" in img[0].page_content
    import tempfile

    with tempfile.TemporaryDirectory() as td:
        docs = pdf_documents(make_rich_pdf(), "report.pdf", describe=describe, image_dir=td)
    text = "\n".join(d.page_content for d in docs if d.metadata["type"] == "text")
    assert "QUARTERLY RESULTS" in text  # CID font decoded via ToUnicode (font dict in an ObjStm)
    assert "TOTAL 215 UNITS" in text
    assert "Revenue grew strongly" in text and "Costs were flat." in text
    assert "HEADER" not in text and "footer" not in text  # header / footer bands cropped
    tables = [d for d in docs if d.metadata["type"] == "table"]
    assert len(tables) == 1
    t = tables[0].page_content
    assert "Region | Sales" in t and "North | 120" in t and "South | 95" in t
    assert "North" not in text  # table cells are not duplicated as free text
    img = [d for d in docs if d.metadata["type"] == "image"]
    assert len(img) == 1 and "bar chart of monthly revenue" in img[0].page_content
    assert seen and seen[0][0] == (12, 8) and "Figure 1" in seen[0][1]


def test_loader_uses_structured_pdf(tmp_path):
    from generativeaiexamples_amd.rag import loaders

    p = tmp_path / "r.pdf"
    p.write_bytes(make_rich_pdf())
    docs = loaders.load(str(p))
    joined = "\n".join(d.page_content for d in docs)
    assert "QUARTERLY RESULTS" in joined and "North | 120" in joined
    assert all(d.metadata["filename"] == "r.pdf" for d in docs)
    # simple PDFs written by make_pdf still load
    q = tmp_path / "s.pdf"
    q.write_bytes(loaders.make_pdf(["hello world", "second page"]))
    assert [d.page_content for d in loaders.load(str(q))] == ["hello world", "second page"]


def test_pptx_slides_notes_tables_pictures(tmp_path):
    calls = []
    docs = pptx_documents(make_pptx(), "deck.pptx", describe=lambda p, c: calls.append(c) or "an architecture diagram",
                          image_dir=str(tmp_path))
    kinds = {d.metadata["type"] for d in docs}
    assert kinds == {"text", "table", "image"}
    text = next(d for d in docs if d.metadata["type"] == "text").page_content
    assert "Roadmap 2025" in text and "Notes: Mention the xGMI all-reduce" in text and "TP serving" not in text
    assert "Q1 | TP serving" in next(d for d in docs if d.metadata["type"] == "table").page_content
    assert "architecture diagram" in next(d for d in docs if d.metadata["type"] == "image").page_content
    assert calls and "Roadmap 2025" in calls[0]


def test_multimodal_example_ingests_pdf(tmp_path, monkeypatch):
    """The multimodal chain ingests every modality of the PDF into searchable chunks."""
    from generativeaiexamples_amd.chain_server import utils as cu
    from generativeaiexamples_amd.examples import multimodal
    from generativeaiexamples_amd.serving.hub import HubSpec, ServiceHub

    monkeypatch.setenv("APP_VECTORSTORE_NAME", "hbm")
    hub = ServiceHub.build(HubSpec(llm="tiny-llama", embedder="tiny-e5", device="cpu", max_num_seqs=4,
                                   max_model_len=512))
    monkeypatch.setattr(cu, "get_hub", lambda: hub)
    monkeypatch.setattr(multimodal, "get_hub", lambda: hub)
    monkeypatch.setattr(multimodal, "IMAGE_DIR", str(tmp_path / "img"))
    try:
        ex = multimodal.MultimodalRAG()
        p = tmp_path / "report.pdf"
        p.write_bytes(make_rich_pdf())
        ex.ingest_docs(str(p), "report.pdf")
        contents = [d.page_content for d in ex.store.documents()] if hasattr(ex.store, "documents") else None
        hits = ex.store.similarity_search("North sales table", k=50) if contents is None else None
        blob = "\n".join(contents if contents is not None else [d.page_content for d in hits])
        assert "QUARTERLY RESULTS" in blob and "North | 120" in blob and "This is an image" in blob
    finally:
        hub.shutdown()


def test_flate_bomb_is_bounded(monkeypatch):
    """A FlateDecode stream inflating past the per-stream budget is skipped, not inflated into memory."""
    import zlib

    from generativeaiexamples_amd.rag import pdf

    monkeypatch.setattr(pdf, "MAX_STREAM_BYTES", 1 << 20)
    bomb = zlib.compress(b"\0" * (8 << 20), 9)  # 8 MiB of zeros in ~8 KiB
    s = pdf.Stream({"Filter": "FlateDecode", "Length": len(bomb)}, bomb)
    doc = pdf.PdfDocument.__new__(pdf.PdfDocument)
    doc.inflated, doc.objs = 0, {}
    assert pdf.decode_stream(s, doc) is None
    ok = pdf.Stream({"Filter": "FlateDecode"}, zlib.compress(b"BT (hi) Tj ET"))
    assert pdf.decode_stream(ok, doc) == b"BT (hi) Tj ET"
