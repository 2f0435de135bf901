"""PDF document understanding without third-party parsers (pdfplumber / PyMuPDF / unstructured are not
available offline): a small PDF object reader and content-stream interpreter that yields, per page,

* positioned text runs decoded through the font's ``/ToUnicode`` CMap (bfchar / bfrange, incl. the
  array form), Type0 / CID fonts (Identity-H two-byte codes), and simple fonts with ``/Differences`` over
  WinAnsi / Standard encodings - so CID-font PDFs (most real ones) do not ingest as glyph codes;
* ruled tables: stroked lines and thin filled rectangles are clustered into a cell grid and the text
  runs are assigned to cells (the reference's ``find_tables(horizontal/vertical_strategy=lines_strict)``);
* embedded raster images (``Do`` of an image XObject, incl. inside form XObjects) with their page
  bounding box: DCT streams come out as JPEG files, Flate RGB / gray as PNG, for the vision model;
* text blocks grouped into lines / paragraphs with font-size headings, header / footer bands cropped
  (10 % of the page height, as the reference does).

Reference behaviour: RAG/examples/advanced_rag/multimodal_rag/vectorstore/custom_pdf_parser.py
(get_pdf_documents:312-370, parse_all_tables / parse_all_images, extract_text_around_item, stringify_table).
Objects are found by scanning for ``N G obj`` plus the contents of object streams (``/Type /ObjStm``), so
cross-reference tables and xref streams are not needed.
"""
from __future__ import annotations

import base64
import re
import struct
import zlib
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

# ------------------------------------------------------------------------------------------------ lexer
_WS = b" \t\r\n\x0c\x00"
_DELIM = b"()<>[]{}/%"


class Name(str):
    pass


@dataclass(frozen=True)
class Ref:
    num: int
    gen: int = 0


@dataclass
class Stream:
    dic: Dict[str, Any]
    raw: bytes


class Lexer:
    def __init__(self, data: bytes, pos: int = 0):
        self.d, self.p = data, pos

    def skip(self):
        d, n = self.d, len(self.d)
        while self.p < n:
            c = d[self.p]
            if c in _WS:
                self.p += 1
            elif c == 0x25:  # % comment
                while self.p < n and d[self.p] not in b"\r\n":
                    self.p += 1
            else:
                break

    def token(self):
        """Next raw token: ('num', v) ('name', s) ('str', b) ('op', s) or delimiters '[' ']' '<<' '>>'."""
        self.skip()
        d, p = self.d, self.p
        if p >= len(d):
            return None
        c = d[p]
        if c == 0x2F:  # /Name
            q = p + 1
            while q < len(d) and d[q] not in _WS and d[q] not in _DELIM:
                q += 1
            self.p = q
            raw = d[p + 1:q]
            name = re.sub(rb"#([0-9A-Fa-f]{2})", lambda m: bytes([int(m.group(1), 16)]), raw)
            return ("name", Name(name.decode("latin-1")))
        if c == 0x28:  # (literal string)
            depth, q, out = 1, p + 1, bytearray()
            while q < len(d) and depth:
                ch = d[q]
                if ch == 0x5C and q + 1 < len(d):
                    nx = d[q + 1]
                    esc = {0x6E: 10, 0x72: 13, 0x74: 9, 0x62: 8, 0x66: 12}
                    if nx in esc:
                        out.append(esc[nx])
                        q += 2
                    elif 0x30 <= nx <= 0x37:
                        j, v = q + 1, 0
                        while j < len(d) and j < q + 4 and 0x30 <= d[j] <= 0x37:
                            v = v * 8 + d[j] - 0x30
                            j += 1
                        out.append(v & 255)
                        q = j
                    elif nx in b"\r\n":  # line continuation
                        q += 2
                        if nx == 0x0D and q < len(d) and d[q] == 0x0A:
                            q += 1
                    else:
                        out.append(nx)
                        q += 2
                    continue
                if ch == 0x28:
                    depth += 1
                elif ch == 0x29:
                    depth -= 1
                    if depth == 0:
                        q += 1
                        break
                out.append(ch)
                q += 1
            self.p = q
            return ("str", bytes(out))
        if c == 0x3C:
            if p + 1 < len(d) and d[p + 1] == 0x3C:
                self.p = p + 2
                return ("<<", None)
            q = d.find(b">", p)
            q = len(d) if q < 0 else q
            hexs = re.sub(rb"[^0-9A-Fa-f]", b"", d[p + 1:q])
            if len(hexs) % 2:
                hexs += b"0"
            self.p = q + 1
            return ("str", bytes.fromhex(hexs.decode()))
        if c == 0x3E and p + 1 < len(d) and d[p + 1] == 0x3E:
            self.p = p + 2
            return (">>", None)
        if c in b"[]{}":
            self.p = p + 1
            return (chr(c), None)
        q = p
        while q < len(d) and d[q] not in _WS and d[q] not in _DELIM:
            q += 1
        if q == p:  # stray delimiter
            self.p = p + 1
            return ("op", chr(c))
        self.p = q
        w = d[p:q]
        try:
            return ("num", int(w)) if re.fullmatch(rb"[+-]?\d+", w) else ("num", float(w))
        except ValueError:
            return ("op", w.decode("latin-1"))

    def obj(self, tok=None):
        """Parse one object (resolving 'N G R' references)."""
        tok = tok or self.token()
        if tok is None:
            return None
        k, v = tok
        if k == "num" and isinstance(v, int):
            save = self.p
            t2 = self.token()
            if t2 and t2[0] == "num" and isinstance(t2[1], int):
                t3 = self.token()
                if t3 == ("op", "R"):
                    return Ref(v, t2[1])
            self.p = save
            return v
        if k in ("num", "name", "str"):
            return v
        if k == "[":
            arr = []
            while True:
                t = self.token()
                if t is None or t[0] == "]":
                    return arr
                arr.append(self.obj(t))
        if k == "<<":
            dic = {}
            while True:
                t = self.token()
                if t is None or t[0] == ">>":
                    return dic
                if t[0] == "name":
                    dic[str(t[1])] = self.obj()
        if k == "op":
            return {"true": True, "false": False, "null": None}.get(v, Name(v))
        return None


# ------------------------------------------------------------------------------------------------ filters
def _png_unpredict(data: bytes, columns: int, colors: int = 1, bpc: int = 8) -> bytes:
    bpp = max(1, colors * bpc // 8)
    row = (columns * colors * bpc + 7) // 8
    out, prev = bytearray(), bytearray(row)
    for i in range(0, len(data), row + 1):
        ft, line = data[i], bytearray(data[i + 1:i + 1 + row])
        for j in range(len(line)):
            a = line[j - bpp] if j >= bpp else 0
            b, c = prev[j], (prev[j - bpp] if j >= bpp else 0)
            if ft == 1:
                line[j] = (line[j] + a) & 255
            elif ft == 2:
                line[j] = (line[j] + b) & 255
            elif ft == 3:
                line[j] = (line[j] + (a + b) // 2) & 255
            elif ft == 4:
                pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                line[j] = (line[j] + (a if pa <= pb and pa <= pc else b if pb <= pc else c)) & 255
        out += line
        prev = line
    return bytes(out)


def decode_stream(s: Stream, doc: "PdfDocument" = None) -> Optional[bytes]:
    """Apply the stream's filters; None when a filter is not supported. DCTDecode / JPX data is returned
    as-is (the caller treats it as an image file)."""
    flt = doc.resolve(s.dic.get("Filter")) if doc else s.dic.get("Filter")
    parms = doc.resolve(s.dic.get("DecodeParms")) if doc else s.dic.get("DecodeParms")
    fl = flt if isinstance(flt, list) else ([flt] if flt else [])
    pl = parms if isinstance(parms, list) else [parms] * len(fl)
    data = s.raw
    for f, p in zip(fl, pl):
        f = str(f)
        if f in ("FlateDecode", "Fl"):
            # bounded inflate: a small crafted stream (zip bomb) must not exhaust the ingest server's memory
            budget = doc.inflate_budget() if doc is not None else MAX_STREAM_BYTES
            try:
                z = zlib.decompressobj()
                data = z.decompress(data, budget + 1)
            except zlib.error:
                return None
            if len(data) > budget or z.unconsumed_tail:
                return None  # over the per-stream / per-document budget: skip the stream
            if doc is not None:
                doc.inflated += len(data)
            if isinstance(p, dict) and int(p.get("Predictor", 1)) >= 10:
                data = _png_unpredict(data, int(p.get("Columns", 1)), int(p.get("Colors", 1)),
                                      int(p.get("BitsPerComponent", 8)))
        elif f in ("ASCIIHexDecode", "AHx"):
            h = re.sub(rb"[^0-9A-Fa-f]", b"", data.split(b">")[0])
            data = bytes.fromhex((h + b"0" * (len(h) % 2)).decode())
        elif f in ("ASCII85Decode", "A85"):
            body = data.strip()
            if body.startswith(b"<~"):
                body = body[2:]
            data = base64.a85decode(body.split(b"~>")[0] + b"~>", adobe=True)
        elif f in ("DCTDecode", "DCT", "JPXDecode"):
            return data
        else:
            return None
    return data


# ------------------------------------------------------------------------------------------------ fonts
_WINANSI_HI = {0x80: "€", 0x82: "‚", 0x83: "ƒ", 0x84: "„", 0x85: "…", 0x86: "†",
               0x87: "‡", 0x88: "ˆ", 0x89: "‰", 0x8A: "Š", 0x8B: "‹", 0x8C: "Œ",
               0x8E: "Ž", 0x91: "‘", 0x92: "’", 0x93: "“", 0x94: "”", 0x95: "•",
               0x96: "–", 0x97: "—", 0x98: "˜", 0x99: "™", 0x9A: "š", 0x9B: "›",
               0x9C: "œ", 0x9E: "ž", 0x9F: "Ÿ"}
# glyph names of /Differences beyond uniXXXX / single letters
_GLYPHS = {"space": " ", "exclam": "!", "quotedbl": '"', "numbersign": "#", "dollar": "$", "percent": "%",
           "ampersand": "&", "quotesingle": "'", "parenleft": "(", "parenright": ")", "asterisk": "*", "plus": "+",
           "comma": ",", "hyphen": "-", "period": ".", "slash": "/", "zero": "0", "one": "1", "two": "2",
           "three": "3", "four": "4", "five": "5", "six": "6", "seven": "7", "eight": "8", "nine": "9",
           "colon": ":", "semicolon": ";", "less": "<", "equal": "=", "greater": ">", "question": "?", "at": "@",
           "bracketleft": "[", "backslash": "\\", "bracketright": "]", "underscore": "_", "quoteleft": "‘",
           "quoteright": "’", "bullet": "•", "endash": "–", "emdash": "—", "fi": "fi",
           "fl": "fl", "degree": "°", "copyright": "©", "registered": "®", "trademark": "™"}


def _glyph_char(name: str) -> str:
    if name in _GLYPHS:
        return _GLYPHS[name]
    if len(name) == 1:
        return name
    m = re.fullmatch(r"uni([0-9A-Fa-f]{4})+", name)
    if m:
        return "".join(chr(int(name[i:i + 4], 16)) for i in range(3, len(name), 4))
    m = re.fullmatch(r"u([0-9A-Fa-f]{4,6})", name)
    return chr(int(m.group(1), 16)) if m else ""


def parse_cmap(data: bytes) -> Tuple[Dict[int, str], int]:
    """ToUnicode CMap -> ({code: text}, code byte width)."""
    out: Dict[int, str] = {}
    width = 1
    for m in re.finditer(rb"begincodespacerange(.*?)endcodespacerange", data, re.S):
        hx = re.findall(rb"<([0-9A-Fa-f]+)>", m.group(1))
        if hx:
            width = max(width, len(hx[0]) // 2)

    def u16(h: bytes) -> str:
        b = bytes.fromhex(h.decode())
        try:
            return b.decode("utf-16-be")
        except UnicodeDecodeError:
            return ""

    for m in re.finditer(rb"beginbfchar(.*?)endbfchar", data, re.S):
        for src, dst in re.findall(rb"<([0-9A-Fa-f]+)>\s*<([0-9A-Fa-f]*)>", m.group(1)):
            out[int(src, 16)] = u16(dst)
            width = max(width, len(src) // 2)
    for m in re.finditer(rb"beginbfrange(.*?)endbfrange", data, re.S):
        body = m.group(1)
        for lo, hi, rest in re.findall(rb"<([0-9A-Fa-f]+)>\s*<([0-9A-Fa-f]+)>\s*(<[0-9A-Fa-f]*>|\[[^\]]*\])", body):
            a, b = int(lo, 16), int(hi, 16)
            width = max(width, len(lo) // 2)
            if rest.startswith(b"["):
                for i, h in enumerate(re.findall(rb"<([0-9A-Fa-f]*)>", rest)):
                    if a + i <= b:
                        out[a + i] = u16(h)
            else:
                base = bytes.fromhex(rest[1:-1].decode())
                for i in range(b - a + 1):
                    v = bytearray(base)
                    if v:
                        v[-1] = (v[-1] + i) & 255
                        if base[-1] + i > 255 and len(v) > 1:
                            v[-2] = (v[-2] + (base[-1] + i) // 256) & 255
                    try:
                        out[a + i] = bytes(v).decode("utf-16-be")
                    except UnicodeDecodeError:
                        pass
    return out, width


class Font:
    def __init__(self, dic: dict, doc: "PdfDocument"):
        self.cmap: Dict[int, str] = {}
        self.width = 1
        self.diff: Dict[int, str] = {}
        sub = str(doc.resolve(dic.get("Subtype", "")))
        self.cid = sub == "Type0"
        tu = doc.resolve(dic.get("ToUnicode"))
        if isinstance(tu, Stream):
            data = decode_stream(tu, doc)
            if data:
                self.cmap, self.width = parse_cmap(data)
        if self.cid:
            self.width = 2 if not self.cmap or self.width < 2 else self.width
        enc = doc.resolve(dic.get("Encoding"))
        if isinstance(enc, dict):
            diffs = doc.resolve(enc.get("Differences")) or []
            code = 0
            for d in diffs:
                if isinstance(d, int):
                    code = d
                else:
                    self.diff[code] = _glyph_char(str(d))
                    code += 1

    def decode(self, s: bytes) -> str:
        w = self.width
        out = []
        for i in range(0, len(s) - w + 1, w):
            code = int.from_bytes(s[i:i + w], "big")
            if code in self.cmap:
                out.append(self.cmap[code])
            elif code in self.diff:
                out.append(self.diff[code])
            elif self.cid:
                continue  # unmapped CID: no text
            elif code in _WINANSI_HI:
                out.append(_WINANSI_HI[code])
            else:
                out.append(chr(code) if code >= 32 else (" " if code in (9, 10, 13) else ""))
        return "".join(out)


# ------------------------------------------------------------------------------------------------ document
@dataclass
class TextRun:
    x: float
    y: float
    size: float
    text: str


@dataclass
class PdfImage:
    bbox: Tuple[float, float, float, float]  # x0, y0, x1, y1 (PDF user space, y up)
    data: bytes                              # a JPEG or PNG file
    ext: str
    width: int
    height: int


@dataclass
class PdfTable:
    bbox: Tuple[float, float, float, float]
    rows: List[List[str]]


@dataclass
class PdfPage:
    number: int
    width: float
    height: float
    runs: List[TextRun] = field(default_factory=list)
    images: List[PdfImage] = field(default_factory=list)
    hlines: List[Tuple[float, float, float]] = field(default_factory=list)  # y, x0, x1
    vlines: List[Tuple[float, float, float]] = field(default_factory=list)  # x, y0, y1
    tables: List[PdfTable] = field(default_factory=list)


_OBJ_RE = re.compile(rb"(\d+)\s+(\d+)\s+obj\b")


MAX_STREAM_BYTES = 64 << 20     # inflated bytes per stream
MAX_DOCUMENT_BYTES = 512 << 20  # inflated bytes per document


class PdfDocument:
    def __init__(self, data: bytes):
        self.data = data
        self.inflated = 0
        self.objs: Dict[int, Any] = {}
        self._scan()
        self.fonts: Dict[int, Font] = {}

    def inflate_budget(self) -> int:
        return max(0, min(MAX_STREAM_BYTES, MAX_DOCUMENT_BYTES - self.inflated))

    # ---- objects
    def _parse_at(self, pos: int):
        lx = Lexer(self.data, pos)
        o = lx.obj()
        if isinstance(o, dict):
            save = lx.p
            t = lx.token()
            if t == ("op", "stream"):
                p = lx.p
                if self.data[p:p + 2] == b"\r\n":
                    p += 2
                elif self.data[p:p + 1] in (b"\n", b"\r"):
                    p += 1
                n = o.get("Length")
                end = -1
                if isinstance(n, int) and self.data[p + n:p + n + 20].lstrip().startswith(b"endstream"):
                    end = p + n
                if end < 0:
                    end = self.data.find(b"endstream", p)
                    end = len(self.data) if end < 0 else end
                    while end > p and self.data[end - 1] in b"\r\n":
                        end -= 1
                return Stream(o, self.data[p:end])
            lx.p = save
        return o

    def _scan(self):
        for m in _OBJ_RE.finditer(self.data):
            num = int(m.group(1))
            try:
                self.objs[num] = self._parse_at(m.end())
            except Exception:  # a damaged object: skip it
                continue
        for num, o in list(self.objs.items()):  # object streams (PDF 1.5)
            if isinstance(o, Stream) and str(o.dic.get("Type")) == "ObjStm":
                data = decode_stream(o, self)
                if not data:
                    continue
                n, first = int(self.resolve(o.dic.get("N", 0))), int(self.resolve(o.dic.get("First", 0)))
                hdr = Lexer(data[:first])
                pairs = []
                for _ in range(n):
                    a, b = hdr.token(), hdr.token()
                    if not a or not b:
                        break
                    pairs.append((a[1], b[1]))
                for onum, off in pairs:
                    if onum not in self.objs:
                        try:
                            self.objs[onum] = Lexer(data, first + off).obj()
                        except Exception:
                            continue

    def resolve(self, o, depth: int = 0):
        while isinstance(o, Ref) and depth < 32:
            o = self.objs.get(o.num)
            depth += 1
        return o

    def font(self, ref_or_dic) -> Font:
        key = ref_or_dic.num if isinstance(ref_or_dic, Ref) else id(ref_or_dic)
        f = self.fonts.get(key)
        if f is None:
            d = self.resolve(ref_or_dic)
            f = Font(d if isinstance(d, dict) else {}, self)
            self.fonts[key] = f
        return f

    # ---- pages
    def pages(self) -> List[dict]:
        root = None
        for o in self.objs.values():
            if isinstance(o, dict) and str(o.get("Type")) == "Catalog":
                root = o
                break
        out: List[dict] = []

        def walk(node, inherited, depth=0):
            node = self.resolve(node)
            if not isinstance(node, dict) or depth > 64:
                return
            inh = dict(inherited)
            for k in ("Resources", "MediaBox"):
                if k in node:
                    inh[k] = node[k]
            if str(node.get("Type")) == "Pages" or "Kids" in node:
                for kid in self.resolve(node.get("Kids")) or []:
                    walk(kid, inh, depth + 1)
            else:
                p = dict(node)
                for k, v in inh.items():
                    p.setdefault(k, v)
                out.append(p)

        if root is not None:
            walk(root.get("Pages"), {})
        if not out:  # no catalog: every page object in file order
            out = [o for o in self.objs.values() if isinstance(o, dict) and str(o.get("Type")) == "Page"]
        return out

    def page(self, i: int, pdict: dict) -> PdfPage:
        mb = [float(self.resolve(v)) for v in (self.resolve(pdict.get("MediaBox")) or [0, 0, 612, 792])]
        pg = PdfPage(i + 1, mb[2] - mb[0], mb[3] - mb[1])
        contents = self.resolve(pdict.get("Contents"))
        streams = contents if isinstance(contents, list) else [contents]
        data = b"\n".join(d for d in (decode_stream(self.resolve(s), self) if isinstance(self.resolve(s), Stream)
                                      else None for s in streams) if d)
        _Interp(self, pg).run(data, self.resolve(pdict.get("Resources")) or {}, [1, 0, 0, 1, 0, 0])
        pg.tables = find_tables(pg)
        return pg


def _mul(a, b):  # 2-D affine [a b c d e f] products: a then b
    return [a[0] * b[0] + a[1] * b[2], a[0] * b[1] + a[1] * b[3], a[2] * b[0] + a[3] * b[2],
            a[2] * b[1] + a[3] * b[3], a[4] * b[0] + a[5] * b[2] + b[4], a[4] * b[1] + a[5] * b[3] + b[5]]


def _apply(m, x, y):
    return m[0] * x + m[2] * y + m[4], m[1] * x + m[3] * y + m[5]


class _Interp:
    """Content-stream interpreter: text runs (position, size, decoded text), image placements, lines."""

    def __init__(self, doc: PdfDocument, page: PdfPage):
        self.doc, self.pg = doc, page

    def run(self, data: bytes, res: dict, ctm: list, depth: int = 0):
        doc = self.doc
        fonts = doc.resolve(res.get("Font")) or {}
        xobjs = doc.resolve(res.get("XObject")) or {}
        lx = Lexer(data)
        ops: List[Any] = []
        stack = []
        font, size, leading = None, 12.0, 0.0
        tm = lm = [1, 0, 0, 1, 0, 0]
        path: List[Tuple[str, list]] = []
        cur = (0.0, 0.0)
        while True:
            t = lx.token()
            if t is None:
                break
            k, v = t
            if k != "op":
                lx_obj = lx.obj(t) if k in ("[", "<<") else v
                ops.append(lx_obj)
                continue
            op = v
            if op == "BI":  # inline image: skip to EI
                end = data.find(b"EI", lx.p)
                lx.p = len(data) if end < 0 else end + 2
                ops = []
                continue
            a = ops
            ops = []
            try:
                if op == "q":
                    stack.append(ctm)
                elif op == "Q":
                    ctm = stack.pop() if stack else ctm
                elif op == "cm" and len(a) >= 6:
                    ctm = _mul([float(x) for x in a[-6:]], ctm)
                elif op == "BT":
                    tm = lm = [1, 0, 0, 1, 0, 0]
                elif op == "Tf" and len(a) >= 2:
                    f = fonts.get(str(a[-2])) if isinstance(fonts, dict) else None
                    font = doc.font(f) if f is not None else None
                    size = float(a[-1])
                elif op == "TL" and a:
                    leading = float(a[-1])
                elif op in ("Td", "TD") and len(a) >= 2:
                    if op == "TD":
                        leading = -float(a[-1])
                    lm = _mul([1, 0, 0, 1, float(a[-2]), float(a[-1])], lm)
                    tm = lm
                elif op == "Tm" and len(a) >= 6:
                    lm = tm = [float(x) for x in a[-6:]]
                elif op == "T*":
                    lm = tm = _mul([1, 0, 0, 1, 0, -leading], lm)
                elif op in ("Tj", "'", '"', "TJ"):
                    if op in ("'", '"'):
                        lm = tm = _mul([1, 0, 0, 1, 0, -leading], lm)
                    items = a[-1] if op == "TJ" and a and isinstance(a[-1], list) else a[-1:]
                    text = []
                    for it in items:
                        if isinstance(it, bytes):
                            text.append(font.decode(it) if font else it.decode("latin-1"))
                        elif isinstance(it, (int, float)) and it < -200 and text and not text[-1].endswith(" "):
                            text.append(" ")  # a kerning gap wider than a fifth of an em is a word break
                    s = "".join(text)
                    m = _mul(tm, ctm)
                    x, y = _apply(m, 0, 0)
                    eff = size * (abs(m[3]) or abs(m[0]) or 1.0)
                    if s.strip():
                        self.pg.runs.append(TextRun(x, y, eff, s))
                    adv = 0.5 * size * len(s)  # approximate advance (glyph widths are not parsed)
                    tm = _mul([1, 0, 0, 1, adv, 0], tm)
                elif op == "Do" and a:
                    xo = xobjs.get(str(a[-1])) if isinstance(xobjs, dict) else None
                    xs = doc.resolve(xo)
                    if isinstance(xs, Stream):
                        sub = str(xs.dic.get("Subtype"))
                        if sub == "Image":
                            self._image(xs, ctm)
                        elif sub == "Form" and depth < 8:
                            fm = [float(x) for x in (doc.resolve(xs.dic.get("Matrix")) or [1, 0, 0, 1, 0, 0])]
                            body = decode_stream(xs, doc)
                            if body:
                                self.run(body, doc.resolve(xs.dic.get("Resources")) or res, _mul(fm, ctm), depth + 1)
                # ---- paths (for ruled tables)
                elif op == "m" and len(a) >= 2:
                    cur = (float(a[-2]), float(a[-1]))
                    path.append(("m", [cur]))
                elif op == "l" and len(a) >= 2:
                    nxt = (float(a[-2]), float(a[-1]))
                    path.append(("l", [cur, nxt]))
                    cur = nxt
                elif op == "re" and len(a) >= 4:
                    x, y, w, h = (float(z) for z in a[-4:])
                    path.append(("re", [(x, y), (x + w, y + h)]))
                elif op in ("S", "s", "f", "F", "f*", "B", "B*", "b", "b*"):
                    self._paint(path, ctm, stroke=op in ("S", "s", "B", "B*", "b", "b*"))
                    path = []
                elif op == "n":
                    path = []
            except (ValueError, TypeError, IndexError, AttributeError):
                continue

    def _paint(self, path, ctm, stroke: bool):
        for kind, pts in path:
            if kind == "l":
                (x0, y0), (x1, y1) = (_apply(ctm, *pts[0]), _apply(ctm, *pts[1]))
                self._seg(x0, y0, x1, y1)
            elif kind == "re":
                (x0, y0), (x1, y1) = (_apply(ctm, *pts[0]), _apply(ctm, *pts[1]))
                x0, x1 = sorted((x0, x1))
                y0, y1 = sorted((y0, y1))
                if stroke:
                    for seg in ((x0, y0, x1, y0), (x0, y1, x1, y1), (x0, y0, x0, y1), (x1, y0, x1, y1)):
                        self._seg(*seg)
                elif y1 - y0 <= 3 and x1 - x0 > 3:  # filled hairline rectangles are rules too
                    self._seg(x0, (y0 + y1) / 2, x1, (y0 + y1) / 2)
                elif x1 - x0 <= 3 and y1 - y0 > 3:
                    self._seg((x0 + x1) / 2, y0, (x0 + x1) / 2, y1)

    def _seg(self, x0, y0, x1, y1):
        if abs(y1 - y0) < 1.0 and abs(x1 - x0) > 2:
            self.pg.hlines.append(((y0 + y1) / 2, min(x0, x1), max(x0, x1)))
        elif abs(x1 - x0) < 1.0 and abs(y1 - y0) > 2:
            self.pg.vlines.append(((x0 + x1) / 2, min(y0, y1), max(y0, y1)))

    def _image(self, xs: Stream, ctm):
        doc = self.doc
        w, h = int(doc.resolve(xs.dic.get("Width", 0)) or 0), int(doc.resolve(xs.dic.get("Height", 0)) or 0)
        pts = [_apply(ctm, x, y) for x, y in ((0, 0), (1, 0), (0, 1), (1, 1))]
        xs_, ys_ = [p[0] for p in pts], [p[1] for p in pts]
        bbox = (min(xs_), min(ys_), max(xs_), max(ys_))
        flt = doc.resolve(xs.dic.get("Filter"))
        fl = [str(f) for f in (flt if isinstance(flt, list) else [flt] if flt else [])]
        data = decode_stream(xs, doc)
        if data is None:
            return
        if fl and fl[-1] in ("DCTDecode", "DCT"):
            self.pg.images.append(PdfImage(bbox, data, ".jpg", w, h))
            return
        if fl and fl[-1] == "JPXDecode":
            self.pg.images.append(PdfImage(bbox, data, ".jp2", w, h))
            return
        cs = doc.resolve(xs.dic.get("ColorSpace"))
        csn = str(cs[0] if isinstance(cs, list) and cs else cs)
        bpc = int(doc.resolve(xs.dic.get("BitsPerComponent", 8)) or 8)
        comps = {"DeviceRGB": 3, "DeviceGray": 1, "CalRGB": 3, "CalGray": 1}.get(csn)
        if comps is None and isinstance(cs, list) and str(cs[0]) == "ICCBased":
            icc = doc.resolve(cs[1])
            comps = int(doc.resolve(icc.dic.get("N", 3))) if isinstance(icc, Stream) else 3
        if comps in (1, 3) and bpc == 8 and w and h and len(data) >= w * h * comps:
            self.pg.images.append(PdfImage(bbox, encode_png(data[:w * h * comps], w, h, comps), ".png", w, h))


def encode_png(pixels: bytes, w: int, h: int, comps: int) -> bytes:
    """Raw 8-bit gray / RGB rows -> a PNG file."""
    raw = b"".join(b"\x00" + pixels[r * w * comps:(r + 1) * w * comps] for r in range(h))

    def chunk(tag, body):
        return struct.pack(">I", len(body)) + tag + body + struct.pack(">I", zlib.crc32(tag + body) & 0xFFFFFFFF)

    ihdr = struct.pack(">IIBBBBB", w, h, 8, 2 if comps == 3 else 0, 0, 0, 0)
    return b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b"")


# ------------------------------------------------------------------------------------------------ tables
def _cluster(vals: List[float], tol: float) -> List[float]:
    out: List[float] = []
    for v in sorted(vals):
        if out and v - out[-1] <= tol:
            continue
        out.append(v)
    return out


def find_tables(pg: PdfPage, tol: float = 2.0) -> List[PdfTable]:
    """Grids of ruling lines -> tables: rows between consecutive horizontal rules, columns between
    consecutive vertical rules, text runs assigned by their start point."""
    if len(pg.hlines) < 2 or len(pg.vlines) < 2:
        return []
    # connected groups of lines by bounding-box overlap
    segs = [("h", y, x0, x1) for y, x0, x1 in pg.hlines] + [("v", x, y0, y1) for x, y0, y1 in pg.vlines]
    boxes = []
    for s in segs:
        if s[0] == "h":
            boxes.append([s[2], s[1], s[3], s[1]])
        else:
            boxes.append([s[1], s[2], s[1], s[3]])
    parent = list(range(len(segs)))

    def find(i):
        while parent[i] != i:
            parent[i] = parent[parent[i]]
            i = parent[i]
        return i

    for i in range(len(segs)):
        for j in range(i + 1, len(segs)):
            a, b = boxes[i], boxes[j]
            if a[0] - tol <= b[2] and b[0] - tol <= a[2] and a[1] - tol <= b[3] and b[1] - tol <= a[3]:
                parent[find(i)] = find(j)
    groups: Dict[int, List[int]] = {}
    for i in range(len(segs)):
        groups.setdefault(find(i), []).append(i)
    tables = []
    for idx in groups.values():
        ys = _cluster([segs[i][1] for i in idx if segs[i][0] == "h"], tol)
        xs = _cluster([segs[i][1] for i in idx if segs[i][0] == "v"], tol)
        if len(ys) < 2 or len(xs) < 2:
            continue
        ys = sorted(ys, reverse=True)  # top row first
        grid = [["" for _ in range(len(xs) - 1)] for _ in range(len(ys) - 1)]
        for r in pg.runs:
            if not (xs[0] - tol <= r.x <= xs[-1] + tol and ys[-1] - tol <= r.y <= ys[0] + tol):
                continue
            row = next((i for i in range(len(ys) - 1) if ys[i + 1] - tol <= r.y <= ys[i] + tol), None)
            col = next((j for j in range(len(xs) - 1) if xs[j] - tol <= r.x <= xs[j + 1] + tol), None)
            if row is not None and col is not None:
                grid[row][col] = (grid[row][col] + " " + r.text.strip()).strip()
        if any(any(c for c in row) for row in grid):
            tables.append(PdfTable((xs[0], ys[-1], xs[-1], ys[0]), grid))
    return tables


# ------------------------------------------------------------------------------------------------ layout
def _inside(r: TextRun, bbox, tol=2.0) -> bool:
    return bbox[0] - tol <= r.x <= bbox[2] + tol and bbox[1] - tol <= r.y <= bbox[3] + tol


def page_lines(pg: PdfPage, runs: List[TextRun], tol: float = 2.5) -> List[Tuple[float, float, str]]:
    """Runs -> lines (y, max font size, text), top to bottom."""
    lines: List[List[TextRun]] = []
    for r in sorted(runs, key=lambda r: (-r.y, r.x)):
        if lines and abs(lines[-1][0].y - r.y) <= tol:
            lines[-1].append(r)
        else:
            lines.append([r])
    out = []
    for ln in lines:
        ln.sort(key=lambda r: r.x)
        txt = " ".join(r.text.strip() for r in ln if r.text.strip())
        out.append((ln[0].y, max(r.size for r in ln), re.sub(r"\s+", " ", txt)))
    return out


def text_blocks(lines: List[Tuple[float, float, str]]) -> List[Tuple[str, str]]:
    """Lines -> (heading, body) blocks; a line in a font larger than the body text starts a block."""
    if not lines:
        return []
    sizes = sorted(s for _, s, _ in lines)
    body = sizes[len(sizes) // 2]
    blocks: List[Tuple[str, List[str]]] = []
    prev_y = None
    for y, s, t in lines:
        gap = prev_y - y if prev_y is not None else 0
        if s > body * 1.15 or not blocks or gap > 2.2 * max(s, body):
            blocks.append((t if s > body * 1.15 else "", [] if s > body * 1.15 else [t]))
        else:
            blocks[-1][1].append(t)
        prev_y = y
    return [(h, "\n".join(b)) for h, b in blocks]


def around(lines, bbox, page_h, frac=0.1) -> Tuple[str, str]:
    """Nearest text line above and below a bounding box (within frac of the page height)."""
    lim = page_h * frac
    above = [t for y, _, t in lines if bbox[3] < y <= bbox[3] + lim]
    below = [t for y, _, t in lines if bbox[1] - lim <= y < bbox[1]]
    return (above[-1] if above else ""), (below[0] if below else "")


def parse_pdf(data: bytes) -> List[PdfPage]:
    doc = PdfDocument(data)
    out = []
    for i, p in enumerate(doc.pages()):
        try:
            out.append(doc.page(i, p))
        except Exception:  # keep the other pages of a damaged file
            continue
    return out
