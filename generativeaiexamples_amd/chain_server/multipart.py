"""multipart/form-data parser (python-multipart is not available in this image, so FastAPI's
UploadFile cannot be used; ``POST /documents`` parses the body itself)."""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import List, Optional


@dataclass
class Part:
    name: Optional[str]
    filename: Optional[str]
    content_type: Optional[str]
    data: bytes


_DISP = re.compile(r'(\w+)\*?=(?:"((?:[^"\\]|\\.)*)"|([^;\s]+))')


def parse_multipart(content_type: str, body: bytes) -> List[Part]:
    m = re.search(r'boundary="?([^";]+)"?', content_type or "")
    if not m:
        raise ValueError("multipart request without boundary")
    delim = b"--" + m.group(1).encode("latin-1")
    parts: List[Part] = []
    for chunk in body.split(delim)[1:]:
        if chunk.startswith(b"--"):
            break
        chunk = chunk[2:] if chunk.startswith(b"\r\n") else chunk.lstrip(b"\n")
        head, sep, data = chunk.partition(b"\r\n\r\n")
        if not sep:
            head, sep, data = chunk.partition(b"\n\n")
        if data.endswith(b"\r\n"):
            data = data[:-2]
        elif data.endswith(b"\n"):
            data = data[:-1]
        name = filename = ctype = None
        for line in head.decode("utf-8", "replace").splitlines():
            k, _, v = line.partition(":")
            k = k.strip().lower()
            if k == "content-disposition":
                for pm in _DISP.finditer(v):
                    val = pm.group(2) if pm.group(2) is not None else pm.group(3)
                    if pm.group(1).lower() == "name":
                        name = val
                    elif pm.group(1).lower() == "filename":
                        filename = val
            elif k == "content-type":
                ctype = v.strip()
        parts.append(Part(name, filename, ctype, data))
    return parts
