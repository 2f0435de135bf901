"""HTML sanitisation of user text (the behaviour of ``bleach.clean(value, strip=True)`` with bleach's
default allow-list, which the reference applies to every request field; bleach is not available).

Allowed tags keep their markup; every other tag is stripped; bare ``<``, ``>`` and ``&`` that are
not part of allowed markup or an existing entity are escaped; comments are dropped.
"""
from __future__ import annotations

import re

ALLOWED = {"a", "abbr", "acronym", "b", "blockquote", "code", "em", "i", "li", "ol", "strong", "ul"}
_TAG = re.compile(r"<(/?)([a-zA-Z][a-zA-Z0-9]*)([^<>]*)>")
_COMMENT = re.compile(r"<!--.*?-->", re.S)
_ENTITY = re.compile(r"&(#\d+|#x[0-9a-fA-F]+|[a-zA-Z][a-zA-Z0-9]*);")


def _escape_text(s: str) -> str:
    out, last = [], 0
    for m in _ENTITY.finditer(s):
        out.append(s[last:m.start()].replace("&", "&amp;"))
        out.append(m.group(0))
        last = m.end()
    out.append(s[last:].replace("&", "&amp;"))
    return "".join(out).replace("<", "&lt;").replace(">", "&gt;")


def clean(value: str) -> str:
    if not isinstance(value, str):
        value = str(value)
    value = _COMMENT.sub("", value)
    out, last = [], 0
    for m in _TAG.finditer(value):
        out.append(_escape_text(value[last:m.start()]))
        if m.group(2).lower() in ALLOWED:
            attrs = ""
            if m.group(2).lower() in ("a", "abbr", "acronym") and m.group(1) == "":
                keep = re.findall(r'\s(href|title)\s*=\s*("[^"]*"|\'[^\']*\')', m.group(3))
                attrs = "".join(f' {k}="{v.strip(chr(34)).strip(chr(39))}"' for k, v in keep)
            out.append(f"<{m.group(1)}{m.group(2).lower()}{attrs}>")
        last = m.end()
    out.append(_escape_text(value[last:]))
    return "".join(out)
