"""CVE -> exploitability checklist (reference: /root/reference/community/event-driven-rag-cve-analysis/cyber_dev_day/
checklist_node.py:44-266 - a few-shot prompt that turns CVE details into a Python-list checklist, a quote-repair pass
and ``ast.literal_eval`` of the reply).

``parse_checklist`` takes the reply apart without trusting its syntax: a bracketed list (Python or JSON, with
unescaped inner quotes repaired), else a numbered / bulleted list, else one item per non-empty line.
"""
from __future__ import annotations

import ast
import json
import re
from typing import List

CHECKLIST_PROMPT = (
    "You are a security analyst. Given the details of one CVE, write the checklist an analyst follows to decide "
    "whether a specific container image is exploitable. Each item starts with an action verb and names concrete "
    "things to verify: whether the affected package is present, whether its version is in the vulnerable range, "
    "whether dependent components are in their vulnerable ranges, whether the vulnerable function or configuration "
    "is used, and whether any mitigating condition the CVE mentions is in place. Only include checks that follow "
    "from the CVE details.\n"
    "Example CVE: a path traversal in the web framework 'fastweb' before 2.4.1 when serving static routes with "
    "symlink following enabled; setting follow_symlinks=False mitigates it.\n"
    'Example checklist: ["Check for fastweb: confirm whether the image installs the fastweb package; if not, it is '
    'not affected.", "Check the fastweb version: versions before 2.4.1 are vulnerable.", "Review static routes: '
    'check whether static file routes are configured with follow_symlinks enabled (mitigated when False)."]\n'
    "Reply with the checklist only, as a Python list of strings.")

_QUOTED = re.compile(r"""(['"])((?:\\.|[^\\])*?)\1(?=\s*,|\s*\])""", re.S)
_ENUM = re.compile(r"^\s*(?:\d+[.)]|[-*•])\s+(.*\S)\s*$")


def repair_list_string(s: str) -> str:
    """Bracket a list body and escape stray quotes inside its string items."""
    s = s.strip()
    if not s.startswith("["):
        s = "[" + s
    if not s.endswith("]"):
        s = s + "]"

    def fix(m):
        q, body = m.group(1), m.group(2)
        return q + re.sub(r"(?<!\\)" + re.escape(q), "\\\\" + q, body) + q

    return _QUOTED.sub(fix, s)


def _as_items(obj) -> List[str]:
    if not isinstance(obj, list):
        return []
    out = []
    for x in obj:
        if isinstance(x, list) and len(x) == 1:
            x = x[0]
        if isinstance(x, (str, int, float)) and str(x).strip():
            out.append(str(x).strip())
    return out


def parse_checklist(text: str) -> List[str]:
    text = getattr(text, "content", text) or ""
    m = re.search(r"```(?:python|json)?\s*(.*?)```", text, re.S)
    body = m.group(1) if m else text
    start, end = body.find("["), body.rfind("]")
    if start >= 0:
        cand = body[start:end + 1] if end > start else body[start:]
        for s in (cand, repair_list_string(cand)):
            for parse in (json.loads, ast.literal_eval):
                try:
                    items = _as_items(parse(s))
                except (ValueError, SyntaxError, TypeError, MemoryError, RecursionError):
                    continue
                if items:
                    return items
    lines = [ln for ln in body.splitlines() if ln.strip()]
    enum = [m.group(1) for m in (_ENUM.match(ln) for ln in lines) if m]
    return enum or [ln.strip() for ln in lines]


def generate_checklist(cve_info: str, llm, **kw) -> List[str]:
    reply = llm.invoke([{"role": "system", "content": CHECKLIST_PROMPT},
                        {"role": "user", "content": f"CVE details:\n{cve_info}\n\nChecklist:"}],
                       temperature=kw.pop("temperature", 0.0), max_tokens=kw.pop("max_tokens", 512), **kw)
    return parse_checklist(reply)
