"""Agent tools of the CVE triage pipeline (reference: /root/reference/community/event-driven-rag-cve-analysis/
cyber_dev_day/tools.py:25-191 and pipeline_utils.py:43-112): the container's software bill of materials (SBOM)
lookup, version-range comparison (PEP 440, then Debian ordering, then string order) and a code-search tool over the
container's source indexed in an HBM collection.

``debian_compare`` implements dpkg's ordering itself (epoch, upstream, revision; '~' sorts before everything, letters
before other characters, digit runs numerically) - the reference imports a third-party package for it.
"""
from __future__ import annotations

import re
from typing import Callable, Dict, List, Optional, Union

from packaging.version import InvalidVersion, Version

_DEB = re.compile(r"^(?:(\d+):)?([0-9][A-Za-z0-9.+~:-]*?)(?:-([A-Za-z0-9.+~]+))?$")


def _order(c: str) -> int:
    if c == "~":
        return -1
    if c.isalpha():
        return ord(c)
    return ord(c) + 256


def _cmp_part(a: str, b: str) -> int:
    i = j = 0
    while i < len(a) or j < len(b):
        # non-digit prefix, compared character by character ("end" sorts after '~' and before anything else)
        while (i < len(a) and not a[i].isdigit()) or (j < len(b) and not b[j].isdigit()):
            ca = _order(a[i]) if i < len(a) and not a[i].isdigit() else 0
            cb = _order(b[j]) if j < len(b) and not b[j].isdigit() else 0
            if ca != cb:
                return -1 if ca < cb else 1
            i += i < len(a) and not a[i].isdigit()
            j += j < len(b) and not b[j].isdigit()
        da = re.match(r"\d*", a[i:]).group(0)
        db = re.match(r"\d*", b[j:]).group(0)
        i, j = i + len(da), j + len(db)
        na, nb = int(da or 0), int(db or 0)
        if na != nb:
            return -1 if na < nb else 1
    return 0


class DebianVersionError(ValueError):
    pass


def _parse_deb(v: str):
    m = _DEB.match(str(v).strip())
    if not m:
        raise DebianVersionError(f"not a Debian version: {v!r}")
    return int(m.group(1) or 0), m.group(2), m.group(3) or "0"


def debian_compare(a: str, b: str) -> int:
    """-1 / 0 / 1 as dpkg --compare-versions orders ``a`` and ``b``."""
    ea, ua, ra = _parse_deb(a)
    eb, ub, rb = _parse_deb(b)
    if ea != eb:
        return -1 if ea < eb else 1
    return _cmp_part(ua, ub) or _cmp_part(ra, rb)


def _compare(a: str, b: str) -> int:
    try:
        va, vb = Version(str(a)), Version(str(b))
        return (va > vb) - (va < vb)
    except InvalidVersion:
        pass
    try:
        return debian_compare(a, b)
    except DebianVersionError:
        sa, sb = str(a), str(b)
        return (sa > sb) - (sa < sb)


def in_range(version: str, lower: str, upper: str) -> bool:
    """lower <= version <= upper."""
    return _compare(version, lower) >= 0 and _compare(version, upper) <= 0


def at_most(version: str, vulnerable: str) -> bool:
    return _compare(version, vulnerable) <= 0


def version_comparison(spec: str) -> Union[bool, str]:
    """``"have,vuln"`` -> have <= vuln; ``"have,lo,hi"`` -> lo <= have <= hi; ``"have,v1,v2,v3,..."`` -> have is one
    of the listed versions (the reference's tool contract)."""
    v = [x.strip() for x in str(spec).split(",")]
    if len(v) == 2:
        return at_most(v[0], v[1])
    if len(v) == 3:
        return in_range(v[0], v[1], v[2])
    if len(v) > 3:
        return any(v[0] == x for x in v[1:])
    return "Could not compare versions: give the installed version and the vulnerable version(s), comma separated"


class SBOMChecker:
    description = ("Looks a package up in the container's software bill of materials. Input: the package name "
                   "only. Returns the installed version, or says the package is not present.")

    def __init__(self, sbom: Dict[str, str]):
        self.sbom = {str(k).lower().strip(): str(v) for k, v in sbom.items()}

    def __call__(self, package: str) -> str:
        words = str(package).strip().strip("'\"`").split()
        if not words:
            return "Give a package name."
        if len(words) > 1:
            return (f"Input must be the package name only; drop {' '.join(words[1:])!r} and call again with "
                    f"{words[0]!r}.")
        name = words[0].lower()
        return self.sbom.get(name, f"The package '{name}' was not found in the SBOM")

    @classmethod
    def from_csv(cls, path: str, package_col: str = "package", version_col: str = "version") -> "SBOMChecker":
        import csv

        with open(path, newline="") as f:
            return cls({r[package_col]: r[version_col] for r in csv.DictReader(f)})


class CodeSearch:
    """Retriever tool over the container's source code (a chain-server VectorStore of code chunks)."""
    description = ("Searches the container's source code. Input: a question about the code, or a code snippet such "
                   "as an import or a function call. Returns the most relevant source excerpts.")

    def __init__(self, store, k: int = 4, max_chars: int = 1200):
        self.store, self.k, self.max_chars = store, k, max_chars

    def __call__(self, query: str) -> str:
        if self.store is None or len(self.store) == 0:
            return "No source code is indexed."
        hits = self.store.similarity_search_with_relevance_scores(str(query), self.k)
        parts = [f"[{d.metadata.get('source', d.metadata.get('filename', '?'))}]\n{d.page_content[:self.max_chars]}"
                 for d, _ in hits]
        return "\n\n".join(parts) or "No matching code."


class Tool:
    def __init__(self, name: str, fn: Callable[[str], object], description: str):
        self.name, self.fn, self.description = name, fn, description

    def __call__(self, arg: str) -> str:
        try:
            return str(self.fn(arg))
        except Exception as e:  # noqa: BLE001 - tool errors go back to the agent as observations
            return f"Tool error: {e}"


def default_tools(sbom: Optional[SBOMChecker] = None, code: Optional[CodeSearch] = None) -> List[Tool]:
    tools = [Tool("Version Comparator", version_comparison,
                  "Compares versions. Input: 'installed,vulnerable' (true if installed <= vulnerable), "
                  "'installed,lower,upper' (true if inside the range) or 'installed,v1,v2,...' (true if listed).")]
    if sbom is not None:
        tools.append(Tool("SBOM Package Checker", sbom, SBOMChecker.description))
    if code is not None:
        tools.append(Tool("Container Code Search", code, CodeSearch.description))
    return tools
