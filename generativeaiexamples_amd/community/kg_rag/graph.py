"""Knowledge graph of LLM-extracted triples for graph-augmented RAG (reference: /root/reference/community/
knowledge_graph_rag/backend/utils/lc_graph.py:27-199 - triples -> entities / relations / triples CSVs -> a directed
networkx graph saved as GraphML and queried with LangChain's NetworkxEntityGraph.get_entity_knowledge).

``KnowledgeGraph`` is a small directed multigraph with typed entities (no networkx in this image): entity names are
matched case- and whitespace-insensitively and keep their first spelling; ``entity_knowledge(e, depth)`` lists the
"head relation tail" facts reachable from ``e`` along out-edges within ``depth`` hops (depth-first, like
``nx.dfs_edges(G, e, depth_limit=depth)``), optionally also along in-edges. GraphML read / write interoperates with the
reference's ``knowledge_graph.graphml`` (node ids = entity names, edge attribute ``relation``, node attribute
``type``); ``to_csvs`` writes its entities / relations / triples tables.
"""
from __future__ import annotations

import csv
import os
import re
import threading
import xml.etree.ElementTree as ET
from collections import defaultdict
from typing import Dict, Iterable, List, Optional, Tuple

Triple = Tuple[str, str, str, str, str]  # (head, head_type, relation, tail, tail_type)

_GML_NS = "http://graphml.graphdrawing.org/xmlns"


def _key(name: str) -> str:
    return re.sub(r"\s+", " ", str(name)).strip().lower()


_WORD = re.compile(r"\w")


def _occurs(k: str, text: str) -> bool:
    """``k`` occurs in ``text`` with no word character on either side (the regex ``(?<!\\w)k(?!\\w)`` without
    compiling one pattern per entity)."""
    i = text.find(k)
    while i >= 0:
        j = i + len(k)
        if (i == 0 or not _WORD.match(text[i - 1])) and (j >= len(text) or not _WORD.match(text[j])):
            return True
        i = text.find(k, i + 1)
    return False


class KnowledgeGraph:
    def __init__(self):
        self.names: Dict[str, str] = {}           # key -> display name
        self.types: Dict[str, str] = {}           # key -> entity type
        self.out: Dict[str, List[Tuple[str, str]]] = defaultdict(list)  # key -> [(relation, tail key)]
        self.inc: Dict[str, List[Tuple[str, str]]] = defaultdict(list)  # key -> [(relation, head key)]
        self.edges: set = set()                   # (head key, relation, tail key): O(1) duplicate check on hubs
        self.lock = threading.Lock()
        self._first: Optional[Dict[Optional[str], List[str]]] = None  # first word -> keys (find_entities index)

    # ---- building
    def _entity(self, name: str, etype: Optional[str]) -> Optional[str]:
        k = _key(name)
        if not k or k in ("nan", "none", "null"):
            return None
        if k not in self.names:
            self.names[k] = re.sub(r"\s+", " ", str(name)).strip()
            self._first = None
        if etype and (k not in self.types or self.types[k] in ("", "Unknown")):
            self.types[k] = str(etype)
        return k

    def add_triple(self, head: str, head_type: Optional[str], relation: str, tail: str,
                   tail_type: Optional[str] = None) -> bool:
        with self.lock:
            h, t = self._entity(head, head_type), self._entity(tail, tail_type)
            rel = str(relation).strip()
            if h is None or t is None or not rel or (h, rel, t) in self.edges:
                return False
            self.edges.add((h, rel, t))
            self.out[h].append((rel, t))
            self.inc[t].append((rel, h))
            return True

    def add_triples(self, triples: Iterable) -> int:
        n = 0
        for tr in triples:
            if isinstance(tr, dict):
                tr = (tr.get("subject"), tr.get("subject_type"), tr.get("relation"), tr.get("object"),
                      tr.get("object_type"))
            if len(tr) == 3:
                tr = (tr[0], None, tr[1], tr[2], None)
            n += self.add_triple(*tr)
        return n

    def merge(self, other: "KnowledgeGraph") -> int:
        """Add every edge of ``other`` (with its entity types); returns the number of new edges."""
        n = 0
        for h, es in other.out.items():
            for r, t in es:
                n += self.add_triple(other.names[h], other.types.get(h), r, other.names[t], other.types.get(t))
        return n

    # ---- queries
    def __contains__(self, name: str) -> bool:
        return _key(name) in self.names

    def __len__(self) -> int:
        return len(self.names)

    @property
    def num_edges(self) -> int:
        return sum(len(v) for v in self.out.values())

    def triples(self) -> List[Tuple[str, str, str]]:
        return [(self.names[h], r, self.names[t]) for h, es in self.out.items() for r, t in es]

    def _first_word_index(self) -> Dict[Optional[str], List[str]]:
        idx = self._first
        if idx is None:
            idx = defaultdict(list)
            for k in list(self.names):
                m = re.match(r"\w+", k)
                idx[m.group(0) if m else None].append(k)
            self._first = idx
        return idx

    def find_entities(self, text: str) -> List[str]:
        """Entities whose name occurs in ``text`` (word-bounded, longest first). Only the names whose first word is a
        word of the text are tried (a word-bounded match starts exactly at one of the text's words), so a query costs
        O(its words), not O(entities)."""
        low = " " + _key(text) + " "
        idx = self._first_word_index()
        cands = set(idx.get(None, ()))
        for w in set(re.findall(r"\w+", low)):
            cands.update(idx.get(w, ()))
        hits = [k for k in cands if len(k) > 1 and _occurs(k, low)]
        return [self.names[k] for k in sorted(hits, key=lambda k: (-len(k), k))]

    def entity_knowledge(self, entity: str, depth: int = 2, both_directions: bool = False) -> List[str]:
        """Facts "head relation tail" within ``depth`` hops of ``entity`` (depth-first from it, each edge once)."""
        start = _key(entity)
        if start not in self.names:
            return []
        facts, seen_edges, visited = [], set(), {start}

        def visit(k: str, d: int):
            if d == 0:
                return
            nbrs = [(r, t, True) for r, t in self.out.get(k, [])]
            if both_directions:
                nbrs += [(r, h, False) for r, h in self.inc.get(k, [])]
            for r, other, forward in nbrs:
                e = (k, r, other) if forward else (other, r, k)
                if e in seen_edges:
                    continue
                seen_edges.add(e)
                facts.append(f"{self.names[e[0]]} {r} {self.names[e[2]]}")
                if other not in visited:
                    visited.add(other)
                    visit(other, d - 1)

        visit(start, depth)
        return facts

    # ---- persistence
    def write_graphml(self, path: str) -> None:
        ET.register_namespace("", _GML_NS)
        root = ET.Element(f"{{{_GML_NS}}}graphml")
        for kid, dom, name in (("d0", "node", "type"), ("d1", "edge", "relation")):
            ET.SubElement(root, f"{{{_GML_NS}}}key", {"id": kid, "for": dom, "attr.name": name, "attr.type": "string"})
        g = ET.SubElement(root, f"{{{_GML_NS}}}graph", {"edgedefault": "directed"})
        for k, name in self.names.items():
            n = ET.SubElement(g, f"{{{_GML_NS}}}node", {"id": name})
            if k in self.types:
                ET.SubElement(n, f"{{{_GML_NS}}}data", {"key": "d0"}).text = self.types[k]
        for h, es in self.out.items():
            for r, t in es:
                e = ET.SubElement(g, f"{{{_GML_NS}}}edge", {"source": self.names[h], "target": self.names[t]})
                ET.SubElement(e, f"{{{_GML_NS}}}data", {"key": "d1"}).text = r
        ET.ElementTree(root).write(path, encoding="utf-8", xml_declaration=True)

    @classmethod
    def read_graphml(cls, path: str) -> "KnowledgeGraph":
        """GraphML with node ids as entity names and a string edge attribute named ``relation`` (and optionally a node
        attribute ``type``) - the reference's knowledge_graph.graphml."""
        tree = ET.parse(path)
        root = tree.getroot()
        ns = root.tag[: root.tag.index("}") + 1] if root.tag.startswith("{") else ""
        keys = {k.get("id"): (k.get("for"), k.get("attr.name")) for k in root.iter(f"{ns}key")}
        kg = cls()
        types = {}
        for n in root.iter(f"{ns}node"):
            for d in n.iter(f"{ns}data"):
                if keys.get(d.get("key"), (None, None))[1] == "type":
                    types[n.get("id")] = d.text or ""
            kg._entity(n.get("id"), types.get(n.get("id")))
        for e in root.iter(f"{ns}edge"):
            rel = next((d.text or "" for d in e.iter(f"{ns}data")
                        if keys.get(d.get("key"), (None, None))[1] == "relation"), "related_to")
            kg.add_triple(e.get("source"), types.get(e.get("source")), rel, e.get("target"), types.get(e.get("target")))
        return kg

    def to_csvs(self, directory: str) -> None:
        """entities.csv (entity_id, entity_name, entity_type), relations.csv (relation_id, relation_name) and
        triples.csv (entity_id_1, relation_id, entity_id_2), as the reference's save_triples_to_csvs writes."""
        os.makedirs(directory, exist_ok=True)
        ids = {k: i for i, k in enumerate(self.names)}
        rels: Dict[str, int] = {}
        for es in self.out.values():
            for r, _ in es:
                rels.setdefault(r, len(rels))
        with open(os.path.join(directory, "entities.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["entity_id", "entity_name", "entity_type"])
            for k, i in ids.items():
                w.writerow([i, self.names[k], self.types.get(k, "Unknown")])
        with open(os.path.join(directory, "relations.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["relation_id", "relation_name"])
            for r, i in rels.items():
                w.writerow([i, r])
        with open(os.path.join(directory, "triples.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["entity_id_1", "relation_id", "entity_id_2"])
            for h, es in self.out.items():
                for r, t in es:
                    w.writerow([ids[h], rels[r], ids[t]])
