"""Constrained (guided) decoding: JSON-schema / JSON-object / tool-call grammars.

The reference's agent notebooks depend on the OpenAI structured-output contract:
``llm.with_structured_output(Schema)`` and ``llm.bind_tools(tools, tool_choice=...)``
(RAG/notebooks/langchain/Agent_use_tools_leveraging_NVIDIA_AI_endpoints.ipynb:271-272,325-326,
agentic_rag_with_nemo_retriever_nim.ipynb:278,346,395). Prompting alone does not guarantee valid
output; here the generator is *forced*:

* :func:`compile_schema` lowers a JSON schema (object / array / string / number / integer / boolean /
  null / enum / const / anyOf / oneOf / $ref to $defs, nullable ``type`` lists) into a node table;
* ``_rt.Grammar`` (csrc/runtime/grammar.cpp) builds the vocabulary byte trie once per (schema,
  tokenizer); each request gets a ``_rt.Matcher`` that walks its output byte by byte;
* every decode step the engine asks the matcher for the allowed-token bitmask (budget-aware: a token is
  allowed only if the shortest completion still fits in the tokens left, so outputs always close) and
  the ``token_mask`` HIP kernel writes -inf into the logits of every other token before sampling.

Object properties are generated in declared order (required ones mandatory); whitespace is limited to
one optional space after ':' and ','. Tool calls use the Llama-3.1 JSON form the API layer parses,
``{"name": <tool>, "parameters": {...}}``, with the parameters schema selected by the name (tagged
union).
"""
from __future__ import annotations

import json
import threading
from collections import OrderedDict
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

# node kinds (grammar.h GNodeKind)
ANY, OBJECT, ARRAY, STRING, NUMBER, INTEGER, BOOLEAN, NULL, ENUM, ANYOF, OBJECT_ANY = range(11)

DEFAULT_MAX_STRING = 256
_KIND_OF_TYPE = {"string": STRING, "number": NUMBER, "integer": INTEGER, "boolean": BOOLEAN, "null": NULL}


class SchemaError(ValueError):
    pass


def _lit(v: Any) -> str:
    return json.dumps(v, ensure_ascii=False, separators=(",", ":"))


class _Compiler:
    def __init__(self, root_schema: dict, max_string: int):
        self.nodes: List[dict] = []
        self.root_schema = root_schema
        self.defs = dict(root_schema.get("$defs", {}))
        self.defs.update(root_schema.get("definitions", {}))
        self.max_string = max_string
        self.ref_nodes: Dict[str, int] = {}

    def add(self, d: dict) -> int:
        self.nodes.append(d)
        return len(self.nodes) - 1

    def compile(self, s: Any, depth: int = 0) -> int:
        if depth > 32:
            raise SchemaError("schema nests too deeply")
        if s is True or s == {} or s is None:
            return self.add({"kind": ANY})
        if not isinstance(s, dict):
            raise SchemaError(f"unsupported schema: {s!r}")
        if "$ref" in s:
            ref = s["$ref"]
            if ref in self.ref_nodes:
                return self.ref_nodes[ref]
            name = ref.split("/")[-1]
            if ref == "#":
                target = self.root_schema
            elif name in self.defs:
                target = self.defs[name]
            else:
                raise SchemaError(f"unresolved $ref {ref}")
            idx = self.add({"kind": ANY})  # placeholder for recursion
            self.ref_nodes[ref] = idx
            real = self.compile(target, depth + 1)
            self.nodes[idx] = dict(self.nodes[real])
            return idx
        if "const" in s:
            return self.add({"kind": ENUM, "lits": [_lit(s["const"])]})
        if "enum" in s:
            lits = [_lit(v) for v in s["enum"]]
            if not lits:
                raise SchemaError("empty enum")
            return self.add({"kind": ENUM, "lits": lits[:64]})
        for key in ("anyOf", "oneOf"):
            if key in s:
                alts = [self.compile(a, depth + 1) for a in s[key]]
                return self._anyof(alts)
        if "allOf" in s and len(s["allOf"]) == 1:
            return self.compile(s["allOf"][0], depth + 1)
        t = s.get("type")
        if isinstance(t, list):
            alts = [self.compile({**s, "type": x}, depth + 1) for x in t]
            return self._anyof(alts)
        if t is None:
            t = "object" if "properties" in s else "array" if "items" in s else None
        if t is None:
            return self.add({"kind": ANY})
        if t == "object":
            props = s.get("properties") or {}
            if not props:
                return self.add({"kind": OBJECT_ANY})
            req = set(s.get("required", []))
            keys = list(props)[:64]
            kids = [self.compile(props[k], depth + 1) for k in keys]
            return self.add({"kind": OBJECT, "keys": [_lit(k) for k in keys], "props": kids,
                             "required": [k in req for k in keys]})
        if t == "array":
            item = self.compile(s.get("items", True), depth + 1)
            d = {"kind": ARRAY, "item": item, "min_items": int(s.get("minItems", 0))}
            if "maxItems" in s:
                d["max_items"] = int(s["maxItems"])
            return self.add(d)
        if t == "string":
            return self.add({"kind": STRING, "min_len": int(s.get("minLength", 0)),
                             "max_len": int(s.get("maxLength", self.max_string))})
        if t in _KIND_OF_TYPE:
            return self.add({"kind": _KIND_OF_TYPE[t]})
        raise SchemaError(f"unsupported type {t!r}")

    def _anyof(self, alts: List[int]) -> int:
        if len(alts) == 1:
            return alts[0]
        return self.add({"kind": ANYOF, "alts": alts})


def compile_schema(schema: Any, max_string: int = DEFAULT_MAX_STRING):
    """JSON schema -> (nodes, root) for ``_rt.Grammar``."""
    c = _Compiler(schema if isinstance(schema, dict) else {}, max_string)
    root = c.compile(schema)
    return c.nodes, root


def compile_json_object():
    """OpenAI ``response_format: {"type": "json_object"}``: any JSON object."""
    return [{"kind": OBJECT_ANY}], 0


def compile_tool_call(tools: Sequence[dict], name: Optional[str] = None, max_string: int = DEFAULT_MAX_STRING):
    """``{"name": <tool>, "parameters": <that tool's arguments schema>}``; ``name`` forces one tool."""
    fns = [t.get("function", t) for t in tools if t.get("type", "function") == "function"]
    if name is not None:
        fns = [f for f in fns if f.get("name") == name]
    if not fns:
        raise SchemaError("no matching tool")
    c = _Compiler({}, max_string)
    name_node = c.add({"kind": ENUM, "lits": [_lit(f["name"]) for f in fns][:64]})
    alts = [c.compile(f.get("parameters") or {"type": "object"}) for f in fns[:64]]
    root = c.add({"kind": OBJECT, "keys": [_lit("name"), _lit("parameters")], "props": [name_node, alts[0]],
                  "required": [True, True], "disc_prop": 0, "dep_prop": 1, "dep_alts": alts})
    return c.nodes, root


# ----------------------------------------------------------------------------------------- vocab bytes
def _gpt2_byte_decoder() -> Dict[str, int]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {chr(c): b for b, c in zip(bs, cs)}


_VOCAB_CACHE: "OrderedDict[int, tuple]" = OrderedDict()
_LOCK = threading.Lock()


def vocab_bytes(tok) -> List[Optional[bytes]]:
    """Bytes each token id decodes to (None: special / unrenderable, never allowed inside the value)."""
    key = id(tok)
    with _LOCK:
        hit = _VOCAB_CACHE.get(key)
        if hit is not None and hit[0] is tok:
            return hit[1]
    V = int(getattr(tok, "vocab_size", 0))
    out: List[Optional[bytes]] = [None] * V
    if hasattr(tok, "offset") and hasattr(tok, "inv_special"):  # ByteTokenizer: ids offset..offset+255
        for b in range(256):
            if tok.offset + b < V:
                out[tok.offset + b] = bytes([b])
    elif hasattr(tok, "tk"):  # HF tokenizers
        tk = tok.tk
        V = max(V, tk.get_vocab_size(with_added_tokens=True))
        out = [None] * V
        dec = _gpt2_byte_decoder()
        special = set()
        try:
            special = {t.content for t in tk.get_added_tokens_decoder().values() if t.special}
        except Exception:  # older tokenizers
            pass
        for s, i in tk.get_vocab(with_added_tokens=True).items():
            if i >= V or s in special:
                continue
            if s.startswith("<0x") and s.endswith(">") and len(s) == 6:  # sentencepiece byte fallback
                out[i] = bytes([int(s[3:5], 16)])
            elif all(ch in dec for ch in s):  # byte-level BPE (GPT-2 / Llama-3)
                out[i] = bytes(dec[ch] for ch in s)
            else:  # sentencepiece pieces
                out[i] = s.replace("▁", " ").encode("utf-8")
    else:
        for i in range(V):
            try:
                b = tok.decode_bytes([i])
            except Exception:
                b = b""
            out[i] = b or None
    with _LOCK:
        _VOCAB_CACHE[key] = (tok, out)
        while len(_VOCAB_CACHE) > 8:
            _VOCAB_CACHE.popitem(last=False)
    return out


# ----------------------------------------------------------------------------------------- guide
class Guide:
    """A compiled grammar bound to one tokenizer; ``SamplingParams.guided`` holds one. Requests get
    their own :meth:`matcher`."""

    _cache: "OrderedDict[tuple, Guide]" = OrderedDict()

    def __init__(self, nodes, root, tok, kind: str, spec: Any = None):
        from .. import _rt

        eos = [int(e) for e in getattr(tok, "eos_ids", ())]
        self.grammar = _rt.Grammar(nodes, int(root), vocab_bytes(tok), eos)
        self.vocab_size = self.grammar.vocab_size
        self.words = (self.vocab_size + 31) // 32
        self.kind, self.spec = kind, spec

    def matcher(self):
        from .. import _rt

        return _rt.Matcher(self.grammar)

    @property
    def min_tokens(self) -> int:
        """Token budget below which a request cannot be guaranteed to close its value: the mask walk counts
        one character per remaining token, so the shortest completion needs this many tokens."""
        if not hasattr(self, "_min_tokens"):
            self._min_tokens = int(self.matcher().min_chars) + 1  # + the end-of-sequence token
        return self._min_tokens

    @classmethod
    def _get(cls, key, build):
        with _LOCK:
            g = cls._cache.get(key)
            if g is not None:
                cls._cache.move_to_end(key)
                return g
        g = build()
        with _LOCK:
            cls._cache[key] = g
            while len(cls._cache) > 64:
                cls._cache.popitem(last=False)
        return g

    @classmethod
    def json_schema(cls, schema: dict, tok) -> "Guide":
        key = ("schema", json.dumps(schema, sort_keys=True), id(tok))
        return cls._get(key, lambda: cls(*compile_schema(schema), tok, "json_schema", schema))

    @classmethod
    def json_object(cls, tok) -> "Guide":
        return cls._get(("object", id(tok)), lambda: cls(*compile_json_object(), tok, "json_object"))

    @classmethod
    def tool_call(cls, tools: Sequence[dict], tok, name: Optional[str] = None) -> "Guide":
        key = ("tool", json.dumps(list(tools), sort_keys=True), name, id(tok))
        return cls._get(key, lambda: cls(*compile_tool_call(tools, name), tok, "tool_call", name))


class MaskBuilder:
    """Per-step allowed-token masks of the guided rows of a batch (host side, int32 words)."""

    def __init__(self):
        self.buf = np.zeros((0, 0), np.uint32)

    def build(self, rows: List[int], matchers: List[Any], budgets: List[int], words: int) -> np.ndarray:
        n = len(rows)
        if self.buf.shape[0] < n or self.buf.shape[1] != words:
            self.buf = np.zeros((max(n, 8), words), np.uint32)
        for j, (m, b) in enumerate(zip(matchers, budgets)):
            m.fill_mask(max(1, int(b)), self.buf[j])
        return self.buf[:n].view(np.int32)


# ----------------------------------------------------------------------------------------- validation
def validate(value: Any, schema: Any, root: Optional[dict] = None) -> bool:
    """Minimal JSON-schema check for the subset :func:`compile_schema` supports (tests / API guard)."""
    root = root if root is not None else (schema if isinstance(schema, dict) else {})
    if schema is True or schema == {} or schema is None:
        return True
    if "$ref" in schema:
        ref = schema["$ref"]
        if ref == "#":
            return validate(value, root, root)
        name = ref.split("/")[-1]
        defs = {**root.get("definitions", {}), **root.get("$defs", {})}
        return validate(value, defs[name], root)
    if "const" in schema:
        return value == schema["const"]
    if "enum" in schema:
        return value in schema["enum"]
    for key in ("anyOf", "oneOf"):
        if key in schema:
            return any(validate(value, a, root) for a in schema[key])
    t = schema.get("type")
    if isinstance(t, list):
        return any(validate(value, {**schema, "type": x}, root) for x in t)
    if t is None:
        t = "object" if "properties" in schema else "array" if "items" in schema else None
    if t == "object":
        if not isinstance(value, dict):
            return False
        props = schema.get("properties") or {}
        if any(r not in value for r in schema.get("required", [])):
            return False
        if props and any(k not in props for k in value):
            return False
        return all(validate(v, props.get(k, True), root) for k, v in value.items())
    if t == "array":
        if not isinstance(value, list):
            return False
        if len(value) < schema.get("minItems", 0) or len(value) > schema.get("maxItems", 1 << 30):
            return False
        return all(validate(v, schema.get("items", True), root) for v in value)
    if t == "string":
        return isinstance(value, str) and schema.get("minLength", 0) <= len(value) <= schema.get("maxLength", 1 << 30)
    if t == "integer":
        return isinstance(value, int) and not isinstance(value, bool)
    if t == "number":
        return isinstance(value, (int, float)) and not isinstance(value, bool)
    if t == "boolean":
        return isinstance(value, bool)
    if t == "null":
        return value is None
    return True
