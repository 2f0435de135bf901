"""Typed configuration from a JSON/YAML file overlaid with ``APP_*`` environment variables.

Behavioural parity with the reference's ConfigWizard (RAG/src/chain_server/configuration_wizard.py):
* config sections are frozen dataclasses; each field has a JSON key (camelCase) and may be
  settable from the environment;
* env var name = ``APP`` + ``_<SECTION>`` ... + ``_<FIELDKEY>`` upper-cased, e.g. the
  ``vector_store.index_type`` field with key ``indexType`` is ``APP_VECTORSTORE_INDEXTYPE``;
* precedence: value in the file > environment variable > dataclass default (env vars only fill
  keys the file does not set);
* env values are JSON-decoded when they parse as JSON (``APP_RETRIEVER_TOPK=8`` is an int);
* ``APP_CONFIG_FILE`` names the file (JSON or YAML; missing / empty -> defaults).
"""
from __future__ import annotations

import dataclasses
import json
import os
import sys
from typing import Any, Dict, Iterator, List, Optional, TextIO, Tuple, Type, TypeVar, get_type_hints

import yaml

ENV_BASE = "APP"
T = TypeVar("T")


def configclass(cls):
    """Decorator: a frozen dataclass usable as a config section."""
    return dataclasses.dataclass(frozen=True)(cls)


def configfield(name: str, *, env: bool = True, help_txt: str = "", **kw):
    """A config field. ``name`` is its JSON key and the last component of its env var name."""
    md = dict(kw.pop("metadata", {}) or {})
    md.update({"gai_key": name, "gai_env": env, "gai_help": help_txt})
    return dataclasses.field(metadata=md, **kw)


def _key(f: dataclasses.Field) -> str:
    return f.metadata.get("gai_key", f.name)


def _is_section(tp) -> bool:
    return isinstance(tp, type) and dataclasses.is_dataclass(tp)


def try_json_load(v: str) -> Any:
    try:
        return json.loads(v)
    except (json.JSONDecodeError, TypeError):
        return v


def read_json_or_yaml(stream: TextIO) -> Dict[str, Any]:
    txt = stream.read()
    if not txt.strip():
        return {}
    try:
        data = json.loads(txt)
    except json.JSONDecodeError:
        try:
            data = yaml.safe_load(txt)
        except yaml.YAMLError as e:
            raise ValueError(f"config is neither valid JSON nor YAML: {e}") from e
    if data is None:
        return {}
    if not isinstance(data, dict):
        raise ValueError("config file must contain a mapping at the top level")
    return data


class ConfigWizard:
    """Mixin for the top-level config dataclass."""

    @classmethod
    def envvars(cls, prefix: str = ENV_BASE) -> Iterator[Tuple[str, Tuple[str, ...], Any, str]]:
        """Yield (env var name, key path, field type, help) for every env-settable leaf field."""
        hints = get_type_hints(cls)
        for f in dataclasses.fields(cls):
            tp = hints[f.name]
            k = _key(f)
            name = f"{prefix}_{k.upper()}"
            if _is_section(tp):
                for sub_name, path, t2, h in tp.envvars(name) if hasattr(tp, "envvars") else ConfigWizard.envvars.__func__(tp, name):
                    yield sub_name, (k,) + path, t2, h
            elif f.metadata.get("gai_env", True):
                yield name, (k,), tp, f.metadata.get("gai_help", "")

    @classmethod
    def from_dict(cls: Type[T], data: Dict[str, Any]) -> T:
        data = json.loads(json.dumps(data or {}))  # deep copy, plain types
        for var, path, _tp, _h in ConfigWizard.envvars.__func__(cls):
            if var in os.environ:
                update_dict(data, path, try_json_load(os.environ[var]), overwrite=False)
        return _build(cls, data)

    @classmethod
    def from_file(cls: Type[T], path: Optional[str]) -> T:
        data: Dict[str, Any] = {}
        if path and os.path.isfile(path):
            with open(path) as f:
                data = read_json_or_yaml(f)
        return cls.from_dict(data)

    @classmethod
    def print_help(cls, out: TextIO = sys.stdout) -> None:
        out.write(f"Configuration for {cls.__name__}\n")
        out.write("(file value > environment variable > default)\n\n")
        for var, path, tp, h in ConfigWizard.envvars.__func__(cls):
            default = _default_at(cls, path)
            tname = getattr(tp, "__name__", str(tp))
            out.write(f"  {'.'.join(path):40s} {var:45s} {tname:8s} default={default!r}\n")
            if h:
                out.write(f"      {h}\n")


def update_dict(data: Dict[str, Any], path: Tuple[str, ...], value: Any, overwrite: bool = False) -> None:
    cur = data
    for k in path[:-1]:
        nxt = cur.get(k)
        if not isinstance(nxt, dict):
            nxt = {}
            cur[k] = nxt
        cur = nxt
    if overwrite or path[-1] not in cur:
        cur[path[-1]] = value


def _coerce(tp, v):
    if v is None:
        return None
    origin = getattr(tp, "__origin__", None)
    try:
        if tp in (int, float, str):
            return tp(v)
        if tp is bool:
            return v if isinstance(v, bool) else str(v).lower() in ("1", "true", "yes", "on")
        if origin in (list, List):
            return list(v) if isinstance(v, (list, tuple)) else [v]
    except (TypeError, ValueError):
        return v
    return v


def _build(cls, data: Dict[str, Any]):
    hints = get_type_hints(cls)
    kw = {}
    for f in dataclasses.fields(cls):
        tp = hints[f.name]
        k = _key(f)
        if _is_section(tp):
            kw[f.name] = _build(tp, data.get(k) or {})
        elif k in data:
            kw[f.name] = _coerce(tp, data[k])
    return cls(**kw)


def _default_at(cls, path):
    hints = get_type_hints(cls)
    for f in dataclasses.fields(cls):
        if _key(f) == path[0]:
            if len(path) > 1:
                return _default_at(hints[f.name], path[1:])
            if f.default is not dataclasses.MISSING:
                return f.default
            if f.default_factory is not dataclasses.MISSING:  # type: ignore[misc]
                return f.default_factory()  # type: ignore[misc]
    return None
