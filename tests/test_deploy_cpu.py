"""Deployment assets: compose files parse, every service command names an importable module entrypoint,
and per-example compose files point EXAMPLE_PATH at an existing example."""
import glob
import importlib
import os

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _services():
    for f in glob.glob(f"{ROOT}/deploy/compose/*.yaml") + glob.glob(f"{ROOT}/RAG/examples/**/docker-compose.yaml", recursive=True):
        doc = yaml.safe_load(open(f))
        for name, svc in (doc.get("services") or {}).items():
            yield f, name, svc


def test_compose_entrypoints_importable():
    n = 0
    for f, name, svc in _services():
        cmd = svc.get("command")
        if isinstance(cmd, list) and cmd and cmd[0].startswith("generativeaiexamples_amd"):
            spec = importlib.util.find_spec(cmd[0] + ".__main__") or importlib.util.find_spec(cmd[0])
            assert spec is not None, f"{f}:{name} -> {cmd[0]}"
            n += 1
    assert n >= 10


def test_examples_exist():
    for f, name, svc in _services():
        ex = (svc.get("environment") or {}).get("EXAMPLE_PATH")
        if ex:
            assert os.path.isfile(os.path.join(ROOT, "RAG/examples", ex, "chains.py")), ex
            assert os.path.samefile(os.path.dirname(f), os.path.join(ROOT, "RAG/examples", ex))
