"""Constrained decoding: schema compiler, native matcher (csrc/runtime/grammar.cpp), token masks, engine.

Random walks pick a uniformly random *allowed* token every step (the worst case for termination: no
model preference for closing anything); every walk must end in JSON that parses and validates."""
import json
import random

import numpy as np
import pytest
import torch

from generativeaiexamples_amd.engine import guided
from generativeaiexamples_amd.engine.guided import Guide, validate
from generativeaiexamples_amd.engine.tokenizer import llama3_byte_tokenizer, small_byte_tokenizer

PERSON = {
    "type": "object",
    "properties": {
        "name": {"type": "string", "maxLength": 12},
        "age": {"type": "integer"},
        "email": {"type": ["string", "null"]},
        "tags": {"type": "array", "items": {"type": "string", "maxLength": 6}, "maxItems": 3},
        "role": {"enum": ["admin", "user", 7, None]},
        "score": {"type": "number"},
        "active": {"type": "boolean"},
    },
    "required": ["name", "age", "role"],
}
NESTED = {
    "type": "object",
    "properties": {
        "items": {"type": "array", "minItems": 1, "maxItems": 2,
                  "items": {"$ref": "#/$defs/item"}},
        "note": {"anyOf": [{"type": "string", "maxLength": 5}, {"type": "integer"}]},
    },
    "required": ["items"],
    "$defs": {"item": {"type": "object", "properties": {"id": {"type": "integer"}, "ok": {"const": True}},
                       "required": ["id", "ok"]}},
}
TOOLS = [
    {"type": "function", "function": {"name": "get_weather", "parameters": {
        "type": "object", "properties": {"city": {"type": "string", "maxLength": 10},
                                         "unit": {"enum": ["c", "f"]}}, "required": ["city", "unit"]}}},
    {"type": "function", "function": {"name": "add", "parameters": {
        "type": "object", "properties": {"a": {"type": "number"}, "b": {"type": "number"}}, "required": ["a", "b"]}}},
]


def _walk(guide, tok, budget, rng):
    m = guide.matcher()
    mask = np.zeros(guide.words, np.uint32)
    out = []
    for step in range(budget):
        m.fill_mask(budget - step, mask)
        bits = np.unpackbits(mask.view(np.uint8), bitorder="little")[: guide.vocab_size]
        allowed = np.nonzero(bits)[0]
        assert len(allowed), f"no allowed token after {tok.decode_bytes(out)!r}"
        t = int(rng.choice(allowed))
        if t in tok.eos_ids:
            break
        assert m.advance(t)
        out.append(t)
        if m.done:
            break
    return tok.decode_bytes(out).decode("utf-8", "replace"), m


@pytest.mark.parametrize("schema", [PERSON, NESTED], ids=["person", "nested"])
@pytest.mark.parametrize("budget", [120, 400])
def test_random_walks_are_valid(schema, budget):
    tok = small_byte_tokenizer(512)
    g = Guide.json_schema(schema, tok)
    rng = np.random.default_rng(budget)
    for _ in range(40):
        text, m = _walk(g, tok, budget, rng)
        v = json.loads(text)
        assert validate(v, schema), text
        assert m.done or m.can_finish


def test_tool_call_tagged_union():
    tok = llama3_byte_tokenizer()
    g = Guide.tool_call(TOOLS, tok)
    rng = np.random.default_rng(1)
    names = set()
    for _ in range(30):
        text, _ = _walk(g, tok, 200, rng)
        v = json.loads(text)
        names.add(v["name"])
        fn = next(t["function"] for t in TOOLS if t["function"]["name"] == v["name"])
        assert set(v) == {"name", "parameters"}
        assert validate(v["parameters"], fn["parameters"]), text
    assert names == {"get_weather", "add"}
    forced = Guide.tool_call(TOOLS, tok, name="add")
    text, _ = _walk(forced, tok, 200, rng)
    assert json.loads(text)["name"] == "add"


def test_json_object_mode():
    tok = small_byte_tokenizer(512)
    g = Guide.json_object(tok)
    rng = np.random.default_rng(3)
    for _ in range(40):
        text, _ = _walk(g, tok, 150, rng)
        assert isinstance(json.loads(text), dict), text


def test_matcher_accepts_and_rejects():
    tok = small_byte_tokenizer(512)
    g = Guide.json_schema(PERSON, tok)
    m = g.matcher()
    assert m.feed_bytes(b'{"name": "Ann", "age": -12, "role": "user", "active": true}')
    assert m.done
    for bad in [b'{"age": 1}', b'{"name": 5', b'{"name": "A", "age": 1.5', b'{"name": "A", "age": 1, "role": "root"',
                b'{"name": "A", "age": 1, "role": 7, "zzz"']:
        m = g.matcher()
        assert not m.feed_bytes(bad), bad
        assert m.dead
    # key order follows the schema; optional properties may be skipped
    assert g.matcher().feed_bytes(b'{"name":"x","age":0,"role":null}')


def test_budget_forces_completion():
    """With a tight budget the mask only leaves tokens whose shortest completion still fits."""
    tok = small_byte_tokenizer(512)
    schema = {"type": "object", "properties": {"s": {"type": "string"}}, "required": ["s"]}
    g = Guide.json_schema(schema, tok)
    m = g.matcher()
    assert m.feed_bytes(b'{"s": "abc')
    assert m.min_chars == 2  # '"' '}'
    mask = np.zeros(g.words, np.uint32)
    m.fill_mask(2, mask)
    bits = np.unpackbits(mask.view(np.uint8), bitorder="little")[: g.vocab_size]
    assert set(np.nonzero(bits)[0]) == {tok.encode('"')[0]}


def test_hf_style_vocab_bytes():
    class Fake:
        vocab_size = 6
        eos_ids = (5,)

        def decode_bytes(self, ids):
            return [b"{", b"}", b'"a"', b":", b"1", b""][ids[0]]

    vb = guided.vocab_bytes(Fake())
    assert vb[:5] == [b"{", b"}", b'"a"', b":", b"1"] and vb[5] is None


def test_token_mask_reference():
    from generativeaiexamples_amd import ops

    logits = torch.randn(3, 70)
    mask = torch.zeros(2, 3, dtype=torch.int32)
    mask[0, 0] = 0b101
    mask[1, 2] = 1 << 3  # token 67
    ops.token_mask(logits, torch.tensor([2, 0], dtype=torch.int32), mask)
    assert torch.isfinite(logits[2]).tolist() == [i in (0, 2) for i in range(70)]
    assert torch.isfinite(logits[0]).tolist() == [i == 67 for i in range(70)]
    assert torch.isfinite(logits[1]).all()


def test_engine_guided_generation_cpu():
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel

    torch.manual_seed(0)
    tok = small_byte_tokenizer(512)
    model = LlamaModel(LlamaConfig.tiny(), device=torch.device("cpu"), dtype=torch.float32).random_init(0)
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=4, num_blocks=128, max_model_len=512, use_graphs=False))
    g = Guide.json_schema(PERSON, tok)
    prompts = [tok.encode(f"person {i}:") for i in range(3)]
    ps = [SamplingParams(temperature=1.0, top_p=1.0, max_tokens=m, guided=g, seed=i) for i, m in
          enumerate((60, 90, 150))]
    reqs = eng.generate(prompts, ps)
    for r in reqs:
        v = json.loads(r.text)
        assert validate(v, PERSON), r.text
        assert r.finish_reason == "stop"
    # unguided request in the same engine is unaffected
    r = eng.generate([tok.encode("x")], SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True))[0]
    assert len(r.output_ids) == 5


def test_engine_guided_exhausted_budget_ends_with_length():
    """Engine-level (no API admission check): once the grammar allows no token within the remaining budget
    the request ends with finish_reason 'length' instead of sampling from an all -inf row."""
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel

    tok = small_byte_tokenizer(512)
    model = LlamaModel(LlamaConfig.tiny(), device=torch.device("cpu"), dtype=torch.float32).random_init(0)
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=2, num_blocks=64, max_model_len=256, use_graphs=False))
    g = Guide.json_schema(PERSON, tok)
    assert g.min_tokens > 3
    r = eng.generate([tok.encode("p:")], SamplingParams(temperature=1.0, max_tokens=3, guided=g, seed=1))[0]
    assert r.finished and r.finish_reason == "length"
    assert eng.sched.num_free_blocks() == eng.sched.num_blocks()
