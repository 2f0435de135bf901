"""NIM / OpenAI-compatible ``/v1`` API on the in-process MI355X engines.

What the reference's clients call (ChatNVIDIA / NVIDIAEmbeddings / NVIDIARerank with
``base_url=http://host:8000/v1``, the OpenAI SDK, curl in the notebooks):

* ``POST /v1/chat/completions`` - stream (SSE ``data:`` ... ``data: [DONE]``) and non-stream,
  temperature / top_p / max_tokens / stop / seed / frequency & presence penalties, ``tools`` +
  ``tool_choice`` (tool calls parsed from the model's JSON answer), ``response_format``.
* ``POST /v1/completions`` - raw prompt completion.
* ``POST /v1/embeddings`` - ``input_type`` query|passage, ``truncate`` NONE|START|END, float or
  base64 encoding.
* ``POST /v1/ranking`` (and the hosted alias ``/v1/retrieval/nvidia/reranking``) -
  ``{"query":{"text"},"passages":[{"text"}]}`` -> ``{"rankings":[{"index","logit"}]}``.
* ``GET /v1/models``, ``GET /v1/health/ready``, ``GET /v1/health/live``, ``GET /metrics``.
"""
from __future__ import annotations

import asyncio
import base64
import json
import re
import struct
import time
import uuid
from typing import Any, Dict, List, Optional, Union

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, Response, StreamingResponse
from pydantic import BaseModel, Field
from starlette.concurrency import run_in_threadpool

from ..engine.sampling import SamplingParams
from ..engine.tokenizer import apply_chat_template, image_token_of
from ..utils.metrics import METRICS
from .hub import ServiceHub


# ------------------------------------------------------------------------------------ schemas
class ChatMessage(BaseModel):
    role: str
    content: Optional[Union[str, List[Dict[str, Any]]]] = None
    name: Optional[str] = None
    tool_calls: Optional[List[Dict[str, Any]]] = None
    tool_call_id: Optional[str] = None


class ChatRequest(BaseModel):
    model: Optional[str] = None
    messages: List[ChatMessage]
    temperature: Optional[float] = Field(None, ge=0.0, le=2.0)
    top_p: Optional[float] = Field(None, gt=0.0, le=1.0)
    top_k: Optional[int] = None
    max_tokens: Optional[int] = Field(None, ge=1)
    max_completion_tokens: Optional[int] = Field(None, ge=1)
    stop: Optional[Union[str, List[str]]] = None
    stream: bool = False
    seed: Optional[int] = None
    n: int = 1
    frequency_penalty: float = 0.0
    presence_penalty: float = 0.0
    repetition_penalty: float = 1.0
    tools: Optional[List[Dict[str, Any]]] = None
    tool_choice: Optional[Union[str, Dict[str, Any]]] = None
    response_format: Optional[Dict[str, Any]] = None
    stream_options: Optional[Dict[str, Any]] = None
    ignore_eos: bool = False
    min_tokens: int = 0
    # NIM / vLLM structured-generation extensions: {"guided_json": <schema>}
    nvext: Optional[Dict[str, Any]] = None
    guided_json: Optional[Union[Dict[str, Any], str]] = None


class CompletionRequest(BaseModel):
    model: Optional[str] = None
    prompt: Union[str, List[str], List[int]]
    temperature: Optional[float] = Field(None, ge=0.0, le=2.0)
    top_p: Optional[float] = Field(None, gt=0.0, le=1.0)
    max_tokens: Optional[int] = Field(16, ge=1)
    stop: Optional[Union[str, List[str]]] = None
    stream: bool = False
    seed: Optional[int] = None
    echo: bool = False
    frequency_penalty: float = 0.0
    presence_penalty: float = 0.0
    ignore_eos: bool = False


class EmbeddingRequest(BaseModel):
    model: Optional[str] = None
    input: Union[str, List[str]]
    input_type: Optional[str] = "query"
    truncate: Optional[str] = "NONE"
    encoding_format: Optional[str] = "float"
    dimensions: Optional[int] = None
    user: Optional[str] = None


class RankingText(BaseModel):
    text: str


class RankingRequest(BaseModel):
    model: Optional[str] = None
    query: RankingText
    passages: List[RankingText]
    truncate: Optional[str] = "END"
    top_n: Optional[int] = None


# ------------------------------------------------------------------------------------ helpers
def _err(status: int, msg: str, typ: str = "invalid_request_error"):
    return JSONResponse(status_code=status, content={"error": {"message": msg, "type": typ, "code": status},
                                                     "object": "error", "message": msg})


def _stops(stop) -> List[str]:
    if stop is None:
        return []
    return [stop] if isinstance(stop, str) else list(stop)


def _params(req, default_max: int) -> SamplingParams:
    mt = getattr(req, "max_completion_tokens", None) or req.max_tokens or default_max
    return SamplingParams(
        temperature=1.0 if req.temperature is None else req.temperature,
        top_p=1.0 if req.top_p is None else req.top_p,
        top_k=getattr(req, "top_k", None) or 0,
        max_tokens=mt, stop=_stops(req.stop), seed=req.seed,
        frequency_penalty=req.frequency_penalty, presence_penalty=req.presence_penalty,
        repetition_penalty=getattr(req, "repetition_penalty", 1.0), ignore_eos=getattr(req, "ignore_eos", False),
        min_tokens=getattr(req, "min_tokens", 0))


def _tool_system_prompt(tools: List[Dict[str, Any]], choice) -> str:
    """Llama-3.1-style JSON function-calling instructions."""
    fns = [t.get("function", t) for t in tools if t.get("type", "function") == "function"]
    forced = ""
    if isinstance(choice, dict):
        forced = f" You MUST call the function `{choice.get('function', {}).get('name')}`."
    elif choice == "required":
        forced = " You MUST call one of the functions."
    return ("You have access to the following functions. To call a function, respond ONLY with a JSON object "
            'of the form {"name": <function name>, "parameters": <arguments object>}. If no function is '
            "needed, answer normally." + forced + "\n\n" + "\n".join(json.dumps(f) for f in fns))


_JSON_OBJ = re.compile(r"\{.*\}", re.S)


def parse_tool_calls(text: str, tools: List[Dict[str, Any]]) -> Optional[List[Dict[str, Any]]]:
    names = {t.get("function", t).get("name") for t in tools}
    cand = text.strip()
    if cand.startswith("<|python_tag|>"):
        cand = cand[len("<|python_tag|>"):]
    m = _JSON_OBJ.search(cand)
    if not m:
        return None
    # one JSON object, or several separated by ';' (Llama 3.1 style): decoded one after another, so a ';' inside
    # an argument string is data, not a separator
    objs, dec, i = [], json.JSONDecoder(), m.start()
    while i < len(cand) and cand[i] == "{":  # text after the last call is ignored
        try:
            o, i = dec.raw_decode(cand, i)
        except json.JSONDecodeError:
            return None
        objs.append(o)
        while i < len(cand) and (cand[i].isspace() or cand[i] == ";"):
            i += 1
    calls = []
    for o in objs:
        if not isinstance(o, dict):
            return None
        name = o.get("name")
        args = o.get("parameters", o.get("arguments", {}))
        if name not in names:
            return None
        calls.append({"id": f"call_{uuid.uuid4().hex[:24]}", "type": "function",
                      "function": {"name": name, "arguments": json.dumps(args)}})
    return calls or None


def guide_for(req, tok):
    """Constrained-decoding grammar a chat request asks for (engine/guided.py), or None:
    ``tool_choice: "required"`` / ``{"type": "function", "function": {"name": ...}}`` -> a tool-call
    object whose parameters follow the chosen tool's schema; ``response_format`` json_schema /
    json_object; ``guided_json`` (top level or under ``nvext``). ``tool_choice: "auto"`` stays free."""
    from ..engine.guided import Guide

    tools = getattr(req, "tools", None)
    choice = getattr(req, "tool_choice", None)
    if tools and choice not in (None, "auto", "none"):
        name = None
        if isinstance(choice, dict):
            name = (choice.get("function") or {}).get("name")
            if name is None:
                raise ValueError("tool_choice object needs function.name")
        elif choice != "required":
            raise ValueError(f"unsupported tool_choice {choice!r}")
        return Guide.tool_call(tools, tok, name)
    gj = getattr(req, "guided_json", None) or ((getattr(req, "nvext", None) or {}).get("guided_json"))
    if gj is not None:
        return Guide.json_schema(json.loads(gj) if isinstance(gj, str) else gj, tok)
    rf = getattr(req, "response_format", None) or {}
    if rf.get("type") == "json_schema":
        js = rf.get("json_schema") or {}
        schema = js.get("schema", js if "type" in js or "properties" in js else None)
        return Guide.json_schema(schema, tok) if schema else Guide.json_object(tok)
    if rf.get("type") == "json_object":
        return Guide.json_object(tok)
    return None


def _images_of(req: ChatRequest) -> List[str]:
    """OpenAI/NIM vision content parts: {"type": "image_url", "image_url": {"url": "data:image/...;base64,..."}}
    (W12 image_url chat); also accepts a bare string url field."""
    out = []
    for m in req.messages:
        if isinstance(m.content, list):
            for p in m.content:
                if p.get("type") == "image_url":
                    u = p.get("image_url")
                    out.append(u.get("url") if isinstance(u, dict) else u)
    return out


def _messages_for_template(req: ChatRequest) -> List[dict]:
    msgs = []
    for m in req.messages:
        content = m.content
        if isinstance(content, list):  # text parts joined; image parts kept as markers for the image token
            imgs = [{"type": "image"} for p in content if p.get("type") in ("image_url", "image")]
            text = "".join(p.get("text", "") for p in content if p.get("type") in ("text", None))
            content = imgs + [{"type": "text", "text": text}] if imgs else text
        if m.role == "tool":
            msgs.append({"role": "ipython", "content": content or ""})
        elif m.tool_calls:
            msgs.append({"role": "assistant", "content": json.dumps(
                [{"name": c["function"]["name"], "parameters": json.loads(c["function"].get("arguments") or "{}")}
                 for c in m.tool_calls])})
        else:
            msgs.append({"role": m.role, "content": content or ""})
    if req.tools and req.tool_choice != "none":
        sys_txt = _tool_system_prompt(req.tools, req.tool_choice)
        if msgs and msgs[0]["role"] == "system":
            msgs[0] = {"role": "system", "content": msgs[0]["content"] + "\n\n" + sys_txt}
        else:
            msgs.insert(0, {"role": "system", "content": sys_txt})
    if req.response_format and req.response_format.get("type") in ("json_object", "json_schema"):
        schema = req.response_format.get("json_schema", {}).get("schema")
        hint = "Respond only with a valid JSON object" + (f" matching this JSON schema: {json.dumps(schema)}" if schema else ".")
        msgs.insert(0, {"role": "system", "content": hint})
    return msgs


def _embedding_payload(vecs, fmt: str):
    out = []
    for i, v in enumerate(vecs):
        if fmt == "base64":
            emb = base64.b64encode(struct.pack(f"<{len(v)}f", *v)).decode()
        else:
            emb = v
        out.append({"object": "embedding", "index": i, "embedding": emb})
    return out


# ------------------------------------------------------------------------------------ app
def create_openai_app(hub: ServiceHub) -> FastAPI:
    app = FastAPI(title="generativeaiexamples_amd NIM-compatible API", version="1.0")
    app.state.hub = hub

    @app.middleware("http")
    async def count(request: Request, call_next):
        METRICS.api_requests.labels(request.url.path).inc()
        return await call_next(request)

    @app.get("/v1/health/ready")
    async def ready():
        if not hub.ready():
            return JSONResponse(status_code=503, content={"object": "health.response", "message": "Service is not ready."})
        return {"object": "health.response", "message": "Service is ready."}

    @app.get("/v1/health/live")
    async def live():
        return {"object": "health.response", "message": "Service is live."}

    @app.get("/health")
    async def health():
        return {"message": "Service is up."}

    @app.get("/metrics")
    async def metrics():
        hub.update_gauges()
        return Response(METRICS.render(), media_type="text/plain; version=0.0.4")

    @app.get("/v1/models")
    async def models():
        now = int(time.time())
        data = [{"id": m, "object": "model", "created": now, "owned_by": "generativeaiexamples_amd", "root": root,
                 "parent": None if root == m else root, "max_model_len": hub.max_model_len(m)}
                for m, root in hub.model_list()]
        return {"object": "list", "data": data}

    # ---------------------------------------------------------------- chat
    @app.post("/v1/chat/completions")
    async def chat(req: ChatRequest):
        llm = hub.llm(req.model)
        if llm is None:
            return _err(404, f"model '{req.model}' is not served here")
        if req.n != 1:
            return _err(400, "only n=1 is supported")
        tok = llm.tokenizer
        ids = apply_chat_template(_messages_for_template(req), tok, image_token_id=image_token_of(llm.engine.model))
        params = _params(req, hub.default_max_tokens)
        try:
            params.guided = guide_for(req, tok)
        except (ValueError, KeyError) as e:  # SchemaError is a ValueError
            return _err(400, f"structured output: {e}")
        if params.guided is not None and params.max_tokens < params.guided.min_tokens:
            return _err(400, f"structured output: max_tokens={params.max_tokens} cannot hold the shortest valid "
                             f"output ({params.guided.min_tokens} tokens)")
        # elastic re-queue (serving/router.py): the router asks for token ids in the stream and resumes a
        # completion a failed replica started by sending the ids it already delivered
        nv = req.nvext or {}
        want_ids = bool(nv.get("return_token_ids"))
        resume = [int(t) for t in nv.get("resume_token_ids") or []]
        if resume:
            params.max_tokens = max(0, params.max_tokens - len(resume))
            params.min_tokens = max(0, params.min_tokens - len(resume))
            params.resume_ids, params.resume_sent_chars = resume, nv.get("resume_text_chars")
        images = _images_of(req) or None
        lora = hub.lora_for(req.model)
        if images and not hasattr(llm.engine.model, "register_request"):
            return _err(400, f"model '{req.model or hub.default_llm_name}' does not accept image inputs")
        rid = f"chatcmpl-{uuid.uuid4().hex}"
        created = int(time.time())
        model = req.model or hub.default_llm_name
        use_tools = bool(req.tools) and req.tool_choice != "none"
        if req.stream and not use_tools:
            include_usage = bool(req.stream_options and req.stream_options.get("include_usage"))

            async def gen():
                head = {"id": rid, "object": "chat.completion.chunk", "created": created, "model": model,
                        "choices": [{"index": 0, "delta": {"role": "assistant", "content": ""}, "logprobs": None,
                                     "finish_reason": None}]}
                yield f"data: {json.dumps(head)}\n\n"
                n = 0
                try:
                    async for it in llm.generate(ids, params, rid, images, lora):
                        n += it.token_id >= 0
                        ch = {"id": rid, "object": "chat.completion.chunk", "created": created, "model": model,
                              "choices": [{"index": 0, "delta": {"content": it.delta} if it.delta else {},
                                           "logprobs": None, "finish_reason": it.finish_reason if it.finished else None}]}
                        if want_ids and it.token_id >= 0:
                            ch["nvext"] = {"token_ids": [it.token_id]}
                        if it.delta or it.finished or "nvext" in ch:
                            yield f"data: {json.dumps(ch)}\n\n"
                except Exception as e:  # report in-band, SSE cannot change status mid-stream
                    yield f"data: {json.dumps({'error': {'message': str(e)}})}\n\n"
                if include_usage:
                    u = {"id": rid, "object": "chat.completion.chunk", "created": created, "model": model,
                         "choices": [], "usage": {"prompt_tokens": len(ids), "completion_tokens": n,
                                                  "total_tokens": len(ids) + n}}
                    yield f"data: {json.dumps(u)}\n\n"
                yield "data: [DONE]\n\n"

            return StreamingResponse(gen(), media_type="text/event-stream")

        text, out_ids, reason = await llm.complete(ids, params, rid, images, lora)
        msg: Dict[str, Any] = {"role": "assistant", "content": text}
        if use_tools:
            calls = parse_tool_calls(text, req.tools)
            if calls:
                msg = {"role": "assistant", "content": None, "tool_calls": calls}
                reason = "tool_calls"
        body = {"id": rid, "object": "chat.completion", "created": created, "model": model,
                "choices": [{"index": 0, "message": msg, "logprobs": None, "finish_reason": reason}],
                "usage": {"prompt_tokens": len(ids), "completion_tokens": len(out_ids),
                          "total_tokens": len(ids) + len(out_ids)}}
        if req.stream:  # tools + stream: emit the finished message as one chunk
            async def one():
                ch = dict(body, object="chat.completion.chunk")
                ch["choices"] = [{"index": 0, "delta": msg, "finish_reason": reason}]
                yield f"data: {json.dumps(ch)}\n\n"
                yield "data: [DONE]\n\n"

            return StreamingResponse(one(), media_type="text/event-stream")
        return body

    # ---------------------------------------------------------------- completions
    @app.post("/v1/completions")
    async def completions(req: CompletionRequest):
        llm = hub.llm(req.model)
        if llm is None:
            return _err(404, f"model '{req.model}' is not served here")
        tok = llm.tokenizer
        prompts = req.prompt if isinstance(req.prompt, list) and req.prompt and isinstance(req.prompt[0], str) else [req.prompt]
        params = _params(req, 16)
        rid = f"cmpl-{uuid.uuid4().hex}"
        created, model = int(time.time()), req.model or hub.default_llm_name
        enc = [p if isinstance(p, list) else ([tok.bos_id] if tok.bos_id is not None else []) + tok.encode(p)
               for p in prompts]
        if req.stream:
            async def gen():
                for i, ids in enumerate(enc):
                    async for it in llm.generate(ids, params, f"{rid}-{i}"):
                        ch = {"id": rid, "object": "text_completion", "created": created, "model": model,
                              "choices": [{"index": i, "text": it.delta, "logprobs": None,
                                           "finish_reason": it.finish_reason if it.finished else None}]}
                        yield f"data: {json.dumps(ch)}\n\n"
                yield "data: [DONE]\n\n"

            return StreamingResponse(gen(), media_type="text/event-stream")
        res = await asyncio.gather(*[llm.complete(ids, params, f"{rid}-{i}") for i, ids in enumerate(enc)])
        choices, ntok = [], 0
        for i, ((text, oids, reason), p) in enumerate(zip(res, prompts)):
            ntok += len(oids)
            choices.append({"index": i, "text": (p + text) if req.echo and isinstance(p, str) else text,
                            "logprobs": None, "finish_reason": reason})
        npr = sum(len(e) for e in enc)
        return {"id": rid, "object": "text_completion", "created": created, "model": model, "choices": choices,
                "usage": {"prompt_tokens": npr, "completion_tokens": ntok, "total_tokens": npr + ntok}}

    # ---------------------------------------------------------------- embeddings
    @app.post("/v1/embeddings")
    async def embeddings(req: EmbeddingRequest):
        emb = hub.embedder(req.model)
        if emb is None:
            return _err(404, f"embedding model '{req.model}' is not served here")
        texts = [req.input] if isinstance(req.input, str) else list(req.input)
        if any(isinstance(t, str) and t.startswith("data:image") for t in texts) and not getattr(emb, "accepts_images", False):
            return _err(400, f"embedding model '{req.model or emb.name}' does not accept image inputs")
        itype = (req.input_type or "query").lower()
        if itype not in ("query", "passage"):
            return _err(400, "input_type must be 'query' or 'passage'")
        t0 = time.perf_counter()
        try:
            # concurrent /v1/embeddings calls coalesce into one encoder batch (Triton dynamic batching semantics)
            fn = getattr(emb, "embed_coalesced", emb.embed)
            vecs = await run_in_threadpool(lambda: fn(texts, itype, req.truncate or "NONE"))
        except ValueError as e:
            return _err(400, str(e))
        METRICS.embed.observe(time.perf_counter() - t0)
        v = vecs.float().cpu()
        if req.dimensions:
            v = v[:, : req.dimensions]
        ntok = sum(len(emb.tokenize(t, itype, "END")) for t in texts)
        return {"object": "list", "data": _embedding_payload(v.tolist(), req.encoding_format or "float"),
                "model": req.model or emb.name, "usage": {"prompt_tokens": ntok, "total_tokens": ntok}}

    # ---------------------------------------------------------------- ranking
    async def _rank(req: RankingRequest):
        rr = hub.reranker(req.model)
        if rr is None:
            return _err(404, f"ranking model '{req.model}' is not served here")
        t0 = time.perf_counter()
        ranked = await run_in_threadpool(lambda: rr.rank(req.query.text, [p.text for p in req.passages],
                                                         req.top_n, req.truncate or "END"))
        METRICS.rerank.observe(time.perf_counter() - t0)
        return {"rankings": [{"index": i, "logit": float(s)} for i, s in ranked]}

    app.post("/v1/ranking")(_rank)
    app.post("/v1/retrieval/nvidia/reranking")(_rank)
    return app
