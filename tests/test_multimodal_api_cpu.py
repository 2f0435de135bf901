"""Multimodal /v1 API on tiny CPU models: image_url chat on the vision LLM (W12) and NV-CLIP-style
text + image embeddings in one space (W14), plus rejection of images on text-only models."""
import base64
import io

import numpy as np
import pytest


def _png_uri(seed=0, h=48, w=64):
    from PIL import Image
    arr = np.random.RandomState(seed).randint(0, 255, (h, w, 3), dtype=np.uint8)
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="PNG")
    return "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()


@pytest.fixture(scope="module")
def client():
    from fastapi.testclient import TestClient

    from generativeaiexamples_amd.serving.hub import HubSpec, ServiceHub
    from generativeaiexamples_amd.serving.openai_api import create_openai_app

    hub = ServiceHub.build(HubSpec(llm="tiny-mllama", embedder="tiny-clip", reranker=None, device="cpu",
                                   served_llm_name="meta/llama-3.2-11b-vision-instruct",
                                   served_embedder_name="nvidia/nvclip", max_num_seqs=4, max_model_len=512))
    with TestClient(create_openai_app(hub)) as c:
        yield c, hub
    hub.shutdown()


def test_image_chat(client):
    c, hub = client
    body = {"model": "meta/llama-3.2-11b-vision-instruct", "max_tokens": 4, "temperature": 0,
            "messages": [{"role": "user", "content": [
                {"type": "text", "text": "Describe the chart."},
                {"type": "image_url", "image_url": {"url": _png_uri(1)}}]}]}
    r = c.post("/v1/chat/completions", json=body)
    assert r.status_code == 200, r.text
    assert r.json()["usage"]["completion_tokens"] >= 1
    r = c.post("/v1/chat/completions", json=dict(body, stream=True))
    assert r.status_code == 200 and r.text.rstrip().endswith("data: [DONE]")
    model = hub.llm().engine.model
    assert not model.cross.seqs  # cross-attention cache released after both requests


def test_clip_embeddings_text_and_image(client):
    c, _ = client
    r = c.post("/v1/embeddings", json={"model": "nvidia/nvclip", "input": ["a red square", _png_uri(2)]})
    assert r.status_code == 200, r.text
    data = r.json()["data"]
    assert len(data) == 2 and len(data[0]["embedding"]) == len(data[1]["embedding"]) == 128
    n = [float(np.linalg.norm(d["embedding"])) for d in data]
    assert all(abs(x - 1) < 1e-3 for x in n)
