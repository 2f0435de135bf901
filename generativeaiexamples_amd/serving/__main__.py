"""``python -m generativeaiexamples_amd.serving`` - the NIM-compatible model server (port 8000).

Equivalent of the reference's ``nemollm-inference`` + ``nemollm-embedding`` + ``ranking-ms``
containers in one MI355X process. Example:

    python -m generativeaiexamples_amd.serving --llm llama3-8b --embedder e5-large-v2 \\
        --reranker nv-rerankqa-mistral-4b --port 8000

``--tp N`` serves the generator tensor-parallel over N GPUs of this node (the reference's LLM NIM spans
``INFERENCE_GPU_COUNT`` GPUs, RAG/examples/local_deploy/docker-compose-nim-ms.yaml:20): the command
re-runs itself as N ranks; rank 0 serves the API and plans every engine step, ranks 1..N-1 execute the
plans it broadcasts (LLMEngine.follow) until it shuts down.
"""
from __future__ import annotations

import argparse
import logging
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--llm", default=os.environ.get("APP_ENGINE_LLM", "llama3-8b"))
    ap.add_argument("--llm-weights", default=os.environ.get("APP_ENGINE_LLMWEIGHTS"))
    ap.add_argument("--embedder", default=os.environ.get("APP_ENGINE_EMBEDDER", "e5-large-v2"))
    ap.add_argument("--embedder-weights", default=os.environ.get("APP_ENGINE_EMBEDDERWEIGHTS"))
    ap.add_argument("--reranker", default=os.environ.get("APP_ENGINE_RERANKER"))
    ap.add_argument("--reranker-weights", default=os.environ.get("APP_ENGINE_RERANKERWEIGHTS"))
    ap.add_argument("--served-model-name", default=None)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--lora", action="append", default=[],
                    help="NAME=DIR serves a trained LoRA adapter (unmerged, per request); NAME alone aliases the base model")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--device", default=None)
    ap.add_argument("--tp", type=int, default=int(os.environ.get("APP_ENGINE_TP", "1")),
                    help="tensor-parallel degree of the generator (one process per GPU)")
    ap.add_argument("--dtype", default=None, help="generator dtype override, e.g. float32")
    ap.add_argument("--kv-cache-dtype", default=os.environ.get("APP_ENGINE_KVCACHEDTYPE", "auto"),
                    help="auto | fp8 (OCP e4m3fn paged KV cache: 2x cached tokens, half the decode KV bytes)")
    a = ap.parse_args()
    if a.tp > 1 and "WORLD_SIZE" not in os.environ:
        import sys

        from ..parallel.launch import spawn_ranks

        sys.exit(spawn_ranks(a.tp, script="-m generativeaiexamples_amd.serving"))
    logging.basicConfig(level=os.environ.get("LOGLEVEL", "INFO").upper())

    import uvicorn

    from .hub import HubSpec, ServiceHub
    from .openai_api import create_openai_app

    spec = HubSpec(llm=a.llm or None, llm_weights=a.llm_weights, embedder=a.embedder or None,
                   embedder_weights=a.embedder_weights, reranker=a.reranker, reranker_weights=a.reranker_weights,
                   served_llm_name=a.served_model_name, max_num_seqs=a.max_num_seqs, max_model_len=a.max_model_len,
                   use_graphs=not a.no_graphs, lora_adapters=dict((x.split("=", 1) + [""])[:2] for x in a.lora), device=a.device,
                   tp=a.tp, dtype=a.dtype, kv_cache_dtype=a.kv_cache_dtype)
    hub = ServiceHub.build(spec)
    if hub.is_follower:
        hub.serve_follower()
        return
    try:
        uvicorn.run(create_openai_app(hub), host=a.host, port=a.port, log_level="info")
    finally:
        hub.shutdown()


if __name__ == "__main__":
    main()
