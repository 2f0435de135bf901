"""Benchmarks of the BASELINE.json configurations beyond the headline (which lives in bench.py):

* config 3 - :mod:`.rag70b`: Llama-3-70B (TP over the ranks) + cross-encoder rerank of the top-40 +
  a 10M-vector index sharded over the ranks.
* config 4 - :mod:`.multimodal`: NV-CLIP ViT-L/14 retrieval + Llama-3.2-11B-Vision generation, fp8 MFMA.
* config 5 - :mod:`.agentic`: Mixtral-8x7B tool-calling loop (plan -> retrieve tool -> answer).

Each module exposes ``add_args(ap)`` and ``run(args, ctx) -> dict`` (the bench.py JSON line).
"""
CONFIGS = {3: "rag70b", 4: "multimodal", 5: "agentic"}


def module(config: int):
    import importlib
    return importlib.import_module(f"{__name__}.{CONFIGS[config]}")
