"""Chain-server configuration tree (same sections, keys and env names as the reference's
RAG/src/chain_server/configuration.py, plus an ``engine`` section for the in-process MI355X engines).

Env examples: APP_VECTORSTORE_NAME, APP_LLM_SERVERURL, APP_LLM_MODELNAME, APP_LLM_MODELENGINE,
APP_TEXTSPLITTER_CHUNKSIZE, APP_EMBEDDINGS_MODELENGINE, APP_RANKING_SERVERURL, APP_RETRIEVER_TOPK,
APP_RETRIEVER_SCORETHRESHOLD, APP_ENGINE_LLM, APP_ENGINE_TP ...
"""
from __future__ import annotations

from .configuration_wizard import ConfigWizard, configclass, configfield


@configclass
class VectorStoreConfig(ConfigWizard):
    name: str = configfield("name", default="hbm",
                            help_txt="hbm (exact HBM index). milvus / faiss / pgvector are accepted aliases.")
    url: str = configfield("url", default="", help_txt="unused by the in-process HBM store")
    nlist: int = configfield("nlist", default=64, help_txt="kept for compatibility (the HBM index is exact)")
    nprobe: int = configfield("nprobe", default=16, help_txt="kept for compatibility (the HBM index is exact)")
    index_type: str = configfield("indexType", default="FLAT", help_txt="exact brute-force (FLAT)")
    metric: str = configfield("metric", default="cosine", help_txt="cosine | ip | l2")
    persist_dir: str = configfield("persistDir", default="", help_txt="directory for index snapshots + WAL")
    hybrid: bool = configfield("hybrid", default=False,
                               help_txt="also keep a BM25 sparse index (enables retriever nrPipeline hybrid / ranked_hybrid)")


@configclass
class LLMConfig(ConfigWizard):
    server_url: str = configfield("serverUrl", default="", help_txt="host:port of a NIM-compatible /v1 server")
    model_name: str = configfield("modelName", default="meta/llama3-8b-instruct", help_txt="served model name")
    model_engine: str = configfield("modelEngine", default="mi355x",
                                    help_txt="mi355x (in-process) | nvidia-ai-endpoints | openai")
    model_name_pandas_ai: str = configfield("modelNamePandasAI", default="meta/llama3-8b-instruct",
                                            help_txt="model used by the structured-data (CSV) example")
    ignore_eos: bool = configfield("ignoreEos", default=False,
                                   help_txt="benchmarking only: every answer generates exactly max_tokens")


@configclass
class TextSplitterConfig(ConfigWizard):
    model_name: str = configfield("modelName", default="Snowflake/snowflake-arctic-embed-l",
                                  help_txt="tokenizer used to count chunk tokens")
    chunk_size: int = configfield("chunkSize", default=510, help_txt="chunk size in tokens")
    chunk_overlap: int = configfield("chunkOverlap", default=200, help_txt="overlap in tokens")


@configclass
class EmbeddingConfig(ConfigWizard):
    model_name: str = configfield("modelName", default="nvidia/nv-embedqa-e5-v5", help_txt="embedding model")
    model_engine: str = configfield("modelEngine", default="mi355x",
                                    help_txt="mi355x | huggingface (both in-process) | nvidia-ai-endpoints")
    dimensions: int = configfield("dimensions", default=1024, help_txt="embedding width")
    server_url: str = configfield("serverUrl", default="", help_txt="host:port of a /v1/embeddings server")


@configclass
class RankingConfig(ConfigWizard):
    model_name: str = configfield("modelName", default="nv-rerank-qa-mistral-4b:1", help_txt="reranker name")
    model_engine: str = configfield("modelEngine", default="mi355x", help_txt="mi355x | nvidia-ai-endpoints")
    server_url: str = configfield("serverUrl", default="", help_txt="host:port of a /v1/ranking server")


@configclass
class RetrieverConfig(ConfigWizard):
    top_k: int = configfield("topK", default=4, help_txt="chunks returned to the prompt")
    score_threshold: float = configfield("scoreThreshold", default=0.25, help_txt="minimum relevance score")
    nr_url: str = configfield("nrUrl", default="", help_txt="NeMo-Retriever-compatible service (optional)")
    nr_pipeline: str = configfield("nrPipeline", default="ranked_hybrid", help_txt="ranked_hybrid | hybrid")


@configclass
class EngineSection(ConfigWizard):
    llm: str = configfield("llm", default="llama3-8b", help_txt="generator preset (llama3-8b, llama3-70b, opt-125m, ...)")
    llm_weights: str = configfield("llmWeights", default="", help_txt="local HF directory (empty: random init)")
    embedder: str = configfield("embedder", default="e5-large-v2", help_txt="encoder preset")
    embedder_weights: str = configfield("embedderWeights", default="", help_txt="local HF directory")
    reranker: str = configfield("reranker", default="", help_txt="cross-encoder preset (empty: no reranker)")
    reranker_weights: str = configfield("rerankerWeights", default="", help_txt="local HF directory")
    device: str = configfield("device", default="", help_txt="cuda:N | cpu (empty: auto)")
    tp: int = configfield("tp", default=1, help_txt="tensor-parallel degree of the generator")
    max_batch: int = configfield("maxBatch", default=256, help_txt="max concurrent sequences")
    max_model_len: int = configfield("maxModelLen", default=8192, help_txt="context length")
    kv_fraction: float = configfield("kvFraction", default=0.6, help_txt="share of free HBM for the KV cache")


@configclass
class AppConfig(ConfigWizard):
    vector_store: VectorStoreConfig = configfield("vectorStore", env=False, default=VectorStoreConfig())
    llm: LLMConfig = configfield("llm", env=False, default=LLMConfig())
    text_splitter: TextSplitterConfig = configfield("textSplitter", env=False, default=TextSplitterConfig())
    embeddings: EmbeddingConfig = configfield("embeddings", env=False, default=EmbeddingConfig())
    ranking: RankingConfig = configfield("ranking", env=False, default=RankingConfig())
    retriever: RetrieverConfig = configfield("retriever", env=False, default=RetrieverConfig())
    engine: EngineSection = configfield("engine", env=False, default=EngineSection())
