"""Deployment sizing for MI355X: memory fit, TP degree, TTFT / TPOT / throughput estimates for a RAG stack
(SURVEY §2.9 vgpu-sizing-advisor; reference community/vgpu-sizing-advisor/src/calculator.py:714-803).

Two models of the same request:

* :func:`plan` - MI355X-first planner. KV bytes per token come from the real attention geometry
  (layers x KV heads x head_dim x K/V, so GQA counts), weights from the model's parameter count, and
  the time terms are rooflines scaled by efficiencies MEASURED on this framework's kernels
  (profiles/r1: hipBLASLt prefill GEMMs 1.55 PF/s bf16, decode attention ~5.4 TB/s, weight-streaming
  decode GEMMs ~4.5 TB/s). Prefill = 2 x params x prompt FLOPs (+ causal attention); a decode step
  reads the weights once and every live sequence's KV.
* :func:`reference_estimate` - the reference advisor's own analytic formulas, kept so the
  "other hardware" rows of BASELINE.md (rows 2-7) can be regenerated: prefill time = params x
  bytes / FLOPS, TPOT = params x bytes / bandwidth, e2e = (prompt x prefill + response x TPOT) / 1000.

``python -m generativeaiexamples_amd.sizing --model llama3-70b --gpu MI355X --concurrency 64``
"""
from __future__ import annotations

import argparse
import json
import math
from dataclasses import asdict, dataclass
from typing import Dict, Optional

GB = 1e9


@dataclass(frozen=True)
class GPUSpec:
    name: str
    memory_gb: float
    bandwidth_tbs: float        # peak HBM / GDDR bandwidth
    bf16_tflops: float          # dense (no sparsity)
    fp8_tflops: float
    # achieved fractions (measured on MI355X by this framework; vendor-typical defaults elsewhere)
    gemm_eff: float = 0.60
    bw_eff: float = 0.70
    link_gbs: float = 0.0       # per-GPU scale-up bandwidth (xGMI / NVLink), GB/s


GPUS: Dict[str, GPUSpec] = {
    # MI355X: 288 GB HBM3E, 8 TB/s, 2.5 PF dense bf16 / 5 PF fp8; 7 xGMI links x ~153 GB/s.
    # gemm_eff 0.62 = 1.55 PF/s hipBLASLt prefill GEMMs; bw_eff 0.68 = 5.4 TB/s decode attention (profiles/r1).
    "MI355X": GPUSpec("MI355X", 288, 8.0, 2500, 5000, gemm_eff=0.62, bw_eff=0.68, link_gbs=7 * 153),
    "MI325X": GPUSpec("MI325X", 256, 6.0, 1307, 2615, link_gbs=7 * 128),
    "MI300X": GPUSpec("MI300X", 192, 5.3, 1307, 2615, link_gbs=7 * 128),
    # the reference advisor's GPUs (gpu_specs.json values: memory, fp16 TFLOPS, bandwidth)
    "L40S": GPUSpec("L40S", 48, 0.864, 366, 733),
    "A40": GPUSpec("A40", 48, 0.696, 299, 299),
    "L4": GPUSpec("L4", 24, 0.300, 242, 485),
    "RTX-PRO-6000": GPUSpec("RTX-PRO-6000", 96, 1.600, 500, 1000),
}


@dataclass(frozen=True)
class ModelSpec:
    name: str
    params_b: float
    layers: int
    kv_heads: int
    head_dim: int
    hidden: int
    heads: int

    @staticmethod
    def from_preset(preset: str) -> "ModelSpec":
        from .models.registry import LLM_PRESETS

        name, mk = LLM_PRESETS[preset]
        c = mk()
        c = getattr(c, "text", c)  # Mllama: text decoder geometry
        params = _llama_params(c)
        return ModelSpec(name, params / 1e9, c.num_layers, c.num_kv_heads, c.head_dim, c.hidden_size, c.num_heads)

    def kv_bytes_per_token(self, kv_bytes: float = 2.0) -> float:
        return 2 * self.layers * self.kv_heads * self.head_dim * kv_bytes


def _llama_params(c) -> float:
    D, I, L = c.hidden_size, c.intermediate_size, c.num_layers
    attn = D * (c.num_heads + 2 * c.num_kv_heads) * c.head_dim + c.num_heads * c.head_dim * D
    mlp_mult = 3 if getattr(c, "mlp", "swiglu") in ("swiglu", "geglu") else 2
    experts = getattr(c, "num_experts", 1) or 1
    mlp = mlp_mult * D * I * experts
    emb = c.vocab_size * D * (1 if c.tie_embeddings else 2)
    return L * (attn + mlp + 2 * D) + emb


ENCODER_GB = {"e5-large-v2": 0.67, "e5-base-v2": 0.22, "all-minilm-l6-v2": 0.05, "nvclip": 0.86}
RERANKER_GB = {"nv-rerankqa-mistral-4b": 7.1, "bge-reranker-large": 1.1}


def plan(model: str | ModelSpec, gpu: str = "MI355X", num_gpus: Optional[int] = None, concurrency: int = 64,
         prompt: int = 2400, response: int = 256, dtype: str = "bf16", kv_dtype: str = "bf16",
         embedder: Optional[str] = "e5-large-v2", reranker: Optional[str] = None, index_vectors: int = 0,
         index_dim: int = 1024, runtime_reserve_gb: float = 6.0) -> dict:
    """Memory + latency plan. ``num_gpus`` None -> the smallest TP degree (power of two) that fits."""
    m = model if isinstance(model, ModelSpec) else ModelSpec.from_preset(model)
    g = GPUS[gpu]
    wbytes = 1.0 if dtype == "fp8" else 2.0
    kvb = 1.0 if kv_dtype == "fp8" else 2.0
    weights_gb = m.params_b * 1e9 * wbytes / GB
    kv_tok = m.kv_bytes_per_token(kvb)
    ctx = prompt + response
    kv_gb = kv_tok * ctx * concurrency / GB
    emb_gb = ENCODER_GB.get(embedder, 0.0) if embedder else 0.0
    rr_gb = RERANKER_GB.get(reranker, 0.0) if reranker else 0.0
    index_gb = index_vectors * index_dim * 2 / GB
    # weights and KV shard over TP; embedder / reranker / index replicate (DP embedder, sharded index)
    fixed_gb = emb_gb + rr_gb + runtime_reserve_gb

    def fits(n):
        return weights_gb / n + kv_gb / n + fixed_gb + index_gb / n <= g.memory_gb

    tp = num_gpus
    if tp is None:
        tp = next((n for n in (1, 2, 4, 8) if fits(n) and m.kv_heads % n == 0), 8)
    free_for_kv = g.memory_gb * tp - weights_gb - fixed_gb * tp - index_gb
    max_seqs = int(max(0.0, free_for_kv) * GB // (kv_tok * ctx)) if kv_tok else 0

    peak = (g.fp8_tflops if dtype == "fp8" else g.bf16_tflops) * 1e12 * g.gemm_eff * tp
    bw = g.bandwidth_tbs * 1e12 * g.bw_eff * tp
    gemm_flops = 2 * m.params_b * 1e9 * prompt
    attn_flops = 2 * 2 * m.layers * m.heads * m.head_dim * prompt * prompt / 2  # causal QK^T + PV
    prefill_s = (gemm_flops + attn_flops) / peak
    # a decode step reads the weights once and the KV of every live sequence (mean context)
    mean_ctx = prompt + response / 2
    step_s = (weights_gb * GB + kv_tok * mean_ctx * concurrency) / bw
    comm_s = 0.0
    if tp > 1 and g.link_gbs:
        # two ring all-reduces of [concurrency, hidden] bf16 per layer on the decode step
        comm_s = 2 * m.layers * 2 * (tp - 1) / tp * concurrency * m.hidden * 2 / (g.link_gbs * 1e9)
    tpot_s = step_s + comm_s
    # wave schedule: all `concurrency` prompts prefilled back to back, then decoded together
    wave_s = concurrency * prefill_s + response * tpot_s
    return {
        "model": m.name, "gpu": g.name, "tp": tp, "dtype": dtype, "kv_dtype": kv_dtype,
        "memory_gb": {"weights": round(weights_gb, 2), "kv_cache": round(kv_gb, 2), "embedder": emb_gb,
                      "reranker": rr_gb, "index": round(index_gb, 2), "runtime": runtime_reserve_gb,
                      "per_gpu": round((weights_gb + kv_gb + index_gb) / tp + fixed_gb, 2),
                      "capacity_per_gpu": g.memory_gb},
        "fits": fits(tp), "kv_bytes_per_token": kv_tok, "max_concurrent_sequences": max_seqs,
        "ttft_s_single": round(prefill_s + tpot_s, 4), "tpot_ms": round(1000 * tpot_s, 3),
        "decode_tokens_per_s": round(concurrency / tpot_s, 1),
        "wave_s": round(wave_s, 3), "queries_per_s": round(concurrency / wave_s, 3),
        "p50_ttft_s_wave": round(concurrency / 2 * prefill_s + tpot_s, 3),
    }


def reference_estimate(params_b: float, gpu: str, num_gpus: int = 1, prompt: int = 1024, response: int = 250,
                       bytes_per_param: float = 2.0) -> dict:
    """The reference advisor's formulas (calculator.py:781-803) - reproduces BASELINE.md rows 2-7."""
    g = GPUS[gpu]
    prefill = params_b * bytes_per_param / g.bf16_tflops / num_gpus          # "seconds" per prompt token x 1e3
    tpot_ms = params_b * bytes_per_param / (g.bandwidth_tbs * 1000) / num_gpus * 1000
    e2e = (prompt * prefill + response * tpot_ms) / 1000
    return {"gpu": gpu, "num_gpus": num_gpus, "ttft_s": round(prefill + tpot_ms / 1000, 3),
            "tpot_ms": round(tpot_ms, 1), "e2e_s": round(e2e, 2), "tokens_per_s": round(response / e2e, 1),
            "queries_per_s": round(1 / e2e, 4)}


def main(argv=None):
    ap = argparse.ArgumentParser(description="MI355X deployment sizing for a RAG stack")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--gpu", default="MI355X", choices=sorted(GPUS))
    ap.add_argument("--num-gpus", type=int, default=None)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=2400)
    ap.add_argument("--response", type=int, default=256)
    ap.add_argument("--dtype", choices=["bf16", "fp8"], default="bf16")
    ap.add_argument("--kv-dtype", choices=["bf16", "fp8"], default="bf16")
    ap.add_argument("--embedder", default="e5-large-v2")
    ap.add_argument("--reranker", default=None)
    ap.add_argument("--index-vectors", type=int, default=1_000_000)
    ap.add_argument("--index-dim", type=int, default=1024)
    ap.add_argument("--reference", action="store_true", help="also print the reference advisor's estimate")
    a = ap.parse_args(argv)
    out = plan(a.model, a.gpu, a.num_gpus, a.concurrency, a.prompt, a.response, a.dtype, a.kv_dtype, a.embedder,
               a.reranker, a.index_vectors, a.index_dim)
    if a.reference:
        m = ModelSpec.from_preset(a.model)
        out["reference_formula"] = {g: reference_estimate(round(m.params_b), g, a.num_gpus or 1)
                                    for g in ("L40S", "A40", "L4", "RTX-PRO-6000")}
    print(json.dumps(out, indent=2))


if __name__ == "__main__":
    main()
