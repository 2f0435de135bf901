"""Long-context serving profile on one GPU (VERDICT r5 missing #3 / next #5): Llama-3.1-8B (32 layers, llama3 RoPE
scaling, random-init bf16 weights) serving ONE request with a ``--ctx``-token prompt through the engine: chunked
prefill (``--chunk`` tokens per step), then ``--decode`` greedy tokens on the captured decode graphs.

Reports TTFT (add_request -> first token, host clock after a device sync), TPOT (mean decode step), and the prefill
attention's useful FLOPs (causal: 4 * head_dim * q_heads * T (T + 1) / 2 per layer) so that a rocprofv3 kernel table
of the same run gives the attention kernel's TF/s. The reference serves max-model-len 131072
(/root/reference/community/chat-llama-nemotron/backend-dynamo/config/agg_llama_nemotron_4b.yaml:21).

  python tools/long_context.py --ctx 32768 --json-out gpurun_out/lc32k.json
  python tools/long_context.py --ctx 131072 --chunk 16384
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=32768)
    ap.add_argument("--chunk", type=int, default=16384)
    ap.add_argument("--decode", type=int, default=64)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--json-out", default="")
    args = ap.parse_args()

    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import llama3_byte_tokenizer
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel

    dev = torch.device("cuda", 0)
    cfg = LlamaConfig.llama31_8b(num_layers=args.layers)
    m = LlamaModel(cfg, device=dev).random_init(3)
    tok = llama3_byte_tokenizer(cfg.vocab_size)
    # the prompt and its generated tokens must fit the model's 131,072 positions: --ctx 131072 means the longest
    # prompt that leaves room for --decode new tokens
    T = min(args.ctx, cfg.max_position - args.decode - 16)
    eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=4, max_batched_tokens=args.chunk, prefill_chunk=args.chunk,
                                         max_model_len=T + args.decode + 16, prefix_cache=False, decode_steps=8,
                                         graph_batch_sizes=(1,), kv_memory_fraction=0.3))
    eng.capture_graphs()
    g = torch.Generator().manual_seed(1)
    sp = SamplingParams(temperature=0.0, max_tokens=args.decode, ignore_eos=True)
    # warm-up: a short request (kernel attributes, workspaces), untimed
    eng.generate([torch.randint(1000, 120000, (2048,), generator=g).tolist()], SamplingParams(max_tokens=8,
                                                                                             ignore_eos=True))
    prompt = torch.randint(1000, 120000, (T,), generator=g).tolist()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    req = eng.add_request(prompt, sp)
    t_first = None
    n_first = 0
    while eng.has_work():
        eng.step()
        if t_first is None and req.output_ids:
            torch.cuda.synchronize(dev)
            t_first = time.perf_counter()
            n_first = len(req.output_ids)
    torch.cuda.synchronize(dev)
    t_end = time.perf_counter()
    assert len(req.output_ids) == args.decode, len(req.output_ids)
    tpot = (t_end - t_first) / max(1, args.decode - n_first)
    attn_flops = 4 * cfg.head_dim * cfg.num_heads * T * (T + 1) / 2 * args.layers
    gemm_flops = 2 * T * args.layers * (cfg.hidden_size * (cfg.num_heads + 2 * cfg.num_kv_heads) * cfg.head_dim
                                        + cfg.hidden_size * cfg.num_heads * cfg.head_dim
                                        + 3 * cfg.hidden_size * cfg.intermediate_size)
    kv_bytes = T * args.layers * 2 * cfg.num_kv_heads * cfg.head_dim * 2
    res = {"model": cfg.name, "layers": args.layers, "ctx": T, "chunk": args.chunk, "decode_tokens": args.decode,
           "ttft_s": round(t_first - t0, 4), "tpot_ms": round(1e3 * tpot, 3),
           "prefill_tok_s": round(T / (t_first - t0)), "prefill_attention_tflop": round(attn_flops / 1e12, 2),
           "prefill_gemm_tflop": round(gemm_flops / 1e12, 2), "kv_cache_gb_at_ctx": round(kv_bytes / 1e9, 2),
           "decode_kv_tb_s_floor_note": "decode step streams the KV cache + 16 GB of weights",
           "data": "random-init weights, random prompt tokens"}
    print(json.dumps(res), flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
