"""Training CLI: ``--mode lora`` (LoRA SFT, :mod:`.trainer`), ``--mode sft`` (full-weight SFT) and
``--mode pretrain`` (from-scratch causal-LM pretraining on a text corpus), both in :mod:`.full`.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m generativeaiexamples_amd.training --mode sft --model gemma-7b --tp 4 --data dolly.jsonl \\
        --global-batch 128 --micro-batch 1 --seq-len 2048 --steps 50 --out runs/gemma-sft
"""
import argparse
import logging

from ..models.registry import build_llm
from ..parallel.dist import init_distributed
from .data import load_jsonl
from .lora import LoRAConfig
from .trainer import LoRATrainer, TrainConfig


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="lora", choices=["lora", "sft", "pretrain"])
    ap.add_argument("--corpus", default=None, help="pretraining text: .txt files / a directory / JSONL with 'text'")
    ap.add_argument("--weight-decay", type=float, default=None)
    ap.add_argument("--export-hf", default=None, help="full modes: write an HF checkpoint (TP=1) at the end")
    ap.add_argument("--model", default="tiny-llama")
    ap.add_argument("--weights", default=None)
    ap.add_argument("--data", default=None, help="JSONL (prompt/response or instruction/context/response)")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--global-batch", type=int, default=8)
    ap.add_argument("--micro-batch", type=int, default=1)
    ap.add_argument("--seq-len", type=int, default=512)
    ap.add_argument("--lr", type=float, default=2e-4)
    ap.add_argument("--rank", type=int, default=16)
    ap.add_argument("--alpha", type=float, default=32)
    ap.add_argument("--targets", default="qkv,o")
    ap.add_argument("--out", default=None)
    ap.add_argument("--save-every", type=int, default=25)
    ap.add_argument("--checkpoint-activations", action="store_true")
    ap.add_argument("--merge-export", default=None)
    a = ap.parse_args()
    logging.basicConfig(level=logging.INFO)
    ctx = init_distributed(tp_size=a.tp)
    import torch
    from ..models.llama import LlamaModel
    m, tok, _ = build_llm(a.model, a.weights, device=ctx.device) if a.tp == 1 else (None, None, None)
    if a.tp > 1:  # TP-sharded model: build with the distributed context
        from ..models.registry import LLM_PRESETS, llama3_byte_tokenizer, small_byte_tokenizer
        cfg = LLM_PRESETS[a.model][1]()
        m = LlamaModel(cfg, device=ctx.device, dist_ctx=ctx).random_init(seed=0)
        tok = llama3_byte_tokenizer(cfg.vocab_size) if cfg.vocab_size >= 128256 else small_byte_tokenizer(cfg.vocab_size)
    rows = load_jsonl(a.data) if a.data else None
    if a.mode != "lora":
        from .data import batches, synthetic_rows
        from .full import FullTrainer, pretrain_batches

        tcfg = TrainConfig(steps=a.steps, global_batch=a.global_batch, micro_batch=a.micro_batch,
                           seq_len=a.seq_len, lr=a.lr, save_every=a.save_every, out=a.out,
                           checkpoint_activations=a.checkpoint_activations)
        dp, dpn = ctx.dp_rank, ctx.dp_size
        if a.mode == "pretrain":
            texts = _corpus(a.corpus) if a.corpus else _synthetic_corpus()
            data = pretrain_batches(texts[dp::dpn], tok, a.seq_len, a.micro_batch, seed=dp)
        else:
            rows = rows if rows is not None else synthetic_rows(512)
            data = batches(rows[dp::dpn], tok, a.seq_len, a.micro_batch, seed=dp, pad_id=tok.pad_id or 0)
        tr = FullTrainer(m, tok, tcfg, data, weight_decay=a.weight_decay if a.weight_decay is not None
                         else (0.1 if a.mode == "pretrain" else 0.0))
        hist = tr.train()
        if ctx.rank == 0:
            print(f"{a.mode}: {tr.num_params() * ctx.tp_size / 1e6:.1f}M params, final loss {hist[-1]:.4f} "
                  f"(first {hist[0]:.4f})" if hist else "nothing to do")
        if a.export_hf:
            tr.export_hf(a.export_hf)
        return
    tr = LoRATrainer(m, tok, LoRAConfig(r=a.rank, alpha=a.alpha, targets=tuple(a.targets.split(","))),
                     TrainConfig(steps=a.steps, global_batch=a.global_batch, micro_batch=a.micro_batch,
                                 seq_len=a.seq_len, lr=a.lr, save_every=a.save_every, out=a.out,
                                 checkpoint_activations=a.checkpoint_activations), rows)
    hist = tr.train()
    if ctx.rank == 0:
        print(f"final loss {hist[-1]:.4f} (first {hist[0]:.4f})" if hist else "nothing to do")
    if a.merge_export:
        tr.merge_and_export(a.merge_export)
    del torch


def _corpus(path):
    import json
    import os

    files = [os.path.join(path, f) for f in sorted(os.listdir(path))] if os.path.isdir(path) else [path]
    out = []
    for f in files:
        if f.endswith(".jsonl"):
            with open(f, encoding="utf-8") as fh:
                out += [json.loads(x).get("text", "") for x in fh if x.strip()]
        elif f.endswith((".txt", ".md")):
            with open(f, encoding="utf-8", errors="replace") as fh:
                out.append(fh.read())
    return [t for t in out if t]


def _synthetic_corpus(n=2000):
    from ..rag import synthetic

    return [synthetic.chunk_document(i, 256).page_content for i in range(n)]


if __name__ == "__main__":
    main()
