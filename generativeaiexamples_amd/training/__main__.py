"""CLI of the LoRA SFT trainer (see :mod:`.trainer`)."""
import argparse
import logging

from ..models.registry import build_llm
from ..parallel.dist import init_distributed
from .data import load_jsonl
from .lora import LoRAConfig
from .trainer import LoRATrainer, TrainConfig


def main():
    ap = argparse.ArgumentParser()
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


if __name__ == "__main__":
    main()
