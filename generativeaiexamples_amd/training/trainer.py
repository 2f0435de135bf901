"""LoRA SFT trainer (TP x DP over RCCL; gloo on the CPU test tier).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m generativeaiexamples_amd.training --model llama3-8b --tp 4 --data dolly.jsonl \\
        --global-batch 128 --micro-batch 1 --seq-len 2048 --steps 50 --out runs/llama3-lora

Global batch = micro_batch x grad_accum x dp_size (the reference: global_batch_size=128,
micro_batch_size=1, TP=4 on 8 devices -> DP=2). ``--out`` holds ``step_<n>/`` checkpoints (LoRA
safetensors per TP rank + optimizer/scheduler/RNG state); an existing run resumes from its latest
checkpoint (NeMo ``resume_if_exists``). ``--merge-export DIR`` folds the adapter into the base weights
and writes HF safetensors (TP=1).
"""
from __future__ import annotations

import json
import logging
import math
import os
import time
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from .data import batches, load_jsonl, synthetic_rows
from .ddp import GradBucketer
from .forward import lm_loss
from .lora import LoRAAdapter, LoRAConfig

log = logging.getLogger(__name__)


@dataclass
class TrainConfig:
    steps: int = 50
    global_batch: int = 8
    micro_batch: int = 1
    seq_len: int = 512
    lr: float = 2e-4
    warmup: int = 5
    weight_decay: float = 0.0
    clip: float = 1.0
    save_every: int = 25
    out: Optional[str] = None
    checkpoint_activations: bool = False
    seed: int = 0


def lr_at(step: int, cfg: TrainConfig) -> float:
    if step < cfg.warmup:
        return cfg.lr * (step + 1) / cfg.warmup
    t = (step - cfg.warmup) / max(1, cfg.steps - cfg.warmup)
    return cfg.lr * 0.5 * (1 + math.cos(math.pi * min(1.0, t)))


class LoRATrainer:
    def __init__(self, model, tokenizer, lora_cfg: LoRAConfig, cfg: TrainConfig, rows=None):
        self.model, self.tok, self.cfg = model, tokenizer, cfg
        self.ctx = model.ctx
        torch.manual_seed(cfg.seed)
        self.lora = LoRAAdapter(model, lora_cfg, seed=cfg.seed + self.ctx.tp_rank * 0)
        params = self.lora.parameters()
        self.opt = torch.optim.AdamW(params, lr=cfg.lr, weight_decay=cfg.weight_decay, betas=(0.9, 0.999))
        dp = self.ctx.dp_size
        assert cfg.global_batch % (cfg.micro_batch * dp) == 0, "global_batch must be micro_batch x dp x accum"
        self.accum = cfg.global_batch // (cfg.micro_batch * dp)
        self.bucketer = GradBucketer(params, group=self.ctx.dp_group) if dp > 1 else None
        self.step = 0
        rows = rows if rows is not None else synthetic_rows(512, seed=cfg.seed)
        self.data = batches(rows[self.ctx.dp_rank::dp], tokenizer, cfg.seq_len, cfg.micro_batch,
                            seed=cfg.seed + self.ctx.dp_rank, pad_id=tokenizer.pad_id or 0)
        self.history = []
        if cfg.out:
            self.maybe_resume()

    # ---------------------------------------------------------------- checkpoint / resume
    def _ckpt_dir(self, step: int) -> str:
        return os.path.join(self.cfg.out, f"step_{step:06d}")

    def save(self):
        d = self._ckpt_dir(self.step)
        r = self.ctx.tp_rank
        if self.ctx.dp_rank == 0:  # DP replicas hold identical adapters
            os.makedirs(d, exist_ok=True)
            from safetensors.torch import save_file
            save_file(self.lora.state_dict(), os.path.join(d, f"adapter.tp{r}.safetensors"))
            torch.save({"opt": self.opt.state_dict(), "step": self.step, "rng": torch.get_rng_state()},
                       os.path.join(d, f"trainer.tp{r}.pt"))
            if r == 0:
                with open(os.path.join(d, "meta.json"), "w") as f:
                    json.dump({"step": self.step, "tp": self.ctx.tp_size, "dp": self.ctx.dp_size,
                               "lora": {"r": self.lora.cfg.r, "alpha": self.lora.cfg.alpha,
                                        "targets": list(self.lora.cfg.targets)}}, f)
        if self.ctx.is_distributed:
            self.ctx.barrier()

    def maybe_resume(self) -> bool:
        if not os.path.isdir(self.cfg.out):
            return False
        done = sorted(x for x in os.listdir(self.cfg.out)
                      if x.startswith("step_") and os.path.exists(os.path.join(self.cfg.out, x, "meta.json")))
        if not done:
            return False
        d = os.path.join(self.cfg.out, done[-1])
        r = self.ctx.tp_rank
        from safetensors.torch import load_file
        self.lora.load_state_dict(load_file(os.path.join(d, f"adapter.tp{r}.safetensors")))
        st = torch.load(os.path.join(d, f"trainer.tp{r}.pt"), weights_only=True)
        self.opt.load_state_dict(st["opt"])
        self.step = int(st["step"])
        torch.set_rng_state(st["rng"])
        for _ in range(self.step * self.accum):  # replay the data stream to the resume point
            next(self.data)
        log.info("resumed from %s (step %d)", d, self.step)
        return True

    # ---------------------------------------------------------------- training
    def train_step(self) -> float:
        dev = self.model.device
        total = 0.0
        for g in self.opt.param_groups:
            g["lr"] = lr_at(self.step, self.cfg)
        for mi in range(self.accum):
            ids, labels = next(self.data)
            if self.bucketer is not None:
                self.bucketer.sync = mi == self.accum - 1
            loss = lm_loss(self.model, self.lora, ids.to(dev), labels.to(dev), self.cfg.checkpoint_activations)
            (loss / self.accum).backward()
            total += float(loss.detach()) / self.accum
        if self.ctx.tp_size > 1:  # partial grads of TP-replicated LoRA factors
            for p in self.lora.tp_replicated():
                if p.grad is not None:
                    dist.all_reduce(p.grad, group=self.ctx.tp_group)
        if self.bucketer is not None:
            self.bucketer.finish()
        torch.nn.utils.clip_grad_norm_(self.lora.parameters(), self.cfg.clip)
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        self.step += 1
        if self.ctx.dp_size > 1:
            t = torch.tensor([total], device=dev)
            dist.all_reduce(t, group=self.ctx.dp_group)
            total = float(t) / self.ctx.dp_size
        return total

    def train(self):
        t0 = time.perf_counter()
        while self.step < self.cfg.steps:
            loss = self.train_step()
            self.history.append(loss)
            if self.ctx.rank == 0 and (self.step % 10 == 0 or self.step == self.cfg.steps):
                toks = self.step * self.cfg.global_batch * self.cfg.seq_len
                log.info("step %d loss %.4f lr %.2e %.0f tok/s", self.step, loss, self.opt.param_groups[0]["lr"],
                         toks / (time.perf_counter() - t0))
            if self.cfg.out and (self.step % self.cfg.save_every == 0 or self.step == self.cfg.steps):
                self.save()
        return self.history

    def merge_and_export(self, path: str):
        self.lora.merge_into(self.model)
        if self.ctx.tp_size == 1:
            from safetensors.torch import save_file
            os.makedirs(path, exist_ok=True)
            save_file({k: v.contiguous().cpu() for k, v in self.model.export_hf_state().items()},
                      os.path.join(path, "model.safetensors"))
