"""Full-weight training of decoder LMs: supervised fine-tuning and from-scratch pretraining (TP x DP).

The reference runs full-parameter SFT of Gemma with NeMo on 8 devices at TP=4 (finetuning/Gemma/
sft.ipynb:279-284: tensor_model_parallel_size=4, global_batch_size=128, micro_batch_size=1) and the
NeMo SLM notebook pretrains a small GPT from scratch and then fine-tunes it
(finetuning/NeMo/slm/slm_pretraining_sft.ipynb:449-459). Here both run on the same differentiable
forward as the LoRA trainer (training/forward.py), MI355X-first:

* bf16 weights are the autograd leaves; fp32 master weights + AdamW moments live beside them (16 B per
  parameter: a TP=4 shard of Llama-3-8B is ~32 GB of HBM), the optimizer steps the masters and writes the
  bf16 copies back;
* TP shards follow the inference layout (column-parallel QKV / gate-up, row-parallel O / down,
  vocab-parallel embedding / LM head); replicated tensors (norms) get identical gradients on every TP
  rank by construction of the TP collectives; the global gradient norm sums sharded squares over the TP
  group and counts replicated ones once;
* DP gradients go through the bucketed, backward-overlapped all-reduce (training/ddp.py);
* checkpoints: per-TP-rank safetensors of the bf16 weights + masters / optimizer / RNG / data position
  (``step_<n>/``, resumed automatically, NeMo ``resume_if_exists``); ``export_hf`` writes an HF
  checkpoint at TP=1.

Pretraining data (:func:`pretrain_batches`): documents are tokenised, joined with EOS and cut into
``seq_len`` blocks, every token trained (NeMo's packed GPT dataset); SFT data: training/data.py.
"""
from __future__ import annotations

import json
import logging
import math
import os
import random
import time
from typing import Dict, Iterator, List, Optional, Tuple

import torch
import torch.distributed as dist

from .ddp import GradBucketer
from .forward import lm_loss
from .trainer import TrainConfig, lr_at

log = logging.getLogger(__name__)


def _replicated(name: str) -> bool:
    """Tensors every TP rank holds in full with identical gradients (norm scales / shifts)."""
    return name.endswith("norm") or name.endswith("norm_b")


def pretrain_batches(texts: List[str], tok, seq_len: int, micro_batch: int, seed: int = 0
                     ) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
    """Packed causal-LM blocks: every token is a target (labels = ids)."""
    eos = tok.eos_ids[0] if getattr(tok, "eos_ids", None) else 0
    stream: List[int] = []
    for t in texts:
        stream += tok.encode(t) + [eos]
    n = len(stream) // seq_len
    if n == 0:
        raise ValueError("pretraining corpus shorter than one block")
    blocks = [stream[i * seq_len:(i + 1) * seq_len] for i in range(n)]
    rng = random.Random(seed)
    while True:
        order = list(range(n))
        rng.shuffle(order)
        for i in range(0, n - micro_batch + 1, micro_batch):
            ids = torch.tensor([blocks[j] for j in order[i:i + micro_batch]])
            yield ids, ids.clone()


class FullTrainer:
    """Full-weight SFT / pretraining of a (TP-sharded) LlamaModel; ``data`` yields (ids, labels) micro-batches
    for this DP rank."""

    def __init__(self, model, tokenizer, cfg: TrainConfig, data: Iterator, weight_decay: Optional[float] = None):
        self.model, self.tok, self.cfg, self.data = model, tokenizer, cfg, data
        self.ctx = model.ctx
        torch.manual_seed(cfg.seed)
        seen, self.names, self.params = set(), [], []
        for k, t in model.w.items():
            if getattr(t, "_gai_frag", False):
                raise ValueError(f"{k} is stored in the fragment-ordered inference layout (an LLMEngine rewrote it): "
                                 "train a model no engine has served, or EngineConfig.weight_layout='dual'")
            if t.data_ptr() in seen:  # tied embeddings: one leaf
                continue
            seen.add(t.data_ptr())
            t.requires_grad_(True)
            self.names.append(k)
            self.params.append(t)
        self.master = [p.detach().float().clone() for p in self.params]
        wd = cfg.weight_decay if weight_decay is None else weight_decay
        decay = [m for k, m in zip(self.names, self.master) if m.dim() >= 2]
        no_decay = [m for k, m in zip(self.names, self.master) if m.dim() < 2]
        self.opt = torch.optim.AdamW([{"params": decay, "weight_decay": wd}, {"params": no_decay, "weight_decay": 0.0}],
                                     lr=cfg.lr, betas=(0.9, 0.95), eps=1e-8)
        dp = self.ctx.dp_size
        assert cfg.global_batch % (cfg.micro_batch * dp) == 0, "global_batch must be micro_batch x dp x accum"
        self.accum = cfg.global_batch // (cfg.micro_batch * dp)
        self.bucketer = GradBucketer(self.params, group=self.ctx.dp_group) if dp > 1 else None
        self.step = 0
        self.history: List[float] = []
        if cfg.out:
            self.maybe_resume()

    def num_params(self) -> int:
        return sum(p.numel() for p in self.params)

    # ---------------------------------------------------------------- step
    def _grad_norm(self) -> float:
        dev = self.params[0].device
        sh = torch.zeros((), device=dev, dtype=torch.float32)
        rep = torch.zeros((), device=dev, dtype=torch.float32)
        for k, p in zip(self.names, self.params):
            if p.grad is None:
                continue
            s = p.grad.float().pow(2).sum()
            if _replicated(k):
                rep += s
            else:
                sh += s
        if self.ctx.tp_size > 1:
            dist.all_reduce(sh, group=self.ctx.tp_group)
        return float((sh + rep).sqrt())

    def train_step(self) -> float:
        dev = self.model.device
        total = 0.0
        for g in self.opt.param_groups:
            g["lr"] = lr_at(self.step, self.cfg)
        for mi in range(self.accum):
            ids, labels = next(self.data)
            if self.bucketer is not None:
                self.bucketer.sync = mi == self.accum - 1
            loss = lm_loss(self.model, None, ids.to(dev), labels.to(dev), self.cfg.checkpoint_activations)
            (loss / self.accum).backward()
            total += float(loss.detach()) / self.accum
        if self.bucketer is not None:
            self.bucketer.finish()
        gn = self._grad_norm()
        scale = min(1.0, self.cfg.clip / (gn + 1e-6)) if self.cfg.clip > 0 else 1.0
        for p, m in zip(self.params, self.master):
            m.grad = None if p.grad is None else p.grad.float().mul_(scale)
        self.opt.step()
        with torch.no_grad():
            for p, m in zip(self.params, self.master):
                p.copy_(m)
                p.grad = None
        self.step += 1
        if self.ctx.dp_size > 1:
            t = torch.tensor([total], device=dev)
            dist.all_reduce(t, group=self.ctx.dp_group)
            total = float(t) / self.ctx.dp_size
        return total

    def train(self) -> List[float]:
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

    # ---------------------------------------------------------------- checkpoint / resume / export
    def _dir(self, step: int) -> str:
        return os.path.join(self.cfg.out, f"step_{step:06d}")

    def save(self):
        d = self._dir(self.step)
        r = self.ctx.tp_rank
        if self.ctx.dp_rank == 0:  # DP replicas hold identical weights
            os.makedirs(d, exist_ok=True)
            from safetensors.torch import save_file

            save_file({k: p.detach().contiguous() for k, p in zip(self.names, self.params)},
                      os.path.join(d, f"model.tp{r}.safetensors"))
            save_file({k: m.contiguous() for k, m in zip(self.names, self.master)},
                      os.path.join(d, f"master.tp{r}.safetensors"))
            torch.save({"opt": self.opt.state_dict(), "step": self.step, "rng": torch.get_rng_state()},
                       os.path.join(d, f"trainer.tp{r}.pt"))
        # meta.json is the "checkpoint complete" marker maybe_resume relies on: written only after every rank
        # has flushed its files (barrier), and atomically (temp file + rename)
        if self.ctx.is_distributed:
            self.ctx.barrier()
        if self.ctx.dp_rank == 0 and r == 0:
            tmp = os.path.join(d, "meta.json.tmp")
            with open(tmp, "w") as f:
                json.dump({"step": self.step, "tp": self.ctx.tp_size, "dp": self.ctx.dp_size, "mode": "full",
                           "params": self.num_params()}, f)
                f.flush()
                os.fsync(f.fileno())
            os.replace(tmp, os.path.join(d, "meta.json"))
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

        w = load_file(os.path.join(d, f"model.tp{r}.safetensors"))
        mst = load_file(os.path.join(d, f"master.tp{r}.safetensors"))
        with torch.no_grad():
            for k, p, m in zip(self.names, self.params, self.master):
                p.copy_(w[k])
                m.copy_(mst[k])
        st = torch.load(os.path.join(d, f"trainer.tp{r}.pt"), weights_only=True)
        self.opt.load_state_dict(st["opt"])
        self.step = int(st["step"])
        torch.set_rng_state(st["rng"])
        for _ in range(self.step * self.accum):  # replay the data stream to the resume point
            next(self.data)
        log.info("resumed from %s (step %d)", d, self.step)
        return True

    def export_hf(self, path: str):
        """HF safetensors checkpoint of the trained weights (TP = 1)."""
        if self.ctx.tp_size != 1:
            raise ValueError("export_hf needs TP = 1 (load the TP checkpoint at TP = 1 first)")
        from safetensors.torch import save_file

        os.makedirs(path, exist_ok=True)
        with torch.no_grad():
            sd = {k: v.detach().contiguous().cpu() for k, v in self.model.export_hf_state().items()}
        save_file(sd, os.path.join(path, "model.safetensors"))
