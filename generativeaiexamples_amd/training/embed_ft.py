"""Full-weight contrastive fine-tuning of the BERT/E5 embedders (reference
nemo/data-flywheel/embedding-finetuning: ``{"query", "pos_doc", "neg_doc": [...]}`` JSONL, all-weights SFT,
batch 256, lr 5e-6, 1 epoch, bf16 — 2_finetuning_and_inference.ipynb:548-624).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m generativeaiexamples_amd.training.embed_ft --embedder e5-large-v2 --data train.jsonl \\
        --global-batch 256 --micro-batch 32 --lr 5e-6 --epochs 1 --out runs/e5-ft --export runs/e5-ft/hf

Loss: InfoNCE over the query's positive against every other passage of the (micro-)batch — the other
queries' positives and all hard negatives (``neg_doc``) — at temperature ``tau``; with
``gather_negatives`` the passage embeddings of every DP rank are all-gathered (autograd-aware) so each
query also sees the other ranks' passages. Queries / passages get the E5 ``query: `` / ``passage: ``
prefixes of :class:`~..engine.embedder.Embedder`, so the tuned weights serve unchanged.

Execution: fp32 master weights (a copy of the serving model's bf16 tensors), bf16 autocast on the GPU,
padded micro-batches through PyTorch SDPA (training needs autograd; the serving path keeps the varlen
HIP kernels), bucketed DP gradient all-reduce overlapped with backward (:class:`~.ddp.GradBucketer`),
AdamW + warmup/cosine, grad clipping. ``--out`` holds ``step_<n>/`` checkpoints (weights + optimizer
+ RNG) and an existing run resumes from the latest one; ``export_hf`` writes a ``config.json`` +
``model.safetensors`` directory that :func:`~..models.registry.build_encoder` loads.
"""
from __future__ import annotations

import argparse
import json
import logging
import math
import os
import random
from dataclasses import asdict, dataclass
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .ddp import GradBucketer

log = logging.getLogger(__name__)


@dataclass
class EmbedFTConfig:
    epochs: int = 1
    global_batch: int = 256
    micro_batch: int = 8
    lr: float = 5e-6
    warmup: int = 0
    weight_decay: float = 0.0
    clip: float = 1.0
    tau: float = 0.02
    max_len: int = 512
    gather_negatives: bool = False
    save_every: int = 0
    out: Optional[str] = None
    seed: int = 0
    max_steps: Optional[int] = None


def load_pairs(path: str) -> List[dict]:
    rows = []
    with open(path, encoding="utf-8") as f:
        for line in f:
            if line.strip():
                r = json.loads(line)
                neg = r.get("neg_doc") or []
                rows.append({"query": r["query"], "pos_doc": r["pos_doc"],
                             "neg_doc": [neg] if isinstance(neg, str) else list(neg)})
    return rows


def encoder_forward(model, w: Dict[str, torch.Tensor], ids: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """Differentiable BERT forward on padded ids [B, S] / mask [B, S] (bool) -> pooled embeddings [B, D]
    with the serving model's pooling + normalisation (same weights layout, padded head dims included)."""
    c = model.cfg
    B, S = ids.shape
    H, hp = c.num_heads, c.head_dim_padded
    pos = torch.arange(S, device=ids.device)
    h = F.embedding(ids, w["word"]) + w["pos"][pos][None] + w["type"][0]
    h = F.layer_norm(h, (c.hidden_size,), w["emb_ln_w"], w["emb_ln_b"], c.ln_eps)
    am = mask[:, None, None, :]  # [B, 1, 1, S] keys
    for i in range(c.num_layers):
        p = f"l{i}."
        qkv = F.linear(h, w[p + "qkv"], w[p + "qkv_b"]).view(B, S, 3, H, hp)
        q, k, v = (qkv[:, :, j].transpose(1, 2) for j in range(3))
        a = F.scaled_dot_product_attention(q, k, v, attn_mask=am, scale=model.scale)
        x = F.linear(a.transpose(1, 2).reshape(B, S, H * hp), w[p + "o"], w[p + "o_b"]) + h
        h = F.layer_norm(x, (c.hidden_size,), w[p + "ln1_w"], w[p + "ln1_b"], c.ln_eps)
        f = F.gelu(F.linear(h, w[p + "up"], w[p + "up_b"]))
        x = F.linear(f, w[p + "down"], w[p + "down_b"]) + h
        h = F.layer_norm(x, (c.hidden_size,), w[p + "ln2_w"], w[p + "ln2_b"], c.ln_eps)
    m = mask[..., None].to(h.dtype)
    if c.pooling == "cls":
        e = h[:, 0]
    elif c.pooling == "last":
        e = h[torch.arange(B, device=h.device), mask.sum(1) - 1]
    else:
        e = (h * m).sum(1) / m.sum(1).clamp_min(1.0)
    e = e.float()
    return F.normalize(e, dim=-1, eps=1e-12) if c.normalize else e


def info_nce(q: torch.Tensor, docs: torch.Tensor, pos_index: torch.Tensor, tau: float) -> torch.Tensor:
    """q [B, D], docs [N, D] (positives and negatives, any order), pos_index [B] -> mean InfoNCE."""
    return F.cross_entropy((q @ docs.t()) / tau, pos_index)


class EmbedFineTuner:
    def __init__(self, embedder, cfg: EmbedFTConfig, rows: Sequence[dict], group=None):
        self.emb, self.model, self.cfg = embedder, embedder.model, cfg
        self.rows = list(rows)
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        dev = self.model.device
        self.device = dev
        # fp32 master copies of every weight (the serving model keeps its bf16 tensors)
        self.w = {k: t.detach().float().clone().requires_grad_(True) for k, t in self.model.w.items()
                  if not k.startswith("cls_")}
        self.params = list(self.w.values())
        self.opt = torch.optim.AdamW(self.params, lr=cfg.lr, weight_decay=cfg.weight_decay)
        if self.world > 1:  # identical starting point on every rank
            for p in self.params:
                dist.broadcast(p.data, 0, group=group)
        self.bucketer = GradBucketer(self.params, group=group)
        self.step = 0
        assert cfg.global_batch % (cfg.micro_batch * self.world) == 0, "global batch must split over micro x DP"
        self.accum = cfg.global_batch // (cfg.micro_batch * self.world)
        per_epoch = max(1, len(self.rows) // cfg.global_batch)
        self.total_steps = cfg.max_steps or per_epoch * cfg.epochs
        self.history: List[float] = []

    # ------------------------------------------------------------------ data
    def _pad(self, seqs: List[List[int]]):
        S = max(len(s) for s in seqs)
        ids = torch.zeros(len(seqs), S, dtype=torch.long)
        mask = torch.zeros(len(seqs), S, dtype=torch.bool)
        for i, s in enumerate(seqs):
            ids[i, : len(s)] = torch.tensor(s)
            mask[i, : len(s)] = True
        return ids.to(self.device), mask.to(self.device)

    def _encode(self, texts: List[str], kind: str) -> torch.Tensor:
        seqs = [self.emb.tokenize(t, kind, "END")[: self.cfg.max_len] for t in texts]
        ids, mask = self._pad(seqs)
        if self.device.type == "cuda":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return encoder_forward(self.model, self.w, ids, mask)
        return encoder_forward(self.model, self.w, ids, mask)

    def micro_loss(self, batch: List[dict]) -> torch.Tensor:
        q = self._encode([r["query"] for r in batch], "query")
        docs, pos_index = [], []
        for r in batch:
            pos_index.append(len(docs))
            docs.append(r["pos_doc"])
            docs += r["neg_doc"]
        d = self._encode(docs, "passage")
        pi = torch.tensor(pos_index, device=d.device)
        if self.cfg.gather_negatives and self.world > 1:
            from torch.distributed.nn.functional import all_gather

            parts = all_gather(d, group=self.group)  # equal sizes: same micro-batch shape on every rank
            offset = sum(p.shape[0] for p in parts[: self.rank])
            d = torch.cat(parts)
            pi = pi + offset
        return info_nce(q, d, pi, self.cfg.tau)

    def _lr(self) -> float:
        c = self.cfg
        if self.step < c.warmup:
            return c.lr * (self.step + 1) / c.warmup
        t = (self.step - c.warmup) / max(1, self.total_steps - c.warmup)
        return c.lr * 0.5 * (1 + math.cos(math.pi * min(1.0, t)))

    # ------------------------------------------------------------------ loop
    def train_step(self, rows: List[dict]) -> float:
        """One optimizer step over this rank's share of a global batch (micro-batch accumulation)."""
        mb = self.cfg.micro_batch
        mine = rows[self.rank::self.world]
        total = 0.0
        self.opt.zero_grad(set_to_none=True)
        for a in range(self.accum):
            self.bucketer.sync = a == self.accum - 1
            loss = self.micro_loss(mine[a * mb:(a + 1) * mb]) / self.accum
            loss.backward()
            total += float(loss.detach())
        self.bucketer.finish()
        if self.cfg.clip:
            torch.nn.utils.clip_grad_norm_(self.params, self.cfg.clip)
        for g in self.opt.param_groups:
            g["lr"] = self._lr()
        self.opt.step()
        self.step += 1
        if self.world > 1:
            t = torch.tensor([total], device=self.device)
            dist.all_reduce(t, group=self.group)
            total = float(t) / self.world
        self.history.append(total)
        return total

    def fit(self) -> List[float]:
        self._maybe_resume()
        rng = random.Random(self.cfg.seed)
        order = list(range(len(self.rows)))
        gb = self.cfg.global_batch
        epoch_of = lambda s: s // max(1, len(self.rows) // gb)  # noqa: E731
        while self.step < self.total_steps:
            e = epoch_of(self.step)
            rng.seed(self.cfg.seed + e)
            rng.shuffle(order)
            b = self.step % max(1, len(self.rows) // gb)
            rows = [self.rows[i] for i in order[b * gb:(b + 1) * gb]]
            loss = self.train_step(rows)
            if self.rank == 0:
                log.info("step %d/%d loss %.4f lr %.2e", self.step, self.total_steps, loss, self._lr())
            if self.cfg.out and self.cfg.save_every and self.step % self.cfg.save_every == 0:
                self.save()
        if self.cfg.out:
            self.save()
        self.sync_to_model()
        return self.history

    # ------------------------------------------------------------------ weights / checkpoints
    @torch.no_grad()
    def sync_to_model(self):
        """Copy the fp32 master weights into the serving model (bf16), ready for /v1/embeddings."""
        for k, t in self.w.items():
            self.model.w[k].copy_(t.to(self.model.w[k].dtype))

    def save(self):
        from safetensors.torch import save_file

        d = os.path.join(self.cfg.out, f"step_{self.step}")
        if self.rank == 0:
            os.makedirs(d, exist_ok=True)
            save_file({k: v.detach().cpu().contiguous() for k, v in self.w.items()}, os.path.join(d, "weights.safetensors"))
            torch.save({"opt": self.opt.state_dict(), "step": self.step, "history": self.history,
                        "cfg": asdict(self.cfg)}, os.path.join(d, "state.pt"))
        if dist.is_initialized():
            dist.barrier(group=self.group)

    def _maybe_resume(self):
        from safetensors.torch import load_file

        if not self.cfg.out or not os.path.isdir(self.cfg.out):
            return
        steps = sorted(int(n[5:]) for n in os.listdir(self.cfg.out) if n.startswith("step_") and n[5:].isdigit())
        if not steps:
            return
        d = os.path.join(self.cfg.out, f"step_{steps[-1]}")
        sd = load_file(os.path.join(d, "weights.safetensors"))
        with torch.no_grad():
            for k, t in self.w.items():
                t.copy_(sd[k].to(t.device))
        st = torch.load(os.path.join(d, "state.pt"), map_location=self.device, weights_only=True)
        self.opt.load_state_dict(st["opt"])
        self.step, self.history = int(st["step"]), list(st["history"])
        log.info("resumed from %s", d)

    def export_hf(self, out_dir: str):
        """HF BERT layout (``config.json`` + ``model.safetensors``), loadable by build_encoder(weights=...)."""
        from safetensors.torch import save_file

        self.sync_to_model()
        if self.rank != 0:
            return
        os.makedirs(out_dir, exist_ok=True)
        sd = self.model.export_hf_state()
        save_file({k: v.float().cpu().contiguous() for k, v in sd.items()}, os.path.join(out_dir, "model.safetensors"))
        c = self.model.cfg
        with open(os.path.join(out_dir, "config.json"), "w") as f:
            json.dump({"architectures": ["BertModel"], "model_type": "bert", "vocab_size": c.vocab_size,
                       "hidden_size": c.hidden_size, "intermediate_size": c.intermediate_size,
                       "num_hidden_layers": c.num_layers, "num_attention_heads": c.num_heads,
                       "max_position_embeddings": c.max_position, "type_vocab_size": c.type_vocab_size,
                       "layer_norm_eps": c.ln_eps, "hidden_act": "gelu"}, f, indent=2)


def recall_at_k(embedder, rows: Sequence[dict], k: int = 1) -> float:
    """Fraction of queries whose positive ranks in the top k among all positives + negatives of ``rows``."""
    docs, pos = [], []
    for r in rows:
        pos.append(len(docs))
        docs.append(r["pos_doc"])
        docs += r["neg_doc"]
    q = embedder.embed([r["query"] for r in rows], "query").float()
    d = embedder.embed(docs, "passage").float()
    top = (q @ d.t()).topk(min(k, len(docs)), dim=1).indices.cpu()
    return float(sum(int(pos[i] in top[i].tolist()) for i in range(len(rows)))) / max(1, len(rows))


def main(argv=None):
    ap = argparse.ArgumentParser(description="contrastive full-weight fine-tuning of an embedder")
    ap.add_argument("--embedder", default="e5-large-v2")
    ap.add_argument("--weights", default=None, help="HF BERT directory (default: random init of the preset)")
    ap.add_argument("--data", default=None, help='JSONL {"query", "pos_doc", "neg_doc": [...]} (default: synthetic)')
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--global-batch", type=int, default=256)
    ap.add_argument("--micro-batch", type=int, default=8)
    ap.add_argument("--lr", type=float, default=5e-6)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--tau", type=float, default=0.02)
    ap.add_argument("--max-len", type=int, default=512)
    ap.add_argument("--max-steps", type=int, default=None)
    ap.add_argument("--gather-negatives", action="store_true")
    ap.add_argument("--save-every", type=int, default=0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--export", default=None)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    from ..engine.embedder import Embedder
    from ..models.registry import build_encoder
    from ..parallel.dist import init_distributed

    ctx = init_distributed(tp_size=1)
    enc, tok, _ = build_encoder(a.embedder, a.weights, device=ctx.device)
    emb = Embedder(enc, tok)
    rows = load_pairs(a.data) if a.data else synthetic_pairs(a.global_batch * 4)
    cfg = EmbedFTConfig(epochs=a.epochs, global_batch=a.global_batch, micro_batch=a.micro_batch, lr=a.lr,
                        warmup=a.warmup, tau=a.tau, max_len=a.max_len, gather_negatives=a.gather_negatives,
                        save_every=a.save_every, out=a.out, max_steps=a.max_steps)
    ft = EmbedFineTuner(emb, cfg, rows)
    hist = ft.fit()
    if a.export:
        ft.export_hf(a.export)
    if ft.rank == 0:
        print(json.dumps({"steps": ft.step, "loss_first": hist[0] if hist else None, "loss_last": hist[-1] if hist
                          else None}))


def synthetic_pairs(n: int, seed: int = 0) -> List[dict]:
    """Synthetic retrieval pairs: the positive shares the query's rare entity tokens, the hard negative
    shares its template words only (a learnable lexical-overlap signal for smoke runs / tests)."""
    rng = random.Random(seed)
    words = [f"w{i}" for i in range(400)]
    rows = []
    for i in range(n):
        ent = rng.sample(words, 3)
        other = rng.sample(words, 3)
        rows.append({"query": f"what is known about {' '.join(ent)}",
                     "pos_doc": f"{' '.join(ent)} is described in this passage number {i}",
                     "neg_doc": [f"{' '.join(other)} is described in this passage number {i + 1}"]})
    return rows


if __name__ == "__main__":
    main()
