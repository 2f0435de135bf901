"""Digital-fingerprinting autoencoder (reference: /root/reference/community/digital-human-security-analyst/
workspace/dfp/stages/dfp_training.py:53-157, which trains Morpheus' dfencoder ``AutoEncoder`` per user with
encoder [512, 500], decoder [512], relu, swap noise 0.2, SGD lr 1e-3 with 0.99 per-epoch decay, batch 512,
standard scaling, 30 epochs).

A denoising autoencoder over a mixed tabular feature frame: numeric columns standard-scaled (MSE), boolean columns
(BCE), categorical columns embedded (cross-entropy over the categories seen in training; categories rarer than
``min_cats`` map to one "other" slot). Training corrupts each row by swap noise - every cell is replaced, with
probability ``swap_probability``, by the same column's value from a random other row - and reconstructs the clean
row. Scoring returns each feature's reconstruction loss, its z-score against the training losses and the row's
mean / max |z| (the anomaly score), as dfencoder's ``get_results`` does. PyTorch on the GPU when available.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch
from torch import nn


@dataclass
class AEConfig:
    encoder_layers: List[int] = field(default_factory=lambda: [512, 500])
    decoder_layers: List[int] = field(default_factory=lambda: [512])
    activation: str = "relu"
    swap_probability: float = 0.2
    learning_rate: float = 1e-3
    learning_rate_decay: float = 0.99
    batch_size: int = 512
    optimizer: str = "sgd"
    min_cats: int = 1
    seed: int = 0


def _act(name: str) -> nn.Module:
    return {"relu": nn.ReLU(), "tanh": nn.Tanh(), "leaky_relu": nn.LeakyReLU(), "gelu": nn.GELU(),
            "selu": nn.SELU()}[name]


class _Net(nn.Module):
    def __init__(self, n_num: int, n_bin: int, cats: List[int], cfg: AEConfig):
        super().__init__()
        self.embs = nn.ModuleList([nn.Embedding(c, min(32, math.ceil(1.6 * c ** 0.56))) for c in cats])
        d_in = n_num + n_bin + sum(e.embedding_dim for e in self.embs)
        layers, d = [], d_in
        for w in cfg.encoder_layers + cfg.decoder_layers:
            layers += [nn.Linear(d, w), _act(cfg.activation)]
            d = w
        self.body = nn.Sequential(*layers)
        self.num_out = nn.Linear(d, n_num) if n_num else None
        self.bin_out = nn.Linear(d, n_bin) if n_bin else None
        self.cat_out = nn.ModuleList([nn.Linear(d, c) for c in cats])

    def forward(self, num, binf, cat):
        parts = [num, binf] + [e(cat[:, i]) for i, e in enumerate(self.embs)]
        h = self.body(torch.cat([p for p in parts if p.shape[1]], dim=1))
        return (self.num_out(h) if self.num_out is not None else num[:, :0],
                self.bin_out(h) if self.bin_out is not None else binf[:, :0],
                [o(h) for o in self.cat_out])


class TabularAutoEncoder:
    def __init__(self, cfg: Optional[AEConfig] = None, device=None, **overrides):
        self.cfg = cfg or AEConfig()
        for k, v in overrides.items():
            setattr(self.cfg, k, v)
        self.device = torch.device(device) if device else torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.net: Optional[_Net] = None
        self.loss_stats: Dict[str, tuple] = {}

    # ---- feature encoding
    def _fit_schema(self, df):
        self.num_cols = [c for c in df.columns if df[c].dtype.kind in "fiu" and df[c].dtype != bool]
        self.bin_cols = [c for c in df.columns if df[c].dtype == bool]
        self.cat_cols = [c for c in df.columns if c not in self.num_cols and c not in self.bin_cols]
        self.mean = {c: float(df[c].mean()) for c in self.num_cols}
        self.std = {c: float(df[c].std(ddof=0)) or 1.0 for c in self.num_cols}
        self.cat_maps = {}
        for c in self.cat_cols:
            vc = df[c].astype(str).value_counts()
            keep = [v for v, n in vc.items() if n >= self.cfg.min_cats]
            self.cat_maps[c] = {v: i + 1 for i, v in enumerate(sorted(keep))}  # 0 = other / unseen

    def _encode(self, df):
        n = len(df)
        num = np.stack([(df[c].to_numpy(np.float64) - self.mean[c]) / self.std[c] for c in self.num_cols], 1) \
            if self.num_cols else np.zeros((n, 0))
        binf = np.stack([df[c].to_numpy().astype(np.float64) for c in self.bin_cols], 1) if self.bin_cols \
            else np.zeros((n, 0))
        cat = np.stack([df[c].astype(str).map(self.cat_maps[c]).fillna(0).to_numpy(np.int64) for c in self.cat_cols],
                       1) if self.cat_cols else np.zeros((n, 0), np.int64)
        t = lambda a, dt: torch.as_tensor(a, dtype=dt, device=self.device)  # noqa: E731
        return t(num, torch.float32), t(binf, torch.float32), t(cat, torch.long)

    def _swap(self, x: torch.Tensor, g: torch.Generator) -> torch.Tensor:
        if x.shape[1] == 0 or self.cfg.swap_probability <= 0:
            return x
        mask = torch.rand(x.shape, generator=g, device=x.device) < self.cfg.swap_probability
        rows = torch.randint(0, x.shape[0], x.shape, generator=g, device=x.device)
        other = torch.gather(x, 0, rows)
        return torch.where(mask, other, x)

    def _losses(self, out, num, binf, cat) -> torch.Tensor:
        """Per-row, per-feature losses [B, n_features] in column order num | bin | cat."""
        pn, pb, pc = out
        cols = [(pn - num) ** 2] if num.shape[1] else []
        if binf.shape[1]:
            cols.append(nn.functional.binary_cross_entropy_with_logits(pb, binf, reduction="none"))
        for i, logits in enumerate(pc):
            cols.append(nn.functional.cross_entropy(logits, cat[:, i], reduction="none")[:, None])
        return torch.cat(cols, dim=1)

    @property
    def feature_names(self) -> List[str]:
        return self.num_cols + self.bin_cols + self.cat_cols

    # ---- training / scoring
    def fit(self, df, epochs: int = 30, validation_data=None) -> List[float]:
        self._fit_schema(df)
        torch.manual_seed(self.cfg.seed)
        g = torch.Generator(device=self.device).manual_seed(self.cfg.seed)
        num, binf, cat = self._encode(df)
        self.net = _Net(len(self.num_cols), len(self.bin_cols), [len(self.cat_maps[c]) + 1 for c in self.cat_cols],
                        self.cfg).to(self.device)
        n, bs = num.shape[0], self.cfg.batch_size
        if self.cfg.optimizer == "sgd" and torch.device(self.device).type == "cuda" and n >= 4 * bs:
            history = self._fit_graphed(num, binf, cat, epochs, g)
        else:
            history = self._fit_eager(num, binf, cat, epochs, g)
        # z-score statistics of each feature's loss over the (clean) training rows
        losses = self.feature_losses(df)
        self.loss_stats = {c: (float(losses[:, j].mean()), float(losses[:, j].std()) or 1.0)
                           for j, c in enumerate(self.feature_names)}
        if validation_data is not None:
            self.validation_loss = float(self.feature_losses(validation_data).mean())
        return history

    def _fit_graphed(self, num, binf, cat, epochs: int, g: torch.Generator) -> List[float]:
        """SGD with every full 512-row step replayed from one captured HIP graph (the step is ~100 small launches:
        launch-bound when issued one by one). Same update as ``torch.optim.SGD`` without momentum, p -= lr * grad,
        with lr a device scalar so the per-epoch decay needs no re-capture; the swap noise draws from the default
        device generator (graph-safe) instead of ``g``; the last partial batch of an epoch runs eagerly."""
        from ...utils.graphs import hip_graph_capture

        n, bs, history = num.shape[0], self.cfg.batch_size, []
        params = [p for p in self.net.parameters() if p.requires_grad]
        lr = torch.tensor(self.cfg.learning_rate, dtype=torch.float32, device=self.device)
        s_num, s_bin, s_cat = num[:bs].clone(), binf[:bs].clone(), cat[:bs].clone()
        s_loss = torch.zeros((), device=self.device)

        def step(bn, bb, bc, gen):
            out = self.net(self._swap(bn, gen), self._swap(bb, gen), self._swap(bc, gen))
            loss = self._losses(out, bn, bb, bc).mean()
            grads = torch.autograd.grad(loss, params)
            with torch.no_grad():
                torch._foreach_sub_(params, torch._foreach_mul(grads, lr))
            return loss.detach()

        self.net.train()
        graph = None
        for _ in range(epochs):
            perm = torch.randperm(n, generator=g, device=self.device)
            tot = torch.zeros((), device=self.device)
            full = n // bs
            for b in range(full):
                idx = perm[b * bs:(b + 1) * bs]
                torch.index_select(num, 0, idx, out=s_num)
                torch.index_select(binf, 0, idx, out=s_bin)
                torch.index_select(cat, 0, idx, out=s_cat)
                if graph is None:
                    # first step: run once on a side stream (allocator / library warm-up - a real training step),
                    # then capture the same step; replays start with the next batch
                    side = torch.cuda.Stream(device=self.device)
                    side.wait_stream(torch.cuda.current_stream(self.device))
                    with torch.cuda.stream(side):
                        s_loss.copy_(step(s_num, s_bin, s_cat, None))
                    torch.cuda.current_stream(self.device).wait_stream(side)
                    tot += s_loss * bs
                    graph = torch.cuda.CUDAGraph()
                    with hip_graph_capture(graph, side):
                        s_loss.copy_(step(s_num, s_bin, s_cat, None))
                    continue
                graph.replay()
                tot += s_loss * bs
            if n % bs:
                idx = perm[full * bs:]
                tot += step(num[idx], binf[idx], cat[idx], g) * (n - full * bs)
            lr.mul_(self.cfg.learning_rate_decay)
            history.append(float(tot) / n)
        return history

    def _fit_eager(self, num, binf, cat, epochs: int, g: torch.Generator) -> List[float]:
        opt_cls = {"sgd": torch.optim.SGD, "adam": torch.optim.Adam, "adamw": torch.optim.AdamW}[self.cfg.optimizer]
        opt = opt_cls(self.net.parameters(), lr=self.cfg.learning_rate)
        sched = torch.optim.lr_scheduler.ExponentialLR(opt, gamma=self.cfg.learning_rate_decay)
        n, bs, history = num.shape[0], self.cfg.batch_size, []
        for _ in range(epochs):
            self.net.train()
            perm = torch.randperm(n, generator=g, device=self.device)
            # the epoch loss is summed on the device and read once per epoch: a host read per batch would stall the
            # launch-bound loop (512-row batches) on every step
            tot = torch.zeros((), device=self.device)
            for i in range(0, n, bs):
                idx = perm[i:i + bs]
                bn, bb, bc = num[idx], binf[idx], cat[idx]
                out = self.net(self._swap(bn, g), self._swap(bb, g), self._swap(bc, g))
                loss = self._losses(out, bn, bb, bc).mean()
                opt.zero_grad(set_to_none=True)
                loss.backward()
                opt.step()
                tot += loss.detach() * len(idx)
            sched.step()
            history.append(float(tot) / n)
        return history

    @torch.no_grad()
    def feature_losses(self, df) -> np.ndarray:
        self.net.eval()
        num, binf, cat = self._encode(df)
        return self._losses(self.net(num, binf, cat), num, binf, cat).cpu().numpy()

    def get_results(self, df):
        """A frame with <feature>_loss, <feature>_z_loss, mean_abs_z and max_abs_z per row (the anomaly scores)."""
        import pandas as pd

        losses = self.feature_losses(df)
        out = {}
        zs = []
        for j, c in enumerate(self.feature_names):
            mu, sd = self.loss_stats[c]
            z = (losses[:, j] - mu) / sd
            out[f"{c}_loss"], out[f"{c}_z_loss"] = losses[:, j], z
            zs.append(np.abs(z))
        za = np.stack(zs, 1)
        out["mean_abs_z"], out["max_abs_z"] = za.mean(1), za.max(1)
        return pd.DataFrame(out, index=df.index)


def train_per_user(df, user_column: str, feature_columns: List[str], epochs: int = 30, min_rows: int = 1,
                   **ae_kwargs) -> Dict[str, TabularAutoEncoder]:
    """One model per user over its own rows (the reference's per-user DFP training stage)."""
    models = {}
    for user, part in df.groupby(user_column):
        if len(part) < min_rows:
            continue
        m = TabularAutoEncoder(**ae_kwargs)
        m.fit(part[feature_columns], epochs=epochs)
        models[str(user)] = m
    return models
