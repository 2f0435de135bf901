"""LoRA adapters for the Llama-family weight layout of :class:`~..models.llama.LlamaModel`."""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, field
from typing import Dict, Tuple

import torch

from .. import ops

DEFAULT_TARGETS = ("qkv", "o")


@dataclass
class LoRAConfig:
    r: int = 16
    alpha: float = 32.0
    targets: Tuple[str, ...] = DEFAULT_TARGETS  # subset of qkv, o, gate_up (or fc: non-gated MLP), down
    dropout: float = 0.0

    @property
    def scale(self) -> float:
        return self.alpha / self.r


class LoRAAdapter:
    """fp32 master adapter weights for every (layer, target): ``A`` [r, in], ``B`` [out, r]."""

    def __init__(self, model, cfg: LoRAConfig, device=None, init: bool = True, seed: int = 0):
        self.cfg = cfg
        self.params: Dict[str, torch.Tensor] = {}
        dev = device or model.device
        g = torch.Generator().manual_seed(seed)
        for i in range(model.cfg.num_layers):
            for t in cfg.targets:
                w = model.w.get(f"l{i}.{t}")
                if w is None:
                    continue
                out_f, in_f = w.shape
                a = torch.empty(cfg.r, in_f)
                if init:
                    torch.nn.init.kaiming_uniform_(a, a=math.sqrt(5), generator=g)
                else:
                    a.zero_()
                self.params[f"l{i}.{t}.A"] = a.to(dev).requires_grad_(True)
                self.params[f"l{i}.{t}.B"] = torch.zeros(out_f, cfg.r, device=dev).requires_grad_(True)

    def parameters(self):
        return list(self.params.values())

    def tp_replicated(self):
        """Factors replicated over the TP group (their gradients are partial sums over ranks): A of the
        column-parallel qkv / gate_up, B of the row-parallel o / down."""
        out = []
        for k, v in self.params.items():
            t = k.split(".")[1]
            if (k.endswith(".A") and t in ("qkv", "gate_up", "fc")) or (k.endswith(".B") and t in ("o", "down")):
                out.append(v)
        return out

    def delta_weight(self, layer: int, target: str) -> torch.Tensor | None:
        a = self.params.get(f"l{layer}.{target}.A")
        if a is None:
            return None
        return (self.params[f"l{layer}.{target}.B"] @ a) * self.cfg.scale

    @torch.no_grad()
    def merge_into(self, model):
        """W += scale * B A for every adapted weight (the reference merges .nemo adapters before export)."""
        for key in list(self.params):
            if not key.endswith(".A"):
                continue
            base = key[:-2]
            li, t = base.split(".", 1)
            d = self.delta_weight(int(li[1:]), t)
            w = model.w[base]
            # a weight an engine rewrote into the fragment-ordered inference layout: add the row-major delta to its
            # row-major values, then store them fragment-ordered again (LlamaModel._put does the same on loads)
            merged = (ops.natural_weight(w).float() + d.to(w.device)).to(w.dtype)
            w.copy_(ops.shuffle_fragments(merged) if ops.is_frag(w) else merged)

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {k: v.detach().float().cpu().contiguous() for k, v in self.params.items()}

    def load_state_dict(self, sd: Dict[str, torch.Tensor]):
        with torch.no_grad():
            for k, v in sd.items():
                self.params[k].copy_(v.to(self.params[k].device))

    def save(self, path: str):
        import json
        import os

        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        save_file(self.state_dict(), os.path.join(path, "adapter_model.safetensors"))
        with open(os.path.join(path, "adapter_config.json"), "w") as f:
            json.dump(dict(asdict(self.cfg), targets=list(self.cfg.targets)), f)

    @classmethod
    def load(cls, path: str, model, device=None) -> "LoRAAdapter":
        import json
        import os

        from safetensors.torch import load_file
        with open(os.path.join(path, "adapter_config.json")) as f:
            c = json.load(f)
        ad = cls(model, LoRAConfig(r=c["r"], alpha=c["alpha"], targets=tuple(c["targets"]),
                                   dropout=c.get("dropout", 0.0)), device=device, init=False)
        ad.load_state_dict(load_file(os.path.join(path, "adapter_model.safetensors")))
        return ad
