"""Mixtral-8x7B family (sparse MoE decoder; BASELINE config 5).

Attention is the Llama block. The MLP is a top-2-of-8 mixture: router GEMM (fp32 logits) ->
``moe_route`` (softmax, top-k, renormalise) -> device-side dispatch plan (expert-sorted rows, no
host sync) -> grouped GEMM w1|w3 with the SwiGLU epilogue gathering token rows -> grouped GEMM w2
-> weighted combine (+ residual). 47B parameters = 94 GB bf16: fits ONE 288 GB MI355X.

Expert parallelism, two modes:

* TP mode (``dist_ctx`` with tp > 1): experts are sharded over the TP group (rank r owns experts
  [r*E/tp, (r+1)*E/tp)); hidden states are replicated by the attention all-reduce, so each rank
  computes only the (token, expert) pairs it owns and the row-parallel all-reduce sums the expert
  outputs - no extra collective.
* EP mode (``ep_group``): data-parallel attention (every rank holds attention / embeddings and serves
  its own requests) + experts sharded over the EP group, tokens exchanged with all-to-all
  (:mod:`..parallel.ep`): every step uses the fixed-capacity, sync-free padded exchange (capacity = the
  step's largest per-rank token count, agreed by the engine's EP lockstep, ``LLMEngine``); prefill steps
  exchange the per-peer counts on the device and move only the valid rows. Ranks step in lockstep; a rank without work runs a one-token dummy
  forward so every all-to-all has all its peers.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict

import torch

from .. import ops
from .common import ForwardBatch, randn_like_
from .llama import LlamaConfig, LlamaModel


@dataclass
class MixtralConfig(LlamaConfig):
    num_experts: int = 8
    top_k: int = 2

    @staticmethod
    def mixtral_8x7b(**kw):
        return MixtralConfig(name="mistralai/mixtral-8x7b-instruct-v0.1", vocab_size=32000, rope_theta=1e6,
                             max_position=32768, bos_token_id=1, eos_token_ids=(2,), **kw)

    @staticmethod
    def from_hf(path: str) -> "MixtralConfig":
        import json
        with open(os.path.join(path, "config.json")) as f:
            c = json.load(f)
        return MixtralConfig(**LlamaConfig.hf_fields(c, os.path.basename(path.rstrip("/"))),
                             num_experts=c.get("num_local_experts", 8), top_k=c.get("num_experts_per_tok", 2))

    @staticmethod
    def tiny_moe(**kw):
        base = dict(vocab_size=512, hidden_size=256, intermediate_size=256, num_layers=2, num_heads=4, num_kv_heads=2,
                    head_dim=64, max_position=2048, bos_token_id=1, eos_token_ids=(2,), name="tiny-moe",
                    num_experts=4, top_k=2)
        base.update(kw)
        return MixtralConfig(**base)


# MoE steps with at least this many (token, expert) rows run each expert on the dense prefill GEMMs
# (GAI_MOE_DENSE_PREFILL_ROWS; a huge value keeps every step on the grouped kernel)
_DENSE_PREFILL_MIN_ROWS = int(os.environ.get("GAI_MOE_DENSE_PREFILL_ROWS", "2048"))


class MixtralModel(LlamaModel):
    supports_fp8_kv = False  # own attention call sites (no per-layer KV scales)

    def __init__(self, cfg, device=None, dtype=torch.bfloat16, dist_ctx=None, ep_group=None):
        import torch.distributed as dist

        self.ep_group = ep_group
        self.ep_size = dist.get_world_size(ep_group) if ep_group is not None else 1
        self.ep_rank = dist.get_rank(ep_group) if ep_group is not None else 0
        self.ep_capacity_tokens = 0   # EP lockstep: the step's largest per-rank token count (set by the engine)
        self.ep_exact = False         # EP lockstep: some rank prefills this step -> exact-count exchange
        super().__init__(cfg, device, dtype, dist_ctx)
        # decode-time token exchange: the one-shot peer-memory all-to-all (direct xGMI writes, graph-capturable even
        # over a gloo control plane); GAI_EP_A2A=rccl keeps RCCL's all_to_all_single
        self.ep_xchg = None
        if (ep_group is not None and self.ep_size > 1 and self.device.type == "cuda"
                and os.environ.get("GAI_EP_A2A", "peer") != "rccl"):
            from ..parallel.custom_ar import CustomAllReduce
            # slots for the prefill slabs too (GAI_EP_A2A_MAX_MB per peer segment; larger slabs go to RCCL)
            a2a_mb = int(os.environ.get("GAI_EP_A2A_MAX_MB", "64"))
            self.ep_xchg = CustomAllReduce(group=ep_group, device=self.device, a2a_max_bytes=a2a_mb << 20)

    def _alloc(self):
        c = self.cfg
        if self.ep_group is not None:
            assert self.ctx.tp_size == 1, "EP mode runs data-parallel attention (tp = 1)"
            shards, r = self.ep_size, self.ep_rank
        else:
            shards, r = self.ctx.tp_size, self.ctx.tp_rank
        assert c.num_experts % shards == 0, "experts must divide the TP/EP group"
        self.e_local = c.num_experts // shards
        self.e_start = r * self.e_local
        # the dense MLP of LlamaModel is replaced by experts: allocate attention etc. via the parent,
        # then drop its MLP weights
        inter = self.inter
        self.inter = 16  # tiny placeholder for the parent allocation
        super()._alloc()
        self.inter = inter
        d, dt, D, I = self.device, self.dtype, c.hidden_size, c.intermediate_size
        for i in range(c.num_layers):
            p = f"l{i}."
            del self.w[p + "gate_up"], self.w[p + "down"]
            self.w[p + "router"] = torch.empty(c.num_experts, D, device=d, dtype=dt)
            self.w[p + "w13"] = torch.empty(self.e_local, 2 * I, D, device=d, dtype=dt)  # interleaved per 16
            self.w[p + "w2"] = torch.empty(self.e_local, D, I, device=d, dtype=dt)

    def random_init(self, seed: int = 0):
        s = seed * 1000 + self.ctx.tp_rank + 100 * self.ep_rank
        for k, t in self.w.items():
            if k.endswith("norm"):
                t.fill_(1.0)
            elif k in ("embed",):
                randn_like_(t, s, 0.02)
            else:
                randn_like_(t, s, 1.0 / math.sqrt(t.shape[-1]))
            s += 1
        return self

    def _load_mlp(self, sd: Dict[str, torch.Tensor], i: int):
        p, h = f"l{i}.", f"model.layers.{i}.block_sparse_moe."
        self.w[p + "router"].copy_(sd[h + "gate.weight"].to(self.dtype))
        for j in range(self.e_local):
            e = self.e_start + j
            g, u = sd[h + f"experts.{e}.w1.weight"], sd[h + f"experts.{e}.w3.weight"]
            self.w[p + "w13"][j].copy_(ops.interleave_gate_up(g, u).to(self.dtype))
            self.w[p + "w2"][j].copy_(sd[h + f"experts.{e}.w2.weight"].to(self.dtype))

    def moe_mlp(self, x: torch.Tensor, layer: int, residual: torch.Tensor | None) -> torch.Tensor:
        c, w, p = self.cfg, self.w, f"l{layer}."
        T = x.shape[0]
        logits = ops.linear(x, w[p + "router"], out_dtype=torch.float32)
        ids, wts = ops.moe_route(logits, c.top_k, True)
        k = c.top_k
        if self.ep_group is not None:
            return self._moe_ep(x, ids, wts, w[p + "w13"], w[p + "w2"], residual)
        if self.e_local != c.num_experts:  # EP: keep only local experts; others -> sentinel bin, weight 0
            loc = ids - self.e_start
            mine = (loc >= 0) & (loc < self.e_local)
            ids = torch.where(mine, loc, torch.full_like(loc, self.e_local)).to(torch.int32)
            wts = torch.where(mine, wts, torch.zeros_like(wts))
            a_rows, offs, pos = ops.moe_dispatch(ids, self.e_local + 1)
        else:
            a_rows, offs, pos = ops.moe_dispatch(ids, c.num_experts)
        if (x.is_cuda and self.e_local == c.num_experts and T * k >= _DENSE_PREFILL_MIN_ROWS
                and not torch.cuda.is_current_stream_capturing()):
            y = self._moe_dense_prefill(x, a_rows, offs, w[p + "w13"], w[p + "w2"], T * k)
            return ops.moe_combine(y, pos, wts, residual)
        h1 = ops.moe_gemm(x, a_rows, w[p + "w13"], offs, T * k, swiglu=True)
        y = ops.moe_gemm(h1, None, w[p + "w2"], offs, T * k, swiglu=False) if self.e_local == c.num_experts else \
            self._moe_down_ep(h1, w[p + "w2"], offs, T * k)
        return ops.moe_combine(y, pos, wts, residual)

    @staticmethod
    def _moe_dense_prefill(x, a_rows, offs, w13, w2, rows: int) -> torch.Tensor:
        """Prefill-sized steps: the expert-sorted rows are gathered once and every expert's slice runs on the
        dense persistent 256x256 GEMMs (SwiGLU epilogue on the interleaved w1|w3), ~1.6 vs ~1.0 PF/s for the
        128x128 grouped kernel at Mixtral widths. Reads the expert row ranges on the host: one sync per layer,
        prefill only (decode steps keep the graph-capturable grouped path)."""
        bounds = offs.tolist()
        xs = x.index_select(0, a_rows.long())
        h1 = torch.empty(rows, w13.shape[1] // 2, dtype=x.dtype, device=x.device)
        y = torch.empty(rows, w2.shape[1], dtype=x.dtype, device=x.device)
        for e in range(w13.shape[0]):
            lo, hi = bounds[e], bounds[e + 1]
            if hi > lo:
                ops.linear(xs[lo:hi], w13[e], act="swiglu", out=h1[lo:hi])
                ops.linear(h1[lo:hi], w2[e], out=y[lo:hi])
        return y

    def _moe_ep(self, x, ids, wts, w13, w2, residual):
        """All-to-all expert parallelism: pairs go to the rank owning their expert and come back weighted."""
        c = self.cfg
        # capacity: the step's largest per-rank token count (EP lockstep) x top-k - never drops a pair. Prefill-sized
        # steps (ep_exact) exchange the per-peer counts on the device and move only the valid rows; decode steps
        # move whole slabs (graph-capturable). Neither synchronises the host.
        cap_tok = max(self.ep_capacity_tokens, x.shape[0])
        chunk = self._ep_chunk_tokens(x, cap_tok)
        if chunk >= cap_tok:
            return self._moe_ep_slab(x, ids, wts, w13, w2, residual, cap_tok * c.top_k)
        # a prefill step whose per-peer segments would overflow the peer-memory buffers runs in row chunks that fit
        # them: every rank makes the same number of exchanges (cap_tok is agreed by the lockstep), the slabs and the
        # expert GEMM intermediates are sized by the chunk, never by W x the whole step; a rank whose
        # rows ran out joins with one zero-weight row and drops its output
        T, outs = x.shape[0], []
        for lo in range(0, cap_tok, chunk):
            hi = min(lo + chunk, T)
            if hi > lo:
                outs.append(self._moe_ep_slab(x[lo:hi], ids[lo:hi], wts[lo:hi], w13, w2,
                                              None if residual is None else residual[lo:hi], chunk * c.top_k))
            else:
                self._moe_ep_slab(x[:1], ids[:1], torch.zeros_like(wts[:1]), w13, w2, None, chunk * c.top_k)
        return torch.cat(outs)

    def _ep_chunk_tokens(self, x, cap_tok: int) -> int:
        """Tokens per MoE exchange of a prefill-sized EP step: all of them while one per-peer segment of capacity
        cap_tok x top_k rows (D + 8 bf16 lanes each) fits the peer-memory slot, else as many as fit.
        GAI_EP_PREFILL_CHUNK_TOKENS forces a chunk size (tests; the gloo control plane has no slot)."""
        forced = int(os.environ.get("GAI_EP_PREFILL_CHUNK_TOKENS", "0"))
        if forced > 0 and self.ep_exact:
            return forced
        if not (self.ep_exact and self.ep_xchg is not None and x.is_cuda):
            return cap_tok
        row_bytes = (x.shape[1] + 8) * x.element_size()
        return max(1, self.ep_xchg.slot_bytes // (row_bytes * self.cfg.top_k))

    def _moe_ep_slab(self, x, ids, wts, w13, w2, residual, cap: int):
        from ..parallel import ep

        c = self.cfg
        rows, eid, plan = ep.dispatch_padded(x, ids, c.num_experts, capacity=cap, group=self.ep_group,
                                             xchg=self.ep_xchg, exact_counts=self.ep_exact)
        y = ep.local_experts_padded(rows, eid, w13, w2)
        return ep.combine_padded(y, wts, plan, group=self.ep_group, xchg=self.ep_xchg, residual=residual)

    def _moe_down_ep(self, h1, w2, offs, rows):
        y = ops.moe_gemm(h1, None, w2, offs, rows, swiglu=False)
        # rows of non-local pairs were never written: zero them (their combine weight is 0)
        valid = torch.arange(rows, device=y.device) < offs[self.e_local].to(torch.int64)
        return torch.where(valid[:, None], y, torch.zeros((), dtype=y.dtype, device=y.device))

    def forward(self, fb: ForwardBatch, kv, decode_ws=None) -> torch.Tensor:
        c, w, ctx = self.cfg, self.w, self.ctx
        T, P = fb.num_tokens, fb.num_prefill_tokens
        hd = c.head_dim
        res = ops.embedding(fb.token_ids, w["embed"], self.vstart, self.vstart + self.vocab_local)
        ctx.tp_all_reduce(res)
        q = torch.empty(T, self.hq, hd, device=res.device, dtype=self.dtype)
        attn = torch.empty_like(q)
        h = None
        for i in range(c.num_layers):
            p = f"l{i}."
            x = ops.rms_norm(res, w[p + "attn_norm"], c.rms_eps) if h is None else \
                ops.rms_norm(h, w[p + "attn_norm"], c.rms_eps, residual=res)
            qkv = ops.linear(x, w[p + "qkv"])
            kc, vc = kv.layer(i)
            ops.rope_kv_write(qkv, fb.positions, self.cos_sin, fb.slots, q, kc, vc, self.hq, self.hkv, hd, True)
            if P > 0:
                ops.attention_prefill(q[:P], kc, vc, fb.prefill_block_tables, fb.cu_q, fb.prefill_ctx, self.scale,
                                      True, tiles=fb.prefill_tiles, q_lens=fb.prefill_qlen, out=attn[:P])
            if T > P:
                ops.attention_decode(q[P:], kc, vc, fb.decode_block_tables, fb.decode_ctx, self.scale, ws=decode_ws,
                                     max_ctx=fb.max_decode_ctx, out=attn[P:])
            h = ops.linear(attn.view(T, -1), w[p + "o"])
            ctx.tp_all_reduce(h)
            x = ops.rms_norm(h, w[p + "mlp_norm"], c.rms_eps, residual=res)
            h = self.moe_mlp(x, i, None)
            ctx.tp_all_reduce(h)
        if fb.sample_rows is not None:
            h = h.index_select(0, fb.sample_rows)
            res = res.index_select(0, fb.sample_rows)
        x = ops.rms_norm(h, w["norm"], c.rms_eps, residual=res)
        logits = ops.linear(x, w["lm_head"], out_dtype=torch.float32)
        if fb.tp_local_logits and ctx.tp_size > 1:
            return logits
        logits = ctx.tp_all_gather_last(logits)
        return logits[:, : c.vocab_size]

    @torch.no_grad()
    def reference_forward(self, token_ids: torch.Tensor, router_margin: list | None = None,
                          device: str | torch.device = "cpu") -> torch.Tensor:
        """Dense fp32 oracle (TP=1), plain PyTorch ops on ``device`` (the GPU for full-width layers, where the CPU
        would copy ~8 GB of fp32 experts per layer per call). ``router_margin`` (a list) receives, per token, the
        smallest gap over the layers between the router logits of its k-th and (k+1)-th expert: where that gap is
        within bf16 noise the bf16 engine may route the token to a different expert, a discontinuity no logit
        tolerance covers. Returns CPU fp32 logits."""
        c = self.cfg
        dev = torch.device(device)
        wf = {k: ops.natural_weight(v).to(dev, torch.float32) for k, v in self.w.items()}
        T, hd = token_ids.numel(), c.head_dim
        h = wf["embed"][token_ids.long().to(dev)]
        cs = self.cos_sin.to(dev)[:T]
        cos, sin = cs[:, None, : hd // 2], cs[:, None, hd // 2:]

        def rope(t):
            a, b = t[..., : hd // 2], t[..., hd // 2:]
            return torch.cat([a * cos - b * sin, b * cos + a * sin], -1)

        def rms(x, g):
            return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + c.rms_eps) * g

        for i in range(c.num_layers):
            p = f"l{i}."
            x = rms(h, wf[p + "attn_norm"])
            qkv = (x @ wf[p + "qkv"].t()).view(T, self.hq + 2 * self.hkv, hd)
            q, k_, v = qkv[:, : self.hq], qkv[:, self.hq: self.hq + self.hkv], qkv[:, self.hq + self.hkv:]
            q, k_ = rope(q), rope(k_)
            rep = self.hq // self.hkv
            k_, v = k_.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1)
            att = torch.einsum("qhd,khd->hqk", q, k_) * self.scale
            att = att.masked_fill(torch.ones(T, T, dtype=torch.bool, device=dev).triu(1)[None], float("-inf"))
            h = h + torch.einsum("hqk,khd->qhd", att.softmax(-1), v).reshape(T, -1) @ wf[p + "o"].t()
            x = rms(h, wf[p + "mlp_norm"])
            rl = x @ wf[p + "router"].t()
            if router_margin is not None:
                top = torch.topk(rl, min(c.top_k + 1, rl.shape[-1]), -1).values
                gap = top[:, c.top_k - 1] - top[:, -1] if top.shape[-1] > c.top_k else \
                    torch.full((T,), float("inf"), device=dev)
                margin = gap if i == 0 else torch.minimum(margin, gap)
            pr = rl.softmax(-1)
            tw, ti = torch.topk(pr, c.top_k, -1)
            tw = tw / tw.sum(-1, keepdim=True)
            out = torch.zeros_like(x)
            for e in range(c.num_experts):  # every expert over the tokens routed to it (same math per token)
                sel = (ti == e).nonzero()
                if sel.numel() == 0:
                    continue
                t_idx, j_idx = sel[:, 0], sel[:, 1]
                gu = (x[t_idx] @ wf[p + "w13"][e].t()).reshape(len(t_idx), -1, 2, 16)
                g = (torch.nn.functional.silu(gu[:, :, 0]) * gu[:, :, 1]).reshape(len(t_idx), -1)
                out.index_add_(0, t_idx, tw[t_idx, j_idx][:, None] * (g @ wf[p + "w2"][e].t()))
            h = h + out
        if router_margin is not None:
            router_margin.append(margin.cpu())
        return (rms(h, wf["norm"]) @ wf["lm_head"].t()).cpu()
