"""Op layer: every hot op of the framework, dispatched by tensor device.

* GPU tensors run the hand-written gfx950 HIP kernels in ``generativeaiexamples_amd._C``.
  If the extension is missing on a machine with a GPU this module raises - there
  is no silent PyTorch fallback for device tensors.
* CPU tensors run the fp32 reference implementations in :mod:`.reference` (the
  CPU plumbing configuration and the CPU test tier).
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import torch

from . import reference as ref
from .reference import BLOCK, interleave_gate_up, rope_cos_sin  # noqa: F401

_C = None
_C_ERR: Exception | None = None


def _into(out, y):
    """CPU path: honour a caller-provided output buffer."""
    if out is None:
        return y
    out.copy_(y.reshape(out.shape))
    return out


def native():
    """Return the loaded native module (raises if unavailable)."""
    global _C, _C_ERR
    if _C is None and _C_ERR is None:
        try:
            from .. import _C as mod  # type: ignore

            _C = mod
        except Exception as e:  # pragma: no cover - depends on build state
            _C_ERR = e
    if _C is None:
        raise RuntimeError(
            "generativeaiexamples_amd._C (gfx950 HIP kernels) is not built/loadable: "
            f"{_C_ERR!r}. Run `python -m generativeaiexamples_amd._build`."
        )
    return _C


def native_available() -> bool:
    try:
        native()
        return True
    except RuntimeError:
        return False


EPI = {None: 0, "bias": 1, "gelu": 2, "residual": 3, "swiglu": 4, "bias_residual": 5, "relu": 6}
_GEMM_FORCE = {"auto": 0, "skinny": 1, "tiled": 2}[os.environ.get("GAI_GEMM_KERNEL", "auto")]
# Plain (epilogue-free) GEMMs may use hipBLASLt when GAI_PLAIN_GEMM=hipblaslt; fused ones are always native.
_PLAIN_GEMM = os.environ.get("GAI_PLAIN_GEMM", "native")


# ---------------------------------------------------------------------------------------------
# normalisation
# ---------------------------------------------------------------------------------------------
def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None):
    """y = rmsnorm(x [+ residual]) * w. With ``residual``, it is updated in place to x + residual."""
    if not x.is_cuda:
        return _into(out, ref.rms_norm(x, w, eps, residual))
    out = torch.empty_like(x) if out is None else out
    native().rmsnorm(x, w, eps, out, residual, residual)
    return out


def layer_norm(x, w, b, eps, residual=None, out=None):
    if not x.is_cuda:
        return _into(out, ref.layer_norm(x, w, b, eps, residual))
    out = torch.empty_like(x) if out is None else out
    native().layernorm(x, w, b, eps, out, residual, residual)
    return out


# ---------------------------------------------------------------------------------------------
# GEMM
# ---------------------------------------------------------------------------------------------
def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
           residual: Optional[torch.Tensor] = None, act: Optional[str] = None, out_dtype=None,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = act(x @ w^T + bias) + residual on the MFMA GEMM with a fused epilogue.

    act: None | 'gelu' | 'relu' | 'swiglu' (w interleaved per 16 rows, see interleave_gate_up).
    """
    if not x.is_cuda:
        return _into(out, ref.linear(x, w, bias, residual, act, out_dtype))
    K = x.shape[-1]
    N = w.shape[0]
    lead = x.shape[:-1]
    M = x.numel() // K
    out_dtype = out_dtype or x.dtype
    if act == "swiglu":
        epi = EPI["swiglu"]
        assert bias is None and residual is None
        ncol = N // 2
    elif act == "gelu":
        assert bias is not None and residual is None
        epi, ncol = EPI["gelu"], N
    elif act == "relu":
        assert bias is not None and residual is None
        epi, ncol = EPI["relu"], N
    elif residual is not None:
        epi, ncol = (EPI["bias_residual"] if bias is not None else EPI["residual"]), N
    else:
        epi, ncol = (EPI["bias"] if bias is not None else 0), N
    if epi == 0 and _PLAIN_GEMM == "hipblaslt" and out is None and out_dtype == x.dtype:
        return torch.matmul(x, w.t())
    if out is None:
        out = torch.empty(*lead, ncol, dtype=out_dtype, device=x.device)
    if M == 0:
        return out
    x2 = x.reshape(M, K)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    native().gemm(x2, w, out, bias, residual, epi, _GEMM_FORCE)
    return out


# ---------------------------------------------------------------------------------------------
# RoPE + paged KV write, attention
# ---------------------------------------------------------------------------------------------
def rope_kv_write(qkv, positions, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, D, rope=True):
    if not qkv.is_cuda:
        return ref.rope_kv_write(qkv, positions, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, D, rope)
    native().rope_kv_write(qkv, positions, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, D, rope)


def prefill_rows_per_tile(Hq: int, Hkv: int) -> int:
    r = Hq // Hkv
    hpw = 4 if r >= 4 else 2 if r >= 2 else 1
    return 32 * (4 // hpw)


def build_prefill_tiles(q_lens: Sequence[int], Hq: int, Hkv: int, device) -> torch.Tensor:
    """Host-side varlen tile list [(seq, q_start), ...] for attention_prefill."""
    rows = prefill_rows_per_tile(Hq, Hkv)
    t = [(b, s) for b, n in enumerate(q_lens) for s in range(0, n, rows)]
    return torch.tensor(t, dtype=torch.int32).reshape(-1).to(device, non_blocking=True)


def attention_prefill(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale, causal=True, tiles=None,
                      q_lens: Sequence[int] | None = None, out=None):
    if not q.is_cuda:
        return _into(out, ref.attention_prefill(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale, causal))
    Hq, Hkv = q.shape[1], k_cache.shape[1]
    if tiles is None:
        if q_lens is None:
            cu = cu_q.tolist()
            q_lens = [cu[i + 1] - cu[i] for i in range(len(cu) - 1)]
        tiles = build_prefill_tiles(q_lens, Hq, Hkv, q.device)
    out = torch.empty_like(q) if out is None else out
    native().attn_prefill(q, k_cache, v_cache, block_tables, tiles, cu_q, ctx_lens, out, Hq, Hkv, scale, causal)
    return out


class DecodeWorkspace:
    """Split-KV partial buffers for attention_decode (sized once; graph-capture safe)."""

    def __init__(self, max_batch: int, Hq: int, D: int, max_ctx: int, device, split_keys: int | None = None):
        self.split_keys = split_keys or self.choose_split(max_ctx)
        self.max_splits = max(1, (max_ctx + self.split_keys - 1) // self.split_keys)
        self.o = torch.empty(self.max_splits * max_batch * Hq * D, dtype=torch.float32, device=device)
        self.ml = torch.empty(self.max_splits * max_batch * Hq * 2, dtype=torch.float32, device=device)

    @staticmethod
    def choose_split(max_ctx: int) -> int:
        # ~8-16 splits over the longest context, each a multiple of 128 keys (4 waves x 32)
        s = max(128, ((max_ctx // 12) + 127) // 128 * 128)
        return min(s, 2048)


def attention_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale, ws: DecodeWorkspace | None = None,
                     max_ctx: int | None = None, out=None):
    if not q.is_cuda:
        return _into(out, ref.attention_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale))
    B, Hq, D = q.shape
    if ws is None:
        mc = max_ctx if max_ctx is not None else int(ctx_lens.max())
        ws = DecodeWorkspace(B, Hq, D, mc, q.device)
    out = torch.empty_like(q) if out is None else out
    native().attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, out, ws.o, ws.ml, scale, ws.split_keys,
                         ws.max_splits)
    return out


# ---------------------------------------------------------------------------------------------
# sampling
# ---------------------------------------------------------------------------------------------
def sample(logits, temperature, top_p, top_k, seeds, step: int, out=None):
    if not logits.is_cuda:
        return ref.sample(logits, temperature, top_p, top_k, seeds, step)
    out = torch.empty(logits.shape[0], dtype=torch.int32, device=logits.device) if out is None else out
    native().sample(logits, temperature, top_p, top_k, seeds, int(step), out)
    return out


def apply_penalties(logits, tok_ids, tok_cnt, n, freq, pres, rep):
    if not logits.is_cuda:
        return ref.apply_penalties(logits, tok_ids, tok_cnt, n, freq, pres, rep)
    native().apply_penalties(logits, tok_ids, tok_cnt, n, freq, pres, rep)
    return logits


# ---------------------------------------------------------------------------------------------
# vector search
# ---------------------------------------------------------------------------------------------
def topk_cap(k: int) -> int:
    return 4 if k <= 4 else 8 if k <= 8 else 16 if k <= 16 else 32 if k <= 32 else 64


def sim_topk(Q: torch.Tensor, X: torch.Tensor, bias: torch.Tensor, n_rows: int, k: int, ws=None):
    """Top-k of Q @ X[:n_rows]^T + bias (exact). Returns (scores fp32 [nq,k], ids int64 [nq,k])."""
    if k > 64:
        raise ValueError("sim_topk supports k <= 64")
    k_eff = min(k, n_rows)
    if not Q.is_cuda or n_rows == 0:
        return ref.sim_topk(Q, X, bias, n_rows, k_eff)
    nq = Q.shape[0]
    rows_per_wg = max(128, ((n_rows + 1023) // 1024 + 127) // 128 * 128)
    rows_per_wg = min(rows_per_wg, 8192)
    nwg = (n_rows + rows_per_wg - 1) // rows_per_wg
    cap = topk_cap(k_eff)
    ws_v = torch.empty(nwg * nq * cap, dtype=torch.float32, device=Q.device)
    ws_i = torch.empty(nwg * nq * cap, dtype=torch.int32, device=Q.device)
    out_v = torch.empty(nq, k_eff, dtype=torch.float32, device=Q.device)
    out_i = torch.empty(nq, k_eff, dtype=torch.int64, device=Q.device)
    native().sim_topk(Q.contiguous(), X, bias, n_rows, k_eff, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i)
    return out_v, out_i


# ---------------------------------------------------------------------------------------------
# misc
# ---------------------------------------------------------------------------------------------
def embedding(ids, table, vstart: int = 0, vend: int | None = None, out=None):
    if not ids.is_cuda:
        return _into(out, ref.embedding(ids, table, vstart, vend))
    vend = table.shape[0] + vstart if vend is None else vend
    out = torch.empty(ids.numel(), table.shape[1], dtype=table.dtype, device=ids.device) if out is None else out
    native().embedding(ids.int().contiguous() if ids.dtype != torch.int32 else ids, table, out, vstart, vend)
    return out


POOL_MODES = {"mean": 0, "cls": 1, "last": 2}


def pool(h, cu_seqlens, mode: str = "mean", normalize: bool = True):
    if not h.is_cuda:
        return ref.pool(h, cu_seqlens, mode, normalize)
    out = torch.empty(cu_seqlens.numel() - 1, h.shape[-1], dtype=torch.float32, device=h.device)
    native().pool(h, cu_seqlens, out, POOL_MODES[mode], normalize)
    return out


def silu_mul(x):
    if not x.is_cuda:
        return ref.silu_mul(x)
    y = torch.empty(*x.shape[:-1], x.shape[-1] // 2, dtype=x.dtype, device=x.device)
    native().silu_mul(x, y)
    return y


def gelu(x):
    if not x.is_cuda:
        return ref.gelu(x)
    y = torch.empty_like(x)
    native().gelu(x, y)
    return y
