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

import numpy as np
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


EPI = {None: 0, "bias": 1, "gelu": 2, "residual": 3, "swiglu": 4, "bias_residual": 5, "relu": 6, "quick_gelu": 7}
_GEMM_KERNELS = {"auto": 0, "skinny": 1, "tiled": 2, "w4p": 8, "w4d": 9, "w4r": 10, "w4s": 11, "w4x": 12, "w4d192": 13,
                 # names of round-3 kernels that the persistent 256x256 kernels replaced
                 "large": 9, "ring": 10}


def _gemm_force(name: str) -> int:
    if name not in _GEMM_KERNELS:
        raise ValueError(f"GAI_GEMM_KERNEL={name!r}: expected one of {sorted(_GEMM_KERNELS)}")
    return _GEMM_KERNELS[name]


_GEMM_FORCE = _gemm_force(os.environ.get("GAI_GEMM_KERNEL", "auto"))


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

    act: None | 'gelu' | 'relu' | 'quick_gelu' | 'swiglu' (w interleaved per 16 rows, see interleave_gate_up).
    An :class:`Fp8Weight` ``w`` routes to the fp8 MFMA GEMM (``linear_fp8``).
    """
    if act in ("geglu", "gelu_tanh"):
        # tanh-GELU family (Gemma GeGLU, StarCoder2 MLP): GEMM (+ bias) then one elementwise kernel
        assert residual is None and out is None
        y = linear(x, w, bias, out_dtype=None)
        y = geglu_interleaved(y) if act == "geglu" else gelu_tanh(y)
        return y if out_dtype in (None, y.dtype) else y.to(out_dtype)
    if isinstance(w, Fp8Weight):
        return linear_fp8(x, w, bias, residual, act, out_dtype, out)
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
    elif act in ("relu", "quick_gelu"):
        assert bias is not None and residual is None
        epi, ncol = EPI[act], N
    elif residual is not None:
        epi, ncol = (EPI["bias_residual"] if bias is not None else EPI["residual"]), N
    else:
        epi, ncol = (EPI["bias"] if bias is not None else 0), N
    if M == 0:
        return torch.empty(*lead, ncol, dtype=out_dtype, device=x.device) if out is None else out
    x2 = x.reshape(M, K)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    psw = decode_operand(w)
    if psw is not None and M <= 64:  # decode: weight stream from the fragment-shuffled copy
        if out is None:
            out = torch.empty(*lead, ncol, dtype=out_dtype, device=x.device)
        nat = native()
        ws = torch.empty(nat.gemm_splitk_ws_floats(M, N, K), dtype=torch.float32, device=x2.device)
        nat.gemm_splitk(x2, psw, out, bias, residual, epi, ws, True)
        return out
    if out is None:
        out = torch.empty(*lead, ncol, dtype=out_dtype, device=x.device)
    _native_gemm(x2, w, out, bias, residual, epi)
    return out


_SPLITK = os.environ.get("GAI_SPLITK", "1") == "1"


def linear_add_rmsnorm(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, norm_w: torch.Tensor, eps: float,
                       bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Decode tail of a row-parallel projection at TP = 1: ``residual += x @ w^T (+ bias)`` (bf16 rounding
    as the unfused pair) and return ``rmsnorm(residual) * norm_w``. For decode-sized M the split-K
    partials are reduced, added and normalised in ONE kernel (no separate reduce / norm launches);
    otherwise ``linear`` + ``rms_norm``."""
    K = x.shape[-1]
    M, N = x.numel() // K, w.shape[0]
    if (x.is_cuda and not isinstance(w, Fp8Weight) and _SPLITK and _GEMM_FORCE == 0 and M <= 64
            and native().gemm_splitk_fusable_norm(M, N, K)):
        nat = native()
        psw = decode_operand(w)
        ws = torch.empty(nat.gemm_splitk_ws_floats(M, N, K), dtype=torch.float32, device=x.device)
        out = torch.empty_like(residual)
        nat.gemm_splitk_add_rmsnorm(x.reshape(M, K).contiguous(), w if psw is None else psw, bias, residual,
                                    norm_w, out, eps, ws, psw is not None)
        return out
    return rms_norm(linear(x, w, bias), norm_w, eps, residual=residual)


def linear_rope_kv(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], positions, cos_sin, slots, q_out,
                   k_cache, v_cache, Hq: int, Hkv: int, D: int, k_scale=1.0, v_scale=1.0) -> None:
    """QKV projection + RoPE + paged KV write. For decode-sized M the split-K QKV partials are summed,
    rotated and scattered into q_out / the K, V^T caches by ONE kernel (no reduce launch, no bf16 qkv
    round trip, no rope_kv launch); for prefill (M >= 1024, head_dim 128, bf16 KV) the 256x256 GEMM's
    epilogue does the same; otherwise ``linear`` + ``rope_kv_write``. Same bf16 roundings."""
    K = x.shape[-1]
    M = x.numel() // K
    if x.is_cuda and not isinstance(w, Fp8Weight) and _SPLITK and _GEMM_FORCE == 0 and 1 <= M <= 64:
        nat = native()
        psw = decode_operand(w)
        ws = torch.empty(nat.gemm_splitk_ws_floats(M, w.shape[0], K), dtype=torch.float32, device=x.device)
        if nat.gemm_rope_kv(x.reshape(M, K).contiguous(), w if psw is None else psw, bias, positions, cos_sin, slots,
                            q_out, k_cache, v_cache, Hq, Hkv, D, k_scale, v_scale, ws, psw is not None,
                            tail_counters(x.device) if _QKV_TAIL else None):
            return
    if (x.is_cuda and not isinstance(w, Fp8Weight) and _GEMM_FORCE == 0 and M >= 1024
            and positions.dtype == torch.int32 and slots.dtype == torch.int32):
        # prefill: RoPE + paged KV write in the 256x256 GEMM's epilogue (no bf16 qkv round trip)
        ws = torch.empty(0, dtype=torch.float32, device=x.device)
        if native().gemm_rope_kv(x.reshape(M, K).contiguous(), w, bias, positions, cos_sin, slots, q_out, k_cache,
                                 v_cache, Hq, Hkv, D, k_scale, v_scale, ws, is_frag(w), None):
            return
    qkv = linear(x, w, bias=bias)
    rope_kv_write(qkv, positions, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, D, True, k_scale, v_scale)


# GAI_QKV_TAIL=1: the decode QKV partials are summed + rotated by the last-arriving K-slice inside the GEMM launch
# instead of the separate splitk_rope_kv launch. Off by default: at Llama-3-8B B = 64 the one reducer per head reads
# 8 x 64 x 128 fp32 slabs (256 KB) serially, 25.5 us vs 16.3 + 6.3 us for GEMM + tail launch
# (profiles/r3/qkv_tail_ab); the tail only pays when K-slices x slab bytes per tile are a few tens of KB.
_QKV_TAIL = os.environ.get("GAI_QKV_TAIL", "0") == "1"
_TAIL_CNT: dict = {}


def tail_counters(device) -> torch.Tensor:
    """Ticket counters of the in-launch split-K tails (one int32 per output tile). Zero between launches: the
    last-arriving K-slice of a tile resets its own counter. One buffer per (device, stream), since launches
    queued on one stream never overlap; graphs capture the buffer of their capture stream."""
    dev = torch.device(device)
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    t = _TAIL_CNT.get(key)
    if t is None:
        t = _TAIL_CNT[key] = torch.zeros(4096, dtype=torch.int32, device=dev)
    return t


def shuffle_fragments(w: torch.Tensor) -> torch.Tensor:
    """[N, K] -> the same [N, K]-shaped storage in MFMA B-fragment order [N/16][K/32][64 lanes][8]:
    lane l of fragment (nt, kt) holds w[16 nt + (l & 15), 32 kt + 8 (l >> 4) : +8]. A decode GEMM wave
    then streams 1 KiB contiguous per k32 step (8 full 128-B lines) instead of 16 half lines."""
    N, K = w.shape
    assert N % 16 == 0 and K % 32 == 0
    return w.view(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().view(N, K)


def shuffle_fragments_(w: torch.Tensor, rows_per_chunk: int = 4096) -> torch.Tensor:
    """shuffle_fragments in place, a chunk of rows (a multiple of 16) at a time: the permutation never leaves a 16-row
    group, so chunk r of the result is the shuffle of chunk r (transient memory: one chunk, not a second weight)."""
    step = max(16, rows_per_chunk - rows_per_chunk % 16)
    with torch.no_grad():
        for r0 in range(0, w.shape[0], step):
            blk = w[r0:r0 + step]
            blk.copy_(shuffle_fragments(blk))
    return w


def unshuffle_fragments(w: torch.Tensor) -> torch.Tensor:
    """Inverse of shuffle_fragments: a fragment-ordered [N, K] weight back in row-major [N, K] order (a new tensor)."""
    N, K = w.shape
    return w.view(N // 16, K // 32, 4, 16, 8).permute(0, 3, 1, 2, 4).contiguous().view(N, K)


def is_frag(w) -> bool:
    """True when ``w`` itself is stored in MFMA fragment order (to_fragment_layout_): every GEMM / GEMV path reads it
    so, and nothing keeps a row-major copy."""
    return bool(getattr(w, "_gai_frag", False))


def natural_weight(w) -> torch.Tensor:
    """``w`` in row-major [N, K] order (a new tensor when it is stored fragment-ordered): for plain-PyTorch references,
    checkpoint export and anything else outside the native kernels."""
    return unshuffle_fragments(w) if is_frag(w) else w


def to_fragment_layout_(w: torch.Tensor, rows_per_chunk: int = 4096) -> bool:
    """Rewrite a bf16 [N, K] CUDA weight IN PLACE into MFMA fragment order (shuffle_fragments) and mark it: the one
    weight layout (no second copy). The prefill GEMMs (tiled / 256x256 walks / stream-K / split walks, the QKV + RoPE
    epilogue), the skinny and split-K decode GEMMs and the batch <= 4 GEMV all read it directly. The permutation stays
    inside 16-row groups, so it runs in row chunks (transient memory: one chunk). Returns False (untouched) when the
    shape does not qualify (psw_qualifies) or the weight is 2 GiB or more (the 32-bit-offset kernels)."""
    if is_frag(w):
        return True
    if not psw_qualifies(w) or isinstance(w, Fp8Weight) or w.numel() * 2 >= (1 << 31) or not w.is_contiguous():
        return False
    shuffle_fragments_(w, rows_per_chunk)
    w._gai_frag = True  # the decode paths' fragment-ordered operand is the weight itself (decode_operand); no
    return True         # self-referencing attribute: that would be a reference cycle keeping the weight alive


def decode_operand(w):
    """The fragment-ordered bf16 operand the decode kernels stream for ``w``: the weight itself when it is stored
    fragment-ordered, its attached decode copy in the two-layout mode, else None."""
    if is_frag(w):
        return w
    return getattr(w, "_gai_psw", None)


def psw_qualifies(w) -> bool:
    """A bf16 [N, K] CUDA weight (or an fp8 one, whose decode copy is bf16) the fragment-shuffled decode layout
    takes (N % 16 == 0, K % 512 == 0, N >= 64)."""
    if isinstance(w, Fp8Weight):
        return w.q.is_cuda and w.q.dim() == 2 and not (w.q.shape[0] % 16 or w.q.shape[1] % 512 or w.q.shape[0] < 64)
    if not (isinstance(w, torch.Tensor) and w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 2):
        return False
    N, K = w.shape
    return not (N % 16 or K % 512 or N < 64)


def psw_bytes(w) -> int:
    """HBM the decode copy of w takes (bf16 for fp8 weights too)."""
    return w.numel() * 2


def preshuffle_weight(w) -> bool:
    """Attach a fragment-shuffled copy of a bf16 weight for the decode GEMM (M <= 64). Costs one extra
    copy of the weight in HBM (16 GB for Llama-3-8B: 288 GB per MI355X buys decode bandwidth). An Fp8Weight gets
    its dequantised values in that layout (Fp8Weight.dec). Returns False when the shape does not qualify
    (psw_qualifies)."""
    if not psw_qualifies(w):
        return False
    if isinstance(w, Fp8Weight):
        w.dec = shuffle_fragments(w.dequantize(torch.bfloat16))
        return True
    w._gai_psw = shuffle_fragments(w)
    return True


def _decode_psw_linear(x, psw, bias, residual, act, out_dtype, out):
    """Decode GEMM (M <= 64) from a fragment-ordered bf16 weight copy, with linear()'s epilogues."""
    K = x.shape[-1]
    M, N = x.numel() // K, psw.shape[0]
    if act == "swiglu":
        epi, ncol = EPI["swiglu"], N // 2
    elif act in ("gelu", "relu", "quick_gelu"):
        epi, ncol = EPI[act], N
    elif residual is not None:
        epi, ncol = (EPI["bias_residual"] if bias is not None else EPI["residual"]), N
    else:
        epi, ncol = (EPI["bias"] if bias is not None else 0), N
    if out is None:
        out = torch.empty(*x.shape[:-1], ncol, dtype=out_dtype or x.dtype, device=x.device)
    if M == 0:
        return out
    nat = native()
    ws = torch.empty(nat.gemm_splitk_ws_floats(M, N, K), dtype=torch.float32, device=x.device)
    nat.gemm_splitk(x.reshape(M, K).contiguous(), psw, out, bias, residual, epi, ws, True)
    return out


def _native_gemm(x2, w, out, bias, residual, epi):
    """Hand-written MFMA GEMM: the weight-streaming split-K kernel for decode-sized M (<= 64),
    otherwise the skinny / 128x128 / 256x256 kernels chosen inside gai_gemm (fragment-ordered weights too)."""
    M, K = x2.shape
    frag = is_frag(w)
    if _SPLITK and _GEMM_FORCE == 0 and M <= 64 and K % 512 == 0:
        nat = native()
        ws = torch.empty(nat.gemm_splitk_ws_floats(M, w.shape[0], K), dtype=torch.float32, device=x2.device)
        nat.gemm_splitk(x2, w, out, bias, residual, epi, ws, frag)
    else:
        native().gemm(x2, w, out, bias, residual, epi, _GEMM_FORCE, frag)


_FP8_FORCE = int(os.environ.get("GAI_FP8_FORCE", "0"))  # 0 auto, 2 tiled, 3 large


class Fp8Weight:
    """Per-output-channel OCP e4m3fn weight, quantised once at load time, plus its fp32 scales [N]. ``dec``:
    optional decode copy (the dequantised bf16 values in MFMA fragment order, preshuffle_weight) that decode-sized
    GEMMs stream instead of running the 128x128 fp8 tile kernel on a few rows."""

    __slots__ = ("q", "scale", "dec")

    def __init__(self, q: torch.Tensor, scale: torch.Tensor):
        self.q, self.scale, self.dec = q, scale, None

    @classmethod
    def quantize(cls, w: torch.Tensor) -> "Fp8Weight":
        q, s = quant_fp8(w)
        return cls(q, s)

    @property
    def shape(self):
        return self.q.shape

    @property
    def device(self):
        return self.q.device

    def data_ptr(self) -> int:
        return self.q.data_ptr()

    def numel(self) -> int:
        return self.q.numel()

    def dequantize(self, dtype=torch.bfloat16) -> torch.Tensor:
        return (self.q.float() * self.scale[:, None]).to(dtype)


def quant_fp8(x: torch.Tensor):
    """Per-row dynamic quantisation -> (q float8_e4m3fn [.., K], scale fp32 [rows])."""
    if not x.is_cuda:
        return ref.quant_rows_fp8(x)
    K = x.shape[-1]
    M = x.numel() // K
    x2 = x.reshape(M, K)
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    q = torch.empty(x.shape, dtype=torch.float8_e4m3fn, device=x.device)
    s = torch.empty(M, dtype=torch.float32, device=x.device)
    native().quant_rows_fp8(x2, q, s)
    return q, s


def linear_fp8(x: torch.Tensor, w: Fp8Weight, bias=None, residual=None, act=None, out_dtype=None, out=None):
    """``linear`` with fp8 operands: x is quantised per token on the fly (one fused pass), the K-loop
    runs on the block-scaled fp8 MFMA and the scales are applied in the fp32 epilogue."""
    out_dtype = out_dtype or x.dtype
    K = x.shape[-1]
    M = x.numel() // K
    if w.dec is not None and x.is_cuda and M <= 64 and act in (None, "swiglu", "gelu", "relu", "quick_gelu"):
        # decode: stream the fragment-ordered bf16 copy of the fp8 values (the 128x128 fp8 tile kernel ran the
        # Llama-3.2-11B decode projections at ~0.4 TB/s on <= 32 rows); bf16 activations, fp32 accumulation
        return _decode_psw_linear(x, w.dec, bias, residual, act, out_dtype, out)
    xq, sx = quant_fp8(x)
    if not x.is_cuda:
        return _into(out, ref.linear_fp8(xq, sx, w.q, w.scale, bias, residual, act, out_dtype))
    N = w.q.shape[0]
    if act == "swiglu":
        epi, ncol = EPI["swiglu"], N // 2
    elif act in ("gelu", "relu", "quick_gelu"):
        assert bias is not None and residual is None
        epi, ncol = EPI[act], N
    elif residual is not None:
        epi, ncol = (EPI["bias_residual"] if bias is not None else EPI["residual"]), N
    else:
        epi, ncol = (EPI["bias"] if bias is not None else 0), N
    if out is None:
        out = torch.empty(*x.shape[:-1], ncol, dtype=out_dtype, device=x.device)
    if M:
        native().gemm_fp8(xq.reshape(M, K), w.q, sx, w.scale, out, bias, residual, epi, _FP8_FORCE)
    return out


# One GEMM backend: every GEMM above is a hand-written gfx950 MFMA kernel (decode M <= 64: gemm_decode.hip /
# gemm_splitk.hip; prefill / encoder: the persistent 256x256 kernels of gemm.hip; fp8: gemm_fp8.hip). The
# same-box A/B against hipBLASLt (the library prefill GEMMs, profiles/r2/policy_ab*) lives in
# tools/blas_ab.py, outside the product code path.


# ---------------------------------------------------------------------------------------------
# RoPE + paged KV write, attention
# ---------------------------------------------------------------------------------------------
def rope_kv_write(qkv, positions, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, D, rope=True, k_scale=1.0,
                  v_scale=1.0):
    """KV caches are bf16, or torch.float8_e4m3fn (fp8 KV option: the cache holds x / {k,v}_scale)."""
    if not qkv.is_cuda:
        return ref.rope_kv_write(qkv, positions, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, D, rope,
                                 k_scale, v_scale)
    native().rope_kv_write(qkv, positions, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, D, rope, k_scale,
                           v_scale)


def kv_pack(qkv, blk_tok, blk_n, k_cache, v_cache, Hq: int, Hkv: int, D: int) -> None:
    """Encoder self-attention K / V (no RoPE) from the packed QKV rows [T, (Hq + 2 Hkv) D] into the pages of a transient
    paged cache: page b holds tokens blk_tok[b] .. + blk_n[b] (K [16][D], V^T [D][16]; rows past blk_n zeroed)."""
    if not qkv.is_cuda:
        kv = qkv.view(qkv.shape[0], Hq + 2 * Hkv, D)
        nb = blk_tok.numel()
        k_cache[:nb].zero_()
        v_cache[:nb].zero_()
        pages = torch.repeat_interleave(torch.arange(nb), blk_n.long())
        rows = torch.cat([torch.arange(n) for n in blk_n.tolist()]) if nb else pages
        tok = blk_tok.long()[pages] + rows
        k_cache[pages, :, rows] = kv[tok, Hq:Hq + Hkv].to(k_cache.dtype)
        v_cache[pages, :, :, rows] = kv[tok, Hq + Hkv:].to(v_cache.dtype)
        return
    native().kv_pack(qkv.contiguous(), blk_tok, blk_n, k_cache, v_cache, Hq, Hkv, D)


def prefill_rows_per_tile(Hq: int, Hkv: int, head_dim: int = 128) -> int:
    """Query rows per attention_prefill tile; the kernel launcher owns the choice (it follows the heads per wave of
    the prefill kernel, attention.hip prefill_hl), so GPU builds ask it."""
    if torch.cuda.is_available():
        return int(native().attn_prefill_rows_per_tile(Hq, Hkv, head_dim))
    r = Hq // Hkv
    hpw = 4 if r >= 4 else 2 if r >= 2 else 1
    waves = 8 if hpw == 4 and head_dim in (64, 128) and os.environ.get("GAI_ATTN_WAVES", "8") == "8" else 4
    return 32 * (waves // hpw)


def set_prefill_heads_per_wave(hl: int) -> None:
    """Prefill attention heads per wave (1 or 2; 2 applies to head_dim 128 with >= 4 q heads per kv head). Tile lists
    built before a change keep the old rows per tile: build them after setting it."""
    native().attn_prefill_set_hl(int(hl))


def prefill_tile_list(q_lens: Sequence[int], rows: int, ctx_lens: Sequence[int] | None = None) -> np.ndarray:
    """Varlen tile list [(seq, q_start), ...] for attention_prefill, longest first: a causal tile's work
    grows with its last query position (ctx - qlen + q_start + rows keys), and workgroups are dispatched
    roughly in tile order, so issuing the long tiles first keeps them off the tail of the grid
    (longest-processing-time-first scheduling). Grouping the tiles by sequence instead (for L2 reuse of a K/V
    prefix on the kernel's per-XCD kv heads) measured 1-7 % slower (profiles/r3/attn_prefill_xcd)."""
    t = [(b, s) for b, n in enumerate(q_lens) for s in range(0, n, rows)]
    if ctx_lens is None:
        ctx_lens = q_lens
    t.sort(key=lambda bs: -(int(ctx_lens[bs[0]]) - int(q_lens[bs[0]]) + bs[1]))
    return np.asarray(t, dtype=np.int32).reshape(-1, 2)


def build_prefill_tiles(q_lens: Sequence[int], Hq: int, Hkv: int, device,
                        ctx_lens: Sequence[int] | None = None, head_dim: int = 128) -> torch.Tensor:
    """Host-side varlen tile list [(seq, q_start), ...] for attention_prefill (longest tile first)."""
    t = prefill_tile_list(q_lens, prefill_rows_per_tile(Hq, Hkv, head_dim), ctx_lens)
    return torch.from_numpy(t).reshape(-1).to(device, non_blocking=True)


def attention_prefill(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale, causal=True, tiles=None,
                      q_lens: Sequence[int] | None = None, out=None, lse=None, k_scale=1.0, v_scale=1.0):
    """Varlen paged flash attention. ``lse`` (optional fp32 [T, Hq]) receives each row's natural-log
    softmax normaliser, used to merge partial attentions (parallel/context_parallel.py)."""
    if not q.is_cuda:
        o, l = ref.attention_prefill(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale, causal, return_lse=True,
                                     k_scale=k_scale, v_scale=v_scale)
        if lse is not None:
            lse.copy_(l)
        return _into(out, o)
    Hq, Hkv = q.shape[1], k_cache.shape[1]
    if tiles is None:
        if q_lens is None:
            cu = cu_q.tolist()
            q_lens = [cu[i + 1] - cu[i] for i in range(len(cu) - 1)]
        tiles = build_prefill_tiles(q_lens, Hq, Hkv, q.device, head_dim=q.shape[2])
    out = torch.empty_like(q) if out is None else out
    native().attn_prefill(q, k_cache, v_cache, block_tables, tiles, cu_q, ctx_lens, out, Hq, Hkv, scale, causal, lse,
                          k_scale, v_scale)
    return out


class DecodeWorkspace:
    """Split-KV partial buffers for attention_decode, sized once for the finest split (128 keys) so the
    split can be chosen per call / per captured batch bucket (graph-capture safe)."""

    MIN_SPLIT = 128

    def __init__(self, max_batch: int, Hq: int, D: int, max_ctx: int, device, split_keys: int | None = None):
        self.fixed_split = split_keys
        self.max_ctx = max_ctx
        self.max_splits = max(1, (max_ctx + self.MIN_SPLIT - 1) // self.MIN_SPLIT)
        self.o = torch.empty(self.max_splits * max_batch * Hq * D, dtype=torch.float32, device=device)
        self.ml = torch.empty(self.max_splits * max_batch * Hq * 2, dtype=torch.float32, device=device)
        # split tickets of the in-launch merge (one per (sequence, kv head) <= max_batch * Hq): zero at
        # allocation, reset by each merge's last split
        self.cnt = torch.zeros(max_batch * Hq, dtype=torch.int32, device=device)

    @property
    def split_keys(self) -> int:
        return self.fixed_split or self.choose_split(self.max_ctx)

    @staticmethod
    def choose_split(max_ctx: int, batch: int = 1, hkv: int = 8, target_wgs: int | None = None) -> int:
        """Split length (multiple of 128) giving ~target_wgs workgroups of (split, kv-head, sequence).
        The head_dim-128 kernel runs 3 workgroups per CU (VGPR-bound), i.e. 768 resident on 256 CUs.
        Round 4 (non-temporal K / V loads): 1024 target workgroups, i.e. 2 splits at B = 64, 8 kv heads. Measured on MI355X (B=64, 8 KV heads, ctx
        2.3-2.6k, profiles/r1/decode_attn_split_sweep_v2.jsonl): 896-key splits (1536 WGs) 5.34 TB/s vs
        768-key splits (2048 WGs = 2.67 waves, a 1/3-empty last wave) 5.04 TB/s; 256-key splits
        4.5 TB/s (per-workgroup prologue / combine not amortised)."""
        if target_wgs is None:
            # few (sequence, kv head) pairs - a TP shard with one kv head per rank, or <= 16 sequences at 8 kv heads -
            # take one resident wave (2 workgroups per CU): Llama-3-70B TP = 8 rank, B = 64, ctx 2500: 10.63 ->
            # 10.27 ms per decode step (profiles/r5/tp8_rank); Llama-3-8B ctx 2471 graph replay, B = 16: 4.51 ->
            # 4.36 ms, B = 8: 4.15 -> 3.92 ms (profiles/r6/decode/small_batch_split/); B = 64 (512 pairs) keeps 1024
            one_wave = batch * hkv <= (64 if hkv <= 2 else _DECODE_ONE_WAVE_PAIRS)
            target_wgs = 512 if one_wave and not _DECODE_TARGET_ENV else _DECODE_TARGET_WGS
        nsplit = max(1, -(-target_wgs // max(1, batch * hkv)))
        s = -(-max_ctx // nsplit)
        s = (s + 127) // 128 * 128
        # a few (sequence, kv head) pairs (batch 1-2 at 8 kv heads): the kernel is latency-bound, and 256-key splits
        # beat 128-key ones: batch 1 10.6-11.0 vs 11.7-12.2 us per layer (profiles/r5/gemv_b1/attn_b1_split_sweep.log),
        # decode step 3.00-3.03 -> 2.97-2.99 ms, batch 2 3.565 -> 3.512 ms (decode_small_batch.txt)
        lo = 256 if batch * hkv <= 16 and not _DECODE_TARGET_ENV else 128
        return int(min(max(s, lo), _DECODE_MAX_SPLIT))

    def split_for(self, batch: int, hkv: int, max_ctx: int) -> int:
        if self.fixed_split:
            return self.fixed_split
        return self.choose_split(max_ctx, batch, hkv)


# With the non-temporal K / V loads (attention.hip) two splits per (sequence, kv head) beat three at B = 64:
# ctx 2535 graph replay 7.68 -> 7.47 ms per step at 1024 target workgroups (768 the same, 2048 7.71;
# profiles/r4/decode/decode_nt_split_ab.txt). GAI_DECODE_TARGET_WGS overrides (sweeps).
_DECODE_TARGET_ENV = "GAI_DECODE_TARGET_WGS" in os.environ
_DECODE_TARGET_WGS = int(os.environ.get("GAI_DECODE_TARGET_WGS", "1024"))
_DECODE_MAX_SPLIT = int(os.environ.get("GAI_DECODE_MAX_SPLIT", "2048"))  # keys per split, upper bound (sweeps)
# up to this many (sequence, kv head) pairs the split targets one resident wave of workgroups (512) instead of 1024
_DECODE_ONE_WAVE_PAIRS = int(os.environ.get("GAI_DECODE_ONE_WAVE_PAIRS", "128"))
_DECODE_ADAPTIVE = os.environ.get("GAI_DECODE_ADAPTIVE", "1") == "1"


def attention_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale, ws: DecodeWorkspace | None = None,
                     max_ctx: int | None = None, out=None, k_scale=1.0, v_scale=1.0, qkv_fold=None):
    """qkv_fold = (slabs, ks, positions, cos_sin, slots) from :func:`qkv_fold_partials`: q is computed inside the
    launch from the QKV split-K partials (sum, bf16, RoPE) and the new key / value are written to the caches there;
    ``q`` is then only read for its shape."""
    if not q.is_cuda:
        return _into(out, ref.attention_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale, k_scale, v_scale))
    B, Hq, D = q.shape
    mc = max_ctx if max_ctx is not None else int(ctx_lens.max())
    if ws is None:
        ws = DecodeWorkspace(B, Hq, D, mc, q.device)
    split = ws.split_for(B, k_cache.shape[1], mc)
    nsplit = (mc + split - 1) // split
    if qkv_fold is not None:
        nsplit = max(nsplit, 2)  # the fold runs in the fused-merge kernel; surplus splits exit at once
    assert nsplit <= ws.max_splits, "decode workspace too small for this context"
    out = torch.empty_like(q) if out is None else out
    # adaptive (split_keys 0): the kernel cuts each sequence's ACTUAL context into nsplit equal parts, so graphs
    # captured for max_ctx balance their splits at every replay (GAI_DECODE_ADAPTIVE=0: fixed split_keys)
    f = qkv_fold if qkv_fold is not None else (None, 0, None, None, None)
    native().attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, out, ws.o, ws.ml, scale,
                         0 if (_DECODE_ADAPTIVE and ws.fixed_split is None) else split, nsplit, k_scale, v_scale,
                         ws.cnt if _ATTN_FUSE else None, f[0], f[1], f[2], f[3], f[4])
    return out


# Decode QKV tail folded into the decode-attention launch (attention.hip QP): the QKV projection writes only its split-K
# partial slabs, and attention_decode sums them, applies RoPE and writes the new key / value itself - one launch per
# layer fewer than the split-K RoPE / KV-write tail (GAI_QKV_FOLD=0: the tail kernel). Needs the default fused,
# non-temporal bf16 decode kernel.
_QKV_FOLD = (os.environ.get("GAI_QKV_FOLD", "1") == "1" and os.environ.get("GAI_DECODE_NT", "1") != "0"
             and os.environ.get("GAI_DECODE_VARIANT", "1") == "1")


def qkv_fold_partials(x: torch.Tensor, w, bias, k_cache, head_dim: int, ws: "DecodeWorkspace | None", k_scale=1.0,
                      v_scale=1.0):
    """Decode QKV projection for attention_decode(qkv_fold=...): launches the split-K partial slabs and returns
    (slabs, ks), or None when the fold does not apply (the caller then runs linear_rope_kv)."""
    if not (_QKV_FOLD and _ATTN_FUSE and _SPLITK and _GEMM_FORCE == 0 and x.is_cuda and bias is None
            and head_dim == 128 and k_cache.dtype == torch.bfloat16 and k_scale == 1.0 and v_scale == 1.0
            and ws is not None and ws.max_splits >= 2 and not isinstance(w, Fp8Weight)):
        return None
    K = x.shape[-1]
    M, N = x.numel() // K, w.shape[0]
    if not 1 <= M <= 64:
        return None
    nat = native()
    psw = decode_operand(w)
    slabs = torch.empty(nat.gemm_splitk_ws_floats(M, N, K), dtype=torch.float32, device=x.device)
    ks = nat.gemm_qkv_partials(x.reshape(M, K).contiguous(), w if psw is None else psw, slabs, psw is not None)
    return (slabs, int(ks)) if ks else None


def gemv_qkv_partials(x, W, gamma, eps: float, k_cache, head_dim: int, ws: "DecodeWorkspace | None", k_scale=1.0,
                      v_scale=1.0, ks: int = 2, out=None):
    """Batch-1 decode QKV as a K-split GEMV (gemv.hip GV_PART, the attention RMSNorm staged in) for
    attention_decode(qkv_fold=...): (slabs [ks, M, N] fp32, ks), or None when the fold does not apply (the caller
    then runs gemv_rope_kv). 2 K parts x N / 16 columns of 4 waves: 768 workgroups for Llama-3-8B's 6144 rows instead
    of gemv_rope_kv's 192 column pairs, and the RoPE / KV-write epilogue moves into the attention prologue."""
    if not (_QKV_FOLD and _ATTN_FUSE and x.is_cuda and is_frag(W) and head_dim == 128
            and k_cache.dtype == torch.bfloat16 and k_scale == 1.0 and v_scale == 1.0 and ws is not None
            and ws.max_splits >= 2 and (W.shape[1] // 32) % (ks * 16) == 0):
        return None
    return gemv(x, W, gamma, eps, "part", out=out, ks=ks), ks


# Decode-attention splits are merged inside the attention launch by the last-arriving split (write-through sc1
# partials + a relaxed ticket, no fence): Llama-3-8B B = 64, ctx 2600 eager forward 7.918 -> 7.738 ms, headline
# 16.92 -> 17.08 q/s (profiles/r3/attn_fused_merge_ab). The first form, with a per-workgroup agent release, was
# 192.6 vs 117.4 us per layer. GAI_ATTN_FUSE=0: the separate attn_decode_reduce launch.
_ATTN_FUSE = os.environ.get("GAI_ATTN_FUSE", "1") == "1"


# ---------------------------------------------------------------------------------------------
# sampling
# ---------------------------------------------------------------------------------------------
def sample(logits, temperature, top_p, top_k, seeds, step: int, out=None):
    if not logits.is_cuda:
        return _into(out, ref.sample(logits, temperature, top_p, top_k, seeds, step).to(torch.int32))
    out = torch.empty(logits.shape[0], dtype=torch.int32, device=logits.device) if out is None else out
    nat = native()
    nb = nat.sample_ws_bytes(logits.shape[0], logits.shape[1])  # split-row path (V >= 16K): 3 small kernels
    ws = torch.empty(nb, dtype=torch.uint8, device=logits.device) if nb else None
    nat.sample(logits, temperature, top_p, top_k, seeds, int(step), out, ws)
    return out


TP_SAMPLE_CANDIDATES = int(os.environ.get("GAI_TP_SAMPLE_CANDIDATES", "64"))
_TP_FLAGS: dict = {}


def tp_sample_flags(device) -> torch.Tensor:
    """Device counter of TP-sampled rows whose nucleus / top-k reached past the gathered candidates (the draw
    was then restricted to them); 0 means every draw was exact."""
    key = str(device)
    if key not in _TP_FLAGS:
        _TP_FLAGS[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return _TP_FLAGS[key]


def sample_tp(logits_local, ctx, vstart: int, vocab: int, temperature, top_p, top_k, seeds, step: int, out=None,
              candidates: int | None = None):
    """Sampling from vocab-parallel logits [B, V/tp] without gathering them (Llama TP decode).

    Each rank reduces its shard to a small packet per row: max, softmax mass, its Gumbel-max (exact pure
    temperature sampling) and its top-C logits with global ids. The packets are gathered with ONE small
    TP all-reduce of a zero-padded [tp, B, W] buffer (the peer-memory kernel on GPU: graph-capturable, no
    RCCL), and every rank resolves the same token with ``sample_tp_resolve`` - the whole-row sampler's
    nucleus and Gumbel noise, exact whenever the cut lies inside the candidates (flagged otherwise,
    :func:`tp_sample_flags`). At Llama-3-70B TP=8, B=64 that is 8 x 64 x 528 B instead of a
    [64, 128256] fp32 all-gather (32 MB) per decode step. CPU tensors: full gather + the reference sampler."""
    B = logits_local.shape[0]
    if not logits_local.is_cuda:
        full = ctx.tp_all_gather_last(logits_local.contiguous())[:, :vocab]
        return sample(full.contiguous(), temperature, top_p, top_k, seeds, step, out=out)
    C = int(candidates or TP_SAMPLE_CANDIDATES)
    nat = native()
    n = max(1, min(logits_local.shape[1], vocab - vstart))
    c = min(C, n)
    W = (4 + 2 * C + 3) // 4 * 4
    R = ctx.tp_size
    buf = torch.zeros(R, B, W, dtype=torch.float32, device=logits_local.device)
    pk = buf[ctx.tp_rank]
    nat.sample_tp_stats(logits_local, int(vstart), int(vocab), temperature, seeds, int(step), pk[:, :4])
    vals, idx = torch.topk(logits_local[:, :n], c, dim=-1)
    pk[:, 4:4 + c] = vals
    pk[:, 4 + c:4 + C] = float("-inf")
    pk[:, 4 + C:4 + C + c] = (idx + vstart).float()
    ctx.tp_all_reduce(buf)
    out = torch.empty(B, dtype=torch.int32, device=logits_local.device) if out is None else out
    nat.sample_tp_resolve(buf, C, int(vocab), temperature, top_p, top_k, seeds, int(step), out,
                          tp_sample_flags(logits_local.device))
    return out


def token_mask(logits, rows, mask):
    """Constrained decoding: logits[rows[r], t] = -inf where bit t of mask[r] (int32 words) is clear."""
    if not logits.is_cuda:
        return ref.token_mask(logits, rows, mask)
    native().token_mask(logits, rows, mask)
    return logits


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
    if topk_cap(k_eff) <= 8:
        # streaming kernel: ~one workgroup per CU, its bias rows staged in LDS (<= 4096 rows)
        rows_per_wg = min(4096, max(128, ((n_rows + 255) // 256 + 127) // 128 * 128))
    else:
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


def topk_merge(vals: torch.Tensor, k: int):
    """Merge W descending-sorted candidate lists per query: vals [W, Q, n] fp32 -> (top values [Q, k], positions
    [Q, k] int64 into the flattened [W * n] candidates of the query, w * n + j). On the GPU: the similarity top-k's
    second-stage kernel (topk.hip sim_topk_stage2). The sharded index's cross-shard merge."""
    W, Q, n = vals.shape
    k = min(k, W * n)
    if not vals.is_cuda or Q == 0 or k > 64:
        flat = vals.permute(1, 0, 2).reshape(Q, W * n)
        return torch.topk(flat, k, dim=1)
    cap = topk_cap(k)
    v = vals.float()
    if n != cap:  # every list holds exactly `cap` entries (the kernel's K), padded with -inf
        pad = v.new_full((W, Q, cap), float("-inf"))
        pad[:, :, : min(n, cap)] = v[:, :, :cap]
        v = pad
    pos = (torch.arange(W, device=v.device, dtype=torch.int32)[:, None, None] * n
           + torch.arange(cap, device=v.device, dtype=torch.int32)[None, None, :]).expand(W, Q, cap).contiguous()
    out_v = torch.empty(Q, k, dtype=torch.float32, device=v.device)
    out_i = torch.empty(Q, k, dtype=torch.int64, device=v.device)
    native().topk_merge(v.contiguous(), pos, k, out_v, out_i)
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


def decode_advance(toks, ids, pos, ctx, slots, block_tables, n_valid):
    """In-place multi-step decode update for rows < n_valid[0]: ids <- toks, pos += 1, ctx = pos + 1,
    slots from block_tables (int32 tensors; graph-capturable: the row count is read on device)."""
    if not ids.is_cuda:
        return ref.decode_advance(toks, ids, pos, ctx, slots, block_tables, n_valid, BLOCK)
    native().decode_advance(toks, ids, pos, ctx, slots, block_tables, n_valid, BLOCK)


def moe_route(logits: torch.Tensor, k: int, renorm: bool = True):
    """Router softmax + top-k -> (expert ids int32 [T,k], weights fp32 [T,k])."""
    if not logits.is_cuda:
        return ref.moe_route(logits, k, renorm)
    T = logits.shape[0]
    ids = torch.empty(T, k, dtype=torch.int32, device=logits.device)
    w = torch.empty(T, k, dtype=torch.float32, device=logits.device)
    native().moe_route(logits.float().contiguous(), k, renorm, ids, w)
    return ids, w


_MOE_DISPATCH_MAX = int(os.environ.get("GAI_MOE_DISPATCH_MAX", "8192"))


def moe_dispatch(ids: torch.Tensor, num_experts: int):
    """Expert-sorted dispatch plan without host sync: (a_rows [T*k], offsets [E+1], pos [T,k]).
    Up to _MOE_DISPATCH_MAX rows (decode steps) one single-workgroup counting-sort kernel builds it; larger
    steps keep the stable argsort (the one workgroup walks rows 256 at a time: level at ~16K rows,
    profiles/r3/moe_dispatch/dispatch_microbench.txt)."""
    T, k = ids.shape
    if ids.is_cuda and 0 < T * k <= _MOE_DISPATCH_MAX:
        dev = ids.device
        a_rows = torch.empty(T * k, dtype=torch.int32, device=dev)
        offs = torch.empty(num_experts + 1, dtype=torch.int32, device=dev)
        pos = torch.empty(T, k, dtype=torch.int32, device=dev)
        native().moe_dispatch(ids.to(torch.int32).contiguous(), num_experts, a_rows, offs, pos)
        return a_rows, offs, pos
    flat = ids.reshape(-1).long()
    order = torch.argsort(flat, stable=True)
    a_rows = (order // k).to(torch.int32)
    counts = torch.zeros(num_experts, dtype=torch.int64, device=ids.device).scatter_add_(0, flat, torch.ones_like(flat))
    offs = torch.zeros(num_experts + 1, dtype=torch.int32, device=ids.device)
    offs[1:] = counts.cumsum(0).to(torch.int32)
    pos = torch.empty(T * k, dtype=torch.int32, device=ids.device)
    pos[order] = torch.arange(T * k, dtype=torch.int32, device=ids.device)
    return a_rows, offs, pos.view(T, k)


_GEMV_EPI = {"plain": 0, "residual": 1, "swiglu": 2, "f32": 4, "part": 5}


def gemv_ok(M: int, N: int, K: int, normed: bool = False) -> bool:
    """Shapes the small-batch decode GEMV (gemv.hip) takes: 1..4 rows, K a multiple of 2048, the staged activation
    rows within LDS, K <= 8192 when it normalises its input."""
    return (1 <= M <= 4 and N % 2 == 0 and K % 2048 == 0 and M * K * 2 <= 160 * 1024
            and (not normed or K <= 8192))


def gemv(x, W, gamma=None, eps: float = 1e-5, epi: str = "plain", res=None, out=None, swi=None, ks: int = 1):
    """Decode GEMV for 1..4 token rows with the consumer's RMSNorm staged in (``gamma``) and the epilogue fused:
    plain bf16, ``residual`` (res = bf16(bf16(x W^T) + res) in place), ``swiglu`` on the [gate16 | up16]
    interleave, ``f32`` logits, ``part`` = fp32 partial sums of ``ks`` K parts [ks, M, N] (the QKV slabs
    attention_decode(qkv_fold=...) folds). ``swi`` (fragment-ordered W): the input is bf16(silu(g) * u) of that fp32
    [M, 2K] gate_up interleave, computed while staging (x is then ignored)."""
    src = swi if swi is not None else x
    if not src.is_cuda:
        r = ref.gemv(x, W, gamma, eps, epi, res, swi, ks)
        return _into(out, r) if epi != "residual" else r
    M, N = src.shape[0], W.shape[0]
    xa = src if swi is not None else x.contiguous()  # (not read when swi is given)
    if epi == "residual":
        native().gemv(xa, gamma, eps, W, 1, None, res, is_frag(W), swi, ks)
        return res
    if out is None:
        cols = N // 2 if epi == "swiglu" else N
        shape = (ks, M, N) if epi == "part" else (M, cols)
        out = torch.empty(shape, dtype=torch.float32 if epi in ("f32", "part") else x.dtype, device=src.device)
    native().gemv(xa, gamma, eps, W, _GEMV_EPI[epi], out, None, is_frag(W), swi, ks)
    return out


def gemv_rope_kv(x, W, gamma, eps, positions, cos_sin, slots, q_out, k_cache, v_cache, Hq: int, Hkv: int):
    """QKV GEMV (+ the attention RMSNorm staged in) + RoPE + q / paged K, V^T stores: the batch <= 4 decode
    counterpart of linear_rope_kv, no split-K slabs and no tail launch."""
    native().gemv_rope_kv(x.contiguous(), gamma, eps, W, positions, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv,
                          is_frag(W))


def ep_dispatch_plan(ids: torch.Tensor, world: int, e_local: int):
    """Expert-parallel send plan of the (token, choice) pairs: (offs [W+1], pos [T, k], a_pairs [T*k]) = the pairs
    counting-sorted by destination rank id // e_local (moe_dispatch's kernel with a bucket divisor), sync-free."""
    T, k = ids.shape
    if ids.is_cuda and 0 < T * k <= _MOE_DISPATCH_MAX:
        dev = ids.device
        a_rows = torch.empty(T * k, dtype=torch.int32, device=dev)
        a_pairs = torch.empty(T * k, dtype=torch.int32, device=dev)
        offs = torch.empty(world + 1, dtype=torch.int32, device=dev)
        pos = torch.empty(T, k, dtype=torch.int32, device=dev)
        native().moe_dispatch_by(ids.to(torch.int32).contiguous(), world, e_local, a_rows, offs, pos, a_pairs)
        return offs, pos, a_pairs
    return ref.ep_dispatch_plan(ids, world, e_local)


def ep_pack(x: torch.Tensor, ids: torch.Tensor, offs, a_pairs, world: int, capacity: int, e_local: int,
            ids_in_rows: bool = False):
    """-> (send slabs [W*C, D], local expert ids [W*C] int32; padding rows carry the sentinel e_local).
    ids_in_rows: slabs are [W*C, D + 8] with each row's expert id stored as an int32 in its tail (one exchange
    moves rows and ids); the second result is then None."""
    if not x.is_cuda:
        send, eid = ref.ep_pack(x, ids, offs, a_pairs, world, capacity, e_local)
        if ids_in_rows:
            tail = torch.zeros(send.shape[0], 8, dtype=send.dtype)
            tail[:, :2] = eid.view(torch.bfloat16).view(-1, 2)
            return torch.cat([send, tail], 1), None
        return send, eid
    D = x.shape[1]
    send = torch.empty(world * capacity, D + 8 if ids_in_rows else D, dtype=x.dtype, device=x.device)
    eid = None if ids_in_rows else torch.empty(world * capacity, dtype=torch.int32, device=x.device)
    native().ep_pack(x.contiguous(), ids.to(torch.int32).contiguous(), offs, a_pairs, world, capacity, e_local, send,
                     eid)
    return send, eid


def ep_combine(back, ids, pos, offs, w, residual, e_local: int, capacity: int):
    """out[t] = sum_j w[t, j] * back[slab row of (t, j)] (+ residual): the returned expert outputs, weighted."""
    if not back.is_cuda:
        return ref.ep_combine(back, ids, pos, offs, w, residual, e_local, capacity)
    out = torch.empty(ids.shape[0], back.shape[1], dtype=back.dtype, device=back.device)
    native().ep_combine(back.contiguous(), ids.to(torch.int32).contiguous(), pos.contiguous(), offs,
                        w.to(torch.float32).contiguous(), residual, e_local, capacity, out)
    return out


def moe_gemm(A, a_rows, W, offs, rows_total: int, swiglu: bool):
    """Grouped expert GEMM over expert-sorted rows (A rows gathered through a_rows when given)."""
    if not A.is_cuda:
        return ref.moe_gemm(A, a_rows, W, offs, rows_total, swiglu)
    N = W.shape[1]
    C = torch.empty(rows_total, N // 2 if swiglu else N, dtype=A.dtype, device=A.device)
    native().moe_gemm(A.contiguous(), a_rows, W, C, offs, rows_total, swiglu)
    return C


def moe_combine(Y, pos, w, residual=None):
    if not Y.is_cuda:
        return ref.moe_combine(Y, pos, w, residual)
    out = torch.empty(pos.shape[0], Y.shape[1], dtype=Y.dtype, device=Y.device)
    native().moe_combine(Y, pos, w, residual, out)
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


def gelu_tanh(x):
    """tanh-approximated GELU (HF ``gelu_pytorch_tanh``: StarCoder2, Gemma)."""
    if not x.is_cuda:
        return ref.gelu_tanh(x)
    y = torch.empty_like(x)
    native().gelu_tanh(x, y)
    return y


def geglu_interleaved(x):
    """gelu_tanh(gate) * up on the interleaved-per-16 [gate16|up16] layout -> width / 2 (Gemma MLP)."""
    if not x.is_cuda:
        return ref.geglu_interleaved(x)
    y = torch.empty(*x.shape[:-1], x.shape[-1] // 2, dtype=x.dtype, device=x.device)
    native().geglu_interleaved(x, y)
    return y


# ---------------------------------------------------------------------------------------------- vision
def patchify(img: torch.Tensor, patch: int, mean: torch.Tensor, inv_std: torch.Tensor, Kp: int) -> torch.Tensor:
    """Normalise + im2col an image batch [B, C, H, W] fp32 into bf16 patch rows [B * gh * gw, Kp]."""
    if not img.is_cuda:
        return ref.patchify(img, patch, mean, inv_std, Kp)
    B, C, H, W = img.shape
    out = torch.empty(B * (H // patch) * (W // patch), Kp, dtype=torch.bfloat16, device=img.device)
    native().patchify(img.contiguous(), patch, mean, inv_std, out)
    return out


def vit_embed(patches: torch.Tensor, cls: torch.Tensor, pos: torch.Tensor, B: int) -> torch.Tensor:
    """[CLS | patch embeddings] + position embeddings -> packed token rows [B * (NP + 1), D]."""
    if not patches.is_cuda:
        return ref.vit_embed(patches, cls, pos, B)
    D = cls.numel()
    NP = patches.numel() // (B * D)
    out = torch.empty(B * (NP + 1), D, dtype=torch.bfloat16, device=patches.device)
    native().vit_embed(patches, cls, pos, out, B)
    return out
