"""FM-radio baseband processing for the streaming ingest demo: the signal chain of the reference's
Holoscan SDR application (/root/reference/community/fm-asr-streaming-rag/sdr-holoscan/operators.py:42-73, 206-327;
parameters sdr-holoscan/params.yml) - a Hamming-window FIR low-pass of the complex64 bursts, FM demodulation by the
discrete-time phase differentiator, rational resampling to the 16 kHz the speech recogniser takes, and the float ->
PCM16 conversion.

GPU tensors run the HIP kernels of ``csrc/kernels/dsp.hip``; CPU tensors (the test tier) run the same math in torch.
Semantics follow the reference's cupyx.scipy.signal calls: ``lowpass`` = lfilter(taps, [1], x) with zero initial
state per burst, ``fm_demod`` = diff(unwrap(angle(x))), ``resample_poly`` = scipy's polyphase resampler with the
filter padded and offset the same way (length ceil(n up / down)). One deliberate difference: the reference derives
(up, down) = (1, round(fs_in / fs_out)) (1 / 62 for 1 MS/s -> 16 kHz, i.e. 16,129 Hz audio); ``rational_factors``
reduces fs_out / fs_in exactly (2 / 125).
"""
from __future__ import annotations

import functools
import math
from fractions import Fraction
from typing import Tuple

import numpy as np
import torch

_CPU_BLOCK = 1 << 18  # CPU fallbacks work in blocks of outputs (bounded temporary memory)

__all__ = ["firwin", "lowpass", "fm_demod", "resample_poly", "rational_factors", "float_to_pcm16", "resample_filter"]


def firwin(numtaps: int, cutoff: float, fs: float = 2.0, window: str = "hamming") -> np.ndarray:
    """Linear-phase low-pass FIR by the window method, unit gain at DC (scipy.signal.firwin's default
    ``pass_zero=True, scale=True`` form). ``cutoff`` in the units of ``fs``."""
    if numtaps < 1:
        raise ValueError("numtaps >= 1")
    fc = 2.0 * float(cutoff) / float(fs)  # relative to Nyquist
    if not 0.0 < fc < 1.0:
        raise ValueError("cutoff must lie strictly between 0 and fs / 2")
    m = np.arange(numtaps, dtype=np.float64) - (numtaps - 1) / 2.0
    h = fc * np.sinc(fc * m)
    if window == "hamming":
        w = 0.54 - 0.46 * np.cos(2.0 * np.pi * np.arange(numtaps) / max(numtaps - 1, 1)) if numtaps > 1 else np.ones(1)
    elif window in ("boxcar", "rect", None):
        w = np.ones(numtaps)
    else:
        raise ValueError(f"unsupported window {window!r}")
    h = h * w
    return h / h.sum()


def _native():
    from ... import ops

    return ops.native()


def lowpass(taps, x: torch.Tensor) -> torch.Tensor:
    """Causal FIR of a complex64 burst, zero initial state: y[n] = sum_j taps[j] x[n - j]."""
    if x.dtype != torch.complex64 or x.dim() != 1:
        raise ValueError("lowpass: 1-D complex64 input")
    h = taps.to(x.device, torch.float32) if isinstance(taps, torch.Tensor) else \
        torch.as_tensor(np.asarray(taps, dtype=np.float32), device=x.device)
    if x.is_cuda:
        y = torch.empty_like(x)
        _native().dsp_fir_complex(torch.view_as_real(x.contiguous()), h.contiguous(), torch.view_as_real(y))
        return y
    xr = torch.view_as_real(x).double()  # [n, 2]
    T, n = h.numel(), x.numel()
    xp = torch.nn.functional.pad(xr.t().unsqueeze(1), (T - 1, 0))  # [2, 1, n + T - 1]
    w = h.double().flip(0).view(1, 1, -1)
    # blocks of _CPU_BLOCK outputs (each reads T - 1 samples of history): bounded im2col memory for long inputs
    y = torch.cat([torch.nn.functional.conv1d(xp[..., s:s + min(_CPU_BLOCK, n - s) + T - 1], w)
                   for s in range(0, n, _CPU_BLOCK)], dim=-1) if n else xp[..., :0]
    return torch.view_as_complex(y.squeeze(1).t().float().contiguous())


def fm_demod(x: torch.Tensor) -> torch.Tensor:
    """FM discriminator: the phase step between consecutive samples (n - 1 outputs), diff(unwrap(angle(x)))."""
    if not torch.is_complex(x) or x.dim() != 1:
        raise ValueError("fm_demod: 1-D complex input")
    x = x.to(torch.complex64)
    if x.is_cuda:
        y = torch.empty(max(x.numel() - 1, 0), dtype=torch.float32, device=x.device)
        _native().dsp_fm_demod(torch.view_as_real(x.contiguous()), y)
        return y
    return torch.angle(x[1:] * torch.conj(x[:-1])).float()


def rational_factors(fs_in: float, fs_out: float, max_den: int = 100_000) -> Tuple[int, int]:
    """(up, down) with fs_in * up / down == fs_out (reduced)."""
    f = Fraction(fs_out / fs_in).limit_denominator(max_den) if not (float(fs_in).is_integer() and float(fs_out).is_integer()) \
        else Fraction(int(fs_out), int(fs_in))
    return f.numerator, f.denominator


def _upfirdn_len(ntaps: int, n_in: int, up: int, down: int) -> int:
    return ((n_in - 1) * up + ntaps - 1) // down + 1


def resample_filter(up: int, down: int, window: str = "hamming") -> Tuple[np.ndarray, int, int]:
    """The polyphase filter scipy.signal.resample_poly designs for (up, down) - firwin(20 max + 1, 1 / max) * up -
    with its leading zero padding: returns (taps, pre_remove, pad) for an input of any length (post padding is added
    per call)."""
    g = math.gcd(up, down)
    up, down = up // g, down // g
    max_rate = max(up, down)
    half_len = 10 * max_rate
    h = firwin(2 * half_len + 1, 1.0 / max_rate, window=window) * up
    n_pre_pad = down - half_len % down
    n_pre_remove = (half_len + n_pre_pad) // down
    return np.concatenate([np.zeros(n_pre_pad), h]), n_pre_remove, n_pre_pad


_DEVICE_TAPS: dict = {}


@functools.lru_cache(maxsize=64)
def _padded_filter(up: int, down: int, window: str, n: int) -> Tuple[np.ndarray, int, int]:
    h, pre_remove, _ = resample_filter(up, down, window)
    n_out = -(-n * up // down)
    while _upfirdn_len(len(h), n, up, down) < n_out + pre_remove:  # post padding, as scipy does
        h = np.concatenate([h, np.zeros(1)])
    return h, pre_remove, n_out


def resample_poly(x: torch.Tensor, up: int, down: int, window: str = "hamming", gain: float = 1.0) -> torch.Tensor:
    """Rational resampling of a real signal by up / down (scipy.signal.resample_poly semantics; output length
    ceil(n up / down)), times ``gain``."""
    if x.dim() != 1 or torch.is_complex(x):
        raise ValueError("resample_poly: 1-D real input")
    g = math.gcd(int(up), int(down))
    up, down = int(up) // g, int(down) // g
    x = x.float()
    if up == down == 1:
        return x * gain if gain != 1.0 else x.clone()
    n = x.numel()
    h, pre_remove, n_out = _padded_filter(up, down, window, n)
    if x.is_cuda:
        key = (up, down, window, n, str(x.device))
        ht = _DEVICE_TAPS.get(key)
        if ht is None:  # bursts have one size: the filter goes to the device once, not per call
            ht = _DEVICE_TAPS[key] = torch.as_tensor(h.astype(np.float32), device=x.device)
        y = torch.empty(n_out, dtype=torch.float32, device=x.device)
        _native().dsp_upfirdn(x.contiguous(), ht.contiguous(), up, down, pre_remove, float(gain), y)
        return y
    # CPU: only the kept outputs, polyphase - output m sits at t = (m + pre_remove) down of the zero-stuffed
    # convolution, where only taps i = t mod up + j up meet nonzero input x[(t - t mod up) / up - j]
    hd = torch.as_tensor(h, dtype=torch.float64)
    L = -(-len(h) // up)
    hp = torch.zeros(up, L, dtype=torch.float64)
    for k in range(up):
        hk = hd[k::up]
        hp[k, :hk.numel()] = hk
    xd = torch.nn.functional.pad(x.double(), (L, L))  # zero history / future
    j = torch.arange(L)
    out = torch.empty(n_out, dtype=torch.float64)
    for s0 in range(0, n_out, _CPU_BLOCK // 8):
        m = torch.arange(s0, min(n_out, s0 + _CPU_BLOCK // 8))
        t = (m + pre_remove) * down
        k = t % up
        base = (t - k) // up
        idx = (base[:, None] - j[None, :] + L).clamp_(0, xd.numel() - 1)
        out[m] = (xd[idx] * hp[k]).sum(1)
    return (out * gain).float()


def float_to_pcm16(x: torch.Tensor) -> torch.Tensor:
    """[-1, 1) float audio -> int16 PCM (clipped), the format the speech recogniser takes."""
    return torch.clamp(x * 32768.0, -32768.0, 32767.0).to(torch.int16)
