"""MoE kernels on MI355X vs the fp32 reference: routing, grouped GEMM with row gather, combine; and the
interleaved SwiGLU epilogue kernel used with library GEMMs."""
import math

import pytest
import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _close(a, b, atol, rtol, what):
    err = (a.float().cpu() - b.float().cpu()).abs()
    assert (err <= atol + rtol * b.float().cpu().abs()).all(), f"{what}: max err {err.max():.4g}"


def test_moe_route(cuda):
    torch.manual_seed(0)
    logits = torch.randn(300, 8, device=cuda)
    ids, w = ops.moe_route(logits, 2)
    ids_r, w_r = ref.moe_route(logits.cpu(), 2)
    assert torch.equal(ids.cpu(), ids_r)
    _close(w, w_r, 1e-5, 1e-5, "route weights")


@pytest.mark.parametrize("T,E,k,D,I", [(1, 8, 2, 256, 512), (37, 8, 2, 512, 256), (700, 4, 2, 1024, 1024)])
def test_moe_gemm_and_combine(cuda, T, E, k, D, I):
    torch.manual_seed(T)
    x = torch.randn(T, D, device=cuda, dtype=torch.bfloat16)
    w13 = (torch.randn(E, 2 * I, D, device=cuda) / math.sqrt(D)).to(torch.bfloat16)
    w2 = (torch.randn(E, D, I, device=cuda) / math.sqrt(I)).to(torch.bfloat16)
    ids, w = ops.moe_route(torch.randn(T, E, device=cuda), k)
    a_rows, offs, pos = ops.moe_dispatch(ids, E)
    h1 = ops.moe_gemm(x, a_rows, w13, offs, T * k, True)
    h1_r = ref.moe_gemm(x.cpu(), a_rows.cpu(), w13.cpu(), offs.cpu(), T * k, True)
    _close(h1, h1_r, 3e-2, 2e-2, "w13 swiglu")
    y = ops.moe_gemm(h1, None, w2, offs, T * k, False)
    y_r = ref.moe_gemm(h1.cpu(), None, w2.cpu(), offs.cpu(), T * k, False)
    _close(y, y_r, 3e-2, 2e-2, "w2")
    res = torch.randn(T, D, device=cuda, dtype=torch.bfloat16)
    o = ops.moe_combine(y, pos, w, res)
    _close(o, ref.moe_combine(y.cpu(), pos.cpu(), w.cpu(), res.cpu()), 2e-2, 1e-2, "combine")


def test_silu_mul_interleaved(cuda):
    x = torch.randn(9, 2 * 512, device=cuda, dtype=torch.bfloat16)
    y = torch.empty(9, 512, device=cuda, dtype=torch.bfloat16)
    ops.native().silu_mul_interleaved(x, y)
    x4 = x.float().cpu().reshape(9, -1, 2, 16)
    _close(y, (torch.nn.functional.silu(x4[:, :, 0]) * x4[:, :, 1]).reshape(9, 512), 2e-2, 1e-2, "interleaved swiglu")


def test_tuned_linear_paths_agree(cuda):
    """Both GEMM paths the tuner may pick produce the same result for every epilogue."""
    torch.manual_seed(1)
    x = torch.randn(300, 1024, device=cuda, dtype=torch.bfloat16)
    w = (torch.randn(2048, 1024, device=cuda) / 32).to(torch.bfloat16)
    b = torch.randn(2048, device=cuda, dtype=torch.bfloat16)
    for act, bias in ((None, None), (None, b), ("swiglu", None), ("gelu", b)):
        old = ops.TUNER.mode
        try:
            ops.TUNER.mode = "native"
            y1 = ops.linear(x, w, bias=bias, act=act)
            ops.TUNER.mode = "hipblaslt"
            y2 = ops.linear(x, w, bias=bias, act=act)
        finally:
            ops.TUNER.mode = old
        _close(y1, y2, 3e-2, 2e-2, f"paths {act}")
