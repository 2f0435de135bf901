"""fp8 (OCP e4m3fn) quantiser + block-scaled MFMA GEMM vs fp32 references of the same op."""
import math

import pytest
import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def test_quant_rows_fp8_matches_reference(cuda):
    torch.manual_seed(5)
    x = torch.randn(77, 1024, device="cuda", dtype=torch.bfloat16) * 3
    q, s = ops.quant_fp8(x)
    qr, sr = ref.quant_rows_fp8(x.cpu())
    torch.testing.assert_close(s.cpu(), sr, rtol=1e-6, atol=0)
    # same reciprocal multiply and RNE rounding: at most a handful of codes one ulp apart
    diff = (q.cpu().float() - qr.float()).abs()
    assert (diff > 0).float().mean() < 1e-4
    rel = diff / qr.float().abs().clamp_min(1e-3)
    assert rel.max() <= 0.13


def test_gemm_fp8_exact_integers(cuda):
    """Small integers are exact in e4m3: with unit scales the GEMM must be exact (layout check with an
    asymmetric B)."""
    M, N, K = 64, 48, 256
    a = torch.randint(-3, 4, (M, K), device="cuda").float()
    b = (torch.arange(N, device="cuda")[:, None] % 5 - 2).float() * (torch.arange(K, device="cuda")[None] % 3 - 1)
    aq, bq = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
    one_m = torch.ones(M, device="cuda")
    one_n = torch.ones(N, device="cuda")
    out = torch.empty(M, N, device="cuda", dtype=torch.float32)
    ops.native().gemm_fp8(aq, bq, one_m, one_n, out, None, None, 0, 0)
    torch.testing.assert_close(out, a @ b.t(), rtol=0, atol=0)


@pytest.mark.parametrize("M,N,K", [(1, 256, 128), (77, 1000, 1024), (128, 4096, 4096), (300, 512, 1152),
                                   (2048, 1024, 4096)])
@pytest.mark.parametrize("act", [None, "bias", "quick_gelu", "swiglu", "residual"])
def test_linear_fp8_vs_reference(cuda, M, N, K, act):
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16) if act in ("bias", "quick_gelu") else None
    res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16) if act == "residual" else None
    a = act if act in ("quick_gelu", "swiglu") else None
    if a == "swiglu" and N % 32:
        pytest.skip("swiglu needs N % 32 == 0")
    W = ops.Fp8Weight.quantize(w)
    y = ops.linear_fp8(x, W, bias=bias, residual=res, act=a)
    xq, sx = ops.quant_fp8(x)
    r = ref.linear_fp8(xq.cpu(), sx.cpu(), W.q.cpu(), W.scale.cpu(), None if bias is None else bias.cpu(),
                       None if res is None else res.cpu(), a, torch.float32)
    torch.testing.assert_close(y.float().cpu(), r, rtol=2e-2, atol=2e-2)
    # and the fp8 result stays close to the bf16 op itself
    full = ref.linear(x.cpu(), w.cpu(), None if bias is None else bias.cpu(), None if res is None else res.cpu(), a,
                      torch.float32)
    err = (y.float().cpu() - full).norm() / full.norm().clamp_min(1e-6)
    assert err < 0.08, float(err)


@pytest.mark.parametrize("force", [2, 3])
@pytest.mark.parametrize("act", [None, "swiglu", "residual"])
def test_gemm_fp8_tiled_vs_large(cuda, force, act):
    """Both kernels (128x128 tiled, 256x256 pipelined) on a shape that is ragged in M and N."""
    M, N, K = 1100, 800, 1024
    torch.manual_seed(7)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16)
    res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16) if act == "residual" else None
    W = ops.Fp8Weight.quantize(w)
    xq, sx = ops.quant_fp8(x)
    ncol = N // 2 if act == "swiglu" else N
    out = torch.empty(M, ncol, device="cuda", dtype=torch.float32)
    epi = {None: 0, "swiglu": 4, "residual": 3}[act]
    ops.native().gemm_fp8(xq, W.q, sx, W.scale, out, None, res, epi, force)
    r = ref.linear_fp8(xq.cpu(), sx.cpu(), W.q.cpu(), W.scale.cpu(), None, None if res is None else res.cpu(),
                       act if act == "swiglu" else None, torch.float32)
    torch.testing.assert_close(out.cpu(), r, rtol=1e-3, atol=1e-3)


def test_gemm_fp8_large_exact_integers(cuda):
    M, N, K = 1024, 512, 512
    a = torch.randint(-3, 4, (M, K), device="cuda").float()
    b = (torch.arange(N, device="cuda")[:, None] % 5 - 2).float() * (torch.arange(K, device="cuda")[None] % 3 - 1)
    out = torch.empty(M, N, device="cuda", dtype=torch.float32)
    ops.native().gemm_fp8(a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn), torch.ones(M, device="cuda"),
                          torch.ones(N, device="cuda"), out, None, None, 0, 3)
    torch.testing.assert_close(out, a @ b.t(), rtol=0, atol=0)


@pytest.mark.parametrize("epi,what", [(1, "bias"), (3, "residual"), (5, "bias"), (9, "unknown")])
def test_gemm_epilogue_missing_operand_refused(cuda, epi, what):
    """An epilogue whose bias / residual operand is absent is refused on the host (the kernel would read
    address 0), for the bf16, split-K and fp8 GEMM entry points alike."""
    M, N, K = 256, 256, 256
    nat = ops.native()
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match=what):
        nat.gemm(x, w, out, None, None, epi, 0)
    W = ops.Fp8Weight.quantize(w)
    xq, sx = ops.quant_fp8(x)
    with pytest.raises(RuntimeError, match=what):
        nat.gemm_fp8(xq, W.q, sx, W.scale, out, None, None, epi, 0)
    ws = torch.empty(1 << 20, device="cuda", dtype=torch.float32)
    with pytest.raises(RuntimeError, match=what):
        nat.gemm_splitk(x[:8], w, out[:8], None, None, epi, ws, False)
    torch.cuda.synchronize()


def test_gemm_fp8_large_rule_deep_grid(cuda):
    """K = 1280 (the vision encoder's width): both fp8 kernels agree. The auto rule sends such a GEMM to the
    256x256 pipelined kernel once its grid is >= 8 waves of 256 tiles (e.g. the 204928 x 5120 fc1)."""
    M, N, K = 4096, 1280, 1280
    torch.manual_seed(3)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    W = ops.Fp8Weight.quantize((torch.randn(N, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16))
    xq, sx = ops.quant_fp8(x)
    outs = []
    for force in (2, 3):
        out = torch.empty(M, N, device="cuda", dtype=torch.float32)
        ops.native().gemm_fp8(xq, W.q, sx, W.scale, out, None, None, 0, force)
        outs.append(out)
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M", [1, 32, 64])
@pytest.mark.parametrize("act", [None, "swiglu"])
def test_fp8_weight_decode_copy(cuda, M, act):
    """Decode-sized GEMMs of an fp8 weight stream its dequantised bf16 copy in fragment order (Fp8Weight.dec):
    equal to the fp32 GEMM on the dequantised weight; wider rows keep the fp8 MFMA path."""
    torch.manual_seed(M)
    N, K = 4096, 4096
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    W = ops.Fp8Weight.quantize(w)
    assert ops.preshuffle_weight(W) and W.dec is not None and W.dec.dtype == torch.bfloat16
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    got = ops.linear(x, W, act=act).float()
    want = ref.linear(x.float().cpu(), W.dequantize(torch.float32).cpu(), act=act).float()
    torch.testing.assert_close(got.cpu(), want, rtol=2e-2, atol=2e-2)
    xl = torch.randn(200, K, device=cuda, dtype=torch.bfloat16)  # prefill-sized: fp8 operands as before
    got_l = ops.linear(xl, W, act=act).float().cpu()
    want_l = ref.linear(xl.float().cpu(), W.dequantize(torch.float32).cpu(), act=act).float()
    assert (got_l - want_l).abs().max() <= 0.1 * want_l.abs().max() + 0.05
