"""Persistent 256x256 prefill GEMMs (csrc/kernels/gemm.hip: w4p / w4d / w4r) against the fp32 reference.

Covers every epilogue, bf16 and fp32 output, partial M / N tiles, the ring tail (K / 32 close to the
ring depth) and launch-to-launch bit-repeatability (race screen for the counted-vmcnt pipeline)."""
import math

import pytest
import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
# force codes in gai_gemm: persistent 4-wave ring (tile walk per CU), persistent full-line double-unit kernel, and
# its 5-part LDS ring variant (the default for M >= 1024), and that ring on the stream-K walk (K % 128 == 0; forced
# onto shapes with K % 128 != 0 it takes the tile walk)
KERNELS = {"w4p": 8, "w4d": 9, "w4r": 10, "w4s": 11, "w4x": 12,  # w4x: the split walk (k-parts per tile)
           "w4d192": 13}  # the double-slot walk on 192-row tiles (6 A fragments per wave)

SHAPES = [(1024, 256, 192), (1280, 1040, 256), (2048, 2304, 1024), (1100, 4096, 4096), (4096, 6144, 320),
          (1536, 512, 14336), (4608, 4096, 192), (8192, 8448, 256),  # last two: > 256 tiles, multi-tile walks
          (2406, 4096, 1024)]  # the 2406-token O / down row count: 192-row tiles by the auto policy


def _run(x, w, bias, res, act, out_dtype=torch.bfloat16, force=4):
    M, N = x.shape[0], w.shape[0]
    ncol = N // 2 if act == "swiglu" else N
    if act == "swiglu":
        epi = ops.EPI["swiglu"]
    elif act in ("gelu", "relu"):
        epi = ops.EPI[act]
    elif res is not None:
        epi = ops.EPI["bias_residual"] if bias is not None else ops.EPI["residual"]
    else:
        epi = ops.EPI["bias"] if bias is not None else 0
    out = torch.full((M, ncol), float("nan"), device=x.device, dtype=out_dtype)
    ops.native().gemm(x, w, out, bias, res, epi, force)
    return out


@pytest.mark.parametrize("kern", list(KERNELS))
@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("act", [None, "bias", "gelu", "relu", "residual", "bias_residual", "swiglu"])
def test_ring_gemm(cuda, M, N, K, act, kern):
    if act == "swiglu" and N % 32:
        pytest.skip("SwiGLU weights interleave in 32-row groups")
    torch.manual_seed(M + 3 * N + K)
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda, dtype=torch.bfloat16) if act in ("bias", "gelu", "relu", "bias_residual") else None
    res = torch.randn(M, N, device=cuda, dtype=torch.bfloat16) if act in ("residual", "bias_residual") else None
    a = act if act in ("gelu", "relu", "swiglu") else None
    y = _run(x, w, bias, res, a, force=KERNELS[kern])
    y_ref = ref.linear(x.cpu(), w.cpu(), None if bias is None else bias.cpu(), None if res is None else res.cpu(), a)
    err = (y.float().cpu() - y_ref.float()).abs()
    tol = 3e-2 + 2e-2 * y_ref.float().abs()
    assert not torch.isnan(y).any(), "unwritten output elements"
    assert (err <= tol).all(), f"ring {M}x{N}x{K} {act}: max err {err.max():.4g}, {(err > tol).sum()} bad"


@pytest.mark.parametrize("kern", list(KERNELS))
@pytest.mark.parametrize("M,N,K", [(1024, 1024, 512), (1300, 2000, 1024)])
def test_ring_gemm_fp32_out(cuda, M, N, K, kern):
    torch.manual_seed(5)
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    y = _run(x, w, None, None, None, torch.float32, KERNELS[kern])
    y_ref = x.float().cpu() @ w.float().cpu().t()
    assert (y.cpu() - y_ref).abs().max() < 2e-3 + 2e-3 * y_ref.abs().max()


@pytest.mark.parametrize("kern", list(KERNELS))
@pytest.mark.parametrize("M,N,K", [(1024, 512, 256), (8192, 4352, 448)])
def test_ring_gemm_exact_layout(cuda, kern, M, N, K):
    """Small-integer operands make every product exact in fp32: any row/column mix-up in the swapped
    operand order or the permlane16 epilogue shows as a wrong integer (the second shape walks 2-3 tiles
    per CU in the persistent kernel, so a ring hand-over between tiles is checked exactly too)."""
    torch.manual_seed(9)
    x = torch.randint(-3, 4, (M, K), device=cuda).to(torch.bfloat16)
    w = torch.randint(-3, 4, (N, K), device=cuda).to(torch.bfloat16)
    y = _run(x, w, None, None, None, torch.float32, KERNELS[kern])
    assert torch.equal(y.cpu(), x.float().cpu() @ w.float().cpu().t())


@pytest.mark.parametrize("kern", list(KERNELS))
@pytest.mark.parametrize("M,N,K", [(4096, 4096, 4096), (2304, 6144, 1024)])
def test_ring_gemm_repeatable(cuda, M, N, K, kern):
    torch.manual_seed(11)
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    f = KERNELS[kern]
    y0 = _run(x, w, None, None, None, force=f)
    for _ in range(20):
        assert torch.equal(_run(x, w, None, None, None, force=f), y0)
    y_ref = ref.linear(x.cpu(), w.cpu())
    assert ((y0.float().cpu() - y_ref.float()).abs() <= 3e-2 + 2e-2 * y_ref.float().abs()).all()


@pytest.mark.parametrize("walk", ["w4s", "w4x"])
@pytest.mark.parametrize("M,N,K", [(256, 256, 8192), (300, 512, 1024), (2406, 4096, 14336), (1111, 1040, 640)])
@pytest.mark.parametrize("act", [None, "residual", "swiglu"])
def test_stream_k_split_tiles(cuda, M, N, K, act, walk):
    """Stream-K walk with tiles split many ways (64 contributors on the single tile of the first shape, 8 per tile
    on the second, the 2406-token down projection, odd tile edges on the last): small-integer operands make the
    fp32 partial sums exact, so any lost, doubled or misplaced partial quadrant shows as a wrong integer; then
    launch-to-launch bit equality (the sum order does not depend on which contributor finishes last). The split walk
    (w4x) cuts each tile into up to 8 k-parts over the same hand-off."""
    if act == "swiglu" and N % 32:
        pytest.skip("SwiGLU weights interleave in 32-row groups")
    torch.manual_seed(M + N + K)
    x = torch.randint(-2, 3, (M, K), device=cuda).to(torch.bfloat16)
    w = torch.randint(-2, 3, (N, K), device=cuda).to(torch.bfloat16)
    res = torch.randint(-8, 9, (M, N), device=cuda).to(torch.bfloat16) if act == "residual" else None
    out_dtype = torch.bfloat16 if act == "swiglu" else torch.float32  # the SwiGLU epilogue writes bf16
    y = _run(x, w, None, res, act, out_dtype, force=KERNELS[walk])
    acc = x.float().cpu() @ w.float().cpu().t()
    if act == "swiglu":
        g = acc.view(M, N // 32, 2, 16)
        ref_y = (torch.nn.functional.silu(g[:, :, 0]) * g[:, :, 1]).reshape(M, N // 2)
        torch.testing.assert_close(y.float().cpu(), ref_y, rtol=1e-2, atol=1e-2)
    else:
        assert torch.equal(y.cpu(), acc + (0 if res is None else res.float().cpu()))
    for _ in range(5):
        assert torch.equal(_run(x, w, None, res, act, out_dtype, force=KERNELS[walk]), y)


# one tile per workgroup (8192 x 1024: 128 tiles; 1300 x 6144; 2406 x 6144 with bias) and a multi-tile walk
# (8192 x 6144: 768 tiles, 3 per workgroup - the epilogue reads the next tile's first fragments after its stores)
@pytest.mark.parametrize("M,K,Hq,Hkv,with_bias", [(8192, 512, 4, 2, False), (1300, 4096, 32, 8, False),
                                                  (2406, 1024, 32, 8, True), (8192, 256, 32, 8, False)])
def test_prefill_qkv_rope_kv_fused(cuda, M, K, Hq, Hkv, with_bias):
    """Prefill QKV GEMM with RoPE + paged K / V^T write in its epilogue == gemm + rope_kv_write (same
    accumulators, same bf16 roundings); skipped slots (-1) leave the caches untouched."""
    torch.manual_seed(M + K)
    D, nblk = 128, (M + 15) // 16 + 8
    N = (Hq + 2 * Hkv) * D
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda, dtype=torch.bfloat16) if with_bias else None
    pos = torch.randint(0, 4096, (M,), device=cuda, dtype=torch.int32)
    slots = torch.randperm(nblk * 16, device=cuda)[:M].to(torch.int32)
    slots[::7] = -1
    cs = ops.rope_cos_sin(4096, D, 500000.0, device=cuda)
    outs = []
    for fused in (True, False):
        q = torch.full((M, Hq, D), float("nan"), device=cuda, dtype=torch.bfloat16)
        kc = torch.zeros(nblk, Hkv, 16, D, device=cuda, dtype=torch.bfloat16)
        vc = torch.zeros(nblk, Hkv, D, 16, device=cuda, dtype=torch.bfloat16)
        if fused:
            assert ops.native().gemm_rope_kv(x, w, bias, pos, cs, slots, q, kc, vc, Hq, Hkv, D, 1.0, 1.0,
                                             torch.empty(0, device=cuda), False, None)
        else:
            qkv = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
            # the fused kernel's tile walk (w4d): same accumulation order (the auto policy may pick the stream-K
            # walk, whose partial sums round differently)
            ops.native().gemm(x, w, qkv, bias, None, ops.EPI["bias"] if with_bias else 0, KERNELS["w4d"])
            ops.rope_kv_write(qkv, pos, cs, slots, q, kc, vc, Hq, Hkv, D, True)
        outs.append((q, kc, vc))
    # same accumulators and roundings; hipcc may contract the rotation's mul-sub into an FMA differently at
    # the two call sites, so a value that cancels to ~0 can differ in its last bit (as the decode test)
    for a, b in zip(*outs):
        torch.testing.assert_close(a.float(), b.float(), rtol=1e-2, atol=1e-5)
        assert (a != b).sum().item() <= max(2, a.numel() // 10000)
    assert not torch.isnan(outs[0][0]).any()
    assert outs[0][1].float().abs().sum() > 0 and outs[0][2].float().abs().sum() > 0  # caches written


def test_prefill_qkv_rope_kv_narrow_declines(cuda):
    """A QKV projection whose 256x256 tiles fill less than half the CUs (1024 x 1024: 16 tiles) is not fused: the
    call returns False and ops.linear_rope_kv takes the plain GEMM + rope_kv path, with the same results."""
    torch.manual_seed(2)
    M, K, Hq, Hkv, D = 1024, 512, 4, 2, 128
    N, nblk = (Hq + 2 * Hkv) * D, 1024 // 16 + 4
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    pos = torch.arange(M, device=cuda, dtype=torch.int32)
    slots = torch.arange(M, device=cuda, dtype=torch.int32)
    cs = ops.rope_cos_sin(4096, D, 500000.0, device=cuda)
    q = torch.empty(M, Hq, D, device=cuda, dtype=torch.bfloat16)
    kc = torch.zeros(nblk, Hkv, 16, D, device=cuda, dtype=torch.bfloat16)
    vc = torch.zeros(nblk, Hkv, D, 16, device=cuda, dtype=torch.bfloat16)
    assert not ops.native().gemm_rope_kv(x, w, None, pos, cs, slots, q, kc, vc, Hq, Hkv, D, 1.0, 1.0,
                                         torch.empty(0, device=cuda), False, None)
    ops.linear_rope_kv(x, w, None, pos, cs, slots, q, kc, vc, Hq, Hkv, D)
    qkv = ref.linear(x.cpu(), w.cpu())
    q2, k2, v2 = torch.empty(M, Hq, D), kc.cpu().float().zero_(), vc.cpu().float().zero_()
    ref.rope_kv_write(qkv, pos.cpu(), cs.cpu(), slots.cpu(), q2, k2, v2, Hq, Hkv, D)
    assert (q.float().cpu() - q2).abs().max().item() < 5e-2
    assert (kc.float().cpu() - k2).abs().max().item() < 5e-2
    assert (vc.float().cpu() - v2).abs().max().item() < 5e-2
