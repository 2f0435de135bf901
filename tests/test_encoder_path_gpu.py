"""Encoder self-attention path (BERT / E5 / CLIP / ViT): the page-packing kernel (ops.kv_pack) against the
per-(token, head) RoPE/KV writer with rotation off, the prefill attention reading q straight from the packed QKV rows
(strided q) against a contiguous q, and the fast branch-free GELU epilogue against PyTorch's exact erf GELU."""
import math

import pytest
import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.models.common import PackedAttention

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D,H", [(64, 16), (128, 8), (96, 4)])
def test_kv_pack_matches_rope_kv_writer(cuda, D, H):
    torch.manual_seed(D)
    lens = [1, 16, 17, 83, 130]
    T = sum(lens)
    qkv = torch.randn(T, 3 * H * D, device=cuda).to(torch.bfloat16)
    a = PackedAttention(lens, H, D, cuda)
    assert a.pack is not None
    ops.kv_pack(qkv, a.pack[0], a.pack[1], a.k_cache, a.v_cache, H, H, D)
    k2, v2 = torch.zeros_like(a.k_cache), torch.zeros_like(a.v_cache)
    q2 = torch.empty(T, H, D, device=cuda, dtype=torch.bfloat16)
    ops.rope_kv_write(qkv, a.positions, a.cs, a.slots, q2, k2, v2, H, H, D, rope=False)
    assert torch.equal(a.k_cache, k2) and torch.equal(a.v_cache, v2)
    # the CPU path of the op agrees too
    kc, vc = torch.zeros_like(a.k_cache).cpu(), torch.zeros_like(a.v_cache).cpu()
    ops.kv_pack(qkv.cpu(), a.pack[0].cpu(), a.pack[1].cpu(), kc, vc, H, H, D)
    assert torch.equal(kc, k2.cpu()) and torch.equal(vc, v2.cpu())


@pytest.mark.parametrize("D,H", [(64, 16), (128, 8)])
def test_packed_attention_strided_q_matches_fp32(cuda, D, H):
    torch.manual_seed(3)
    lens = [5, 64, 77, 512]
    T = sum(lens)
    qkv = torch.randn(T, 3 * H * D, device=cuda).to(torch.bfloat16)
    a = PackedAttention(lens, H, D, cuda)
    out = a(qkv, 1.0 / math.sqrt(D))
    kv = qkv.float().view(T, 3, H, D)
    ref, t0 = [], 0
    for n in lens:
        q, k, v = kv[t0:t0 + n, 0], kv[t0:t0 + n, 1], kv[t0:t0 + n, 2]
        s = torch.einsum("qhd,khd->hqk", q, k) / math.sqrt(D)
        ref.append(torch.einsum("hqk,khd->qhd", s.softmax(-1), v).reshape(n, H * D))
        t0 += n
    ref = torch.cat(ref)
    err = (out.float() - ref).abs().max().item()
    assert err < 2e-2, err


@pytest.mark.parametrize("M,N,K", [(8192, 4096, 1024), (300, 1024, 4096)])
def test_gelu_epilogue_matches_exact_erf(cuda, M, N, K):
    torch.manual_seed(M)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = (torch.randn(N, device=cuda) * 0.5).to(torch.bfloat16)
    y = ops.linear(x, w, bias=b, act="gelu")
    ref = torch.nn.functional.gelu(x.float() @ w.float().t() + b.float())
    err = (y.float() - ref).abs().max().item()
    assert err <= 2e-2 * max(1.0, ref.abs().max().item()), err
