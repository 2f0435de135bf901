"""The one weight layout (ops.to_fragment_layout_): the in-place, row-chunked fragment shuffle equals the
out-of-place one, unshuffle_fragments inverts it, and natural_weight hands row-major data to everything outside
the native kernels (references, checkpoint export). The kernels that read the layout are covered by
tests/test_weight_layout_gpu.py."""
import torch

from generativeaiexamples_amd import ops


def test_in_place_chunked_shuffle_matches_and_inverts():
    torch.manual_seed(0)
    w = torch.randn(208, 1024).to(torch.bfloat16)
    want = ops.shuffle_fragments(w)
    for chunk in (16, 48, 100, 4096):  # 100 rounds down to 96: chunks stay inside 16-row groups
        got = ops.shuffle_fragments_(w.clone(), rows_per_chunk=chunk)
        assert torch.equal(got, want)
    assert torch.equal(ops.unshuffle_fragments(want), w)
    # fragment (nt, kt), lane l holds w[16 nt + (l & 15), 32 kt + 8 (l >> 4) : + 8]
    K = w.shape[1]
    nt, kt, lane = 3, 5, 37
    off = (nt * (K // 32) + kt) * 512 + lane * 8
    r, k = 16 * nt + (lane & 15), 32 * kt + 8 * (lane >> 4)
    assert torch.equal(want.view(-1)[off:off + 8], w[r, k:k + 8])


def test_natural_weight_of_marked_tensor():
    w = torch.randn(64, 512).to(torch.bfloat16)
    f = ops.shuffle_fragments(w)
    f._gai_frag = True
    assert ops.is_frag(f) and not ops.is_frag(w)
    assert torch.equal(ops.natural_weight(f), w)
    assert ops.natural_weight(w) is w


def test_cpu_weights_are_never_rewritten():
    w = torch.randn(64, 512).to(torch.bfloat16)
    w0 = w.clone()
    assert not ops.to_fragment_layout_(w)  # CPU tensors keep the row-major layout the reference ops read
    assert torch.equal(w, w0) and not ops.is_frag(w)
