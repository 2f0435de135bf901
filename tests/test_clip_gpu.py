"""CLIP (ViT-L/14 geometry) on the HIP kernels vs an fp32 PyTorch reference of the same weights."""
import pytest
import torch
import torch.nn.functional as F

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.models.clip import CLIP_MEAN, CLIP_STD, ClipConfig, ClipModel
from generativeaiexamples_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def test_patchify_and_vit_embed(cuda):
    img = torch.rand(3, 3, 56, 70, device="cuda")
    mean = torch.tensor(CLIP_MEAN, device="cuda")
    inv = 1 / torch.tensor(CLIP_STD, device="cuda")
    got = ops.patchify(img, 14, mean, inv, 640)
    exp = ref.patchify(img.cpu(), 14, mean.cpu(), inv.cpu(), 640)
    torch.testing.assert_close(got.cpu().float(), exp.float(), rtol=1e-2, atol=1e-2)
    D = 256
    pe = torch.randn(3 * 20, D, device="cuda", dtype=torch.bfloat16)
    cls = torch.randn(D, device="cuda", dtype=torch.bfloat16)
    pos = torch.randn(21, D, device="cuda", dtype=torch.bfloat16)
    torch.testing.assert_close(ops.vit_embed(pe, cls, pos, 3).cpu().float(),
                               ref.vit_embed(pe.cpu(), cls.cpu(), pos.cpu(), 3).float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("cfg_name", ["tiny", "vit_l_14"])
def test_clip_image_embeddings_match_reference(cuda, cfg_name):
    cfg = getattr(ClipConfig, cfg_name)()
    m = ClipModel(cfg, device="cuda").random_init(seed=5)
    px = torch.rand(2, 3, cfg.image_size, cfg.image_size, device="cuda")
    e = m.encode_image(px)
    r = m.reference_encode_image(px)
    cos = F.cosine_similarity(e.cpu(), r, dim=-1)
    assert cos.min() > 0.995, cos


def test_clip_fp8_weights(cuda):
    m = ClipModel(ClipConfig.vit_l_14(), device="cuda").random_init(seed=6)
    px = torch.rand(2, 3, 224, 224, device="cuda")
    e16 = m.encode_image(px)
    m.quantize_fp8("v")
    assert isinstance(m.w["v0.fc1"], ops.Fp8Weight)
    e8 = m.encode_image(px)
    r = m.reference_encode_image(px)  # reference on the dequantised fp8 weights
    assert F.cosine_similarity(e8.cpu(), r, dim=-1).min() > 0.99
    assert F.cosine_similarity(e8, e16, dim=-1).min() > 0.95


def test_clip_text_and_preprocess(cuda):
    import numpy as np
    m = ClipModel(ClipConfig.tiny(), device="cuda").random_init(seed=7)
    t = m.encode_text([[1, 2, 3, 4, 5], [9, 8, 7]])
    assert t.shape == (2, 128) and torch.allclose(t.norm(dim=-1), torch.ones(2, device="cuda"), atol=1e-3)
    px = m.preprocess([np.random.randint(0, 255, (90, 120, 3), dtype=np.uint8)])
    assert px.shape == (1, 3, 56, 56) and px.is_cuda
