"""CPU tier: CLIP tiny forward vs its fp32 reference, preprocessing, fp8 CPU reference path."""
import base64
import io

import numpy as np
import torch
import torch.nn.functional as F

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.models.clip import ClipConfig, ClipModel


def test_clip_tiny_cpu_matches_reference():
    m = ClipModel(ClipConfig.tiny(), device="cpu").random_init(seed=3)
    px = torch.rand(2, 3, 56, 56)
    e, r = m.encode_image(px), m.reference_encode_image(px)
    assert F.cosine_similarity(e, r, dim=-1).min() > 0.999


def test_clip_preprocess_inputs():
    from PIL import Image
    m = ClipModel(ClipConfig.tiny(), device="cpu")
    arr = np.random.randint(0, 255, (64, 100, 3), dtype=np.uint8)
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="PNG")
    uri = "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()
    px = m.preprocess([arr, Image.fromarray(arr), uri])
    assert px.shape == (3, 3, 56, 56)
    assert torch.allclose(px[0], px[1]) and torch.allclose(px[0], px[2])


def test_fp8_linear_cpu_reference():
    x = torch.randn(7, 256, dtype=torch.bfloat16)
    w = torch.randn(64, 256, dtype=torch.bfloat16) / 16
    W = ops.Fp8Weight.quantize(w)
    y = ops.linear(x, W)  # routes to linear_fp8
    r = ops.reference.linear(x, w, out_dtype=torch.float32)
    assert ((y.float() - r).norm() / r.norm()) < 0.08
