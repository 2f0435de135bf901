// Vision front-end kernels (ViT patch-embed as a GEMM).
//
// patchify: normalise pixels ((x - mean[c]) * inv_std[c]) and im2col the non-overlapping PxP
// patches of an image batch [B, C, H, W] (fp32) into bf16 rows [B * gh * gw, Kp] ordered
// (c, ky, kx) - the flattening of a Conv2d(C, D, P, stride P) weight [D, C, P, P] - zero-padded to
// Kp (a multiple of 128) so the patch projection runs as one MFMA GEMM against the padded weight.
// vit_embed: [CLS | patches] + absolute position embedding, written as the encoder's packed
// token rows [B * (1 + gh * gw), D], 16-B vectors.
#include "gai_common.h"
#include "gai_kernels.h"

using namespace gai;

namespace {

__global__ __launch_bounds__(256) void patchify_kernel(const float* __restrict__ img, int C, int H, int W, int P,
                                                       int gh, int gw, int Kp, const float* __restrict__ mean,
                                                       const float* __restrict__ inv_std, bf16* __restrict__ out) {
  const int row = blockIdx.x;  // b * gh * gw + py * gw + px
  const int per = gh * gw;
  const int b = row / per, pr = row % per, py = pr / gw, px = pr % gw;
  const int PP = P * P, Kr = C * PP;
  bf16* o = out + (size_t)row * Kp;
  for (int k = threadIdx.x; k < Kp; k += 256) {
    float v = 0.f;
    if (k < Kr) {
      const int c = k / PP, r = k % PP, ky = r / P, kx = r % P;
      const float x = img[(((size_t)b * C + c) * H + py * P + ky) * W + px * P + kx];
      v = (x - mean[c]) * inv_std[c];
    }
    o[k] = (bf16)v;
  }
}

__global__ __launch_bounds__(256) void vit_embed_kernel(const bf16* __restrict__ patches, const bf16* __restrict__ cls,
                                                        const bf16* __restrict__ pos, bf16* __restrict__ out, int B,
                                                        int NP, int D) {
  const int units = D / 8;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)B * (NP + 1) * units;
  if (e >= total) return;
  const int u = (int)(e % units);
  const long t = e / units;
  const int b = (int)(t / (NP + 1)), s = (int)(t % (NP + 1));
  const bf16x8 src = s == 0 ? load8(cls + u * 8) : load8(patches + ((size_t)b * NP + s - 1) * D + u * 8);
  const bf16x8 p = load8(pos + (size_t)s * D + u * 8);
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = (bf16)((float)src[i] + (float)p[i]);
  store8(out + (size_t)t * D + u * 8, r);
}

}  // namespace

void gai_patchify(const float* img, int B, int C, int H, int W, int P, int Kp, const float* mean,
                  const float* inv_std, void* out, hipStream_t st) {
  const int gh = H / P, gw = W / P;
  if (B == 0 || gh == 0 || gw == 0) return;
  patchify_kernel<<<B * gh * gw, 256, 0, st>>>(img, C, H, W, P, gh, gw, Kp, mean, inv_std, (bf16*)out);
  GAI_LAUNCH_CHECK();
}

void gai_vit_embed(const void* patches, const void* cls, const void* pos, void* out, int B, int NP, int D,
                   hipStream_t st) {
  const long total = (long)B * (NP + 1) * (D / 8);
  if (total == 0) return;
  vit_embed_kernel<<<(unsigned)((total + 255) / 256), 256, 0, st>>>((const bf16*)patches, (const bf16*)cls,
                                                                     (const bf16*)pos, (bf16*)out, B, NP, D);
  GAI_LAUNCH_CHECK();
}
