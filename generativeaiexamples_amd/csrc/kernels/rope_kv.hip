// Fused RoPE + paged KV-cache write.
//
// Input is the packed output of the fused QKV projection, [T, (Hq + 2*Hkv) * D].
// Per token it (1) rotates q and k (neox rotate-half pairs (i, i + D/2) with a
// host-precomputed fp32 cos/sin table [max_pos, D] = [cos(D/2) | sin(D/2)]),
// (2) writes q to q_out [T, Hq, D], (3) writes k into the paged K cache laid out
// [num_blocks, Hkv, 16, D] and v into the *transposed* paged V cache
// [num_blocks, Hkv, D, 16] -- the V^T layout lets both attention kernels feed
// P.V MFMAs with 8-byte contiguous loads (no LDS transpose).
// slot_mapping[t] = block * 16 + offset, or < 0 to skip the cache write.
// rope == 0 skips the rotation (encoder / BERT path).
// KV = fp8: the cache holds OCP e4m3fn values x / scale (per-layer k / v scales, saturated) -- the fp8 KV
// cache option, half the bytes per token for decode attention.
#include "gai_common.h"
#include "gai_kernels.h"

using namespace gai;

namespace {

constexpr int kBS = 16;  // KV block size (tokens per page)

template <int D, typename KV>
__global__ __launch_bounds__(256) void rope_kv_kernel(const bf16* __restrict__ qkv, const int* __restrict__ pos,
                                                      const float* __restrict__ cos_sin,
                                                      const int* __restrict__ slots, bf16* __restrict__ q_out,
                                                      KV* __restrict__ k_cache, KV* __restrict__ v_cache,
                                                      int T, int Hq, int Hkv, int rope, float inv_ks, float inv_vs) {
  constexpr int LPH = D / 8;  // lanes per head: each lane owns 4 rotation pairs
  constexpr int HPB = 256 / LPH;
  const int H = Hq + 2 * Hkv;
  const long item = (long)blockIdx.x * HPB + threadIdx.x / LPH;  // (token, head)
  if (item >= (long)T * H) return;
  const int t = (int)(item / H), h = (int)(item % H);
  const int l = threadIdx.x % LPH;
  const int i0 = l * 4;  // pair indices i0..i0+3 and i0+D/2..
  const bf16* src = qkv + ((size_t)t * H + h) * D;
  bf16x4 x1 = *reinterpret_cast<const bf16x4*>(src + i0);
  bf16x4 x2 = *reinterpret_cast<const bf16x4*>(src + i0 + D / 2);
  const bool is_v = h >= Hq + Hkv;
  if (rope && !is_v) {
    const int p = pos[t];
    const float4 c = *reinterpret_cast<const float4*>(cos_sin + (size_t)p * D + i0);
    const float4 s = *reinterpret_cast<const float4*>(cos_sin + (size_t)p * D + D / 2 + i0);
    const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = (float)x1[j], b = (float)x2[j];
      x1[j] = (bf16)(a * cc[j] - b * ss[j]);
      x2[j] = (bf16)(b * cc[j] + a * ss[j]);
    }
  }
  if (h < Hq) {
    bf16* dst = q_out + ((size_t)t * Hq + h) * D;
    *reinterpret_cast<bf16x4*>(dst + i0) = x1;
    *reinterpret_cast<bf16x4*>(dst + i0 + D / 2) = x2;
    return;
  }
  const int slot = slots[t];
  if (slot < 0) return;
  const int blk = slot / kBS, off = slot % kBS;
  constexpr bool F8 = sizeof(KV) == 1;
  if (!is_v) {
    const int g = h - Hq;
    KV* dst = k_cache + (((size_t)blk * Hkv + g) * kBS + off) * D;
    if constexpr (F8) {
      *reinterpret_cast<uint32_t*>(dst + i0) = f32x4_to_fp8(x1[0], x1[1], x1[2], x1[3], inv_ks);
      *reinterpret_cast<uint32_t*>(dst + i0 + D / 2) = f32x4_to_fp8(x2[0], x2[1], x2[2], x2[3], inv_ks);
    } else {
      *reinterpret_cast<bf16x4*>(dst + i0) = x1;
      *reinterpret_cast<bf16x4*>(dst + i0 + D / 2) = x2;
    }
  } else {
    const int g = h - Hq - Hkv;
    KV* dst = v_cache + ((size_t)blk * Hkv + g) * D * kBS + off;
    if constexpr (F8) {
      const uint32_t lo = f32x4_to_fp8(x1[0], x1[1], x1[2], x1[3], inv_vs);
      const uint32_t hi = f32x4_to_fp8(x2[0], x2[1], x2[2], x2[3], inv_vs);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dst[(size_t)(i0 + j) * kBS] = (KV)(lo >> (8 * j));
        dst[(size_t)(i0 + D / 2 + j) * kBS] = (KV)(hi >> (8 * j));
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dst[(size_t)(i0 + j) * kBS] = x1[j];
        dst[(size_t)(i0 + D / 2 + j) * kBS] = x2[j];
      }
    }
  }
}

}  // namespace

void gai_rope_kv_write(const void* qkv, const int* pos, const float* cos_sin, const int* slots, void* q_out,
                       void* k_cache, void* v_cache, int T, int Hq, int Hkv, int D, int rope, int kv_fp8,
                       float k_scale, float v_scale, hipStream_t st) {
  if (T == 0) return;
  const long items = (long)T * (Hq + 2 * Hkv);
  const float iks = 1.f / k_scale, ivs = 1.f / v_scale;
#define GAI_ROPE_CASE(DD)                                                                                   \
  if (D == DD) {                                                                                            \
    constexpr int HPB = 256 / (DD / 8);                                                                     \
    const unsigned grid = (unsigned)((items + HPB - 1) / HPB);                                              \
    if (kv_fp8)                                                                                             \
      rope_kv_kernel<DD, fp8><<<grid, 256, 0, st>>>((const bf16*)qkv, pos, cos_sin, slots, (bf16*)q_out,   \
                                                     (fp8*)k_cache, (fp8*)v_cache, T, Hq, Hkv, rope, iks, ivs); \
    else                                                                                                    \
      rope_kv_kernel<DD, bf16><<<grid, 256, 0, st>>>((const bf16*)qkv, pos, cos_sin, slots, (bf16*)q_out,  \
                                                      (bf16*)k_cache, (bf16*)v_cache, T, Hq, Hkv, rope, iks, ivs); \
    GAI_LAUNCH_CHECK();                                                                                     \
    return;                                                                                                 \
  }
  GAI_ROPE_CASE(64)
  GAI_ROPE_CASE(128)
  GAI_ROPE_CASE(256)
#undef GAI_ROPE_CASE
  gai_launch_error(__FILE__, __LINE__, "rope_kv: head_dim must be 64, 128 or 256");
}
