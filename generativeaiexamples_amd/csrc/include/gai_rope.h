// RoPE + paged KV-cache store of one (token, head) quarter-row, shared by the stand-alone rope_kv kernel
// (rope_kv.hip) and the decode QKV split-K reduce that fuses it (gemm_splitk.hip).
//
// A thread owns rotation pairs (i0 .. i0+3, i0+D/2 .. i0+D/2+3) of head h of token t: it rotates q and k
// (neox rotate-half, fp32 cos/sin table [max_pos, D] = [cos(D/2) | sin(D/2)]), writes q to q_out
// [T, Hq, D], k into the paged K cache [num_blocks, Hkv, 16, D] and v into the transposed paged V cache
// [num_blocks, Hkv, D, 16]; slot_mapping[t] = block * 16 + offset, < 0 skips the cache write. KV = fp8:
// the cache holds OCP e4m3fn x / scale.
#pragma once
#include "gai_common.h"

namespace gai {

constexpr int kKvBlock = 16;  // KV block size (tokens per page)

template <int D, typename KV>
__device__ __forceinline__ void rope_kv_store(bf16x4 x1, bf16x4 x2, int t, int h, int i0, const int* __restrict__ pos,
                                              const float* __restrict__ cos_sin, const int* __restrict__ slots,
                                              bf16* __restrict__ q_out, KV* __restrict__ k_cache,
                                              KV* __restrict__ v_cache, int Hq, int Hkv, int rope, float inv_ks,
                                              float inv_vs) {
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
  const int blk = slot / kKvBlock, off = slot % kKvBlock;
  constexpr bool F8 = sizeof(KV) == 1;
  if (!is_v) {
    const int g = h - Hq;
    KV* dst = k_cache + (((size_t)blk * Hkv + g) * kKvBlock + off) * D;
    if constexpr (F8) {
      *reinterpret_cast<uint32_t*>(dst + i0) = f32x4_to_fp8(x1[0], x1[1], x1[2], x1[3], inv_ks);
      *reinterpret_cast<uint32_t*>(dst + i0 + D / 2) = f32x4_to_fp8(x2[0], x2[1], x2[2], x2[3], inv_ks);
    } else {
      *reinterpret_cast<bf16x4*>(dst + i0) = x1;
      *reinterpret_cast<bf16x4*>(dst + i0 + D / 2) = x2;
    }
  } else {
    const int g = h - Hq - Hkv;
    KV* dst = v_cache + ((size_t)blk * Hkv + g) * D * kKvBlock + off;
    if constexpr (F8) {
      const uint32_t lo = f32x4_to_fp8(x1[0], x1[1], x1[2], x1[3], inv_vs);
      const uint32_t hi = f32x4_to_fp8(x2[0], x2[1], x2[2], x2[3], inv_vs);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dst[(size_t)(i0 + j) * kKvBlock] = (KV)(lo >> (8 * j));
        dst[(size_t)(i0 + D / 2 + j) * kKvBlock] = (KV)(hi >> (8 * j));
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dst[(size_t)(i0 + j) * kKvBlock] = x1[j];
        dst[(size_t)(i0 + D / 2 + j) * kKvBlock] = x2[j];
      }
    }
  }
}

}  // namespace gai
