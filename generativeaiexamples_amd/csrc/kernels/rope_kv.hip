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
#include "gai_rope.h"

using namespace gai;

namespace {

template <int D, typename KV>
__global__ __launch_bounds__(256) void rope_kv_kernel(const bf16* __restrict__ qkv, const int* __restrict__ pos,
                                                      const float* __restrict__ cos_sin,
                                                      const int* __restrict__ slots, bf16* __restrict__ q_out,
                                                      KV* __restrict__ k_cache, KV* __restrict__ v_cache,
                                                      int T, int Hq, int Hkv, int rope, float inv_ks, float inv_vs) {
  constexpr int LPH = D / 8;  // lanes per head: each lane owns 4 rotation pairs
  constexpr int HPB = 256 / LPH;
  if (threadIdx.x >= HPB * LPH) return;  // D = 96: 12 lanes per head, 21 heads per block, 4 idle lanes
  const int H = Hq + 2 * Hkv;
  const long item = (long)blockIdx.x * HPB + threadIdx.x / LPH;  // (token, head)
  if (item >= (long)T * H) return;
  const int t = (int)(item / H), h = (int)(item % H);
  const int i0 = (threadIdx.x % LPH) * 4;  // pair indices i0..i0+3 and i0+D/2..
  const bf16* src = qkv + ((size_t)t * H + h) * D;
  const bf16x4 x1 = *reinterpret_cast<const bf16x4*>(src + i0);
  const bf16x4 x2 = *reinterpret_cast<const bf16x4*>(src + i0 + D / 2);
  rope_kv_store<D>(x1, x2, t, h, i0, pos, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, rope, inv_ks, inv_vs);
}

// Encoder self-attention (no RoPE, K / V straight from the packed QKV rows): one workgroup per (transient page, kv
// head) writes the page's K image [16][D] and V^T image [D][16] whole, with 16-B stores; V is transposed through LDS.
// Replaces rope_kv_kernel's per-(token, head) scatter for encoders, whose V^T half is 2-B stores 32 B apart and which
// also copied q (the attention reads q from the QKV rows, q_ld): e5-large ingest at 65536 tokens spent 379 us per
// layer there (profiles/r6).
template <int D>
__global__ __launch_bounds__(64) void kv_pack_kernel(const bf16* __restrict__ qkv, int ld, int koff, int voff,
                                                     const int* __restrict__ blk_tok, const int* __restrict__ blk_n,
                                                     bf16* __restrict__ k_cache, bf16* __restrict__ v_cache, int Hkv) {
  constexpr int CPR = D / 8;       // 16-B chunks per row
  constexpr int PIECES = 16 * CPR;
  __shared__ __attribute__((aligned(16))) bf16 vs[16][D + 8];  // V rows, padded against bank conflicts
  const int b = blockIdx.x, g = blockIdx.y, lane = threadIdx.x;
  const int t0 = blk_tok[b], n = blk_n[b];
  bf16* kp = k_cache + ((size_t)b * Hkv + g) * 16 * D;
  bf16* vp = v_cache + ((size_t)b * Hkv + g) * D * 16;
#pragma unroll
  for (int p = lane; p < PIECES; p += 64) {
    const int r = p / CPR, c = (p % CPR) * 8;
    bf16x8 kv = {}, vv = {};
    if (r < n) {
      const bf16* src = qkv + (size_t)(t0 + r) * ld + (size_t)g * D + c;
      kv = load8(src + koff);
      vv = load8(src + voff);
    }
    store8(kp + r * D + c, kv);
    *reinterpret_cast<bf16x8*>(&vs[r][c]) = vv;
  }
  __syncthreads();
#pragma unroll
  for (int p = lane; p < PIECES; p += 64) {  // V^T row d = 16 tokens = two 16-B pieces
    const int d = p >> 1, h8 = (p & 1) * 8;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = vs[h8 + e][d];
    store8(vp + d * 16 + h8, o);
  }
}

}  // namespace

void gai_kv_pack(const void* qkv, int ld, int koff, int voff, const int* blk_tok, const int* blk_n, int nblk,
                 void* k_cache, void* v_cache, int Hkv, int D, hipStream_t st) {
  if (nblk == 0) return;
  const dim3 grid(nblk, Hkv);
#define GAI_KVP(DD)                                                                                          \
  if (D == DD) {                                                                                             \
    kv_pack_kernel<DD><<<grid, 64, 0, st>>>((const bf16*)qkv, ld, koff, voff, blk_tok, blk_n, (bf16*)k_cache, \
                                            (bf16*)v_cache, Hkv);                                            \
    GAI_LAUNCH_CHECK();                                                                                      \
    return;                                                                                                  \
  }
  GAI_KVP(64)
  GAI_KVP(96)
  GAI_KVP(128)
  GAI_KVP(256)
#undef GAI_KVP
  gai_launch_error(__FILE__, __LINE__, "kv_pack: head_dim must be 64, 96, 128 or 256");
}

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
  GAI_ROPE_CASE(96)
  GAI_ROPE_CASE(128)
  GAI_ROPE_CASE(256)
#undef GAI_ROPE_CASE
  gai_launch_error(__FILE__, __LINE__, "rope_kv: head_dim must be 64, 96, 128 or 256");
}
