// Small-batch decode GEMV (M = 1..4 token rows): C[M, N] = A[M, K] . W[N, K]^T with the layer's neighbours fused.
//
// At batch 1 a decode layer is a pure weight stream (Llama-3-8B: 436 MB per layer, 16 KB of activations). The
// MFMA decode kernels (gemm_splitk / gemm_decode) load 16 weight rows x 64 B per instruction and split K over
// workgroups, so every projection also pays an fp32 partial-slab round trip and a tail launch (split-K reduce +
// RoPE / residual add + RMSNorm): four tails per layer at batch 1, each latency-bound. Here:
//  * a wave owns two weight rows and streams each as whole 1 KiB rows pieces (64 lanes x 16 B contiguous,
//    non-temporal: read once), kG = 4 pieces per row in flight ahead of the arithmetic (v_dot2_f32_bf16);
//  * the activation rows are staged ONCE per workgroup in LDS; with `gamma` the kernel stages the RMSNorm of the
//    residual stream instead (sum of squares reduced in the workgroup, x_hat * gamma rounded to bf16 exactly as
//    the norm kernel does) - the norm launch disappears, its input is the residual the previous projection's
//    epilogue updated in place;
//  * the wave's row pair is chosen so the epilogue has everything it needs: (2p, 2p+1) for plain / fp32 /
//    residual outputs, the interleaved (gate, up) rows for SwiGLU, and the rotate-half partners (d, d + 64) of
//    one head for RoPE + q / paged K / V^T stores - no split-K, no slabs, no tail launch.
// A Llama decode layer at batch <= 4 is then five launches: QKV(+norm, +RoPE/KV) -> attention -> O(+residual)
// -> gate_up(+norm, +SwiGLU) -> down(+residual).
#include <cstdlib>

#include "gai_common.h"
#include "gai_kernels.h"

using namespace gai;

namespace {

constexpr int kGvWaves = 8;  // waves per workgroup (default); 12 where 8 leaves the grid unbalanced (gemv_waves)
constexpr int kGvThreads = 64 * kGvWaves;
constexpr int kPiece = 512;  // K elements of one wave load (64 lanes x 8 bf16)
constexpr int kG = 4;        // pieces per row per pipeline group
// dynamic LDS cap: the 160 KiB of a CU minus the kernel's static reduction arrays (asking for all 160 KiB fails the
// attribute call, and its error would surface at the next launch check)
constexpr int kGvMaxDyn = 160 * 1024 - 1024;

// GV_PART (fragment-ordered weights): K is split over KS workgroups per column, each storing its fp32 row sums as
// slab h of out [KS][M][N] - the QKV split-K partials the decode-attention launch folds (sum, RoPE, KV write).
enum { GV_PLAIN = 0, GV_RESIDUAL = 1, GV_SWIGLU = 2, GV_ROPE = 3, GV_F32 = 4, GV_PART = 5 };

struct GemvArgs {
  const bf16* x;      // [M, K] activations, or the residual stream to normalise when gamma != null
  const bf16* gamma;  // RMSNorm weight [K] (null: x is used as is)
  float eps;
  const bf16* W;      // [N, K]
  int M, N, K;
  void* out;          // GV_PLAIN / GV_SWIGLU: bf16 [M, N or N / 2]; GV_F32: fp32 [M, N]
  bf16* res;          // GV_RESIDUAL: [M, N], res = bf16(bf16(acc) + res) in place
  const int* pos;     // GV_ROPE
  const float* cos_sin;
  const int* slots;
  bf16* q_out;
  bf16* k_cache;
  bf16* v_cache;
  int Hq, Hkv;
  // swi != null: the staged activations are bf16(silu(g) * u) of an fp32 [M, 2K] gate_up output in the [gate16 | up16]
  // interleave (the GV_F32 gate_up GEMV), i.e. the down projection does the SwiGLU while staging its input
  const float* swi;
  int ks;  // GV_PART: K parts per column
};

__device__ __forceinline__ float dot8(const bf16x8& a, const bf16x8& b, float acc) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    acc = __builtin_amdgcn_fdot2_f32_bf16(bf16x2{a[2 * i], a[2 * i + 1]}, bf16x2{b[2 * i], b[2 * i + 1]}, acc, false);
  return acc;
}

// The epilogue of row pair p (rows r0, r1: their fp32 dot products v0, v1) for token row m; shared by the row-pair and
// the fragment-ordered kernels.
template <int EPI>
__device__ __forceinline__ void gv_epilogue(const GemvArgs& a, int m, int p, int r0, int r1, float v0, float v1) {
  const int N = a.N;
  if constexpr (EPI == GV_PLAIN) {
    bf16* o = reinterpret_cast<bf16*>(a.out) + (size_t)m * N;
    o[r0] = (bf16)v0;
    o[r1] = (bf16)v1;
  } else if constexpr (EPI == GV_F32) {
    float* o = reinterpret_cast<float*>(a.out) + (size_t)m * N;
    o[r0] = v0;
    o[r1] = v1;
  } else if constexpr (EPI == GV_RESIDUAL) {  // the rounding of the split-K add + norm tail: bf16(bf16(h) + r)
    bf16* r = a.res + (size_t)m * N;
    r[r0] = (bf16)((float)(bf16)v0 + (float)r[r0]);
    r[r1] = (bf16)((float)(bf16)v1 + (float)r[r1]);
  } else if constexpr (EPI == GV_SWIGLU) {
    reinterpret_cast<bf16*>(a.out)[(size_t)m * (N / 2) + p] = (bf16)(silu(v0) * v1);
  } else if constexpr (EPI == GV_ROPE) {  // x = bf16(qkv) as the unfused GEMM output, then rotate (neox halves), store
    constexpr int D = 128, kBS = 16;
    const int h = p >> 6, i = p & 63;
    float x1 = (float)(bf16)v0, x2 = (float)(bf16)v1;
    if (h < a.Hq + a.Hkv) {
      const int ps = a.pos[m];
      const float c = a.cos_sin[(size_t)ps * D + i], s = a.cos_sin[(size_t)ps * D + D / 2 + i];
      const float y1 = x1 * c - x2 * s, y2 = x2 * c + x1 * s;
      x1 = y1;
      x2 = y2;
    }
    if (h < a.Hq) {
      bf16* q = a.q_out + ((size_t)m * a.Hq + h) * D;
      q[i] = (bf16)x1;
      q[i + D / 2] = (bf16)x2;
      return;
    }
    const int slot = a.slots[m];
    if (slot < 0) return;
    const int blk = slot / kBS, off = slot % kBS;
    if (h < a.Hq + a.Hkv) {
      bf16* kd = a.k_cache + (((size_t)blk * a.Hkv + (h - a.Hq)) * kBS + off) * D;
      kd[i] = (bf16)x1;
      kd[i + D / 2] = (bf16)x2;
    } else {
      bf16* vd = a.v_cache + ((size_t)blk * a.Hkv + (h - a.Hq - a.Hkv)) * D * kBS + off;
      vd[(size_t)i * kBS] = (bf16)x1;
      vd[(size_t)(i + D / 2) * kBS] = (bf16)x2;
    }
  }
}

// Stage the MR activation rows in LDS (xs, [MR][K] bf16), normalised (x_hat * gamma rounded to bf16 exactly as the norm
// kernel does) when a.gamma is given; red [NW][MR] / inv_s [MR] are the workgroup's reduction scratch. No trailing barrier.
template <int MR, int NW>
__device__ __forceinline__ void gv_stage(const GemvArgs& a, bf16* xs, float* red, float* inv_s) {
  constexpr int kThr = 64 * NW;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int K = a.K, nch = K / 8;
  // the host keeps K <= 8192 for the norm form
  if (a.gamma != nullptr) {
    constexpr int kMaxC = (8192 + 8 * kThr - 1) / (8 * kThr);  // chunks per thread per row: K <= 8192
    bf16x8 v[MR][kMaxC];
    float ss[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      ss[m] = 0.f;
#pragma unroll
      for (int c = 0; c < kMaxC; ++c) {
        const int ch = c * kThr + tid;
        if (ch < nch) {
          v[m][c] = load8(a.x + (size_t)m * K + 8 * ch);
#pragma unroll
          for (int e = 0; e < 8; ++e) ss[m] += (float)v[m][c][e] * (float)v[m][c][e];
        }
      }
      ss[m] = wave_sum(ss[m]);
      if (lane == 0) red[wid * MR + m] = ss[m];
    }
    __syncthreads();
    if (tid < MR) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += red[w * MR + tid];
      inv_s[tid] = rsqrtf(t / K + a.eps);
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const float inv = inv_s[m];
#pragma unroll
      for (int c = 0; c < kMaxC; ++c) {
        const int ch = c * kThr + tid;
        if (ch < nch) {
          const bf16x8 g = load8(a.gamma + 8 * ch);
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (bf16)((float)v[m][c][e] * inv * (float)g[e]);
          *reinterpret_cast<bf16x8*>(xs + (size_t)m * K + 8 * ch) = o;
        }
      }
    }
  } else if (a.swi != nullptr) {
    // chunk c = k 8c .. 8c + 7, inside one 16-group: gate at 32 (k / 16) + k % 16, up 16 further; the rounding of the
    // GV_SWIGLU epilogue (bf16(silu(g) * u) of the fp32 sums)
    for (int ch = tid; ch < MR * nch; ch += kThr) {
      const int m = ch / nch, c = ch % nch, k0 = 8 * c;
      const float* gp = a.swi + (size_t)m * 2 * K + 32 * (k0 >> 4) + (k0 & 15);
      const float4 g0 = *reinterpret_cast<const float4*>(gp), g1 = *reinterpret_cast<const float4*>(gp + 4);
      const float4 u0 = *reinterpret_cast<const float4*>(gp + 16), u1 = *reinterpret_cast<const float4*>(gp + 20);
      const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float u[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)(silu(g[e]) * u[e]);
      *reinterpret_cast<bf16x8*>(xs + (size_t)m * K + k0) = o;
    }
  } else {
    for (int ch = tid; ch < MR * nch; ch += kThr) {
      const int m = ch / nch, c = ch % nch;
      *reinterpret_cast<bf16x8*>(xs + (size_t)m * K + 8 * c) = load8(a.x + (size_t)m * K + 8 * c);
    }
  }
}

template <int MR, int EPI, int NW = kGvWaves>
__global__ __launch_bounds__(64 * NW) void gemv_kernel(GemvArgs a) {
  constexpr int kThr = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [MR][K] bf16 activation image
  __shared__ float red[NW][MR];
  __shared__ float inv_s[MR];
  bf16* xs = reinterpret_cast<bf16*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int K = a.K, nch = K / 8;

  // ---- this wave's row pair; its first weight group is issued BEFORE the activation staging, so the HBM
  // latency of the weight stream overlaps the staging (and the RMSNorm reduction) instead of following it
  const int p = blockIdx.x * NW + wid;
  const int npairs = a.N / 2;
  const bool live = p < npairs;
  int r0, r1;
  if (EPI == GV_SWIGLU) {  // rows interleaved per 16: [gate16 | up16]; output column p
    r0 = 32 * (p >> 4) + (p & 15);
    r1 = r0 + 16;
  } else if (EPI == GV_ROPE) {  // head p / 64, rotate-half pair (i, i + 64)
    r0 = 128 * (p >> 6) + (p & 63);
    r1 = r0 + 64;
  } else {
    r0 = 2 * p;
    r1 = r0 + 1;
  }
  const bf16* w0 = a.W + (size_t)(live ? r0 : 0) * K + 8 * lane;
  const bf16* w1 = a.W + (size_t)(live ? r1 : 0) * K + 8 * lane;
  const int ngroups = K / (kPiece * kG);  // host: K % 2048 == 0
  bf16x8 cur0[kG], cur1[kG], nxt0[kG], nxt1[kG];
  auto load_group = [&](int g, bf16x8(&b0)[kG], bf16x8(&b1)[kG]) {
#pragma unroll
    for (int c = 0; c < kG; ++c) {
      const int off = (g * kG + c) * kPiece;
      b0[c] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(w0 + off));
      b1[c] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(w1 + off));
    }
  };
  if (live) load_group(0, cur0, cur1);

  gv_stage<MR, NW>(a, xs, &red[0][0], inv_s);
  __syncthreads();
  if (!live) return;  // no barrier below

  float acc[MR][2];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc[m][0] = acc[m][1] = 0.f;
  auto compute_group = [&](int g, const bf16x8(&b0)[kG], const bf16x8(&b1)[kG]) {
#pragma unroll
    for (int c = 0; c < kG; ++c) {
      const int k0 = (g * kG + c) * kPiece + 8 * lane;
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xs + (size_t)m * K + k0);
        acc[m][0] = dot8(xv, b0[c], acc[m][0]);
        acc[m][1] = dot8(xv, b1[c], acc[m][1]);
      }
    }
  };
  int g = 0;  // group 0 is in flight since the kernel start
  for (; g + 2 <= ngroups; g += 2) {
    load_group(g + 1, nxt0, nxt1);
    compute_group(g, cur0, cur1);
    if (g + 2 < ngroups) load_group(g + 2, cur0, cur1);
    compute_group(g + 1, nxt0, nxt1);
  }
  if (g < ngroups) compute_group(g, cur0, cur1);

#pragma unroll
  for (int m = 0; m < MR; ++m) {
    acc[m][0] = wave_sum(acc[m][0]);
    acc[m][1] = wave_sum(acc[m][1]);
  }
  if (lane >= MR) return;
  // lane m finishes token row m
  float v0 = acc[0][0], v1 = acc[0][1];
#pragma unroll
  for (int m = 1; m < MR; ++m)
    if (lane == m) {
      v0 = acc[m][0];
      v1 = acc[m][1];
    }
  gv_epilogue<EPI>(a, lane, p, r0, r1, v0, v1);
}

// Fragment-ordered weights (ops.shuffle_fragments: [N/16][K/32][64 lanes][8], the one layout of the decode
// projections): a 16-row column of W is K/32 contiguous 1 KiB MFMA fragments, lane l of fragment kt holding row l & 15,
// k 32 kt + 8 (l >> 4) .. + 8. A workgroup owns C whole columns - one for the plain / fp32 / residual epilogues, the
// (gate, up) pair 2b, 2b + 1 for SwiGLU, the rotate-half pair c, c + 4 of one head for RoPE. Each wave streams ONE
// column (a wave streaming two columns at once ran 25-35 % slower: SwiGLU 45-51 vs 36.9 us at any wave count,
// profiles/r5/weight_layout): the NW / C waves of a column split its K range, kG whole 1 KiB fragments in flight ahead
// of the arithmetic (non-temporal), each lane dotting its 8 weights with the staged activation chunk. The 4 lanes of a
// row (l, l + 16, l + 32, l + 48) reduce by cross-lane shuffles, the waves through LDS.
// KS > 1 (opt-in, GAI_GEMV_FRAG_KS: it did not pay where the grid has fewer column groups than CUs - Llama-3-8B
// QKV + RoPE, 192 column pairs for 256 CUs: 13.6 us unsplit, 13.7-16.0 split in two): KS workgroups split K of one group; each stores its fp32 row sums write-through (sc1), waits for them, and draws a
// relaxed agent-scope ticket (the stream-K GEMM's hand-over, gemm_impl.h gemm_w4r_kernel); the last one sums the KS
// partials in K order (deterministic whichever finishes last), resets the ticket, and runs the row-pair epilogue
// gv_epilogue.
template <int EPI>
constexpr int gv_frag_cols() { return (EPI == GV_SWIGLU || EPI == GV_ROPE) ? 2 : 1; }

// fragments per wave per pipeline group (two groups in flight). 8-deep groups: batch-1 SwiGLU 44.2 -> 42.4 us but QKV
// 13.7 -> 16.0, LM head 153 -> 167, the batch-4 step 4.01 -> 4.31 ms (profiles/r5/weight_layout)
constexpr int kGf = 4;
constexpr int kGvfMaxItems = 4096;  // split workspace: (group, K part) items (2 MiB)
__device__ float g_gvf_ws[kGvfMaxItems * 4 * 16 * 2];  // [item][MR <= 4][16 pairs][2] fp32 row sums
__device__ int g_gvf_cnt[kGvfMaxItems];                // tickets per group, zero between launches

template <int MR, int EPI, int NW>
__global__ __launch_bounds__(64 * NW) void gemv_frag_kernel(GemvArgs a, int KS) {
  constexpr int C = gv_frag_cols<EPI>();
  constexpr int NWC = NW / C;                 // waves per column
  constexpr int NP = C == 1 ? 8 : 16;         // row pairs per group: rows (2i, 2i + 1) of one column, or row i of both
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [MR][K] bf16 activation image
  __shared__ float red[NW][MR];
  __shared__ float inv_s[MR];
  __shared__ float part[NW][MR][16];
  __shared__ int last_s;
  bf16* xs = reinterpret_cast<bf16*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int K = a.K, KF = K / 32;
  const int groups = (int)gridDim.x / KS;
  const int b = (int)blockIdx.x % groups, h = (int)blockIdx.x / groups;  // column group, K part
  auto column = [&](int c) {
    if constexpr (EPI == GV_ROPE) return 8 * (b >> 2) + (b & 3) + 4 * c;
    else return C * b + c;
  };
  const int wc = wid / NWC;                    // this wave's column (0 .. C-1)
  const int nf = KF / (KS * NWC);              // fragments per wave (host: a multiple of kGf)
  const int f0 = h * (KF / KS) + (wid % NWC) * nf;
  const bf16* wp = a.W + ((size_t)column(wc) * KF + f0) * 512 + 8 * lane;
  bf16x8 cur[kGf], nxt[kGf];
  auto load_group = [&](int g, bf16x8(&bq)[kGf]) {
#pragma unroll
    for (int j = 0; j < kGf; ++j)
      bq[j] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wp + (size_t)(g * kGf + j) * 512));
  };
  const int ngroups = nf / kGf;
  // both groups in flight during the activation staging (the RMSNorm of the normalised forms takes a few us)
  load_group(0, cur);
  if (ngroups > 1) load_group(1, nxt);
  gv_stage<MR, NW>(a, xs, &red[0][0], inv_s);
  __syncthreads();

  float acc[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc[m] = 0.f;
  const int kl = 8 * (lane >> 4);  // the lane's k offset inside a fragment
  auto compute_group = [&](int g, const bf16x8(&bq)[kGf]) {
#pragma unroll
    for (int j = 0; j < kGf; ++j) {
      const int k0 = (f0 + g * kGf + j) * 32 + kl;
#pragma unroll
      for (int m = 0; m < MR; ++m)
        acc[m] = dot8(*reinterpret_cast<const bf16x8*>(xs + (size_t)m * K + k0), bq[j], acc[m]);
    }
  };
  for (int g = 0; g < ngroups; g += 2) {  // groups g, g + 1 in flight on entry
    compute_group(g, cur);
    if (g + 2 < ngroups) load_group(g + 2, cur);
    if (g + 1 < ngroups) {
      compute_group(g + 1, nxt);
      if (g + 3 < ngroups) load_group(g + 3, nxt);
    }
  }

  // lanes l, l + 16, l + 32, l + 48 hold row l & 15's partials
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    float v = acc[m];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane < 16) part[wid][m][lane] = v;
  }
  __syncthreads();
  const bool epi_thread = tid < MR * NP;
  const int m = tid / NP, i = tid % NP;
  const int ra = C == 1 ? 2 * i : i, rb = C == 1 ? 2 * i + 1 : i;  // rows inside columns 0 / C-1
  float v0 = 0.f, v1 = 0.f;
  if (epi_thread) {
#pragma unroll
    for (int w = 0; w < NWC; ++w) {
      v0 += part[w][m][ra];
      v1 += part[(C - 1) * NWC + w][m][rb];
    }
  }
  if constexpr (EPI == GV_PART) {  // slab h of out [KS][M][N]: this part's row sums, no hand-over
    if (!epi_thread) return;
    const int r0 = 16 * column(0) + ra;
    float* o = reinterpret_cast<float*>(a.out) + ((size_t)h * a.M + m) * a.N + r0;
    *reinterpret_cast<float2*>(o) = float2{v0, v1};
    return;
  }
  if (KS > 1) {
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(g_gvf_ws, (short)0, 0x7fffffff, 0x00020000);
    using f32x2 = __attribute__((ext_vector_type(2))) float;
    auto off = [&](int part_h) { return (unsigned)((((b * KS + part_h) * 4 + m) * 16 + i) * 8); };
    if (epi_thread)  // write-through (sc1): visible to the other XCDs' L2s
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned,
                                                               f32x2{v0, v1}), rw, off(h), 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const int tk = __hip_atomic_fetch_add(&g_gvf_cnt[b], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_s = tk == KS - 1;
      if (tk == KS - 1) __hip_atomic_store(&g_gvf_cnt[b], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last_s) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
    if (epi_thread) {
      v0 = v1 = 0.f;
      for (int q = 0; q < KS; ++q) {  // K order
        const f32x2 t = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rw, off(q), 0, 16));
        v0 += t.x;
        v1 += t.y;
      }
    }
  }
  if (!epi_thread) return;
  const int r0 = 16 * column(0) + ra, r1 = 16 * column(C - 1) + rb;
  int p;
  if constexpr (EPI == GV_SWIGLU)
    p = 16 * b + i;  // output column: gate row r0 = 32 b + i
  else if constexpr (EPI == GV_ROPE)
    p = 64 * (r0 >> 7) + (r0 & 63);  // head r0 / 128, dim r0 % 128 (< 64)
  else
    p = r0 >> 1;
  gv_epilogue<EPI>(a, m, p, r0, r1, v0, v1);
}

// Waves per workgroup: 8, or 12 where that quantises the row pairs onto the CUs better (Llama-3-8B QKV, N 6144: 3072
// pairs = 384 eight-wave workgroups, 1.5 per CU, vs 256 twelve-wave ones). 6-wave workgroups also balance that grid
// (512 = 2 per CU) but stage the normalised activations in 1/3 more workgroups - measured slower (13.2 vs 11.4 us,
// profiles/r5/gemv_b1). Batch 1 only: QKV 11.42 -> 10.53 us, decode step 3.007 -> 2.97 ms; at batch 4 the step
// went 4.466 -> 4.530 ms (profiles/r5/gemv_b1/gemv_12waves_ab.txt). GAI_GEMV_WAVES = 6 / 8 / 12 forces one (sweeps).
int gemv_waves(int N, int M) {
  static const int force = getenv("GAI_GEMV_WAVES") ? atoi(getenv("GAI_GEMV_WAVES")) : 0;
  if (force == 6 || force == 8 || force == 12) return force;
  if (M != 1) return 8;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 8)
      ncu = 256;
  }
  auto fill = [&](int nw) {  // fraction of the workgroup slots (one per CU per round) the grid's rounds use
    const int grid = (N / 2 + nw - 1) / nw;
    return (double)grid / ((double)((grid + ncu - 1) / ncu) * ncu);
  };
  return fill(12) > fill(8) + 0.1 ? 12 : 8;
}

template <int EPI, int NW>
void gemv_launch_nw(const GemvArgs& a, hipStream_t st) {
  const size_t lds = (size_t)a.M * a.K * sizeof(bf16);
  const int grid = (a.N / 2 + NW - 1) / NW;
#define GAI_GV(MRV)                                                                                           \
  if (a.M == MRV) {                                                                                           \
    static bool once = false;                                                                                 \
    if (!once) {                                                                                              \
      hipFuncSetAttribute(reinterpret_cast<const void*>(gemv_kernel<MRV, EPI, NW>),                          \
                          hipFuncAttributeMaxDynamicSharedMemorySize, kGvMaxDyn);                             \
      once = true;                                                                                            \
    }                                                                                                         \
    gemv_kernel<MRV, EPI, NW><<<grid, 64 * NW, lds, st>>>(a);                                                 \
    GAI_LAUNCH_CHECK();                                                                                       \
    return;                                                                                                   \
  }
  GAI_GV(1)
  GAI_GV(2)
  GAI_GV(3)
  GAI_GV(4)
#undef GAI_GV
  gai_launch_error(__FILE__, __LINE__, "gemv: 1 <= M <= 4");
}

// Fragment-ordered launch: N / (16 C) column groups. Waves per workgroup by epilogue (Llama-3-8B sweeps, batch 1 / 4,
// profiles/r5/weight_layout): 16 for the one-column plain / residual forms (O / down 14.9 -> 14.0 us at batch 1,
// 17.0 -> 15.8 at batch 4) and QKV + RoPE (13.1 -> 12.1 / 15.1 -> 14.8); 8 for the fp32 LM head (16: 154 -> 158 /
// 178 -> 218) and batch > 1 SwiGLU (16: 48.1 -> 54.8), 4 for batch-1 SwiGLU (44.0 -> 42.8). GAI_GEMV_FRAG_WAVES =
// 4 / 8 / 16 and GAI_GEMV_FRAG_KS = 2 / 4 / 8 (K parts per group where it fits) force others.
constexpr int kGvFragStatic = 6 * 1024;  // bound on the frag kernel's static LDS (part[16][4][16] + red + inv_s)
constexpr int kGvFragMaxDyn = 160 * 1024 - kGvFragStatic;

template <int EPI, int NW>
void gemv_frag_launch_nw(const GemvArgs& a, int KS, hipStream_t st) {
  const size_t lds = (size_t)a.M * a.K * sizeof(bf16);
  const int grid = a.N / (16 * gv_frag_cols<EPI>()) * KS;
#define GAI_GVF(MRV)                                                                                          \
  if (a.M == MRV) {                                                                                           \
    static bool once = false;                                                                                 \
    if (!once) {                                                                                              \
      hipFuncSetAttribute(reinterpret_cast<const void*>(gemv_frag_kernel<MRV, EPI, NW>),                     \
                          hipFuncAttributeMaxDynamicSharedMemorySize, kGvFragMaxDyn);                         \
      once = true;                                                                                            \
    }                                                                                                         \
    gemv_frag_kernel<MRV, EPI, NW><<<grid, 64 * NW, lds, st>>>(a, KS);                                        \
    GAI_LAUNCH_CHECK();                                                                                       \
    return;                                                                                                   \
  }
  GAI_GVF(1)
  GAI_GVF(2)
  GAI_GVF(3)
  GAI_GVF(4)
#undef GAI_GVF
  gai_launch_error(__FILE__, __LINE__, "gemv: 1 <= M <= 4");
}

template <int EPI>
void gemv_frag_launch(const GemvArgs& a, hipStream_t st) {
  static const int fnw = getenv("GAI_GEMV_FRAG_WAVES") ? atoi(getenv("GAI_GEMV_FRAG_WAVES")) : 0;
  static const int fks = getenv("GAI_GEMV_FRAG_KS") ? atoi(getenv("GAI_GEMV_FRAG_KS")) : 0;
  constexpr int C = gv_frag_cols<EPI>();
  const int groups = a.N / (16 * C), KF = a.K / 32;
  // waves: 4 for the batch-1 gate_up as an fp32 GEMV (1792 one-column workgroups, 7 per CU: the SwiGLU moved into the
  // down projection's staging) and for the QKV partials (K parts x 384 columns); 8 for the LM head
  const int nw = (fnw == 4 || fnw == 8 || fnw == 16) ? fnw
                 : EPI == GV_PART ? 4
                 : EPI == GV_F32 ? (a.M == 1 && a.N <= 65536 ? 4 : 8)
                 : EPI == GV_SWIGLU ? (a.M == 1 ? 4 : 8)
                 : 16;
  auto fits = [&](int ks) { return (ks == 1 || groups * ks <= kGvfMaxItems) && KF % (ks * (nw / C) * kGf) == 0; };
  const int KS = EPI == GV_PART ? a.ks : (fks == 2 || fks == 4 || fks == 8) && fits(fks) ? fks : 1;
  if (!fits(KS)) gai_launch_error(__FILE__, __LINE__, "gemv: fragment-ordered K split");
  if (nw == 4) return gemv_frag_launch_nw<EPI, 4>(a, KS, st);
  if (nw == 16) return gemv_frag_launch_nw<EPI, 16>(a, KS, st);
  gemv_frag_launch_nw<EPI, 8>(a, KS, st);
}

template <int EPI>
void gemv_launch(const GemvArgs& a, hipStream_t st, int wfrag) {
  if (wfrag) {
    const int cols = gv_frag_cols<EPI>();
    if (a.N % (16 * cols) || (a.K / 32) % (8 * kG) || (size_t)a.M * a.K * sizeof(bf16) > (size_t)kGvFragMaxDyn)
      gai_launch_error(__FILE__, __LINE__, "gemv: fragment-ordered weight shape");
    return gemv_frag_launch<EPI>(a, st);
  }
  if constexpr (EPI == GV_PART) gai_launch_error(__FILE__, __LINE__, "gemv: K parts need fragment-ordered weights");
  const int nw = gemv_waves(a.N, a.M);
  if (nw == 6) return gemv_launch_nw<EPI, 6>(a, st);
  if (nw == 12) return gemv_launch_nw<EPI, 12>(a, st);
  gemv_launch_nw<EPI, 8>(a, st);
}

}  // namespace

int gai_gemv_ok(int M, int N, int K, int normed) {
  // (also the shapes of GV_PART and of the swi staging form; their extra conditions are checked in gai_gemv)
  if (M < 1 || M > 4 || N % 2 || K % (kPiece * kG)) return 0;
  if ((size_t)M * K * sizeof(bf16) > (size_t)kGvMaxDyn) return 0;
  if (normed && K > 2 * 8 * kGvThreads) return 0;
  return 1;
}

// epi: 0 plain bf16, 1 residual in place (res), 2 SwiGLU on the [gate16 | up16] interleave, 4 fp32 out.
void gai_gemv(const void* x, const void* gamma, float eps, const void* W, int M, int N, int K, int epi, void* out,
              void* res, hipStream_t st, int wfrag, const float* swi, int ks) {
  if (!gai_gemv_ok(M, N, K, gamma != nullptr)) gai_launch_error(__FILE__, __LINE__, "gemv: shape");
  if (epi == GV_SWIGLU && N % 32) gai_launch_error(__FILE__, __LINE__, "gemv: SwiGLU needs N % 32 == 0");
  if ((epi == GV_PART || swi != nullptr) && !wfrag)
    gai_launch_error(__FILE__, __LINE__, "gemv: K parts / SwiGLU staging need fragment-ordered weights");
  if (swi != nullptr && gamma != nullptr) gai_launch_error(__FILE__, __LINE__, "gemv: SwiGLU staging has no norm");
  if (epi == GV_PART && (ks < 1 || (K / 32) % (ks * 4 * kGf) || (N / 16) * ks > kGvfMaxItems))
    gai_launch_error(__FILE__, __LINE__, "gemv: K parts do not divide the column");
  GemvArgs a{};
  a.swi = swi;
  a.ks = ks;
  a.x = (const bf16*)x;
  a.gamma = (const bf16*)gamma;
  a.eps = eps;
  a.W = (const bf16*)W;
  a.M = M;
  a.N = N;
  a.K = K;
  a.out = out;
  a.res = (bf16*)res;
  switch (epi) {
    case GV_PLAIN: gemv_launch<GV_PLAIN>(a, st, wfrag); return;
    case GV_RESIDUAL: gemv_launch<GV_RESIDUAL>(a, st, wfrag); return;
    case GV_SWIGLU: gemv_launch<GV_SWIGLU>(a, st, wfrag); return;
    case GV_F32: gemv_launch<GV_F32>(a, st, wfrag); return;
    case GV_PART: gemv_launch<GV_PART>(a, st, wfrag); return;
    default: gai_launch_error(__FILE__, __LINE__, "gemv: unknown epilogue");
  }
}

// QKV projection + RoPE + q / paged K, V^T stores (head_dim 128, bf16 cache), normalised input when gamma.
void gai_gemv_rope_kv(const void* x, const void* gamma, float eps, const void* W, int M, int K, const int* pos,
                      const float* cos_sin, const int* slots, void* q_out, void* k_cache, void* v_cache, int Hq,
                      int Hkv, hipStream_t st, int wfrag) {
  const int N = (Hq + 2 * Hkv) * 128;
  if (!gai_gemv_ok(M, N, K, gamma != nullptr)) gai_launch_error(__FILE__, __LINE__, "gemv_rope_kv: shape");
  GemvArgs a{};
  a.x = (const bf16*)x;
  a.gamma = (const bf16*)gamma;
  a.eps = eps;
  a.W = (const bf16*)W;
  a.M = M;
  a.N = N;
  a.K = K;
  a.pos = pos;
  a.cos_sin = cos_sin;
  a.slots = slots;
  a.q_out = (bf16*)q_out;
  a.k_cache = (bf16*)k_cache;
  a.v_cache = (bf16*)v_cache;
  a.Hq = Hq;
  a.Hkv = Hkv;
  gemv_launch<GV_ROPE>(a, st, wfrag);
}
