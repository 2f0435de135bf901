// Weight-streaming split-K GEMM for decode-sized M (<= 64): C[M, N] = A[M, K] . W[N, K]^T (+ epilogue).
//
// Decode GEMMs read every weight byte once and do ~M MACs per byte, so they are HBM-bound; the
// library kernels leave the small-N projections (QKV, O, down) at 1.7-2.4 TB/s because a grid that
// fills 256 CUs with 16-64-column tiles re-reads the activation rows far more than the weights.
// Here:
//  * a workgroup (4 waves) owns 64 output columns x one K-slice; each wave owns 16 columns and
//    streams its 16 weight rows straight from HBM into MFMA B-fragments (lane l: row l&15, 16 B at
//    k = 8(l>>4)) through a 16-deep register ring (16 KiB in flight per wave, no LDS for W);
//  * the activation K-slice [16*MB x KL] is staged ONCE per workgroup into LDS with global_load_lds
//    (XOR-swizzled 16-B chunks, conflict-free ds_read_b128 of the A-fragments), so activation
//    traffic is 1/4 of the weight traffic even at M = 64;
//  * K is split over gridDim.y so every projection launches >= ~512 workgroups; fp32 partials land
//    in a workspace [KS, M, N] and a reduce kernel sums them and applies the fused epilogue
//    (bias / GELU / ReLU / quick-GELU / residual / interleaved SwiGLU), writing bf16 or fp32.
#include <type_traits>

#include "gai_common.h"
#include "gai_epilogue.h"
#include "gai_kernels.h"
#include "gai_rope.h"

using namespace gai;

namespace {

constexpr int kRing = 16;            // k-steps (of 32) of weight fragments in flight per wave
constexpr int kKAlign = kRing * 32;  // K-slice granularity

// Pre-shuffled weight layout [N/16][K/32][64 lanes][8]: fragment (nt, kt) holds, for lane l,
// W[16 nt + (l & 15)][32 kt + 8 (l >> 4) .. +7] - exactly the B operand of v_mfma_f32_16x16x32_bf16.
__device__ __forceinline__ size_t psw_offset(int nt, int kt, int K, int lane) {
  return (((size_t)nt * (K / 32) + kt) * 64 + lane) * 8;
}

// In-launch decode QKV tail (RopeTail): the K-slices of a 128-column tile (= one head at head_dim 128) hand their
// partials to the slice that finishes last, which sums them (+ bias), rounds to bf16, applies RoPE and writes q /
// the paged K, V^T caches - the work of splitk_rope_kv_kernel without its launch. Hand-off as the decode-attention
// split merge (cdna_hip_programming Guideline 16, R1): write-through (sc1) partial stores, every wave vmcnt(0),
// barrier, lane 0 relaxed agent ticket; the last arriver reads the slabs with sc1 loads. cnt[tile] is zero between
// launches (zeroed at allocation, reset by the last arriver).
struct RopeTail {
  int* cnt;
  const bf16* bias;
  const int* pos;
  const float* cos_sin;
  const int* slots;
  bf16* q_out;
  void* k_cache;
  void* v_cache;
  int Hq, Hkv;
  float inv_ks, inv_vs;
};
constexpr int kTailMaxKS = 8;  // K-slices one last arriver sums (legacy_ks never exceeds 8 at K <= 4096)

// Reducer of one 128-column tile = head h: 16 threads per token row, each owning rotation pairs (i0..i0+3,
// i0+64..i0+67), slabs summed in slice order from 0 (the rounding of sum_slabs / splitk_rope_kv_kernel).
template <typename KV>
__device__ void rope_tail_reduce(const float* part, int KS, int M, int N, int h, const RopeTail& t, int tid,
                                 int nthreads) {
  constexpr int D = 128, LPH = D / 8;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(part), (short)0, 0x7fffffff,
                                                                     0x00020000);
  for (int e = tid; e < M * LPH; e += nthreads) {
    const int row = e / LPH, i0 = (e % LPH) * 4;
    const int c1 = h * D + i0, c2 = c1 + D / 2;
    float4 x[kTailMaxKS][2];
#pragma unroll
    for (int k = 0; k < kTailMaxKS; ++k) {  // every slab load issued before the sums (sc1: past this CU's L1)
      const unsigned base = (unsigned)((((size_t)min(k, KS - 1) * M + row) * N) * 4);
      x[k][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, base + c1 * 4, 0, 16));
      x[k][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, base + c2 * 4, 0, 16));
    }
    float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < kTailMaxKS; ++k) {
      if (k < KS) {
        a[0] += x[k][0].x; a[1] += x[k][0].y; a[2] += x[k][0].z; a[3] += x[k][0].w;  // NOLINT
        b[0] += x[k][1].x; b[1] += x[k][1].y; b[2] += x[k][1].z; b[3] += x[k][1].w;  // NOLINT
      }
    }
    bf16x4 x1, x2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x1[j] = (bf16)(t.bias ? a[j] + (float)t.bias[c1 + j] : a[j]);
      x2[j] = (bf16)(t.bias ? b[j] + (float)t.bias[c2 + j] : b[j]);
    }
    rope_kv_store<D>(x1, x2, row, h, i0, t.pos, t.cos_sin, t.slots, t.q_out, reinterpret_cast<KV*>(t.k_cache),
                     reinterpret_cast<KV*>(t.v_cache), t.Hq, t.Hkv, 1, t.inv_ks, t.inv_vs);
  }
}

// NTW: the pre-shuffled weight stream is loaded non-temporally (read once per decode step), as gemm_dec2 does
template <int MB, bool PSW, int WPG, typename TAILKV = void, bool NTW = false>
__global__ __launch_bounds__(64 * WPG) void gemm_splitk_kernel(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                                               float* __restrict__ part, int M, int N, int K, int KL,
                                                               RopeTail tail = RopeTail{}) {
  constexpr bool TAIL = !std::is_void<TAILKV>::value;
  static_assert(!TAIL || WPG == 8, "the QKV tail owns one 128-column head per workgroup");
  extern __shared__ __attribute__((aligned(16))) char smem[];  // A slice [16*MB][KL] bf16, swizzled chunks
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = blockIdx.x * 16 * WPG;  // WPG waves x 16 columns share one staged activation slice
  const int ks = blockIdx.y;
  const int k0 = ks * KL;
  const int cpr = KL / 8;  // 16-B chunks per staged row (multiple of 64)
  constexpr int ROWS = 16 * MB;

  // ---- stage the activation slice: chunk p -> row p / cpr, physical chunk pc, logical pc ^ (row & 15)
  const int chunks = ROWS * cpr;  // multiple of 256 (cpr % 64 == 0, ROWS % 16 == 0)
  for (int base = wid * 64; base < chunks; base += 64 * WPG) {
    const int p = base + lane;
    const int row = p / cpr, pc = p % cpr, c = pc ^ (row & 15);
    const bf16* src = A + (size_t)min(row, M - 1) * K + k0 + c * 8;
    __builtin_amdgcn_global_load_lds(src, GAI_LDS(smem + (size_t)base * 16), 16, 0, 0);
  }

  // ---- weight stream of this wave: rows n0 + 16*wid + (lane & 15)
  // PSW: W is pre-shuffled into MFMA fragments (psw_offset): one k32 step of a 16-row tile is 1 KiB
  // contiguous, so a wave load is 8 whole 128-B lines instead of 16 half lines of 16 rows.
  const int n = min(n0 + 16 * wid + (lane & 15), N - 1);
  const bf16* wp = PSW ? W + psw_offset(min(n0 / 16 + wid, N / 16 - 1), k0 / 32, K, lane)
                       : W + (size_t)n * K + k0 + 8 * (lane >> 4);
  constexpr int kStepW = PSW ? 512 : 32;  // elements between consecutive k32 steps of one lane
  const int nsteps = KL / 32;  // multiple of kRing
  auto wload = [&](const bf16* p) -> bf16x8 {
    if constexpr (PSW && NTW) return __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(p));
    else return load8(p);
  };
  bf16x8 ring[kRing];
#pragma unroll
  for (int u = 0; u < kRing; ++u) ring[u] = wload(wp + u * kStepW);

  f32x4 acc[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // staged slice (and the first ring) landed
  __syncthreads();

  // A-fragment LDS offsets: row 16i + (lane & 15), logical chunk 4s + (lane >> 4)
  int arow[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) arow[i] = (16 * i + (lane & 15)) * cpr;
  const int rsw = lane & 15, cq = lane >> 4;

  auto step = [&](int s, const bf16x8& b) {
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int c = (4 * s + cq) ^ rsw;
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(smem + (size_t)(arow[i] + c) * 16);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
    }
  };

  int s = 0;
  for (; s + kRing < nsteps; s += kRing) {
#pragma unroll
    for (int u = 0; u < kRing; ++u) {
      const bf16x8 b = ring[u];
      ring[u] = wload(wp + (s + kRing + u) * kStepW);
      step(s + u, b);
    }
  }
#pragma unroll
  for (int u = 0; u < kRing; ++u) step(s + u, ring[u]);

  // ---- partials: lane holds D[m = 16i + 4(lane>>4) + r][n = 16*wid + (lane&15)]
  const int nc = n0 + 16 * wid + (lane & 15);
  if constexpr (!TAIL) {
    if (nc < N) {
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * i + 4 * (lane >> 4) + r;
          if (m < M) part[((size_t)ks * M + m) * N + nc] = acc[i][r];
        }
    }
  } else {
    // write-through partials as whole 16-B stores (a per-lane dword sc1 store is one fabric write each, ~6x the
    // time per byte): the [ROWS][128] fp32 tile goes through LDS (row stride 132 floats), then each thread
    // stores 16-B row pieces with sc1
    constexpr int TS = 16 * WPG + 4;
    float* tile = reinterpret_cast<float*>(smem);
    __syncthreads();  // every wave is done reading the staged activation slice
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) tile[(16 * i + 4 * (lane >> 4) + r) * TS + 16 * wid + (lane & 15)] = acc[i][r];
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(part, (short)0, 0x7fffffff, 0x00020000);
    for (int e = tid; e < ROWS * 4 * WPG; e += 64 * WPG) {
      const int m = e / (4 * WPG), c = 4 * (e % (4 * WPG));
      if (m < M) {
        const float4 v = *reinterpret_cast<const float4*>(tile + m * TS + c);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), rs,
                                               (unsigned)((((size_t)ks * M + m) * N + n0 + c) * 4), 0, 16);
      }
    }
  }
  if constexpr (TAIL) {
    // the flag word sits past the staged slice in the ONE dynamic LDS array (a second __shared__ object next to
    // global_load_lds staging can make hipcc wait vmcnt(0) in the k-loop)
    int* s_last = reinterpret_cast<int*>(smem + (size_t)chunks * 16);  // past the slice (>= the partial tile)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through partials have landed
    __syncthreads();
    if (tid == 0)
      *s_last = __hip_atomic_fetch_add(tail.cnt + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                (int)gridDim.y - 1;
    __syncthreads();
    if (!*s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
    rope_tail_reduce<TAILKV>(part, gridDim.y, M, N, blockIdx.x, tail, tid, 64 * WPG);
    if (tid == 0) __hip_atomic_store(tail.cnt + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------------------------------------
// Register-streamed variant (default). The kernel above stages the WHOLE activation K-slice in LDS,
// so at M = 64 the slice is capped at 1024 columns (128 KiB, one workgroup per CU): K is split
// 4-8 ways, the fp32 partials add 12-25 % to the weight traffic of the K = 4096 projections, and
// every wave streams a single 16 KiB ring fill before it drains. Here nothing is staged:
//  * a wave owns a 16*MB x 64 output tile (MB x 4 MFMA 16x16x32 blocks), so each k32 step loads
//    4 weight fragments from HBM and MB activation fragments (L2-resident, 1:1 with the weights at
//    M = 64) straight into a 3-deep register ring; only ordinary loads, so the compiler's counted
//    vmcnt keeps 3 steps in flight (no LDS-DMA / barrier in the loop);
//  * the 4 waves of a workgroup split K four ways over the SAME 64 columns and reduce through LDS
//    (row stride 68 floats: conflict-free), so a workgroup covers its whole K-slice with no global
//    partials; cross-workgroup KS > 1 is used only when the column tiles give < 256 workgroups;
//  * with KS = 1 the epilogue (SwiGLU on the [gate16|up16] interleave, bias, GELU, residual, fp32
//    logits) is applied by the workgroup itself: no reduce launch.
constexpr int kDepth = 3;    // k32 steps in flight per wave
constexpr int kSlots = kDepth + 1;  // register sets of the ring
constexpr int kLdsRow = 68;  // fp32 row stride of the reduction tiles

template <int MB>
constexpr int dec_lds_bytes() { return 4 * 16 * MB * kLdsRow * 4; }

template <int MB, int EPI, bool OUTF32, bool PSW>
__global__ __launch_bounds__(256, 2) void gemm_dec_kernel(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                                          float* __restrict__ part, void* __restrict__ C,
                                                          const bf16* __restrict__ bias, const bf16* R, int M, int N,
                                                          int K, int KW, int ldc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int ROWS = 16 * MB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = blockIdx.x * 64;
  const int ks = blockIdx.y, KS = gridDim.y;
  const int kbeg = (ks * 4 + wid) * KW;  // this wave's K range [kbeg, kbeg + KW)
  const int nsteps = KW / 32;
  const int kq = 8 * (lane >> 4);

  const bf16* ap[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) ap[i] = A + (size_t)min(16 * i + (lane & 15), M - 1) * K + kbeg + kq;
  const bf16* wp[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    wp[j] = PSW ? W + psw_offset(min(n0 / 16 + j, N / 16 - 1), kbeg / 32, K, lane)
                : W + (size_t)min(n0 + 16 * j + (lane & 15), N - 1) * K + kbeg + kq;
  constexpr int kStepW = PSW ? 512 : 32;

  bf16x8 ra[kSlots][MB], rw[kSlots][4];
  auto load = [&](int s, bf16x8 (&a)[MB], bf16x8 (&w)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = load8(wp[j] + kStepW * s);
#pragma unroll
    for (int i = 0; i < MB; ++i) a[i] = load8(ap[i] + 32 * s);
  };
  f32x4 acc[MB][4];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const bf16x8 (&a)[MB], const bf16x8 (&w)[4]) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], w[j], acc[i][j], 0, 0, 0);
  };

  // prologue, then per step: MFMAs on the oldest ring slot, refill that slot kDepth steps ahead.
  // The ring has kSlots = kDepth + 1 register sets: step s first issues the loads of step s + kDepth
  // into the set step s - 1 has just released, then runs its MFMAs, so kDepth steps are always in
  // flight. The loop is branch-free (past the end a load re-reads the last step, an L2 hit) and each
  // step is pinned by a sched_barrier: with a refill under a branch, or reusing the set being
  // multiplied, hipcc sank the refills below later MFMAs and waited vmcnt(0..3) at the top of every
  // ring turn, draining the pipeline (measured 2.7-3.5 TB/s at M = 64).
#pragma unroll
  for (int d = 0; d < kDepth; ++d) load(min(d, nsteps - 1), ra[d], rw[d]);
  int s = 0;
  for (; s + kSlots <= nsteps; s += kSlots) {
#pragma unroll
    for (int d = 0; d < kSlots; ++d) {
      load(min(s + d + kDepth, nsteps - 1), ra[(d + kDepth) % kSlots], rw[(d + kDepth) % kSlots]);
      mma(ra[d], rw[d]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // tail (< kSlots <= kDepth + 1 steps, all already loaded into sets 0, 1, ...)
#pragma unroll
  for (int d = 0; d < kSlots - 1; ++d)
    if (s + d < nsteps) mma(ra[d], rw[d]);

  // in-workgroup K reduction: tile[w][m][n] (row stride kLdsRow)
  float* tile = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        tile[(wid * ROWS + 16 * i + 4 * (lane >> 4) + r) * kLdsRow + 16 * j + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  // thread -> (row m, 16-column group q); ROWS * 4 items
  for (int e = tid; e < ROWS * 4; e += 256) {
    const int m = e >> 2, q = e & 3;
    float v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float* t = tile + (w * ROWS + m) * kLdsRow + 16 * q;
#pragma unroll
      for (int c = 0; c < 16; c += 4) {
        const float4 x = *reinterpret_cast<const float4*>(t + c);
        v[c] += x.x;
        v[c + 1] += x.y;
        v[c + 2] += x.z;
        v[c + 3] += x.w;
      }
    }
    if (m >= M) continue;
    if (KS > 1) {
      float* dst = part + ((size_t)ks * M + m) * N + n0 + 16 * q;
      if (n0 + 16 * q + 16 <= N) {
#pragma unroll
        for (int c = 0; c < 16; c += 4) *reinterpret_cast<float4*>(dst + c) = float4{v[c], v[c + 1], v[c + 2], v[c + 3]};
      } else {
        for (int c = 0; c < 16; ++c)
          if (n0 + 16 * q + c < N) dst[c] = v[c];
      }
      continue;
    }
    if (EPI == EPI_SWIGLU) {
      // columns [g16 u16 g16 u16]: the gate lanes (q even) pull the up half from the next group
      if (q & 1) continue;
      const float* up = tile + m * kLdsRow + 16 * (q + 1);
      float u[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) u[c] = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int c = 0; c < 16; ++c) u[c] += up[w * ROWS * kLdsRow + c];
      const int oc = n0 / 2 + 8 * q;
      if (n0 + 16 * q + 32 <= N && !OUTF32) {
        bf16x8 o0, o1;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          o0[c] = (bf16)(silu(v[c]) * u[c]);
          o1[c] = (bf16)(silu(v[8 + c]) * u[8 + c]);
        }
        store8(reinterpret_cast<bf16*>(C) + (size_t)m * ldc + oc, o0);
        store8(reinterpret_cast<bf16*>(C) + (size_t)m * ldc + oc + 8, o1);
      } else {
        for (int c = 0; c < 16; ++c)
          if (n0 + 16 * q + 16 + c < N) store_out<EPI_NONE, OUTF32>(C, nullptr, nullptr, ldc, m, oc + c, silu(v[c]) * u[c]);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if (n0 + 16 * q + c < N) store_out<EPI, OUTF32>(C, bias, R, ldc, m, n0 + 16 * q + c, v[c]);
    }
  }
}

// Sum the KS fp32 partial slabs (stride floats apart) of W consecutive values at p, slab 0 first (the
// same order as a plain loop, so every reduce path rounds identically). A runtime-trip loop waits for
// each slab's load before issuing the next; here 4 slabs are in flight at a time.
template <int W>
__device__ __forceinline__ void sum_slabs(const float* p, size_t stride, int KS, float (&v)[W]) {
  static_assert(W == 1 || W % 4 == 0, "W: 1 or a multiple of 4");
  int k = 0;
  for (; k + 4 <= KS; k += 4) {
    float x[4][W];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float* q = p + (size_t)(k + u) * stride;
      if constexpr (W == 1) {
        x[u][0] = q[0];
      } else {
#pragma unroll
        for (int c = 0; c < W; c += 4) {
          const float4 t = *reinterpret_cast<const float4*>(q + c);
          x[u][c] = t.x; x[u][c + 1] = t.y; x[u][c + 2] = t.z; x[u][c + 3] = t.w;  // NOLINT
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int c = 0; c < W; ++c) v[c] += x[u][c];
  }
  for (; k < KS; ++k) {
    const float* q = p + (size_t)k * stride;
#pragma unroll
    for (int c = 0; c < W; ++c) v[c] += q[c];
  }
}

// The same sum with the slab count known at compile time (the decode tails: KS = 4 for down, 8 for QKV / O):
// every slab load is issued before the first add - one memory round trip instead of KS / 4.
template <int W, int KSC>
__device__ __forceinline__ void sum_slabs_c(const float* p, size_t stride, float (&v)[W]) {
  float x[KSC][W];
#pragma unroll
  for (int u = 0; u < KSC; ++u) {
    const float* q = p + (size_t)u * stride;
#pragma unroll
    for (int c = 0; c < W; c += 4) {
      const float4 t = *reinterpret_cast<const float4*>(q + c);
      x[u][c] = t.x; x[u][c + 1] = t.y; x[u][c + 2] = t.z; x[u][c + 3] = t.w;  // NOLINT
    }
  }
#pragma unroll
  for (int u = 0; u < KSC; ++u)
#pragma unroll
    for (int c = 0; c < W; ++c) v[c] += x[u][c];
}

template <int W, int KSC>
__device__ __forceinline__ void sum_slabs_any(const float* p, size_t stride, int KS, float (&v)[W]) {
  if constexpr (KSC > 0) sum_slabs_c<W, KSC>(p, stride, v);
  else sum_slabs<W>(p, stride, KS, v);
}

// Sum the KS partial slabs and apply the epilogue. One thread per output element.
template <int EPI, bool OUTF32>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int KS, int M, int N,
                                                            void* C, const bf16* bias, const bf16* R, int ldc) {
  const int ncol = EPI == EPI_SWIGLU ? N / 2 : N;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)M * ncol) return;
  const int m = (int)(e / ncol), j = (int)(e % ncol);
  if (EPI == EPI_SWIGLU) {
    const int g = (j >> 4) * 32 + (j & 15);  // interleaved per 16: [gate16 | up16]
    float vg[1] = {0.f}, vu[1] = {0.f};
    sum_slabs<1>(part + (size_t)m * N + g, (size_t)M * N, KS, vg);
    sum_slabs<1>(part + (size_t)m * N + g + 16, (size_t)M * N, KS, vu);
    store_out<EPI_NONE, OUTF32>(C, nullptr, nullptr, ldc, m, j, silu(vg[0]) * vu[0]);
  } else {
    float v[1] = {0.f};
    sum_slabs<1>(part + (size_t)m * N + j, (size_t)M * N, KS, v);
    store_out<EPI, OUTF32>(C, bias, R, ldc, m, j, v[0]);
  }
}

template <int EPI, bool OUTF32>
void launch_reduce(const float* part, int KS, int M, int N, void* C, const void* bias, const void* R, int ldc,
                   hipStream_t st) {
  const int ncol = EPI == EPI_SWIGLU ? N / 2 : N;
  const long total = (long)M * ncol;
  splitk_reduce_kernel<EPI, OUTF32><<<(unsigned)((total + 255) / 256), 256, 0, st>>>(
      part, KS, M, N, C, (const bf16*)bias, (const bf16*)R, ldc);
  GAI_LAUNCH_CHECK();
}

}  // namespace

namespace {

// Waves per workgroup of the slice-staging kernel: every workgroup stages its activation K-slice once,
// so 8 waves (128 columns) halve the activation bytes per weight byte of 4 waves (64 columns).
int splitk_wpg() {
  static const int v = getenv("GAI_SPLITK_WPG") ? atoi(getenv("GAI_SPLITK_WPG")) : 8;
  return v == 4 ? 4 : 8;
}

// Legacy (whole-slice staging) K-split: the grid reaches ~2 workgroups per CU while the slice fits LDS.
int legacy_ks(int M, int N, int K) {
  if (K % kKAlign) return 0;
  const int MB = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  const int kl_max = (128 * 1024) / (16 * MB * 2);  // LDS bytes / row bytes
  const int units = K / kKAlign;
  const int tiles = (N + 16 * splitk_wpg() - 1) / (16 * splitk_wpg());
  // 192: Llama-3-8B B = 64 QKV takes 4 K-slices (192 workgroups, half the fp32 partial traffic of 8), O keeps 8
  // (4 would leave 128 workgroups): decode step 7.325 -> 7.226 ms (512: 8 slices for both; 128: 4 for both, 7.294;
  // profiles/r4/decode/decode_nt_split_ab.txt)
  // M <= 16 (16-row activation slab: less partial traffic per slice) takes twice the workgroups: Llama-3-8B ctx 2471
  // graph replay B = 8 3.921 -> 3.863 ms, B = 16 4.349 -> 4.309-4.322 ms (profiles/r6/decode/small_batch_split/)
  static const int env_wg = getenv("GAI_SPLITK_LEGACY_MINWG") ? atoi(getenv("GAI_SPLITK_LEGACY_MINWG")) : 0;
  const int min_wg = env_wg ? env_wg : (M <= 16 ? 384 : 192);
  int best = units;  // KS = units / d for a divisor d of units
  for (int d = units; d >= 1; --d) {
    if (units % d) continue;
    const int KS = units / d, KL = d * kKAlign;
    if (KL > kl_max) continue;
    best = KS;
    if ((long)tiles * KS >= min_wg) break;  // largest slice that still fills the chip
  }
  return best;
}

// Which variant serves a shape (measured on MI355X, profiles/r1/kernel_bench_decode_gemm_v2.jsonl): the
// register-streamed kernel wins on the wide (gate_up, lm_head: 1.1-1.3x) and deep (down: 1.1-1.4x)
// projections; the LDS-staged one stays ahead on the square K = 4096 ones (QKV, O) by 2-10 %.
// GAI_SPLITK_V = 1 / 2 forces the legacy / streamed variant.
bool use_legacy(int N, int K) {
  static const int v = getenv("GAI_SPLITK_V") ? atoi(getenv("GAI_SPLITK_V")) : 0;
  if (v) return v == 1;
  return K % kKAlign == 0 && K <= 4096 && N <= 8192;
}

// Register-streamed K-split across workgroups (each workgroup already splits its slice 4 ways over
// its waves): the smallest KS with K / (4 KS) a multiple of 32 that reaches kMinWG workgroups.
int stream_ks(int N, int K) {
  static const int min_wg = getenv("GAI_SPLITK_MINWG") ? atoi(getenv("GAI_SPLITK_MINWG")) : 256;
  if (K % 128) return 0;
  const int tiles = (N + 63) / 64;
  const int units = K / 128;
  for (int KS = 1; KS <= units; ++KS) {
    if (units % KS) continue;
    if ((long)tiles * KS >= min_wg) return KS;
  }
  return units;
}

}  // namespace

int gai_gemm_splitk_ks(int M, int N, int K) { return use_legacy(N, K) ? legacy_ks(M, N, K) : stream_ks(N, K); }

size_t gai_gemm_splitk_ws_bytes(int M, int N, int K) {
  const int KS = max(gai_gemm_splitk_ks(M, N, K), gai_gemm_dec2_partials_ks(M, N, K));
  return (size_t)(KS > 1 ? KS : 1) * M * N * sizeof(float);
}

namespace {

template <int MB, int EPI, bool OUTF32>
void launch_stream(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                   int ldc, int KS, float* ws, bool psw, hipStream_t st) {
  auto kern = psw ? gemm_dec_kernel<MB, EPI, OUTF32, true> : gemm_dec_kernel<MB, EPI, OUTF32, false>;
  static bool once[2] = {false, false};
  if (!once[psw]) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                        dec_lds_bytes<MB>());
    once[psw] = true;
  }
  dim3 grid((N + 63) / 64, KS);
  kern<<<grid, 256, dec_lds_bytes<MB>(), st>>>((const bf16*)A, (const bf16*)B, ws, C, (const bf16*)bias,
                                               (const bf16*)R, M, N, K, K / (4 * KS), ldc);
  GAI_LAUNCH_CHECK();
}

template <int MB>
void dispatch_stream_ks1(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                         int ldc, int epi, int out_f32, bool psw, hipStream_t st) {
#define GAI_SS(E)                                                                           \
  case E:                                                                                   \
    if (out_f32)                                                                            \
      launch_stream<MB, E, true>(A, B, C, bias, R, M, N, K, ldc, 1, nullptr, psw, st);      \
    else                                                                                    \
      launch_stream<MB, E, false>(A, B, C, bias, R, M, N, K, ldc, 1, nullptr, psw, st);     \
    return;
  switch (epi) {
    GAI_SS(EPI_NONE)
    GAI_SS(EPI_BIAS)
    GAI_SS(EPI_BIAS_GELU)
    GAI_SS(EPI_RESIDUAL)
    GAI_SS(EPI_SWIGLU)
    GAI_SS(EPI_BIAS_RESIDUAL)
    GAI_SS(EPI_BIAS_RELU)
    GAI_SS(EPI_BIAS_QUICKGELU)
    default:
      gai_launch_error(__FILE__, __LINE__, "gemm_splitk: unknown epilogue");
  }
#undef GAI_SS
}

}  // namespace

namespace {

// fp32 partials [KS, M, N] of A . W^T into ws (KS > 1), either kernel variant.
// Non-temporal loads of the pre-shuffled weight stream in the LDS-staged split-K kernel (GAI_SPLITK_NT=0: plain):
// Llama-3-8B B = 64 decode step 7.466 -> 7.398 ms (QKV / O projections; profiles/r4/decode/decode_nt_split_ab.txt)
bool splitk_ntw() {
  static const bool on = !(getenv("GAI_SPLITK_NT") && atoi(getenv("GAI_SPLITK_NT")) == 0);
  return on;
}

void launch_partials(const void* A, const void* B, int M, int N, int K, int KS, float* ws, int psw, hipStream_t st) {
  const int MB = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  if (!use_legacy(N, K)) {
    if (MB == 1) launch_stream<1, EPI_NONE, true>(A, B, nullptr, nullptr, nullptr, M, N, K, 0, KS, ws, psw, st);
    else if (MB == 2) launch_stream<2, EPI_NONE, true>(A, B, nullptr, nullptr, nullptr, M, N, K, 0, KS, ws, psw, st);
    else launch_stream<4, EPI_NONE, true>(A, B, nullptr, nullptr, nullptr, M, N, K, 0, KS, ws, psw, st);
    return;
  }
  const int KL = K / KS;
  const size_t lds = (size_t)16 * MB * KL * 2;
  const int wpg = splitk_wpg();
  dim3 grid((N + 16 * wpg - 1) / (16 * wpg), KS);
#define GAI_SK1(MBV, WPGV)                                                                                       \
  {                                                                                                              \
    static bool once = false;                                                                                    \
    if (!once) {                                                                                                 \
      hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_splitk_kernel<MBV, false, WPGV>),                   \
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);                               \
      hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_splitk_kernel<MBV, true, WPGV>),                    \
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);                               \
      hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_splitk_kernel<MBV, true, WPGV, void, true>),        \
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);                               \
      once = true;                                                                                               \
    }                                                                                                            \
    if (psw && splitk_ntw())                                                                                     \
      gemm_splitk_kernel<MBV, true, WPGV, void, true><<<grid, 64 * WPGV, lds, st>>>((const bf16*)A, (const bf16*)B, \
                                                                                    ws, M, N, K, KL);            \
    else if (psw)                                                                                                \
      gemm_splitk_kernel<MBV, true, WPGV><<<grid, 64 * WPGV, lds, st>>>((const bf16*)A, (const bf16*)B, ws, M, N, \
                                                                        K, KL);                                  \
    else                                                                                                         \
      gemm_splitk_kernel<MBV, false, WPGV><<<grid, 64 * WPGV, lds, st>>>((const bf16*)A, (const bf16*)B, ws, M,   \
                                                                         N, K, KL);                              \
    GAI_LAUNCH_CHECK();                                                                                          \
  }
#define GAI_SK(MBV)                   \
  case MBV:                           \
    if (wpg == 4) GAI_SK1(MBV, 4)     \
    else GAI_SK1(MBV, 8)              \
    break;
  switch (MB) {
    GAI_SK(1)
    GAI_SK(2)
    GAI_SK(4)
  }
#undef GAI_SK1
#undef GAI_SK
}

// Fused decode tail for TP = 1: h = sum_k partials (+ bias) rounded to bf16, r = bf16(h + res) written
// back to res, out = rmsnorm(r) * g. One 256-thread workgroup per row (16 columns per thread at
// N = 4096, NCH chunks of 8): replaces the split-K reduce launch AND the norm launch (whose 64-row
// grid is 16 workgroups) with one 64-workgroup kernel that issues every load of the row up front.
template <int NCH>
__global__ __launch_bounds__(256) void splitk_add_rmsnorm_kernel(const float* __restrict__ part, int KS, int M, int N,
                                                                 const bf16* __restrict__ bias, bf16* res,
                                                                 const bf16* __restrict__ g, float eps,
                                                                 bf16* __restrict__ out) {
  __shared__ float scratch[16];
  const int m = blockIdx.x, tid = threadIdx.x;
  float v[NCH][8];
  bf16x8 rr[NCH], gg[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < N) {
      rr[c] = load8(res + (size_t)m * N + idx);
      gg[c] = load8(g + idx);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
      sum_slabs<8>(part + (size_t)m * N + idx, (size_t)M * N, KS, v[c]);
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < N) {
      bf16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float h = v[c][j];
        if (bias) h += (float)bias[idx + j];
        r[j] = (bf16)((float)(bf16)h + (float)rr[c][j]);
        v[c][j] = (float)r[j];
        ss += v[c][j] * v[c][j];
      }
      store8(res + (size_t)m * N + idx, r);
    }
  }
  const float inv = rsqrtf(block_sum(ss, scratch) / N + eps);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int idx = (c * 256 + tid) * 8;
    if (idx < N) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)(v[c][j] * inv * (float)gg[c][j]);
      store8(out + (size_t)m * N + idx, o);
    }
  }
}

// The same tail with 1024 threads x 4 columns (N <= 4096): one workgroup per row is all the parallelism
// a batch-64 decode step has, so the row's slab loads are spread over 4x the waves to keep more of them
// in flight per CU.
template <int KSC>
__global__ __launch_bounds__(1024) void splitk_add_rmsnorm_w4_kernel(const float* __restrict__ part, int KS, int M,
                                                                     int N, const bf16* __restrict__ bias, bf16* res,
                                                                     const bf16* __restrict__ g, float eps,
                                                                     bf16* __restrict__ out) {
  __shared__ float scratch[16];
  const int m = blockIdx.x, idx = threadIdx.x * 4;
  const bool live = idx < N;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  bf16x4 rr, gg;
  if (live) {
    rr = *reinterpret_cast<const bf16x4*>(res + (size_t)m * N + idx);
    gg = *reinterpret_cast<const bf16x4*>(g + idx);
    sum_slabs_any<4, KSC>(part + (size_t)m * N + idx, (size_t)M * N, KS, v);
  }
  float ss = 0.f;
  if (live) {
    bf16x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float h = v[j];
      if (bias) h += (float)bias[idx + j];
      r[j] = (bf16)((float)(bf16)h + (float)rr[j]);
      v[j] = (float)r[j];
      ss += v[j] * v[j];
    }
    *reinterpret_cast<bf16x4*>(res + (size_t)m * N + idx) = r;
  }
  const float inv = rsqrtf(block_sum(ss, scratch) / N + eps);
  if (live) {
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (bf16)(v[j] * inv * (float)gg[j]);
    *reinterpret_cast<bf16x4*>(out + (size_t)m * N + idx) = o;
  }
}

}  // namespace

int gai_gemm_splitk_fusable_norm(int M, int N, int K) {
  return M >= 1 && M <= 64 && N % 8 == 0 && N <= 256 * 8 * 4 && gai_gemm_splitk_ks(M, N, K) > 1;
}

void gai_gemm_splitk_add_rmsnorm(const void* A, const void* B, const void* bias, void* res, const void* g, void* out,
                                 int M, int N, int K, float eps, float* ws, int psw, hipStream_t st) {
  if (M == 0) return;
  if (!gai_gemm_splitk_fusable_norm(M, N, K)) gai_launch_error(__FILE__, __LINE__, "gemm_splitk_add_rmsnorm: shape");
  if (gai_gemm_dec2_ok(M, N, K, bias ? EPI_BIAS : EPI_NONE)) {
    // decode GEMM into a bf16 scratch h (the workspace), then the residual-add RMSNorm kernel:
    // res = bf16(h + res), out = rmsnorm(res) * g - the same roundings as the fused tail
    bf16* h = reinterpret_cast<bf16*>(ws);
    gai_gemm_dec2(A, B, h, bias, nullptr, M, N, K, N, bias ? EPI_BIAS : EPI_NONE, 0, st, psw);
    gai_rmsnorm(h, res, res, g, out, M, N, eps, st);
    return;
  }
  // deep K (down): LDS-staged decode kernel writing K-split slabs
  const int ks2 = gai_gemm_dec2_partials(A, B, M, N, K, ws, st, psw);
  const int KS = ks2 ? ks2 : gai_gemm_splitk_ks(M, N, K);
  if (!ks2) launch_partials(A, B, M, N, K, KS, ws, psw, st);
  if (N <= 4096 && N % 4 == 0 && getenv("GAI_NORM_TAIL_256") == nullptr) {
#define GAI_W4(KC)                                                                                              \
    splitk_add_rmsnorm_w4_kernel<KC><<<M, 1024, 0, st>>>(ws, KS, M, N, (const bf16*)bias, (bf16*)res,          \
                                                         (const bf16*)g, eps, (bf16*)out);
    if (KS == 4) GAI_W4(4) else if (KS == 8) GAI_W4(8) else GAI_W4(0)
#undef GAI_W4
    GAI_LAUNCH_CHECK();
    return;
  }
  const int nch = (N + 2047) / 2048;
#define GAI_FN(NC)                                                                                          \
  if (nch == NC) {                                                                                          \
    splitk_add_rmsnorm_kernel<NC><<<M, 256, 0, st>>>(ws, KS, M, N, (const bf16*)bias, (bf16*)res,           \
                                                     (const bf16*)g, eps, (bf16*)out);                       \
    GAI_LAUNCH_CHECK();                                                                                     \
    return;                                                                                                 \
  }
  GAI_FN(1)
  GAI_FN(2)
  GAI_FN(3)
  GAI_FN(4)
#undef GAI_FN
}

namespace {

// Fused decode QKV tail: sum the KS partial slabs of the QKV projection (+ bias), round to bf16 exactly as
// the unfused GEMM output, then RoPE + q store + paged K / V^T cache write (gai_rope.h) - replaces the
// split-K reduce launch, the bf16 qkv round trip and the rope_kv launch. Thread mapping as rope_kv_kernel.
template <int D, typename KV, int KSC>
__global__ __launch_bounds__(256) void splitk_rope_kv_kernel(const float* __restrict__ part, int KS, int M, int N,
                                                             const bf16* __restrict__ bias, const int* __restrict__ pos,
                                                             const float* __restrict__ cos_sin,
                                                             const int* __restrict__ slots, bf16* __restrict__ q_out,
                                                             KV* __restrict__ k_cache, KV* __restrict__ v_cache, int Hq,
                                                             int Hkv, float inv_ks, float inv_vs) {
  constexpr int LPH = D / 8;
  constexpr int HPB = 256 / LPH;
  const int H = Hq + 2 * Hkv;
  const long item = (long)blockIdx.x * HPB + threadIdx.x / LPH;
  if (item >= (long)M * H) return;
  const int t = (int)(item / H), h = (int)(item % H);
  const int i0 = (threadIdx.x % LPH) * 4;
  const int c1 = h * D + i0, c2 = c1 + D / 2;
  float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
  sum_slabs_any<4, KSC>(part + (size_t)t * N + c1, (size_t)M * N, KS, a);
  sum_slabs_any<4, KSC>(part + (size_t)t * N + c2, (size_t)M * N, KS, b);
  bf16x4 x1, x2;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    x1[j] = (bf16)(bias ? a[j] + (float)bias[c1 + j] : a[j]);
    x2[j] = (bf16)(bias ? b[j] + (float)bias[c2 + j] : b[j]);
  }
  rope_kv_store<D>(x1, x2, t, h, i0, pos, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, 1, inv_ks, inv_vs);
}

}  // namespace

namespace {

// LDS-staged split-K QKV with the in-launch reduce + RoPE tail (RopeTail). Returns false when the shape is not
// the one the tail is written for (head_dim 128 = the 128-column tile, legacy kernel, 2..8 K-slices).
template <typename KV>
bool launch_rope_tail(const void* A, const void* B, int M, int N, int K, float* ws, int psw, const RopeTail& t,
                      hipStream_t st) {
  if (!use_legacy(N, K) || splitk_wpg() != 8 || N % 128) return false;
  const int KS = legacy_ks(M, N, K);
  if (KS < 2 || KS > kTailMaxKS) return false;
  const int MB = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  const int KL = K / KS;
  const size_t lds = (size_t)16 * MB * KL * 2 + 16;  // + the last-arriver flag
  dim3 grid(N / 128, KS);
#define GAI_RT(MBV)                                                                                           \
  if (MB == MBV) {                                                                                            \
    static bool once = false;                                                                                 \
    if (!once) {                                                                                              \
      hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_splitk_kernel<MBV, false, 8, KV>),               \
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);                            \
      hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_splitk_kernel<MBV, true, 8, KV>),                \
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);                            \
      once = true;                                                                                            \
    }                                                                                                         \
    if (psw)                                                                                                  \
      gemm_splitk_kernel<MBV, true, 8, KV><<<grid, 512, lds, st>>>((const bf16*)A, (const bf16*)B, ws, M, N, K, \
                                                                   KL, t);                                    \
    else                                                                                                      \
      gemm_splitk_kernel<MBV, false, 8, KV><<<grid, 512, lds, st>>>((const bf16*)A, (const bf16*)B, ws, M, N,   \
                                                                    K, KL, t);                                \
    GAI_LAUNCH_CHECK();                                                                                       \
    return true;                                                                                              \
  }
  GAI_RT(1)
  GAI_RT(2)
  GAI_RT(4)
#undef GAI_RT
  return false;
}

}  // namespace

int gai_gemm_splitk_rope_kv(const void* A, const void* B, const void* bias, const int* pos, const float* cos_sin,
                            const int* slots, void* q_out, void* k_cache, void* v_cache, int M, int Hq, int Hkv,
                            int D, int kv_fp8, float k_scale, float v_scale, float* ws, int psw, hipStream_t st,
                            int K, int* tail_cnt) {
  const int N = (Hq + 2 * Hkv) * D;
  if (M < 1 || M > 64 || (D != 64 && D != 128 && D != 256) || N % 16) return 0;
  if (gai_gemm_dec2_ok(M, N, K, bias ? EPI_BIAS : EPI_NONE)) return 0;  // single-pass kernel owns it
  const int ks2 = gai_gemm_dec2_partials_ks(M, N, K);
  if (tail_cnt != nullptr && D == 128 && !ks2) {
    const RopeTail t{tail_cnt, (const bf16*)bias, pos, cos_sin, slots, (bf16*)q_out, k_cache, v_cache, Hq, Hkv,
                     1.f / k_scale, 1.f / v_scale};
    if (kv_fp8 ? launch_rope_tail<fp8>(A, B, M, N, K, ws, psw, t, st)
               : launch_rope_tail<bf16>(A, B, M, N, K, ws, psw, t, st))
      return 1;
  }
  const int KS = ks2 ? ks2 : gai_gemm_splitk_ks(M, N, K);
  if (KS <= 1) return 0;
  if (ks2)
    gai_gemm_dec2_partials(A, B, M, N, K, ws, st, psw);
  else
    launch_partials(A, B, M, N, K, KS, ws, psw, st);
  const long items = (long)M * (Hq + 2 * Hkv);
  const float iks = 1.f / k_scale, ivs = 1.f / v_scale;
#define GAI_SRK(DD)                                                                                               \
  if (D == DD) {                                                                                                  \
    constexpr int HPB = 256 / (DD / 8);                                                                           \
    const unsigned grid = (unsigned)((items + HPB - 1) / HPB);                                                    \
    if (kv_fp8)                                                                                                   \
      splitk_rope_kv_kernel<DD, fp8, 0><<<grid, 256, 0, st>>>(ws, KS, M, N, (const bf16*)bias, pos, cos_sin,      \
                                                              slots, (bf16*)q_out, (fp8*)k_cache, (fp8*)v_cache,  \
                                                              Hq, Hkv, iks, ivs);                                 \
    else if (KS == 8)                                                                                             \
      splitk_rope_kv_kernel<DD, bf16, 8><<<grid, 256, 0, st>>>(ws, KS, M, N, (const bf16*)bias, pos, cos_sin,     \
                                                               slots, (bf16*)q_out, (bf16*)k_cache,               \
                                                               (bf16*)v_cache, Hq, Hkv, iks, ivs);                \
    else if (KS == 4)  /* Llama-3-8B QKV at B = 64 (legacy_ks, min 192 workgroups) */                             \
      splitk_rope_kv_kernel<DD, bf16, 4><<<grid, 256, 0, st>>>(ws, KS, M, N, (const bf16*)bias, pos, cos_sin,     \
                                                               slots, (bf16*)q_out, (bf16*)k_cache,               \
                                                               (bf16*)v_cache, Hq, Hkv, iks, ivs);                \
    else                                                                                                          \
      splitk_rope_kv_kernel<DD, bf16, 0><<<grid, 256, 0, st>>>(ws, KS, M, N, (const bf16*)bias, pos, cos_sin,     \
                                                               slots, (bf16*)q_out, (bf16*)k_cache,               \
                                                               (bf16*)v_cache, Hq, Hkv, iks, ivs);                \
    GAI_LAUNCH_CHECK();                                                                                           \
    return 1;                                                                                                     \
  }
  GAI_SRK(64)
  GAI_SRK(128)
  GAI_SRK(256)
#undef GAI_SRK
  return 0;
}

int gai_gemm_qkv_partials(const void* A, const void* B, int M, int N, int K, float* ws, int psw, hipStream_t st) {
  if (M < 1 || M > 64 || N % 16) return 0;
  if (gai_gemm_dec2_ok(M, N, K, EPI_NONE)) return 0;  // single-pass kernel owns it
  const int ks2 = gai_gemm_dec2_partials_ks(M, N, K);
  const int KS = ks2 ? ks2 : gai_gemm_splitk_ks(M, N, K);
  // up to 16 slabs: the TP = 8 shard of Llama-3-70B (N 1280, K 8192) takes 16 K-slices to reach 192 workgroups;
  // GAI_QKV_FOLD_MAXKS = 8 restores the round-5 limit (A/B)
  static const int max_ks = getenv("GAI_QKV_FOLD_MAXKS") ? atoi(getenv("GAI_QKV_FOLD_MAXKS")) : 16;
  if (KS < 2 || KS > max_ks) return 0;
  if (ks2)
    gai_gemm_dec2_partials(A, B, M, N, K, ws, st, psw);
  else
    launch_partials(A, B, M, N, K, KS, ws, psw, st);
  return KS;
}

void gai_gemm_splitk(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                     int ldc, int epi, int out_f32, float* ws, int psw, hipStream_t st) {
  if (psw && N % 16) gai_launch_error(__FILE__, __LINE__, "gemm_splitk: pre-shuffled weights need N % 16 == 0");
  if (M == 0 || N == 0) return;
  if (M > 64) gai_launch_error(__FILE__, __LINE__, "gemm_splitk: M must be <= 64");
  // natural weight layout: the LDS-staged decode kernel (gemm_decode.hip) when the shape fits - single
  // pass for the wide projections, K-split slabs for the deep ones
  if (gai_gemm_dec2(A, B, C, bias, R, M, N, K, ldc, epi, out_f32, st, psw)) return;
  const int ks2 = gai_gemm_dec2_partials(A, B, M, N, K, ws, st, psw);
  const int KS = ks2 ? ks2 : gai_gemm_splitk_ks(M, N, K);
  if (KS == 0) gai_launch_error(__FILE__, __LINE__, "gemm_splitk: K must be a multiple of 512");
  const int MB = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  if (!use_legacy(N, K) && KS == 1) {
    if (MB == 1) dispatch_stream_ks1<1>(A, B, C, bias, R, M, N, K, ldc, epi, out_f32, psw, st);
    else if (MB == 2) dispatch_stream_ks1<2>(A, B, C, bias, R, M, N, K, ldc, epi, out_f32, psw, st);
    else dispatch_stream_ks1<4>(A, B, C, bias, R, M, N, K, ldc, epi, out_f32, psw, st);
    return;
  }
  if (!ks2) launch_partials(A, B, M, N, K, KS, ws, psw, st);
#define GAI_SKR(E)                                                         \
  case E:                                                                  \
    if (out_f32)                                                           \
      launch_reduce<E, true>(ws, KS, M, N, C, bias, R, ldc, st);           \
    else                                                                   \
      launch_reduce<E, false>(ws, KS, M, N, C, bias, R, ldc, st);          \
    return;
  switch (epi) {
    GAI_SKR(EPI_NONE)
    GAI_SKR(EPI_BIAS)
    GAI_SKR(EPI_BIAS_GELU)
    GAI_SKR(EPI_RESIDUAL)
    GAI_SKR(EPI_SWIGLU)
    GAI_SKR(EPI_BIAS_RESIDUAL)
    GAI_SKR(EPI_BIAS_RELU)
    GAI_SKR(EPI_BIAS_QUICKGELU)
    default:
      gai_launch_error(__FILE__, __LINE__, "gemm_splitk: unknown epilogue");
  }
#undef GAI_SKR
}
