// bf16 GEMM on MFMA with fused epilogues (SURVEY K1, K8, K9 epilogues).
//
// C[M, N] = A[M, K] . B[N, K]^T  (torch Linear convention: weights are [out, in]).
//
// Two kernels, chosen by M:
//  * gemm_tiled  (M > 128, prefill / encoder): 128x128x64 block tile, 4 waves as
//    2x2, each wave 64x64 = 4x4 v_mfma_f32_16x16x32_bf16 tiles. Both operands are
//    staged global->LDS with global_load_lds_dwordx4 (16 B/lane, lane-linear LDS
//    image, XOR swizzle applied on the *source* address and on the ds_read side,
//    cdna_hip_programming §5 rule 21 / T2), double-buffered, one barrier per K
//    tile; XCD-aware bijective block remap + grouped-M raster for L2 reuse (T1).
//  * gemm_skinny (M <= 128, decode): the weight stream dominates. 8 waves per
//    workgroup split K eight ways *inside* the workgroup (no global split-K
//    slabs, no atomics); operands are loaded straight to VGPRs (decode GEMV row
//    of the glds-vs-register table); partials are reduced through LDS and the
//    epilogue writes coalesced rows.
// Epilogues: none | +bias | +bias,GELU | +bias,ReLU | +residual | SwiGLU (weights interleaved
// per 16 rows [gate16 | up16 | ...], output width N/2) | +bias+residual, bf16 or
// fp32 output (fp32 for LM-head logits).
#include "gai_common.h"
#include "gai_kernels.h"
#include "gai_epilogue.h"

using namespace gai;

namespace {

// ----------------------------------------------------------------------------------------------
// Tiled kernel
// ----------------------------------------------------------------------------------------------
constexpr int TBM = 128, TBN = 128, TBK = 64;
constexpr int kTileBytes = TBM * TBK * 2;  // 16 KiB per operand tile

__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, GAI_LDS(lds), 16, 0, 0);
}

template <int EPI, bool OUTF32>
__global__ __launch_bounds__(256, 2) void gemm_tiled_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                            void* C, const bf16* bias, const bf16* R, int M, int N,
                                                            int K, int ldc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 x (A 16K + B 16K)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = (M + TBM - 1) / TBM, tiles_n = (N + TBN - 1) / TBN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 8;
  const int group = wg / (GM * tiles_n);
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int pin = wg % (GM * tiles_n);
  const int tm = first_m + pin % gsz, tn = pin / gsz;
  const int m0 = tm * TBM, n0 = tn * TBN;

  // per-lane staging source offsets (4 glds per operand per wave per K tile)
  size_t a_off[4], b_off[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = (wid * 4 + q) * 64 + lane;
    const int row = p >> 3, cl = p & 7, cg = cl ^ (row & 7);
    a_off[q] = (size_t)min(m0 + row, M - 1) * K + cg * 8;
    b_off[q] = (size_t)min(n0 + row, N - 1) * K + cg * 8;
  }
  auto stage = [&](int kt, int buf) {
    char* sa = smem + buf * 2 * kTileBytes;
    char* sb = sa + kTileBytes;
    const int k0 = kt * TBK;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      glds16(A + a_off[q] + k0, sa + (wid * 4 + q) * 1024);
      glds16(B + b_off[q] + k0, sb + (wid * 4 + q) * 1024);
    }
  };

  const int wm = wid >> 1, wn = wid & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (bytes inside a tile) for k-step s: chunk c = 4s + (lane>>4)
  int a_rd[4][2], b_rd[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 4 * s + (lane >> 4);
      const int ra = wm * 64 + 16 * i + (lane & 15);
      const int rb = wn * 64 + 16 * i + (lane & 15);
      a_rd[i][s] = ra * 128 + ((c ^ (ra & 7)) << 4);
      b_rd[i][s] = rb * 128 + ((c ^ (rb & 7)) << 4);
    }

  const int nk = K / TBK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const char* sa = smem + cur * 2 * kTileBytes;
    const char* sb = sa + kTileBytes;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = *reinterpret_cast<const bf16x8*>(sa + a_rd[i][s]);
        bfr[i] = *reinterpret_cast<const bf16x8*>(sb + b_rd[i][s]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane holds D[m = 4(lane>>4)+r][n = lane&15] of each 16x16 tile
  if (EPI == EPI_SWIGLU) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int nout = (n0 + wn * 64) / 2 + 16 * jp + (lane & 15);
        if (2 * nout >= N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
          if (m >= M) continue;
          const float g = acc[i][2 * jp][r], u = acc[i][2 * jp + 1][r];
          store_out<EPI_NONE, OUTF32>(C, nullptr, nullptr, ldc, m, nout, silu(g) * u);
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + 16 * j + (lane & 15);
        if (n >= N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
          if (m < M) store_out<EPI, OUTF32>(C, bias, R, ldc, m, n, acc[i][j][r]);
        }
      }
  }
}

// ----------------------------------------------------------------------------------------------
// Large kernel (prefill, M >= 1024): 256x256x64 block tile, 8 waves as 2(M) x 4(N), each wave
// 128x64 = 8x4 MFMA 16x16x32 tiles (128 accumulator VGPRs). A K-tile is held as four 16 KiB
// K-halves [A-k0 | B-k0 | A-k1 | B-k1] (256 rows x 32 k, 64-B rows); two buffers = 128 KiB LDS.
// Each K-tile runs 4 phases of 16 MFMAs (k-half x {top, bottom} 64 rows of the wave's A), and each
// phase issues ONE K-half of the next K-tile by global_load_lds (2 per wave): a K-half is issued
// 3-4 phases before its first read, so loads stay in flight across the phase barriers (raw
// s_barrier + counted vmcnt(4) at the end of phases 2 and 4; never a __syncthreads() vmcnt(0) drain,
// cdna_hip_programming §5 "Pipelining across barriers", T3/T4). 64-B rows are XOR-swizzled by
// G[(row>>2)&3] = {0,3,2,1} on the 16-B chunk: conflict-free for all four ds_read_b128 lane groups.
// ----------------------------------------------------------------------------------------------
constexpr int LBM = 256, LBN = 256, LBK = 64;
constexpr int kHalfBytes = 256 * 32 * 2;  // one K-half of one operand

__device__ __forceinline__ int lswz(int r) { return (4 - ((r >> 2) & 3)) & 3; }

template <int EPI, bool OUTF32>
__global__ __launch_bounds__(512, 1) void gemm_large_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                            void* C, const bf16* bias, const bf16* R, int M, int N,
                                                            int K, int ldc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 buffers x [A-k0 | B-k0 | A-k1 | B-k1]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = (M + LBM - 1) / LBM, tiles_n = (N + LBN - 1) / LBN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 4;
  const int group = wg / (GM * tiles_n);
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int pin = wg % (GM * tiles_n);
  const int tm = first_m + pin % gsz, tn = pin / gsz;
  const int m0 = tm * LBM, n0 = tn * LBN;

  // staging: each wave issues 2 x 1 KiB (16 rows x 64 B) per K-half; lane -> (row, physical chunk)
  size_t a_src[2], b_src[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int q = wid * 2 + j;
    const int row = q * 16 + (lane >> 2);
    const int cg = (lane & 3) ^ lswz(row);
    a_src[j] = (size_t)min(m0 + row, M - 1) * K + cg * 8;
    b_src[j] = (size_t)min(n0 + row, N - 1) * K + cg * 8;
  }
  // K-half h (0: A-k0, 1: B-k0, 2: A-k1, 3: B-k1) of K-tile kt into buffer buf
  auto stage = [&](int kt, int h, int buf) {
    const bf16* src = (h & 1) ? B : A;
    const size_t* off = (h & 1) ? b_src : a_src;
    char* dst = smem + buf * 4 * kHalfBytes + h * kHalfBytes;
    const int k0 = kt * LBK + (h >> 1) * 32;
#pragma unroll
    for (int j = 0; j < 2; ++j) glds16(src + off[j] + k0, dst + (wid * 2 + j) * 1024);
  };

  const int wm = wid >> 2, wn = wid & 3;
  // fragment read byte offsets inside a K-half: row r, logical chunk c = lane>>4
  int a_rd[8], b_rd[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = wm * 128 + 16 * i + (lane & 15);
    a_rd[i] = r * 64 + (((lane >> 4) ^ lswz(r)) << 4);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = wn * 64 + 16 * j + (lane & 15);
    b_rd[j] = r * 64 + (((lane >> 4) ^ lswz(r)) << 4);
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / LBK;
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h, 0);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // k0 halves of tile 0 landed
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  // Register double-buffering: every phase first issues the ds_reads of the NEXT phase's
  // fragments, then runs its 16 MFMAs on fragments read one phase earlier, so LDS latency hides
  // under the MFMAs. Data a prefetch reads must be valid one phase earlier than its use, hence
  // the counted waits at the end of phases 1 and 3 (vmcnt(2): the one younger K-half may fly on).
  auto rd_a = [&](bf16x8* f, const char* buf, int kh, int hm) {
    const char* s = buf + (2 * kh) * kHalfBytes;
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = *reinterpret_cast<const bf16x8*>(s + a_rd[4 * hm + i]);
  };
  auto rd_b = [&](bf16x8* f, const char* buf, int kh) {
    const char* s = buf + (2 * kh + 1) * kHalfBytes;
#pragma unroll
    for (int j = 0; j < 4; ++j) f[j] = *reinterpret_cast<const bf16x8*>(s + b_rd[j]);
  };
  auto mma = [&](const bf16x8* af, const bf16x8* bfr, int hm) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[4 * hm + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[4 * hm + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  bf16x8 bk0[4], bk1[4], aT0[4], aB0[4], aT1[4], aB1[4];
  rd_b(bk0, smem, 0);
  rd_a(aT0, smem, 0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    const char* base = smem + cur * 4 * kHalfBytes;
    const char* nbase = smem + (cur ^ 1) * 4 * kHalfBytes;
    // phase 1: k0 x top rows
    if (more) stage(kt + 1, 0, cur ^ 1);
    rd_a(aB0, base, 0, 1);
    mma(aT0, bk0, 0);
    if (more) {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // k1 halves of this tile landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();
    // phase 2: k0 x bottom rows; prefetch k1 operands
    if (more) stage(kt + 1, 1, cur ^ 1);
    rd_b(bk1, base, 1);
    rd_a(aT1, base, 1, 0);
    mma(aB0, bk0, 1);
    barrier();
    // phase 3: k1 x top rows
    if (more) stage(kt + 1, 2, cur ^ 1);
    rd_a(aB1, base, 1, 1);
    mma(aT1, bk1, 0);
    if (more) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // k0 halves of the next tile landed
    barrier();
    // phase 4: k1 x bottom rows; prefetch the next tile's k0 operands
    if (more) {
      stage(kt + 1, 3, cur ^ 1);
      rd_b(bk0, nbase, 0);
      rd_a(aT0, nbase, 0, 0);
    }
    mma(aB1, bk1, 1);
    barrier();
  }

  if (EPI == EPI_SWIGLU) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int nout = (n0 + wn * 64) / 2 + 16 * jp + (lane & 15);
        if (2 * nout >= N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 128 + 16 * i + 4 * (lane >> 4) + r;
          if (m >= M) continue;
          store_out<EPI_NONE, OUTF32>(C, nullptr, nullptr, ldc, m, nout, silu(acc[i][2 * jp][r]) * acc[i][2 * jp + 1][r]);
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + 16 * j + (lane & 15);
        if (n >= N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 128 + 16 * i + 4 * (lane >> 4) + r;
          if (m < M) store_out<EPI, OUTF32>(C, bias, R, ldc, m, n, acc[i][j][r]);
        }
      }
  }
}

// ----------------------------------------------------------------------------------------------
// Skinny kernel (decode): 8 waves split K inside the workgroup
// ----------------------------------------------------------------------------------------------
template <int MT, int NF, int EPI, bool OUTF32>
__global__ __launch_bounds__(512) void gemm_skinny_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                          void* C, const bf16* bias, const bf16* R, int M, int N,
                                                          int K, int ldc) {
  constexpr int NB = 16 * NF;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* part = reinterpret_cast<float*>(smem);  // [8 waves][MT][NF][4][64 lanes]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nb = xcd_remap(blockIdx.x, gridDim.x);
  const int n0 = nb * NB;
  const int KS = K / 8;
  const int kbeg = wid * KS, kend = kbeg + KS;

  const bf16* bp[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) bp[f] = B + (size_t)min(n0 + 16 * f + (lane & 15), N - 1) * K + 8 * (lane >> 4);
  const bf16* ap[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) ap[i] = A + (size_t)min(16 * i + (lane & 15), M - 1) * K + 8 * (lane >> 4);

  f32x4 acc[MT][NF];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 4
  for (int k = kbeg; k < kend; k += 32) {
    bf16x8 bfr[NF], af[MT];
#pragma unroll
    for (int f = 0; f < NF; ++f) bfr[f] = load8(bp[f] + k);
#pragma unroll
    for (int i = 0; i < MT; ++i) af[i] = load8(ap[i] + k);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int f = 0; f < NF; ++f) acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[f], acc[i][f], 0, 0, 0);
  }

#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[(((wid * MT + i) * NF + f) * 4 + r) * 64 + lane] = acc[i][f][r];
  __syncthreads();

  // element (m, n): i = m>>4, r = m&3, lane = ((m&15)>>2)*16 + (n&15), f = n>>4
  if (EPI == EPI_SWIGLU) {
    constexpr int NO = NB / 2;
    for (int e = tid; e < M * NO; e += 512) {
      const int m = e / NO, no = e % NO;
      const int fp = no >> 4, c = no & 15;
      const int i = m >> 4, r = m & 3, l = ((m & 15) >> 2) * 16 + c;
      float g = 0.f, u = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        g += part[(((w * MT + i) * NF + 2 * fp) * 4 + r) * 64 + l];
        u += part[(((w * MT + i) * NF + 2 * fp + 1) * 4 + r) * 64 + l];
      }
      const int nout = n0 / 2 + no;
      if (2 * nout < N) store_out<EPI_NONE, OUTF32>(C, nullptr, nullptr, ldc, m, nout, silu(g) * u);
    }
  } else {
    for (int e = tid; e < M * NB; e += 512) {
      const int m = e / NB, nn = e % NB;
      const int n = n0 + nn;
      if (n >= N) continue;
      const int i = m >> 4, r = m & 3, f = nn >> 4, l = ((m & 15) >> 2) * 16 + (nn & 15);
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += part[(((w * MT + i) * NF + f) * 4 + r) * 64 + l];
      store_out<EPI, OUTF32>(C, bias, R, ldc, m, n, v);
    }
  }
}

template <typename F>
void set_max_lds(F* f) {
  hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <int EPI, bool OUTF32>
void launch_tiled(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
                  hipStream_t st) {
  const int tiles = ((M + TBM - 1) / TBM) * ((N + TBN - 1) / TBN);
  static bool once = false;
  if (!once) {
    set_max_lds(gemm_tiled_kernel<EPI, OUTF32>);
    once = true;
  }
  gemm_tiled_kernel<EPI, OUTF32><<<tiles, 256, 4 * kTileBytes, st>>>((const bf16*)A, (const bf16*)B, C,
                                                                      (const bf16*)bias, (const bf16*)R, M, N, K, ldc);
  GAI_LAUNCH_CHECK();
}

template <int EPI, bool OUTF32>
void launch_large(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
                  hipStream_t st) {
  const int tiles = ((M + LBM - 1) / LBM) * ((N + LBN - 1) / LBN);
  static bool once = false;
  if (!once) {
    set_max_lds(gemm_large_kernel<EPI, OUTF32>);
    once = true;
  }
  gemm_large_kernel<EPI, OUTF32><<<tiles, 512, 8 * kHalfBytes, st>>>((const bf16*)A, (const bf16*)B, C,
                                                                      (const bf16*)bias, (const bf16*)R, M, N, K, ldc);
  GAI_LAUNCH_CHECK();
}

template <int MT, int NF, int EPI, bool OUTF32>
void launch_skinny_mt(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                      int ldc, hipStream_t st) {
  const int nblk = (N + 16 * NF - 1) / (16 * NF);
  const size_t lds = (size_t)8 * MT * NF * 4 * 64 * sizeof(float);
  static bool once = false;
  if (!once) {
    set_max_lds(gemm_skinny_kernel<MT, NF, EPI, OUTF32>);
    once = true;
  }
  gemm_skinny_kernel<MT, NF, EPI, OUTF32><<<nblk, 512, lds, st>>>((const bf16*)A, (const bf16*)B, C,
                                                                  (const bf16*)bias, (const bf16*)R, M, N, K, ldc);
  GAI_LAUNCH_CHECK();
}

template <int NF, int EPI, bool OUTF32>
void launch_skinny_nf(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                      int ldc, hipStream_t st) {
  if (M <= 16) return launch_skinny_mt<1, NF, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st);
  if (M <= 32) return launch_skinny_mt<2, NF, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st);
  if (M <= 64) return launch_skinny_mt<4, NF, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st);
  return launch_skinny_mt<8, NF, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st);
}

template <int EPI, bool OUTF32>
void launch_gemm(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                 int ldc, int force, hipStream_t st) {
  const bool skinny_ok = (K % 256) == 0 && M <= 128;
  const bool use_skinny = force == 1 || (force == 0 && skinny_ok);
  if (use_skinny) {
    if (!skinny_ok) gai_launch_error(__FILE__, __LINE__, "gemm_skinny: needs M<=128 and K%256==0");
    // two 16-row fragments per wave when there are enough column blocks to fill the chip
    if (EPI != EPI_SWIGLU && N / 32 >= 512)
      return launch_skinny_nf<2, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st);
    if (EPI == EPI_SWIGLU) return launch_skinny_nf<2, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st);
    return launch_skinny_nf<1, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st);
  }
  if (K % TBK) gai_launch_error(__FILE__, __LINE__, "gemm_tiled: K must be a multiple of 64");
  const bool large_ok = M >= 1024 && N >= 256;
  if (force == 3 || (force == 0 && large_ok)) return launch_large<EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st);
  launch_tiled<EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st);
}

}  // namespace

void gai_gemm(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
              int epi, int out_f32, int force, hipStream_t st) {
  if (M == 0 || N == 0) return;
#define GAI_GEMM_EPI(E)                                                              \
  case E:                                                                            \
    if (out_f32)                                                                     \
      launch_gemm<E, true>(A, B, C, bias, R, M, N, K, ldc, force, st);               \
    else                                                                             \
      launch_gemm<E, false>(A, B, C, bias, R, M, N, K, ldc, force, st);              \
    return;
  switch (epi) {
    GAI_GEMM_EPI(EPI_NONE)
    GAI_GEMM_EPI(EPI_BIAS)
    GAI_GEMM_EPI(EPI_BIAS_GELU)
    GAI_GEMM_EPI(EPI_RESIDUAL)
    GAI_GEMM_EPI(EPI_SWIGLU)
    GAI_GEMM_EPI(EPI_BIAS_RESIDUAL)
    GAI_GEMM_EPI(EPI_BIAS_RELU)
    GAI_GEMM_EPI(EPI_BIAS_QUICKGELU)
    default:
      gai_launch_error(__FILE__, __LINE__, "gemm: unknown epilogue");
  }
#undef GAI_GEMM_EPI
}
