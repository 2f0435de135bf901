// FP8 (OCP e4m3fn) GEMM on the block-scaled CDNA4 MFMA (BASELINE config 4 "CDNA4 fp8 MFMA").
//
// C[M, N] = (Aq[M, K] . Bq[N, K]^T) * sa[m] * sb[n]  (+ the bf16 GEMM epilogues)
//
// Aq is a per-token (row) quantised activation produced by quant_rows_fp8 below, Bq a per-output-
// channel quantised weight (quantised once at load time by the same kernel). The K-loop runs on
// v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales (e8m0 127 = 2^0): on gfx950 the scaled
// form issues twice the K per cycle of the bf16 MFMA (MI355X_MICROARCH "FP8 ~5 PF dense"), while the
// non-scaled fp8 MFMA only runs at the bf16 rate. Per-row / per-channel scales are applied once in
// the fp32 epilogue, so the inner loop is pure MFMA.
//
// Structure: 128x128 block tile with BK = 128 k (= 128 bytes per row, the same LDS image as the bf16
// tiled kernel's 64 bf16), 4 waves as 2x2, each wave 64x64 = 4x4 MFMA tiles; operands staged by
// global_load_lds_dwordx4 into a lane-linear, XOR-swizzled image, double buffered. The MFMA's A/B
// fragment is 32 fp8 per lane (lane l: row l&15, k-bytes 32*(l>>4) .. +31), i.e. two adjacent 16-B
// chunks of one row, read with two ds_read_b128.
#include "gai_common.h"
#include "gai_epilogue.h"
#include "gai_kernels.h"

using namespace gai;

namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int FBM = 128, FBN = 128, FBK = 128;  // BK in fp8 elements == bytes
constexpr int kFTile = FBM * FBK;                // 16 KiB per operand tile
constexpr float kFp8Max = 448.f;
constexpr int kUnitScale = 127;                  // e8m0 encoding of 2^0

__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, GAI_LDS(lds), 16, 0, 0);
}

template <int EPI, bool OUTF32>
__global__ __launch_bounds__(256, 2) void gemm_fp8_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                          const float* __restrict__ sa, const float* __restrict__ sb,
                                                          void* C, const bf16* bias, const bf16* R, int M, int N,
                                                          int K, int ldc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 x (A 16K + B 16K)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = (M + FBM - 1) / FBM, tiles_n = (N + FBN - 1) / FBN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 8;
  const int group = wg / (GM * tiles_n);
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int pin = wg % (GM * tiles_n);
  const int tm = first_m + pin % gsz, tn = pin / gsz;
  const int m0 = tm * FBM, n0 = tn * FBN;

  size_t a_off[4], b_off[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = (wid * 4 + q) * 64 + lane;
    const int row = p >> 3, cl = p & 7, cg = cl ^ (row & 7);
    a_off[q] = (size_t)min(m0 + row, M - 1) * K + cg * 16;
    b_off[q] = (size_t)min(n0 + row, N - 1) * K + cg * 16;
  }
  auto stage = [&](int kt, int buf) {
    char* s_a = smem + buf * 2 * kFTile;
    char* s_b = s_a + kFTile;
    const size_t k0 = (size_t)kt * FBK;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      glds16(A + a_off[q] + k0, s_a + (wid * 4 + q) * 1024);
      glds16(B + b_off[q] + k0, s_b + (wid * 4 + q) * 1024);
    }
  };

  const int wm = wid >> 1, wn = wid & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LDS byte offsets of the two 16-B chunks (2g, 2g+1) of each fragment row
  int a_rd[4][2], b_rd[4][2];
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = 2 * g + h;
      const int ra = wm * 64 + 16 * i + (lane & 15);
      const int rb = wn * 64 + 16 * i + (lane & 15);
      a_rd[i][h] = ra * 128 + ((c ^ (ra & 7)) << 4);
      b_rd[i][h] = rb * 128 + ((c ^ (rb & 7)) << 4);
    }

  const int nk = K / FBK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const char* s_a = smem + cur * 2 * kFTile;
    const char* s_b = s_a + kFTile;
    i32x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const i32x4 a0 = *reinterpret_cast<const i32x4*>(s_a + a_rd[i][0]);
      const i32x4 a1 = *reinterpret_cast<const i32x4*>(s_a + a_rd[i][1]);
      const i32x4 b0 = *reinterpret_cast<const i32x4*>(s_b + b_rd[i][0]);
      const i32x4 b1 = *reinterpret_cast<const i32x4*>(s_b + b_rd[i][1]);
      af[i] = i32x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      bfr[i] = i32x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, kUnitScale,
                                                                     0, kUnitScale);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane holds D[m = 4(lane>>4)+r][n = lane&15] of each 16x16 tile
  float srow[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
      srow[i][r] = m < M ? sa[m] : 0.f;
    }
  if (EPI == EPI_SWIGLU) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int nout = (n0 + wn * 64) / 2 + 16 * jp + (lane & 15);
        if (2 * nout >= N) continue;
        const int ng = n0 + wn * 64 + 32 * jp + (lane & 15);
        const float sg = sb[ng], su = sb[ng + 16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
          if (m >= M) continue;
          const float gt = acc[i][2 * jp][r] * srow[i][r] * sg, u = acc[i][2 * jp + 1][r] * srow[i][r] * su;
          store_out<EPI_NONE, OUTF32>(C, nullptr, nullptr, ldc, m, nout, silu(gt) * u);
        }
      }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + 16 * j + (lane & 15);
      if (n >= N) continue;
      const float scol = sb[n];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
          if (m < M) store_out<EPI, OUTF32>(C, bias, R, ldc, m, n, acc[i][j][r] * srow[i][r] * scol);
        }
    }
  }
}

// ----------------------------------------------------------------------------------------------
// Large fp8 kernel (M >= 1024): the 256x256 four-phase pipeline of gemm.hip's gemm_large_kernel on
// v_mfma_scale_f32_32x32x64_f8f6f4. A K-tile is 128 k held as four 16 KiB K-halves
// [A-k0 | B-k0 | A-k1 | B-k1] of 256 rows x 64 fp8 (64-B rows: byte-identical to the bf16 kernel's
// 32-k halves), so staging, swizzle and the counted-vmcnt barrier schedule carry over unchanged while
// every phase issues twice the FLOPs (4 MFMAs 32x32x64 at 64 cycles = the bf16 phase's 16 x 16x16x32).
// 8 waves as 2(M) x 4(N), each 128x64 = 4x2 tiles of 32x32 (8 x f32x16 = 128 accumulator VGPRs).
// Fragment of lane l: row l&31, k-bytes 32*(l>>5) .. +31 = logical 16-B chunks 2(l>>5), 2(l>>5)+1.
// ----------------------------------------------------------------------------------------------
constexpr int LBM = 256, LBN = 256, LBK = 128;
constexpr int kHalfBytes = 256 * 64;

__device__ __forceinline__ int lswz(int r) { return (4 - ((r >> 2) & 3)) & 3; }

template <int EPI, bool OUTF32>
__global__ __launch_bounds__(512, 1) void gemm_fp8_large_kernel(const uint8_t* __restrict__ A,
                                                                const uint8_t* __restrict__ B,
                                                                const float* __restrict__ sa,
                                                                const float* __restrict__ sb, void* C,
                                                                const bf16* bias, const bf16* R, int M, int N, int K,
                                                                int ldc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
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

  size_t a_src[2], b_src[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int q = wid * 2 + j;
    const int row = q * 16 + (lane >> 2);
    const int cg = (lane & 3) ^ lswz(row);
    a_src[j] = (size_t)min(m0 + row, M - 1) * K + cg * 16;
    b_src[j] = (size_t)min(n0 + row, N - 1) * K + cg * 16;
  }
  auto stage = [&](int kt, int h, int buf) {
    const uint8_t* src = (h & 1) ? B : A;
    const size_t* off = (h & 1) ? b_src : a_src;
    char* dst = smem + buf * 4 * kHalfBytes + h * kHalfBytes;
    const size_t k0 = (size_t)kt * LBK + (h >> 1) * 64;
#pragma unroll
    for (int j = 0; j < 2; ++j) glds16(src + off[j] + k0, dst + (wid * 2 + j) * 1024);
  };

  const int wm = wid >> 2, wn = wid & 3;
  const int hl = lane >> 5;
  // chunk 2hl+1 sits at (chunk 2hl's physical position) ^ 1, i.e. byte offset ^ 16
  int a_rd[4], b_rd[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wm * 128 + 32 * i + (lane & 31);
    a_rd[i] = r * 64 + (((2 * hl) ^ lswz(r)) << 4);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = wn * 64 + 32 * j + (lane & 31);
    b_rd[j] = r * 64 + (((2 * hl) ^ lswz(r)) << 4);
  }

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = K / LBK;
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h, 0);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  auto frag = [&](const char* s, int off) -> i32x8 {
    const i32x4 x0 = *reinterpret_cast<const i32x4*>(s + off);
    const i32x4 x1 = *reinterpret_cast<const i32x4*>(s + (off ^ 16));
    return __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto rd_a = [&](i32x8* f, const char* buf, int kh, int hm) {
    const char* s = buf + (2 * kh) * kHalfBytes;
#pragma unroll
    for (int i = 0; i < 2; ++i) f[i] = frag(s, a_rd[2 * hm + i]);
  };
  auto rd_b = [&](i32x8* f, const char* buf, int kh) {
    const char* s = buf + (2 * kh + 1) * kHalfBytes;
#pragma unroll
    for (int j = 0; j < 2; ++j) f[j] = frag(s, b_rd[j]);
  };
  auto mma = [&](const i32x8* af, const i32x8* bfr, int hm) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[2 * hm + i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af[i], bfr[j], acc[2 * hm + i][j], 0, 0,
                                                                             0, kUnitScale, 0, kUnitScale);
    // the MFMAs have no side effects: without this pin LLVM sinks all 16 of them below the phase
    // barriers (de-pipelining the loop and spilling the prefetched fragments)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[2 * hm + i][j]));
    __builtin_amdgcn_s_setprio(0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  i32x8 bk0[2], bk1[2], aT0[2], aB0[2], aT1[2], aB1[2];
  rd_b(bk0, smem, 0);
  rd_a(aT0, smem, 0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    const char* base = smem + cur * 4 * kHalfBytes;
    const char* nbase = smem + (cur ^ 1) * 4 * kHalfBytes;
    if (more) stage(kt + 1, 0, cur ^ 1);
    rd_a(aB0, base, 0, 1);
    mma(aT0, bk0, 0);
    if (more) {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();
    if (more) stage(kt + 1, 1, cur ^ 1);
    rd_b(bk1, base, 1);
    rd_a(aT1, base, 1, 0);
    mma(aB0, bk0, 1);
    barrier();
    if (more) stage(kt + 1, 2, cur ^ 1);
    rd_a(aB1, base, 1, 1);
    mma(aT1, bk1, 0);
    if (more) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    barrier();
    if (more) {
      stage(kt + 1, 3, cur ^ 1);
      rd_b(bk0, nbase, 0);
      rd_a(aT0, nbase, 0, 0);
    }
    mma(aB1, bk1, 1);
    barrier();
  }

  // epilogue: 32x32 tile element (row (r&3) + 8(r>>2) + 4*hl, col lane&31)
  const int col = lane & 31;
  if (EPI == EPI_SWIGLU) {
    // per 32-col tile: cols 0-15 gate, 16-31 up of the same 16 outputs -> pair lanes l and l^16
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ng = n0 + wn * 64 + 32 * j + (col & 15);
      const int nout = (n0 + wn * 64) / 2 + 16 * j + (col & 15);
      const bool valid = 2 * nout < N;
      const float sg = valid ? sb[ng] : 0.f, su = valid ? sb[ng + 16] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float other = __shfl_xor(acc[i][j][r], 16, 64);
          const int m = m0 + wm * 128 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if ((col & 16) || !valid || m >= M) continue;
          const float s_m = sa[m];
          store_out<EPI_NONE, OUTF32>(C, nullptr, nullptr, ldc, m, nout,
                                      silu(acc[i][j][r] * s_m * sg) * (other * s_m * su));
        }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + 32 * j + col;
      if (n >= N) continue;
      const float scol = sb[n];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 128 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (m < M) store_out<EPI, OUTF32>(C, bias, R, ldc, m, n, acc[i][j][r] * sa[m] * scol);
        }
    }
  }
}

// ----------------------------------------------------------------------------------------------
// Per-row dynamic quantisation bf16 -> fp8 e4m3fn (+ fp32 scale = amax / 448). One 256-thread block
// per row: 16-B bf16 loads, block amax, then packed conversions (v_cvt_pk_fp8_f32, OCP on gfx950)
// written 8 bytes per lane. Used for activations (per token) and for weights (per output channel).
// ----------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void quant_rows_fp8_kernel(const bf16* __restrict__ x, int K, long ldx,
                                                             uint8_t* __restrict__ q, float* __restrict__ scale) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const bf16* xr = x + (size_t)row * ldx;
  float amax = 0.f;
  for (int c = threadIdx.x * 8; c < K; c += 256 * 8) {
    const bf16x8 v = load8(xr + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf((float)v[e]));
  }
  amax = block_max(amax, red);
  const float s = fmaxf(amax, 1e-12f) / kFp8Max;
  // x * (1 / s), one multiply per element (ops.reference.quant_rows_fp8 does the same) instead of an IEEE x / s
  // (~10 VALU per element) on every prefill activation
  const float inv = 1.f / s;
  if (threadIdx.x == 0) scale[row] = s;
  uint8_t* qr = q + (size_t)row * K;
  for (int c = threadIdx.x * 8; c < K; c += 256 * 8) {
    const bf16x8 v = load8(xr + c);
    int w0 = 0, w1 = 0;
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[0] * inv, (float)v[1] * inv, w0, false);
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[2] * inv, (float)v[3] * inv, w0, true);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[4] * inv, (float)v[5] * inv, w1, false);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[6] * inv, (float)v[7] * inv, w1, true);
    *reinterpret_cast<int2*>(qr + c) = make_int2(w0, w1);
  }
}

template <int EPI, bool OUTF32>
void launch_fp8(const void* A, const void* B, const float* sa, const float* sb, void* C, const void* bias,
                const void* R, int M, int N, int K, int ldc, int force, hipStream_t st) {
  // 256x256 pipeline when the grid fills whole waves of the 256 CUs and K amortises its prologue
  // (measured: 1.5-wave grids and K = 1024 run faster on the 128x128 kernel; a K = 1280 grid of many
  // waves, the vision encoder's 204928 x 5120 fc1, runs 3.32 ms here vs 3.84 ms on the 128x128 kernel)
  const int t256 = ((M + LBM - 1) / LBM) * ((N + LBN - 1) / LBN);
  const float fill = (float)t256 / (float)(((t256 + 255) / 256) * 256);
  const bool deep_k = K >= 2048 || (K >= 1024 && t256 >= 8 * 256);
  const bool large_ok = M >= 1024 && N >= 256 && deep_k && fill >= 0.8f;
  if (force == 3 || (force == 0 && large_ok)) {
    static bool once = false;
    if (!once) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_fp8_large_kernel<EPI, OUTF32>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      once = true;
    }
    const int tiles = ((M + LBM - 1) / LBM) * ((N + LBN - 1) / LBN);
    gemm_fp8_large_kernel<EPI, OUTF32><<<tiles, 512, 8 * kHalfBytes, st>>>(
        (const uint8_t*)A, (const uint8_t*)B, sa, sb, C, (const bf16*)bias, (const bf16*)R, M, N, K, ldc);
    GAI_LAUNCH_CHECK();
    return;
  }
  const int tiles = ((M + FBM - 1) / FBM) * ((N + FBN - 1) / FBN);
  gemm_fp8_kernel<EPI, OUTF32><<<tiles, 256, 4 * kFTile, st>>>((const uint8_t*)A, (const uint8_t*)B, sa, sb, C,
                                                                (const bf16*)bias, (const bf16*)R, M, N, K, ldc);
  GAI_LAUNCH_CHECK();
}

}  // namespace

void gai_quant_rows_fp8(const void* x, int M, int K, long ldx, void* q, float* scale, hipStream_t st) {
  if (M == 0) return;
  if (K % 8) gai_launch_error(__FILE__, __LINE__, "quant_rows_fp8: K must be a multiple of 8");
  quant_rows_fp8_kernel<<<M, 256, 0, st>>>((const bf16*)x, K, ldx, (uint8_t*)q, scale);
  GAI_LAUNCH_CHECK();
}

void gai_gemm_fp8(const void* A, const void* B, const float* sa, const float* sb, void* C, const void* bias,
                  const void* R, int M, int N, int K, int ldc, int epi, int out_f32, int force, hipStream_t st) {
  if (M == 0 || N == 0) return;
  if (K % FBK) gai_launch_error(__FILE__, __LINE__, "gemm_fp8: K must be a multiple of 128");
#define GAI_FP8_EPI(E)                                                         \
  case E:                                                                      \
    if (out_f32)                                                               \
      launch_fp8<E, true>(A, B, sa, sb, C, bias, R, M, N, K, ldc, force, st);         \
    else                                                                       \
      launch_fp8<E, false>(A, B, sa, sb, C, bias, R, M, N, K, ldc, force, st);        \
    return;
  switch (epi) {
    GAI_FP8_EPI(EPI_NONE)
    GAI_FP8_EPI(EPI_BIAS)
    GAI_FP8_EPI(EPI_BIAS_GELU)
    GAI_FP8_EPI(EPI_RESIDUAL)
    GAI_FP8_EPI(EPI_SWIGLU)
    GAI_FP8_EPI(EPI_BIAS_RESIDUAL)
    GAI_FP8_EPI(EPI_BIAS_QUICKGELU)
    default:
      gai_launch_error(__FILE__, __LINE__, "gemm_fp8: unsupported epilogue");
  }
#undef GAI_FP8_EPI
}
