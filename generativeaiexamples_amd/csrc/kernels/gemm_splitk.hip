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
#include "gai_common.h"
#include "gai_epilogue.h"
#include "gai_kernels.h"

using namespace gai;

namespace {

constexpr int kRing = 16;            // k-steps (of 32) of weight fragments in flight per wave
constexpr int kKAlign = kRing * 32;  // K-slice granularity

template <int MB>
__global__ __launch_bounds__(256) void gemm_splitk_kernel(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                                          float* __restrict__ part, int M, int N, int K, int KL) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // A slice [16*MB][KL] bf16, swizzled chunks
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = blockIdx.x * 64;
  const int ks = blockIdx.y;
  const int k0 = ks * KL;
  const int cpr = KL / 8;  // 16-B chunks per staged row (multiple of 64)
  constexpr int ROWS = 16 * MB;

  // ---- stage the activation slice: chunk p -> row p / cpr, physical chunk pc, logical pc ^ (row & 15)
  const int chunks = ROWS * cpr;  // multiple of 256 (cpr % 64 == 0, ROWS % 16 == 0)
  for (int base = wid * 64; base < chunks; base += 256) {
    const int p = base + lane;
    const int row = p / cpr, pc = p % cpr, c = pc ^ (row & 15);
    const bf16* src = A + (size_t)min(row, M - 1) * K + k0 + c * 8;
    __builtin_amdgcn_global_load_lds(src, GAI_LDS(smem + (size_t)base * 16), 16, 0, 0);
  }

  // ---- weight stream of this wave: rows n0 + 16*wid + (lane & 15)
  const int n = min(n0 + 16 * wid + (lane & 15), N - 1);
  const bf16* wp = W + (size_t)n * K + k0 + 8 * (lane >> 4);
  const int nsteps = KL / 32;  // multiple of kRing
  bf16x8 ring[kRing];
#pragma unroll
  for (int u = 0; u < kRing; ++u) ring[u] = load8(wp + u * 32);

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
      ring[u] = load8(wp + (s + kRing + u) * 32);
      step(s + u, b);
    }
  }
#pragma unroll
  for (int u = 0; u < kRing; ++u) step(s + u, ring[u]);

  // ---- partials: lane holds D[m = 16i + 4(lane>>4) + r][n = 16*wid + (lane&15)]
  const int nc = n0 + 16 * wid + (lane & 15);
  if (nc < N) {
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * i + 4 * (lane >> 4) + r;
        if (m < M) part[((size_t)ks * M + m) * N + nc] = acc[i][r];
      }
  }
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
    float vg = 0.f, vu = 0.f;
    for (int s = 0; s < KS; ++s) {
      const float* p = part + ((size_t)s * M + m) * N;
      vg += p[g];
      vu += p[g + 16];
    }
    store_out<EPI_NONE, OUTF32>(C, nullptr, nullptr, ldc, m, j, silu(vg) * vu);
  } else {
    float v = 0.f;
    for (int s = 0; s < KS; ++s) v += part[((size_t)s * M + m) * N + j];
    store_out<EPI, OUTF32>(C, bias, R, ldc, m, j, v);
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

// K-split chosen so the grid reaches ~2 workgroups per CU while the staged slice fits the LDS.
int gai_gemm_splitk_ks(int M, int N, int K) {
  if (K % kKAlign) return 0;
  const int MB = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  const int kl_max = (128 * 1024) / (16 * MB * 2);  // LDS bytes / row bytes
  const int units = K / kKAlign;
  const int tiles = (N + 63) / 64;
  int best = units;  // KS = units / d for a divisor d of units
  for (int d = units; d >= 1; --d) {
    if (units % d) continue;
    const int KS = units / d, KL = d * kKAlign;
    if (KL > kl_max) continue;
    best = KS;
    if ((long)tiles * KS >= 512) break;  // largest slice that still fills the chip
  }
  return best;
}

size_t gai_gemm_splitk_ws_bytes(int M, int N, int K) {
  const int KS = gai_gemm_splitk_ks(M, N, K);
  return (size_t)KS * M * N * sizeof(float);
}

void gai_gemm_splitk(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                     int ldc, int epi, int out_f32, float* ws, hipStream_t st) {
  if (M == 0 || N == 0) return;
  if (M > 64) gai_launch_error(__FILE__, __LINE__, "gemm_splitk: M must be <= 64");
  const int KS = gai_gemm_splitk_ks(M, N, K);
  if (KS == 0) gai_launch_error(__FILE__, __LINE__, "gemm_splitk: K must be a multiple of 512");
  const int KL = K / KS;
  const int MB = M <= 16 ? 1 : M <= 32 ? 2 : 4;
  const size_t lds = (size_t)16 * MB * KL * 2;
  dim3 grid((N + 63) / 64, KS);
#define GAI_SK(MBV)                                                                                          \
  case MBV: {                                                                                                \
    static bool once = false;                                                                                \
    if (!once) {                                                                                             \
      hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_splitk_kernel<MBV>),                            \
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);                           \
      once = true;                                                                                           \
    }                                                                                                        \
    gemm_splitk_kernel<MBV><<<grid, 256, lds, st>>>((const bf16*)A, (const bf16*)B, ws, M, N, K, KL);        \
    GAI_LAUNCH_CHECK();                                                                                      \
    break;                                                                                                   \
  }
  switch (MB) {
    GAI_SK(1)
    GAI_SK(2)
    GAI_SK(4)
  }
#undef GAI_SK
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
