// Decode-GEMM streaming microbenchmark (M <= 64 rows of activations, weights [N][K] bf16 from HBM).
// Question it answers: which load shape / ring depth / occupancy lets a weight-streaming MFMA kernel
// reach HBM speed at M = 64, where the framework's split-K kernel measured 2.9 TB/s.
// Each wave owns 16 output columns x the whole K and streams its weight rows through a register ring
// (branch-free, kSlots = DEPTH + 1 sets). Variants:
//   MODE 0: W fragment-shaped loads (16 rows x 64 B per wave load), A fragments held in registers
//   MODE 1: W fragment-shaped + A fragment loads from global (L2-resident), as the framework kernel
//   MODE 2: W pre-shuffled (1 KiB contiguous per wave load), A in registers
//   MODE 3: W fragment-shaped + A from an LDS copy (staged once per block, ds_read_b128)
// build: hipcc -O3 --offload-arch=gfx950 -o /tmp/dec_stream tools/microbench/dec_stream.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int MODE, int DEPTH, int MB, int WPB, bool NTL = false>
__global__ __launch_bounds__(64 * WPB) void stream_kernel(const bf16* __restrict__ W, const bf16* __restrict__ A,
                                                          float* __restrict__ out, int N, int K) {
  constexpr int kSlots = DEPTH + 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nt = blockIdx.x * WPB + wid;  // 16-column tile of this wave
  const int nsteps = K / 32;
  const bf16* wp = MODE == 2 ? W + ((size_t)nt * nsteps * 64 + lane) * 8
                             : W + (size_t)(nt * 16 + (lane & 15)) * K + 8 * (lane >> 4);
  constexpr int kStepW = MODE == 2 ? 512 : 32;
  const bf16* ap = A + (size_t)(lane & 15) * K + 8 * (lane >> 4);
  // MODE 4 = MODE 1 with each wave walking K in a rotated order (start step differs per wave), so the
  // chip's waves do not all hit the same activation lines (one L2 channel) at the same moment
  const int rot = MODE == 4 ? (nt * 5) & (nsteps - 1) : 0;
  if (MODE == 3) {  // stage A [16*MB][K] rows once (K*2 B per row), plain copy
    const int bytes = 16 * MB * K * 2;
    for (int o = threadIdx.x * 16; o < bytes; o += 64 * WPB * 16)
      *reinterpret_cast<bf16x8*>(smem + o) = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(A) + o);
    __syncthreads();
  }
  bf16x8 areg[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) areg[i] = *reinterpret_cast<const bf16x8*>(ap + (size_t)16 * i * K);
  bf16x8 rw[kSlots], ra[kSlots][MB];
  f32x4 acc[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto load = [&](int s, int slot) {
    s = (s + rot) & (nsteps - 1);
    if (NTL)
      rw[slot] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(wp + (size_t)kStepW * s));
    else
      rw[slot] = *reinterpret_cast<const bf16x8*>(wp + (size_t)kStepW * s);
    if (MODE == 1 || MODE == 4) {
#pragma unroll
      for (int i = 0; i < MB; ++i) ra[slot][i] = *reinterpret_cast<const bf16x8*>(ap + (size_t)16 * i * K + 32 * s);
    }
  };
  auto mma = [&](int s, int slot) {
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      bf16x8 a = areg[i];
      if (MODE == 1 || MODE == 4) a = ra[slot][i];
      if (MODE == 3)
        a = *reinterpret_cast<const bf16x8*>(smem + ((size_t)(16 * i + (lane & 15)) * K + 32 * s + 8 * (lane >> 4)) * 2);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, rw[slot], acc[i], 0, 0, 0);
    }
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) load(d, d);
  int s = 0;
  for (; s + kSlots <= nsteps; s += kSlots) {
#pragma unroll
    for (int d = 0; d < kSlots; ++d) {
      load(min(s + d + DEPTH, nsteps - 1), (d + DEPTH) % kSlots);
      mma(s + d, d);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int d = 0; d < kSlots - 1; ++d)
    if (s + d < nsteps) mma(s + d, d);
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < MB; ++i) v += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[(size_t)nt * 64 + lane] = v;
}

template <int MODE, int DEPTH, int MB, int WPB, bool NTL = false>
void run(const char* name, int N, int K, std::vector<bf16*>& Ws, const bf16* A, float* out) {
  const int tiles = N / 16;
  const int blocks = tiles / WPB;
  const int lds = MODE == 3 ? 16 * MB * K * 2 : 0;
  auto kern = stream_kernel<MODE, DEPTH, MB, WPB, NTL>;
  if (lds) CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 40;
  for (int w = 0; w < 4; ++w) kern<<<blocks, 64 * WPB, lds>>>(Ws[w % Ws.size()], A, out, N, K);
  CK(hipEventRecord(e0));
  for (int it = 0; it < iters; ++it) kern<<<blocks, 64 * WPB, lds>>>(Ws[it % Ws.size()], A, out, N, K);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / iters;
  printf("{\"kernel\": \"%s\", \"nt\": %d, \"mode\": %d, \"depth\": %d, \"MB\": %d, \"wpb\": %d, \"N\": %d, \"K\": %d, \"blocks\": %d, "
         "\"us\": %.2f, \"TBps\": %.3f}\n", name, (int)NTL, MODE, DEPTH, MB, WPB, N, K, blocks, us, (double)N * K * 2 / (us * 1e6));
  fflush(stdout);
}

int main() {
  const int K = 4096;
  const int Ns[2] = {28672, 6144};
  const int NMAX = 28672;
  std::vector<bf16*> Ws;
  const int copies = 4;  // 4 x 235 MB: beyond the 256 MB Infinity Cache
  std::vector<uint16_t> h((size_t)NMAX * K);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 0x3c00 + (uint16_t)((i * 2654435761u) >> 24 & 0x7f);  // ~[0.0078, 0.016)
  for (int c = 0; c < copies; ++c) {
    bf16* w;
    CK(hipMalloc(&w, (size_t)NMAX * K * 2));
    CK(hipMemcpy(w, h.data(), (size_t)NMAX * K * 2, hipMemcpyHostToDevice));
    Ws.push_back(w);
  }
  bf16* A;
  CK(hipMalloc(&A, (size_t)64 * K * 2));
  CK(hipMemcpy(A, h.data(), (size_t)64 * K * 2, hipMemcpyHostToDevice));
  float* out;
  CK(hipMalloc(&out, (size_t)NMAX * 64 * 4));
  for (int N : Ns) {
    run<0, 8, 4, 4>("wfrag_areg", N, K, Ws, A, out);
    run<1, 6, 4, 4>("wfrag_aglobal", N, K, Ws, A, out);
    run<4, 6, 4, 4>("wfrag_aglobal_rot", N, K, Ws, A, out);
    run<4, 6, 4, 1>("wfrag_aglobal_rot", N, K, Ws, A, out);
    run<4, 8, 4, 2>("wfrag_aglobal_rot", N, K, Ws, A, out);
    run<4, 6, 1, 4>("wfrag_aglobal_rot", N, K, Ws, A, out);
    run<4, 6, 2, 4>("wfrag_aglobal_rot", N, K, Ws, A, out);
    run<2, 8, 4, 1, true>("wpsw_areg", N, K, Ws, A, out);
    run<2, 8, 4, 1>("wpsw_areg", N, K, Ws, A, out);
  }
  printf("done\n");
  return 0;
}
