// Ablation microbenchmark of the persistent 4-wave prefill GEMM (gemm.hip gemm_w4p_kernel): where do
// the matrix-pipe idle cycles come from? Each variant drops one part of the main loop (results are
// garbage for VAR != 0; only the time matters):
//   VAR 0: the framework kernel         VAR 1: no global->LDS loads / vmcnt waits in the loop
//   VAR 2: no barriers at phase ends    VAR 4: no fragment ds_reads (MFMAs on stale registers)
//   VAR 8: full-line (128 B) glds requests, k64 double-unit request count (wrong data)
//   combinations OR the bits (VAR 7 = MFMAs + loop control only); w4d = the full-line double-unit kernel
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I generativeaiexamples_amd/csrc/include \
//          -o /tmp/gemm_w4p_ab tools/microbench/gemm_w4p_ab.hip
#define GAI_GEMM_KERNELS_ONLY
#include "../../generativeaiexamples_amd/csrc/kernels/gemm_impl.h"

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill_kernel(bf16* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = (bf16)(((int)(h & 1023) - 512) / 512.f);
  }
}

template <int VAR>
float run(const bf16* A, const bf16* B, bf16* C, int M, int N, int K, int grid, int iters) {
  auto k = gemm_w4p_kernel<EPI_NONE, false, VAR>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, RNS * kUnitBytes));
  hipEvent_t ev0, ev1;
  CK(hipEventCreate(&ev0));
  CK(hipEventCreate(&ev1));
  k<<<grid, 256, RNS * kUnitBytes>>>(A, B, C, nullptr, nullptr, M, N, K, N);
  CK(hipEventRecord(ev0));
  for (int i = 0; i < iters; ++i) k<<<grid, 256, RNS * kUnitBytes>>>(A, B, C, nullptr, nullptr, M, N, K, N);
  CK(hipEventRecord(ev1));
  CK(hipEventSynchronize(ev1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, ev0, ev1));
  return ms / iters;
}

template <int WV>
float run_w4d(const bf16* A, const bf16* B, bf16* C, int M, int N, int K, int grid, int iters) {
  auto k = gemm_w4d_kernel<EPI_NONE, false, WV>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kDblBytes));
  hipEvent_t ev0, ev1;
  CK(hipEventCreate(&ev0));
  CK(hipEventCreate(&ev1));
  k<<<grid, 256, 2 * kDblBytes>>>(A, B, C, nullptr, nullptr, M, N, K, N, RopeKvArgs{}, 0);
  CK(hipEventRecord(ev0));
  for (int i = 0; i < iters; ++i) k<<<grid, 256, 2 * kDblBytes>>>(A, B, C, nullptr, nullptr, M, N, K, N, RopeKvArgs{}, 0);
  CK(hipEventRecord(ev1));
  CK(hipEventSynchronize(ev1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, ev0, ev1));
  return ms / iters;
}

float run_w4r(const bf16* A, const bf16* B, bf16* C, int M, int N, int K, int grid, int iters) {
  auto k = gemm_w4r_kernel<EPI_NONE, false>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 5 * kPart));
  hipEvent_t ev0, ev1;
  CK(hipEventCreate(&ev0));
  CK(hipEventCreate(&ev1));
  k<<<grid, 256, 5 * kPart>>>(A, B, C, nullptr, nullptr, M, N, K, N, nullptr, nullptr, 1, 0);
  CK(hipEventRecord(ev0));
  for (int i = 0; i < iters; ++i) k<<<grid, 256, 5 * kPart>>>(A, B, C, nullptr, nullptr, M, N, K, N, nullptr, nullptr, 1, 0);
  CK(hipEventRecord(ev1));
  CK(hipEventSynchronize(ev1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, ev0, ev1));
  return ms / iters;
}

int main() {
  const int shapes[][3] = {{16384, 4096, 4096}, {16384, 4096, 14336}, {16384, 28672, 4096}};
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  for (auto& sh : shapes) {
    const int M = sh[0], N = sh[1], K = sh[2];
    bf16 *A, *B, *C;
    CK(hipMalloc(&A, (size_t)M * K * 2));
    CK(hipMalloc(&B, (size_t)N * K * 2));
    CK(hipMalloc(&C, (size_t)M * N * 2));
    fill_kernel<<<1024, 256>>>(A, (size_t)M * K, 1);
    fill_kernel<<<1024, 256>>>(B, (size_t)N * K, 2);
    CK(hipDeviceSynchronize());
    const int tiles = (M / 256) * (N / 256);
    const int grid = tiles <= ncu ? tiles : (ncu & ~7);
    const double fl = 2.0 * M * N * K;
    float t[8] = {0};  // slots: VAR 0 1 2 3 4 8 10 7
    float tw4d[4] = {0}, tw4r = 0;
    for (int r = 0; r < 3; ++r) {  // interleaved rounds, best of 3
      float v[8] = {run<0>(A, B, C, M, N, K, grid, 10), run<1>(A, B, C, M, N, K, grid, 10),
                    run<2>(A, B, C, M, N, K, grid, 10), run<3>(A, B, C, M, N, K, grid, 10),
                    run<4>(A, B, C, M, N, K, grid, 10), run<8>(A, B, C, M, N, K, grid, 10), run<10>(A, B, C, M, N, K, grid, 10), run<7>(A, B, C, M, N, K, grid, 10)};
      for (int i = 0; i < 8; ++i)
        if (v[i] > 0 && (t[i] == 0 || v[i] < t[i])) t[i] = v[i];
      const float w[4] = {run_w4d<0>(A, B, C, M, N, K, grid, 10), run_w4d<1>(A, B, C, M, N, K, grid, 10),
                          run_w4d<2>(A, B, C, M, N, K, grid, 10), run_w4d<3>(A, B, C, M, N, K, grid, 10)};
      for (int i = 0; i < 4; ++i)
        if (tw4d[i] == 0 || w[i] < tw4d[i]) tw4d[i] = w[i];
      const float wr = run_w4r(A, B, C, M, N, K, grid, 10);
      if (tw4r == 0 || wr < tw4r) tw4r = wr;
    }
    printf("{\"M\": %d, \"N\": %d, \"K\": %d", M, N, K);
    const int vars[] = {0, 1, 2, 3, 4, 8, 10, 7};
    for (int i = 0; i < 8; ++i) printf(", \"var%d_tflops\": %.1f", vars[i], fl / t[i] / 1e9);
    for (int i = 0; i < 4; ++i) printf(", \"w4d_v%d_tflops\": %.1f", i, fl / tw4d[i] / 1e9);
    printf(", \"w4r_tflops\": %.1f", fl / tw4r / 1e9);
    printf("}\n");
    fflush(stdout);
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
  }
  return 0;
}
