// bf16 GEMM entry points: epilogue dispatch, the stream-K workspace pool and the prefill QKV GEMM with
// RoPE + paged-KV write in its epilogue. The kernels and launchers are in gemm_impl.h; the per-epilogue
// instantiations in gemm_epi_*.hip.
#include "gemm_impl.h"

#ifndef GAI_GEMM_KERNELS_ONLY
bool gai_sk_workspace(hipStream_t st, size_t ws_bytes, size_t cnt_n, float** ws_out, int** cnt_out) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, SkWorkspace> pool;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  std::lock_guard<std::mutex> lk(mu);
  SkWorkspace& w = pool[{dev, st}];
  if (w.ws_bytes < ws_bytes || w.cnt_n < cnt_n) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
    if (hipStreamSynchronize(st) != hipSuccess) return false;  // earlier launches may still use the old one
    if (w.ws) (void)hipFree(w.ws);
    if (w.cnt) (void)hipFree(w.cnt);
    w = SkWorkspace{};
    const size_t nb = std::max(ws_bytes, w.ws_bytes), nc = std::max<size_t>(cnt_n, 4096);
    if (hipMalloc(&w.ws, nb) != hipSuccess) return false;
    if (hipMalloc(&w.cnt, nc * sizeof(int)) != hipSuccess || hipMemset(w.cnt, 0, nc * sizeof(int)) != hipSuccess) {
      (void)hipFree(w.ws);
      w = SkWorkspace{};
      return false;
    }
    w.ws_bytes = nb;
    w.cnt_n = nc;
  }
  *ws_out = w.ws;
  *cnt_out = w.cnt;
  return true;
}

void gai_gemm(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
              int epi, int out_f32, int force, hipStream_t st, int bfrag) {
  if (M == 0 || N == 0) return;
  static_assert(EPI_NONE == 0 && EPI_BIAS == 1 && EPI_BIAS_GELU == 2 && EPI_RESIDUAL == 3 && EPI_SWIGLU == 4 &&
                    EPI_BIAS_RESIDUAL == 5 && EPI_BIAS_RELU == 6 && EPI_BIAS_QUICKGELU == 7,
                "gai_gemm_run<E> numbering");
  switch (epi) {
    case 0: return gai_gemm_run0(A, B, C, bias, R, M, N, K, ldc, out_f32, force, st, bfrag);
    case 1: return gai_gemm_run1(A, B, C, bias, R, M, N, K, ldc, out_f32, force, st, bfrag);
    case 2: return gai_gemm_run2(A, B, C, bias, R, M, N, K, ldc, out_f32, force, st, bfrag);
    case 3: return gai_gemm_run3(A, B, C, bias, R, M, N, K, ldc, out_f32, force, st, bfrag);
    case 4: return gai_gemm_run4(A, B, C, bias, R, M, N, K, ldc, out_f32, force, st, bfrag);
    case 5: return gai_gemm_run5(A, B, C, bias, R, M, N, K, ldc, out_f32, force, st, bfrag);
    case 6: return gai_gemm_run6(A, B, C, bias, R, M, N, K, ldc, out_f32, force, st, bfrag);
    case 7: return gai_gemm_run7(A, B, C, bias, R, M, N, K, ldc, out_f32, force, st, bfrag);
    default:
      gai_launch_error(__FILE__, __LINE__, "gemm: unknown epilogue");
  }
}

int gai_gemm_prefill_rope_kv(const void* A, const void* B, const void* bias, const int* pos, const float* cos_sin,
                             const int* slots, void* q_out, void* k_cache, void* v_cache, int M, int K, int Hq,
                             int Hkv, int D, int kv_fp8, hipStream_t st, int bfrag) {
  const int N = (Hq + 2 * Hkv) * D;
  if (D != 128 || kv_fp8 || M < 1024 || K % 64 || K < 192 || (size_t)M * K * 2 >= (1ull << 31) ||
      (size_t)N * K * 2 >= (1ull << 31))
    return 0;
  // the fused epilogue rides on the 256x256 tile walk; when its tiles fill less than half the grid (QKV of a TP = 8
  // Llama-3-70B shard: N 1280, 50 tiles at M = 2407 -> 169 us, 0.3 PF/s) the caller's plain GEMM (stream-K for deep K)
  // plus the rope_kv kernel is faster
  if (2 * ring_tiles(M, N) < sk_grid()) return 0;
  RopeKvArgs rk;
  rk.pos = pos;
  rk.cos_sin = cos_sin;
  rk.slots = slots;
  rk.q_out = (bf16*)q_out;
  rk.k_cache = (bf16*)k_cache;
  rk.v_cache = (bf16*)v_cache;
  rk.Hq = Hq;
  rk.Hkv = Hkv;
  launch_w4d<EPI_ROPE_KV, false>(A, B, nullptr, bias, nullptr, M, N, K, N, st, rk, 0, bfrag);
  return 1;
}
#endif  // GAI_GEMM_KERNELS_ONLY
