// Streaming-SDR signal processing for the FM-radio ingest pipeline (the reference runs these as CuPy /
// cupyx.scipy.signal calls inside Holoscan operators, /root/reference/community/fm-asr-streaming-rag/sdr-holoscan/
// operators.py:42-53, 206-327). Three launches per burst of complex64 baseband samples:
//  * fir_complex_kernel: causal FIR y[n] = sum_j h[j] x[n - j] with zero initial state (lfilter with a = [1]) - a
//    workgroup stages its output block's input window and the taps in LDS once, each thread then produces 4 outputs;
//  * fm_demod_kernel: the discrete-time FM discriminator angle(x[n + 1] conj(x[n])), which equals
//    diff(unwrap(angle(x))) sample for sample (the unwrap only removes the 2 pi jumps the principal angle of the
//    product never has);
//  * upfirdn_kernel: polyphase rational resampling of a real signal (zero-stuff by `up`, FIR, keep every `down`-th
//    sample) evaluated only at the kept outputs: output i sums the taps k = (i down) mod up, + up, ... against
//    x[(i down - k) / up]; the host pads and offsets the filter exactly as scipy.signal.resample_poly does.
// Bursts are ~62.5K samples (500 KB of complex64) every 62.5 ms at 1 MS/s: latency, not bandwidth, is what matters,
// so the kernels favour one pass and few launches over tiling tricks.
#include "gai_common.h"
#include "gai_kernels.h"

namespace {

constexpr int kFirThreads = 256;

// kFirPer outputs per thread: 4 for long blocks (taps amortised over more outputs), 1 for a burst (62.5K samples ->
// ~245 workgroups instead of ~62, so the whole chip takes part)
template <int kFirPer>
__global__ __launch_bounds__(kFirThreads) void fir_complex_kernel(const float2* __restrict__ x,
                                                                  const float* __restrict__ h, int n, int ntaps,
                                                                  float2* __restrict__ y) {
  constexpr int kFirBlock = kFirThreads * kFirPer;  // outputs per workgroup
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* hs = reinterpret_cast<float*>(smem);                                  // [ntaps]
  float2* xs = reinterpret_cast<float2*>(smem + ((ntaps * 4 + 15) & ~15));     // [ntaps - 1 + kFirBlock]
  const int n0 = blockIdx.x * kFirBlock;
  const int win = ntaps - 1 + kFirBlock;
  for (int i = threadIdx.x; i < ntaps; i += kFirThreads) hs[i] = h[i];
  for (int i = threadIdx.x; i < win; i += kFirThreads) {
    const int src = n0 - (ntaps - 1) + i;
    xs[i] = (src >= 0 && src < n) ? x[src] : float2{0.f, 0.f};
  }
  __syncthreads();
  float2 acc[kFirPer];
#pragma unroll
  for (int r = 0; r < kFirPer; ++r) acc[r] = float2{0.f, 0.f};
  // output n0 + t + 256 r reads xs[t + 256 r + ntaps - 1 - j]
  for (int j = 0; j < ntaps; ++j) {
    const float hj = hs[j];
#pragma unroll
    for (int r = 0; r < kFirPer; ++r) {
      const float2 v = xs[threadIdx.x + kFirThreads * r + ntaps - 1 - j];
      acc[r].x = fmaf(hj, v.x, acc[r].x);
      acc[r].y = fmaf(hj, v.y, acc[r].y);
    }
  }
#pragma unroll
  for (int r = 0; r < kFirPer; ++r) {
    const int o = n0 + threadIdx.x + kFirThreads * r;
    if (o < n) y[o] = acc[r];
  }
}

__global__ __launch_bounds__(256) void fm_demod_kernel(const float2* __restrict__ x, int n, float* __restrict__ y) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n - 1) return;
  const float2 a = x[i], b = x[i + 1];
  // b * conj(a)
  const float re = b.x * a.x + b.y * a.y, im = b.y * a.x - b.x * a.y;
  y[i] = atan2f(im, re);
}

// One wavefront per output: lane l takes taps k + l up, k + (l + 64) up, ... (samples j - l, j - l - 64, ...), so the
// ~1,250 taps of the 1 MS/s -> 16 kHz filter are 20 FMAs per lane and x is read as contiguous 64-sample runs; a
// burst's ~1,000 outputs are ~250 workgroups (one thread per output left ~4 workgroups busy for the whole filter).
constexpr int kRsWaves = 4;

__global__ __launch_bounds__(64 * kRsWaves) void upfirdn_kernel(const float* __restrict__ x, int n,
                                                                 const float* __restrict__ h, int ntaps, int up,
                                                                 int down, int offset, int nout, float gain,
                                                                 float* __restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* hs = reinterpret_cast<float*>(smem);
  for (int i = threadIdx.x; i < ntaps; i += 64 * kRsWaves) hs[i] = h[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * kRsWaves + (threadIdx.x >> 6);  // wave-uniform
  if (m >= nout) return;
  const long long t = (long long)(m + offset) * down;  // position in the zero-stuffed signal
  int k = (int)(t % up);                              // first tap that meets a real sample
  long long j = (t - k) / up;                         // that sample
  // taps k, k + up, ... meet samples j, j - 1, ...; skip the ones past the end of x, stop at x[0]
  if (j >= n) {
    const long long skip = j - (n - 1);
    k += (int)(skip * up);
    j = n - 1;
  }
  float acc = 0.f;
  long long jj = j - lane;
  for (long long kk = k + (long long)lane * up; kk < ntaps && jj >= 0; kk += 64LL * up, jj -= 64)
    acc = fmaf(hs[kk], x[jj], acc);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) y[m] = gain * acc;
}

}  // namespace

template <int PER>
static void fir_launch(const void* x, const float* taps, int n, int ntaps, void* y, hipStream_t st) {
  constexpr int block = kFirThreads * PER;
  const size_t lds = (size_t)((ntaps * 4 + 15) & ~15) + (size_t)(ntaps - 1 + block) * sizeof(float2);
  static bool once = false;  // one static per instantiation: each kernel gets its LDS limit raised once
  if (!once) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(fir_complex_kernel<PER>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  fir_complex_kernel<PER><<<(n + block - 1) / block, kFirThreads, lds, st>>>((const float2*)x, taps, n, ntaps,
                                                                            (float2*)y);
  GAI_LAUNCH_CHECK();
}

void gai_dsp_fir_complex(const void* x, const float* taps, int n, int ntaps, void* y, hipStream_t st) {
  if (n <= 0) return;
  if (ntaps < 1 || ntaps > 4096) gai_launch_error(__FILE__, __LINE__, "dsp_fir: 1 <= taps <= 4096");
  if (n < 1024 * 1024)
    fir_launch<1>(x, taps, n, ntaps, y, st);
  else
    fir_launch<4>(x, taps, n, ntaps, y, st);
}

void gai_dsp_fm_demod(const void* x, int n, float* y, hipStream_t st) {
  if (n < 2) return;
  fm_demod_kernel<<<(n - 1 + 255) / 256, 256, 0, st>>>((const float2*)x, n, y);
  GAI_LAUNCH_CHECK();
}

void gai_dsp_upfirdn(const float* x, int n, const float* taps, int ntaps, int up, int down, int offset, int nout,
                     float gain, float* y, hipStream_t st) {
  if (nout <= 0) return;
  if (up < 1 || down < 1 || ntaps < 1 || ntaps > 32768 || offset < 0)
    gai_launch_error(__FILE__, __LINE__, "dsp_upfirdn: up, down >= 1, 1 <= taps <= 32768, offset >= 0");
  const size_t lds = (size_t)ntaps * sizeof(float);
  static bool once = false;
  if (!once) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(upfirdn_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    once = true;
  }
  upfirdn_kernel<<<(nout + kRsWaves - 1) / kRsWaves, 64 * kRsWaves, lds, st>>>(x, n, taps, ntaps, up, down, offset,
                                                                              nout, gain, y);
  GAI_LAUNCH_CHECK();
}
