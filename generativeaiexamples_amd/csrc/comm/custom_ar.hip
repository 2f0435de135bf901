// One-shot peer-memory all-reduce over xGMI (SURVEY §2.4 D1 / P1, §5.8 "small messages").
//
// Decode-time TP all-reduces are latency bound (Llama-3-70B TP8, batch 64: 1 MiB, 160 per token).
// A ring all-reduce crosses N-1 hops in sequence; on a fully connected xGMI mesh every rank can
// instead push its whole input to all N-1 peers at once (one link each, concurrently) and reduce
// locally: one hop of latency.
//
// Memory (per rank, allocated uncached so no L2 of any GPU holds a stale copy, IPC-exported):
//   data  [2 parity][W src][slot_bytes]   peers write their contribution into slot `src`
//   sig   [kArMaxBlocks][8] uint32         peer `src` stores the epoch of block b into sig[b][src]
// plus a local, never shared, uint32 counter per block that carries the epoch between launches, so
// the launch has no per-call scalar argument and replays correctly from a captured HIP graph.
//
// Block b owns the fixed byte range [b * kArChunk, (b + 1) * kArChunk) of every call. Per call:
//   1. e = ++counter[b]; parity p = e & 1
//   2. push own chunk to data_q[p][rank] of every peer q (16-B stores, remote for q != rank)
//   3. s_waitcnt vmcnt(0) in every wave, barrier, then lane q stores sig_q[b][rank] = e (system scope)
//   4. lanes 0..W-1 poll the local sig[b][q] until it equals e (bounded: a timeout sets *err and the
//      block proceeds, so a broken peer can never hang the GPU), barrier
//   5. out chunk = sum_q data_local[p][q] (fp32 accumulate in peer order 0..W-1: every rank computes
//      bit-identical results)
// Reuse of parity p at call e+2 is safe without a closing barrier: a peer's block b can only reach
// e+2 after seeing our signal for e+1, which we send after finishing our reads of call e (same
// stream, kernels serialised). Flags hold e-1, e or e+1 while we wait for e (a peer can finish call e and
// signal the next call, but cannot reach e+2 without our e+1 signal), so the wait accepts any epoch >= e.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "gai_common.h"
#include "gai_kernels.h"

namespace {

constexpr int kArThreads = 256;

typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void acc_bf16x8(float (&a)[8], const uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[2 * i] += __uint_as_float(w[i] << 16);
    a[2 * i + 1] += __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  // round-to-nearest-even, NaN kept quiet
  auto rn = [](float f) -> uint32_t {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
  };
  return rn(lo) | (rn(hi) << 16);
}

struct ArPtrs {
  char* data[GAI_AR_MAX_WORLD];
  uint32_t* sig[GAI_AR_MAX_WORLD];
  uint32_t spin_limit;  // bounded peer wait (s_sleep polls) before the error flag is raised
};

// 2^26 polls (~2 s) by default; GAI_AR_SPIN_LOG2 raises it where ranks legitimately lag by seconds (every
// rank of a TP rehearsal time-slicing ONE GPU and a few CPU cores)
static uint32_t ar_spin_limit() {
  static const uint32_t v = [] {
    const char* e = getenv("GAI_AR_SPIN_LOG2");
    const int l = e ? atoi(e) : 26;
    return 1u << (l < 20 ? 20 : l > 31 ? 31 : l);
  }();
  return v;
}

// Poll a peer's signal until it reaches epoch e. "Reaches" is `flag - e >= 0` (wrap-safe), not equality: a peer
// that saw OUR epoch-e signal may finish call e and the next collective on the same counters, storing e + 1 here
// before this wave reads e (a rank descheduled mid-poll, e.g. ranks time-slicing one GPU). e + 1 implies the peer's
// epoch-e data landed first (it signals in order), and it cannot reach e + 2 without our e + 1 signal.
__device__ __forceinline__ void wait_epoch(uint32_t* f, uint32_t e, uint32_t limit, int* err) {
  uint32_t spins = 0;
  while ((int32_t)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > limit) {
      atomicOr(err, 1);
      break;
    }
  }
}

// Workgroups of one all-to-all launch (they loop over the chunks). Every workgroup spin-waits for its peers', so all
// ranks' workgroups must be resident at once: one GPU per rank holds 512 easily, but W ranks sharing ONE GPU (the
// one-GPU rehearsals: 8 workgroups of 256 threads per CU = 2048 on 256 CUs) need GAI_AR_MAX_GRID <= 2048 / W.
static int ar_max_grid() {
  static const int v = [] {
    const char* e = getenv("GAI_AR_MAX_GRID");
    const int g = e ? atoi(e) : GAI_AR_MAX_BLOCKS;
    return g < 1 ? 1 : g > GAI_AR_MAX_BLOCKS ? GAI_AR_MAX_BLOCKS : g;
  }();
  return v;
}

template <int W, bool F32>
__global__ __launch_bounds__(kArThreads) void ar_oneshot_kernel(const uint4* in, uint4* out,
                                                                ArPtrs p, uint32_t* __restrict__ counters, int rank,
                                                                int64_t n16, int64_t slot_bytes, int* err) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ uint32_t e_sh;
  if (tid == 0) e_sh = counters[b] + 1u;
  __syncthreads();
  const uint32_t e = e_sh;
  const int par = (int)(e & 1u);
  constexpr int64_t kVec = GAI_AR_CHUNK / 16;
  const int64_t v0 = (int64_t)b * kVec, v1 = min(v0 + kVec, n16);
  const int64_t my_off = ((int64_t)par * W + rank) * slot_bytes;

  // 2. push
  for (int64_t v = v0 + tid; v < v1; v += kArThreads) {
    const uint4 x = in[v];
#pragma unroll
    for (int q = 0; q < W; ++q) reinterpret_cast<uint4*>(p.data[q] + my_off)[v] = x;
  }
  // 3. drain this wave's stores, join the workgroup, signal every peer
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (tid < W) __hip_atomic_store(p.sig[tid] + b * GAI_AR_MAX_WORLD + rank, e, __ATOMIC_RELEASE,
                                  __HIP_MEMORY_SCOPE_SYSTEM);
  // 4. wait for every peer's chunk
  if (tid < W) {
    uint32_t* f = p.sig[rank] + b * GAI_AR_MAX_WORLD + tid;
    wait_epoch(f, e, p.spin_limit, err);  // ~seconds bound: a peer died or diverged; never hang the GPU
  }
  __syncthreads();
  // 5. reduce the W local slots in rank order
  const char* base = p.data[rank] + (int64_t)par * W * slot_bytes;
  for (int64_t v = v0 + tid; v < v1; v += kArThreads) {
    if (F32) {
      f32x4_t s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const uint4 x = reinterpret_cast<const uint4*>(base + q * slot_bytes)[v];
        s += f32x4_t{__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), __uint_as_float(x.w)};
      }
      out[v] = uint4{__float_as_uint(s[0]), __float_as_uint(s[1]), __float_as_uint(s[2]), __float_as_uint(s[3])};
    } else {
      float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < W; ++q) acc_bf16x8(a, reinterpret_cast<const uint4*>(base + q * slot_bytes)[v]);
      out[v] = uint4{pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]), pack_bf16x2(a[4], a[5]),
                     pack_bf16x2(a[6], a[7])};
    }
  }
  if (tid == 0) counters[b] = e;
}

// Fused all-reduce + residual add + RMSNorm (the TP block boundary: row-parallel projection ->
// all-reduce -> h + residual -> rmsnorm). Steps 1-4 are the one-shot kernel's (same buffers, same
// block -> byte mapping, so the parity argument above holds across both kernels); step 5 reduces whole
// rows (the caller guarantees GAI_AR_CHUNK % row_bytes == 0, so a chunk holds complete rows) and
// applies, with the rounding of the unfused path: h = bf16(sum), r = bf16(h + residual) -> residual,
// y = bf16(r * rsqrt(mean(r^2) + eps) * w). VPT = 16-byte vectors per thread per row (D = 2048 * VPT).
template <int W, int VPT>
__global__ __launch_bounds__(kArThreads) void ar_rmsnorm_kernel(const uint4* in, uint4* out, uint4* residual,
                                                                const uint4* __restrict__ wgt, ArPtrs p,
                                                                uint32_t* __restrict__ counters, int rank,
                                                                int64_t n16, int64_t slot_bytes, float eps, int* err) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ uint32_t e_sh;
  __shared__ float red[kArThreads / 64];
  if (tid == 0) e_sh = counters[b] + 1u;
  __syncthreads();
  const uint32_t e = e_sh;
  const int par = (int)(e & 1u);
  constexpr int64_t kVec = GAI_AR_CHUNK / 16;
  constexpr int kRowVec = VPT * kArThreads;  // 16-B vectors per row
  const int64_t v0 = (int64_t)b * kVec, v1 = min(v0 + kVec, n16);
  const int64_t my_off = ((int64_t)par * W + rank) * slot_bytes;
  for (int64_t v = v0 + tid; v < v1; v += kArThreads) {
    const uint4 x = in[v];
#pragma unroll
    for (int q = 0; q < W; ++q) reinterpret_cast<uint4*>(p.data[q] + my_off)[v] = x;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (tid < W) __hip_atomic_store(p.sig[tid] + b * GAI_AR_MAX_WORLD + rank, e, __ATOMIC_RELEASE,
                                  __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < W) {
    uint32_t* f = p.sig[rank] + b * GAI_AR_MAX_WORLD + tid;
    wait_epoch(f, e, p.spin_limit, err);
  }
  __syncthreads();
  const char* base = p.data[rank] + (int64_t)par * W * slot_bytes;
  const float inv_d = 1.f / (float)(kRowVec * 8);
  for (int64_t r0 = v0; r0 < v1; r0 += kRowVec) {
    float rv[VPT][8];
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int64_t v = r0 + j * kArThreads + tid;
      float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < W; ++q) acc_bf16x8(a, reinterpret_cast<const uint4*>(base + q * slot_bytes)[v]);
      const uint4 h = uint4{pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]), pack_bf16x2(a[4], a[5]),
                            pack_bf16x2(a[6], a[7])};
      float hr[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      acc_bf16x8(hr, h);
      acc_bf16x8(hr, residual[v]);
      const uint4 r = uint4{pack_bf16x2(hr[0], hr[1]), pack_bf16x2(hr[2], hr[3]), pack_bf16x2(hr[4], hr[5]),
                            pack_bf16x2(hr[6], hr[7])};
      residual[v] = r;
#pragma unroll
      for (int i = 0; i < 8; ++i) rv[j][i] = 0.f;
      acc_bf16x8(rv[j], r);
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += rv[j][i] * rv[j][i];
    }
    ss = gai::wave_sum(ss);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < kArThreads / 64; ++i) tot += red[i];
    __syncthreads();
    const float rs = rsqrtf(tot * inv_d + eps);
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int64_t v = r0 + j * kArThreads + tid;
      float wv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      acc_bf16x8(wv, wgt[(v - r0)]);
      out[v] = uint4{pack_bf16x2(rv[j][0] * rs * wv[0], rv[j][1] * rs * wv[1]),
                     pack_bf16x2(rv[j][2] * rs * wv[2], rv[j][3] * rs * wv[3]),
                     pack_bf16x2(rv[j][4] * rs * wv[4], rv[j][5] * rs * wv[5]),
                     pack_bf16x2(rv[j][6] * rs * wv[6], rv[j][7] * rs * wv[7])};
    }
  }
  if (tid == 0) counters[b] = e;
}

// Two-shot all-reduce for bandwidth-bound messages: reduce-scatter then all-gather, each over direct
// peer writes. The one-shot kernel moves the whole message over every link; here each link carries
// 2/W of it (rank r reduces segment r), at the price of a second signal round. Own buffers (region 0:
// reduce-scatter inputs, region 1: gathered segments, both [2 parity][W src][region]) and own per-block
// epochs / signals [block][phase][src]; block b owns bytes [b * CHUNK, (b + 1) * CHUNK) of every
// segment in both regions, so the one-shot parity argument applies per region.
template <int W, bool F32>
__global__ __launch_bounds__(kArThreads) void ar_twoshot_kernel(const uint4* in, uint4* out, ArPtrs p,
                                                                uint32_t* __restrict__ counters, int rank,
                                                                int64_t seg16, int64_t region_bytes, int* err) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ uint32_t e_sh;
  if (tid == 0) e_sh = counters[b] + 1u;
  __syncthreads();
  const uint32_t e = e_sh;
  const int par = (int)(e & 1u);
  constexpr int64_t kVec = GAI_AR_CHUNK / 16;
  const int64_t v0 = (int64_t)b * kVec, v1 = min(v0 + kVec, seg16);
  const int64_t slot = 2 * region_bytes;
  const int64_t pbase = (int64_t)par * W * slot;
  auto wait_phase = [&](int ph) {
    if (tid < W) {
      uint32_t* f = p.sig[rank] + (b * 2 + ph) * GAI_AR_MAX_WORLD + tid;
      wait_epoch(f, e, p.spin_limit, err);
    }
    __syncthreads();
  };
  auto signal_phase = [&](int ph) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    if (tid < W)
      __hip_atomic_store(p.sig[tid] + (b * 2 + ph) * GAI_AR_MAX_WORLD + rank, e, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  };
  // 1. reduce-scatter: segment q of my input goes to peer q (region 0, slot `rank`)
#pragma unroll
  for (int q = 0; q < W; ++q) {
    uint4* dst = reinterpret_cast<uint4*>(p.data[q] + pbase + rank * slot);
    for (int64_t v = v0 + tid; v < v1; v += kArThreads) dst[v] = in[q * seg16 + v];
  }
  signal_phase(0);
  wait_phase(0);
  // 2. reduce my segment, keep it, push it to every peer (region 1, slot `rank`)
  const char* lb = p.data[rank] + pbase;
  for (int64_t v = v0 + tid; v < v1; v += kArThreads) {
    uint4 res;
    if (F32) {
      f32x4_t s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const uint4 x = reinterpret_cast<const uint4*>(lb + q * slot)[v];
        s += f32x4_t{__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z), __uint_as_float(x.w)};
      }
      res = uint4{__float_as_uint(s[0]), __float_as_uint(s[1]), __float_as_uint(s[2]), __float_as_uint(s[3])};
    } else {
      float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < W; ++q) acc_bf16x8(a, reinterpret_cast<const uint4*>(lb + q * slot)[v]);
      res = uint4{pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]), pack_bf16x2(a[4], a[5]), pack_bf16x2(a[6], a[7])};
    }
    out[rank * seg16 + v] = res;
#pragma unroll
    for (int q = 0; q < W; ++q)
      if (q != rank) reinterpret_cast<uint4*>(p.data[q] + pbase + rank * slot + region_bytes)[v] = res;
  }
  signal_phase(1);
  wait_phase(1);
  // 3. all-gather: the other ranks' reduced segments
#pragma unroll
  for (int q = 0; q < W; ++q) {
    if (q == rank) continue;
    const uint4* src = reinterpret_cast<const uint4*>(lb + q * slot + region_bytes);
    for (int64_t v = v0 + tid; v < v1; v += kArThreads) out[q * seg16 + v] = src[v];
  }
  if (tid == 0) counters[b] = e;
}


// One-shot all-to-all on the same buffers (expert-parallel token exchange, parallel/ep.py): the input is W
// equal segments, segment q bound for rank q. Block b owns chunks b, b + G, ... of every segment: it pushes them
// into slot `rank` of peer q's data area (direct xGMI writes, all peers at once), signals every peer with the
// block's epoch, waits for all of them, then copies the same chunks of every local slot q into output segment q.
// Epochs, parities and the bounded wait are the one-shot all-reduce's (shared counters and signals: every rank
// issues the same sequence of collectives), so it replays from a HIP graph too.
// Variable segments (send_rows / recv_rows, device int32 [W], optional): only the first send_rows[q] rows
// (row16 16-B vectors each) of segment q are pushed and only the first recv_rows[q] rows of slot q are copied out
// - a capacity-sized slab of which only the valid rows cross xGMI, with the counts known on the device only (the
// expert-parallel prefill exchange needs no host round trip). Rows past a count are left untouched in `out`.
template <int W>
__global__ __launch_bounds__(kArThreads) void a2a_oneshot_kernel(const uint4* in, uint4* out, ArPtrs p,
                                                                 uint32_t* __restrict__ counters, int rank,
                                                                 int64_t seg16, int64_t slot_bytes, int* err,
                                                                 const int* __restrict__ send_rows,
                                                                 const int* __restrict__ recv_rows, int64_t row16,
                                                                 int nchunks) {
  const int b = blockIdx.x, tid = threadIdx.x, G = gridDim.x;
  __shared__ uint32_t e_sh;
  if (tid == 0) e_sh = counters[b] + 1u;
  __syncthreads();
  const uint32_t e = e_sh;
  const int par = (int)(e & 1u);
  constexpr int64_t kVec = GAI_AR_CHUNK / 16;
  const int64_t my_off = ((int64_t)par * W + rank) * slot_bytes;
#pragma unroll
  for (int q = 0; q < W; ++q) {
    uint4* dst = reinterpret_cast<uint4*>(p.data[q] + my_off);
    const uint4* src = in + (int64_t)q * seg16;
    const int64_t lim = send_rows ? min(seg16, (int64_t)send_rows[q] * row16) : seg16;
    for (int c = b; c < nchunks; c += G) {
      const int64_t v1 = min((int64_t)(c + 1) * kVec, lim);
      for (int64_t v = (int64_t)c * kVec + tid; v < v1; v += kArThreads) dst[v] = src[v];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (tid < W) __hip_atomic_store(p.sig[tid] + b * GAI_AR_MAX_WORLD + rank, e, __ATOMIC_RELEASE,
                                  __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < W) {
    uint32_t* f = p.sig[rank] + b * GAI_AR_MAX_WORLD + tid;
    wait_epoch(f, e, p.spin_limit, err);
  }
  __syncthreads();
  const char* base = p.data[rank] + (int64_t)par * W * slot_bytes;
#pragma unroll
  for (int q = 0; q < W; ++q) {
    const uint4* src = reinterpret_cast<const uint4*>(base + q * slot_bytes);
    uint4* dst = out + (int64_t)q * seg16;
    const int64_t lim = recv_rows ? min(seg16, (int64_t)recv_rows[q] * row16) : seg16;
    for (int c = b; c < nchunks; c += G) {
      const int64_t v1 = min((int64_t)(c + 1) * kVec, lim);
      for (int64_t v = (int64_t)c * kVec + tid; v < v1; v += kArThreads) dst[v] = src[v];
    }
  }
  if (tid == 0) counters[b] = e;
}

}  // namespace

void gai_custom_all_to_all(const void* in, void* out, int64_t seg_bytes, void* const* peer_data,
                           uint32_t* const* peer_sig, uint32_t* counters, int rank, int world, int64_t slot_bytes,
                           int* err, hipStream_t st, const int* send_rows, const int* recv_rows, int64_t row_bytes) {
  if (seg_bytes == 0) return;
  if (seg_bytes % 16 || seg_bytes > slot_bytes) gai_launch_error(__FILE__, __LINE__, "custom_all_to_all: segment size");
  if ((send_rows || recv_rows) && (row_bytes <= 0 || row_bytes % 16))
    gai_launch_error(__FILE__, __LINE__, "custom_all_to_all: row_bytes must be a positive multiple of 16");
  const int64_t nchunks = (seg_bytes + GAI_AR_CHUNK - 1) / GAI_AR_CHUNK;
  if (nchunks > (int64_t)1 << 30) gai_launch_error(__FILE__, __LINE__, "custom_all_to_all: segment too large");
  const int nblk = (int)std::min<int64_t>(nchunks, ar_max_grid());  // blocks loop over the chunks
  ArPtrs p{};
  p.spin_limit = ar_spin_limit();
  for (int q = 0; q < world; ++q) {
    p.data[q] = static_cast<char*>(peer_data[q]);
    p.sig[q] = peer_sig[q];
  }
#define GAI_A2A(WW)                                                                                             \
  if (world == WW) {                                                                                            \
    a2a_oneshot_kernel<WW><<<nblk, kArThreads, 0, st>>>((const uint4*)in, (uint4*)out, p, counters, rank,       \
                                                        seg_bytes / 16, slot_bytes, err, send_rows, recv_rows,  \
                                                        row_bytes / 16, (int)nchunks);                         \
    GAI_LAUNCH_CHECK();                                                                                         \
    return;                                                                                                     \
  }
  GAI_A2A(2)
  GAI_A2A(4)
  GAI_A2A(8)
  GAI_A2A(3)
  GAI_A2A(5)
  GAI_A2A(6)
  GAI_A2A(7)
#undef GAI_A2A
  gai_launch_error(__FILE__, __LINE__, "custom_all_to_all: world size must be 2..8");
}

void gai_custom_allreduce(const void* in, void* out, int64_t bytes, int f32, void* const* peer_data,
                          uint32_t* const* peer_sig, uint32_t* counters, int rank, int world, int64_t slot_bytes,
                          int* err, hipStream_t st) {
  if (bytes == 0) return;
  if (bytes % 16 || bytes > slot_bytes) gai_launch_error(__FILE__, __LINE__, "custom_allreduce: bad message size");
  const int64_t nblk = (bytes + GAI_AR_CHUNK - 1) / GAI_AR_CHUNK;
  if (nblk > GAI_AR_MAX_BLOCKS) gai_launch_error(__FILE__, __LINE__, "custom_allreduce: message too large");
  ArPtrs p{};
  p.spin_limit = ar_spin_limit();
  for (int q = 0; q < world; ++q) {
    p.data[q] = static_cast<char*>(peer_data[q]);
    p.sig[q] = peer_sig[q];
  }
  const int64_t n16 = bytes / 16;
#define GAI_AR(WW)                                                                                            \
  if (world == WW) {                                                                                          \
    if (f32)                                                                                                  \
      ar_oneshot_kernel<WW, true><<<(int)nblk, kArThreads, 0, st>>>((const uint4*)in, (uint4*)out, p, counters, \
                                                                    rank, n16, slot_bytes, err);              \
    else                                                                                                      \
      ar_oneshot_kernel<WW, false><<<(int)nblk, kArThreads, 0, st>>>((const uint4*)in, (uint4*)out, p,          \
                                                                     counters, rank, n16, slot_bytes, err);   \
    GAI_LAUNCH_CHECK();                                                                                       \
    return;                                                                                                   \
  }
  GAI_AR(2)
  GAI_AR(4)
  GAI_AR(8)
  GAI_AR(3)
  GAI_AR(5)
  GAI_AR(6)
  GAI_AR(7)
#undef GAI_AR
  gai_launch_error(__FILE__, __LINE__, "custom_allreduce: world size must be 2..8");
}

void gai_custom_allreduce_twoshot(const void* in, void* out, int64_t bytes, int f32, void* const* peer_data,
                                  uint32_t* const* peer_sig, uint32_t* counters, int rank, int world,
                                  int64_t region_bytes, int* err, hipStream_t st) {
  if (bytes == 0) return;
  if (bytes % (16 * world)) gai_launch_error(__FILE__, __LINE__, "allreduce two-shot: bytes % (16 * world) != 0");
  const int64_t seg = bytes / world;
  if (seg > region_bytes) gai_launch_error(__FILE__, __LINE__, "allreduce two-shot: message too large");
  const int64_t nblk = (seg + GAI_AR_CHUNK - 1) / GAI_AR_CHUNK;
  if (nblk > GAI_AR_MAX_BLOCKS) gai_launch_error(__FILE__, __LINE__, "allreduce two-shot: too many blocks");
  ArPtrs p{};
  p.spin_limit = ar_spin_limit();
  for (int q = 0; q < world; ++q) {
    p.data[q] = static_cast<char*>(peer_data[q]);
    p.sig[q] = peer_sig[q];
  }
#define GAI_AR2(WW)                                                                                          \
  if (world == WW) {                                                                                         \
    if (f32)                                                                                                 \
      ar_twoshot_kernel<WW, true><<<(int)nblk, kArThreads, 0, st>>>((const uint4*)in, (uint4*)out, p, counters, \
                                                                    rank, seg / 16, region_bytes, err);      \
    else                                                                                                     \
      ar_twoshot_kernel<WW, false><<<(int)nblk, kArThreads, 0, st>>>((const uint4*)in, (uint4*)out, p,         \
                                                                     counters, rank, seg / 16, region_bytes, err); \
    GAI_LAUNCH_CHECK();                                                                                      \
    return;                                                                                                  \
  }
  GAI_AR2(2)
  GAI_AR2(4)
  GAI_AR2(8)
  GAI_AR2(3)
  GAI_AR2(5)
  GAI_AR2(6)
  GAI_AR2(7)
#undef GAI_AR2
  gai_launch_error(__FILE__, __LINE__, "allreduce two-shot: world size must be 2..8");
}

void gai_custom_allreduce_rmsnorm(const void* in, void* out, void* residual, const void* w, int64_t rows, int D,
                                  float eps, void* const* peer_data, uint32_t* const* peer_sig, uint32_t* counters,
                                  int rank, int world, int64_t slot_bytes, int* err, hipStream_t st) {
  if (rows == 0) return;
  const int64_t row_bytes = (int64_t)D * 2, bytes = rows * row_bytes;
  if (D % 2048 || GAI_AR_CHUNK % row_bytes || bytes > slot_bytes)
    gai_launch_error(__FILE__, __LINE__, "allreduce_rmsnorm: D must be 2048 or 4096*k with rows inside a chunk");
  const int64_t nblk = (bytes + GAI_AR_CHUNK - 1) / GAI_AR_CHUNK;
  if (nblk > GAI_AR_MAX_BLOCKS) gai_launch_error(__FILE__, __LINE__, "allreduce_rmsnorm: message too large");
  ArPtrs p{};
  p.spin_limit = ar_spin_limit();
  for (int q = 0; q < world; ++q) {
    p.data[q] = static_cast<char*>(peer_data[q]);
    p.sig[q] = peer_sig[q];
  }
  const int vpt = D / 2048;
#define GAI_ARN(WW, VV)                                                                                       \
  if (world == WW && vpt == VV) {                                                                             \
    ar_rmsnorm_kernel<WW, VV><<<(int)nblk, kArThreads, 0, st>>>((const uint4*)in, (uint4*)out, (uint4*)residual, \
                                                                (const uint4*)w, p, counters, rank, bytes / 16,  \
                                                                slot_bytes, eps, err);                        \
    GAI_LAUNCH_CHECK();                                                                                       \
    return;                                                                                                   \
  }
#define GAI_ARN_W(WW) GAI_ARN(WW, 1) GAI_ARN(WW, 2) GAI_ARN(WW, 4)
  GAI_ARN_W(2)
  GAI_ARN_W(3)
  GAI_ARN_W(4)
  GAI_ARN_W(5)
  GAI_ARN_W(6)
  GAI_ARN_W(7)
  GAI_ARN_W(8)
#undef GAI_ARN_W
#undef GAI_ARN
  gai_launch_error(__FILE__, __LINE__, "allreduce_rmsnorm: unsupported world / hidden size");
}

// --- IPC buffer management (host) ---------------------------------------------------------------
void* gai_ipc_malloc(int64_t bytes) {
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess)
    gai_launch_error(__FILE__, __LINE__, "ipc_malloc: hipExtMallocWithFlags(uncached) failed");
  if (hipMemset(p, 0, bytes) != hipSuccess) gai_launch_error(__FILE__, __LINE__, "ipc_malloc: memset failed");
  if (hipDeviceSynchronize() != hipSuccess) gai_launch_error(__FILE__, __LINE__, "ipc_malloc: sync failed");
  return p;
}

void gai_ipc_free(void* p) { (void)hipFree(p); }

void gai_ipc_get_handle(void* p, char* handle64) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) gai_launch_error(__FILE__, __LINE__, "hipIpcGetMemHandle failed");
  static_assert(sizeof(h) <= 64, "ipc handle size");
  for (size_t i = 0; i < sizeof(h); ++i) handle64[i] = reinterpret_cast<const char*>(&h)[i];
}

void* gai_ipc_open(const char* handle64) {
  hipIpcMemHandle_t h;
  for (size_t i = 0; i < sizeof(h); ++i) reinterpret_cast<char*>(&h)[i] = handle64[i];
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess)
    gai_launch_error(__FILE__, __LINE__, "hipIpcOpenMemHandle failed");
  return p;
}

void gai_ipc_close(void* p) { (void)hipIpcCloseMemHandle(p); }
