// Exact brute-force vector search: fused similarity GEMM + top-k.
//
// scores[q, x] = Q[q] . X[x] + bias[x]  with bias = 0 (inner product / cosine on
// normalised vectors), -0.5*|x|^2 (L2 ranking) or -inf (deleted row), so one
// kernel serves IP / cosine / L2 and tombstones. The [nq, N] score matrix is
// never materialised:
//   stage 1: a 512-thread workgroup keeps a tile of up to 64 queries in LDS
//   (XOR-swizzled rows), each wave streams 16-row groups of X straight to VGPRs
//   (X is read once from HBM per query tile: the index is bandwidth-bound),
//   v_mfma_f32_16x16x32_bf16 produces the 16x(16*MT) score block, the block is
//   transposed through a per-wave LDS scratch so each lane owns one query, and
//   every lane keeps a sorted top-K list in registers (statically indexed
//   insertion; after warm-up almost every candidate is rejected by one compare).
//   The workgroup's lists are merged through LDS into one list per query.
//   stage 2: one workgroup per query merges the per-workgroup lists.
#include <algorithm>

#include "gai_common.h"
#include "gai_kernels.h"

using namespace gai;

namespace {

template <int K>
struct TopK {
  float v[K];
  int i[K];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      v[j] = -INFINITY;
      i[j] = -1;
    }
  }
  __device__ __forceinline__ void insert(float s, int id) {
    if (!(s > v[K - 1])) return;
    v[K - 1] = s;
    i[K - 1] = id;
#pragma unroll
    for (int j = K - 1; j > 0; --j) {
      if (v[j] > v[j - 1]) {
        const float tv = v[j];
        v[j] = v[j - 1];
        v[j - 1] = tv;
        const int ti = i[j];
        i[j] = i[j - 1];
        i[j - 1] = ti;
      }
    }
  }
};

// LDS layout: [Q image: NQ*D*2 bytes][score scratch: 8 waves * NQ * 17 floats]; the merge
// buffer (64 lanes * K * 8 bytes) aliases the Q image after the main loop.
template <int MT, int K>
__global__ __launch_bounds__(512) void sim_topk_stage1(const bf16* __restrict__ Q, const bf16* __restrict__ X,
                                                       const float* __restrict__ bias, int nq, int N, int D,
                                                       int rows_per_wg, float* __restrict__ ws_v,
                                                       int* __restrict__ ws_i) {
  constexpr int NQ = 16 * MT;
  constexpr int LPQ = 64 / NQ;  // lanes per query
  constexpr int XPL = 16 / LPQ;  // x-columns per lane per group
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* qimg = smem;
  float* scratch = reinterpret_cast<float*>(smem + (size_t)NQ * D * 2);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q0 = blockIdx.y * NQ;
  const int ncols = D / 8;  // 16-B units per row

  // stage the query tile (zero rows beyond nq)
  for (int e = tid; e < NQ * ncols; e += 512) {
    const int r = e / ncols, u = e % ncols;
    bf16x8 v = (q0 + r < nq) ? load8(Q + (size_t)(q0 + r) * D + u * 8) : bf16x8{};
    *reinterpret_cast<bf16x8*>(qimg + (size_t)r * D * 2 + ((u ^ (r & 15)) << 4)) = v;
  }
  __syncthreads();

  const int my_q = lane % NQ, my_sub = lane / NQ;
  TopK<K> tk;
  tk.init();
  float* scr = scratch + wid * NQ * 17;
  const int wg_row0 = blockIdx.x * rows_per_wg;
  const int wave_rows = rows_per_wg / 8;
  const int r_begin = wg_row0 + wid * wave_rows;
  const int r_end = min(N, r_begin + wave_rows);

  for (int rb = r_begin; rb < r_end; rb += 16) {
    const int xr = min(rb + (lane & 15), N - 1);
    const bf16* xp = X + (size_t)xr * D + 8 * (lane >> 4);
    f32x4 acc[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int t = 0; t < D / 32; ++t) {
      const bf16x8 xf = load8(xp + 32 * t);
      const int u = 4 * t + (lane >> 4);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int qr = 16 * i + (lane & 15);
        const bf16x8 qf = *reinterpret_cast<const bf16x8*>(qimg + (size_t)qr * D * 2 + ((u ^ (qr & 15)) << 4));
        // D[row = query][col = x row]
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf, xf, acc[i], 0, 0, 0);
      }
    }
    // transpose through LDS: scr[q][x]
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) scr[(16 * i + 4 * (lane >> 4) + r) * 17 + (lane & 15)] = acc[i][r];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int c = 0; c < XPL; ++c) {
      const int xc = my_sub * XPL + c;
      const int row = rb + xc;
      if (row < r_end) tk.insert(scr[my_q * 17 + xc] + bias[row], row);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }

  // merge: owner of query q = wave 0, lane q (sub 0). Buffer aliases the Q image.
  __syncthreads();
  float* mv = reinterpret_cast<float*>(qimg);
  int* mi = reinterpret_cast<int*>(qimg + 64 * K * 4);
#pragma unroll 1
  for (int w = 0; w < 8; ++w) {
    if (wid == w && !(w == 0 && my_sub == 0)) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        mv[lane * K + j] = tk.v[j];
        mi[lane * K + j] = tk.i[j];
      }
    }
    __syncthreads();
    if (wid == 0 && my_sub == 0) {
#pragma unroll 1
      for (int s = (w == 0 ? 1 : 0); s < LPQ; ++s) {
        const int src = s * NQ + my_q;
        for (int j = 0; j < K; ++j) {
          const float v = mv[src * K + j];
          if (!(v > tk.v[K - 1])) break;
          tk.insert(v, mi[src * K + j]);
        }
      }
    }
    __syncthreads();
  }
  if (wid == 0 && my_sub == 0 && q0 + my_q < nq) {
    const size_t base = ((size_t)blockIdx.x * nq + q0 + my_q) * K;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      ws_v[base + j] = tk.v[j];
      ws_i[base + j] = tk.i[j];
    }
  }
}


// ------------------------------------------------------------------------------------------------
// Streaming stage 1 for k <= 8 (the RAG path: top-4 of 1M-10M rows): one workgroup per CU-sized row
// range, X streamed at HBM rate.
//  * operands swapped (MFMA A = 16 X rows, B = 16 queries): lane l ends a 16-row group owning query
//    l&15 (+16i) and rows 4(l>>4)..+3 - it inserts its 4 candidates straight from the accumulator, no LDS
//    transpose, no wave barrier per group;
//  * X fragments flow through a 16-deep register ring (16 KiB in flight per wave) that runs across
//    group boundaries: the two 64-B halves of every 128-B X line are issued back to back;
//  * per-lane register top-K lists; the 32 lists of a query (8 waves x 4 row-lanes) are merged in LDS
//    once at the end.
// ------------------------------------------------------------------------------------------------
template <int MT, int K, int RING>
__global__ __launch_bounds__(512) void sim_topk_stream(const bf16* __restrict__ Q, const bf16* __restrict__ X,
                                                       const float* __restrict__ bias, int nq, int N, int D,
                                                       int rows_per_wg, float* __restrict__ ws_v,
                                                       int* __restrict__ ws_i) {
  constexpr int NQ = 16 * MT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* qimg = smem;
  float* bsm = reinterpret_cast<float*>(smem + (size_t)NQ * D * 2);  // this workgroup's bias rows
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q0 = blockIdx.y * NQ;
  const int ncols = D / 8;
  const int wg_row0 = blockIdx.x * rows_per_wg;
  for (int e = tid; e < NQ * ncols; e += 512) {
    const int r = e / ncols, u = e % ncols;
    bf16x8 v = (q0 + r < nq) ? load8(Q + (size_t)(q0 + r) * D + u * 8) : bf16x8{};
    *reinterpret_cast<bf16x8*>(qimg + (size_t)r * D * 2 + ((u ^ (r & 15)) << 4)) = v;
  }
  // bias through LDS: a global load inside the X stream would make every wait drain the ring
  for (int r = tid; r < rows_per_wg; r += 512) bsm[r] = wg_row0 + r < N ? bias[wg_row0 + r] : -INFINITY;
  __syncthreads();

  TopK<K> tk[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) tk[i].init();
  const int wave_rows = rows_per_wg / 8;  // multiple of 16
  const int r_begin = wg_row0 + wid * wave_rows;
  const int r_end = min(N, r_begin + wave_rows);
  const int ngroups = r_end > r_begin ? (r_end - r_begin + 15) / 16 : 0;
  const int nk = D / 32;             // k-steps per 16-row group; RING divides it
  const int total = ngroups * nk;    // a multiple of RING: no tail guard inside the stream
  // the stream position advances by RING k-steps per chunk; pointers are stepped, never divided
  const bf16* const xlast = X + (size_t)(N - 1) * D + (D - 32) + 8 * (lane >> 4);
  const bf16* xrow = X + (size_t)min(r_begin + (lane & 15), N - 1) * D + 8 * (lane >> 4);  // group g row
  const size_t gstep = (size_t)16 * D;                                                    // next group
  int pf_t = 0;                  // k-step of the prefetch pointer within its group
  const bf16* pf = xrow;         // prefetch pointer (k-step j0 + RING)
  auto advance_pf = [&]() {      // RING k-steps ahead
    pf_t += RING;
    if (pf_t == nk) {
      pf_t = 0;
      pf += gstep - (size_t)32 * (nk - RING);
    } else {
      pf += 32 * RING;
    }
  };
  bf16x8 ring[RING];
#pragma unroll
  for (int u = 0; u < RING; ++u) ring[u] = load8(pf + 32 * u);
  advance_pf();
  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  int g = 0, t0 = 0;
  for (int j0 = 0; j0 < total; j0 += RING) {
    // past the stream's end the prefetch re-reads the last row (clamped, harmless)
    const bf16* p = j0 + RING < total ? pf : xlast - 32 * (RING - 1);
    // query fragments one k-step ahead (LDS latency hides under the previous step's MFMAs)
    auto rdq = [&](bf16x8* qf, int t) {
      const int uu = 4 * t + (lane >> 4);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int qr = 16 * i + (lane & 15);
        qf[i] = *reinterpret_cast<const bf16x8*>(qimg + (size_t)qr * D * 2 + ((uu ^ (qr & 15)) << 4));
      }
    };
    bf16x8 qa[MT], qb[MT];
    rdq(qa, t0);
#pragma unroll
    for (int u = 0; u < RING; ++u) {
      bf16x8* qc = (u & 1) ? qb : qa;
      bf16x8* qn = (u & 1) ? qa : qb;
      if (u + 1 < RING) rdq(qn, t0 + u + 1);
#pragma unroll
      for (int i = 0; i < MT; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[u], qc[i], acc[i], 0, 0, 0);  // D[x row][query]
      ring[u] = load8(p + 32 * u);  // consumed first, then refilled: the slot keeps its registers
    }
    advance_pf();
    t0 += RING;
    if (t0 == nk) {  // a 16-row group is complete: 4 candidate rows per lane and query tile
      const int rl = r_begin - wg_row0 + 16 * g + 4 * (lane >> 4);
      const f32x4 bv = *reinterpret_cast<const f32x4*>(bsm + rl);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wg_row0 + rl + r;
        if (row < r_end) {
#pragma unroll
          for (int i = 0; i < MT; ++i) tk[i].insert(acc[i][r] + bv[r], row);
        }
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      t0 = 0;
      ++g;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // merge the 32 lists of every query (list = 4 * wave + row-lane group) in LDS (aliases the Q image)
  __syncthreads();
  float* mv = reinterpret_cast<float*>(smem);
  int* mi = reinterpret_cast<int*>(smem + (size_t)NQ * 32 * K * 4);
  const int list = wid * 4 + (lane >> 4);
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int q = 16 * i + (lane & 15);
#pragma unroll
    for (int jj = 0; jj < K; ++jj) {
      mv[(q * 32 + list) * K + jj] = tk[i].v[jj];
      mi[(q * 32 + list) * K + jj] = tk[i].i[jj];
    }
  }
  __syncthreads();
  if (tid < NQ && q0 + tid < nq) {
    TopK<K> m;
    m.init();
    for (int l = 0; l < 32; ++l)
      for (int jj = 0; jj < K; ++jj) {
        const float v = mv[(tid * 32 + l) * K + jj];
        if (!(v > m.v[K - 1])) break;
        m.insert(v, mi[(tid * 32 + l) * K + jj]);
      }
    const size_t base = ((size_t)blockIdx.x * nq + q0 + tid) * K;
#pragma unroll
    for (int jj = 0; jj < K; ++jj) {
      ws_v[base + jj] = m.v[jj];
      ws_i[base + jj] = m.i[jj];
    }
  }
}

// stage 2: one 256-thread workgroup per query merges nwg lists of K.
template <int K>
__global__ __launch_bounds__(256) void sim_topk_stage2(const float* __restrict__ ws_v, const int* __restrict__ ws_i,
                                                       int nwg, int nq, int k_out, float* __restrict__ out_v,
                                                       int64_t* __restrict__ out_i) {
  __shared__ float mv[128 * K];
  __shared__ int mi[128 * K];
  const int q = blockIdx.x, tid = threadIdx.x;
  TopK<K> tk;
  tk.init();
  for (int w = tid; w < nwg; w += 256) {
    const size_t base = ((size_t)w * nq + q) * K;
    for (int j = 0; j < K; ++j) {
      const float v = ws_v[base + j];
      if (!(v > tk.v[K - 1])) break;
      tk.insert(v, ws_i[base + j]);
    }
  }
  // tree merge: 256 -> 128 -> ... -> 1
#pragma unroll 1
  for (int half = 128; half >= 1; half >>= 1) {
    if (tid >= half && tid < 2 * half) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        mv[(tid - half) * K + j] = tk.v[j];
        mi[(tid - half) * K + j] = tk.i[j];
      }
    }
    __syncthreads();
    if (tid < half) {
      for (int j = 0; j < K; ++j) {
        const float v = mv[tid * K + j];
        if (!(v > tk.v[K - 1])) break;
        tk.insert(v, mi[tid * K + j]);
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (j < k_out) {
        out_v[(size_t)q * k_out + j] = tk.v[j];
        out_i[(size_t)q * k_out + j] = tk.i[j];
      }
  }
}

template <typename F>
void set_max_lds(F* f, int bytes) {
  hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

template <int MT, int K>
void run_topk(const void* Q, const void* X, const float* bias, int nq, int N, int D, int k, float* ws_v, int* ws_i,
              int nwg, int rows_per_wg, float* out_v, int64_t* out_i, hipStream_t st) {
  constexpr int NQ = 16 * MT;
  const size_t lds = (size_t)NQ * D * 2 + (size_t)8 * NQ * 17 * 4;
  auto k1 = sim_topk_stage1<MT, K>;
  static bool once = false;
  if (!once) {
    set_max_lds(k1, 160 * 1024);
    once = true;
  }
  const int qtiles = (nq + NQ - 1) / NQ;
  k1<<<dim3(nwg, qtiles), 512, lds, st>>>((const bf16*)Q, (const bf16*)X, bias, nq, N, D, rows_per_wg, ws_v, ws_i);
  GAI_LAUNCH_CHECK();
  sim_topk_stage2<K><<<nq, 256, 0, st>>>(ws_v, ws_i, nwg, nq, k, out_v, out_i);
  GAI_LAUNCH_CHECK();
}

template <int MT, int K, int RING>
void run_stream_r(const void* Q, const void* X, const float* bias, int nq, int N, int D, int k, float* ws_v,
                  int* ws_i, int nwg, int rows_per_wg, float* out_v, int64_t* out_i, hipStream_t st) {
  constexpr int NQ = 16 * MT;
  const size_t lds = std::max((size_t)NQ * D * 2 + (size_t)rows_per_wg * 4, (size_t)NQ * 32 * K * 8);
  auto k1 = sim_topk_stream<MT, K, RING>;
  static bool once = false;
  if (!once) {
    set_max_lds(k1, 160 * 1024);
    once = true;
  }
  const int qtiles = (nq + NQ - 1) / NQ;
  k1<<<dim3(nwg, qtiles), 512, lds, st>>>((const bf16*)Q, (const bf16*)X, bias, nq, N, D, rows_per_wg, ws_v, ws_i);
  GAI_LAUNCH_CHECK();
  sim_topk_stage2<K><<<nq, 256, 0, st>>>(ws_v, ws_i, nwg, nq, k, out_v, out_i);
  GAI_LAUNCH_CHECK();
}

template <int MT, int K>
void run_stream(const void* Q, const void* X, const float* bias, int nq, int N, int D, int k, float* ws_v, int* ws_i,
                int nwg, int rows_per_wg, float* out_v, int64_t* out_i, hipStream_t st) {
  const int nk = D / 32;
  if (nk % 16 == 0) return run_stream_r<MT, K, 16>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
  if (nk % 8 == 0) return run_stream_r<MT, K, 8>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
  if (nk % 4 == 0) return run_stream_r<MT, K, 4>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
  return run_stream_r<MT, K, 1>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
}

template <int K>
void run_topk_k(const void* Q, const void* X, const float* bias, int nq, int N, int D, int k, float* ws_v, int* ws_i,
                int nwg, int rows_per_wg, float* out_v, int64_t* out_i, hipStream_t st) {
  if constexpr (K <= 8) {
    // streaming kernel (host sizes rows_per_wg as a multiple of 128 for it)
    if (rows_per_wg % 128 == 0 && rows_per_wg <= 8192) {
      auto fits = [&](int nq_tile) { return (size_t)nq_tile * D * 2 + (size_t)rows_per_wg * 4 <= 160 * 1024; };
      if (nq > 32 && fits(64))
        return run_stream<4, K>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
      if (nq > 16 && fits(32))
        return run_stream<2, K>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
      if (fits(16))
        return run_stream<1, K>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
    }
  }
  // largest query tile that fits LDS (Q image + scratch, with room for the K-merge buffer)
  auto fits = [&](int mt) {
    const size_t lds = (size_t)16 * mt * D * 2 + (size_t)8 * 16 * mt * 17 * 4;
    return lds <= 160 * 1024 && (size_t)16 * mt * D * 2 >= (size_t)64 * K * 8;
  };
  if (nq > 16 && fits(4)) return run_topk<4, K>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
  if (nq > 16 && fits(2)) return run_topk<2, K>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
  if (fits(1)) return run_topk<1, K>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
  gai_launch_error(__FILE__, __LINE__, "sim_topk: dimension too large for the LDS query tile");
}

}  // namespace

// Cross-list merge (the sharded index's W shard lists per query): stage 2 alone over ws [nlists][nq][cap].
void gai_topk_merge(const float* vals, const int* idx, int nlists, int nq, int cap, int k, float* out_v, int64_t* out_i,
                    hipStream_t st) {
  if (nq == 0) return;
  switch (cap) {
    case 4: sim_topk_stage2<4><<<nq, 256, 0, st>>>(vals, idx, nlists, nq, k, out_v, out_i); break;
    case 8: sim_topk_stage2<8><<<nq, 256, 0, st>>>(vals, idx, nlists, nq, k, out_v, out_i); break;
    case 16: sim_topk_stage2<16><<<nq, 256, 0, st>>>(vals, idx, nlists, nq, k, out_v, out_i); break;
    case 32: sim_topk_stage2<32><<<nq, 256, 0, st>>>(vals, idx, nlists, nq, k, out_v, out_i); break;
    case 64: sim_topk_stage2<64><<<nq, 256, 0, st>>>(vals, idx, nlists, nq, k, out_v, out_i); break;
    default: gai_launch_error(__FILE__, __LINE__, "topk_merge: cap must be 4, 8, 16, 32 or 64");
  }
  GAI_LAUNCH_CHECK();
}

int gai_topk_cap(int k) { return k <= 4 ? 4 : k <= 8 ? 8 : k <= 16 ? 16 : k <= 32 ? 32 : 64; }

void gai_sim_topk(const void* Q, const void* X, const float* bias, int nq, int N, int D, int k, float* ws_v,
                  int* ws_i, int nwg, int rows_per_wg, float* out_v, int64_t* out_i, hipStream_t st) {
  if (nq == 0) return;
  if (D % 32) gai_launch_error(__FILE__, __LINE__, "sim_topk: D must be a multiple of 32");
  switch (gai_topk_cap(k)) {
    case 4: return run_topk_k<4>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
    case 8: return run_topk_k<8>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
    case 16: return run_topk_k<16>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
    case 32: return run_topk_k<32>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
    default: return run_topk_k<64>(Q, X, bias, nq, N, D, k, ws_v, ws_i, nwg, rows_per_wg, out_v, out_i, st);
  }
}
