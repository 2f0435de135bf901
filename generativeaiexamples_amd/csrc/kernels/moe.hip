// Mixture-of-experts kernels (SURVEY K17 router top-k + permute, K18 grouped GEMM).
//
// moe_route:   softmax over the E router logits of each token, top-k experts, renormalised
//              weights (Mixtral), one lane per token.
// moe_gemm:    grouped GEMM over expert-sorted rows: Y[r] = act(A[row(r)] . W[e(r)]^T). The A rows
//              are gathered through an index list (dispatch permutation fused into the operand
//              staging: global_load_lds takes a per-lane source address), W is [E, N, K]. The work
//              list is derived on the device from the expert offsets (each 128-row tile finds its
//              expert by a prefix walk), so there is no host synchronisation and the launch can be
//              captured in a HIP graph. Same 128x128x64 MFMA tile as gemm_tiled; SwiGLU epilogue for
//              the fused w1|w3 projection.
// moe_combine: out[t] = sum_j w[t, j] * Y[pos[t, j]] (+ residual), bf16x8 vectorised.
#include "gai_common.h"
#include "gai_kernels.h"

using namespace gai;

namespace {

constexpr int MBM = 128, MBN = 128, MBK = 64;
constexpr int kMTile = MBM * MBK * 2;

__global__ void moe_route_kernel(const float* __restrict__ logits, int T, int E, int k, int renorm,
                                 int* __restrict__ ids, float* __restrict__ w) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const float* x = logits + (size_t)t * E;
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) mx = fmaxf(mx, x[e]);
  float s = 0.f;
  for (int e = 0; e < E; ++e) s += __expf(x[e] - mx);
  float bv[8];
  int bi[8];
  for (int j = 0; j < k; ++j) {
    bv[j] = -INFINITY;
    bi[j] = 0;
  }
  for (int e = 0; e < E; ++e) {
    const float p = __expf(x[e] - mx) / s;
    if (p > bv[k - 1]) {
      int j = k - 1;
      while (j > 0 && bv[j - 1] < p) {
        bv[j] = bv[j - 1];
        bi[j] = bi[j - 1];
        --j;
      }
      bv[j] = p;
      bi[j] = e;
    }
  }
  float tot = 0.f;
  for (int j = 0; j < k; ++j) tot += bv[j];
  for (int j = 0; j < k; ++j) {
    ids[(size_t)t * k + j] = bi[j];
    w[(size_t)t * k + j] = renorm ? bv[j] / tot : bv[j];
  }
}

__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, GAI_LDS(lds), 16, 0, 0);
}

template <bool SWIGLU>
__global__ __launch_bounds__(256, 2) void moe_gemm_kernel(const bf16* __restrict__ A, const int* __restrict__ a_rows,
                                                          const bf16* __restrict__ W, bf16* __restrict__ C,
                                                          const int* __restrict__ offs, int E, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // ---- which (expert, row tile) is this block?
  int t = blockIdx.x, e = 0, r0 = 0, rend = 0;
  {
    bool found = false;
    for (; e < E; ++e) {
      const int cnt = offs[e + 1] - offs[e];
      const int nt = (cnt + MBM - 1) / MBM;
      if (t < nt) {
        r0 = offs[e] + t * MBM;
        rend = offs[e + 1];
        found = true;
        break;
      }
      t -= nt;
    }
    if (!found) return;
  }
  const int n0 = blockIdx.y * MBN;
  const bf16* B = W + (size_t)e * N * K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

  size_t a_off[4], b_off[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = (wid * 4 + q) * 64 + lane;
    const int row = p >> 3, cl = p & 7, cg = cl ^ (row & 7);
    const int r = min(r0 + row, rend - 1);
    const int src_row = a_rows ? a_rows[r] : r;
    a_off[q] = (size_t)src_row * K + cg * 8;
    b_off[q] = (size_t)min(n0 + row, N - 1) * K + cg * 8;
  }
  auto stage = [&](int kt, int buf) {
    char* sa = smem + buf * 2 * kMTile;
    char* sb = sa + kMTile;
    const int k0 = kt * MBK;
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
  const int nk = K / MBK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const char* sa = smem + cur * 2 * kMTile;
    const char* sb = sa + kMTile;
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
  const int ldc = SWIGLU ? N / 2 : N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = r0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
      if (m >= rend) continue;
      if (SWIGLU) {
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const int nout = (n0 + wn * 64) / 2 + 16 * jp + (lane & 15);
          if (2 * nout < N) C[(size_t)m * ldc + nout] = (bf16)(silu(acc[i][2 * jp][r]) * acc[i][2 * jp + 1][r]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + wn * 64 + 16 * j + (lane & 15);
          if (n < N) C[(size_t)m * ldc + n] = (bf16)acc[i][j][r];
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void moe_combine_kernel(const bf16* __restrict__ Y, const int* __restrict__ pos,
                                                          const float* __restrict__ w, const bf16* residual,
                                                          bf16* __restrict__ out, int T, int k, int D) {
  const int units = D / 8;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)T * units) return;
  const int t = (int)(e / units), u = (int)(e % units);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < k; ++j) {
    const float wj = w[(size_t)t * k + j];
    const bf16x8 y = load8(Y + (size_t)pos[(size_t)t * k + j] * D + u * 8);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += wj * (float)y[q];
  }
  if (residual) {
    const bf16x8 r = load8(residual + (size_t)t * D + u * 8);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += (float)r[q];
  }
  bf16x8 o;
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = (bf16)acc[q];
  store8(out + (size_t)t * D + u * 8, o);
}


// Expert-sorted dispatch plan for small steps (decode: T*k rows) in ONE workgroup, replacing a stable
// argsort + scatter_add + cumsum + index_put (~10 launches and a radix sort per MoE layer). Counting sort:
// per-expert counts in LDS -> exclusive offsets -> chunks of 256 rows placed in flat order, each row's rank
// = expert cursor + rows of the same expert in earlier waves of the chunk + earlier lanes of its own wave
// (wave ballot per distinct expert), so rows of one expert keep their (token, slot) order like the stable
// argsort. Out-of-range ids are clamped so every output stays defined (moe_route never produces them).
// div > 1 buckets id / div instead of id (expert parallelism: the destination rank of a global expert id);
// a_pairs (optional) receives the flat pair index i of every sorted row next to its token i / k.
__global__ __launch_bounds__(256) void moe_dispatch_kernel(const int* __restrict__ ids, int n, int k, int E,
                                                           int* __restrict__ a_rows, int* __restrict__ offs,
                                                           int* __restrict__ pos, int div, int* __restrict__ a_pairs) {
  extern __shared__ int dsm[];  // cursor[E] | wave counts [4][E]
  int* cursor = dsm;
  int* wcnt = dsm + E;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int e = tid; e < E; e += 256) cursor[e] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += 256) atomicAdd(&cursor[min(max(ids[i] / div, 0), E - 1)], 1);
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int e = 0; e < E; ++e) {
      const int c = cursor[e];
      cursor[e] = run;
      offs[e] = run;
      run += c;
    }
    offs[E] = run;
  }
  for (int base = 0; base < n; base += 256) {
    for (int x = tid; x < 4 * E; x += 256) wcnt[x] = 0;
    __syncthreads();  // cursors final (first chunk) / advanced; wave counts cleared
    const int i = base + tid;
    const int e = i < n ? min(max(ids[i] / div, 0), E - 1) : -1;
    unsigned long long rest = __ballot(e >= 0);
    int rank = 0;
    while (rest) {  // wave-uniform: one pass per distinct expert in the wave
      const int leader = __builtin_ctzll(rest);
      const int le = __shfl(e, leader, 64);
      const unsigned long long m = __ballot(e == le);
      if (e == le) rank = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == leader) wcnt[wid * E + le] = __popcll(m);
      rest &= ~m;
    }
    __syncthreads();
    if (e >= 0) {
      int r = cursor[e] + rank;
      for (int w = 0; w < wid; ++w) r += wcnt[w * E + e];
      a_rows[r] = i / k;
      if (a_pairs != nullptr) a_pairs[r] = i;
      pos[i] = r;
    }
    __syncthreads();
    for (int x = tid; x < E; x += 256) cursor[x] += wcnt[x] + wcnt[E + x] + wcnt[2 * E + x] + wcnt[3 * E + x];
    __syncthreads();  // every cursor update has read its wave counts before the next chunk clears them
  }
}

// Expert-parallel send slab (decode, graph-capturable; parallel/ep.py dispatch_padded): W destination slabs
// of C rows. Slab row s = dest * C + r holds the r-th pair bound for rank dest in (token, choice) order (the
// moe_dispatch plan of the pairs bucketed by dest: offs / a_pairs), or padding past that rank's count: its
// local expert id is then the sentinel e_local, which the receiver's grouped GEMM skips (its row is not read).
// One wave per slab row, 16 B per lane. Rows are ld elements apart; with ld > D the local expert id is also
// stored as an int32 in the row's tail (element D), so rows and ids cross the wire in ONE exchange.
__global__ __launch_bounds__(256) void ep_pack_kernel(const bf16* __restrict__ x, const int* __restrict__ ids,
                                                      const int* __restrict__ offs, const int* __restrict__ a_pairs,
                                                      int rows, int C, int k, int D, int ld, int e_local,
                                                      bf16* __restrict__ send, int* __restrict__ send_eid) {
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (s >= rows) return;
  const int dest = s / C, j = offs[dest] + s % C;
  const bool live = j < offs[dest + 1];
  const int pair = live ? a_pairs[j] : 0;
  const int eid = live ? ids[pair] - dest * e_local : e_local;
  if (lane == 0) {
    if (send_eid != nullptr) send_eid[s] = eid;
    if (ld > D) *reinterpret_cast<int*>(send + (size_t)s * ld + D) = eid;
  }
  if (!live) return;
  const bf16* src = x + (size_t)(pair / k) * D;
  bf16* dst = send + (size_t)s * ld;
  for (int c = lane * 8; c < D; c += 512) store8(dst + c, load8(src + c));
}

// Expert-parallel combine: out[t] = sum_j w[t, j] * back[slab row of pair (t, j)] (+ residual), the slab row
// recomputed from the same plan (dest = id / e_local, r = pos - offs[dest]; pairs past the capacity C were
// dropped and contribute nothing). fp32 accumulation in choice order, like moe_combine.
__global__ __launch_bounds__(256) void ep_combine_kernel(const bf16* __restrict__ back, const int* __restrict__ ids,
                                                         const int* __restrict__ pos, const int* __restrict__ offs,
                                                         const float* __restrict__ w, const bf16* residual,
                                                         bf16* __restrict__ out, int T, int k, int D, int e_local,
                                                         int C) {
  const int units = D / 8;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)T * units) return;
  const int t = (int)(e / units), u = (int)(e % units);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < k; ++j) {
    const int i = t * k + j, dest = ids[i] / e_local, r = pos[i] - offs[dest];
    if (r >= C) continue;
    const float wj = w[i];
    const bf16x8 y = load8(back + (size_t)(dest * C + r) * D + u * 8);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += wj * (float)y[q];
  }
  if (residual) {
    const bf16x8 r = load8(residual + (size_t)t * D + u * 8);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += (float)r[q];
  }
  bf16x8 o;
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = (bf16)acc[q];
  store8(out + (size_t)t * D + u * 8, o);
}

}  // namespace

void gai_ep_pack(const void* x, const int* ids, const int* offs, const int* a_pairs, int W, int C, int k, int D,
                 int ld, int e_local, void* send, int* send_eid, hipStream_t st) {
  if (D % 8 || ld % 8 || ld < D || (ld > D && ld < D + 2))
    gai_launch_error(__FILE__, __LINE__, "ep_pack: D and the row stride must be multiples of 8 (stride D or >= D + 8)");
  if (send_eid == nullptr && ld == D) gai_launch_error(__FILE__, __LINE__, "ep_pack: nowhere to store expert ids");
  const int rows = W * C;
  if (rows == 0) return;
  ep_pack_kernel<<<(rows + 3) / 4, 256, 0, st>>>((const bf16*)x, ids, offs, a_pairs, rows, C, k, D, ld, e_local,
                                                 (bf16*)send, send_eid);
  GAI_LAUNCH_CHECK();
}

void gai_ep_combine(const void* back, const int* ids, const int* pos, const int* offs, const float* w,
                    const void* residual, void* out, int T, int k, int D, int e_local, int C, hipStream_t st) {
  if (T == 0) return;
  if (D % 8) gai_launch_error(__FILE__, __LINE__, "ep_combine: hidden size must be a multiple of 8");
  const long n = (long)T * (D / 8);
  ep_combine_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>((const bf16*)back, ids, pos, offs, w,
                                                                 (const bf16*)residual, (bf16*)out, T, k, D, e_local,
                                                                 C);
  GAI_LAUNCH_CHECK();
}

void gai_moe_dispatch(const int* ids, int n, int k, int E, int* a_rows, int* offs, int* pos, hipStream_t st,
                      int div, int* a_pairs) {
  if (E < 1 || E > 2048) gai_launch_error(__FILE__, __LINE__, "moe_dispatch: 1 <= experts <= 2048");
  if (div < 1) gai_launch_error(__FILE__, __LINE__, "moe_dispatch: bucket divisor >= 1");
  moe_dispatch_kernel<<<1, 256, 5 * E * sizeof(int), st>>>(ids, n, k, E, a_rows, offs, pos, div, a_pairs);
  GAI_LAUNCH_CHECK();
}

void gai_moe_route(const float* logits, int T, int E, int k, int renorm, int* ids, float* w, hipStream_t st) {
  if (T == 0) return;
  if (k > 8) gai_launch_error(__FILE__, __LINE__, "moe_route: top-k > 8 unsupported");
  moe_route_kernel<<<(T + 255) / 256, 256, 0, st>>>(logits, T, E, k, renorm, ids, w);
  GAI_LAUNCH_CHECK();
}

void gai_moe_gemm(const void* A, const int* a_rows, const void* W, void* C, const int* offs, int E, int rows_total,
                  int N, int K, int swiglu, hipStream_t st) {
  if (rows_total == 0) return;
  // decode steps (<= 64 expert rows in all): every expert's weights streamed once by the decode kernel
  if (gai_moe_gemm_dec2(A, a_rows, W, C, offs, E, rows_total, N, K, swiglu, st)) return;
  if (K % MBK) gai_launch_error(__FILE__, __LINE__, "moe_gemm: K must be a multiple of 64");
  const dim3 grid((rows_total + MBM - 1) / MBM + E, (N + MBN - 1) / MBN);
  const int lds = 4 * kMTile;
  static bool once = false;
  if (!once) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(moe_gemm_kernel<true>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipFuncSetAttribute(reinterpret_cast<const void*>(moe_gemm_kernel<false>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    once = true;
  }
  if (swiglu) {
    moe_gemm_kernel<true><<<grid, 256, lds, st>>>((const bf16*)A, a_rows, (const bf16*)W, (bf16*)C, offs, E, N, K);
  } else {
    moe_gemm_kernel<false><<<grid, 256, lds, st>>>((const bf16*)A, a_rows, (const bf16*)W, (bf16*)C, offs, E, N, K);
  }
  GAI_LAUNCH_CHECK();
}

void gai_moe_combine(const void* Y, const int* pos, const float* w, const void* residual, void* out, int T, int k,
                     int D, hipStream_t st) {
  if (T == 0) return;
  const long n = (long)T * (D / 8);
  moe_combine_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>((const bf16*)Y, pos, w, (const bf16*)residual,
                                                                   (bf16*)out, T, k, D);
  GAI_LAUNCH_CHECK();
}
