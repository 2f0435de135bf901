// Decode GEMM for M <= 64 on the natural weight layout: C[M, N] = A[M, K] . W[N, K]^T (+ fused epilogue).
//
// At decode sizes every weight byte is read once and the activations (<= 64 x K, L2-resident) are tiny,
// so the kernel is an HBM weight stream with MFMAs riding along. Measured on MI355X
// (tools/microbench/dec_stream.hip, profiles/r2/dec_stream_microbench.jsonl): a wave streaming its 16
// weight rows into a register ring reaches 5.1-5.4 TB/s on the plain [N][K] layout (5.8-5.9 on a
// fragment-shuffled copy), but as soon as the same wave ALSO loads its activation fragments from global
// memory (16 rows x 64 B per load, the shape of an MFMA operand) the stream collapses to 1.6 TB/s at
// M = 64: the per-CU load path, not HBM, is the limit. So here the activations never take that path:
//  * a workgroup = 8 waves = NT column tiles (16 columns each) x KQ = 8 / NT K-quarters; every wave
//    streams its 16 weight rows over its K range through a branch-free 8-set register ring (7 k32
//    steps in flight, one 16-B load per lane per step);
//  * the activation K-slices all waves need are staged ONCE per workgroup into LDS in 32 KiB stages
//    (full 128-B lines, register-staged: the loads are ordinary loads, so hipcc's counted vmcnt stays
//    exact beside the weight loads - cdna_hip_programming §5 'Projection GEMM at M = 256' 4(b)), two
//    stages in flight in registers, two LDS slots, one barrier per stage; A fragments come from LDS
//    with ds_read_b128 on an XOR-swizzled image (conflict-free for every row width);
//  * the KQ partial sums are combined in LDS and the epilogue (bias, GELU / ReLU / quick-GELU,
//    residual, interleaved SwiGLU, fp32 logits) is applied in the same kernel: no split-K slabs, no
//    reduce launch, no second copy of the weights.
#include "gai_common.h"
#include "gai_epilogue.h"
#include "gai_kernels.h"

#include <cstdlib>
#include <type_traits>

using namespace gai;

namespace {

constexpr int kThreads = 512;  // 8 waves
constexpr int kStage = 32768;  // activation bytes per LDS stage
constexpr int kD = 7;          // weight k32 steps in flight per wave
constexpr int kSets = kD + 1;  // register sets of the weight ring

template <int MB, int KQ>
struct DecCfg {
  static constexpr int ROWS = 16 * MB;
  static constexpr int BKS = kStage / (ROWS * KQ * 2);  // k per K-quarter per stage
  static constexpr int SPS = BKS / 32;                  // k32 steps per stage
  static constexpr int RB = BKS * 2;                    // bytes per staged row
  static constexpr int CPR = BKS / 8;                   // 16-B chunks per staged row
  static constexpr int L = 2 * SPS > kSets ? 2 * SPS : kSets;  // steps per unrolled loop body
  static constexpr int Q = RB >= 256 ? 1 : 256 / RB;   // rows sharing one 256-B bank row
  static_assert(SPS >= 1 && (SPS & (SPS - 1)) == 0, "stage must hold a power-of-two number of k32 steps");
};

// XOR swizzle of the 16-B chunk index of staged row r: the 16 rows one ds_read_b128 lane group reads at
// the same logical chunk land on 16 distinct 16-B bank slots.
template <int MB, int KQ>
__device__ __forceinline__ int dec_swz(int r) {
  using C = DecCfg<MB, KQ>;
  return C::RB >= 256 ? (r & 15) : ((r / C::Q) & (C::CPR - 1));
}

template <int EPI>
__device__ __forceinline__ float dec_act(float v, const bf16* bias, int n) {
  if (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RESIDUAL || EPI == EPI_BIAS_RELU ||
      EPI == EPI_BIAS_QUICKGELU)
    v += (float)bias[n];
  if (EPI == EPI_BIAS_GELU) v = gelu_erf(v);
  if (EPI == EPI_BIAS_RELU) v = fmaxf(v, 0.f);
  if (EPI == EPI_BIAS_QUICKGELU) v = quick_gelu(v);
  return v;
}

template <bool OUTF32>
__device__ __forceinline__ void dec_store8(void* C, size_t off, const float (&v)[8]) {
  if (OUTF32) {
    float* p = reinterpret_cast<float*>(C) + off;
    *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<float4*>(p + 4) = float4{v[4], v[5], v[6], v[7]};
  } else {
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
    store8(reinterpret_cast<bf16*>(C) + off, o);
  }
}

// PART: K is also split over gridDim.y workgroups (deep-K projections: down); each writes its fp32 partial
// slab [ks][M][N] instead of the epilogue, reduced by the split-K tail kernels (gemm_splitk.hip).
// PSW: W is the fragment-shuffled copy [N/16][K/32][64 lanes][8] (ops.shuffle_fragments): a wave's k32 step
// is ONE contiguous KiB (8 full 128-B lines) instead of 16 half lines, loaded non-temporally (read once;
// profiles/r2/dec_stream_microbench.jsonl: 5.8-6.5 TB/s shuffled + nt vs 5.0-5.4 on the natural layout).
// MoE (moe_offs != nullptr): blockIdx.z = expert e of W [E, N, K]; its rows are moe_offs[e] .. moe_offs[e + 1] of the
// expert-sorted order (<= 16 MB of them, host-checked), gathered from A through moe_rows when given, and written to
// C rows moe_offs[e] + m: the grouped expert GEMM of a decode step as a weight stream (moe.hip routes it here).
template <int MB, int NT, int EPI, bool OUTF32, bool PART = false, bool PSW = false>
__global__ __launch_bounds__(kThreads, 1) void gemm_dec2_kernel(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                                                void* C, const bf16* __restrict__ bias, const bf16* R,
                                                                int M, int N, int K, int ldc, float* __restrict__ part,
                                                                const int* __restrict__ moe_rows,
                                                                const int* __restrict__ moe_offs) {
  constexpr int KQ = 8 / NT;
  int row0 = 0;
  if (moe_offs != nullptr) {  // wave-uniform: the whole workgroup leaves before any barrier when the expert is idle
    const int e = blockIdx.z;
    row0 = moe_offs[e];
    M = moe_offs[e + 1] - row0;
    if (M <= 0) return;
    W += (size_t)e * N * K;
    if constexpr (OUTF32) C = reinterpret_cast<float*>(C) + (size_t)row0 * ldc;
    else C = reinterpret_cast<bf16*>(C) + (size_t)row0 * ldc;
  }
  using Cf = DecCfg<MB, KQ>;
  constexpr int ROWS = Cf::ROWS, SPS = Cf::SPS, RB = Cf::RB, CPR = Cf::CPR, L = Cf::L, BKS = Cf::BKS;
  constexpr int BN = 16 * NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 x [KQ][ROWS][RB] A stages; epilogue tile
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntl = wid % NT, kq = wid / NT;
  const int nb = blockIdx.x * BN;
  const int ks = blockIdx.y, KR = K / gridDim.y, kbase = ks * KR;  // this workgroup's K range
  const int KW = KR / KQ;
  const int nsteps = KW / 32;  // host: multiple of L
  const int nstages = nsteps / SPS;

  // ---- weight stream: rows nb + 16 ntl + (lane & 15), k = kq KW + 32 s + 8 (lane >> 4)
  constexpr int WSTEP = PSW ? 512 : 32;  // elements per k32 step of one wave's stream
  const bf16* wp = PSW ? W + ((size_t)min((nb >> 4) + ntl, (N >> 4) - 1) * (K >> 5) + ((kbase + kq * KW) >> 5)) * 512 +
                             8 * lane
                       : W + (size_t)min(nb + 16 * ntl + (lane & 15), N - 1) * K + kbase + (size_t)kq * KW +
                             8 * (lane >> 4);
  auto wload = [&](int s) -> bf16x8 {
    const bf16x8* p = reinterpret_cast<const bf16x8*>(wp + (size_t)WSTEP * s);
    if constexpr (PSW) return __builtin_nontemporal_load(p);
    else return *p;
  };

  // ---- activation staging: chunk p = (4 wid + j) 64 + lane of a stage's [KQ][ROWS][CPR] chunks
  const bf16* asrc[4];
  int adst[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = (wid * 4 + j) * 64 + lane;
    const int strip = p / (ROWS * CPR), rem = p % (ROWS * CPR), r = rem / CPR, c = rem % CPR;
    const int rr = min(r, M - 1);
    const int src = moe_offs == nullptr ? rr : moe_rows != nullptr ? moe_rows[row0 + rr] : row0 + rr;
    asrc[j] = A + (size_t)src * K + kbase + (size_t)strip * KW + 8 * c;
    adst[j] = strip * ROWS * RB + r * RB + 16 * (c ^ dec_swz<MB, KQ>(r));
  }
  bf16x8 ast[2][4];
  auto a_load = [&](int st, bf16x8(&v)[4]) {
    const int o = min(st, nstages - 1) * BKS;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = load8(asrc[j] + o);
  };
  auto a_write = [&](int slot, const bf16x8(&v)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<bf16x8*>(smem + slot * kStage + adst[j]) = v[j];
  };
  // A-fragment reads: row 16 i + (lane & 15) of this wave's K-quarter, logical chunk 4 ss + (lane >> 4)
  int ard[MB], asw[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) {
    const int r = 16 * i + (lane & 15);
    ard[i] = kq * ROWS * RB + r * RB;
    asw[i] = dec_swz<MB, KQ>(r);
  }
  const int cq = lane >> 4;

  f32x4 acc[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 rw[kSets];

  a_load(0, ast[0]);
  a_write(0, ast[0]);
  a_load(1, ast[1]);
#pragma unroll
  for (int d = 0; d < kD; ++d) rw[d] = wload(min(d, nsteps - 1));
  __syncthreads();

  // Stage st: at its first step issue the loads of stage st + 2 (register set st & 1); at its last
  // step write stage st + 1 (loaded one stage earlier) into LDS slot (st + 1) & 1, then the barrier.
  // Branch-free: past the end the loads re-read the last stage / step (L2 hits).
  for (int s0 = 0; s0 < nsteps; s0 += L) {
#pragma unroll
    for (int u = 0; u < L; ++u) {
      const int s = s0 + u;
      const int st = s / SPS;
      if (u % SPS == 0) a_load(st + 2, ast[(u / SPS) & 1]);
      rw[(u + kD) % kSets] = wload(min(s + kD, nsteps - 1));
      const char* sb = smem + (st & 1) * kStage;
      const int c = 4 * (u % SPS) + cq;
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(sb + ard[i] + 16 * (c ^ asw[i]));
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, rw[u % kSets], acc[i], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (u % SPS == SPS - 1) {
        a_write((st + 1) & 1, ast[(u / SPS + 1) & 1]);
        __syncthreads();
      }
    }
  }

  // ---- combine the KQ partial tiles and apply the epilogue: red[kq][m][n], row stride BN + 4 floats
  constexpr int RS = BN + 4;
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(kq * ROWS + 16 * i + 4 * cq + r) * RS + 16 * ntl + (lane & 15)] = acc[i][r];
  __syncthreads();
  if constexpr (PART) {
    constexpr int ITEMS = ROWS * BN / 8;
    for (int e = tid; e < ITEMS; e += kThreads) {
      const int m = e / (BN / 8), c0 = 8 * (e % (BN / 8));
      const int n = nb + c0;
      if (m >= M || n >= N) continue;
      float v[8];
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < KQ; ++q) t += red[(q * ROWS + m) * RS + c0 + x];
        v[x] = t;
      }
      dec_store8<true>(part, ((size_t)ks * M + m) * N + n, v);
    }
  } else if (EPI == EPI_SWIGLU) {
    // 16-column tiles (2j, 2j + 1) are (gate, up); output columns nb / 2 + 16 j + 8 h .. + 7
    constexpr int ITEMS = ROWS * NT;  // (m, j, h)
    for (int e = tid; e < ITEMS; e += kThreads) {
      const int m = e / NT, jh = e % NT, j = jh >> 1, h = jh & 1;
      const int gc = 32 * j + 8 * h;
      if (m >= M || nb + gc >= N) continue;
      float v[8];
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        float g = 0.f, up = 0.f;
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
          g += red[(q * ROWS + m) * RS + gc + x];
          up += red[(q * ROWS + m) * RS + gc + 16 + x];
        }
        v[x] = silu(g) * up;
      }
      dec_store8<OUTF32>(C, (size_t)m * ldc + nb / 2 + 16 * j + 8 * h, v);
    }
  } else {
    constexpr int ITEMS = ROWS * BN / 8;  // (m, 8-column group)
    for (int e = tid; e < ITEMS; e += kThreads) {
      const int m = e / (BN / 8), c0 = 8 * (e % (BN / 8));
      const int n = nb + c0;
      if (m >= M || n >= N) continue;
      float v[8];
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < KQ; ++q) t += red[(q * ROWS + m) * RS + c0 + x];
        v[x] = dec_act<EPI>(t, bias, n + x);
      }
      if (EPI == EPI_RESIDUAL || EPI == EPI_BIAS_RESIDUAL) {  // bf16 output: bf16(bf16(acc) + R) (store_out)
        const bf16x8 rv = load8(R + (size_t)m * ldc + n);
#pragma unroll
        for (int x = 0; x < 8; ++x) v[x] = (OUTF32 ? v[x] : (float)(bf16)v[x]) + (float)rv[x];
      }
      dec_store8<OUTF32>(C, (size_t)m * ldc + n, v);
    }
  }
}

template <int MB, int NT>
constexpr int dec2_steps_multiple() { return DecCfg<MB, 8 / NT>::L; }

template <int MB, int NT, int EPI, bool OUTF32, bool PART = false, bool PSW = false>
void dec2_launch(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
                 hipStream_t st, int KS = 1, float* part = nullptr, const int* moe_rows = nullptr,
                 const int* moe_offs = nullptr, int E = 1) {
  auto kern = gemm_dec2_kernel<MB, NT, EPI, OUTF32, PART, PSW>;
  constexpr int lds = 2 * kStage;
  static bool once = false;
  if (!once) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    once = true;
  }
  const int blocks = (N + 16 * NT - 1) / (16 * NT);
  kern<<<dim3(blocks, KS, E), kThreads, lds, st>>>((const bf16*)A, (const bf16*)W, C, (const bf16*)bias,
                                                   (const bf16*)R, M, N, K, ldc, part, moe_rows, moe_offs);
  GAI_LAUNCH_CHECK();
}

template <int MB, int NT, bool PSW>
bool dec2_dispatch_epi(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                       int ldc, int epi, int out_f32, hipStream_t st) {
#define GAI_D2(E)                                                                    \
  case E:                                                                            \
    if (out_f32)                                                                     \
      dec2_launch<MB, NT, E, true, false, PSW>(A, W, C, bias, R, M, N, K, ldc, st);  \
    else                                                                             \
      dec2_launch<MB, NT, E, false, false, PSW>(A, W, C, bias, R, M, N, K, ldc, st); \
    return true;
  switch (epi) {
    GAI_D2(EPI_NONE)
    GAI_D2(EPI_BIAS)
    GAI_D2(EPI_BIAS_GELU)
    GAI_D2(EPI_RESIDUAL)
    GAI_D2(EPI_BIAS_RESIDUAL)
    GAI_D2(EPI_BIAS_RELU)
    GAI_D2(EPI_BIAS_QUICKGELU)
    case EPI_SWIGLU:
      if constexpr (NT >= 2) {
        if (out_f32)
          dec2_launch<MB, NT, EPI_SWIGLU, true, false, PSW>(A, W, C, bias, R, M, N, K, ldc, st);
        else
          dec2_launch<MB, NT, EPI_SWIGLU, false, false, PSW>(A, W, C, bias, R, M, N, K, ldc, st);
        return true;
      }
      return false;
    default:
      return false;
  }
#undef GAI_D2
}

template <int MB>
bool dec2_shape_ok(int NT, int K) {
  const int KQ = 8 / NT;
  if (K % KQ) return false;
  const int KW = K / KQ;
  if (KW % 32) return false;
  const int L = NT == 8 ? dec2_steps_multiple<MB, 8>() : NT == 4 ? dec2_steps_multiple<MB, 4>()
              : NT == 2 ? dec2_steps_multiple<MB, 2>() : dec2_steps_multiple<MB, 1>();
  return (KW / 32) % L == 0;
}

template <int MB>
int dec2_pick_nt(int N, int K, bool swiglu) {
  static const int force = getenv("GAI_DEC2_NT") ? atoi(getenv("GAI_DEC2_NT")) : 0;
  // 64: measured on MI355X (profiles/r2/dec2_minwg_sweep.txt) the widest tile wins on the wide shapes
  // (gate_up+SwiGLU at M = 64: 54.9 us with 224 workgroups vs 66.4 us with 448): every workgroup re-stages
  // the whole activation K range, so fewer, wider workgroups move fewer bytes through the load path
  // 128 since round 5: at TP = 8 shard widths (LM head N 16032, O / down N 8192) the 64-workgroup tile left half
  // the CUs idle (LM head 53.2 -> 49.6 us, O 14.7 -> 10.5, down 28.8 -> 22.2; Llama-3-8B shapes pick the same tile)
  static const int min_wg = getenv("GAI_DEC2_MINWG") ? atoi(getenv("GAI_DEC2_MINWG")) : 128;
  if (force) return dec2_shape_ok<MB>(force, K) && !(swiglu && force < 2) ? force : 0;
  // widest column tile (least activation re-staging) that still gives every CU a workgroup; at MB = 1
  // the NT = 8 body (64 unrolled steps, 186 VGPRs) ran 4.6x slower than NT = 4 (lm_head, M = 1)
  for (int NT = MB == 1 ? 4 : 8; NT >= (swiglu ? 2 : 1); NT >>= 1)
    if ((N + 16 * NT - 1) / (16 * NT) >= min_wg && dec2_shape_ok<MB>(NT, K)) return NT;
  for (int NT = swiglu ? 2 : 1; NT <= (MB == 1 ? 4 : 8); NT <<= 1)
    if (dec2_shape_ok<MB>(NT, K)) return NT;
  return 0;
}

template <int MB, bool PSW>
bool dec2_run(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
              int epi, int out_f32, hipStream_t st) {
  const int NT = dec2_pick_nt<MB>(N, K, epi == EPI_SWIGLU);
  switch (NT) {
    case 8: return dec2_dispatch_epi<MB, 8, PSW>(A, W, C, bias, R, M, N, K, ldc, epi, out_f32, st);
    case 4: return dec2_dispatch_epi<MB, 4, PSW>(A, W, C, bias, R, M, N, K, ldc, epi, out_f32, st);
    case 2: return dec2_dispatch_epi<MB, 2, PSW>(A, W, C, bias, R, M, N, K, ldc, epi, out_f32, st);
    case 1: return dec2_dispatch_epi<MB, 1, PSW>(A, W, C, bias, R, M, N, K, ldc, epi, out_f32, st);
    default: return false;
  }
}

}  // namespace

// Wide projections only (gate_up, LM head: N >= 16384 by default; TP-shard O / down: N >= 8192 at K <= 4096): there the activation re-staging is
// <= 1/2 of the weight bytes and this kernel beats the split-K kernels (gate_up+SwiGLU 54.9 vs 80.9 us,
// LM head 233 vs 327 us at M = 64). On the narrow ones (QKV, O, down) every column tile needs the whole
// activation K range, 2-4x the weight bytes, and the split-K kernels stay ahead.
int gai_gemm_dec2_ok(int M, int N, int K, int epi) {
  // Also 8192 <= N < 16384 at shallow K (<= 4096) since round 5: the O and down projections of a Llama-3-70B TP = 8
  // shard (K 1024 / 3584) run faster here than split-K (profiles/r5/tp8_rank). At deep K the full-K tile leaves half
  // the CUs idle on a long stream: Llama-3-70B on one GPU (QKV / O, K 8192) config 3 1.57 -> 1.49 q/s when they ran
  // here (profiles/r5/config3_dec2_ab) - those keep the split-K kernels.
  static const int min_n = getenv("GAI_DEC2_MINN") ? atoi(getenv("GAI_DEC2_MINN")) : 16384;
  const bool shallow_shard = N >= 8192 && K <= 4096 && !getenv("GAI_DEC2_MINN");
  if (M < 1 || M > 64 || N % 16 || (N < min_n && !shallow_shard) || (epi == EPI_SWIGLU && N % 32)) return 0;
  static const bool off = getenv("GAI_DEC2") && atoi(getenv("GAI_DEC2")) == 0;
  if (off) return 0;
  const bool sw = epi == EPI_SWIGLU;
  if (M <= 16) return dec2_pick_nt<1>(N, K, sw) > 0;
  if (M <= 32) return dec2_pick_nt<2>(N, K, sw) > 0;
  return dec2_pick_nt<4>(N, K, sw) > 0;
}

bool gai_gemm_dec2(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
                   int epi, int out_f32, hipStream_t st, int psw) {
  if (!gai_gemm_dec2_ok(M, N, K, epi)) return false;
  if (psw) {
    if (M <= 16) return dec2_run<1, true>(A, W, C, bias, R, M, N, K, ldc, epi, out_f32, st);
    if (M <= 32) return dec2_run<2, true>(A, W, C, bias, R, M, N, K, ldc, epi, out_f32, st);
    return dec2_run<4, true>(A, W, C, bias, R, M, N, K, ldc, epi, out_f32, st);
  }
  if (M <= 16) return dec2_run<1, false>(A, W, C, bias, R, M, N, K, ldc, epi, out_f32, st);
  if (M <= 32) return dec2_run<2, false>(A, W, C, bias, R, M, N, K, ldc, epi, out_f32, st);
  return dec2_run<4, false>(A, W, C, bias, R, M, N, K, ldc, epi, out_f32, st);
}

namespace {

// K split for the partial-slab mode. Preferred: a KS giving EXACTLY a multiple of 256 workgroups (every CU
// streams; down at N = 4096: NT = 4 x KS = 4 = 256), else the smallest KS (2..16) whose per-workgroup K range
// fits the unrolled loop and that gives >= 192 workgroups (a K range per CU long enough to stream, few slabs;
// NT = 8 x KS = 7 = 224, 1/8 of the CUs idle).
// The exact split is taken only while its fp32 slabs (written, then read by the tail: 8 KS M N bytes) stay within
// 1/8 of the weight bytes (2 N K): a TP = 8 shard of Llama-3-70B gate_up (N 7168, K 8192) has its only exact split at
// KS = 16, whose slabs are half the weight stream - 47.8 us vs 30.6 us at KS = 2 (224 workgroups;
// profiles/r5/tp8_rank/dec_hbm_sweep.txt).
template <int MB>
int dec2_part_ks(int N, int K, int NT, bool exact) {
  const int blocks = (N + 16 * NT - 1) / (16 * NT);
  static const int force_ks = getenv("GAI_DEC2_PART_KS") ? atoi(getenv("GAI_DEC2_PART_KS")) : 0;  // A/B sweeps
  if (force_ks > 1)
    return K % force_ks == 0 && (K / force_ks) % 32 == 0 && dec2_shape_ok<MB>(NT, K / force_ks) ? force_ks : 0;
  for (int KS = 2; KS <= 16; ++KS) {
    if (K % KS || (K / KS) % 32 || !dec2_shape_ok<MB>(NT, K / KS)) continue;
    if (exact ? (blocks * KS) % 256 == 0 && 4 * KS * 16 * MB * 8 <= K : blocks * KS >= 192) return KS;
  }
  return 0;
}

// GAI_DEC2_PART_NT = 4 | 8 forces the column tile; default: the 256-exact NT = 4 split when it exists
int dec2_part_nt_env() {
  static const int v = getenv("GAI_DEC2_PART_NT") ? atoi(getenv("GAI_DEC2_PART_NT")) : 0;
  return v;
}

template <int MB, bool PSW>
int dec2_part_run(const void* A, const void* W, int M, int N, int K, float* ws, hipStream_t st, bool launch) {
  const int force = dec2_part_nt_env();
  if (MB > 1 && force != 8) {
    int KS4 = dec2_part_ks<MB>(N, K, 4, force != 4);
    if (!KS4 && force != 4) KS4 = dec2_part_ks<MB>(N, K, 4, false);  // no cheap exact split: >= 192 workgroups
    if (KS4) {
      if (launch)
        dec2_launch<MB, 4, EPI_NONE, true, true, PSW>(A, W, nullptr, nullptr, nullptr, M, N, K, N, st, KS4, ws);
      return KS4;
    }
  }
  constexpr int NT = MB == 1 ? 4 : 8;
  const int KS = dec2_part_ks<MB>(N, K, NT, false);
  if (KS && launch)
    dec2_launch<MB, NT, EPI_NONE, true, true, PSW>(A, W, nullptr, nullptr, nullptr, M, N, K, N, st, KS, ws);
  return KS;
}

int dec2_part_dispatch(const void* A, const void* W, int M, int N, int K, float* ws, hipStream_t st, bool launch,
                       bool psw = false) {
  static const int min_k = getenv("GAI_DEC2_PART_MINK") ? atoi(getenv("GAI_DEC2_PART_MINK")) : 8192;
  static const bool off = getenv("GAI_DEC2") && atoi(getenv("GAI_DEC2")) == 0;
  // M <= 16: the register-streamed split-K kernel is faster (down at M = 1: 30 vs 34 us)
  if (off || M <= 16 || M > 64 || N % 16 || K < min_k) return 0;
  if (psw) return M <= 32 ? dec2_part_run<2, true>(A, W, M, N, K, ws, st, launch)
                          : dec2_part_run<4, true>(A, W, M, N, K, ws, st, launch);
  if (M <= 32) return dec2_part_run<2, false>(A, W, M, N, K, ws, st, launch);
  return dec2_part_run<4, false>(A, W, M, N, K, ws, st, launch);
}

}  // namespace

// Deep-K decode projections (down: K = 14336) on the natural layout: LDS-staged activations, K split over
// KS workgroups writing fp32 slabs ws[KS][M][N] for the split-K tail kernels. Returns KS (0: shape not
// handled, nothing launched).
int gai_gemm_dec2_partials_ks(int M, int N, int K) { return dec2_part_dispatch(nullptr, nullptr, M, N, K, nullptr, 0, false); }
int gai_gemm_dec2_partials(const void* A, const void* W, int M, int N, int K, float* ws, hipStream_t st, int psw) {
  return dec2_part_dispatch(A, W, M, N, K, ws, st, true, psw != 0);
}

// Decode-sized grouped expert GEMM (moe.hip: rows_total <= 64, so no expert holds more than 64 rows): one weight
// stream per (expert, column tile) on the LDS-staged decode kernel, instead of 128 x 128 tiles that stage 128 A rows
// for a handful of live ones and keep one 32 KB stage in flight per CU. swiglu: W rows interleaved per 16
// [gate16 | up16] (ops.interleave_gate_up), C = silu(gate) * up. Returns 0 when the shape does not fit.
int gai_moe_gemm_dec2(const void* A, const int* a_rows, const void* W, void* C, const int* offs, int E,
                      int rows_total, int N, int K, int swiglu, hipStream_t st) {
  if (rows_total < 1 || rows_total > 64 || N % 32) return 0;
  const int ldc = swiglu ? N / 2 : N;
  const int epi = swiglu ? EPI_SWIGLU : EPI_NONE;
#define GAI_MOE(MBV)                                                                                             \
  {                                                                                                              \
    const int NT = dec2_pick_nt<MBV>(N, K, swiglu != 0);                                                          \
    if (NT == 0 || (swiglu && NT < 2)) return 0;                                                                  \
    auto go = [&](auto ntc) {                                                                                     \
      constexpr int NTV = decltype(ntc)::value;                                                                   \
      if (epi == EPI_SWIGLU) {                                                                                    \
        if constexpr (NTV >= 2)                                                                                   \
          dec2_launch<MBV, NTV, EPI_SWIGLU, false>(A, W, C, nullptr, nullptr, rows_total, N, K, ldc, st, 1,       \
                                                   nullptr, a_rows, offs, E);                                     \
      } else {                                                                                                    \
        dec2_launch<MBV, NTV, EPI_NONE, false>(A, W, C, nullptr, nullptr, rows_total, N, K, ldc, st, 1, nullptr,  \
                                               a_rows, offs, E);                                                  \
      }                                                                                                           \
    };                                                                                                            \
    switch (NT) {                                                                                                 \
      case 8: go(std::integral_constant<int, 8>{}); return 1;                                                     \
      case 4: go(std::integral_constant<int, 4>{}); return 1;                                                     \
      case 2: go(std::integral_constant<int, 2>{}); return 1;                                                     \
      case 1: if (!swiglu) { go(std::integral_constant<int, 1>{}); return 1; } return 0;                          \
      default: return 0;                                                                                          \
    }                                                                                                             \
  }
  static const bool off = getenv("GAI_MOE_DEC2") && atoi(getenv("GAI_MOE_DEC2")) == 0;
  if (off) return 0;
  if (rows_total <= 16) GAI_MOE(1)
  if (rows_total <= 32) GAI_MOE(2)
  GAI_MOE(4)
#undef GAI_MOE
}
