// Paged flash attention for gfx950.
//
// KV cache layout (written by rope_kv.hip): K [num_blocks, Hkv, 16, D],
// V^T [num_blocks, Hkv, D, 16] (16 tokens per page).
//
// attn_prefill: varlen, causal or bidirectional, GQA. Workgroup = 4 waves; each
// wave owns 32 query rows of one q-head, the workgroup shares 64-key K / V^T tiles
// in LDS (register-staged, issue-early / write-late: K then V^T through one register set,
// one barrier per tile, row-padded images). S^T = K.Q^T on v_mfma_f32_32x32x16_bf16 puts a full query row
// in one lane (swapped QK^T), so the online softmax is in-register; P^T is fed to
// the P.V MFMA straight from the S accumulator (k-order permuted on the V side,
// cdna_hip_programming §3 "accumulator tile as the next MFMA's operand"). exp2
// domain, fp32 statistics. Used for LLM prefill (incl. chunked prefill over a
// cached prefix) and for encoder self-attention (bidirectional, varlen).
//
// attn_decode: one query token per sequence, split-KV flash-decoding. Workgroup =
// (split, kv head, sequence); the GQA group (<= 16 q heads) is the 16-wide MFMA
// column, so K and V^T are read once per kv head with 16-B / 8-B loads straight to
// VGPRs (memory-bound decode row of the glds-vs-register table); the 4 waves
// combine through LDS, splits are merged by attn_decode_reduce.
#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "gai_common.h"
#include "gai_rope.h"
#include "gai_kernels.h"

using namespace gai;

namespace {

constexpr int kBS = 16;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNeg = -1e30f;
constexpr float kRescaleTh = 8.f;  // deferred running-max update of the prefill softmax (log2 domain)

// Raw v_exp_f32 (2^x). exp2f wraps it in a denormal range fix-up (cmp, 2x cndmask, add, ldexp: 6 VALU
// ops per element); softmax arguments are <= 0, and results below 2^-126 are irrelevant next to the
// row maximum's 1.0, so the bare instruction is exact enough and 6x cheaper on the VALU.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// max / sum of lane l and lane l ^ 32 in every lane: one v_permlane32_swap (lanes 32-63 of the first operand <->
// lanes 0-31 of the second) instead of a ds_bpermute round trip through the LDS unit
__device__ __forceinline__ float max_halves(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_halves(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ----------------------------------------------------------------------------------------------
// Prefill
// ----------------------------------------------------------------------------------------------
// LDS images are padded by 16 B per row instead of XOR-swizzled: the 16 rows one ds_read_b128 lane group
// reads at the same column then fall on 16 distinct 4-bank slots (row strides of 4 mod 64 or 36 mod 64
// banks), and every fragment address is one per-lane base plus a compile-time offset (no per-read
// address VALU in the loop).
template <int D>
struct PrefillCfg {
  static constexpr int KT = 64;                  // keys per tile
  static constexpr int KRS = D * 2 + 16;         // K image row stride (bytes)
  static constexpr int VRS = KT * 2 + 16;        // V^T image row stride (bytes)
  static constexpr int KBYTES = KT * KRS;        // K tile image
  static constexpr int VBYTES = D * VRS;         // V^T tile image
  static constexpr int BUF = KBYTES + VBYTES;
  static constexpr int CH = D / 32;              // 16-B chunks per thread per operand
  static constexpr int KU = D / 8;               // 16-B units per K row
};

// K image: row = key, 16-B unit u at 16u
template <int D>
__device__ __forceinline__ int k_lds_off(int key, int u) {
  return key * PrefillCfg<D>::KRS + (u << 4);
}
// V^T image: row = d (64 keys) of 8-B units u (4 keys each). Unit u = 4st + 2b1 + b0 is stored at position
// 4st + 2b0 + b1, so the two units one P.V MFMA operand takes (u = 4st + h and 4st + 2 + h) are one
// aligned 16-B pair read by a single ds_read_b128 (no register shuffles).
template <int D>
__device__ __forceinline__ int v_lds_off(int d, int u) {
  const int p = (u & ~3) | ((u & 1) << 1) | ((u >> 1) & 1);
  return d * PrefillCfg<D>::VRS + (p << 3);
}

// 16 (bf16 cache) or 8 (fp8 cache) bytes at base + off through a buffer resource built from the wave-uniform
// page base: the load's only VGPR operand is the loop-invariant lane offset, so no per-tile 64-bit address
// registers exist for the compiler to recycle (and then wait on) while the load is in flight.
template <typename T>
__device__ __forceinline__ T buf_load(const void* base, unsigned off) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
  if constexpr (sizeof(T) == 16) {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
  }
}

__device__ __forceinline__ bf16x8 kv_to_bf16(bf16x8 v, float) { return v; }
__device__ __forceinline__ bf16x8 kv_to_bf16(uint2 v, float s) { return fp8x8_to_bf16(v, s); }

// KV = bf16 or fp8 (OCP e4m3fn cache, dequantised by the per-layer scale when the tile is written to LDS)
// HL = q heads per wave (1 or 2, same 32 query rows): with 2, every K / V^T fragment a wave reads from LDS feeds two
// MFMAs, halving the LDS read traffic per FLOP (with one head per wave the fragment reads + tile writes, ~2.5K LDS
// cycles per CU per 64-key tile, exceed the ~2K MFMA cycles per SIMD); twice the registers, so one wave per SIMD.
// PIPE (HL == 1): software-pipelined main loop - tile kt+1's QK^T MFMAs are issued interleaved with tile kt's softmax
// exponentials and P.V MFMAs, so the matrix pipe has independent work while the VALU runs the softmax (the one-tile
// loop serialised them: 36.5 % MFMA busy, 7.5 VALU per MFMA, profiles/r5 section 10). K runs one tile ahead of V in
// LDS; the next K and V tiles are staged in two register sets during the iteration.
// NWV = waves per workgroup: 4 (two workgroups per CU) or 8 (one; the row groups of two 4-wave workgroups share each
// staged K / V^T tile, halving the tile loads and LDS writes per FLOP; head_dim 64 / 128, one head per wave)
template <int D, int HPW, typename KV, int HL = 1, bool PIPE = false, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, (D > 128 || HL > 1 || NWV == 8) ? 1 : 2) void attn_prefill_kernel(
    const bf16* __restrict__ q, const KV* __restrict__ kc, const KV* __restrict__ vc,
    const int* __restrict__ block_tables, int max_blocks, const int* __restrict__ tiles,
    const int* __restrict__ cu_q, const int* __restrict__ ctx_lens, bf16* __restrict__ out, int Hq, int Hkv,
    float scale, int causal, float* __restrict__ lse, float k_scale, float v_scale, int xcd, int q_ld) {
  using Cfg = PrefillCfg<D>;
  static_assert(HL == 1 || HPW % HL == 0, "a wave's heads come from one workgroup head group");
  constexpr int WPR = HPW / HL;  // waves per row group
  constexpr int RPW = NWV / WPR;  // row groups per workgroup
  constexpr int NTH = 64 * NWV;   // threads
  static_assert(NWV == 4 || (NWV == 8 && HL == 1 && !PIPE && (D == 64 || D == 128)), "8-wave workgroups: D 64 / 128");
  constexpr int CH = Cfg::CH * 4 / NWV;  // 16-B staging pieces per thread per tile half
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5;
  // xcd: head group = linear workgroup id mod gridDim.y. Workgroups go to the 8 XCDs round-robin by linear id, so
  // with 8 (or a multiple of 8) head groups every XCD serves one kv head (or two): the q tiles running together
  // on it re-read that head's K/V prefixes from the XCD's own L2 instead of all heads' prefixes streaming through
  // every XCD. MI355X (profiles/r3/attn_prefill_xcd): B 4 x S 2048 GQA 32/8 D 128 604 -> 660 TF/s, the headline
  // chunk (7 x 2406) 703 -> 728, Gemma D 256 315 -> 473; 64 x 512 MHA D 64 413 -> 394. GAI_ATTN_XCD=0: off.
  // xcd bits 1-2: wave priority around the MFMA phases (A/B, GAI_ATTN_PRIO): 1 = QK^T at priority 1, 2 = QK^T and P.V
  // xcd bit 3: exact running maximum (GAI_ATTN_RESCALE_TH=0). Otherwise the running maximum only moves when a tile
  // raises it by more than kRescaleTh (log2 units): probabilities then stay <= 2^kRescaleTh (bf16 / fp32 keep their
  // relative precision) and the O / l rescale almost never runs after the first tiles
  const float th = (xcd & 8) ? 0.f : kRescaleTh;
  const int xcd_flags = xcd;
  const int prio = (xcd >> 1) & 3;
  xcd &= 1;
  int bx = blockIdx.x, by = blockIdx.y;
  if (xcd) {
    const int L = blockIdx.y * gridDim.x + blockIdx.x;
    bx = L / gridDim.y;
    by = L % gridDim.y;
  }
  const int seq = tiles[2 * bx], qs = tiles[2 * bx + 1];
  const int qbeg = cu_q[seq], qlen = cu_q[seq + 1] - qbeg;
  const int ctx = ctx_lens[seq];
  const int head = by * HPW + HL * (wid % WPR);  // first of this wave's HL heads
  const int g = (by * HPW) / (Hq / Hkv);
  const int r0 = qs + 32 * (wid / WPR);  // first q row (within the sequence) of this wave
  const int qrow = r0 + (lane & 31);
  const int qpos = ctx - qlen + qrow;  // absolute position of this lane's query
  const int* bt = block_tables + (size_t)seq * max_blocks;

  // rows covered by the whole workgroup -> number of key tiles
  const int last_row = min(qs + 32 * RPW, qlen) - 1;
  const int kmax = causal ? (ctx - qlen + last_row + 1) : ctx;
  const int ntiles = (kmax + Cfg::KT - 1) / Cfg::KT;

  // Q fragments (B operand of S^T = K.Q^T): lane (q = lane&31, h) holds Q[q][16t + 8h .. +7]
  // HL == 1: the Q fragments live in registers. HL == 2: in this wave's LDS region (padded rows like the K image),
  // read once per tile per (head, k-step) - two heads' fragments in registers spill.
  constexpr int QL = HL == 1 ? 1 : 0;  // heads whose fragments stay in registers
  bf16x8 qf[QL ? HL : 1][D / 16];
  char* sq = smem + 2 * Cfg::BUF + wid * (HL * 32 * Cfg::KRS);
#pragma unroll
  for (int j = 0; j < HL; ++j) {
    // q rows are q_ld elements apart: Hq * D for a q tensor of its own, the packed QKV row for encoders
    const bf16* qp = q + (size_t)(qbeg + min(qrow, qlen - 1)) * q_ld + (size_t)(head + j) * D + 8 * h;
#pragma unroll
    for (int t = 0; t < D / 16; ++t) {
      const bf16x8 v = load8(qp + 16 * t);
      if constexpr (QL) qf[j][t] = v;
      else *reinterpret_cast<bf16x8*>(sq + (j * 32 + (lane & 31)) * Cfg::KRS + ((2 * t + h) << 4)) = v;
    }
  }

  // One set of staging registers (raw cache bytes: the fp8 conversion happens at the LDS write), used
  // twice per tile: the next tile's K is loaded at the top and written to the free buffer after QK^T,
  // then its V^T is loaded into the same registers and written before the barrier.
  // Piece c of thread tid (16 B of a tile half) lies in page (c*NTH + tid) / 2D of the tile, which is
  // wave-uniform (a wave's 64 pieces never straddle a page): the page's physical block is looked up with a
  // scalar load one tile ahead (nblk), and each load is a buffer load from that block's scalar base at a
  // loop-invariant 32-bit per-lane offset (no per-lane block-table round trip or 64-bit address math in the loop).
  using Stage = typename std::conditional<sizeof(KV) == 1, uint2, bf16x8>::type;
  Stage stg[CH];
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  unsigned voff[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) voff[c] = (unsigned)(((c * NTH + tid) % (2 * D)) * 8 * sizeof(KV));
  int nblk[CH];
  auto lookup_into = [&](int kt, int(&nb)[CH]) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int pidx = kt * 4 + (c * NTH + wid_u * 64) / (2 * D);
      nb[c] = bt[pidx * kBS < ctx ? pidx : 0];
    }
  };
  auto lookup = [&](int kt) { lookup_into(kt, nblk); };
  auto load_half_from = [&](const KV* base, const int(&nb)[CH], Stage(&dst)[CH]) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      // K page is [16][D] contiguous, V^T page [D][16]
      dst[c] = buf_load<Stage>(base + ((size_t)nb[c] * Hkv + g) * (kBS * D), voff[c]);
    }
  };
  auto load_half = [&](const KV* base) { load_half_from(base, nblk, stg); };
  auto write_k_from = [&](int buf, const Stage(&src)[CH]) {
    char* sk = smem + buf * Cfg::BUF;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int id = c * NTH + tid;
      const int page = id / (2 * D), w = id % (2 * D);
      const int key = page * 16 + w / Cfg::KU, u = w % Cfg::KU;
      *reinterpret_cast<bf16x8*>(sk + k_lds_off<D>(key, u)) = kv_to_bf16(src[c], k_scale);
    }
  };
  auto write_v_from = [&](int buf, const Stage(&src)[CH]) {
    char* sv = smem + buf * Cfg::BUF + Cfg::KBYTES;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int id = c * NTH + tid;
      const int page = id / (2 * D), w = id % (2 * D);
      const int d = w >> 1, half = w & 1;
      const int u8 = 4 * page + 2 * half;
      typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
      const bf16x8 vv = kv_to_bf16(src[c], v_scale);
      const bf16x4_t lo = {vv[0], vv[1], vv[2], vv[3]};
      const bf16x4_t hi = {vv[4], vv[5], vv[6], vv[7]};
      *reinterpret_cast<bf16x4_t*>(sv + v_lds_off<D>(d, u8)) = lo;
      *reinterpret_cast<bf16x4_t*>(sv + v_lds_off<D>(d, u8 + 1)) = hi;
    }
  };
  auto write_k = [&](int buf) { write_k_from(buf, stg); };
  auto write_v = [&](int buf) { write_v_from(buf, stg); };

  f32x16 acc_o[HL][D / 32];
  float m_run[HL], l_run[HL];
#pragma unroll
  for (int j = 0; j < HL; ++j) {
#pragma unroll
    for (int i = 0; i < D / 32; ++i) acc_o[j][i] = f32x16{};
    m_run[j] = kNeg;
    l_run[j] = 0.f;
  }
  const float sl2 = scale * kLog2e;

  if constexpr (PIPE) {
    static_assert(HL == 1, "the pipelined loop keeps one head per wave");
    // K(kt + 1) and V(kt) are in LDS at iteration kt: K in slot (kt + 1) & 1, V in slot kt & 1 (each slot = K image,
    // V^T image). During the iteration V(kt + 1) and K(kt + 2) stream into two register sets; after the MFMAs they
    // are written to V slot (kt + 1) & 1 (last read by P.V(kt - 1)) and K slot kt & 1 (last read by QK^T(kt), which ran
    // in iteration kt - 1); one barrier per iteration.
    Stage stv[CH];
    int nb_v[CH], nb_k[CH];
    auto qk_part = [&](int kslot, int sub, int t0, int nt, f32x16& acc) {
      const char* skk = smem + kslot * Cfg::BUF;
      const int key = 32 * sub + (lane & 31);
#pragma unroll
      for (int t = t0; t < t0 + nt; ++t) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(skk + k_lds_off<D>(key, 2 * t + h));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[0][t], acc, 0, 0, 0);
      }
    };
    f32x16 sc[2], sn[2];
    if (ntiles > 0) {
      lookup_into(0, nblk);
      load_half_from(kc, nblk, stg);
      write_k_from(0, stg);
      load_half_from(vc, nblk, stg);
      write_v_from(0, stg);
      if (ntiles > 1) {
        lookup_into(1, nb_v);
        load_half_from(kc, nb_v, stg);
        write_k_from(1, stg);
      }
      lookup_into(2, nb_k);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the Q fragments and the prologue tiles
    __syncthreads();
    sc[0] = f32x16{};
    sc[1] = f32x16{};
    if (ntiles > 0) {
      qk_part(0, 0, 0, D / 16, sc[0]);
      qk_part(0, 1, 0, D / 16, sc[1]);
    }
    __syncthreads();  // every wave has read K(0) before iteration 0 overwrites K slot 0 with K(2)
    for (int kt = 0; kt < ntiles; ++kt) {
      const bool more1 = kt + 1 < ntiles, more2 = kt + 2 < ntiles;
      if (more1) load_half_from(vc, nb_v, stv);  // V(kt + 1)
      if (more2) load_half_from(kc, nb_k, stg);  // K(kt + 2)
      // ---- softmax statistics of tile kt (as the one-tile loop)
      float mt = kNeg;
      const int kend = kt * 64 + 63;
      if (kend < ctx && (!causal || kend <= ctx - qlen + r0)) {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
          for (int r = 0; r < 16; ++r) mt = fmaxf(mt, sc[sub][r]);
      } else {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kt * 64 + 32 * sub + (r & 3) + 8 * (r >> 2) + 4 * h;
            const bool ok = key < ctx && (!causal || key <= qpos);
            const float x = ok ? sc[sub][r] : kNeg;
            sc[sub][r] = x;
            mt = fmaxf(mt, x);
          }
      }
      mt = max_halves(mt) * sl2;
      const float m_new = mt > m_run[0] + th ? mt : m_run[0];
      const float alpha = fexp2(m_run[0] - m_new);
      if (__any(alpha != 1.f)) {
#pragma unroll
        for (int i = 0; i < D / 32; ++i) acc_o[0][i] *= alpha;
      }
      m_run[0] = m_new;
      // ---- tile kt+1's QK^T interleaved with tile kt's exponentials and P.V: per 8-key step, D / 32 QK^T MFMAs
      // (independent of this tile's softmax) beside the step's 8 exps and its D / 32 P.V MFMAs
      sn[0] = f32x16{};
      sn[1] = f32x16{};
      const char* sv = smem + (kt & 1) * Cfg::BUF + Cfg::KBYTES;
      const int kslot = (kt + 1) & 1;
      float rs = 0.f;
      if (prio == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        if (more1) qk_part(kslot, st >> 1, (st & 1) * (D / 32), D / 32, sn[st >> 1]);
        const int sub = st >> 1, sp = st & 1;
        bf16x8 pf;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float pv = fexp2(fmaf(sc[sub][8 * sp + e], sl2, -m_new));
          rs += pv;
          pf[e] = (bf16)pv;
        }
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt) {
          const bf16x8 vf = *reinterpret_cast<const bf16x8*>(sv + v_lds_off<D>(32 * dt + (lane & 31), 4 * st + h));
          acc_o[0][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, acc_o[0][dt], 0, 0, 0);
        }
      }
      if (prio == 2) __builtin_amdgcn_s_setprio(0);
      l_run[0] = l_run[0] * alpha + rs;  // this lane half's keys; the halves are summed after the loop
      if (more2) write_k_from(kt & 1, stg);
      if (more1) write_v_from((kt + 1) & 1, stv);
#pragma unroll
      for (int c = 0; c < CH; ++c) nb_v[c] = nb_k[c];
      lookup_into(kt + 3, nb_k);  // pages past the context resolve to entry 0 (never read unmasked)
      __syncthreads();
      sc[0] = sn[0];
      sc[1] = sn[1];
    }
  } else if constexpr (NWV == 8) {
    // Staggered 8-wave loop (MI355X_MICROARCH "Two waves per SIMD", item 9): waves 4-7 (the second row group, each
    // the SIMD partner of wave w - 4) run half an iteration behind - their P.V of tile kt - 1, then their QK^T of tile
    // kt - so on every SIMD one wave's QK^T MFMAs meet the other's softmax VALU and P.V instead of both waves hitting
    // the matrix pipe, then the VALU, together. Tile j lives in LDS slot j % 3 (3 x 35 KiB): in iteration kt the
    // waves read slots kt % 3 and (kt - 1) % 3 while tile kt + 1 is written to the third; ntiles + 1 iterations, one
    // barrier each. The K / V^T of tile kt + 1 are loaded at the top of iteration kt and written at its end.
    const bool late = wid >= 4 && !(xcd_flags & 16);  // GAI_ATTN_STAGGER=0: every wave in step (A/B)
    Stage stv[CH];
    auto slot = [&](int t) { return smem + (t % 3) * Cfg::BUF; };
    auto qk = [&](const char* sk, f32x16(&sc)[2]) {
      constexpr int NT = D / 16;
      bf16x8 ka[NT], kb[NT];
      const int key = lane & 31;
      sc[0] = f32x16{};
      sc[1] = f32x16{};
#pragma unroll
      for (int t = 0; t < NT; ++t) ka[t] = *reinterpret_cast<const bf16x8*>(sk + k_lds_off<D>(key, 2 * t + h));
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        kb[t] = *reinterpret_cast<const bf16x8*>(sk + k_lds_off<D>(32 + key, 2 * t + h));
        sc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[t], qf[0][t], sc[0], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) sc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kb[t], qf[0][t], sc[1], 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, NT, 0);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NT, 0);
    };
    // masked row max, deferred running max, O and l rescaled at once (l += the tile's sum after its P.V)
    auto stats = [&](int kt, f32x16(&sc)[2]) {
      float mt = kNeg;
      const int kend = kt * 64 + 63;
      if (kend < ctx && (!causal || kend <= ctx - qlen + r0)) {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
          for (int r = 0; r < 16; ++r) mt = fmaxf(mt, sc[sub][r]);
      } else {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kt * 64 + 32 * sub + (r & 3) + 8 * (r >> 2) + 4 * h;
            const bool ok = key < ctx && (!causal || key <= qpos);
            const float x = ok ? sc[sub][r] : kNeg;
            sc[sub][r] = x;
            mt = fmaxf(mt, x);
          }
      }
      mt = max_halves(mt) * sl2;
      const float m_new = mt > m_run[0] + th ? mt : m_run[0];
      const float alpha = fexp2(m_run[0] - m_new);
      if (__any(alpha != 1.f)) {
#pragma unroll
        for (int i = 0; i < D / 32; ++i) acc_o[0][i] *= alpha;
      }
      l_run[0] *= alpha;
      m_run[0] = m_new;
    };
    auto pv = [&](const char* sv, const f32x16(&sc)[2]) {
      float rs = 0.f;
      if (prio == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const int sub = st >> 1, sp = st & 1;
        bf16x8 pf;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float p = fexp2(fmaf(sc[sub][8 * sp + e], sl2, -m_run[0]));
          rs += p;
          pf[e] = (bf16)p;
        }
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt) {
          const bf16x8 vf = *reinterpret_cast<const bf16x8*>(sv + v_lds_off<D>(32 * dt + (lane & 31), 4 * st + h));
          acc_o[0][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, acc_o[0][dt], 0, 0, 0);
        }
      }
      if (prio == 2) __builtin_amdgcn_s_setprio(0);
      l_run[0] += rs;  // per lane half (summed after the loop)
    };
    if (ntiles > 0) {
      lookup(0);
      load_half(kc);
      write_k(0);
      load_half(vc);
      write_v(0);
      lookup(1);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the Q fragments and tile 0
    __syncthreads();
    f32x16 sc[2];
    for (int kt = 0; kt <= ntiles; ++kt) {
      const bool more = kt + 1 < ntiles;
      if (more) {
        load_half(kc);
        load_half_from(vc, nblk, stv);
      }
      if (!late) {
        if (kt < ntiles) {
          if (prio) __builtin_amdgcn_s_setprio(1);
          qk(slot(kt), sc);
          if (prio) __builtin_amdgcn_s_setprio(0);
          stats(kt, sc);
          pv(slot(kt) + Cfg::KBYTES, sc);
        }
      } else {
        if (kt > 0) pv(slot(kt - 1) + Cfg::KBYTES, sc);  // tile kt - 1 (its statistics ran last iteration)
        if (kt < ntiles) {
          if (prio) __builtin_amdgcn_s_setprio(1);
          qk(slot(kt), sc);
          if (prio) __builtin_amdgcn_s_setprio(0);
          stats(kt, sc);
        }
      }
      lookup(kt + 2);  // after the LDS reads (an SMEM load in flight forces full lgkmcnt waits)
      if (more) {
        write_k_from((kt + 1) % 3, stg);
        write_v_from((kt + 1) % 3, stv);
      }
      __syncthreads();
    }
  } else {
  // K and V^T of the next tile staged through two register sets, both written at the end of the iteration (D <= 128,
  // one head per wave: +16 VGPRs)
  constexpr bool ESPLIT = HL == 1 && D <= 128;
  if (ntiles > 0) {
    lookup(0);
    load_half(kc);
    write_k(0);
    load_half(vc);
    write_v(0);
    lookup(1);
  }
  // Q fragments landed: without this wait the ntiles == 0 path reaches the loop header with the Q loads
  // pending, and hipcc's waitcnt pass then keeps vmcnt(7..0) in front of every tile's QK^T MFMAs, which
  // (counters are in order) waits for the next tile's K loads issued just above them.
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < ntiles;
    // tile kt + 1: K and V^T both loaded here and written at the end of the iteration (a whole iteration of load
    // latency cover; writing K right after QK^T left the K loads only the QK^T MFMAs to land in)
    Stage stv[ESPLIT ? CH : 1];
    if (more) {
      load_half(kc);
      if constexpr (ESPLIT) load_half_from(vc, nblk, stv);
    }
    const char* sk = smem + cur * Cfg::BUF;
    const char* sv = sk + Cfg::KBYTES;

    // S^T[key][q] for two 32-key halves (each K fragment feeds the wave's HL heads)
    if (prio) __builtin_amdgcn_s_setprio(1);
    f32x16 s[HL][2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int j = 0; j < HL; ++j) s[j][sub] = f32x16{};
    if constexpr (QL && D <= 128) {
      // The first 32-key half's D / 16 K fragments are read together, the second half's one per first-half MFMA:
      // no MFMA waits on its own LDS round trip (left to the compiler, one fragment register was re-used and
      // every QK^T MFMA waited lgkmcnt(0) behind its read)
      constexpr int NT = D / 16;
      bf16x8 ka[NT], kb[NT];
      const int key = lane & 31;
#pragma unroll
      for (int t = 0; t < NT; ++t) ka[t] = *reinterpret_cast<const bf16x8*>(sk + k_lds_off<D>(key, 2 * t + h));
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        kb[t] = *reinterpret_cast<const bf16x8*>(sk + k_lds_off<D>(32 + key, 2 * t + h));
        s[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[t], qf[0][t], s[0][0], 0, 0, 0);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) s[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kb[t], qf[0][t], s[0][1], 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, NT, 0);  // DS reads: first half
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one second-half read
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one first-half MFMA
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NT, 0);  // second-half MFMAs
    } else if constexpr (QL) {
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const int key = 32 * sub + (lane & 31);
#pragma unroll
        for (int t = 0; t < D / 16; ++t) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(sk + k_lds_off<D>(key, 2 * t + h));
#pragma unroll
          for (int j = 0; j < HL; ++j) s[j][sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[j][t], s[j][sub], 0, 0, 0);
        }
      }
    }
    if constexpr (!QL) {  // k-step outer: each K fragment (both halves) and each Q fragment read once per tile
#pragma unroll
      for (int t = 0; t < D / 16; ++t) {
        const bf16x8 kf0 = *reinterpret_cast<const bf16x8*>(sk + k_lds_off<D>(lane & 31, 2 * t + h));
        const bf16x8 kf1 = *reinterpret_cast<const bf16x8*>(sk + k_lds_off<D>(32 + (lane & 31), 2 * t + h));
#pragma unroll
        for (int j = 0; j < HL; ++j) {
          const bf16x8 qv = *reinterpret_cast<const bf16x8*>(sq + (j * 32 + (lane & 31)) * Cfg::KRS + ((2 * t + h) << 4));
          s[j][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf0, qv, s[j][0], 0, 0, 0);
          s[j][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf1, qv, s[j][1], 0, 0, 0);
        }
      }
    }
    if (prio) __builtin_amdgcn_s_setprio(0);
    if (!ESPLIT && more) {  // buffer cur ^ 1 was released by the previous barrier
      write_k(cur ^ 1);
      load_half(vc);
    }
    // online softmax (exp2 domain); lane owns query (lane&31), keys split across lane halves.
    // Interior tiles (every key < ctx and, causal, <= the wave's first query position) skip the
    // per-element mask: wave-uniform test, so only the diagonal / tail tiles pay for it.
    float mt[HL];
#pragma unroll
    for (int j = 0; j < HL; ++j) mt[j] = kNeg;
    const int kend = kt * 64 + 63;
    if (kend < ctx && (!causal || kend <= ctx - qlen + r0)) {
#pragma unroll
      for (int j = 0; j < HL; ++j)
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
          for (int r = 0; r < 16; ++r) mt[j] = fmaxf(mt[j], s[j][sub][r]);
    } else {
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kt * 64 + 32 * sub + (r & 3) + 8 * (r >> 2) + 4 * h;
          const bool ok = key < ctx && (!causal || key <= qpos);
#pragma unroll
          for (int j = 0; j < HL; ++j) {
            const float x = ok ? s[j][sub][r] : kNeg;
            s[j][sub][r] = x;
            mt[j] = fmaxf(mt[j], x);
          }
        }
    }
    // scores stay unscaled; the scale folds into the max (scale > 0) and into one fma per exp
    float m_new[HL], alpha[HL];
#pragma unroll
    for (int j = 0; j < HL; ++j) {
      mt[j] = max_halves(mt[j]) * sl2;
      m_new[j] = mt[j] > m_run[j] + th ? mt[j] : m_run[j];
      alpha[j] = fexp2(m_run[j] - m_new[j]);
      // lazy rescale: once the running maxima settle (most tiles after the first few) alpha == 1 in
      // every lane and the D/32 x 16 accumulator multiplies are skipped (bit-identical result)
      if (__any(alpha[j] != 1.f)) {
#pragma unroll
        for (int i = 0; i < D / 32; ++i) acc_o[j][i] *= alpha[j];
      }
      m_run[j] = m_new[j];
    }

    // O^T[d][q] += V^T[d][key] . P^T[key][q]. The 8 probabilities of each 8-key step are exponentiated
    // right before that step's MFMAs, so step st's MFMAs run in the matrix pipe while step st+1's
    // v_exp / cvt issue (the row sum is only needed after the tile). Each V^T fragment feeds the HL heads.
    float rs[HL];
#pragma unroll
    for (int j = 0; j < HL; ++j) rs[j] = 0.f;
    if (prio == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const int sub = st >> 1, sp = st & 1;
      bf16x8 pf[HL];
#pragma unroll
      for (int j = 0; j < HL; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float p = fexp2(fmaf(s[j][sub][8 * sp + e], sl2, -m_new[j]));
          rs[j] += p;
          pf[j][e] = (bf16)p;
        }
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
        // units 4st + h (lo) and 4st + 2 + h (hi) of row d: one 16-B pair in the image
        const bf16x8 vf = *reinterpret_cast<const bf16x8*>(sv + v_lds_off<D>(32 * dt + (lane & 31), 4 * st + h));
#pragma unroll
        for (int j = 0; j < HL; ++j)
          acc_o[j][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[j], acc_o[j][dt], 0, 0, 0);
      }
    }
    if (prio == 2) __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int j = 0; j < HL; ++j) l_run[j] = l_run[j] * alpha[j] + rs[j];  // per lane half (summed after the loop)
    // the next-but-one tile's page lookups (scalar loads) after the P.V reads: an SMEM load in flight makes every
    // LDS wait a full lgkmcnt(0) (the two return out of order)
    lookup(kt + 2);  // pages past the context resolve to entry 0 (never read unmasked)
    if (more) {
      if constexpr (ESPLIT) {
        write_k(cur ^ 1);
        write_v_from(cur ^ 1, stv);
      } else {
        write_v(cur ^ 1);
      }
    }
    __syncthreads();
  }
  }  // one-tile loop
  // each lane half accumulated the row sum of its own keys (every tile rescaled both by the same alpha)
#pragma unroll
  for (int j = 0; j < HL; ++j) l_run[j] = sum_halves(l_run[j]);

  if (qrow < qlen) {
#pragma unroll
    for (int j = 0; j < HL; ++j) {
      const float inv = l_run[j] > 0.f ? 1.f / l_run[j] : 0.f;
      bf16* op = out + ((size_t)(qbeg + qrow) * Hq + head + j) * D;
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
          bf16x4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc_o[j][dt][4 * c + r] * inv);
          *reinterpret_cast<bf16x4_t*>(op + 32 * dt + 8 * c + 4 * h) = o;
        }
      // natural-log softmax normaliser per (row, head): merges partial results (ring attention)
      if (lse != nullptr && h == 0)
        lse[(size_t)(qbeg + qrow) * Hq + head + j] =
            l_run[j] > 0.f ? (m_run[j] + __log2f(l_run[j])) * 0.69314718055994531f : kNeg;
    }
  }
}

// ----------------------------------------------------------------------------------------------
// Decode
// ----------------------------------------------------------------------------------------------
// FUSE (split_cnt != nullptr): the splits of a (sequence, kv head) are merged in the same launch by the split
// that finishes last, instead of a separate attn_decode_reduce launch. Hand-off without any fence
// (cdna_hip_programming Guideline 16, R1 form): the partials are stored write-through (sc1, relaxed agent-scope
// stores, so nothing is left dirty in this XCD's L2) -> every wave vmcnt(0) -> barrier -> lane 0 relaxed agent
// ticket fetch_add; the last arriver reads every split with sc1 loads (they bypass the CU's L1, so no acquire
// is needed). The first version published with a per-workgroup agent release (buffer_wbl2: 192.6 vs 117.4 us
// per layer). cnt[seq * Hkv + g] starts at 0 (zeroed at allocation) and the last arriver resets it for the next
// launch (graph replays).
typedef __attribute__((address_space(1))) unsigned gu32_t;
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store((gu32_t*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __uint_as_float(__hip_atomic_load((gu32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// Merge the flash-decoding partials (O, max, sum) of ns splits for one (sequence, q head, dim): groups of
// kMergeGroup splits, every load of a group issued before its math, running-max rescale between groups. The
// separate reduce launch and the in-launch merge (SC1: write-through partials read with sc1 loads) share it,
// so both round identically.
constexpr int kMergeGroup = 8;

// Keys per split. split_keys > 0: fixed. 0: adaptive - each sequence's context is cut into max_splits equal
// 128-key-aligned parts at run time, so a graph captured for the longest context a replay may see (the split count)
// still balances its splits on the contexts it actually runs (a fixed split sized for max_model_len = 3330 left
// a 2500-key context as 1792 + 708 keys: the critical path of the step).
__device__ __forceinline__ int split_len(int split_keys, int ctx, int max_splits) {
  if (split_keys > 0) return split_keys;
  const int per = (ctx + max_splits - 1) / max_splits;
  return max(128, (per + 127) / 128 * 128);
}
template <bool SC1>
__device__ __forceinline__ void merge_splits(const float* ws_o, const float* ws_ml, int B, int Hq, int D, int seq,
                                             int hq, int d, int ns, float& L, float& O) {
  float M = kNeg;
  L = 0.f;
  O = 0.f;
  for (int s0 = 0; s0 < ns; s0 += kMergeGroup) {
    float m[kMergeGroup], l[kMergeGroup], o[kMergeGroup];
#pragma unroll
    for (int j = 0; j < kMergeGroup; ++j) {
      const size_t i = ((size_t)min(s0 + j, ns - 1) * B + seq) * Hq + hq;
      m[j] = SC1 ? ld_sc1(ws_ml + i * 2) : ws_ml[i * 2];
      l[j] = SC1 ? ld_sc1(ws_ml + i * 2 + 1) : ws_ml[i * 2 + 1];
      o[j] = SC1 ? ld_sc1(ws_o + i * D + d) : ws_o[i * D + d];
    }
    float Mn = M;
#pragma unroll
    for (int j = 0; j < kMergeGroup; ++j) Mn = s0 + j < ns ? fmaxf(Mn, m[j]) : Mn;
    if (s0 > 0) {
      const float a = fexp2(M - Mn);
      L *= a;
      O *= a;
    }
#pragma unroll
    for (int j = 0; j < kMergeGroup; ++j) {
      const float f = s0 + j < ns ? fexp2(m[j] - Mn) : 0.f;
      L += l[j] * f;
      O += o[j] * f;
    }
    M = Mn;
  }
}

// NTL: the V^T cache loads are non-temporal (each decode step streams the cache once; keeps it from evicting the
// L2-resident Q / block tables / split partials)
// Occupancy: unconstrained, the compiler takes 138 VGPRs + 32 AGPRs (2 workgroups per CU, 512 resident), and two
// splits per (sequence, kv head) at B = 64 are exactly two rounds. Held to 3 per CU (no spill) with three splits it
// measured 7.424 vs 7.332 ms per step (profiles/r4/decode/decode_nt_split_ab.txt): kept at 2.
// QP (QkvFold): q is not read from memory - the prologue sums the split-K QKV partial slabs of this workgroup's
// GQA group, rounds to bf16 (the rounding of the unfused GEMM output), applies RoPE (the rounding of rope_kv) and
// stages the group's q rows in LDS; the split that holds the newest key also rotates / stores that key and value
// into the paged caches before its own key loop reads them (the only split that reads that page). This replaces
// the separate split-K RoPE / KV-write tail launch of the decode QKV projection.
template <int D, bool PIPE, int H, bool V16, typename KV, bool FUSE = false, bool NTL = false, bool QP = false>
__global__ __launch_bounds__(256) void attn_decode_kernel(
    const bf16* __restrict__ q, const KV* __restrict__ kc, const KV* __restrict__ vc,
    const int* __restrict__ block_tables, int max_blocks, const int* __restrict__ ctx_lens, bf16* __restrict__ out,
    float* __restrict__ ws_o, float* __restrict__ ws_ml, int B, int Hq, int Hkv, float scale, int split_keys,
    int max_splits, float k_scale, float v_scale, int* __restrict__ cnt, GaiQkvFold fold = GaiQkvFold{}) {
  static_assert(sizeof(KV) == 2 || V16, "fp8 KV decode uses the 16-key V^T loads");
  static_assert(!QP || sizeof(KV) == 2, "the folded QKV tail writes bf16 caches");
  __shared__ __attribute__((aligned(16))) float red_o[4][D][16];
  __shared__ float red_m[4][16], red_l[4][16];
  __shared__ int s_last;
  __shared__ __attribute__((aligned(16))) bf16 q_lds[QP ? 16 : 1][QP ? D : 8];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, gq = lane >> 4;
  const int split = blockIdx.x, g = blockIdx.y, seq = blockIdx.z;
  const int ratio = Hq / Hkv;
  const int ctx = ctx_lens[seq];
  split_keys = split_len(split_keys, ctx, max_splits);
  const int kstart = split * split_keys;
  if (kstart >= ctx) return;
  const int kend = min(ctx, kstart + split_keys);
  const int nsplit = (ctx + split_keys - 1) / split_keys;
  const int* bt = block_tables + (size_t)seq * max_blocks;
  const int qi = lane & 15;  // GQA head index inside the group (MFMA column)

  bf16x8 qf[D / 32];
  // QP prologue (called after this wave's first K / V chunk is in flight, so its latency hides under the stream):
  // quarter-row items (4 + 4 rotation partners of one head) of the group's ratio q heads, plus its k and v head in
  // the split that holds key ctx - 1
  auto qp_prologue = [&]() {
    constexpr int LPH = D / 8;
    const int nh = ratio + (split == nsplit - 1 ? 2 : 0);
    const size_t slab = (size_t)B * fold.n;
    for (int it = tid; it < nh * LPH; it += 256) {
      const int hh = it / LPH, i0 = (it % LPH) * 4;
      const int habs = hh < ratio ? g * ratio + hh : hh == ratio ? Hq + g : Hq + Hkv + g;
      const float* p1 = fold.part + (size_t)seq * fold.n + habs * D + i0;
      float x[4] = {0.f, 0.f, 0.f, 0.f}, y[4] = {0.f, 0.f, 0.f, 0.f};
      for (int s0 = 0; s0 < fold.ks; s0 += 4) {  // 4 slabs in flight; slab order from 0 (the split-K tails' rounding)
        float4 a[4], b[4];
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if (s0 + s < fold.ks) {
            a[s] = *reinterpret_cast<const float4*>(p1 + (s0 + s) * slab);
            b[s] = *reinterpret_cast<const float4*>(p1 + (s0 + s) * slab + D / 2);
          }
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if (s0 + s < fold.ks) {
            x[0] += a[s].x; x[1] += a[s].y; x[2] += a[s].z; x[3] += a[s].w;
            y[0] += b[s].x; y[1] += b[s].y; y[2] += b[s].z; y[3] += b[s].w;
          }
      }
      bf16x4 x1, x2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x1[j] = (bf16)x[j];
        x2[j] = (bf16)y[j];
      }
      if (hh < ratio) {
        const int pp = fold.pos[seq];
        const float4 c = *reinterpret_cast<const float4*>(fold.cos_sin + (size_t)pp * D + i0);
        const float4 sn = *reinterpret_cast<const float4*>(fold.cos_sin + (size_t)pp * D + D / 2 + i0);
        const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float u = (float)x1[j], w = (float)x2[j];
          x1[j] = (bf16)(u * cc[j] - w * ss[j]);
          x2[j] = (bf16)(w * cc[j] + u * ss[j]);
        }
        *reinterpret_cast<bf16x4*>(&q_lds[hh][i0]) = x1;
        *reinterpret_cast<bf16x4*>(&q_lds[hh][i0 + D / 2]) = x2;
      } else {
        rope_kv_store<D, bf16>(x1, x2, seq, habs, i0, fold.pos, fold.cos_sin, fold.slots, nullptr,
                               const_cast<bf16*>(reinterpret_cast<const bf16*>(kc)),
                               const_cast<bf16*>(reinterpret_cast<const bf16*>(vc)), Hq, Hkv, 1, 1.f, 1.f);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the new key / value have landed before any wave reads them
    __syncthreads();
    const bool qv = qi < ratio;
#pragma unroll
    for (int t = 0; t < D / 32; ++t)
      qf[t] = qv ? *reinterpret_cast<const bf16x8*>(&q_lds[qi][32 * t + 8 * gq]) : bf16x8{};
  };
  static_assert(!QP || !PIPE, "the folded QKV prologue runs in the non-pipelined loop");
  if constexpr (!QP) {
    const bool qv = qi < ratio;
    const bf16* qp = q + ((size_t)seq * Hq + g * ratio + (qv ? qi : 0)) * D + 8 * gq;
#pragma unroll
    for (int t = 0; t < D / 32; ++t) qf[t] = qv ? load8(qp + 32 * t) : bf16x8{};
  }

  f32x4 acc_o[D / 16];
#pragma unroll
  for (int i = 0; i < D / 16; ++i) acc_o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = kNeg, l_run = 0.f;
  const float sl2 = scale * kLog2e;

  // A wave step covers H halves of 32 keys (2 pages each). Per half: K rows for the QK^T MFMA (lane:
  // key row lane&15, 16 B of dims 32t + 8gq) and V^T columns for the PV MFMA.
  //  * V16 = false: S row m of MFMA i is key 16i + m; P^T's k order is then {4gq..4gq+3, 16+4gq..+3}
  //    and V^T is read as two 8-B pieces (one per page).
  //  * V16 = true: row m of MFMA i is key 8(m>>2) + 4i + (m&3), so lane group gq ends up holding the
  //    8 CONSECUTIVE keys 8gq..8gq+7 of P^T, and its V^T operand is one 16-B load (page gq>>1, keys
  //    8(gq&1)..+7): half the V load instructions.
  // Addresses of a chunk past the split are clamped to its last page (unconditional loads: a
  // data-dependent branch around them would force vmcnt(0) waits), and such keys are masked.
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  // fp8 caches: chunks hold the raw 8-byte pieces, converted to bf16 right before their MFMA
  using Raw = typename std::conditional<sizeof(KV) == 1, uint2, bf16x8>::type;
  struct Chunk {
    Raw k[H][2][D / 32];
    bf16x4_t vlo[H][V16 ? 1 : D / 16], vhi[H][V16 ? 1 : D / 16];
    Raw v8[H][V16 ? D / 16 : 1];
  };
  const int last_page = (kend - 1) / kBS;
  // physical blocks of a chunk's pages (scalar loads). The non-pipelined loop looks the NEXT chunk's blocks up
  // before issuing this chunk's K/V loads, so a K/V load never waits on a block-table round trip of its own.
  struct Blk {
    int b[H][2];
  };
  auto lookup = [&](int kb, Blk& o) {
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int p0 = min(kb / kBS + 2 * h, last_page);
      o.b[h][0] = bt[p0];
      o.b[h][1] = (p0 + 1) * kBS < ctx ? bt[p0 + 1] : o.b[h][0];
    }
  };
  auto load_chunk_blk = [&](int kb, const Blk& bl, Chunk& c) {
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int blk0 = bl.b[h][0], blk1 = bl.b[h][1];
      const size_t pb0 = ((size_t)blk0 * Hkv + g) * kBS * D, pb1 = ((size_t)blk1 * Hkv + g) * kBS * D;
      if (V16) {
        const int m = lane & 15;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int key = 8 * (m >> 2) + 4 * i + (m & 3);  // 0..31 inside the half
          const size_t pb = key < 16 ? pb0 : pb1;
#pragma unroll
          for (int t = 0; t < D / 32; ++t) {
            const Raw* kp = reinterpret_cast<const Raw*>(kc + pb + (size_t)(key & 15) * D + 32 * t + 8 * gq);
            // K is read with the default policy even under NTL: one load instruction covers 16 key rows x 64 B, so
            // each 128-B line is requested in two halves by consecutive instructions, and the second half then hits
            // the line the first one allocated in L2 (B = 64, ctx 2535 graph replay 7.251 / 7.236 -> 7.149 /
            // 7.169 ms per step, profiles/r6/decode/k_policy_ab); V^T loads cover whole lines and stay non-temporal
            c.k[h][i][t] = *kp;
          }
        }
        const size_t pbv = gq < 2 ? pb0 : pb1;
#pragma unroll
        for (int dt = 0; dt < D / 16; ++dt) {
          const Raw* vp = reinterpret_cast<const Raw*>(vc + pbv + (size_t)(16 * dt + (lane & 15)) * kBS + 8 * (gq & 1));
          if constexpr (NTL) c.v8[h][dt] = __builtin_nontemporal_load(vp);
          else c.v8[h][dt] = *vp;
        }
      } else if constexpr (sizeof(KV) == 2) {
#pragma unroll
        for (int t = 0; t < D / 32; ++t) {
          c.k[h][0][t] = load8((const bf16*)kc + pb0 + (size_t)(lane & 15) * D + 32 * t + 8 * gq);
          c.k[h][1][t] = load8((const bf16*)kc + pb1 + (size_t)(lane & 15) * D + 32 * t + 8 * gq);
        }
#pragma unroll
        for (int dt = 0; dt < D / 16; ++dt) {
          const size_t off = (size_t)(16 * dt + (lane & 15)) * kBS + 4 * gq;
          c.vlo[h][dt] = *reinterpret_cast<const bf16x4_t*>((const bf16*)vc + pb0 + off);
          c.vhi[h][dt] = *reinterpret_cast<const bf16x4_t*>((const bf16*)vc + pb1 + off);
        }
      }
    }
  };
  auto load_chunk = [&](int kb, Chunk& c) {
    Blk bl;
    lookup(kb, bl);
    load_chunk_blk(kb, bl, c);
  };
  auto compute_chunk = [&](int kb, const Chunk& c) {
    f32x4 s[H][2];
    float mt = kNeg;
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        s[h][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < D / 32; ++t)
          s[h][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kv_to_bf16(c.k[h][i][t], k_scale), qf[t], s[h][i], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb + 32 * h + (V16 ? 8 * gq + 4 * i + r : 16 * i + 4 * gq + r);
          const float x = key < kend ? s[h][i][r] * sl2 : kNeg;
          s[h][i][r] = x;
          mt = fmaxf(mt, x);
        }
      }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt);
    const float alpha = fexp2(m_run - m_new);
    float rs = 0.f;
    bf16x8 pf[H];
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = fexp2(s[h][i][r] - m_new);
          rs += pv;
          pf[h][4 * i + r] = (bf16)pv;
        }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l_run = l_run * alpha + rs;
    m_run = m_new;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) {
      acc_o[dt] *= alpha;
#pragma unroll
      for (int h = 0; h < H; ++h) {
        bf16x8 vf;
        if constexpr (V16) {
          vf = kv_to_bf16(c.v8[h][dt], v_scale);
        } else {
          vf = bf16x8{c.vlo[h][dt][0], c.vlo[h][dt][1], c.vlo[h][dt][2], c.vlo[h][dt][3],
                      c.vhi[h][dt][0], c.vhi[h][dt][1], c.vhi[h][dt][2], c.vhi[h][dt][3]};
        }
        acc_o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[h], acc_o[dt], 0, 0, 0);
      }
    }
  };

  constexpr int kStep = 128 * H;
  int kb = kstart + 32 * H * wid;
  if (PIPE) {
    if (kb < kend) {
      Chunk ca, cb;
      load_chunk(kb, ca);
      for (;;) {
        load_chunk(kb + kStep, cb);
        compute_chunk(kb, ca);
        kb += kStep;
        if (kb >= kend) break;
        load_chunk(kb + kStep, ca);
        compute_chunk(kb, cb);
        kb += kStep;
        if (kb >= kend) break;
      }
    }
  } else if (!QP) {
    if (kb < kend) {
      Blk nb;
      lookup(kb, nb);
      for (; kb < kend; kb += kStep) {
        Chunk c;
        load_chunk_blk(kb, nb, c);  // blocks looked up one chunk earlier
        // the next chunk's blocks, issued after this chunk's K/V loads (SMEM returns out of order, so a wait for the
        // blocks in use would also wait for these) and landing under this chunk's compute; pages past the split
        // clamp to its last page (looked up, never loaded)
        lookup(kb + kStep, nb);
        compute_chunk(kb, c);
      }
    }
  } else {
    // first chunk in flight before the prologue, unless it holds the newest key, whose value the prologue writes
    Blk nb;
    Chunk c0;
    const bool live = kb < kend;
    const bool pre = live && !(split == nsplit - 1 && kb <= ctx - 1 && ctx - 1 < kb + 32 * H);
    if (live) lookup(kb, nb);
    if (pre) load_chunk_blk(kb, nb, c0);
    qp_prologue();  // every wave (barrier inside)
    for (bool first = true; kb < kend; kb += kStep, first = false) {
      Chunk c;
      if (first && pre) c = c0;
      else load_chunk_blk(kb, nb, c);
      lookup(kb + kStep, nb);
      compute_chunk(kb, c);
    }
  }

  // combine the 4 waves: acc_o lane layout O^T[d = 16dt + 4gq + r][q = lane&15]
  if (lane < 16) {
    red_m[wid][lane] = m_run;
    red_l[wid][lane] = l_run;
  }
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) red_o[wid][16 * dt + 4 * gq + r][qi] = acc_o[dt][r];
  __syncthreads();
  for (int e = tid; e < ratio * D; e += 256) {
    const int qq = e / D, d = e % D;
    float M = kNeg;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, red_m[w][qq]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float f = fexp2(red_m[w][qq] - M);
      L += red_l[w][qq] * f;
      O += red_o[w][d][qq] * f;
    }
    const int hq = g * ratio + qq;
    if (nsplit == 1) {
      out[((size_t)seq * Hq + hq) * D + d] = (bf16)(L > 0.f ? O / L : 0.f);
    } else if constexpr (FUSE) {
      st_sc1(ws_o + (((size_t)split * B + seq) * Hq + hq) * D + d, O);
      if (d == 0) {
        st_sc1(ws_ml + (((size_t)split * B + seq) * Hq + hq) * 2, M);
        st_sc1(ws_ml + (((size_t)split * B + seq) * Hq + hq) * 2 + 1, L);
      }
    } else {
      ws_o[(((size_t)split * B + seq) * Hq + hq) * D + d] = O;
      if (d == 0) {
        ws_ml[(((size_t)split * B + seq) * Hq + hq) * 2] = M;
        ws_ml[(((size_t)split * B + seq) * Hq + hq) * 2 + 1] = L;
      }
    }
  }
  if constexpr (FUSE) {
    if (nsplit == 1) return;  // wave-uniform for the whole workgroup
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through partials have landed
    __syncthreads();
    if (tid == 0) s_last = __hip_atomic_fetch_add(cnt + seq * Hkv + g, 1, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT) == nsplit - 1;
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
    for (int e = tid; e < ratio * D; e += 256) {
      const int qq = e / D, d = e % D, hq = g * ratio + qq;
      float L, O;
      merge_splits<true>(ws_o, ws_ml, B, Hq, D, seq, hq, d, nsplit, L, O);
      out[((size_t)seq * Hq + hq) * D + d] = (bf16)(L > 0.f ? O / L : 0.f);
    }
    if (tid == 0) __hip_atomic_store(cnt + seq * Hkv + g, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int D>
__global__ void attn_decode_reduce_kernel(const float* __restrict__ ws_o, const float* __restrict__ ws_ml,
                                          const int* __restrict__ ctx_lens, bf16* __restrict__ out, int B, int Hq,
                                          int split_keys, int max_splits) {
  const int seq = blockIdx.x, hq = blockIdx.y, d = threadIdx.x;
  const int ctx = ctx_lens[seq];
  split_keys = split_len(split_keys, ctx, max_splits);
  const int ns = (ctx + split_keys - 1) / split_keys;
  if (ns <= 1) return;
  float L, O;
  merge_splits<false>(ws_o, ws_ml, B, Hq, D, seq, hq, d, ns, L, O);
  out[((size_t)seq * Hq + hq) * D + d] = (bf16)(L > 0.f ? O / L : 0.f);
}

// Raise a kernel's dynamic-LDS limit once per KERNEL (a static flag inside a template over the function type would be
// shared by every instantiation with the same signature, e.g. all bf16 prefill kernels).
template <typename F>
void set_max_lds(F* f, int bytes) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> done;
  const void* key = reinterpret_cast<const void*>(f);
  std::lock_guard<std::mutex> lk(mu);
  auto it = done.find(key);
  if (it != done.end() && it->second >= bytes) return;
  hipFuncSetAttribute(key, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  done[key] = bytes;
}

// Heads per wave of the prefill kernel (attn_prefill_kernel HL): 2 for head_dim 128 with >= 4 q heads per kv head when
// enabled (GAI_ATTN_HL=2 or gai_attn_prefill_set_hl), else 1. The tile list's rows per tile follow it
// (gai_attn_prefill_rows_per_tile), so it is read once per process unless set explicitly.
int g_prefill_hl = -1;
int prefill_hl(int D, int ratio) {
  if (g_prefill_hl < 0) g_prefill_hl = getenv("GAI_ATTN_HL") ? atoi(getenv("GAI_ATTN_HL")) : 1;
  return g_prefill_hl == 2 && D == 128 && ratio >= 4 ? 2 : 1;
}

}  // namespace

void gai_attn_prefill_set_hl(int hl) { g_prefill_hl = hl == 2 ? 2 : 1; }

namespace {
// Waves per workgroup of the one-tile prefill kernel: 8 for head_dim 64 / 128 at >= 4 q heads per kv head (one head
// per wave: 2 row groups x 4 heads = 64 rows per tile share each staged K / V^T tile), else 4 (GAI_ATTN_WAVES=4 forces
// it). Same box, interleaved (profiles/r6/attn_prefill/waves_ab_*): headline chunk 7 x 2406 GQA 32/8 782 / 779 ->
// 796 / 828 TF/s, B 4 x 2048 693 / 689 -> 706 / 696. Not for MHA: the 256-row tiles of one head waste up to 3 of
// their causal key tiles on the upper row groups (encoder shape, causal: 415 -> 295). The tile list's rows per tile
// follow it (gai_attn_prefill_rows_per_tile).
int prefill_waves(int D, int ratio) {
  static const int env = getenv("GAI_ATTN_WAVES") ? atoi(getenv("GAI_ATTN_WAVES")) : 8;
  static const int pipe = getenv("GAI_ATTN_PIPE") ? atoi(getenv("GAI_ATTN_PIPE")) : 0;
  return env == 8 && (D == 64 || D == 128) && ratio >= 4 && prefill_hl(D, ratio) == 1 && pipe != 1 ? 8 : 4;
}

template <int DD, int HP, typename KV>
void prefill_launch(const void* q, const void* k_cache, const void* v_cache, const int* block_tables, int max_blocks,
                    const int* tiles, int ntiles, const int* cu_q, const int* ctx_lens, void* out, int Hq, int Hkv,
                    float scale, int causal, float* lse, float k_scale, float v_scale, int xcd, int q_ld, int nwv,
                    hipStream_t st) {
  const int lds = 2 * PrefillCfg<DD>::BUF;
  if constexpr (DD == 64 || DD == 128) {
    if (nwv == 8) {  // the staggered loop keeps three tile slots
      auto kern = attn_prefill_kernel<DD, HP, KV, 1, false, 8>;
      set_max_lds(kern, 3 * PrefillCfg<DD>::BUF);
      kern<<<dim3(ntiles, Hq / HP), 512, 3 * PrefillCfg<DD>::BUF, st>>>((const bf16*)q, (const KV*)k_cache, (const KV*)v_cache,
                                                    block_tables, max_blocks, tiles, cu_q, ctx_lens, (bf16*)out, Hq,
                                                    Hkv, scale, causal, lse, k_scale, v_scale, xcd, q_ld);
      GAI_LAUNCH_CHECK();
      return;
    }
  }
  auto kern = attn_prefill_kernel<DD, HP, KV>;
  set_max_lds(kern, lds);
  kern<<<dim3(ntiles, Hq / HP), 256, lds, st>>>((const bf16*)q, (const KV*)k_cache, (const KV*)v_cache, block_tables,
                                                max_blocks, tiles, cu_q, ctx_lens, (bf16*)out, Hq, Hkv, scale, causal,
                                                lse, k_scale, v_scale, xcd, q_ld);
  GAI_LAUNCH_CHECK();
}
}  // namespace

void gai_attn_prefill(const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                      int max_blocks, const int* tiles, int ntiles, const int* cu_q, const int* ctx_lens, void* out,
                      int Hq, int Hkv, int D, float scale, int causal, float* lse, int kv_fp8, float k_scale,
                      float v_scale, hipStream_t st, int q_ld) {
  if (ntiles == 0) return;
  if (q_ld <= 0) q_ld = Hq * D;
  const int ratio = Hq / Hkv;
  const int hpw = ratio >= 4 ? 4 : ratio >= 2 ? 2 : 1;
  // XCD kv-head placement for causal decoder prefill at head_dim >= 128 (long K/V prefixes re-read by many q tiles).
  // Off for the head_dim-64 encoders (413 -> 394 TF/s with it) and for non-causal attention: config 4 (Mllama
  // cross-attention over the vision tokens) ran 6.69 -> 6.52 q/s with it (profiles/r3/attn_prefill_xcd).
  // GAI_ATTN_XCD=0 / 2: off / on everywhere.
  static const int xcd_env = getenv("GAI_ATTN_XCD") ? atoi(getenv("GAI_ATTN_XCD")) : 1;
  // wave priority 1 while a wave issues its QK^T / P.V MFMAs (0 in the softmax): +1-2 % on every head_dim-64/128 shape
  // (headline chunk 707-714 -> 721 TF/s, profiles/r5/attn_prefill/prio_ab.txt); GAI_ATTN_PRIO = 0 / 1 for A/B
  static const int prio_env = getenv("GAI_ATTN_PRIO") ? atoi(getenv("GAI_ATTN_PRIO")) : 2;
  static const bool exact_max = getenv("GAI_ATTN_RESCALE_TH") && atoi(getenv("GAI_ATTN_RESCALE_TH")) == 0;
  static const bool no_stagger = getenv("GAI_ATTN_STAGGER") && atoi(getenv("GAI_ATTN_STAGGER")) == 0;
  const int xcd = (xcd_env == 2 || (xcd_env == 1 && D >= 128 && causal)) | ((prio_env & 3) << 1) | (exact_max ? 8 : 0) |
                  (no_stagger ? 16 : 0);
  const int hl = prefill_hl(D, ratio);
  const int nwv = prefill_waves(D, ratio);
  if (hl == 2) {  // D == 128, hpw == 4: 64 rows per tile; + the 4 waves' Q images (2 heads x 32 rows each)
    const int lds = 2 * PrefillCfg<128>::BUF + 4 * 2 * 32 * PrefillCfg<128>::KRS;
    if (kv_fp8) {
      auto kern = attn_prefill_kernel<128, 4, fp8, 2>;
      set_max_lds(kern, lds);
      kern<<<dim3(ntiles, Hq / 4), 256, lds, st>>>((const bf16*)q, (const fp8*)k_cache, (const fp8*)v_cache,
                                                   block_tables, max_blocks, tiles, cu_q, ctx_lens, (bf16*)out, Hq,
                                                   Hkv, scale, causal, lse, k_scale, v_scale, xcd, q_ld);
    } else {
      auto kern = attn_prefill_kernel<128, 4, bf16, 2>;
      set_max_lds(kern, lds);
      kern<<<dim3(ntiles, Hq / 4), 256, lds, st>>>((const bf16*)q, (const bf16*)k_cache, (const bf16*)v_cache,
                                                   block_tables, max_blocks, tiles, cu_q, ctx_lens, (bf16*)out, Hq,
                                                   Hkv, scale, causal, lse, k_scale, v_scale, xcd, q_ld);
    }
    GAI_LAUNCH_CHECK();
    return;
  }
  // GAI_ATTN_PIPE = 1: the software-pipelined main loop (attn_prefill_kernel PIPE)
  static const int pipe_env = getenv("GAI_ATTN_PIPE") ? atoi(getenv("GAI_ATTN_PIPE")) : 0;
#define GAI_PF(DD, HP)                                                                                         \
  if (D == DD && hpw == HP && pipe_env == 1) {                                                                 \
    const int lds = 2 * PrefillCfg<DD>::BUF;                                                                   \
    if (kv_fp8) {                                                                                              \
      auto kern = attn_prefill_kernel<DD, HP, fp8, 1, true>;                                                   \
      set_max_lds(kern, lds);                                                                                  \
      kern<<<dim3(ntiles, Hq / HP), 256, lds, st>>>((const bf16*)q, (const fp8*)k_cache, (const fp8*)v_cache,  \
                                                    block_tables, max_blocks, tiles, cu_q, ctx_lens, (bf16*)out, \
                                                    Hq, Hkv, scale, causal, lse, k_scale, v_scale, xcd, q_ld); \
    } else {                                                                                                   \
      auto kern = attn_prefill_kernel<DD, HP, bf16, 1, true>;                                                  \
      set_max_lds(kern, lds);                                                                                  \
      kern<<<dim3(ntiles, Hq / HP), 256, lds, st>>>((const bf16*)q, (const bf16*)k_cache, (const bf16*)v_cache, \
                                                    block_tables, max_blocks, tiles, cu_q, ctx_lens, (bf16*)out, \
                                                    Hq, Hkv, scale, causal, lse, k_scale, v_scale, xcd, q_ld); \
    }                                                                                                          \
    GAI_LAUNCH_CHECK();                                                                                        \
    return;                                                                                                    \
  }                                                                                                            \
  if (D == DD && hpw == HP) {                                                                                  \
    if (kv_fp8)                                                                                                \
      prefill_launch<DD, HP, fp8>(q, k_cache, v_cache, block_tables, max_blocks, tiles, ntiles, cu_q, ctx_lens, \
                                  out, Hq, Hkv, scale, causal, lse, k_scale, v_scale, xcd, q_ld, nwv, st);     \
    else                                                                                                       \
      prefill_launch<DD, HP, bf16>(q, k_cache, v_cache, block_tables, max_blocks, tiles, ntiles, cu_q, ctx_lens, \
                                   out, Hq, Hkv, scale, causal, lse, k_scale, v_scale, xcd, q_ld, nwv, st);    \
    return;                                                                                                    \
  }
  GAI_PF(64, 1)
  GAI_PF(64, 2)
  GAI_PF(64, 4)
  GAI_PF(96, 1)  // Mllama vision encoder: head_dim 80 zero-padded to 96 (not 128): 25 % less MFMA work
  GAI_PF(96, 2)
  GAI_PF(96, 4)
  GAI_PF(128, 1)
  GAI_PF(128, 2)
  GAI_PF(128, 4)
  GAI_PF(256, 1)
  GAI_PF(256, 2)
  GAI_PF(256, 4)
#undef GAI_PF
  gai_launch_error(__FILE__, __LINE__, "attn_prefill: unsupported head_dim");
}

int gai_attn_prefill_rows_per_tile(int Hq, int Hkv, int D) {
  const int ratio = Hq / Hkv;
  const int hpw = ratio >= 4 ? 4 : ratio >= 2 ? 2 : 1;
  return 32 * (prefill_waves(D, ratio) / (hpw / prefill_hl(D, ratio)));
}

void gai_attn_decode(const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                     int max_blocks, const int* ctx_lens, void* out, float* ws_o, float* ws_ml, int B, int Hq,
                     int Hkv, int D, float scale, int split_keys, int max_splits, int kv_fp8, float k_scale,
                     float v_scale, hipStream_t st, int* split_cnt, const GaiQkvFold* fold) {
  if (B == 0) return;
  if (Hq / Hkv > 16) gai_launch_error(__FILE__, __LINE__, "attn_decode: GQA ratio > 16 unsupported");
  if (split_keys < 0 || split_keys % 128)
    gai_launch_error(__FILE__, __LINE__, "attn_decode: split_keys must be 0 (adaptive) or a multiple of 128");
  const dim3 grid(max_splits, Hkv, B);
  // GAI_DECODE_VARIANT: 0 = 8-B V^T pieces, 1 = 16-B V^T loads (default), 2 = 16-B + 64 keys per wave step,
  // 3 = 16-B + register double buffer (software pipelined)
  static const int variant = getenv("GAI_DECODE_VARIANT") ? atoi(getenv("GAI_DECODE_VARIANT")) : 1;
  // in-launch split merge (no attn_decode_reduce launch) when the caller passes the ticket counters
  const bool fuse = split_cnt != nullptr && max_splits > 1 && variant == 1;
  // non-temporal K / V loads in the fused bf16 kernel (GAI_DECODE_NT=0: plain loads). Llama-3-8B B = 64, ctx 2535
  // graph replay 7.84 -> 7.68 ms per step (profiles/r4/decode/decode_nt_split_ab.txt)
  static const bool ntl = !(getenv("GAI_DECODE_NT") && atoi(getenv("GAI_DECODE_NT")) == 0);
  if (fold != nullptr && !(fuse && ntl && !kv_fp8 && D == 128 && fold->ks >= 1 && fold->ks <= 16))
    gai_launch_error(__FILE__, __LINE__, "attn_decode: the folded QKV tail needs the fused non-temporal bf16 kernel");
  if (fold != nullptr) {
    attn_decode_kernel<128, false, 1, true, bf16, true, true, true><<<grid, 256, 0, st>>>(
        (const bf16*)q, (const bf16*)k_cache, (const bf16*)v_cache, block_tables, max_blocks, ctx_lens, (bf16*)out,
        ws_o, ws_ml, B, Hq, Hkv, scale, split_keys, max_splits, k_scale, v_scale, split_cnt, *fold);
    GAI_LAUNCH_CHECK();
    return;
  }
#define GAI_DEC(DD)                                                                                             \
  if (D == DD && fuse && ntl && !kv_fp8) {                                                                      \
    attn_decode_kernel<DD, false, 1, true, bf16, true, true><<<grid, 256, 0, st>>>(                             \
        (const bf16*)q, (const bf16*)k_cache, (const bf16*)v_cache, block_tables, max_blocks, ctx_lens,         \
        (bf16*)out, ws_o, ws_ml, B, Hq, Hkv, scale, split_keys, max_splits, k_scale, v_scale, split_cnt);       \
    GAI_LAUNCH_CHECK();                                                                                         \
    return;                                                                                                     \
  }                                                                                                             \
  if (D == DD && fuse) {                                                                                        \
    if (kv_fp8)                                                                                                 \
      attn_decode_kernel<DD, false, 1, true, fp8, true><<<grid, 256, 0, st>>>(                                  \
          (const bf16*)q, (const fp8*)k_cache, (const fp8*)v_cache, block_tables, max_blocks, ctx_lens,         \
          (bf16*)out, ws_o, ws_ml, B, Hq, Hkv, scale, split_keys, max_splits, k_scale, v_scale, split_cnt);     \
    else                                                                                                        \
      attn_decode_kernel<DD, false, 1, true, bf16, true><<<grid, 256, 0, st>>>(                                 \
          (const bf16*)q, (const bf16*)k_cache, (const bf16*)v_cache, block_tables, max_blocks, ctx_lens,       \
          (bf16*)out, ws_o, ws_ml, B, Hq, Hkv, scale, split_keys, max_splits, k_scale, v_scale, split_cnt);     \
    GAI_LAUNCH_CHECK();                                                                                         \
    return;                                                                                                     \
  }                                                                                                             \
  if (D == DD) {                                                                                                \
    if (kv_fp8) {                                                                                               \
      auto kern = variant == 2   ? attn_decode_kernel<DD, false, 2, true, fp8>                                  \
                  : variant == 3 ? attn_decode_kernel<DD, true, 1, true, fp8>                                   \
                                 : attn_decode_kernel<DD, false, 1, true, fp8>;                                 \
      kern<<<grid, 256, 0, st>>>((const bf16*)q, (const fp8*)k_cache, (const fp8*)v_cache, block_tables,        \
                                 max_blocks, ctx_lens, (bf16*)out, ws_o, ws_ml, B, Hq, Hkv, scale, split_keys,   \
                                 max_splits, k_scale, v_scale, nullptr, GaiQkvFold{});                           \
    } else {                                                                                                    \
      auto kern = variant == 0   ? attn_decode_kernel<DD, false, 1, false, bf16>                                \
                  : variant == 2 ? attn_decode_kernel<DD, false, 2, true, bf16>                                 \
                  : variant == 3 ? attn_decode_kernel<DD, true, 1, true, bf16>                                  \
                                 : attn_decode_kernel<DD, false, 1, true, bf16>;                                \
      kern<<<grid, 256, 0, st>>>((const bf16*)q, (const bf16*)k_cache, (const bf16*)v_cache, block_tables,      \
                                 max_blocks, ctx_lens, (bf16*)out, ws_o, ws_ml, B, Hq, Hkv, scale, split_keys,   \
                                 max_splits, k_scale, v_scale, nullptr, GaiQkvFold{});                           \
    }                                                                                                           \
    GAI_LAUNCH_CHECK();                                                                                         \
    if (max_splits > 1) {                                                                                       \
      attn_decode_reduce_kernel<DD><<<dim3(B, Hq), DD, 0, st>>>(ws_o, ws_ml, ctx_lens, (bf16*)out, B, Hq,       \
                                                                 split_keys, max_splits);                       \
      GAI_LAUNCH_CHECK();                                                                                       \
    }                                                                                                           \
    return;                                                                                                     \
  }
  GAI_DEC(64)
  GAI_DEC(128)
  GAI_DEC(256)
#undef GAI_DEC
  gai_launch_error(__FILE__, __LINE__, "attn_decode: unsupported head_dim");
}
