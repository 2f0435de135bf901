#pragma once
// bf16 GEMM on MFMA with fused epilogues (SURVEY K1, K8, K9 epilogues): kernel templates and launchers, included by
// gemm.hip (dispatch, stream-K workspace pool, prefill QKV + RoPE) and gemm_epi_*.hip (one translation unit per
// group of epilogues, so the build compiles the instantiations in parallel).
//
// C[M, N] = A[M, K] . B[N, K]^T  (torch Linear convention: weights are [out, in]).
//
// Two kernels, chosen by M:
//  * gemm_tiled  (M > 128, prefill / encoder): 128x128x64 block tile, 4 waves as
//    2x2, each wave 64x64 = 4x4 v_mfma_f32_16x16x32_bf16 tiles. Both operands are
//    staged global->LDS with global_load_lds_dwordx4 (16 B/lane, lane-linear LDS
//    image, XOR swizzle applied on the *source* address and on the ds_read side,
//    cdna_hip_programming §5 rule 21 / T2), double-buffered, one barrier per K
//    tile; XCD-aware bijective block remap + grouped-M raster for L2 reuse (T1).
//  * gemm_skinny (M <= 128, decode): the weight stream dominates. 8 waves per
//    workgroup split K eight ways *inside* the workgroup (no global split-K
//    slabs, no atomics); operands are loaded straight to VGPRs (decode GEMV row
//    of the glds-vs-register table); partials are reduced through LDS and the
//    epilogue writes coalesced rows.
// Epilogues: none | +bias | +bias,GELU | +bias,ReLU | +residual | SwiGLU (weights interleaved
// per 16 rows [gate16 | up16 | ...], output width N/2) | +bias+residual, bf16 or
// fp32 output (fp32 for LM-head logits).
#include "gai_common.h"
#include "gai_kernels.h"
#include "gai_epilogue.h"
#include "gai_rope.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

// every AGPR, for the asm-MFMA persistent kernels (w4p / w4d / w4r)
#define GAI_AGPR_CLOBBERS "a0","a1","a2","a3","a4","a5","a6","a7","a8","a9","a10","a11","a12","a13","a14","a15","a16","a17","a18","a19","a20","a21","a22","a23","a24","a25","a26","a27","a28","a29","a30","a31","a32","a33","a34","a35","a36","a37","a38","a39","a40","a41","a42","a43","a44","a45","a46","a47","a48","a49","a50","a51","a52","a53","a54","a55","a56","a57","a58","a59","a60","a61","a62","a63","a64","a65","a66","a67","a68","a69","a70","a71","a72","a73","a74","a75","a76","a77","a78","a79","a80","a81","a82","a83","a84","a85","a86","a87","a88","a89","a90","a91","a92","a93","a94","a95","a96","a97","a98","a99","a100","a101","a102","a103","a104","a105","a106","a107","a108","a109","a110","a111","a112","a113","a114","a115","a116","a117","a118","a119","a120","a121","a122","a123","a124","a125","a126","a127","a128","a129","a130","a131","a132","a133","a134","a135","a136","a137","a138","a139","a140","a141","a142","a143","a144","a145","a146","a147","a148","a149","a150","a151","a152","a153","a154","a155","a156","a157","a158","a159","a160","a161","a162","a163","a164","a165","a166","a167","a168","a169","a170","a171","a172","a173","a174","a175","a176","a177","a178","a179","a180","a181","a182","a183","a184","a185","a186","a187","a188","a189","a190","a191","a192","a193","a194","a195","a196","a197","a198","a199","a200","a201","a202","a203","a204","a205","a206","a207","a208","a209","a210","a211","a212","a213","a214","a215","a216","a217","a218","a219","a220","a221","a222","a223","a224","a225","a226","a227","a228","a229","a230","a231","a232","a233","a234","a235","a236","a237","a238","a239","a240","a241","a242","a243","a244","a245","a246","a247","a248","a249","a250","a251","a252","a253","a254","a255"
#define GAI_AGPR_ZERO "v_accvgpr_write_b32 a0, 0\n\t""v_accvgpr_write_b32 a1, 0\n\t""v_accvgpr_write_b32 a2, 0\n\t""v_accvgpr_write_b32 a3, 0\n\t""v_accvgpr_write_b32 a4, 0\n\t""v_accvgpr_write_b32 a5, 0\n\t""v_accvgpr_write_b32 a6, 0\n\t""v_accvgpr_write_b32 a7, 0\n\t""v_accvgpr_write_b32 a8, 0\n\t""v_accvgpr_write_b32 a9, 0\n\t""v_accvgpr_write_b32 a10, 0\n\t""v_accvgpr_write_b32 a11, 0\n\t""v_accvgpr_write_b32 a12, 0\n\t""v_accvgpr_write_b32 a13, 0\n\t""v_accvgpr_write_b32 a14, 0\n\t""v_accvgpr_write_b32 a15, 0\n\t""v_accvgpr_write_b32 a16, 0\n\t""v_accvgpr_write_b32 a17, 0\n\t""v_accvgpr_write_b32 a18, 0\n\t""v_accvgpr_write_b32 a19, 0\n\t""v_accvgpr_write_b32 a20, 0\n\t""v_accvgpr_write_b32 a21, 0\n\t""v_accvgpr_write_b32 a22, 0\n\t""v_accvgpr_write_b32 a23, 0\n\t""v_accvgpr_write_b32 a24, 0\n\t""v_accvgpr_write_b32 a25, 0\n\t""v_accvgpr_write_b32 a26, 0\n\t""v_accvgpr_write_b32 a27, 0\n\t""v_accvgpr_write_b32 a28, 0\n\t""v_accvgpr_write_b32 a29, 0\n\t""v_accvgpr_write_b32 a30, 0\n\t""v_accvgpr_write_b32 a31, 0\n\t""v_accvgpr_write_b32 a32, 0\n\t""v_accvgpr_write_b32 a33, 0\n\t""v_accvgpr_write_b32 a34, 0\n\t""v_accvgpr_write_b32 a35, 0\n\t""v_accvgpr_write_b32 a36, 0\n\t""v_accvgpr_write_b32 a37, 0\n\t""v_accvgpr_write_b32 a38, 0\n\t""v_accvgpr_write_b32 a39, 0\n\t""v_accvgpr_write_b32 a40, 0\n\t""v_accvgpr_write_b32 a41, 0\n\t""v_accvgpr_write_b32 a42, 0\n\t""v_accvgpr_write_b32 a43, 0\n\t""v_accvgpr_write_b32 a44, 0\n\t""v_accvgpr_write_b32 a45, 0\n\t""v_accvgpr_write_b32 a46, 0\n\t""v_accvgpr_write_b32 a47, 0\n\t""v_accvgpr_write_b32 a48, 0\n\t""v_accvgpr_write_b32 a49, 0\n\t""v_accvgpr_write_b32 a50, 0\n\t""v_accvgpr_write_b32 a51, 0\n\t""v_accvgpr_write_b32 a52, 0\n\t""v_accvgpr_write_b32 a53, 0\n\t""v_accvgpr_write_b32 a54, 0\n\t""v_accvgpr_write_b32 a55, 0\n\t""v_accvgpr_write_b32 a56, 0\n\t""v_accvgpr_write_b32 a57, 0\n\t""v_accvgpr_write_b32 a58, 0\n\t""v_accvgpr_write_b32 a59, 0\n\t""v_accvgpr_write_b32 a60, 0\n\t""v_accvgpr_write_b32 a61, 0\n\t""v_accvgpr_write_b32 a62, 0\n\t""v_accvgpr_write_b32 a63, 0\n\t""v_accvgpr_write_b32 a64, 0\n\t""v_accvgpr_write_b32 a65, 0\n\t""v_accvgpr_write_b32 a66, 0\n\t""v_accvgpr_write_b32 a67, 0\n\t""v_accvgpr_write_b32 a68, 0\n\t""v_accvgpr_write_b32 a69, 0\n\t""v_accvgpr_write_b32 a70, 0\n\t""v_accvgpr_write_b32 a71, 0\n\t""v_accvgpr_write_b32 a72, 0\n\t""v_accvgpr_write_b32 a73, 0\n\t""v_accvgpr_write_b32 a74, 0\n\t""v_accvgpr_write_b32 a75, 0\n\t""v_accvgpr_write_b32 a76, 0\n\t""v_accvgpr_write_b32 a77, 0\n\t""v_accvgpr_write_b32 a78, 0\n\t""v_accvgpr_write_b32 a79, 0\n\t""v_accvgpr_write_b32 a80, 0\n\t""v_accvgpr_write_b32 a81, 0\n\t""v_accvgpr_write_b32 a82, 0\n\t""v_accvgpr_write_b32 a83, 0\n\t""v_accvgpr_write_b32 a84, 0\n\t""v_accvgpr_write_b32 a85, 0\n\t""v_accvgpr_write_b32 a86, 0\n\t""v_accvgpr_write_b32 a87, 0\n\t""v_accvgpr_write_b32 a88, 0\n\t""v_accvgpr_write_b32 a89, 0\n\t""v_accvgpr_write_b32 a90, 0\n\t""v_accvgpr_write_b32 a91, 0\n\t""v_accvgpr_write_b32 a92, 0\n\t""v_accvgpr_write_b32 a93, 0\n\t""v_accvgpr_write_b32 a94, 0\n\t""v_accvgpr_write_b32 a95, 0\n\t""v_accvgpr_write_b32 a96, 0\n\t""v_accvgpr_write_b32 a97, 0\n\t""v_accvgpr_write_b32 a98, 0\n\t""v_accvgpr_write_b32 a99, 0\n\t""v_accvgpr_write_b32 a100, 0\n\t""v_accvgpr_write_b32 a101, 0\n\t""v_accvgpr_write_b32 a102, 0\n\t""v_accvgpr_write_b32 a103, 0\n\t""v_accvgpr_write_b32 a104, 0\n\t""v_accvgpr_write_b32 a105, 0\n\t""v_accvgpr_write_b32 a106, 0\n\t""v_accvgpr_write_b32 a107, 0\n\t""v_accvgpr_write_b32 a108, 0\n\t""v_accvgpr_write_b32 a109, 0\n\t""v_accvgpr_write_b32 a110, 0\n\t""v_accvgpr_write_b32 a111, 0\n\t""v_accvgpr_write_b32 a112, 0\n\t""v_accvgpr_write_b32 a113, 0\n\t""v_accvgpr_write_b32 a114, 0\n\t""v_accvgpr_write_b32 a115, 0\n\t""v_accvgpr_write_b32 a116, 0\n\t""v_accvgpr_write_b32 a117, 0\n\t""v_accvgpr_write_b32 a118, 0\n\t""v_accvgpr_write_b32 a119, 0\n\t""v_accvgpr_write_b32 a120, 0\n\t""v_accvgpr_write_b32 a121, 0\n\t""v_accvgpr_write_b32 a122, 0\n\t""v_accvgpr_write_b32 a123, 0\n\t""v_accvgpr_write_b32 a124, 0\n\t""v_accvgpr_write_b32 a125, 0\n\t""v_accvgpr_write_b32 a126, 0\n\t""v_accvgpr_write_b32 a127, 0\n\t""v_accvgpr_write_b32 a128, 0\n\t""v_accvgpr_write_b32 a129, 0\n\t""v_accvgpr_write_b32 a130, 0\n\t""v_accvgpr_write_b32 a131, 0\n\t""v_accvgpr_write_b32 a132, 0\n\t""v_accvgpr_write_b32 a133, 0\n\t""v_accvgpr_write_b32 a134, 0\n\t""v_accvgpr_write_b32 a135, 0\n\t""v_accvgpr_write_b32 a136, 0\n\t""v_accvgpr_write_b32 a137, 0\n\t""v_accvgpr_write_b32 a138, 0\n\t""v_accvgpr_write_b32 a139, 0\n\t""v_accvgpr_write_b32 a140, 0\n\t""v_accvgpr_write_b32 a141, 0\n\t""v_accvgpr_write_b32 a142, 0\n\t""v_accvgpr_write_b32 a143, 0\n\t""v_accvgpr_write_b32 a144, 0\n\t""v_accvgpr_write_b32 a145, 0\n\t""v_accvgpr_write_b32 a146, 0\n\t""v_accvgpr_write_b32 a147, 0\n\t""v_accvgpr_write_b32 a148, 0\n\t""v_accvgpr_write_b32 a149, 0\n\t""v_accvgpr_write_b32 a150, 0\n\t""v_accvgpr_write_b32 a151, 0\n\t""v_accvgpr_write_b32 a152, 0\n\t""v_accvgpr_write_b32 a153, 0\n\t""v_accvgpr_write_b32 a154, 0\n\t""v_accvgpr_write_b32 a155, 0\n\t""v_accvgpr_write_b32 a156, 0\n\t""v_accvgpr_write_b32 a157, 0\n\t""v_accvgpr_write_b32 a158, 0\n\t""v_accvgpr_write_b32 a159, 0\n\t""v_accvgpr_write_b32 a160, 0\n\t""v_accvgpr_write_b32 a161, 0\n\t""v_accvgpr_write_b32 a162, 0\n\t""v_accvgpr_write_b32 a163, 0\n\t""v_accvgpr_write_b32 a164, 0\n\t""v_accvgpr_write_b32 a165, 0\n\t""v_accvgpr_write_b32 a166, 0\n\t""v_accvgpr_write_b32 a167, 0\n\t""v_accvgpr_write_b32 a168, 0\n\t""v_accvgpr_write_b32 a169, 0\n\t""v_accvgpr_write_b32 a170, 0\n\t""v_accvgpr_write_b32 a171, 0\n\t""v_accvgpr_write_b32 a172, 0\n\t""v_accvgpr_write_b32 a173, 0\n\t""v_accvgpr_write_b32 a174, 0\n\t""v_accvgpr_write_b32 a175, 0\n\t""v_accvgpr_write_b32 a176, 0\n\t""v_accvgpr_write_b32 a177, 0\n\t""v_accvgpr_write_b32 a178, 0\n\t""v_accvgpr_write_b32 a179, 0\n\t""v_accvgpr_write_b32 a180, 0\n\t""v_accvgpr_write_b32 a181, 0\n\t""v_accvgpr_write_b32 a182, 0\n\t""v_accvgpr_write_b32 a183, 0\n\t""v_accvgpr_write_b32 a184, 0\n\t""v_accvgpr_write_b32 a185, 0\n\t""v_accvgpr_write_b32 a186, 0\n\t""v_accvgpr_write_b32 a187, 0\n\t""v_accvgpr_write_b32 a188, 0\n\t""v_accvgpr_write_b32 a189, 0\n\t""v_accvgpr_write_b32 a190, 0\n\t""v_accvgpr_write_b32 a191, 0\n\t""v_accvgpr_write_b32 a192, 0\n\t""v_accvgpr_write_b32 a193, 0\n\t""v_accvgpr_write_b32 a194, 0\n\t""v_accvgpr_write_b32 a195, 0\n\t""v_accvgpr_write_b32 a196, 0\n\t""v_accvgpr_write_b32 a197, 0\n\t""v_accvgpr_write_b32 a198, 0\n\t""v_accvgpr_write_b32 a199, 0\n\t""v_accvgpr_write_b32 a200, 0\n\t""v_accvgpr_write_b32 a201, 0\n\t""v_accvgpr_write_b32 a202, 0\n\t""v_accvgpr_write_b32 a203, 0\n\t""v_accvgpr_write_b32 a204, 0\n\t""v_accvgpr_write_b32 a205, 0\n\t""v_accvgpr_write_b32 a206, 0\n\t""v_accvgpr_write_b32 a207, 0\n\t""v_accvgpr_write_b32 a208, 0\n\t""v_accvgpr_write_b32 a209, 0\n\t""v_accvgpr_write_b32 a210, 0\n\t""v_accvgpr_write_b32 a211, 0\n\t""v_accvgpr_write_b32 a212, 0\n\t""v_accvgpr_write_b32 a213, 0\n\t""v_accvgpr_write_b32 a214, 0\n\t""v_accvgpr_write_b32 a215, 0\n\t""v_accvgpr_write_b32 a216, 0\n\t""v_accvgpr_write_b32 a217, 0\n\t""v_accvgpr_write_b32 a218, 0\n\t""v_accvgpr_write_b32 a219, 0\n\t""v_accvgpr_write_b32 a220, 0\n\t""v_accvgpr_write_b32 a221, 0\n\t""v_accvgpr_write_b32 a222, 0\n\t""v_accvgpr_write_b32 a223, 0\n\t""v_accvgpr_write_b32 a224, 0\n\t""v_accvgpr_write_b32 a225, 0\n\t""v_accvgpr_write_b32 a226, 0\n\t""v_accvgpr_write_b32 a227, 0\n\t""v_accvgpr_write_b32 a228, 0\n\t""v_accvgpr_write_b32 a229, 0\n\t""v_accvgpr_write_b32 a230, 0\n\t""v_accvgpr_write_b32 a231, 0\n\t""v_accvgpr_write_b32 a232, 0\n\t""v_accvgpr_write_b32 a233, 0\n\t""v_accvgpr_write_b32 a234, 0\n\t""v_accvgpr_write_b32 a235, 0\n\t""v_accvgpr_write_b32 a236, 0\n\t""v_accvgpr_write_b32 a237, 0\n\t""v_accvgpr_write_b32 a238, 0\n\t""v_accvgpr_write_b32 a239, 0\n\t""v_accvgpr_write_b32 a240, 0\n\t""v_accvgpr_write_b32 a241, 0\n\t""v_accvgpr_write_b32 a242, 0\n\t""v_accvgpr_write_b32 a243, 0\n\t""v_accvgpr_write_b32 a244, 0\n\t""v_accvgpr_write_b32 a245, 0\n\t""v_accvgpr_write_b32 a246, 0\n\t""v_accvgpr_write_b32 a247, 0\n\t""v_accvgpr_write_b32 a248, 0\n\t""v_accvgpr_write_b32 a249, 0\n\t""v_accvgpr_write_b32 a250, 0\n\t""v_accvgpr_write_b32 a251, 0\n\t""v_accvgpr_write_b32 a252, 0\n\t""v_accvgpr_write_b32 a253, 0\n\t""v_accvgpr_write_b32 a254, 0\n\t""v_accvgpr_write_b32 a255, 0\n\t"

using namespace gai;

namespace {

// ----------------------------------------------------------------------------------------------
// Tiled kernel
// ----------------------------------------------------------------------------------------------
constexpr int TBM = 128, TBN = 128, TBK = 64;
constexpr int kTileBytes = TBM * TBK * 2;  // 16 KiB per operand tile

__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, GAI_LDS(lds), 16, 0, 0);
}

template <int EPI, bool OUTF32>
__global__ __launch_bounds__(256, 2) void gemm_tiled_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                            void* C, const bf16* bias, const bf16* R, int M, int N,
                                                            int K, int ldc, int bfrag) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 x (A 16K + B 16K)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = (M + TBM - 1) / TBM, tiles_n = (N + TBN - 1) / TBN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 8;
  const int group = wg / (GM * tiles_n);
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int pin = wg % (GM * tiles_n);
  const int tm = first_m + pin % gsz, tn = pin / gsz;
  const int m0 = tm * TBM, n0 = tn * TBN;

  // per-lane staging source offsets (4 glds per operand per wave per K tile). bfrag: B is stored in MFMA fragment
  // order (ops.shuffle_fragments: [N/16][K/32][64 lanes][8]); load q of wave w is then the whole 1 KiB fragment
  // (n-tile (4w + q) / 2, k-half q & 1) of the K tile, and the LDS image is fragment-ordered too
  size_t a_off[4], b_off[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = (wid * 4 + q) * 64 + lane;
    const int row = p >> 3, cl = p & 7, cg = cl ^ (row & 7);
    a_off[q] = (size_t)min(m0 + row, M - 1) * K + cg * 8;
    const int f = wid * 4 + q;
    b_off[q] = bfrag ? ((size_t)min(n0 / 16 + (f >> 1), N / 16 - 1) * (K / 32) + (f & 1)) * 512 + lane * 8
                     : (size_t)min(n0 + row, N - 1) * K + cg * 8;
  }
  const size_t bk = bfrag ? 1024 : TBK;  // B elements per K tile
  auto stage = [&](int kt, int buf) {
    char* sa = smem + buf * 2 * kTileBytes;
    char* sb = sa + kTileBytes;
    const int k0 = kt * TBK;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      glds16(A + a_off[q] + k0, sa + (wid * 4 + q) * 1024);
      glds16(B + b_off[q] + kt * bk, sb + (wid * 4 + q) * 1024);
    }
  };

  const int wm = wid >> 1, wn = wid & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (bytes inside a tile) for k-step s: chunk c = 4s + (lane>>4)
  int a_rd[4][2], b_rd[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 4 * s + (lane >> 4);
      const int ra = wm * 64 + 16 * i + (lane & 15);
      const int rb = wn * 64 + 16 * i + (lane & 15);
      a_rd[i][s] = ra * 128 + ((c ^ (ra & 7)) << 4);
      b_rd[i][s] = bfrag ? ((wn * 4 + i) * 2 + s) * 1024 + lane * 16 : rb * 128 + ((c ^ (rb & 7)) << 4);
    }

  const int nk = K / TBK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const char* sa = smem + cur * 2 * kTileBytes;
    const char* sb = sa + kTileBytes;
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

  // epilogue: lane holds D[m = 4(lane>>4)+r][n = lane&15] of each 16x16 tile
  if (EPI == EPI_SWIGLU) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int nout = (n0 + wn * 64) / 2 + 16 * jp + (lane & 15);
        if (2 * nout >= N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
          if (m >= M) continue;
          const float g = acc[i][2 * jp][r], u = acc[i][2 * jp + 1][r];
          store_out<EPI_NONE, OUTF32>(C, nullptr, nullptr, ldc, m, nout, silu(g) * u);
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + 16 * j + (lane & 15);
        if (n >= N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 64 + 16 * i + 4 * (lane >> 4) + r;
          if (m < M) store_out<EPI, OUTF32>(C, bias, R, ldc, m, n, acc[i][j][r]);
        }
      }
  }
}

// ----------------------------------------------------------------------------------------------
// Shared tile geometry of the 256x256 prefill kernels. Round 1-2's stepping stones (the 8-wave 4-phase
// "large" kernel, the 8-wave unit ring and the non-persistent 4-wave ring, measured in profiles/r2/gemm_ring.jsonl
// and gemm_w4p*.jsonl) were superseded by the persistent kernels below and removed from the build.
// ----------------------------------------------------------------------------------------------
constexpr int LBM = 256, LBN = 256, LBK = 64;
constexpr int kHalfBytes = 256 * 32 * 2;  // one K-half of one operand

__device__ __forceinline__ int lswz(int r) { return (4 - ((r >> 2) & 3)) & 3; }

// ----------------------------------------------------------------------------------------------
// Unit ring of the persistent kernels: K is staged in 32-deep *units* (A 256x32 | B 256x32 = 32 KiB) through
// RNS = 5 LDS slots (160 KiB) by global_load_lds, 3-4 units ahead of their use; waits are counted (never a
// vmcnt(0) drain in the loop; cdna_hip_programming §5 "Pipelining across barriers").
//
// Operands are issued *swapped* (MFMA A = weight fragment, B = activation fragment), so each lane
// accumulates C[m][n .. n+3] - four consecutive output columns of one row - instead of one column
// of four rows. The epilogue then needs no LDS round trip: one v_permlane16_swap per fp32 value
// pairs lanes l / l+16 so every lane owns 8 consecutive columns, and each lane writes 16-byte
// stores (bias / GELU / residual / SwiGLU applied in fp32 on the way; one bf16 rounding).
//
// Measured on MI355X at M = 16384 (Llama-3-8B QKV / O / gate_up / down, random operands,
// profiles/r2/gemm_ring.jsonl): the 8-wave ring with this epilogue reached 1.27-1.39 PF/s; the persistent
// kernels below 1.55+ PF/s.
// ----------------------------------------------------------------------------------------------
constexpr int RNS = 5;                       // ring slots
constexpr int kUnitBytes = 2 * 256 * 32 * 2;  // A + B, 32 k
constexpr int kUnitHalf = 256 * 32 * 2;

__device__ __forceinline__ void swap16(float& lo, float& hi) {
  // lanes 16-31 of `lo` <-> lanes 0-15 of `hi` (and 48-63 <-> 32-47)
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
  lo = __uint_as_float(r[0]);
  hi = __uint_as_float(r[1]);
}

template <int EPI>
__device__ __forceinline__ float epi_act(float v, const bf16* bias, int n) {
  if (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RESIDUAL || EPI == EPI_BIAS_RELU ||
      EPI == EPI_BIAS_QUICKGELU)
    v += (float)bias[n];
  if (EPI == EPI_BIAS_GELU) v = gelu_erf(v);
  if (EPI == EPI_BIAS_RELU) v = fmaxf(v, 0.f);
  if (EPI == EPI_BIAS_QUICKGELU) v = quick_gelu(v);
  return v;
}

// epi_act with the bias value already loaded
template <int EPI>
__device__ __forceinline__ float epi_act_b(float v, float b) {
  if (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RESIDUAL || EPI == EPI_BIAS_RELU ||
      EPI == EPI_BIAS_QUICKGELU)
    v += b;
  if (EPI == EPI_BIAS_GELU) v = gelu_erf(v);
  if (EPI == EPI_BIAS_RELU) v = fmaxf(v, 0.f);
  if (EPI == EPI_BIAS_QUICKGELU) v = quick_gelu(v);
  return v;
}

// Epilogue of the swapped-operand 256x256 kernels, one 16-row group: lane holds C[m = mrow + (lane&15)]
// [n = nb + 16j + 4q + r] (q = lane>>4). Tile pairs (2jp, 2jp+1) are merged by one v_permlane16_swap
// per value so each lane owns 8 consecutive columns (16-byte stores); SwiGLU pairs are (gate, up).
template <int EPI, bool OUTF32, int NJ>
__device__ __forceinline__ void epilogue_rows(const f32x4 (&acc_i)[NJ], void* C, const bf16* bias, const bf16* R,
                                              int M, int N, int ldc, int mrow, int nb, int lane) {
  const int q = lane >> 4;
  const int m = mrow + (lane & 15);
  if (OUTF32) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = nb + 16 * j + 4 * q;
      if (m >= M || n >= N) continue;
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = epi_act<EPI>(acc_i[j][r], bias, n + r);
      if (EPI == EPI_RESIDUAL || EPI == EPI_BIAS_RESIDUAL) {
        const bf16x4 rv = *reinterpret_cast<const bf16x4*>(R + (size_t)m * ldc + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)rv[r];
      }
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(C) + (size_t)m * ldc + n) = v;
    }
    return;
  }
  if (EPI == EPI_SWIGLU) {
    // tiles (2jp, 2jp+1) = (gate, up) of output columns nb/2 + 16jp + 4q + r; pair jp = 2t, 2t+1
#pragma unroll
    for (int t = 0; t < NJ / 4; ++t) {
      float h0[4], h1[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        h0[r] = silu(acc_i[4 * t][r]) * acc_i[4 * t + 1][r];
        h1[r] = silu(acc_i[4 * t + 2][r]) * acc_i[4 * t + 3][r];
        swap16(h0[r], h1[r]);
      }
      const int n = nb / 2 + 32 * t + 16 * (q & 1) + 8 * (q >> 1);
      if (m < M && 2 * n < N) {
        bf16x8 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[r] = (bf16)h0[r];
          o[4 + r] = (bf16)h1[r];
        }
        store8(reinterpret_cast<bf16*>(C) + (size_t)m * ldc + n, o);
      }
    }
    return;
  }
  constexpr bool kBias = EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RESIDUAL || EPI == EPI_BIAS_RELU ||
                        EPI == EPI_BIAS_QUICKGELU;
#pragma unroll
  for (int jp = 0; jp < NJ / 2; ++jp) {
    float x0[4], x1[4];
    // the 4 columns a lane holds per tile are consecutive and N % 16 == 0 here: one 8-B bias load each
    bf16x4 b0 = {}, b1 = {};
    if constexpr (kBias) {
      b0 = *reinterpret_cast<const bf16x4*>(bias + min(nb + 32 * jp + 4 * q, N - 4));
      b1 = *reinterpret_cast<const bf16x4*>(bias + min(nb + 32 * jp + 16 + 4 * q, N - 4));
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      x0[r] = epi_act_b<EPI>(acc_i[2 * jp][r], (float)b0[r]);
      x1[r] = epi_act_b<EPI>(acc_i[2 * jp + 1][r], (float)b1[r]);
      swap16(x0[r], x1[r]);
    }
    // lanes q=0/2 now own tile 2jp columns 8(q>>1) .. +7; q=1/3 own tile 2jp+1
    const int n = nb + 32 * jp + 16 * (q & 1) + 8 * (q >> 1);
    if (m < M && n < N) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = x0[r];
        v[4 + r] = x1[r];
      }
      if (EPI == EPI_RESIDUAL || EPI == EPI_BIAS_RESIDUAL) {  // bf16(bf16(acc) + R): gai_epilogue.h store_out
        const bf16x8 rv = load8(R + (size_t)m * ldc + n);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (float)(bf16)v[e] + (float)rv[e];
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
      store8(reinterpret_cast<bf16*>(C) + (size_t)m * ldc + n, o);
    }
  }
}

template <int N, typename F, int... I>
__device__ __forceinline__ void for_each_const_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
// f(std::integral_constant<int, 0>) ... f(std::integral_constant<int, N-1>), fully unrolled
template <int N, typename F>
__device__ __forceinline__ void for_each_const(F&& f) {
  for_each_const_impl<N>(f, std::make_integer_sequence<int, N>{});
}

// AGPRs a[BASE .. BASE+3] -> v (the asm-MFMA kernel's accumulators)
template <int BASE>
__device__ __forceinline__ void read_acc_tile(f32x4& v) {
  float x0, x1, x2, x3;
  asm volatile(
      "v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
      "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
      : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
      : "i"(BASE), "i"(BASE + 1), "i"(BASE + 2), "i"(BASE + 3));
  v = f32x4{x0, x1, x2, x3};
}
// v -> AGPRs a[BASE .. BASE+3]
template <int BASE>
__device__ __forceinline__ void write_acc_tile(const f32x4& v) {
  asm volatile(
      "v_accvgpr_write_b32 a%c0, %4\n\tv_accvgpr_write_b32 a%c1, %5\n\t"
      "v_accvgpr_write_b32 a%c2, %6\n\tv_accvgpr_write_b32 a%c3, %7"
      :
      : "i"(BASE), "i"(BASE + 1), "i"(BASE + 2), "i"(BASE + 3), "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3])
      : GAI_AGPR_CLOBBERS);
}
template <int I, int... J>
__device__ __forceinline__ void read_acc_row(f32x4 (&row)[8], std::integer_sequence<int, J...>) {
  (read_acc_tile<4 * (8 * I + J)>(row[J]), ...);
}

// sched_group_barrier masks (LLVM SchedGroupMask): MFMA 0x8, VMEM 0x10, DS_READ 0x100
template <int N, int MASK>
__device__ __forceinline__ void sgb_pairs() {
  if constexpr (N > 0) {
    __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
    __builtin_amdgcn_sched_group_barrier(MASK, 1, 0);
    sgb_pairs<N - 1, MASK>();
  }
}

// ----------------------------------------------------------------------------------------------
// 4-wave ring kernel: the same 256x256 block tile and 5-slot ring, but 4 waves as 2 x 2, each owning
// a 128x128 output (8 x 8 MFMA 16x16x32 tiles, 256 accumulator registers in AGPRs: one wave per
// SIMD, 512-register budget). Per k32 unit a wave reads 16 fragments for 64 MFMAs (0.25 ds_read_b128
// per MFMA vs 0.375 for 8 waves of 128x64): 1/3 less LDS traffic and fewer LDS/SALU/VALU instructions
// per FLOP, which is what sets the clock of an MFMA-bound loop on random data (cdna_hip_programming
// §5.4 rule 28). One phase per unit: MFMAs on unit u's fragments (registers) interleaved with the
// ds_reads of unit u+1 and the 8 glds of unit u+5 into unit u's own slot (its fragments are already in
// registers); one barrier per phase.
// ----------------------------------------------------------------------------------------------
// ----------------------------------------------------------------------------------------------
// Persistent 4-wave ring kernel: the 4-wave tile (above), waves and phase, but one workgroup per CU
// walking tiles blockIdx.x, +G, +2G, ... with ONE unit ring running across its tiles. The last six
// phases of a tile prefetch units 0..4 of the workgroup's next tile, and the last one reads unit 0's
// fragments, so a tile's epilogue (AGPR reads + 16-B stores) runs while the next tile's operands are
// landing and its first MFMAs start right after it: no per-tile ring fill (the non-persistent kernel
// idles the matrix pipe ~4 phases per tile while units 0..4 load) and no launch tail between
// workgroup waves. Tile v of the walk goes through the same XCD remap (G % 8 == 0, so v % 8 is the
// XCD) and grouped raster: the 32 CUs of an XCD work on 32 neighbouring tiles at a time.
// ----------------------------------------------------------------------------------------------
// VAR (tools/microbench/gemm_w4p_ab.hip ablations only; 0 in the framework): bit 0 = no glds / vmcnt
// waits in the main loop, bit 1 = no barrier at phase ends, bit 2 = no fragment ds_reads in the loop,
// bit 3 = each glds covers 8 rows x 128 B (full lines; even units rows 0-127, odd 128-255: the request
// count of a k64 double-unit layout, wrong data)
template <int EPI, bool OUTF32, int VAR = 0>
__global__ __launch_bounds__(256, 1) void gemm_w4p_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                          void* C, const bf16* bias, const bf16* R, int M, int N,
                                                          int K, int ldc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // RNS slots x [A 16K | B 16K]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = (M + LBM - 1) / LBM, tiles_n = (N + LBN - 1) / LBN;
  const int tiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int n_my = (tiles - (int)blockIdx.x + G - 1) / G;
  auto coords = [&](int it, int& m0, int& n0) {
    const int wg = xcd_remap((int)blockIdx.x + it * G, tiles);
    constexpr int GM = 4;
    const int group = wg / (GM * tiles_n);
    const int first_m = group * GM;
    const int gsz = min(tiles_m - first_m, GM);
    const int pin = wg % (GM * tiles_n);
    m0 = (first_m + pin % gsz) * LBM;
    n0 = (pin / gsz) * LBN;
  };
  auto sources = [&](int m0, int n0, const bf16** as, const bf16** bs) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = VAR & 8 ? (wid * 4 + j) * 8 + (lane >> 3) : (wid * 4 + j) * 16 + (lane >> 2);
      const int cg = VAR & 8 ? (lane & 7) : (lane & 3) ^ lswz(row);
      as[j] = A + (size_t)min(m0 + row, M - 1) * K + cg * 8;
      bs[j] = B + (size_t)min(n0 + row, N - 1) * K + cg * 8;
    }
  };
  // source offset (elements) of k-unit ks
  auto koff = [&](int ks, int ld) -> size_t {
    return VAR & 8 ? (size_t)(ks & 1) * 128 * ld + (ks >> 1) * 64 : (size_t)ks * 32;
  };
  const int wm = wid >> 1, wn = wid & 1;
  const int rsw = (((lane >> 4) ^ lswz(lane & 15)) << 4);
  const int a_rd = (wm * 128 + (lane & 15)) * 64 + rsw;
  const int b_rd = kUnitHalf + (wn * 128 + (lane & 15)) * 64 + rsw;
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto phase_end = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);                  // lgkmcnt(0): next unit's fragments in registers
    if constexpr (!(VAR & 1)) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");  // unit u+2 landed
    if constexpr (!(VAR & 2)) barrier();
    else __builtin_amdgcn_sched_barrier(0);
  };
  // 64 MFMAs on (af, bfr); spread between them: the 8 glds of k-unit ks of (as, bs) into ring slot
  // g_slot and the 16 ds_reads of ring unit g_rd into (naf, nbf). g_* are walk-global unit numbers.
  auto phase = [&](const bf16x8* af, const bf16x8* bfr, bf16x8* naf, bf16x8* nbf, int g_rd, int g_slot,
                   const bf16* const* as, const bf16* const* bs, int ks) {
    char* d = smem + (g_slot % RNS) * kUnitBytes + wid * 4096;
    const char* sr = smem + (g_rd % RNS) * kUnitBytes;
    for_each_const<64>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int i = t >> 3, j = t & 7;
      asm volatile("v_mfma_f32_16x16x32_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
                   :
                   : "i"(4 * t), "i"(4 * t + 3), "v"(bfr[j]), "v"(af[i])
                   : GAI_AGPR_CLOBBERS);
      constexpr int g = (t - 5) / 8, r = t / 2;
      if constexpr (t % 8 == 5 && g < 4) {
        if constexpr (!(VAR & 1)) glds16(as[g] + koff(ks, K), d + g * 1024);
      } else if constexpr (t % 8 == 5) {
        if constexpr (!(VAR & 1)) glds16(bs[g - 4] + koff(ks, K), d + kUnitHalf + (g - 4) * 1024);
      } else if constexpr (t % 2 == 0 && t < 32 && r < 8) {
        if constexpr (!(VAR & 4)) naf[r] = *reinterpret_cast<const bf16x8*>(sr + a_rd + r * 1024);
      } else if constexpr (t % 2 == 0 && t < 32) {
        if constexpr (!(VAR & 4)) nbf[r - 8] = *reinterpret_cast<const bf16x8*>(sr + b_rd + (r - 8) * 1024);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  const int nu = K / 32;  // host guarantees nu even and nu >= 6
  int m0, n0;
  coords(0, m0, n0);
  const bf16 *ca[4], *cb[4], *xa[4], *xb[4];
  sources(m0, n0, ca, cb);
  asm volatile(GAI_AGPR_ZERO "s_nop 7\n\ts_nop 7\n" ::: GAI_AGPR_CLOBBERS);
#pragma unroll
  for (int u = 0; u < RNS; ++u) {
    char* dd = smem + u * kUnitBytes + wid * 4096;
#pragma unroll
    for (int j = 0; j < 4; ++j) glds16(ca[j] + u * 32, dd + j * 1024);
#pragma unroll
    for (int j = 0; j < 4; ++j) glds16(cb[j] + u * 32, dd + kUnitHalf + j * 1024);
  }
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");  // units 0 and 1 landed
  barrier();
  bf16x8 a0[8], b0[8], a1[8], b1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = *reinterpret_cast<const bf16x8*>(smem + a_rd + i * 1024);
#pragma unroll
  for (int j = 0; j < 8; ++j) b0[j] = *reinterpret_cast<const bf16x8*>(smem + b_rd + j * 1024);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  barrier();  // every wave has slot 0 in registers before phase 0 restages it

  for (int it = 0, gb = 0; it < n_my; ++it, gb += nu) {
    // the next tile's operand sources; past the last tile, dummy re-reads of this tile's first units
    // into slots no later phase reads (keeps every phase's glds / vmcnt count uniform)
    int nm0 = m0, nn0 = n0;
    if (it + 1 < n_my) coords(it + 1, nm0, nn0);
    sources(nm0, nn0, xa, xb);
    int u = 0;
    for (; u < nu - 6; u += 2) {
      phase(a0, b0, a1, b1, gb + u + 1, gb + u + RNS, ca, cb, u + RNS);
      phase_end();
      phase(a1, b1, a0, b0, gb + u + 2, gb + u + 1 + RNS, ca, cb, u + 1 + RNS);
      phase_end();
    }
    // u = nu - 6: the ring crosses into the next tile (this tile's unit nu-1, then next units 0..4)
    phase(a0, b0, a1, b1, gb + u + 1, gb + u + RNS, ca, cb, nu - 1);
    phase_end();
    phase(a1, b1, a0, b0, gb + u + 2, gb + u + 1 + RNS, xa, xb, 0);
    phase_end();
#pragma unroll
    for (int s = 1; s < 5; s += 2) {
      u += 2;
      phase(a0, b0, a1, b1, gb + u + 1, gb + u + RNS, xa, xb, s);
      phase_end();
      phase(a1, b1, a0, b0, gb + u + 2, gb + u + 1 + RNS, xa, xb, s + 1);
      phase_end();
    }
    // (a0, b0) now hold the next tile's unit-0 fragments; this tile's accumulators are complete
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // last MFMAs retire
    for_each_const<8>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      f32x4 row[8];
      read_acc_row<i>(row, std::make_integer_sequence<int, 8>{});
      epilogue_rows<EPI, OUTF32, 8>(row, C, bias, R, M, N, ldc, m0 + wm * 128 + 16 * i, n0 + wn * 128, lane);
    });
    asm volatile(GAI_AGPR_ZERO "s_nop 7\n\ts_nop 7\n" ::: GAI_AGPR_CLOBBERS);
    m0 = nm0;
    n0 = nn0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ca[j] = xa[j];
      cb[j] = xb[j];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
}

// ----------------------------------------------------------------------------------------------
// Persistent 4-wave kernel with full-line operand loads (the default prefill GEMM for K < 8192;
// gemm_w4r_kernel below differs only in its LDS ring): gemm_w4p_kernel's
// walk, waves and AGPR accumulators, but operands are staged in 64-deep *double units* (A 256 x 128 B |
// B 256 x 128 B = 64 KiB, two slots = 128 KiB LDS) so that each LDS-DMA load covers 8 whole 128-B rows:
// 8 lanes per line, one full-line L2 request per 8 lanes instead of two 64-B half-line requests. The
// ablation tools/microbench/gemm_w4p_ab.hip measured that request count as the limiter of the 32-deep
// ring (profiles/r2/gemm_w4p_ab.jsonl: same bytes in full-line requests +11-20 %, no operand loads at
// all +20-50 %). Loads are buffer_load ... lds at per-lane row offsets fixed per tile plus a scalar k
// offset (no 64-bit address arithmetic in the loop). LDS rows are 128 B; 16-B chunk c of row r is
// stored at position c ^ ((r >> 1) & 7), so each 16-lane ds_read_b128 group (16 rows, one chunk) hits
// 16 distinct bank groups.
// Schedule per double unit D (k32 units 2D, 2D+1; slot D & 1), fragments double-buffered in registers:
//   even phase (MFMA unit 2D, ds_read unit 2D+1), then vmcnt(0) + the one barrier: double D+1 landed,
//     every wave is done reading slot D;
//   odd phase (MFMA unit 2D+1, ds_read unit 2D+2 from slot D+1, and the 16 loads of double D+2 into
//     slot D, one after every 4th MFMA: a burst of LDS-DMA issues stalls the wave): 1-2 phases of
//     load latency cover.
// The last two odd phases of a tile load the next tile's doubles 0 and 1, so its epilogue overlaps them.
// ----------------------------------------------------------------------------------------------
constexpr int kDblBytes = 2 * 256 * 64 * 2;  // A + B, 64 k

// Prefill QKV epilogue (EPI_ROPE_KV, gemm_w4d_kernel only): (+ bias) -> bf16 -> RoPE -> q_out / paged K,
// V^T caches, exactly the rounding sequence of gemm + rope_kv_write, without the bf16 qkv round trip.
constexpr int EPI_ROPE_KV = 100;
struct RopeKvArgs {
  const int* pos = nullptr;
  const float* cos_sin = nullptr;
  const int* slots = nullptr;
  bf16* q_out = nullptr;
  bf16* k_cache = nullptr;
  bf16* v_cache = nullptr;
  int Hq = 0, Hkv = 0;
};
constexpr int kDblHalf = 256 * 64 * 2;

// VAR (microbench ablations only; 0 in the framework): bit 0 = the 16 loads issued in a burst over the
// odd phase's first 32 MFMAs (measured 3-9 % slower than 1 per 4 MFMAs: an LDS-DMA issue stalls the
// wave), bit 1 = no vmcnt wait at even phase ends (timing only)
//
// MI = 16-row A fragments per wave: 8 = the 256x256 tile; 6 = a 192x256 tile (each wave 96x128, 192 AGPRs,
// 48 MFMAs and 6 + 8 loads / fragment reads per phase). The launcher takes the tile height whose grid of tiles
// quantises best onto the CUs: a 2406-token prefill has 160 O / down tiles of 256 rows (one 62 %-full wave) but
// 208 of 192 rows (81 %, each 3/4 of the work).
template <int EPI, bool OUTF32, int VAR = 0, int MI = 8>
__global__ __launch_bounds__(256, 1) void gemm_w4d_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                          void* C, const bf16* bias, const bf16* R, int M, int N,
                                                          int K, int ldc, RopeKvArgs rk, int bfrag) {
  static_assert(MI == 8 || MI == 6, "tile heights 256 / 192");
  constexpr int BM = 32 * MI;       // tile rows
  constexpr int NT = 8 * MI;        // MFMAs per phase
  constexpr int NL = MI + 8;        // loads (odd phase) and fragment reads per phase
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 2 slots x [A 32K | B 32K] (A: BM rows used)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + LBN - 1) / LBN;
  const int tiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int n_my = (tiles - (int)blockIdx.x + G - 1) / G;
  auto coords = [&](int it, int& m0, int& n0) {
    const int wg = xcd_remap((int)blockIdx.x + it * G, tiles);
    constexpr int GM = 4;
    const int group = wg / (GM * tiles_n);
    const int first_m = group * GM;
    const int gsz = min(tiles_m - first_m, GM);
    const int pin = wg % (GM * tiles_n);
    m0 = (first_m + pin % gsz) * BM;
    n0 = (pin / gsz) * LBN;
  };
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(A), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(B), (short)0, 0x7fffffff, 0x00020000);
  // load j of wave w: A rows (MI w + j) * 8 + lane / 8 (j < MI), B rows (8w + j) * 8 + lane / 8 (j < 8), 16-B
  // chunk (lane & 7) of the LDS row <- global chunk (lane & 7) ^ f(row); byte offsets (rows clamped to the
  // matrix: partial tiles). bfrag (B in MFMA fragment order, ops.shuffle_fragments): B load j of wave w is the whole
  // 1 KiB fragment (n-tile 4w + j / 2, k32 half j & 1) of the double, landing fragment-ordered in LDS
  const int bks = bfrag ? 2048 : 128;  // B bytes per k-double step
  auto offsets = [&](int m0, int n0, int* oa, int* ob) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = (wid * 8 + j) * 8 + (lane >> 3);
      const int gc = (lane & 7) ^ ((row >> 1) & 7);
      ob[j] = bfrag ? (min(n0 / 16 + wid * 4 + (j >> 1), N / 16 - 1) * (K / 32) + (j & 1)) * 1024 + lane * 16
                    : min(n0 + row, N - 1) * K * 2 + gc * 16;
    }
#pragma unroll
    for (int j = 0; j < MI; ++j) {
      const int row = (wid * MI + j) * 8 + (lane >> 3);
      const int gc = (lane & 7) ^ ((row >> 1) & 7);
      oa[j] = min(m0 + row, M - 1) * K * 2 + gc * 16;
    }
  };
  const int wm = wid >> 1, wn = wid & 1;
  // fragment reads: row wm*BM/2 + 16i + (lane & 15) (f depends on lane & 15 only), chunk 4h + lane / 16
  const int fr = (lane & 15) >> 1;
  const int a_rd0 = (wm * 16 * MI + (lane & 15)) * 128 + (((lane >> 4) ^ fr) << 4);
  const int a_rd1 = (wm * 16 * MI + (lane & 15)) * 128 + (((4 + (lane >> 4)) ^ fr) << 4);
  const int b_rd0 = kDblHalf + (bfrag ? wn * 16384 + lane * 16 : (wn * 128 + (lane & 15)) * 128 + (((lane >> 4) ^ fr) << 4));
  const int b_rd1 = bfrag ? b_rd0 + 1024 : kDblHalf + (wn * 128 + (lane & 15)) * 128 + (((4 + (lane >> 4)) ^ fr) << 4);
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // one k32 phase: NT MFMAs on (af, bfr); the NL ds_reads of the next unit (half 1 of slot `rslot` in
  // an even phase, half 0 in an odd one) interleaved in the first 2 NL MFMAs and, in an odd phase, the NL
  // loads of k-double `kd` from (oa, ob) into slot `wslot` spread over all NT
  auto phase = [&](auto odd_c, const bf16x8* af, const bf16x8* bfr, bf16x8* naf, bf16x8* nbf, int rslot,
                   int wslot, const int* oa, const int* ob, int kd, auto rd_c) {
    constexpr bool ODD = decltype(odd_c)::value;
    constexpr bool RD = decltype(rd_c)::value;  // read the next unit's fragments (false: the caller reads them later)
    const char* sr = smem + rslot * kDblBytes;
    char* da = smem + wslot * kDblBytes + wid * MI * 1024;
    char* db = smem + wslot * kDblBytes + kDblHalf + wid * 8192;
    const int ar = ODD ? a_rd0 : a_rd1, br = ODD ? b_rd0 : b_rd1;
    const int soff = kd * 128, soffb = kd * bks;
    for_each_const<NT>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int i = t >> 3, j = t & 7;
      asm volatile("v_mfma_f32_16x16x32_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
                   :
                   : "i"(4 * t), "i"(4 * t + 3), "v"(bfr[j]), "v"(af[i])
                   : GAI_AGPR_CLOBBERS);
      constexpr int g = t >> 1;
      // load issue slots: 1 per 4 MFMAs at MI = 8 (the tuned schedule); NL spread evenly over NT otherwise
      constexpr bool LD = (VAR & 1) ? (t % 2 == 1 && t < 32)
                                    : (MI == 8 ? (t % 4 == 1) : ((t + 1) * NL / NT > t * NL / NT));
      constexpr int gl = (VAR & 1) ? g : (MI == 8 ? (t >> 2) : (t * NL / NT));  // load number 0..NL-1
      // (a load slot and a fragment-read slot may coincide at MI = 6: both issue)
      if constexpr (ODD && LD && gl < MI)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, GAI_LDS(da + gl * 1024), 16, oa[gl], soff, 0, 0);
      else if constexpr (ODD && LD)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, GAI_LDS(db + (gl - MI) * 1024), 16, ob[gl - MI], soffb, 0, 0);
      if constexpr (RD && t % 2 == 0 && g < NL && g < MI)
        naf[g] = *reinterpret_cast<const bf16x8*>(sr + ar + g * 2048);
      else if constexpr (RD && t % 2 == 0 && g < NL)
        nbf[g - MI] = *reinterpret_cast<const bf16x8*>(sr + br + (g - MI) * 2048);
      __builtin_amdgcn_sched_barrier(0);
    });
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): next unit's fragments in registers
    if constexpr (!ODD) {
      if constexpr (!(VAR & 2)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // double D+1 landed (this wave's share)
      barrier();                                         // ... and every wave's; slot D free
    }
  };
  using EvenT = std::integral_constant<bool, false>;
  using OddT = std::integral_constant<bool, true>;
  using RdT = std::integral_constant<bool, true>;
  // the RoPE / KV-write epilogue needs the registers of the next tile's first fragments: those are read after it
  using LastRdT = std::integral_constant<bool, EPI != EPI_ROPE_KV>;

  const int nd = K / 64;  // host guarantees K % 64 == 0, nd >= 2
  int m0, n0;
  coords(0, m0, n0);
  int ca[8], cb[8], xa[8], xb[8];  // A uses MI entries (an MI-sized local array here drops the host launch stub)
  offsets(m0, n0, ca, cb);
  asm volatile(GAI_AGPR_ZERO "s_nop 7\n\ts_nop 7\n" ::: GAI_AGPR_CLOBBERS);
#pragma unroll
  for (int dd = 0; dd < 2; ++dd) {
    char* dst = smem + dd * kDblBytes;
#pragma unroll
    for (int j = 0; j < MI; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, GAI_LDS(dst + (wid * MI + j) * 1024), 16, ca[j], dd * 128, 0, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, GAI_LDS(dst + kDblHalf + (wid * 8 + j) * 1024), 16, cb[j], dd * bks, 0, 0);
  }
  if constexpr (MI == 8)
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // double 0 landed
  else
    asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
  barrier();
  bf16x8 a0[MI], b0[8], a1[MI], b1[8];
#pragma unroll
  for (int i = 0; i < MI; ++i) a0[i] = *reinterpret_cast<const bf16x8*>(smem + a_rd0 + i * 2048);
#pragma unroll
  for (int j = 0; j < 8; ++j) b0[j] = *reinterpret_cast<const bf16x8*>(smem + b_rd0 + j * 2048);
  __builtin_amdgcn_s_waitcnt(0xC07F);

  for (int it = 0, gd = 0; it < n_my; ++it, gd += nd) {
    // next tile's sources; past the last tile, dummy re-loads of this tile's doubles 0 / 1 into a slot
    // no later phase reads
    int nm0 = m0, nn0 = n0;
    if (it + 1 < n_my) coords(it + 1, nm0, nn0);
    offsets(nm0, nn0, xa, xb);
    int D = 0;
    for (; D < nd - 2; ++D) {
      const int s = (gd + D) & 1;
      phase(EvenT{}, a0, b0, a1, b1, s, 0, ca, cb, 0, RdT{});
      phase(OddT{}, a1, b1, a0, b0, s ^ 1, s, ca, cb, D + 2, RdT{});
    }
    int last_rslot = 0;
    {
      const int s = (gd + D) & 1;
      phase(EvenT{}, a0, b0, a1, b1, s, 0, ca, cb, 0, RdT{});
      phase(OddT{}, a1, b1, a0, b0, s ^ 1, s, xa, xb, 0, RdT{});
      ++D;
    }
    {
      const int s = (gd + D) & 1;
      phase(EvenT{}, a0, b0, a1, b1, s, 0, ca, cb, 0, RdT{});
      phase(OddT{}, a1, b1, a0, b0, s ^ 1, s, xa, xb, 1, LastRdT{});
      last_rslot = s ^ 1;
      ++D;
    }
    // (a0, b0) hold the next tile's unit-0 fragments; this tile's accumulators are complete
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // last MFMAs retire
    // RoPE / KV-write epilogue: the wave's 128 columns are one head h of [Hq | Hkv | Hkv]; lane (m, q) holds dims
    // 16j + 4q + r (tile j) and, in tile j + 4, their rotate-half partners 64 further on. Every load is issued ahead
    // of the stores that would otherwise serialise it: each row group's position, slot and 8 cos / sin vectors are
    // loaded one or two groups early, before the earlier group's stores (vmcnt is in order and counts stores: a
    // load issued after a store waits for the store too). Per-call loads cost a load + store round trip per 4 columns:
    // QKV at M = 2406 112.8 vs 90.9 us for the plain GEMM (profiles/r5/c1_prefill_kernels_before_epi.csv). The
    // registers come from the next tile's first fragments, which this epilogue reads after it (LastRdT).
    // the lane id passes an opaque asm: nothing lane-dependent of this epilogue (64-bit store bases, offsets) is
    // hoisted out of the tile walk into registers the main loop needs (it spilled them, and the scratch reloads queued
    // behind the stores)
    int rk_lane = lane;
    asm volatile("" : "+v"(rk_lane));
    const int rk_nb = n0 + wn * 128, rk_h = rk_nb / 128, rk_q = rk_lane >> 4;
    const bool rk_rot = rk_h < rk.Hq + rk.Hkv;  // q and k heads are rotated, v heads only written
    const __amdgpu_buffer_rsrc_t rk_rq = __builtin_amdgcn_make_buffer_rsrc(rk.q_out, (short)0, 0x7fffffff, 0x00020000);
    int rk_pos[8], rk_slot[8];
    float4 rk_cs[2][8];
    auto rk_row = [&](int i) { return min(m0 + wm * 16 * MI + 16 * i + (rk_lane & 15), M - 1); };  // row of group i
    // buffer loads (uniform resource + 32-bit lane offset): no per-lane 64-bit bases for the compiler to hoist out
    // of the tile walk (they spilled at the kernel's 256-VGPR budget)
    const __amdgpu_buffer_rsrc_t rk_rcs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rk.cos_sin), (short)0,
                                                                             0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rk_rpos = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(rk.pos), (short)0,
                                                                              0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rk_rslot = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(rk.slots), (short)0,
                                                                               0x7fffffff, 0x00020000);
    auto rk_load_cs = [&](int i, float4* dst) {
      const int base = (rk_pos[i] * 128 + 4 * rk_q) * 4;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        dst[jj] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rk_rcs, base + 64 * jj, 0, 0));
        dst[4 + jj] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rk_rcs, base + 256 + 64 * jj, 0, 0));
      }
    };
    auto rk_ld_pos = [&](int i) { return (int)__builtin_amdgcn_raw_buffer_load_b32(rk_rpos, rk_row(i) * 4, 0, 0); };
    auto rk_ld_slot = [&](int i) { return (int)__builtin_amdgcn_raw_buffer_load_b32(rk_rslot, rk_row(i) * 4, 0, 0); };
    // positions two row groups ahead, slots one ahead (short live ranges: the epilogue holds 2 x 8 cos / sin vectors
    // and the kernel sits at its 256-VGPR budget)
    if constexpr (EPI == EPI_ROPE_KV) {
      rk_pos[0] = rk_ld_pos(0);
      if (MI > 1) rk_pos[1] = rk_ld_pos(1);
      rk_slot[0] = rk_ld_slot(0);
      if (rk_rot) rk_load_cs(0, rk_cs[0]);
    }
    for_each_const<MI>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (EPI == EPI_ROPE_KV) {  // issued before this group's stores
        if constexpr (i + 2 < MI) rk_pos[i + 2] = rk_ld_pos(i + 2);
        if constexpr (i + 1 < MI) {
          rk_slot[i + 1] = rk_ld_slot(i + 1);
          if (rk_rot) rk_load_cs(i + 1, rk_cs[(i + 1) & 1]);
        }
      }
      f32x4 row[8];
      read_acc_row<i>(row, std::make_integer_sequence<int, 8>{});
      if constexpr (EPI == EPI_ROPE_KV) {
        const int m = m0 + wm * 16 * MI + 16 * i + (rk_lane & 15);
        if (m < M && rk_nb < N) {
          const float4* cs = rk_cs[i & 1];
          const int slot = rk_slot[i];
          const int blk = slot / kKvBlock, off = slot % kKvBlock;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int i0 = 16 * jj + 4 * rk_q;
            bf16x4 x1, x2;
            if (bias) {  // Qwen-style QKV bias (uniform branch)
              const bf16x4 b1 = *reinterpret_cast<const bf16x4*>(bias + rk_nb + i0);
              const bf16x4 b2 = *reinterpret_cast<const bf16x4*>(bias + rk_nb + i0 + 64);
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                x1[r] = (bf16)(row[jj][r] + (float)b1[r]);
                x2[r] = (bf16)(row[jj + 4][r] + (float)b2[r]);
              }
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                x1[r] = (bf16)row[jj][r];
                x2[r] = (bf16)row[jj + 4][r];
              }
            }
            if (rk_rot) {  // the rounding of rope_kv_store: bf16 inputs, fp32 rotation, bf16 result
              const float cc[4] = {cs[jj].x, cs[jj].y, cs[jj].z, cs[jj].w};
              const float ss[4] = {cs[4 + jj].x, cs[4 + jj].y, cs[4 + jj].z, cs[4 + jj].w};
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float a = (float)x1[r], b = (float)x2[r];
                x1[r] = (bf16)(a * cc[r] - b * ss[r]);
                x2[r] = (bf16)(b * cc[r] + a * ss[r]);
              }
            }
            if (rk_h < rk.Hq) {  // q_out [M, Hq, 128] (< 2 GiB: 32-bit buffer offsets)
              const int qo = ((m * rk.Hq + rk_h) * 128 + i0) * 2;
              using u32x2 = __attribute__((ext_vector_type(2))) unsigned;
              __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, x1), rk_rq, qo, 0, 0);
              __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, x2), rk_rq, qo + 128, 0, 0);
            } else if (slot >= 0 && rk_rot) {
              bf16* dst = rk.k_cache + (((size_t)blk * rk.Hkv + (rk_h - rk.Hq)) * kKvBlock + off) * 128;
              *reinterpret_cast<bf16x4*>(dst + i0) = x1;
              *reinterpret_cast<bf16x4*>(dst + i0 + 64) = x2;
            } else if (slot >= 0) {
              bf16* dst = rk.v_cache + ((size_t)blk * rk.Hkv + (rk_h - rk.Hq - rk.Hkv)) * 128 * kKvBlock + off;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                dst[(size_t)(i0 + r) * kKvBlock] = x1[r];
                dst[(size_t)(i0 + 64 + r) * kKvBlock] = x2[r];
              }
            }
          }
        }
      } else {
        epilogue_rows<EPI, OUTF32, 8>(row, C, bias, R, M, N, ldc, m0 + wm * 16 * MI + 16 * i, n0 + wn * 128, lane);
      }
    });
    if constexpr (EPI == EPI_ROPE_KV) {  // the next tile's unit-0 fragments (the last phase skipped them)
      const char* sr = smem + last_rslot * kDblBytes;
#pragma unroll
      for (int g = 0; g < MI; ++g) a0[g] = *reinterpret_cast<const bf16x8*>(sr + a_rd0 + g * 2048);
#pragma unroll
      for (int g = 0; g < 8; ++g) b0[g] = *reinterpret_cast<const bf16x8*>(sr + b_rd0 + g * 2048);
    }
    asm volatile(GAI_AGPR_ZERO "s_nop 7\n\ts_nop 7\n" ::: GAI_AGPR_CLOBBERS);
    m0 = nm0;
    n0 = nn0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ca[j] = xa[j];
      cb[j] = xb[j];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
}

// ----------------------------------------------------------------------------------------------
// Part-ring variant of gemm_w4d_kernel (the default prefill GEMM for K >= 8192 or N >= 16384): the same full-line double units, but the A and B halves of a
// double are separate 32 KiB *parts* in a 5-part ring (160 KiB: all of the LDS), A(D), B(D), A(D+1), ...
// Part q lives in slot q % 5. The A part of double D+2 is loaded during the even phase 2D (into the
// slot B(D-1) left) and its B part during the odd phase 2D+1 (into the slot A(D) left), 8 loads per
// phase, one per 8 MFMAs: A gets 2-3 phases of latency cover, B 1-2 (w4d: 1-2 for both), one barrier
// per double as in w4d (even phase end, after vmcnt(8): double D+1 landed, A(D+2) may fly).
// M = 16384 (profiles/r2/gemm_w4p_ab.jsonl): 1.55-1.56 PF/s on O / down / gate_up; the longer A cover
// lifts the deep-K down projection (activations streamed from HBM) from 1.41 (w4d) to 1.56 PF/s.
//
// SK = true: the stream-K walk, for grids the 256x256 tiles fill badly (a 2406-token prefill has 160 O / down
// tiles for 256 CUs: one 62 %-full wave; gate_up 1120 tiles: 4.4 waves). The k-doubles of all tiles form one
// tile-major sequence of units; logical workgroup g (XCD-contiguous, so neighbouring runs share an L2) owns an
// equal run of unit pairs and walks it as *segments*, one per tile it touches, through the same ring (which
// runs on across segments as it runs across tiles in the tile walk). A tile covered by one segment takes the
// normal epilogue. A split tile's contributors hand fp32 partials over without ever waiting on each other
// (nothing assumes co-residency): each wave stores its 128x128 quadrant write-through (sc1) in fragment order,
// vmcnt(0), then draws one relaxed agent-scope ticket for (tile, wave); the wave that draws the last ticket
// sums the quadrants in contributor order - bitwise the same result whichever contributor finishes - and runs
// the epilogue. The tile's first contributor reaches it at the END of its run, after the others stored theirs
// at the start of theirs, so it first peeks the counter and usually sums without storing its own.
// Workspace [G][2 slots][4 waves][16384] fp32 (slot 0: a run's unaligned first segment, slot 1: a first
// contributor that was not last); counters [tiles][4], zero between launches (the last ticket resets its own).
//
// WALK = 2: the split walk. Stream-K's runs reach their tiles at unrelated k offsets, so the 32 workgroups of an XCD
// stop streaming one k-window through their shared L2 (O at M = 2406: 0.64 PF/s stream-K vs 1.0 tile walk). Here
// every tile is cut into S k-parts (even double counts) and the walk goes over the S x tiles items part-major,
// through the same XCD remap as the tile walk: the items a wave of workgroups runs together are neighbouring tiles
// at the SAME part, all starting at its first double, so they share their k-windows in L2 exactly as the tile walk
// does, while S x tiles items fill the grid's last wave far better (160 tiles, S = 3: 480 items = 94 % of two
// waves instead of 62 % of one). Every part stores its quadrants (slot = item) and draws the (tile, wave)
// ticket; the last one sums the S parts in part order.
// ----------------------------------------------------------------------------------------------
constexpr int kPart = 256 * 64 * 2;  // one operand of a double unit

constexpr int kSkQuad = 128 * 128;  // fp32 of one wave's quadrant partial

template <int EPI, bool OUTF32, int WALK = 0>
__global__ __launch_bounds__(256, 1) void gemm_w4r_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                          void* C, const bf16* bias, const bf16* R, int M, int N,
                                                          int K, int ldc, float* ws, int* cnt, int S, int bfrag) {
  constexpr bool SK = WALK == 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // 5 parts x 32 KiB
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = (M + LBM - 1) / LBM, tiles_n = (N + LBN - 1) / LBN;
  const int tiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int nd = K / 64;  // host guarantees K % 64 == 0, nd >= 2 (WALK 1 / 2: K % 128 == 0; WALK 2: S <= nd / 2)
  const int hp = nd / 2;
  const int items = WALK == 2 ? tiles * S : tiles;
  // walk positions: tile walk index it (tile blockIdx.x + it * G through the XCD remap), or SK unit index
  const long long P = (long long)tiles * (nd / 2);  // SK: unit pairs
  const int lg = SK ? xcd_remap((int)blockIdx.x, G) : 0;
  const int s_beg = SK ? 2 * (int)(lg * P / G) : 0;
  const int s_end = SK ? 2 * (int)((lg + 1) * P / G) : (items - (int)blockIdx.x + G - 1) / G;
  auto owner = [&](int pair) { return (int)(((pair + 1LL) * G - 1) / P); };  // SK: logical wg of a unit pair
  // position -> tile t (grouped-raster index), k-double range [kb, kb + len) (len even for WALK 1 / 2, >= 2) and
  // (WALK 2) the part pt
  auto segment = [&](int s, int& t, int& kb, int& len, int& pt) {
    if constexpr (SK) {
      t = s / nd;
      kb = s - t * nd;
      len = min(s_end, (t + 1) * nd) - s;
    } else if constexpr (WALK == 2) {
      const int item = xcd_remap((int)blockIdx.x + s * G, items);
      pt = item / tiles;
      t = item - pt * tiles;
      kb = 2 * ((pt * hp) / S);
      len = 2 * (((pt + 1) * hp) / S) - kb;
    } else {
      t = xcd_remap((int)blockIdx.x + s * G, tiles);
      kb = 0;
      len = nd;
    }
  };
  auto raster = [&](int t, int& m0, int& n0) {
    constexpr int GM = 4;
    const int group = t / (GM * tiles_n);
    const int first_m = group * GM;
    const int gsz = min(tiles_m - first_m, GM);
    const int pin = t % (GM * tiles_n);
    m0 = (first_m + pin % gsz) * LBM;
    n0 = (pin / gsz) * LBN;
  };
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(A), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(B), (short)0, 0x7fffffff, 0x00020000);
  // bfrag: B in MFMA fragment order (as gemm_w4d_kernel): B load j of wave w = fragment (n-tile 4w + j / 2, half j & 1)
  const int bks = bfrag ? 2048 : 128;  // B bytes per k-double step
  auto offsets = [&](int m0, int n0, int* oa, int* ob) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = (wid * 8 + j) * 8 + (lane >> 3);
      const int gc = (lane & 7) ^ ((row >> 1) & 7);
      oa[j] = min(m0 + row, M - 1) * K * 2 + gc * 16;
      ob[j] = bfrag ? (min(n0 / 16 + wid * 4 + (j >> 1), N / 16 - 1) * (K / 32) + (j & 1)) * 1024 + lane * 16
                    : min(n0 + row, N - 1) * K * 2 + gc * 16;
    }
  };
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = (lane & 15) >> 1;
  const int a_rd0 = (wm * 128 + (lane & 15)) * 128 + (((lane >> 4) ^ fr) << 4);
  const int a_rd1 = (wm * 128 + (lane & 15)) * 128 + (((4 + (lane >> 4)) ^ fr) << 4);
  const int b_rd0 = bfrag ? wn * 16384 + lane * 16 : (wn * 128 + (lane & 15)) * 128 + (((lane >> 4) ^ fr) << 4);
  const int b_rd1 = bfrag ? b_rd0 + 1024 : (wn * 128 + (lane & 15)) * 128 + (((4 + (lane >> 4)) ^ fr) << 4);
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // one k32 phase: 64 MFMAs on (af, bfr); the 16 ds_reads of the next unit (A part in slot sa, B part
  // in slot sb; half 1 in an even phase, half 0 in an odd one) in the first 32 MFMAs; the 8 loads of
  // one part of k-double kd (even: A from oa, odd: B from ob) into slot sw, one per 8 MFMAs
  auto phase = [&](auto odd_c, const bf16x8* af, const bf16x8* bfr, bf16x8* naf, bf16x8* nbf, int sa, int sb,
                   int sw, const int* o, int kd) {
    constexpr bool ODD = decltype(odd_c)::value;
    const char* pa = smem + sa * kPart + (ODD ? a_rd0 : a_rd1);
    const char* pb = smem + sb * kPart + (ODD ? b_rd0 : b_rd1);
    char* d = smem + sw * kPart + wid * 8192;
    const int soff = kd * (ODD ? bks : 128);
    for_each_const<64>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int i = t >> 3, j = t & 7;
      asm volatile("v_mfma_f32_16x16x32_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
                   :
                   : "i"(4 * t), "i"(4 * t + 3), "v"(bfr[j]), "v"(af[i])
                   : GAI_AGPR_CLOBBERS);
      constexpr int g = t >> 1, gl = t >> 3;
      if constexpr (t % 8 == 3)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ODD ? rb : ra, GAI_LDS(d + gl * 1024), 16, o[gl], soff, 0, 0);
      else if constexpr (t % 2 == 0 && t < 32 && g < 8)
        naf[g] = *reinterpret_cast<const bf16x8*>(pa + g * 2048);
      else if constexpr (t % 2 == 0 && t < 32)
        nbf[g - 8] = *reinterpret_cast<const bf16x8*>(pb + (g - 8) * 2048);
      __builtin_amdgcn_sched_barrier(0);
    });
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): next unit's fragments in registers
    if constexpr (!ODD) {
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // double D+1 landed (only A(D+2) in flight)
      barrier();
    }
  };
  using EvenT = std::integral_constant<bool, false>;
  using OddT = std::integral_constant<bool, true>;
  auto sl = [](int q) { return q % 5; };

  int s = s_beg;
  if (s >= s_end) return;  // (the host sizes the grid so that every run is non-empty)
  int t, kb, len, m0, n0, pt = 0;
  segment(s, t, kb, len, pt);
  raster(t, m0, n0);
  int ca[8], cb[8], xa[8], xb[8];
  offsets(m0, n0, ca, cb);
  asm volatile(GAI_AGPR_ZERO "s_nop 7\n\ts_nop 7\n" ::: GAI_AGPR_CLOBBERS);
#pragma unroll
  for (int q = 0; q < 4; ++q) {  // parts A(kb) B(kb) A(kb+1) B(kb+1) -> slots 0..3
    char* dst = smem + q * kPart + wid * 8192;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(q & 1 ? rb : ra, GAI_LDS(dst + j * 1024), 16, q & 1 ? cb[j] : ca[j],
                                               (kb + (q >> 1)) * (q & 1 ? bks : 128), 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // double kb landed
  barrier();
  bf16x8 a0[8], b0[8], a1[8], b1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = *reinterpret_cast<const bf16x8*>(smem + a_rd0 + i * 2048);
#pragma unroll
  for (int j = 0; j < 8; ++j) b0[j] = *reinterpret_cast<const bf16x8*>(smem + kPart + b_rd0 + j * 2048);
  __builtin_amdgcn_s_waitcnt(0xC07F);

  for (int gd = 0; s < s_end;) {
    // next segment's sources; past the last one, dummy re-loads of this segment's first double pair into a
    // slot no later phase reads
    const int sn = SK ? s + len : s + 1;
    int tn = t, kbn = kb, lenn = len, nm0 = m0, nn0 = n0, ptn = pt;
    if (sn < s_end) {
      segment(sn, tn, kbn, lenn, ptn);
      raster(tn, nm0, nn0);
    }
    offsets(nm0, nn0, xa, xb);
    int D = 0;
    for (; D < len - 2; ++D) {
      const int q = 2 * (gd + D);
      phase(EvenT{}, a0, b0, a1, b1, sl(q), sl(q + 1), sl(q + 4), ca, kb + D + 2);
      phase(OddT{}, a1, b1, a0, b0, sl(q + 2), sl(q + 3), sl(q + 5), cb, kb + D + 2);
    }
#pragma unroll
    for (int e = 0; e < 2; ++e, ++D) {
      const int q = 2 * (gd + D);
      phase(EvenT{}, a0, b0, a1, b1, sl(q), sl(q + 1), sl(q + 4), xa, kbn + e);
      phase(OddT{}, a1, b1, a0, b0, sl(q + 2), sl(q + 3), sl(q + 5), xb, kbn + e);
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // last MFMAs retire
    bool epi = true;
    if constexpr (WALK != 0) {
      if (SK ? (kb != 0 || len != nd) : S > 1) {  // split tile: hand the partial over, or (last ticket) sum them
        // contributors cf..cl (stream-K: logical workgroups, this one = lg; split: the parts, this one = pt)
        const int cf = SK ? owner(t * hp) : 0, cl = SK ? owner(t * hp + hp - 1) : S - 1;
        const int me = SK ? lg : pt;
        int* ctr = cnt + t * 4 + wid;
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(ws, (short)0, 0x7fffffff, 0x00020000);
        // (contributor c, this wave, fragment ij) -> scalar byte offset; the lane's 16 B is the one voffset.
        // Quadrant slot: stream-K [workgroup][first-contributor?], split [part][tile]
        const unsigned vo = lane * 16;
        auto woff = [&](int c, int ij) {
          const int q = SK ? c * 2 + (c == cf ? 1 : 0) : c * tiles + t;
          return (unsigned)__builtin_amdgcn_readfirstlane((q * 4 + wid) * (kSkQuad * 4) + ij * 1024);
        };
        bool last = false, stored = false;
        if (SK && kb == 0)  // stream-K first contributor: everyone else (who started their runs here) is usually done
          last = __builtin_amdgcn_readfirstlane(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ==
                 cl - cf;
        if (!last) {
          for_each_const<8>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            f32x4 row[8];
            read_acc_row<i>(row, std::make_integer_sequence<int, 8>{});
#pragma unroll
            for (int j = 0; j < 8; ++j)
              __builtin_amdgcn_raw_buffer_store_b128(
                  __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, row[j]), rw,
                  vo, woff(me, i * 8 + j), 16);
          });
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through partial has landed
          stored = true;
          int tk = 0;
          if (lane == 0) tk = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          last = __builtin_amdgcn_readfirstlane(tk) == cl - cf;
        }
        if (last) {
          if (lane == 0) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
          // sum in contributor order into the AGPRs: after a successful peek they hold the first term (this wave's
          // own, never stored); after the last ticket every partial, this wave's included, is in the workspace
          int c0 = cf + 1;
          if (stored) {
            asm volatile(GAI_AGPR_ZERO "s_nop 7\n\ts_nop 7\n" ::: GAI_AGPR_CLOBBERS);
            c0 = cf;
          }
          // 16-fragment batches; the next batch's 16 loads are in flight while one is added (a serial walk pays one
          // memory latency per few fragments: measured 0.62 vs 1.0 PF/s for the whole GEMM)
          f32x4 bufa[16], bufb[16];
          auto load_batch = [&](int c, int b, f32x4 (&buf)[16]) {
#pragma unroll
            for (int j = 0; j < 16; ++j)
              buf[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, vo, woff(c, 16 * b + j), 16));
          };
          auto add_batch = [&](auto bc, const f32x4 (&buf)[16]) {
            constexpr int b = decltype(bc)::value;
            for_each_const<16>([&](auto jc) {
              constexpr int j = decltype(jc)::value;
              f32x4 v;
              read_acc_tile<4 * (16 * b + j)>(v);
              v += buf[j];
              write_acc_tile<4 * (16 * b + j)>(v);
            });
          };
          if (c0 <= cl) {
            load_batch(c0, 0, bufa);
            for (int c = c0; c <= cl; ++c) {
              load_batch(c, 1, bufb);
              add_batch(std::integral_constant<int, 0>{}, bufa);
              load_batch(c, 2, bufa);
              add_batch(std::integral_constant<int, 1>{}, bufb);
              load_batch(c, 3, bufb);
              add_batch(std::integral_constant<int, 2>{}, bufa);
              if (c < cl) load_batch(c + 1, 0, bufa);
              add_batch(std::integral_constant<int, 3>{}, bufb);
            }
          }
          asm volatile("s_nop 7" ::: "memory");
        }
        epi = last;
      }
    }
    if (epi) {
      for_each_const<8>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        f32x4 row[8];
        read_acc_row<i>(row, std::make_integer_sequence<int, 8>{});
        epilogue_rows<EPI, OUTF32, 8>(row, C, bias, R, M, N, ldc, m0 + wm * 128 + 16 * i, n0 + wn * 128, lane);
      });
    }
    asm volatile(GAI_AGPR_ZERO "s_nop 7\n\ts_nop 7\n" ::: GAI_AGPR_CLOBBERS);
    gd += len;
    s = sn;
    t = tn;
    kb = kbn;
    len = lenn;
    pt = ptn;
    m0 = nm0;
    n0 = nn0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ca[j] = xa[j];
      cb[j] = xb[j];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
}

// ----------------------------------------------------------------------------------------------
// Skinny kernel (decode): 8 waves split K inside the workgroup
// ----------------------------------------------------------------------------------------------
template <int MT, int NF, int EPI, bool OUTF32>
__global__ __launch_bounds__(512) void gemm_skinny_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                          void* C, const bf16* bias, const bf16* R, int M, int N,
                                                          int K, int ldc, int bfrag) {
  constexpr int NB = 16 * NF;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* part = reinterpret_cast<float*>(smem);  // [8 waves][MT][NF][4][64 lanes]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nb = xcd_remap(blockIdx.x, gridDim.x);
  const int n0 = nb * NB;
  const int KS = K / 8;
  const int kbeg = wid * KS, kend = kbeg + KS;

  // bfrag: B in MFMA fragment order, the lane's 16 B of fragment (n-tile, k32 step) = 1 KiB per step
  const bf16* bp[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f)
    bp[f] = bfrag ? B + (size_t)min(n0 / 16 + f, N / 16 - 1) * (K / 32) * 512 + 8 * lane
                  : B + (size_t)min(n0 + 16 * f + (lane & 15), N - 1) * K + 8 * (lane >> 4);
  const int kmul = bfrag ? 16 : 1;
  const bf16* ap[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) ap[i] = A + (size_t)min(16 * i + (lane & 15), M - 1) * K + 8 * (lane >> 4);

  f32x4 acc[MT][NF];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 4
  for (int k = kbeg; k < kend; k += 32) {
    bf16x8 bfr[NF], af[MT];
#pragma unroll
    for (int f = 0; f < NF; ++f) bfr[f] = load8(bp[f] + (size_t)k * kmul);
#pragma unroll
    for (int i = 0; i < MT; ++i) af[i] = load8(ap[i] + k);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int f = 0; f < NF; ++f) acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[f], acc[i][f], 0, 0, 0);
  }

#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[(((wid * MT + i) * NF + f) * 4 + r) * 64 + lane] = acc[i][f][r];
  __syncthreads();

  // element (m, n): i = m>>4, r = m&3, lane = ((m&15)>>2)*16 + (n&15), f = n>>4
  if (EPI == EPI_SWIGLU) {
    constexpr int NO = NB / 2;
    for (int e = tid; e < M * NO; e += 512) {
      const int m = e / NO, no = e % NO;
      const int fp = no >> 4, c = no & 15;
      const int i = m >> 4, r = m & 3, l = ((m & 15) >> 2) * 16 + c;
      float g = 0.f, u = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        g += part[(((w * MT + i) * NF + 2 * fp) * 4 + r) * 64 + l];
        u += part[(((w * MT + i) * NF + 2 * fp + 1) * 4 + r) * 64 + l];
      }
      const int nout = n0 / 2 + no;
      if (2 * nout < N) store_out<EPI_NONE, OUTF32>(C, nullptr, nullptr, ldc, m, nout, silu(g) * u);
    }
  } else {
    for (int e = tid; e < M * NB; e += 512) {
      const int m = e / NB, nn = e % NB;
      const int n = n0 + nn;
      if (n >= N) continue;
      const int i = m >> 4, r = m & 3, f = nn >> 4, l = ((m & 15) >> 2) * 16 + (nn & 15);
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += part[(((w * MT + i) * NF + f) * 4 + r) * 64 + l];
      store_out<EPI, OUTF32>(C, bias, R, ldc, m, n, v);
    }
  }
}

template <typename F>
void set_max_lds(F* f) {
  hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <int EPI, bool OUTF32>
void launch_tiled(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
                  hipStream_t st, int bfrag) {
  const int tiles = ((M + TBM - 1) / TBM) * ((N + TBN - 1) / TBN);
  static bool once = false;
  if (!once) {
    set_max_lds(gemm_tiled_kernel<EPI, OUTF32>);
    once = true;
  }
  gemm_tiled_kernel<EPI, OUTF32><<<tiles, 256, 4 * kTileBytes, st>>>((const bf16*)A, (const bf16*)B, C,
                                                                      (const bf16*)bias, (const bf16*)R, M, N, K, ldc, bfrag);
  GAI_LAUNCH_CHECK();
}

template <int EPI, bool OUTF32>
void launch_w4p(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
                hipStream_t st) {
  const int tiles = ((M + LBM - 1) / LBM) * ((N + LBN - 1) / LBN);
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 8)
      gai_launch_error(__FILE__, __LINE__, "gemm_w4p: cannot query the CU count");
    set_max_lds(gemm_w4p_kernel<EPI, OUTF32>);
  }
  // one workgroup per CU (160 KiB LDS each), a multiple of 8 so that walk index % 8 stays the XCD
  const int grid = tiles <= ncu ? tiles : (ncu & ~7);
  gemm_w4p_kernel<EPI, OUTF32><<<grid, 256, RNS * kUnitBytes, st>>>((const bf16*)A, (const bf16*)B, C,
                                                                    (const bf16*)bias, (const bf16*)R, M, N, K, ldc);
  GAI_LAUNCH_CHECK();
}

// Tile height of the w4d walk: 192 rows when its tiles quantise onto the CUs' waves enough better to pay for the
// smaller tile's lower rate (15 % per FLOP: M = 16384 QKV / O / gate_up 645 / 406 / 3096 us vs 559 / 358 / 2634 on
// 256-row tiles): cost = waves x rows. M = 2406, N = 4096 (O / down): 10 x 16 = 160 tiles of 256 rows (1 wave x 256)
// vs 13 x 16 = 208 of 192 (1 x 192): O 77.9 -> 66.7 us, down 255.1 -> 225.8 us with cache-resident operands
// (profiles/r5/gemm/w4d192.jsonl). QKV (N 6144: 240 tiles vs 312 = 2 waves) and gate_up (1120 vs 1456 tiles: 5 x 256
// vs 6 x 192) keep 256 rows; M = 16384 keeps 256. GAI_GEMM_BM = 192 / 256 forces one.
int w4d_rows(int M, int N, int ncu) {
  // opt-in (GAI_GEMM_BM=0 selects by the model below): with HBM-streamed operands the 192-row tile's shorter latency
  // cover (3 phases of 48 MFMAs) loses more than the better wave quantisation gains (cold M = 2406 down 291.4 us vs
  // 293.3 on 256 rows and 251.8 on the part ring, profiles/r5/gemm/cold_m2406_16384.jsonl)
  static const int env = getenv("GAI_GEMM_BM") ? atoi(getenv("GAI_GEMM_BM")) : 256;
  if (env == 192 || env == 256) return env;
  const int G = ncu & ~7, tn = (N + LBN - 1) / LBN;
  auto cost = [&](int bm) { return (double)((((M + bm - 1) / bm) * tn + G - 1) / G) * bm; };
  return cost(192) * 1.15 < cost(256) ? 192 : 256;
}

template <int EPI, bool OUTF32>
void launch_w4d(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
                hipStream_t st, RopeKvArgs rk, int rows, int bfrag) {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 8)
      gai_launch_error(__FILE__, __LINE__, "gemm_w4d: cannot query the CU count");
    set_max_lds(gemm_w4d_kernel<EPI, OUTF32>);
    set_max_lds(gemm_w4d_kernel<EPI, OUTF32, 0, 6>);
  }
  const int bm = rows ? rows : w4d_rows(M, N, ncu);
  const int tiles = ((M + bm - 1) / bm) * ((N + LBN - 1) / LBN);
  const int grid = tiles <= ncu ? tiles : (ncu & ~7);
  if (bm == 192)
    gemm_w4d_kernel<EPI, OUTF32, 0, 6><<<grid, 256, 2 * kDblBytes, st>>>((const bf16*)A, (const bf16*)B, C,
                                                                        (const bf16*)bias, (const bf16*)R, M, N, K,
                                                                        ldc, rk, bfrag);
  else
    gemm_w4d_kernel<EPI, OUTF32><<<grid, 256, 2 * kDblBytes, st>>>((const bf16*)A, (const bf16*)B, C,
                                                                   (const bf16*)bias, (const bf16*)R, M, N, K, ldc, rk,
                                                                   bfrag);
  GAI_LAUNCH_CHECK();
}

template <int EPI, bool OUTF32>
void launch_w4r(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
                hipStream_t st, int bfrag) {
  const int tiles = ((M + LBM - 1) / LBM) * ((N + LBN - 1) / LBN);
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 8)
      gai_launch_error(__FILE__, __LINE__, "gemm_w4r: cannot query the CU count");
    set_max_lds(gemm_w4r_kernel<EPI, OUTF32>);
  }
  const int grid = tiles <= ncu ? tiles : (ncu & ~7);
  gemm_w4r_kernel<EPI, OUTF32><<<grid, 256, 5 * kPart, st>>>((const bf16*)A, (const bf16*)B, C, (const bf16*)bias,
                                                             (const bf16*)R, M, N, K, ldc, nullptr, nullptr, 1, bfrag);
  GAI_LAUNCH_CHECK();
}

// Stream-K workspace of one (device, stream): partial quadrants [G][2][4][16384] fp32 and per-(tile, wave)
// tickets (gemm.hip owns the one pool every translation unit shares). Two streams never share one (their launches
// could overlap). Grown outside graph capture only; a captured launch that would need a bigger one takes the tile
// walk instead.
struct SkWorkspace {
  float* ws = nullptr;
  int* cnt = nullptr;
  size_t ws_bytes = 0, cnt_n = 0;
};
}  // namespace
bool gai_sk_workspace(hipStream_t st, size_t ws_bytes, size_t cnt_n, float** ws, int** cnt);
namespace {
bool sk_workspace(hipStream_t st, size_t ws_bytes, size_t cnt_n, SkWorkspace& out) {
  return gai_sk_workspace(st, ws_bytes, cnt_n, &out.ws, &out.cnt);
}

int sk_grid() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 8)
      gai_launch_error(__FILE__, __LINE__, "gemm_w4s: cannot query the CU count");
  }
  return ncu & ~7;
}

int ring_tiles(int M, int N) { return ((M + LBM - 1) / LBM) * ((N + LBN - 1) / LBN); }

// Auto policy of the 256x256 kernels (profiles/r4/gemm_policy: Llama-3-8B projections at M = 512 / 1024 / 2406,
// interleaved rounds against the 128x128 tiled kernel):
//  * tile walk when its tiles fill at least half of the grid (M = 2406: 160-1120 tiles, 1.0-1.3 PF/s vs 0.8-0.95
//    tiled; M = 512 gate_up: 224 tiles, 1.29 vs 0.87 PF/s);
//  * stream-K walk when they do not and K is deep (down at M = 512 / 1024: 32 / 64 tiles, 0.79 / 1.15 PF/s vs
//    0.40 / 0.74 tiled, 0.26 / 0.51 tile walk); at K = 4096 the tiled kernel wins there (O at M = 1024: 0.72 vs
//    0.66 stream-K);
//  * never stream-K just to fill the last wave of a well-filled walk: its runs reach the tiles at unrelated k
//    offsets, so the 32 workgroups of an XCD no longer stream the same k-window through their L2 (O at M = 2406:
//    0.64 PF/s stream-K vs 1.0 tile walk, although the walk leaves 38 % of the CUs idle).
bool sk_auto(int M, int N, int K) { return K >= 8192 && K % 128 == 0 && 2 * ring_tiles(M, N) < sk_grid(); }
bool ring_auto(int M, int N, int K) { return M >= 256 && (2 * ring_tiles(M, N) >= sk_grid() || sk_auto(M, N, K)); }

template <int EPI, bool OUTF32>
bool launch_w4s(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
                hipStream_t st, int bfrag) {
  if (K % 128) return false;
  static bool once = false;
  if (!once) {
    set_max_lds(gemm_w4r_kernel<EPI, OUTF32, 1>);
    once = true;
  }
  const int tiles = ((M + LBM - 1) / LBM) * ((N + LBN - 1) / LBN);
  const long long pairs = (long long)tiles * (K / 128);
  // every run non-empty (pairs >= G); a multiple of 8 keeps the logical -> XCD map contiguous
  const int grid = (int)std::min<long long>(sk_grid(), pairs) & ~7;
  if (grid < 8) return false;
  SkWorkspace w;
  if (!sk_workspace(st, (size_t)grid * 2 * 4 * kSkQuad * sizeof(float), (size_t)tiles * 4, w)) return false;
  gemm_w4r_kernel<EPI, OUTF32, 1><<<grid, 256, 5 * kPart, st>>>((const bf16*)A, (const bf16*)B, C,
                                                                   (const bf16*)bias, (const bf16*)R, M, N, K, ldc,
                                                                   w.ws, w.cnt, 1, bfrag);
  GAI_LAUNCH_CHECK();
  return true;
}

// Parts per tile of the split walk: the S in 2..8 (S <= K / 128) with the lowest modelled time, in k-doubles per
// workgroup: waves x doubles per part, plus ~3.5 doubles per 256 KiB quadrant set a workgroup stores (each item)
// or loads (the last part of a tile loads all S); 1 when no split beats the tile walk. GAI_GEMM_SPLIT_S overrides.
int split_parts(int M, int N, int K) {
  if (K % 128) return 1;
  const int G = sk_grid(), T = ring_tiles(M, N), hp = K / 128;
  static const int env = getenv("GAI_GEMM_SPLIT_S") ? atoi(getenv("GAI_GEMM_SPLIT_S")) : 0;
  if (env > 0) return std::min(env, hp);
  auto cost = [&](int S) {
    const double waves = (double)((T * S + G - 1) / G);
    const double dbl = 2.0 * ((hp + S - 1) / S);
    return waves * dbl + (S > 1 ? 3.5 * (waves + (double)S * T / G) : 0.0);
  };
  int best = 1;
  for (int S = 2; S <= std::min(8, hp); ++S)
    if (cost(S) < cost(best)) best = S;
  return best;
}

template <int EPI, bool OUTF32>
bool launch_w4x(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
                hipStream_t st, int S, int bfrag) {
  if (K % 128 || S < 2 || S > K / 128) return false;
  static bool once = false;
  if (!once) {
    set_max_lds(gemm_w4r_kernel<EPI, OUTF32, 2>);
    once = true;
  }
  const int tiles = ring_tiles(M, N);
  const long long items = (long long)tiles * S;
  if (items * 4 * kSkQuad * sizeof(float) >= (1ull << 31)) return false;  // 32-bit workspace offsets
  const int ncu = sk_grid();
  const int grid = items <= ncu ? (int)items : ncu;
  SkWorkspace w;
  if (!sk_workspace(st, (size_t)items * 4 * kSkQuad * sizeof(float), (size_t)tiles * 4, w)) return false;
  gemm_w4r_kernel<EPI, OUTF32, 2><<<grid, 256, 5 * kPart, st>>>((const bf16*)A, (const bf16*)B, C,
                                                                (const bf16*)bias, (const bf16*)R, M, N, K, ldc,
                                                                w.ws, w.cnt, S, bfrag);
  GAI_LAUNCH_CHECK();
  return true;
}

template <int MT, int NF, int EPI, bool OUTF32>
void launch_skinny_mt(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                      int ldc, hipStream_t st, int bfrag) {
  const int nblk = (N + 16 * NF - 1) / (16 * NF);
  const size_t lds = (size_t)8 * MT * NF * 4 * 64 * sizeof(float);
  static bool once = false;
  if (!once) {
    set_max_lds(gemm_skinny_kernel<MT, NF, EPI, OUTF32>);
    once = true;
  }
  gemm_skinny_kernel<MT, NF, EPI, OUTF32><<<nblk, 512, lds, st>>>((const bf16*)A, (const bf16*)B, C,
                                                                  (const bf16*)bias, (const bf16*)R, M, N, K, ldc,
                                                                  bfrag);
  GAI_LAUNCH_CHECK();
}

template <int NF, int EPI, bool OUTF32>
void launch_skinny_nf(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                      int ldc, hipStream_t st, int bfrag) {
  if (M <= 16) return launch_skinny_mt<1, NF, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, bfrag);
  if (M <= 32) return launch_skinny_mt<2, NF, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, bfrag);
  if (M <= 64) return launch_skinny_mt<4, NF, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, bfrag);
  return launch_skinny_mt<8, NF, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, bfrag);
}

template <int EPI, bool OUTF32>
void launch_gemm(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                 int ldc, int force, hipStream_t st, int bfrag) {
  // bfrag: B [N, K] is stored in MFMA fragment order (ops.shuffle_fragments) - the one weight layout of the
  // decode projections, read by every kernel below except the w4p fallback for >= 2 GiB operands
  if (bfrag && (N % 16 || K % 64 || (size_t)N * K * 2 >= (1ull << 31)))
    gai_launch_error(__FILE__, __LINE__, "gemm: a fragment-ordered B needs N%16==0, K%64==0 and < 2 GiB");
  const bool skinny_ok = (K % 256) == 0 && M <= 128;
  const bool use_skinny = force == 1 || (force == 0 && skinny_ok);
  if (use_skinny) {
    if (!skinny_ok) gai_launch_error(__FILE__, __LINE__, "gemm_skinny: needs M<=128 and K%256==0");
    // two 16-row fragments per wave when there are enough column blocks to fill the chip
    if (EPI != EPI_SWIGLU && N / 32 >= 512)
      return launch_skinny_nf<2, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, bfrag);
    if (EPI == EPI_SWIGLU) return launch_skinny_nf<2, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, bfrag);
    return launch_skinny_nf<1, EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, bfrag);
  }
  if (K % TBK) gai_launch_error(__FILE__, __LINE__, "gemm_tiled: K must be a multiple of 64");
  // ring kernel: 16-B epilogue stores need N % 16 == 0; the 2-unit unrolled ring needs K % 64 == 0, K >= 160
  const bool ring_ok = N % 16 == 0 && K % 64 == 0 && K / 32 >= RNS && ldc % 8 == 0;
  if (force >= 8 || (force == 0 && N >= 256 && ring_ok && ring_auto(M, N, K))) {
    if (!ring_ok) gai_launch_error(__FILE__, __LINE__, "gemm_ring: needs N%16==0, K%64==0, K>=192, ldc%8==0");
    const bool big = (size_t)M * K * 2 >= (1ull << 31) || (size_t)N * K * 2 >= (1ull << 31);  // 32-bit buffer offsets
    if (!bfrag && (force == 8 || big)) return launch_w4p<EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st);
    if (big) return launch_tiled<EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, bfrag);  // (64-bit addressing)
    if ((force == 11 || (force == 0 && sk_auto(M, N, K))) &&
        launch_w4s<EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, bfrag))
      return;
    if (force == 12 &&
        launch_w4x<EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, std::max(2, split_parts(M, N, K)), bfrag))
      return;
    // the part ring (its operands get 2-3 phases of latency cover) with the operands streamed from HBM as in the
    // model - every layer's weights are read once per forward, past the 256 MB Infinity Cache: it is the fastest
    // or tied walk on every Llama-3-8B projection at M = 2406 and 16384 (O 78.9 vs 91.0 us double-slot / 88.6 on
    // 192-row tiles, down 251.8 vs 293.3 / 291.4; profiles/r5/gemm/cold_m2406_16384.jsonl, tools/gemm_bench.py
    // --cold). Back-to-back runs on one operand pair (cache-resident) favour the double-slot kernel by 2-15 % and
    // misled the round-4 / early round-5 rules. Exception, measured in the model (profiles/r5/c1_prefill_kernels*.csv):
    // the wide gate_up (N >= 16384, 1120 tiles) of a single 2406-token prompt runs 430.6 us per layer on the double-slot
    // walk vs 445.4 on the part ring.
    if (force == 10 || (force == 0 && !(M < 8192 && N >= 16384)))
      return launch_w4r<EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, bfrag);
    // force 9 / 13: the double-slot walk with 256- / 192-row tiles (tests, A/B); auto: w4d_rows
    return launch_w4d<EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, RopeKvArgs{},
                                   force == 9 ? 256 : force == 13 ? 192 : 0, bfrag);
  }
  launch_tiled<EPI, OUTF32>(A, B, C, bias, R, M, N, K, ldc, st, bfrag);
}

}  // namespace

// per-epilogue entry points (gemm_epi_*.hip), called by gai_gemm
#define GAI_GEMM_RUN_ARGS                                                                                     \
  const void *A, const void *B, void *C, const void *bias, const void *R, int M, int N, int K, int ldc, int out_f32, \
      int force, hipStream_t st, int bfrag
#define GAI_GEMM_RUN(E)                                                                     \
  void gai_gemm_run##E(GAI_GEMM_RUN_ARGS) {                                                 \
    if (out_f32)                                                                            \
      launch_gemm<E, true>(A, B, C, bias, R, M, N, K, ldc, force, st, bfrag);               \
    else                                                                                    \
      launch_gemm<E, false>(A, B, C, bias, R, M, N, K, ldc, force, st, bfrag);              \
  }
void gai_gemm_run0(GAI_GEMM_RUN_ARGS);
void gai_gemm_run1(GAI_GEMM_RUN_ARGS);
void gai_gemm_run2(GAI_GEMM_RUN_ARGS);
void gai_gemm_run3(GAI_GEMM_RUN_ARGS);
void gai_gemm_run4(GAI_GEMM_RUN_ARGS);
void gai_gemm_run5(GAI_GEMM_RUN_ARGS);
void gai_gemm_run6(GAI_GEMM_RUN_ARGS);
void gai_gemm_run7(GAI_GEMM_RUN_ARGS);
