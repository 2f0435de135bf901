// Host-side launchers of the gfx950 kernels. Pointers are raw device pointers;
// every launcher enqueues on `st` and never synchronises (graph-capture safe).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

void gai_launch_error(const char* file, int line, const char* msg);

// norm.hip
void gai_rmsnorm(const void* x, const void* residual_in, void* residual_out, const void* w, void* out, int T, int D,
                 float eps, hipStream_t st);
void gai_layernorm(const void* x, const void* residual_in, void* residual_out, const void* w, const void* b,
                   void* out, int T, int D, float eps, hipStream_t st);

// rope_kv.hip
// kv_fp8: caches hold OCP e4m3fn x / {k,v}_scale (fp8 KV cache option); scales are ignored for bf16 caches
// Encoder self-attention K / V (no RoPE): the packed QKV rows of each transient page's tokens -> the page's K [16][D]
// and V^T [D][16] images, whole-page 16-B stores (rope_kv.hip kv_pack_kernel). blk_tok[b] / blk_n[b]: first token and
// row count of page b (rows past blk_n are zeroed).
void gai_kv_pack(const void* qkv, int ld, int koff, int voff, const int* blk_tok, const int* blk_n, int nblk,
                 void* k_cache, void* v_cache, int Hkv, int D, hipStream_t st);
void gai_rope_kv_write(const void* qkv, const int* pos, const float* cos_sin, const int* slots, void* q_out,
                       void* k_cache, void* v_cache, int T, int Hq, int Hkv, int D, int rope, int kv_fp8,
                       float k_scale, float v_scale, hipStream_t st);

// gemm.hip  (epi: 0 none, 1 bias, 2 bias+gelu, 3 residual, 4 swiglu, 5 bias+residual, 6 bias+relu, 7 bias+quick-gelu;
//            force: 0 auto, 1 skinny, 2 tiled 128x128, 3 large 256x256; bfrag: B stored in MFMA fragment order,
//            ops.shuffle_fragments - the one layout of the decode projection weights)
void gai_gemm(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
              int epi, int out_f32, int force, hipStream_t st, int bfrag = 0);

// gemm.hip prefill QKV projection (M >= 1024, D = 128, bf16 KV) with (+ bias) -> RoPE -> q_out / paged K, V^T
// caches fused into the GEMM epilogue (as gai_gemm + gai_rope_kv_write); returns 0 (nothing launched) otherwise
int gai_gemm_prefill_rope_kv(const void* A, const void* B, const void* bias, const int* pos, const float* cos_sin,
                             const int* slots, void* q_out, void* k_cache, void* v_cache, int M, int K, int Hq,
                             int Hkv, int D, int kv_fp8, hipStream_t st, int bfrag = 0);

// gemm_fp8.hip (force: 0 auto, 2 tiled 128x128, 3 large 256x256; OCP e4m3fn operands, per-row sa[M] x per-channel sb[N] scales; epi as gai_gemm + 7 bias+quick-gelu)
void gai_gemm_fp8(const void* A, const void* B, const float* sa, const float* sb, void* C, const void* bias,
                  const void* R, int M, int N, int K, int ldc, int epi, int out_f32, int force, hipStream_t st);
void gai_quant_rows_fp8(const void* x, int M, int K, long ldx, void* q, float* scale, hipStream_t st);

// gemm_splitk.hip (decode M <= 64: weight-streaming split-K; ws = fp32 [KS, M, N] partials;
//                  psw: B pre-shuffled into MFMA fragments [N/16][K/32][64][8], see ops.preshuffle_weight)
int gai_gemm_splitk_ks(int M, int N, int K);
size_t gai_gemm_splitk_ws_bytes(int M, int N, int K);
void gai_gemm_splitk(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                     int ldc, int epi, int out_f32, float* ws, int psw, hipStream_t st);

// gemm_decode.hip (decode M <= 64 on the natural [N, K] weight layout: activations staged once per
//                  workgroup in LDS, weights streamed through a register ring, epilogue fused; returns false
//                  when the shape does not fit (caller falls back to gai_gemm_splitk's kernels))
int gai_gemm_dec2_ok(int M, int N, int K, int epi);
// gemm_splitk.hip fused decode QKV tail: split-K QKV projection, then ONE kernel sums the partials (+ bias),
// applies RoPE and writes q / the paged K, V^T caches (as gai_rope_kv_write). Returns 0 (nothing launched)
// when the shape does not take the split-K path; ws as gai_gemm_splitk. tail_cnt (zeroed int32 ticket counters,
// >= N / 128, left zeroed): at head_dim 128 the sum + RoPE + KV write runs inside the GEMM launch instead.
int gai_gemm_splitk_rope_kv(const void* A, const void* B, const void* bias, const int* pos, const float* cos_sin,
                            const int* slots, void* q_out, void* k_cache, void* v_cache, int M, int Hq, int Hkv,
                            int D, int kv_fp8, float k_scale, float v_scale, float* ws, int psw, hipStream_t st,
                            int K, int* tail_cnt = nullptr);
bool gai_gemm_dec2(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K, int ldc,
                   int epi, int out_f32, hipStream_t st, int psw = 0);
// deep-K decode projections: K split over workgroups into fp32 slabs ws[KS][M][N]; returns KS (0: not handled)
int gai_gemm_dec2_partials_ks(int M, int N, int K);
int gai_gemm_dec2_partials(const void* A, const void* W, int M, int N, int K, float* ws, hipStream_t st,
                           int psw = 0);

// attention.hip
void gai_attn_prefill(const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                      int max_blocks, const int* tiles, int ntiles, const int* cu_q, const int* ctx_lens, void* out,
                      int Hq, int Hkv, int D, float scale, int causal, float* lse, int kv_fp8, float k_scale,
                      float v_scale, hipStream_t st, int q_ld = 0);
int gai_attn_prefill_rows_per_tile(int Hq, int Hkv, int D = 128);
void gai_attn_prefill_set_hl(int hl);
// Decode QKV tail folded into the decode-attention launch: the split-K QKV partial slabs part[ks][B][n] (n = (Hq +
// 2 Hkv) D, no bias) are summed, rounded to bf16, rotated (RoPE at pos[seq]) inside attn_decode; the split holding
// the newest key also writes that key / value into the paged caches at slots[seq].
struct GaiQkvFold {
  const float* part = nullptr;
  int ks = 0;
  int n = 0;
  const int* pos = nullptr;
  const float* cos_sin = nullptr;
  const int* slots = nullptr;
};
void gai_attn_decode(const void* q, const void* k_cache, const void* v_cache, const int* block_tables,
                     int max_blocks, const int* ctx_lens, void* out, float* ws_o, float* ws_ml, int B, int Hq,
                     int Hkv, int D, float scale, int split_keys, int max_splits, int kv_fp8, float k_scale,
                     float v_scale, hipStream_t st, int* split_cnt = nullptr,
                     const GaiQkvFold* fold = nullptr);
// QKV partial slabs only (for GaiQkvFold): KS (2..8) when launched, 0 when the shape runs elsewhere.
int gai_gemm_qkv_partials(const void* A, const void* B, int M, int N, int K, float* ws, int psw, hipStream_t st);

// sampling.hip
size_t gai_sample_ws_bytes(int B, int V);
void gai_sample_tp_stats(const float* x, long ld, int B, int Vl, int vstart, int V, const float* temperature,
                         const int64_t* seeds, int64_t step, float* out, long ostride, hipStream_t st);
int gai_sample_tp_resolve(const float* packets, int R, int B, int W, int C, int V, const float* temperature,
                          const float* top_p, const int* top_k, const int64_t* seeds, int64_t step, int* out_tokens,
                          int* flags, hipStream_t st);
void gai_sample(const float* logits, int B, int V, long ld, const float* temperature, const float* top_p,
                const int* top_k, const int64_t* seeds, int64_t step, int* out_tokens, void* ws, size_t ws_bytes,
                hipStream_t st);
void gai_token_mask(float* logits, long ld, int V, const int* rows, int R, const uint32_t* mask, int W,
                    hipStream_t st);
void gai_apply_penalties(float* logits, int B, long ld, const int* tok_ids, const int* tok_cnt, const int* n,
                         int max_n, const float* freq, const float* pres, const float* rep, hipStream_t st);

// topk.hip
int gai_topk_cap(int k);
// Streaming-SDR DSP (dsp.hip): complex64 FIR with zero initial state, FM discriminator, polyphase rational resampler
void gai_dsp_fir_complex(const void* x, const float* taps, int n, int ntaps, void* y, hipStream_t st);
void gai_dsp_fm_demod(const void* x, int n, float* y, hipStream_t st);
void gai_dsp_upfirdn(const float* x, int n, const float* taps, int ntaps, int up, int down, int offset, int nout,
                     float gain, float* y, hipStream_t st);
void gai_topk_merge(const float* vals, const int* idx, int nlists, int nq, int cap, int k, float* out_v, int64_t* out_i,
                    hipStream_t st);
void gai_sim_topk(const void* Q, const void* X, const float* bias, int nq, int N, int D, int k, float* ws_v,
                  int* ws_i, int nwg, int rows_per_wg, float* out_v, int64_t* out_i, hipStream_t st);

// moe.hip
void gai_moe_dispatch(const int* ids, int n, int k, int E, int* a_rows, int* offs, int* pos, hipStream_t st,
                      int div = 1, int* a_pairs = nullptr);
// gemv.hip: decode GEMV for 1..4 token rows with the RMSNorm staged in and the epilogue fused
int gai_gemv_ok(int M, int N, int K, int normed);
// wfrag: W stored in MFMA fragment order (ops.shuffle_fragments; N % 16 == 0, 32 for SwiGLU)
// epi 5 (K parts): out = fp32 slabs [ks][M][N]; swi: stage bf16(silu(g) * u) of an fp32 [M, 2K] interleaved gate_up
void gai_gemv(const void* x, const void* gamma, float eps, const void* W, int M, int N, int K, int epi, void* out,
              void* res, hipStream_t st, int wfrag = 0, const float* swi = nullptr, int ks = 1);
void gai_gemv_rope_kv(const void* x, const void* gamma, float eps, const void* W, int M, int K, const int* pos,
                      const float* cos_sin, const int* slots, void* q_out, void* k_cache, void* v_cache, int Hq,
                      int Hkv, hipStream_t st, int wfrag = 0);
// expert parallelism (moe.hip): fixed-capacity send slabs and the weighted combine of the returned slabs
void gai_ep_pack(const void* x, const int* ids, const int* offs, const int* a_pairs, int W, int C, int k, int D,
                 int ld, int e_local, void* send, int* send_eid, hipStream_t st);
void gai_ep_combine(const void* back, const int* ids, const int* pos, const int* offs, const float* w,
                    const void* residual, void* out, int T, int k, int D, int e_local, int C, hipStream_t st);
// gemm_decode.hip: decode-sized grouped GEMM on the weight-streaming decode kernel (0 = shape not handled)
int gai_moe_gemm_dec2(const void* A, const int* a_rows, const void* W, void* C, const int* offs, int E,
                      int rows_total, int N, int K, int swiglu, hipStream_t st);
void gai_moe_route(const float* logits, int T, int E, int k, int renorm, int* ids, float* w, hipStream_t st);
void gai_moe_gemm(const void* A, const int* a_rows, const void* W, void* C, const int* offs, int E, int rows_total,
                  int N, int K, int swiglu, hipStream_t st);
void gai_moe_combine(const void* Y, const int* pos, const float* w, const void* residual, void* out, int T, int k,
                     int D, hipStream_t st);

// misc.hip
void gai_embedding(const int* ids, const void* table, void* out, int T, int D, int vstart, int vend, hipStream_t st);
void gai_pool(const void* h, const int* cu, float* out, int B, int D, int mode, int normalize, hipStream_t st);
void gai_silu_mul(const void* x, void* y, int T, int I, hipStream_t st);
void gai_gelu(const void* x, void* y, int T, int I, hipStream_t st);
void gai_gelu_tanh(const void* x, void* y, int T, int I, hipStream_t st);
void gai_geglu_interleaved(const void* x, void* y, int T, int I, hipStream_t st);
void gai_silu_mul_interleaved(const void* x, void* y, int T, int I, hipStream_t st);
void gai_decode_advance(const int* toks, int* ids, int* pos, int* ctx, int* slots, const int* bt, int max_blocks,
                        const int* n_valid, int B, int block, hipStream_t st);

// vision.hip
void gai_patchify(const float* img, int B, int C, int H, int W, int P, int Kp, const float* mean,
                  const float* inv_std, void* out, hipStream_t st);
void gai_vit_embed(const void* patches, const void* cls, const void* pos, void* out, int B, int NP, int D,
                   hipStream_t st);

// comm/custom_ar.hip (one-shot peer-memory all-reduce; buffers from gai_ipc_malloc, uncached)
#define GAI_AR_MAX_WORLD 8
#define GAI_AR_CHUNK 16384
#define GAI_AR_MAX_BLOCKS 512
void gai_custom_allreduce(const void* in, void* out, int64_t bytes, int f32, void* const* peer_data,
                          uint32_t* const* peer_sig, uint32_t* counters, int rank, int world, int64_t slot_bytes,
                          int* err, hipStream_t st);
// two-shot (reduce-scatter + all-gather) over its own buffers: region_bytes per (parity, src, region)
// one-shot all-to-all of W equal segments over the one-shot all-reduce's buffers / signals
void gai_custom_all_to_all(const void* in, void* out, int64_t seg_bytes, void* const* peer_data,
                           uint32_t* const* peer_sig, uint32_t* counters, int rank, int world, int64_t slot_bytes,
                           int* err, hipStream_t st, const int* send_rows = nullptr, const int* recv_rows = nullptr,
                           int64_t row_bytes = 0);
void gai_custom_allreduce_twoshot(const void* in, void* out, int64_t bytes, int f32, void* const* peer_data,
                                  uint32_t* const* peer_sig, uint32_t* counters, int rank, int world,
                                  int64_t region_bytes, int* err, hipStream_t st);
// one-shot all-reduce fused with residual add + RMSNorm (bf16 rows of D = 2048 * {1,2,4}); same buffers as
// gai_custom_allreduce
void gai_custom_allreduce_rmsnorm(const void* in, void* out, void* residual, const void* w, int64_t rows, int D,
                                  float eps, void* const* peer_data, uint32_t* const* peer_sig, uint32_t* counters,
                                  int rank, int world, int64_t slot_bytes, int* err, hipStream_t st);
void* gai_ipc_malloc(int64_t bytes);
void gai_ipc_free(void* p);
void gai_ipc_get_handle(void* p, char* handle64);
void* gai_ipc_open(const char* handle64);
void gai_ipc_close(void* p);

// gemm_splitk.hip fused decode tail (TP = 1): res = bf16(bf16(A.W^T + bias) + res); out = rmsnorm(res) * g
int gai_gemm_splitk_fusable_norm(int M, int N, int K);
void gai_gemm_splitk_add_rmsnorm(const void* A, const void* B, const void* bias, void* res, const void* g, void* out,
                                 int M, int N, int K, float eps, float* ws, int psw, hipStream_t st);

// gdn.hip (Qwen3-Next gated DeltaNet decode step; state pool [slots, Hv, DK, DV] fp32, updated in place)
void gai_gdn_decode(const float* q, const float* k, const float* v, const float* g, const float* beta, float* state,
                    const int* slots, float* out, int B, int Hv, int DK, int DV, hipStream_t st);
