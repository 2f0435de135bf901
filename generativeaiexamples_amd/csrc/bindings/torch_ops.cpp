// PyTorch bindings for the gfx950 kernels (module `generativeaiexamples_amd._C`).
//
// Thin shape/dtype checks, then a launch on the current HIP stream. No host
// synchronisation and no allocation happens here, so every op can be captured
// into a HIP graph by torch.cuda.graph().
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <stdexcept>
#include <string>

#include "gai_kernels.h"

void gai_launch_error(const char* file, int line, const char* msg) {
  throw std::runtime_error(std::string("gai kernel error at ") + file + ":" + std::to_string(line) + ": " + msg);
}

namespace {

using at::Tensor;
using c10::optional;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_bf16(const Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
}
void check_i32(const Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kInt, name, " must be int32");
}
void check_f32(const Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
}
const void* opt_ptr(const optional<Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

void rmsnorm(const Tensor& x, const Tensor& w, double eps, Tensor& out, const optional<Tensor>& residual_in,
             const optional<Tensor>& residual_out) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(out, "out");
  const int D = x.size(-1);
  const int T = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && w.numel() == D, "rmsnorm: bad hidden size");
  if (residual_in) check_bf16(*residual_in, "residual_in");
  if (residual_out) check_bf16(*residual_out, "residual_out");
  gai_rmsnorm(x.data_ptr(), opt_ptr(residual_in), residual_out ? residual_out->data_ptr() : nullptr, w.data_ptr(),
              out.data_ptr(), T, D, (float)eps, cur_stream());
}

void layernorm(const Tensor& x, const Tensor& w, const optional<Tensor>& b, double eps, Tensor& out,
               const optional<Tensor>& residual_in, const optional<Tensor>& residual_out) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(out, "out");
  const int D = x.size(-1);
  const int T = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && w.numel() == D, "layernorm: bad hidden size");
  gai_layernorm(x.data_ptr(), opt_ptr(residual_in), residual_out ? residual_out->data_ptr() : nullptr, w.data_ptr(),
                opt_ptr(b), out.data_ptr(), T, D, (float)eps, cur_stream());
}

// KV caches are bf16, or 1-byte OCP e4m3fn (torch.float8_e4m3fn / uint8 storage) for the fp8 KV option
int kv_cache_fp8(const Tensor& k, const Tensor& v) {
  check_dev(k, "k_cache");
  check_dev(v, "v_cache");
  TORCH_CHECK(k.scalar_type() == v.scalar_type(), "k / v caches must share a dtype");
  const auto t = k.scalar_type();
  if (t == at::kBFloat16) return 0;
  TORCH_CHECK(t == at::kFloat8_e4m3fn || t == at::kByte, "KV cache must be bf16 or float8_e4m3fn");
  TORCH_CHECK(k.is_contiguous() && v.is_contiguous(), "KV caches must be contiguous");
  return 1;
}

void rope_kv_write(const Tensor& qkv, const Tensor& pos, const Tensor& cos_sin, const Tensor& slots, Tensor& q_out,
                   Tensor& k_cache, Tensor& v_cache, int64_t Hq, int64_t Hkv, int64_t D, bool rope, double k_scale,
                   double v_scale) {
  check_bf16(qkv, "qkv");
  check_i32(pos, "positions");
  check_f32(cos_sin, "cos_sin");
  check_i32(slots, "slot_mapping");
  check_bf16(q_out, "q_out");
  const int f8 = kv_cache_fp8(k_cache, v_cache);
  const int T = qkv.size(0);
  TORCH_CHECK(qkv.size(1) == (Hq + 2 * Hkv) * D, "rope_kv_write: qkv width mismatch");
  TORCH_CHECK(k_cache.size(-2) == 16 && k_cache.size(-1) == D && v_cache.size(-1) == 16, "bad kv cache layout");
  gai_rope_kv_write(qkv.data_ptr(), pos.data_ptr<int>(), cos_sin.data_ptr<float>(), slots.data_ptr<int>(),
                    q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), T, Hq, Hkv, D, rope ? 1 : 0, f8,
                    (float)k_scale, (float)v_scale, cur_stream());
}

// QKV projection fused with RoPE + KV write: split-K path for decode (M <= 64), the prefill GEMM's
// epilogue for M >= 1024. False: nothing launched, the caller runs linear + rope_kv_write.
bool gemm_rope_kv(const Tensor& A, const Tensor& B, const optional<Tensor>& bias, const Tensor& pos,
                  const Tensor& cos_sin, const Tensor& slots, Tensor& q_out, Tensor& k_cache, Tensor& v_cache,
                  int64_t Hq, int64_t Hkv, int64_t D, double k_scale, double v_scale, Tensor& ws, bool psw,
                  const optional<Tensor>& tail_cnt) {
  check_bf16(A, "A");
  check_bf16(B, "B");
  check_i32(pos, "positions");
  check_f32(cos_sin, "cos_sin");
  check_i32(slots, "slot_mapping");
  check_bf16(q_out, "q_out");
  TORCH_CHECK(A.dim() == 2 && A.is_contiguous() && B.is_contiguous(), "gemm_rope_kv: A [M, K] and B contiguous");
  const int M = A.size(0), K = A.size(1);
  TORCH_CHECK(B.size(0) == (Hq + 2 * Hkv) * D && B.size(1) == K, "gemm_rope_kv: weight shape mismatch");
  TORCH_CHECK(pos.numel() >= M && slots.numel() >= M && q_out.size(0) >= M, "gemm_rope_kv: batch mismatch");
  TORCH_CHECK(k_cache.size(-2) == 16 && k_cache.size(-1) == D && v_cache.size(-1) == 16, "bad kv cache layout");
  const int N = B.size(0);
  if (bias) check_bf16(*bias, "bias");
  const int f8 = kv_cache_fp8(k_cache, v_cache);
  if (M > 64)  // prefill: RoPE + KV write in the 256x256 GEMM's epilogue (ws unused)
    return gai_gemm_prefill_rope_kv(A.data_ptr(), B.data_ptr(), opt_ptr(bias), pos.data_ptr<int>(),
                                    cos_sin.data_ptr<float>(), slots.data_ptr<int>(), q_out.data_ptr(),
                                    k_cache.data_ptr(), v_cache.data_ptr(), M, K, Hq, Hkv, D, f8, cur_stream(),
                                    psw ? 1 : 0) != 0;
  TORCH_CHECK(ws.scalar_type() == at::kFloat && (size_t)ws.numel() * 4 >= gai_gemm_splitk_ws_bytes(M, N, K),
              "gemm_rope_kv: workspace too small");
  int* cnt = nullptr;
  if (tail_cnt && tail_cnt->defined()) {
    check_i32(*tail_cnt, "tail_cnt");
    TORCH_CHECK(tail_cnt->numel() >= (N + 127) / 128, "gemm_rope_kv: tail_cnt too small");
    cnt = tail_cnt->data_ptr<int>();
  }
  return gai_gemm_splitk_rope_kv(A.data_ptr(), B.data_ptr(), opt_ptr(bias), pos.data_ptr<int>(),
                                 cos_sin.data_ptr<float>(), slots.data_ptr<int>(), q_out.data_ptr(),
                                 k_cache.data_ptr(), v_cache.data_ptr(), M, Hq, Hkv, D, f8, (float)k_scale,
                                 (float)v_scale, ws.data_ptr<float>(), psw ? 1 : 0, cur_stream(), K, cnt) != 0;
}

// The epilogue reads bias / residual through raw pointers: an epilogue code whose operand is missing
// would read address 0 on the device, so refuse it on the host.
static void check_epi_operands(int64_t epi, const optional<Tensor>& bias, const optional<Tensor>& R,
                               const char* what) {
  TORCH_CHECK(epi >= 0 && epi <= 7, what, ": unknown epilogue ", epi);
  const bool needs_bias = epi == 1 || epi == 2 || epi == 5 || epi == 6 || epi == 7;
  const bool needs_res = epi == 3 || epi == 5;
  TORCH_CHECK(!needs_bias || bias.has_value(), what, ": epilogue ", epi, " needs a bias");
  TORCH_CHECK(!needs_res || R.has_value(), what, ": epilogue ", epi, " needs a residual");
}

void gemm(const Tensor& A, const Tensor& B, Tensor& C, const optional<Tensor>& bias, const optional<Tensor>& R,
          int64_t epi, int64_t force, bool bfrag) {
  check_bf16(A, "A");
  check_bf16(B, "B");
  check_dev(C, "C");
  const int K = A.size(-1);
  const int M = A.numel() / K;
  const int N = B.size(0);
  TORCH_CHECK(B.size(1) == K, "gemm: K mismatch");
  const bool f32 = C.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || C.scalar_type() == at::kBFloat16, "gemm: C must be bf16 or fp32");
  const int ldc = epi == 4 ? N / 2 : N;
  TORCH_CHECK(C.numel() == (int64_t)M * ldc, "gemm: C has wrong size");
  check_epi_operands(epi, bias, R, "gemm");
  if (bias) check_bf16(*bias, "bias");
  if (R) {
    check_bf16(*R, "residual");
    TORCH_CHECK(R->numel() == (int64_t)M * N, "gemm: residual has wrong size");
  }
  gai_gemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), opt_ptr(bias), opt_ptr(R), M, N, K, ldc, (int)epi, f32 ? 1 : 0,
           (int)force, cur_stream(), bfrag ? 1 : 0);
}

void attn_prefill(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& block_tables,
                  const Tensor& tiles, const Tensor& cu_q, const Tensor& ctx_lens, Tensor& out, int64_t Hq,
                  int64_t Hkv, double scale, bool causal, const optional<Tensor>& lse, double k_scale,
                  double v_scale) {
  // q: contiguous, or a row-strided view of the packed QKV rows (checked below)
  TORCH_CHECK(q.is_cuda() && q.scalar_type() == at::kBFloat16, "q must be a bfloat16 GPU tensor");
  const int f8 = kv_cache_fp8(k_cache, v_cache);
  check_i32(block_tables, "block_tables");
  check_i32(tiles, "tiles");
  check_i32(cu_q, "cu_q");
  check_i32(ctx_lens, "ctx_lens");
  check_bf16(out, "out");
  const int D = q.size(-1);
  // q may be a strided view of the packed QKV rows ([T, Hq, D] with row stride q.stride(0)): encoders pass it
  // without a copy
  TORCH_CHECK(q.dim() == 3 && q.stride(2) == 1 && q.stride(1) == D && q.stride(0) >= Hq * D,
              "attn_prefill: q must be [T, Hq, D] with dense heads");
  float* lse_p = nullptr;
  if (lse) {
    check_f32(*lse, "lse");
    TORCH_CHECK(lse->numel() == q.numel() / D, "attn_prefill: lse must be [T, Hq]");
    lse_p = lse->data_ptr<float>();
  }
  gai_attn_prefill(q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr<int>(),
                   block_tables.size(1), tiles.data_ptr<int>(), tiles.numel() / 2, cu_q.data_ptr<int>(),
                   ctx_lens.data_ptr<int>(), out.data_ptr(), Hq, Hkv, D, (float)scale, causal ? 1 : 0, lse_p, f8,
                   (float)k_scale, (float)v_scale, cur_stream(), (int)q.stride(0));
}

void kv_pack(const Tensor& qkv, const Tensor& blk_tok, const Tensor& blk_n, Tensor& k_cache, Tensor& v_cache,
             int64_t Hq, int64_t Hkv, int64_t D) {
  check_bf16(qkv, "qkv");
  check_i32(blk_tok, "blk_tok");
  check_i32(blk_n, "blk_n");
  TORCH_CHECK(kv_cache_fp8(k_cache, v_cache) == 0, "kv_pack: bf16 caches only");
  TORCH_CHECK(qkv.dim() == 2 && qkv.is_contiguous() && qkv.size(1) == (Hq + 2 * Hkv) * D, "kv_pack: qkv [T, (Hq + 2 Hkv) D]");
  TORCH_CHECK(k_cache.size(-2) == 16 && k_cache.size(-1) == D && v_cache.size(-1) == 16 && k_cache.size(1) == Hkv,
              "kv_pack: bad kv cache layout");
  TORCH_CHECK(blk_tok.numel() == blk_n.numel() && blk_tok.numel() <= k_cache.size(0), "kv_pack: page list");
  gai_kv_pack(qkv.data_ptr(), (int)qkv.size(1), (int)(Hq * D), (int)((Hq + Hkv) * D), blk_tok.data_ptr<int>(),
              blk_n.data_ptr<int>(), (int)blk_tok.numel(), k_cache.data_ptr(), v_cache.data_ptr(), (int)Hkv, (int)D,
              cur_stream());
}

void attn_decode(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& block_tables,
                 const Tensor& ctx_lens, Tensor& out, Tensor& ws_o, Tensor& ws_ml, double scale, int64_t split_keys,
                 int64_t max_splits, double k_scale, double v_scale, const c10::optional<Tensor>& split_cnt,
                 const c10::optional<Tensor>& qkv_part, int64_t part_ks, const c10::optional<Tensor>& positions,
                 const c10::optional<Tensor>& cos_sin, const c10::optional<Tensor>& slots) {
  check_bf16(q, "q");
  const int f8 = kv_cache_fp8(k_cache, v_cache);
  check_i32(block_tables, "block_tables");
  check_i32(ctx_lens, "ctx_lens");
  check_bf16(out, "out");
  check_f32(ws_o, "ws_o");
  check_f32(ws_ml, "ws_ml");
  const int B = q.size(0), Hq = q.size(1), D = q.size(2);
  const int Hkv = k_cache.size(1);
  TORCH_CHECK(ws_o.numel() >= (int64_t)max_splits * B * Hq * D, "attn_decode: ws_o too small");
  TORCH_CHECK(ws_ml.numel() >= (int64_t)max_splits * B * Hq * 2, "attn_decode: ws_ml too small");
  int* cnt = nullptr;
  if (split_cnt.has_value() && split_cnt->defined()) {
    check_i32(*split_cnt, "split_cnt");
    TORCH_CHECK(split_cnt->numel() >= (int64_t)B * Hkv, "attn_decode: split_cnt too small");
    cnt = split_cnt->data_ptr<int>();
  }
  GaiQkvFold fold;
  const GaiQkvFold* fp = nullptr;
  if (qkv_part.has_value() && qkv_part->defined()) {
    // decode QKV tail folded into this launch: q comes from the split-K partial slabs [part_ks, B, (Hq + 2 Hkv) D]
    check_f32(*qkv_part, "qkv_part");
    TORCH_CHECK(positions && cos_sin && slots, "attn_decode: the folded QKV tail needs positions, cos_sin, slots");
    check_i32(*positions, "positions");
    check_i32(*slots, "slots");
    check_f32(*cos_sin, "cos_sin");
    const int64_t n = (int64_t)(Hq + 2 * Hkv) * D;
    TORCH_CHECK(f8 == 0 && D == 128, "attn_decode: the folded QKV tail needs head_dim 128 and a bf16 cache");
    TORCH_CHECK(part_ks >= 1 && part_ks <= 16 && qkv_part->numel() >= part_ks * B * n && qkv_part->is_contiguous(),
                "attn_decode: qkv_part must hold part_ks x B x (Hq + 2 Hkv) x D floats");
    TORCH_CHECK(positions->numel() >= B && slots->numel() >= B && cos_sin->size(-1) == D,
                "attn_decode: positions / slots [B], cos_sin [max_pos, D]");
    TORCH_CHECK(cnt != nullptr && max_splits > 1, "attn_decode: the folded QKV tail runs in the fused-merge kernel");
    fold.part = qkv_part->data_ptr<float>();
    fold.ks = (int)part_ks;
    fold.n = (int)n;
    fold.pos = positions->data_ptr<int>();
    fold.cos_sin = cos_sin->data_ptr<float>();
    fold.slots = slots->data_ptr<int>();
    fp = &fold;
  }
  gai_attn_decode(q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr<int>(),
                  block_tables.size(1), ctx_lens.data_ptr<int>(), out.data_ptr(), ws_o.data_ptr<float>(),
                  ws_ml.data_ptr<float>(), B, Hq, Hkv, D, (float)scale, split_keys, max_splits, f8, (float)k_scale,
                  (float)v_scale, cur_stream(), cnt, fp);
}

int64_t gemm_qkv_partials(const Tensor& A, const Tensor& W, Tensor& ws, bool psw) {
  check_bf16(A, "A");
  check_bf16(W, "W");
  check_f32(ws, "ws");
  TORCH_CHECK(A.dim() == 2 && A.is_contiguous(), "gemm_qkv_partials: A [M, K] contiguous");
  const int M = A.size(0), K = A.size(1);
  const int N = W.size(0);  // the fragment-shuffled copy keeps the [N, K] shape
  TORCH_CHECK(W.dim() == 2 && W.size(1) == K && W.is_contiguous(), "gemm_qkv_partials: W [N, K]");
  TORCH_CHECK(ws.numel() >= (int64_t)gai_gemm_splitk_ws_bytes(M, N, K) / 4, "gemm_qkv_partials: workspace");
  return gai_gemm_qkv_partials(A.data_ptr(), W.data_ptr(), M, N, K, ws.data_ptr<float>(), psw ? 1 : 0, cur_stream());
}

void sample(const Tensor& logits, const Tensor& temperature, const Tensor& top_p, const Tensor& top_k,
            const Tensor& seeds, int64_t step, Tensor& out, const c10::optional<Tensor>& ws) {
  check_f32(logits, "logits");
  check_f32(temperature, "temperature");
  check_f32(top_p, "top_p");
  check_i32(top_k, "top_k");
  check_dev(seeds, "seeds");
  TORCH_CHECK(seeds.scalar_type() == at::kLong, "seeds must be int64");
  check_i32(out, "out");
  const int B = logits.size(0), V = logits.size(1);
  TORCH_CHECK(logits.stride(1) == 1, "logits rows must be contiguous");
  void* wp = nullptr;
  size_t wb = 0;
  if (ws.has_value() && ws->defined()) {
    check_dev(*ws, "sample workspace");
    wp = ws->data_ptr();
    wb = ws->numel() * ws->element_size();
  }
  gai_sample(logits.data_ptr<float>(), B, V, logits.stride(0), temperature.data_ptr<float>(),
             top_p.data_ptr<float>(), top_k.data_ptr<int>(), seeds.data_ptr<int64_t>(), step, out.data_ptr<int>(),
             wp, wb, cur_stream());
}

void sample_tp_resolve(const Tensor& packets, int64_t C, int64_t V, const Tensor& temperature, const Tensor& top_p,
                       const Tensor& top_k, const Tensor& seeds, int64_t step, Tensor& out, Tensor& flags) {
  check_f32(packets, "packets");
  TORCH_CHECK(packets.dim() == 3 && packets.is_contiguous(), "packets must be a contiguous [R, B, W] tensor");
  check_f32(temperature, "temperature");
  check_f32(top_p, "top_p");
  check_i32(top_k, "top_k");
  TORCH_CHECK(seeds.scalar_type() == at::kLong, "seeds must be int64");
  check_i32(out, "out");
  check_i32(flags, "flags");
  const int R = packets.size(0), B = packets.size(1), W = packets.size(2);
  TORCH_CHECK(out.numel() >= B, "out too small");
  TORCH_CHECK(gai_sample_tp_resolve(packets.data_ptr<float>(), R, B, W, (int)C, (int)V, temperature.data_ptr<float>(),
                                    top_p.data_ptr<float>(), top_k.data_ptr<int>(), seeds.data_ptr<int64_t>(), step,
                                    out.data_ptr<int>(), flags.data_ptr<int>(), cur_stream()),
              "sample_tp_resolve: R * C must be <= 1024 and W >= 4 + 2C");
}

void sample_tp_stats(const Tensor& logits, int64_t vstart, int64_t V, const Tensor& temperature, const Tensor& seeds,
                     int64_t step, Tensor& out) {
  check_f32(logits, "logits");
  TORCH_CHECK(logits.stride(1) == 1, "logits rows must be contiguous");
  check_f32(temperature, "temperature");
  TORCH_CHECK(seeds.scalar_type() == at::kLong, "seeds must be int64");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat, "out must be a float32 GPU tensor");
  TORCH_CHECK(out.dim() == 2 && out.size(0) >= logits.size(0) && out.size(1) >= 4 && out.stride(1) == 1,
              "out must be a [B, >=4] float view with unit column stride");
  gai_sample_tp_stats(logits.data_ptr<float>(), logits.stride(0), logits.size(0), logits.size(1), (int)vstart, (int)V,
                      temperature.data_ptr<float>(), seeds.data_ptr<int64_t>(), step, out.data_ptr<float>(),
                      out.stride(0), cur_stream());
}

int64_t sample_ws_bytes(int64_t B, int64_t V) { return (int64_t)gai_sample_ws_bytes((int)B, (int)V);
}

void apply_penalties(Tensor& logits, const Tensor& tok_ids, const Tensor& tok_cnt, const Tensor& n,
                     const Tensor& freq, const Tensor& pres, const Tensor& rep) {
  check_f32(logits, "logits");
  check_i32(tok_ids, "tok_ids");
  check_i32(tok_cnt, "tok_cnt");
  check_i32(n, "n");
  gai_apply_penalties(logits.data_ptr<float>(), logits.size(0), logits.stride(0), tok_ids.data_ptr<int>(),
                      tok_cnt.data_ptr<int>(), n.data_ptr<int>(), tok_ids.size(1), freq.data_ptr<float>(),
                      pres.data_ptr<float>(), rep.data_ptr<float>(), cur_stream());
}

void token_mask(Tensor& logits, const Tensor& rows, const Tensor& mask) {
  check_f32(logits, "logits");
  check_i32(rows, "rows");
  TORCH_CHECK(mask.scalar_type() == at::kInt && mask.dim() == 2 && mask.is_contiguous(),
              "token_mask: mask must be int32 [R, W] (uint32 bit words)");
  TORCH_CHECK(mask.size(0) == rows.numel(), "token_mask: one mask row per logits row");
  const int V = logits.size(1), W = mask.size(1);
  TORCH_CHECK((int64_t)W * 32 >= V, "token_mask: mask narrower than the vocabulary");
  gai_token_mask(logits.data_ptr<float>(), logits.stride(0), V, rows.data_ptr<int>(), rows.numel(),
                 reinterpret_cast<const uint32_t*>(mask.data_ptr<int>()), W, cur_stream());
}

void sim_topk(const Tensor& Q, const Tensor& X, const Tensor& bias, int64_t n_rows, int64_t k, Tensor& ws_v,
              Tensor& ws_i, int64_t nwg, int64_t rows_per_wg, Tensor& out_v, Tensor& out_i) {
  check_bf16(Q, "Q");
  check_bf16(X, "X");
  check_f32(bias, "bias");
  check_f32(ws_v, "ws_v");
  check_i32(ws_i, "ws_i");
  check_f32(out_v, "out_v");
  check_dev(out_i, "out_i");
  const int nq = Q.size(0), D = Q.size(1);
  TORCH_CHECK(X.size(1) == D, "sim_topk: dim mismatch");
  TORCH_CHECK(n_rows <= X.size(0) && n_rows <= bias.numel(), "sim_topk: n_rows exceeds storage");
  TORCH_CHECK(rows_per_wg % 128 == 0, "sim_topk: rows_per_wg must be a multiple of 128");
  const int cap = gai_topk_cap(k);
  TORCH_CHECK(ws_v.numel() >= nwg * nq * cap && ws_i.numel() >= nwg * nq * cap, "sim_topk: workspace too small");
  gai_sim_topk(Q.data_ptr(), X.data_ptr(), bias.data_ptr<float>(), nq, n_rows, D, k, ws_v.data_ptr<float>(),
               ws_i.data_ptr<int>(), nwg, rows_per_wg, out_v.data_ptr<float>(), out_i.data_ptr<int64_t>(),
               cur_stream());
}

void moe_route(const Tensor& logits, int64_t k, bool renorm, Tensor& ids, Tensor& w) {
  check_f32(logits, "router logits");
  check_i32(ids, "topk ids");
  check_f32(w, "topk weights");
  gai_moe_route(logits.data_ptr<float>(), logits.size(0), logits.size(1), k, renorm ? 1 : 0, ids.data_ptr<int>(),
                w.data_ptr<float>(), cur_stream());
}

void patchify(const Tensor& img, int64_t P, const Tensor& mean, const Tensor& inv_std, Tensor& out) {
  check_dev(img, "img");
  TORCH_CHECK(img.scalar_type() == at::kFloat && img.dim() == 4 && img.is_contiguous(),
              "patchify: img must be contiguous fp32 [B, C, H, W]");
  check_bf16(out, "out");
  const int B = img.size(0), C = img.size(1), H = img.size(2), W = img.size(3);
  TORCH_CHECK(H % P == 0 && W % P == 0, "patchify: image size must be a multiple of the patch size");
  TORCH_CHECK(mean.numel() >= C && inv_std.numel() >= C && mean.scalar_type() == at::kFloat &&
                  inv_std.scalar_type() == at::kFloat, "patchify: mean/inv_std must be fp32 [C]");
  const int Kp = out.size(-1);
  TORCH_CHECK(Kp >= C * P * P && out.numel() == (int64_t)B * (H / P) * (W / P) * Kp, "patchify: out shape");
  gai_patchify(img.data_ptr<float>(), B, C, H, W, (int)P, Kp, mean.data_ptr<float>(), inv_std.data_ptr<float>(),
               out.data_ptr(), cur_stream());
}

void vit_embed(const Tensor& patches, const Tensor& cls, const Tensor& pos, Tensor& out, int64_t B) {
  check_bf16(patches, "patches");
  check_bf16(cls, "cls");
  check_bf16(pos, "pos");
  check_bf16(out, "out");
  const int D = cls.numel();
  TORCH_CHECK(D % 8 == 0, "vit_embed: dim must be a multiple of 8");
  const int NP = patches.numel() / ((int64_t)B * D);
  TORCH_CHECK(pos.numel() >= (int64_t)(NP + 1) * D && out.numel() == (int64_t)B * (NP + 1) * D, "vit_embed: shapes");
  gai_vit_embed(patches.data_ptr(), cls.data_ptr(), pos.data_ptr(), out.data_ptr(), B, NP, D, cur_stream());
}

void gemm_splitk(const Tensor& A, const Tensor& B, Tensor& C, const optional<Tensor>& bias, const optional<Tensor>& R,
                 int64_t epi, Tensor& ws, bool psw) {
  check_bf16(A, "A");
  check_bf16(B, "B");
  check_dev(C, "C");
  const int K = A.size(-1);
  const int M = A.numel() / K;
  const int N = B.size(0);
  TORCH_CHECK(A.is_contiguous() && B.is_contiguous(), "gemm_splitk: A and B must be contiguous");
  TORCH_CHECK(B.size(1) == K, "gemm_splitk: K mismatch");
  TORCH_CHECK(M <= 64 && gai_gemm_splitk_ks(M, N, K) > 0, "gemm_splitk: needs M <= 64 and K % 128 == 0");
  const bool f32 = C.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || C.scalar_type() == at::kBFloat16, "gemm_splitk: C must be bf16 or fp32");
  const int ldc = epi == 4 ? N / 2 : N;
  TORCH_CHECK(C.numel() == (int64_t)M * ldc, "gemm_splitk: C has wrong size");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_cuda() &&
                  (size_t)ws.numel() * 4 >= gai_gemm_splitk_ws_bytes(M, N, K), "gemm_splitk: workspace too small");
  check_epi_operands(epi, bias, R, "gemm_splitk");
  if (bias) check_bf16(*bias, "bias");
  if (R) {
    check_bf16(*R, "residual");
    TORCH_CHECK(R->numel() == (int64_t)M * N, "gemm_splitk: residual has wrong size");
  }
  gai_gemm_splitk(A.data_ptr(), B.data_ptr(), C.data_ptr(), opt_ptr(bias), opt_ptr(R), M, N, K, ldc, (int)epi,
                  f32 ? 1 : 0, ws.data_ptr<float>(), psw ? 1 : 0, cur_stream());
}

void quant_rows_fp8(const Tensor& x, Tensor& q, Tensor& scale) {
  check_bf16(x, "x");
  check_dev(q, "q");
  TORCH_CHECK(q.element_size() == 1, "quant_rows_fp8: q must be a 1-byte (fp8) tensor");
  TORCH_CHECK(scale.scalar_type() == at::kFloat, "quant_rows_fp8: scale must be fp32");
  const int K = x.size(-1);
  const int M = x.numel() / K;
  TORCH_CHECK(x.stride(-1) == 1 && (x.dim() == 1 || x.stride(-2) >= K), "quant_rows_fp8: rows must be contiguous");
  TORCH_CHECK(q.numel() == (int64_t)M * K && scale.numel() == M, "quant_rows_fp8: output sizes");
  const long ldx = x.dim() > 1 ? x.stride(-2) : K;
  gai_quant_rows_fp8(x.data_ptr(), M, K, ldx, q.data_ptr(), scale.data_ptr<float>(), cur_stream());
}

void gemm_fp8(const Tensor& A, const Tensor& B, const Tensor& sa, const Tensor& sb, Tensor& C,
              const optional<Tensor>& bias, const optional<Tensor>& R, int64_t epi, int64_t force) {
  check_dev(A, "A");
  check_dev(B, "B");
  check_dev(C, "C");
  TORCH_CHECK(A.element_size() == 1 && B.element_size() == 1, "gemm_fp8: A and B must be fp8");
  TORCH_CHECK(A.is_contiguous() && B.is_contiguous(), "gemm_fp8: A and B must be contiguous");
  const int K = A.size(-1);
  const int M = A.numel() / K;
  const int N = B.size(0);
  TORCH_CHECK(B.size(1) == K, "gemm_fp8: K mismatch");
  TORCH_CHECK(sa.scalar_type() == at::kFloat && sa.numel() == M, "gemm_fp8: sa must be fp32 [M]");
  TORCH_CHECK(sb.scalar_type() == at::kFloat && sb.numel() == N, "gemm_fp8: sb must be fp32 [N]");
  const bool f32 = C.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || C.scalar_type() == at::kBFloat16, "gemm_fp8: C must be bf16 or fp32");
  const int ldc = epi == 4 ? N / 2 : N;
  TORCH_CHECK(C.numel() == (int64_t)M * ldc, "gemm_fp8: C has wrong size");
  check_epi_operands(epi, bias, R, "gemm_fp8");
  if (bias) check_bf16(*bias, "bias");
  if (R) {
    check_bf16(*R, "residual");
    TORCH_CHECK(R->numel() == (int64_t)M * N, "gemm_fp8: residual has wrong size");
  }
  gai_gemm_fp8(A.data_ptr(), B.data_ptr(), sa.data_ptr<float>(), sb.data_ptr<float>(), C.data_ptr(), opt_ptr(bias),
               opt_ptr(R), M, N, K, ldc, (int)epi, f32 ? 1 : 0, (int)force, cur_stream());
}

void moe_gemm(const Tensor& A, const optional<Tensor>& a_rows, const Tensor& W, Tensor& C, const Tensor& offs,
              int64_t rows_total, bool swiglu) {
  check_bf16(A, "A");
  check_bf16(W, "W");
  check_bf16(C, "C");
  check_i32(offs, "expert offsets");
  if (a_rows) check_i32(*a_rows, "a_rows");
  TORCH_CHECK(W.dim() == 3 && W.size(2) == A.size(-1), "moe_gemm: W must be [E, N, K]");
  gai_moe_gemm(A.data_ptr(), a_rows ? a_rows->data_ptr<int>() : nullptr, W.data_ptr(), C.data_ptr(),
               offs.data_ptr<int>(), W.size(0), rows_total, W.size(1), W.size(2), swiglu ? 1 : 0, cur_stream());
}

void moe_dispatch(const Tensor& ids, int64_t E, Tensor& a_rows, Tensor& offs, Tensor& pos) {
  check_i32(ids, "expert ids");
  check_i32(a_rows, "a_rows");
  check_i32(offs, "offs");
  check_i32(pos, "pos");
  TORCH_CHECK(ids.is_contiguous() && a_rows.is_contiguous() && offs.is_contiguous() && pos.is_contiguous(),
              "moe_dispatch: tensors must be contiguous");
  TORCH_CHECK(ids.dim() == 2, "moe_dispatch: ids must be [T, k]");
  const int64_t n = ids.numel();
  TORCH_CHECK(E >= 1 && E <= 2048, "moe_dispatch: 1 <= experts <= 2048");
  TORCH_CHECK(a_rows.numel() == n && pos.numel() == n && offs.numel() == E + 1, "moe_dispatch: output sizes");
  if (n == 0) return;
  gai_moe_dispatch(ids.data_ptr<int>(), (int)n, (int)ids.size(1), (int)E, a_rows.data_ptr<int>(),
                   offs.data_ptr<int>(), pos.data_ptr<int>(), cur_stream());
}

void moe_combine(const Tensor& Y, const Tensor& pos, const Tensor& w, const optional<Tensor>& residual, Tensor& out) {
  check_bf16(Y, "Y");
  check_i32(pos, "pos");
  check_f32(w, "w");
  check_bf16(out, "out");
  const int T = pos.size(0), k = pos.size(1), D = out.size(-1);
  gai_moe_combine(Y.data_ptr(), pos.data_ptr<int>(), w.data_ptr<float>(), opt_ptr(residual), out.data_ptr(), T, k, D,
                  cur_stream());
}

void embedding(const Tensor& ids, const Tensor& table, Tensor& out, int64_t vstart, int64_t vend) {
  check_i32(ids, "ids");
  check_bf16(table, "table");
  check_bf16(out, "out");
  const int D = table.size(1);
  TORCH_CHECK(D % 8 == 0, "embedding: dim must be a multiple of 8");
  gai_embedding(ids.data_ptr<int>(), table.data_ptr(), out.data_ptr(), ids.numel(), D, vstart, vend, cur_stream());
}

void decode_advance(const Tensor& toks, Tensor& ids, Tensor& pos, Tensor& ctx, Tensor& slots, const Tensor& bt,
                    const Tensor& n_valid, int64_t block) {
  check_i32(toks, "toks");
  check_i32(ids, "token_ids");
  check_i32(pos, "positions");
  check_i32(ctx, "ctx_lens");
  check_i32(slots, "slots");
  check_i32(bt, "block_tables");
  check_i32(n_valid, "n_valid");
  const int B = ids.numel();
  TORCH_CHECK(toks.numel() >= B && pos.numel() == B && ctx.numel() == B && slots.numel() == B && bt.size(0) == B,
              "decode_advance: row counts differ");
  TORCH_CHECK(bt.is_contiguous(), "decode_advance: block table must be contiguous");
  gai_decode_advance(toks.data_ptr<int>(), ids.data_ptr<int>(), pos.data_ptr<int>(), ctx.data_ptr<int>(),
                     slots.data_ptr<int>(), bt.data_ptr<int>(), bt.size(1), n_valid.data_ptr<int>(), B, block,
                     cur_stream());
}

void pool(const Tensor& h, const Tensor& cu, Tensor& out, int64_t mode, bool normalize) {
  check_bf16(h, "hidden");
  check_i32(cu, "cu_seqlens");
  check_f32(out, "out");
  gai_pool(h.data_ptr(), cu.data_ptr<int>(), out.data_ptr<float>(), cu.numel() - 1, h.size(-1), mode,
           normalize ? 1 : 0, cur_stream());
}

void silu_mul(const Tensor& x, Tensor& y) {
  check_bf16(x, "x");
  check_bf16(y, "y");
  const int I = y.size(-1);
  gai_silu_mul(x.data_ptr(), y.data_ptr(), y.numel() / I, I, cur_stream());
}

void silu_mul_interleaved(const Tensor& x, Tensor& y) {
  check_bf16(x, "x");
  check_bf16(y, "y");
  const int I = y.size(-1);
  TORCH_CHECK(I % 16 == 0 && x.size(-1) == 2 * I, "silu_mul_interleaved: bad widths");
  gai_silu_mul_interleaved(x.data_ptr(), y.data_ptr(), y.numel() / I, I, cur_stream());
}

void gelu(const Tensor& x, Tensor& y) {
  check_bf16(x, "x");
  check_bf16(y, "y");
  const int I = y.size(-1);
  gai_gelu(x.data_ptr(), y.data_ptr(), y.numel() / I, I, cur_stream());
}

void gelu_tanh(const Tensor& x, Tensor& y) {
  check_bf16(x, "x");
  check_bf16(y, "y");
  const int I = y.size(-1);
  TORCH_CHECK(I % 8 == 0 && x.numel() == y.numel(), "gelu_tanh: width must be a multiple of 8");
  gai_gelu_tanh(x.data_ptr(), y.data_ptr(), y.numel() / I, I, cur_stream());
}

void geglu_interleaved(const Tensor& x, Tensor& y) {
  check_bf16(x, "x");
  check_bf16(y, "y");
  const int I = y.size(-1);
  TORCH_CHECK(I % 16 == 0 && x.size(-1) == 2 * I, "geglu_interleaved: bad widths");
  gai_geglu_interleaved(x.data_ptr(), y.data_ptr(), y.numel() / I, I, cur_stream());
}

void gemv(const Tensor& x, const optional<Tensor>& gamma, double eps, const Tensor& W, int64_t epi,
          const optional<Tensor>& out, const optional<Tensor>& res, bool frag, const optional<Tensor>& swi,
          int64_t ks) {
  check_bf16(W, "W");
  const float* swp = nullptr;
  int M, N = W.size(0), K = W.size(1);
  if (swi) {  // the input is bf16(silu(g) * u) of this fp32 [M, 2K] interleaved gate_up output (x is not read)
    check_f32(*swi, "swi");
    TORCH_CHECK(swi->dim() == 2 && swi->size(1) == 2 * (int64_t)K && W.is_contiguous(), "gemv: swi [M, 2K]");
    M = swi->size(0);
    swp = swi->data_ptr<float>();
  } else {
    check_bf16(x, "x");
    TORCH_CHECK(x.dim() == 2 && W.dim() == 2 && x.size(1) == W.size(1) && x.is_contiguous() && W.is_contiguous(),
                "gemv: x [M, K], W [N, K] contiguous");
    M = x.size(0);
  }
  TORCH_CHECK(gai_gemv_ok(M, N, K, gamma.has_value()), "gemv: shape not supported");
  if (gamma) {
    check_bf16(*gamma, "gamma");
    TORCH_CHECK(gamma->numel() == K, "gemv: gamma [K]");
  }
  void* o = nullptr;
  void* r = nullptr;
  if (epi == 1) {
    TORCH_CHECK(res && res->scalar_type() == at::kBFloat16 && res->is_contiguous() && res->numel() == (int64_t)M * N,
                "gemv: residual [M, N] bf16");
    r = res->data_ptr();
  } else {
    TORCH_CHECK(out && out->is_contiguous(), "gemv: out");
    const int64_t cols = epi == 2 ? N / 2 : N;
    TORCH_CHECK(out->numel() == (int64_t)M * cols * (epi == 5 ? ks : 1), "gemv: out size");
    TORCH_CHECK(out->scalar_type() == (epi == 4 || epi == 5 ? at::kFloat : at::kBFloat16), "gemv: out dtype");
    o = out->data_ptr();
  }
  gai_gemv(swi ? nullptr : x.data_ptr(), gamma ? gamma->data_ptr() : nullptr, (float)eps, W.data_ptr(), M, N, K,
           (int)epi, o, r, cur_stream(), frag ? 1 : 0, swp, (int)ks);
}

void gemv_rope_kv(const Tensor& x, const optional<Tensor>& gamma, double eps, const Tensor& W, const Tensor& pos,
                  const Tensor& cos_sin, const Tensor& slots, Tensor& q_out, Tensor& k_cache, Tensor& v_cache,
                  int64_t Hq, int64_t Hkv, bool frag) {
  check_bf16(x, "x");
  check_bf16(W, "W");
  check_i32(pos, "pos");
  check_i32(slots, "slots");
  check_f32(cos_sin, "cos_sin");
  check_bf16(q_out, "q_out");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  TORCH_CHECK(x.dim() == 2 && W.size(1) == x.size(1) && W.size(0) == (Hq + 2 * Hkv) * 128 && cos_sin.size(-1) == 128,
              "gemv_rope_kv: head_dim 128, W [(Hq + 2 Hkv) * 128, K]");
  TORCH_CHECK(pos.numel() == x.size(0) && slots.numel() == x.size(0), "gemv_rope_kv: pos / slots [M]");
  if (gamma) check_bf16(*gamma, "gamma");
  gai_gemv_rope_kv(x.data_ptr(), gamma ? gamma->data_ptr() : nullptr, (float)eps, W.data_ptr(), x.size(0), x.size(1),
                   pos.data_ptr<int>(), cos_sin.data_ptr<float>(), slots.data_ptr<int>(), q_out.data_ptr(),
                   k_cache.data_ptr(), v_cache.data_ptr(), (int)Hq, (int)Hkv, cur_stream(), frag ? 1 : 0);
}

void custom_all_to_all(const Tensor& inp, Tensor& out, const std::vector<int64_t>& data_ptrs,
                       const std::vector<int64_t>& sig_ptrs, Tensor& counters, Tensor& err, int64_t rank,
                       int64_t slot_bytes, const optional<Tensor>& send_rows, const optional<Tensor>& recv_rows,
                       int64_t row_bytes) {
  check_dev(inp, "inp");
  check_dev(out, "out");
  TORCH_CHECK(inp.is_contiguous() && out.is_contiguous(), "custom_all_to_all: contiguous tensors");
  TORCH_CHECK(inp.scalar_type() == out.scalar_type() && inp.numel() == out.numel(), "custom_all_to_all: in/out mismatch");
  TORCH_CHECK(counters.scalar_type() == at::kInt && counters.numel() >= GAI_AR_MAX_BLOCKS, "custom_all_to_all: counters");
  check_i32(err, "err");
  const int world = (int)data_ptrs.size();
  TORCH_CHECK(world >= 2 && world <= GAI_AR_MAX_WORLD && (int)sig_ptrs.size() == world, "custom_all_to_all: world");
  TORCH_CHECK(rank >= 0 && rank < world, "custom_all_to_all: rank");
  const int64_t bytes = inp.numel() * inp.element_size();
  TORCH_CHECK(bytes % world == 0, "custom_all_to_all: the input must split into equal segments");
  void* d[GAI_AR_MAX_WORLD];
  uint32_t* s[GAI_AR_MAX_WORLD];
  for (int q = 0; q < world; ++q) {
    d[q] = reinterpret_cast<void*>(data_ptrs[q]);
    s[q] = reinterpret_cast<uint32_t*>(sig_ptrs[q]);
  }
  const int* sr = nullptr;
  const int* rr = nullptr;
  if (send_rows || recv_rows) {
    TORCH_CHECK(send_rows && recv_rows, "custom_all_to_all: send_rows and recv_rows go together");
    check_i32(*send_rows, "send_rows");
    check_i32(*recv_rows, "recv_rows");
    TORCH_CHECK(send_rows->numel() == world && recv_rows->numel() == world && send_rows->is_contiguous() &&
                    recv_rows->is_contiguous(), "custom_all_to_all: row counts [world]");
    TORCH_CHECK(row_bytes > 0 && row_bytes % 16 == 0 && (bytes / world) % row_bytes == 0,
                "custom_all_to_all: segments must hold whole rows of a multiple of 16 bytes");
    sr = send_rows->data_ptr<int>();
    rr = recv_rows->data_ptr<int>();
  }
  gai_custom_all_to_all(inp.data_ptr(), out.data_ptr(), bytes / world, d, s,
                        reinterpret_cast<uint32_t*>(counters.data_ptr()), (int)rank, world, slot_bytes,
                        err.data_ptr<int>(), cur_stream(), sr, rr, row_bytes);
}

void ep_pack(const Tensor& x, const Tensor& ids, const Tensor& offs, const Tensor& a_pairs, int64_t W, int64_t C,
             int64_t e_local, Tensor& send, const optional<Tensor>& send_eid) {
  check_bf16(x, "x");
  check_i32(ids, "ids");
  check_i32(offs, "offs");
  check_i32(a_pairs, "a_pairs");
  check_bf16(send, "send");
  TORCH_CHECK(ids.dim() == 2 && x.dim() == 2 && ids.size(0) == x.size(0), "ep_pack: ids [T, k] for x [T, D]");
  TORCH_CHECK(offs.numel() == W + 1 && a_pairs.numel() == ids.numel(), "ep_pack: plan sizes");
  TORCH_CHECK(send.dim() == 2 && send.is_contiguous() && send.size(0) == W * C && send.size(1) >= x.size(1),
              "ep_pack: send slabs [W*C, ld >= D]");
  int* eid = nullptr;
  if (send_eid) {
    check_i32(*send_eid, "send_eid");
    TORCH_CHECK(send_eid->numel() == W * C, "ep_pack: send_eid [W*C]");
    eid = send_eid->data_ptr<int>();
  }
  gai_ep_pack(x.data_ptr(), ids.data_ptr<int>(), offs.data_ptr<int>(), a_pairs.data_ptr<int>(), (int)W, (int)C,
              (int)ids.size(1), (int)x.size(1), (int)send.size(1), (int)e_local, send.data_ptr(), eid, cur_stream());
}

void ep_combine(const Tensor& back, const Tensor& ids, const Tensor& pos, const Tensor& offs, const Tensor& w,
                const optional<Tensor>& residual, int64_t e_local, int64_t C, Tensor& out) {
  check_bf16(back, "back");
  check_i32(ids, "ids");
  check_i32(pos, "pos");
  check_i32(offs, "offs");
  check_f32(w, "w");
  check_bf16(out, "out");
  TORCH_CHECK(ids.dim() == 2 && pos.numel() == ids.numel() && w.numel() == ids.numel(), "ep_combine: plan sizes");
  TORCH_CHECK(out.size(0) == ids.size(0) && out.size(1) == back.size(1), "ep_combine: out [T, D]");
  gai_ep_combine(back.data_ptr(), ids.data_ptr<int>(), pos.data_ptr<int>(), offs.data_ptr<int>(), w.data_ptr<float>(),
                 opt_ptr(residual), out.data_ptr(), (int)ids.size(0), (int)ids.size(1), (int)out.size(1),
                 (int)e_local, (int)C, cur_stream());
}

void moe_dispatch_by(const Tensor& ids, int64_t E, int64_t div, Tensor& a_rows, Tensor& offs, Tensor& pos,
                     Tensor& a_pairs) {
  check_i32(ids, "expert ids");
  check_i32(a_pairs, "a_pairs");
  TORCH_CHECK(ids.is_contiguous() && a_rows.is_contiguous() && offs.is_contiguous() && pos.is_contiguous() &&
              a_pairs.is_contiguous(), "moe_dispatch_by: tensors must be contiguous");
  TORCH_CHECK(ids.dim() == 2 && div >= 1, "moe_dispatch_by: ids [T, k], divisor >= 1");
  const int64_t n = ids.numel();
  TORCH_CHECK(E >= 1 && E <= 2048, "moe_dispatch_by: 1 <= buckets <= 2048");
  TORCH_CHECK(a_rows.numel() == n && pos.numel() == n && a_pairs.numel() == n && offs.numel() == E + 1,
              "moe_dispatch_by: output sizes");
  if (n == 0) return;
  gai_moe_dispatch(ids.data_ptr<int>(), (int)n, (int)ids.size(1), (int)E, a_rows.data_ptr<int>(),
                   offs.data_ptr<int>(), pos.data_ptr<int>(), cur_stream(), (int)div, a_pairs.data_ptr<int>());
}

void custom_allreduce(const Tensor& inp, Tensor& out, const std::vector<int64_t>& data_ptrs,
                      const std::vector<int64_t>& sig_ptrs, Tensor& counters, Tensor& err, int64_t rank,
                      int64_t slot_bytes) {
  check_dev(inp, "inp");
  check_dev(out, "out");
  TORCH_CHECK(inp.scalar_type() == out.scalar_type() && inp.numel() == out.numel(), "custom_allreduce: in/out mismatch");
  TORCH_CHECK(inp.scalar_type() == at::kBFloat16 || inp.scalar_type() == at::kFloat, "custom_allreduce: bf16 or fp32");
  TORCH_CHECK(counters.scalar_type() == at::kInt && counters.numel() >= GAI_AR_MAX_BLOCKS, "custom_allreduce: counters");
  check_i32(err, "err");
  const int world = (int)data_ptrs.size();
  TORCH_CHECK(world >= 2 && world <= GAI_AR_MAX_WORLD && (int)sig_ptrs.size() == world, "custom_allreduce: world");
  TORCH_CHECK(rank >= 0 && rank < world, "custom_allreduce: rank");
  void* d[GAI_AR_MAX_WORLD];
  uint32_t* s[GAI_AR_MAX_WORLD];
  for (int q = 0; q < world; ++q) {
    d[q] = reinterpret_cast<void*>(data_ptrs[q]);
    s[q] = reinterpret_cast<uint32_t*>(sig_ptrs[q]);
  }
  gai_custom_allreduce(inp.data_ptr(), out.data_ptr(), inp.numel() * inp.element_size(),
                       inp.scalar_type() == at::kFloat, d, s, reinterpret_cast<uint32_t*>(counters.data_ptr()),
                       (int)rank, world, slot_bytes, err.data_ptr<int>(), cur_stream());
}

static void ar_peers(const std::vector<int64_t>& data_ptrs, const std::vector<int64_t>& sig_ptrs, int64_t rank,
                     void** d, uint32_t** s) {
  const int world = (int)data_ptrs.size();
  TORCH_CHECK(world >= 2 && world <= GAI_AR_MAX_WORLD && (int)sig_ptrs.size() == world, "custom_allreduce: world");
  TORCH_CHECK(rank >= 0 && rank < world, "custom_allreduce: rank");
  for (int q = 0; q < world; ++q) {
    d[q] = reinterpret_cast<void*>(data_ptrs[q]);
    s[q] = reinterpret_cast<uint32_t*>(sig_ptrs[q]);
  }
}

void custom_allreduce_twoshot(const Tensor& inp, Tensor& out, const std::vector<int64_t>& data_ptrs,
                              const std::vector<int64_t>& sig_ptrs, Tensor& counters, Tensor& err, int64_t rank,
                              int64_t region_bytes) {
  check_dev(inp, "inp");
  check_dev(out, "out");
  TORCH_CHECK(inp.scalar_type() == out.scalar_type() && inp.numel() == out.numel(), "two-shot: in/out mismatch");
  TORCH_CHECK(inp.scalar_type() == at::kBFloat16 || inp.scalar_type() == at::kFloat, "two-shot: bf16 or fp32");
  TORCH_CHECK(inp.is_contiguous() && out.is_contiguous(), "two-shot: contiguous tensors");
  TORCH_CHECK(counters.scalar_type() == at::kInt && counters.numel() >= GAI_AR_MAX_BLOCKS, "two-shot: counters");
  check_i32(err, "err");
  void* d[GAI_AR_MAX_WORLD];
  uint32_t* s[GAI_AR_MAX_WORLD];
  ar_peers(data_ptrs, sig_ptrs, rank, d, s);
  gai_custom_allreduce_twoshot(inp.data_ptr(), out.data_ptr(), inp.numel() * inp.element_size(),
                               inp.scalar_type() == at::kFloat, d, s, reinterpret_cast<uint32_t*>(counters.data_ptr()),
                               (int)rank, (int)data_ptrs.size(), region_bytes, err.data_ptr<int>(), cur_stream());
}

void custom_allreduce_rmsnorm(const Tensor& inp, Tensor& out, Tensor& residual, const Tensor& w, double eps,
                              const std::vector<int64_t>& data_ptrs, const std::vector<int64_t>& sig_ptrs,
                              Tensor& counters, Tensor& err, int64_t rank, int64_t slot_bytes) {
  check_bf16(inp, "inp");
  check_bf16(out, "out");
  check_bf16(residual, "residual");
  check_bf16(w, "w");
  const int D = inp.size(-1);
  TORCH_CHECK(inp.is_contiguous() && out.is_contiguous() && residual.is_contiguous(), "ar_rmsnorm: contiguous");
  TORCH_CHECK(out.numel() == inp.numel() && residual.numel() == inp.numel() && w.numel() == D, "ar_rmsnorm: shapes");
  TORCH_CHECK(counters.scalar_type() == at::kInt && counters.numel() >= GAI_AR_MAX_BLOCKS, "ar_rmsnorm: counters");
  check_i32(err, "err");
  void* d[GAI_AR_MAX_WORLD];
  uint32_t* s[GAI_AR_MAX_WORLD];
  ar_peers(data_ptrs, sig_ptrs, rank, d, s);
  gai_custom_allreduce_rmsnorm(inp.data_ptr(), out.data_ptr(), residual.data_ptr(), w.data_ptr(), inp.numel() / D, D,
                               (float)eps, d, s, reinterpret_cast<uint32_t*>(counters.data_ptr()), (int)rank,
                               (int)data_ptrs.size(), slot_bytes, err.data_ptr<int>(), cur_stream());
}

void gemm_splitk_add_rmsnorm(const Tensor& A, const Tensor& B, const optional<Tensor>& bias, Tensor& res,
                             const Tensor& g, Tensor& out, double eps, Tensor& ws, bool psw) {
  check_bf16(A, "A");
  check_bf16(B, "B");
  check_bf16(res, "res");
  check_bf16(g, "g");
  check_bf16(out, "out");
  const int K = A.size(-1);
  const int M = A.numel() / K;
  const int N = B.size(0);
  TORCH_CHECK(B.size(1) == K && res.numel() == (int64_t)M * N && out.numel() == (int64_t)M * N && g.numel() == N,
              "gemm_splitk_add_rmsnorm: shape mismatch");
  TORCH_CHECK(gai_gemm_splitk_fusable_norm(M, N, K), "gemm_splitk_add_rmsnorm: shape not fusable");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && (size_t)ws.numel() * 4 >= gai_gemm_splitk_ws_bytes(M, N, K),
              "gemm_splitk_add_rmsnorm: workspace too small");
  if (bias) check_bf16(*bias, "bias");
  gai_gemm_splitk_add_rmsnorm(A.data_ptr(), B.data_ptr(), opt_ptr(bias), res.data_ptr(), g.data_ptr(),
                              out.data_ptr(), M, N, K, (float)eps, ws.data_ptr<float>(), psw ? 1 : 0, cur_stream());
}

void gdn_decode(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& g, const Tensor& beta, Tensor& state,
                const Tensor& slots, Tensor& out) {
  check_f32(q, "q");
  check_f32(k, "k");
  check_f32(v, "v");
  check_f32(g, "g");
  check_f32(beta, "beta");
  check_f32(state, "state");
  check_f32(out, "out");
  check_i32(slots, "slots");
  TORCH_CHECK(q.dim() == 3 && k.sizes() == q.sizes() && v.dim() == 3 && state.dim() == 4, "gdn_decode: shapes");
  const int B = q.size(0), Hv = q.size(1), DK = q.size(2), DV = v.size(2);
  TORCH_CHECK(v.size(0) == B && v.size(1) == Hv && g.numel() == (int64_t)B * Hv && beta.numel() == (int64_t)B * Hv,
              "gdn_decode: v / g / beta shapes");
  TORCH_CHECK(state.size(1) == Hv && state.size(2) == DK && state.size(3) == DV && slots.numel() == B &&
                  out.numel() == (int64_t)B * Hv * DV, "gdn_decode: state / slots / out shapes");
  gai_gdn_decode(q.data_ptr<float>(), k.data_ptr<float>(), v.data_ptr<float>(), g.data_ptr<float>(),
                 beta.data_ptr<float>(), state.data_ptr<float>(), slots.data_ptr<int>(), out.data_ptr<float>(), B, Hv,
                 DK, DV, cur_stream());
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 (MI355X) HIP kernels for generativeaiexamples_amd";
  m.def("rmsnorm", &rmsnorm);
  m.def("layernorm", &layernorm);
  m.def("rope_kv_write", &rope_kv_write);
  m.def("gemm", &gemm, pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("C"), pybind11::arg("bias"),
        pybind11::arg("R"), pybind11::arg("epi"), pybind11::arg("force"), pybind11::arg("bfrag") = false);
  m.def("gemm_fp8", &gemm_fp8);
  m.def("gemm_splitk", &gemm_splitk, pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("C"), pybind11::arg("bias"),
        pybind11::arg("R"), pybind11::arg("epi"), pybind11::arg("ws"), pybind11::arg("psw") = false);
  m.def("gemm_rope_kv", &gemm_rope_kv);
  m.def("gemm_dec2_ok", [](int64_t M, int64_t N, int64_t K, int64_t epi) {
    return gai_gemm_dec2_ok((int)M, (int)N, (int)K, (int)epi) != 0;
  });
  m.def("gemm_splitk_ws_floats", [](int64_t M, int64_t N, int64_t K) {
    return (int64_t)(gai_gemm_splitk_ws_bytes(M, N, K) / 4);
  });
  m.def("patchify", &patchify);
  m.def("vit_embed", &vit_embed);
  m.def("quant_rows_fp8", &quant_rows_fp8);
  m.def("attn_prefill", &attn_prefill);
  m.def("kv_pack", &kv_pack);
  m.def("attn_prefill_rows_per_tile", [](int64_t hq, int64_t hkv, int64_t d) { return gai_attn_prefill_rows_per_tile(hq, hkv, d); },
        py::arg("hq"), py::arg("hkv"), py::arg("d") = 128);
  m.def("attn_prefill_set_hl", [](int64_t hl) { gai_attn_prefill_set_hl((int)hl); });
  m.def("attn_decode", &attn_decode, py::arg("q"), py::arg("k_cache"), py::arg("v_cache"), py::arg("block_tables"),
        py::arg("ctx_lens"), py::arg("out"), py::arg("ws_o"), py::arg("ws_ml"), py::arg("scale"), py::arg("split_keys"),
        py::arg("max_splits"), py::arg("k_scale"), py::arg("v_scale"), py::arg("split_cnt") = py::none(),
        py::arg("qkv_part") = py::none(), py::arg("part_ks") = 0, py::arg("positions") = py::none(),
        py::arg("cos_sin") = py::none(), py::arg("slots") = py::none());
  m.def("sample", &sample, py::arg("logits"), py::arg("temperature"), py::arg("top_p"), py::arg("top_k"),
        py::arg("seeds"), py::arg("step"), py::arg("out"), py::arg("ws") = py::none());
  m.def("sample_ws_bytes", &sample_ws_bytes);
  m.def("sample_tp_resolve", &sample_tp_resolve);
  m.def("sample_tp_stats", &sample_tp_stats);
  m.def("apply_penalties", &apply_penalties);
  m.def("token_mask", &token_mask);
  m.def("sim_topk", &sim_topk);
  m.def("topk_merge", [](const Tensor& vals, const Tensor& idx, int64_t k, Tensor& out_v, Tensor& out_i) {
    check_f32(vals, "vals");
    check_i32(idx, "idx");
    TORCH_CHECK(vals.dim() == 3 && idx.sizes() == vals.sizes(), "topk_merge: vals / idx [W, Q, cap]");
    const int cap = (int)vals.size(2);
    TORCH_CHECK(cap == gai_topk_cap(cap) && k >= 1 && k <= cap, "topk_merge: cap must be 4, 8, 16, 32 or 64, k <= cap");
    TORCH_CHECK(out_v.numel() == vals.size(1) * k && out_i.numel() == vals.size(1) * k &&
                    out_i.scalar_type() == at::kLong && out_v.scalar_type() == at::kFloat,
                "topk_merge: outputs [Q, k]");
    gai_topk_merge(vals.data_ptr<float>(), idx.data_ptr<int>(), (int)vals.size(0), (int)vals.size(1), cap, (int)k,
                   out_v.data_ptr<float>(), out_i.data_ptr<int64_t>(), cur_stream());
  });
  m.def("topk_cap", [](int64_t k) { return gai_topk_cap(k); });
  // streaming-SDR DSP: complex64 tensors are passed as their float32 [n, 2] views
  m.def("dsp_fir_complex", [](const Tensor& x, const Tensor& taps, Tensor& y) {
    check_f32(x, "x");
    check_f32(taps, "taps");
    check_f32(y, "y");
    TORCH_CHECK(x.dim() == 2 && x.size(1) == 2 && y.sizes() == x.sizes() && taps.dim() == 1 && x.is_contiguous() &&
                    y.is_contiguous() && taps.is_contiguous(),
                "dsp_fir_complex: x / y [n, 2] float32 (complex64 views), taps [T]");
    gai_dsp_fir_complex(x.data_ptr(), taps.data_ptr<float>(), (int)x.size(0), (int)taps.numel(), y.data_ptr(),
                        cur_stream());
  });
  m.def("dsp_fm_demod", [](const Tensor& x, Tensor& y) {
    check_f32(x, "x");
    check_f32(y, "y");
    TORCH_CHECK(x.dim() == 2 && x.size(1) == 2 && y.numel() == std::max<int64_t>(x.size(0) - 1, 0) &&
                    x.is_contiguous() && y.is_contiguous(),
                "dsp_fm_demod: x [n, 2] (complex64 view), y [n - 1]");
    gai_dsp_fm_demod(x.data_ptr(), (int)x.size(0), y.data_ptr<float>(), cur_stream());
  });
  m.def("dsp_upfirdn", [](const Tensor& x, const Tensor& taps, int64_t up, int64_t down, int64_t offset, double gain,
                          Tensor& y) {
    check_f32(x, "x");
    check_f32(taps, "taps");
    check_f32(y, "y");
    TORCH_CHECK(x.dim() == 1 && taps.dim() == 1 && y.dim() == 1 && x.is_contiguous() && taps.is_contiguous() &&
                    y.is_contiguous(),
                "dsp_upfirdn: 1-D contiguous float32 x, taps, y");
    gai_dsp_upfirdn(x.data_ptr<float>(), (int)x.numel(), taps.data_ptr<float>(), (int)taps.numel(), (int)up,
                    (int)down, (int)offset, (int)y.numel(), (float)gain, y.data_ptr<float>(), cur_stream());
  });
  m.def("moe_route", &moe_route);
  m.def("moe_gemm", &moe_gemm);
  m.def("moe_combine", &moe_combine);
  m.def("moe_dispatch", &moe_dispatch);
  m.def("moe_dispatch_by", &moe_dispatch_by);
  m.def("ep_pack", &ep_pack);
  m.def("ep_combine", &ep_combine);
  m.def("custom_all_to_all", &custom_all_to_all);
  m.def("gemm_qkv_partials", &gemm_qkv_partials);
  m.def("gemv", &gemv, pybind11::arg("x"), pybind11::arg("gamma"), pybind11::arg("eps"), pybind11::arg("W"),
        pybind11::arg("epi"), pybind11::arg("out"), pybind11::arg("res"), pybind11::arg("frag") = false,
        pybind11::arg("swi") = pybind11::none(), pybind11::arg("ks") = 1);
  m.def("gemv_rope_kv", &gemv_rope_kv, pybind11::arg("x"), pybind11::arg("gamma"), pybind11::arg("eps"),
        pybind11::arg("W"), pybind11::arg("pos"), pybind11::arg("cos_sin"), pybind11::arg("slots"),
        pybind11::arg("q_out"), pybind11::arg("k_cache"), pybind11::arg("v_cache"), pybind11::arg("Hq"),
        pybind11::arg("Hkv"), pybind11::arg("frag") = false);
  m.def("embedding", &embedding);
  m.def("decode_advance", &decode_advance);
  m.def("pool", &pool);
  m.def("silu_mul", &silu_mul);
  m.def("gelu", &gelu);
  m.def("gelu_tanh", &gelu_tanh);
  m.def("geglu_interleaved", &geglu_interleaved);
  m.def("silu_mul_interleaved", &silu_mul_interleaved);
  m.def("gemm_splitk_add_rmsnorm", &gemm_splitk_add_rmsnorm);
  m.def("gemm_splitk_fusable_norm", [](int64_t M, int64_t N, int64_t K) { return gai_gemm_splitk_fusable_norm(M, N, K) != 0; });
  m.def("gdn_decode", &gdn_decode);
  m.def("custom_allreduce", &custom_allreduce);
  m.def("custom_allreduce_twoshot", &custom_allreduce_twoshot);
  m.def("custom_allreduce_rmsnorm", &custom_allreduce_rmsnorm);
  m.def("ipc_malloc", [](int64_t bytes) { return reinterpret_cast<int64_t>(gai_ipc_malloc(bytes)); });
  m.def("ipc_free", [](int64_t p) { gai_ipc_free(reinterpret_cast<void*>(p)); });
  m.def("ipc_get_handle", [](int64_t p) {
    char h[64] = {0};
    gai_ipc_get_handle(reinterpret_cast<void*>(p), h);
    return pybind11::bytes(h, 64);
  });
  m.def("ipc_open", [](pybind11::bytes h) {
    std::string b = h;
    TORCH_CHECK(b.size() == 64, "ipc_open: handle must be 64 bytes");
    return reinterpret_cast<int64_t>(gai_ipc_open(b.data()));
  });
  m.def("ipc_close", [](int64_t p) { gai_ipc_close(reinterpret_cast<void*>(p)); });
  m.attr("AR_CHUNK") = GAI_AR_CHUNK;
  m.attr("AR_MAX_BLOCKS") = GAI_AR_MAX_BLOCKS;
  m.attr("ARCH") = "gfx950";
}
