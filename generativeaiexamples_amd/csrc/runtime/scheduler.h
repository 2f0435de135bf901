// Continuous-batching scheduler core (native replacement for the in-engine
// scheduler of the reference's TRT-LLM/vLLM NIM containers).
//
// One unified step: running decodes get one token each, partially prefilled
// prompts continue (chunked prefill), then waiting requests are admitted while the
// token budget, the sequence cap and the KV blocks allow (prefix-cache hits are
// skipped over). When a running sequence cannot get a KV slot the youngest running
// sequence is preempted (blocks freed, recomputed later). The step is flattened
// into the int32 arrays the model runner consumes (token ids, positions, slot
// mapping, varlen prefill metadata, decode block tables) so the Python side does
// no per-token work.
#pragma once

#include <cstdint>
#include <deque>
#include <memory>
#include <unordered_map>
#include <vector>

#include "block_manager.h"

namespace gai {

struct Sequence {
  int64_t id;
  std::vector<int> tokens;  // prompt + generated
  int prompt_len;
  int num_computed = 0;     // tokens whose KV is in the cache
  int max_new_tokens;
  std::vector<int> blocks;
  uint64_t last_hash = 0;   // chain hash of the last committed full block
  int num_hashed = 0;       // full blocks committed to the prefix cache
  int priority = 0;
  bool finished = false;
  int num_generated() const { return (int)tokens.size() - prompt_len; }
};

struct StepBatch {
  // flat token arrays: prefill tokens first, then decode tokens
  std::vector<int32_t> token_ids, positions, slots;
  // prefill part
  std::vector<int64_t> prefill_seq_ids;
  std::vector<int32_t> cu_q, prefill_ctx, prefill_qlen;
  std::vector<int32_t> prefill_block_tables;  // [P, max_blocks]
  std::vector<uint8_t> prefill_samples;       // 1 if this chunk completes the prompt (sample a token)
  // decode part
  std::vector<int64_t> decode_seq_ids;
  std::vector<int32_t> decode_ctx;
  std::vector<int32_t> decode_block_tables;   // [D, max_blocks]
  std::vector<int64_t> preempted;
  int max_blocks = 0;
  int num_prefill_tokens = 0;
};

class Scheduler {
 public:
  Scheduler(int num_blocks, int max_num_seqs, int max_batched_tokens, int max_model_len, bool prefix_cache,
            int prefill_chunk);

  void add(int64_t id, const std::vector<int>& prompt, int max_new_tokens, int priority);
  bool abort(int64_t id);
  // Appends sampled tokens for the sequences sampled in the last step. Returns ids that can no longer grow
  // (max_new_tokens or max_model_len reached); the caller decides EOS/stop and calls finish().
  void append_tokens(const std::vector<int64_t>& ids, const std::vector<int>& toks);
  void finish(int64_t id);

  StepBatch schedule();

  // Multi-step decode. After schedule() returned a pure-decode batch for `ids`, reserve KV pages so
  // each of them can run `steps` tokens (positions num_computed-1 .. num_computed+steps-2) with no
  // further scheduling; fills the [ids.size(), max_blocks] block tables. All-or-nothing: returns
  // false and allocates nothing when the free pool is short.
  bool reserve_decode(const std::vector<int64_t>& ids, int steps, std::vector<int32_t>& block_tables,
                      int& max_blocks);
  // After such a run: appends `steps` sampled tokens per id (toks is [ids.size(), steps] row-major)
  // and marks steps-1 more of them as computed (the last sampled token is the next step's input).
  // chained = the run's first input was the previous run's last token, fed on the device (pipelined
  // runs, LLMEngine): that token was not scheduled by schedule(), so all `steps` positions are computed.
  void advance_decode(const std::vector<int64_t>& ids, const std::vector<int>& toks, int steps, bool chained = false);
  // Pipelined multi-step decode: make every sequence ids[i] own the KV pages of its first upto[i] token
  // positions (absolute counts, <= max_model_len), all-or-nothing, and fill the block tables as
  // reserve_decode does. Used to reserve run r+1 while run r is still executing on the device.
  bool reserve_upto(const std::vector<int64_t>& ids, const std::vector<int>& upto, std::vector<int32_t>& block_tables,
                    int& max_blocks);

  int num_waiting() const { return (int)waiting_.size(); }
  int num_running() const { return (int)running_.size(); }
  int num_free_blocks() const { return bm_.num_free(); }
  int num_blocks() const { return bm_.num_blocks(); }
  double prefix_hit_rate() const { return bm_.queries() ? (double)bm_.hits() / bm_.queries() : 0.0; }
  bool has_work() const { return !waiting_.empty() || !running_.empty(); }
  int num_tokens(int64_t id) const;
  int num_generated(int64_t id) const;

 private:
  bool ensure_blocks(Sequence& s, int upto_tokens);
  void release(Sequence& s);
  void commit_full_blocks(Sequence& s);
  void preempt(Sequence& s);

  BlockManager bm_;
  int max_num_seqs_, max_batched_tokens_, max_model_len_, prefill_chunk_;
  std::unordered_map<int64_t, std::unique_ptr<Sequence>> seqs_;
  std::deque<int64_t> waiting_;
  std::vector<int64_t> running_;  // admission order
};

}  // namespace gai
