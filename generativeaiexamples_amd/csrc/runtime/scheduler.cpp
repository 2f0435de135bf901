#include "scheduler.h"

#include <algorithm>
#include <stdexcept>

namespace gai {

Scheduler::Scheduler(int num_blocks, int max_num_seqs, int max_batched_tokens, int max_model_len, bool prefix_cache,
                     int prefill_chunk)
    : bm_(num_blocks, prefix_cache),
      max_num_seqs_(max_num_seqs),
      max_batched_tokens_(max_batched_tokens),
      max_model_len_(max_model_len),
      prefill_chunk_(prefill_chunk > 0 ? prefill_chunk : max_batched_tokens) {}

void Scheduler::add(int64_t id, const std::vector<int>& prompt, int max_new_tokens, int priority) {
  if (prompt.empty()) throw std::runtime_error("Scheduler.add: empty prompt");
  if (seqs_.count(id)) throw std::runtime_error("Scheduler.add: duplicate id");
  if ((int)prompt.size() >= max_model_len_) throw std::runtime_error("Scheduler.add: prompt exceeds max_model_len");
  auto s = std::make_unique<Sequence>();
  s->id = id;
  s->tokens = prompt;
  s->prompt_len = (int)prompt.size();
  s->max_new_tokens = max_new_tokens;
  s->priority = priority;
  seqs_[id] = std::move(s);
  waiting_.push_back(id);
}

void Scheduler::release(Sequence& s) {
  for (int b : s.blocks) bm_.decref(b);
  s.blocks.clear();
}

bool Scheduler::abort(int64_t id) {
  auto it = seqs_.find(id);
  if (it == seqs_.end()) return false;
  release(*it->second);
  running_.erase(std::remove(running_.begin(), running_.end(), id), running_.end());
  waiting_.erase(std::remove(waiting_.begin(), waiting_.end(), id), waiting_.end());
  seqs_.erase(it);
  return true;
}

void Scheduler::finish(int64_t id) { abort(id); }

int Scheduler::num_tokens(int64_t id) const {
  auto it = seqs_.find(id);
  return it == seqs_.end() ? -1 : (int)it->second->tokens.size();
}

int Scheduler::num_generated(int64_t id) const {
  auto it = seqs_.find(id);
  return it == seqs_.end() ? -1 : it->second->num_generated();
}

void Scheduler::append_tokens(const std::vector<int64_t>& ids, const std::vector<int>& toks) {
  if (ids.size() != toks.size()) throw std::runtime_error("append_tokens: size mismatch");
  for (size_t i = 0; i < ids.size(); ++i) {
    auto it = seqs_.find(ids[i]);
    if (it == seqs_.end()) continue;  // aborted meanwhile
    it->second->tokens.push_back(toks[i]);
  }
}

bool Scheduler::ensure_blocks(Sequence& s, int upto_tokens) {
  const int need = (upto_tokens + kBlockSize - 1) / kBlockSize - (int)s.blocks.size();
  if (need <= 0) return true;
  if (!bm_.can_allocate(need)) return false;
  for (int i = 0; i < need; ++i) s.blocks.push_back(bm_.alloc());
  return true;
}

void Scheduler::commit_full_blocks(Sequence& s) {
  const int full = s.num_computed / kBlockSize;
  while (s.num_hashed < full) {
    const int i = s.num_hashed;
    s.last_hash = BlockManager::chain_hash(s.last_hash, s.tokens.data() + (size_t)i * kBlockSize, kBlockSize);
    bm_.commit(s.blocks[i], s.last_hash);
    ++s.num_hashed;
  }
}

void Scheduler::preempt(Sequence& s) {
  release(s);
  s.num_computed = 0;
  s.num_hashed = 0;
  s.last_hash = 0;
  running_.erase(std::remove(running_.begin(), running_.end(), s.id), running_.end());
  waiting_.push_front(s.id);
}

StepBatch Scheduler::schedule() {
  StepBatch b;
  int budget = max_batched_tokens_;

  // ---- 1. make room for all running decodes (preempt youngest first)
  auto decode_block_need = [&]() {
    int n = 0;
    for (int64_t id : running_) {
      const Sequence& s = *seqs_[id];
      const int rem = (int)s.tokens.size() - s.num_computed;
      if (rem == 1 && (int)s.blocks.size() * kBlockSize <= s.num_computed) ++n;
    }
    return n;
  };
  while (!running_.empty() && decode_block_need() > bm_.num_free()) {
    b.preempted.push_back(running_.back());
    preempt(*seqs_[running_.back()]);
  }

  struct Chunk {
    Sequence* s;
    int start, n;
  };
  std::vector<Chunk> prefills;
  std::vector<Sequence*> decodes;

  for (int64_t id : running_) {
    Sequence& s = *seqs_[id];
    const int rem = (int)s.tokens.size() - s.num_computed;
    if (rem == 1 && budget > 0) {
      if (!ensure_blocks(s, s.num_computed + 1)) continue;  // cannot happen after the pre-check
      decodes.push_back(&s);
      --budget;
    }
  }
  // ---- 2. continue partially prefilled running sequences
  for (int64_t id : running_) {
    Sequence& s = *seqs_[id];
    const int rem = (int)s.tokens.size() - s.num_computed;
    if (rem <= 1 || budget <= 0) continue;
    int n = std::min({rem, budget, prefill_chunk_});
    const int room = ((int)s.blocks.size() + bm_.num_free()) * kBlockSize - s.num_computed;
    n = std::min(n, room);
    if (n <= 0) continue;
    ensure_blocks(s, s.num_computed + n);
    prefills.push_back({&s, s.num_computed, n});
    budget -= n;
  }
  // ---- 3. admit waiting sequences
  while (!waiting_.empty() && budget > 0 && (int)running_.size() < max_num_seqs_) {
    Sequence& s = *seqs_[waiting_.front()];
    if (s.blocks.empty() && s.num_computed == 0) {
      // prefix cache: never match the last token (its logits are needed)
      const int maxb = ((int)s.tokens.size() - 1) / kBlockSize;
      s.blocks = bm_.match_prefix(s.tokens, maxb);
      s.num_computed = (int)s.blocks.size() * kBlockSize;
      s.num_hashed = (int)s.blocks.size();
      s.last_hash = 0;
      for (int i = 0; i < s.num_hashed; ++i)
        s.last_hash = BlockManager::chain_hash(s.last_hash, s.tokens.data() + (size_t)i * kBlockSize, kBlockSize);
    }
    const int rem = (int)s.tokens.size() - s.num_computed;
    int n = std::min({rem, budget, prefill_chunk_});
    const int room = ((int)s.blocks.size() + bm_.num_free()) * kBlockSize - s.num_computed;
    n = std::min(n, room);
    if (n <= 0) break;  // out of KV blocks: wait for running sequences to finish
    waiting_.pop_front();
    running_.push_back(s.id);
    ensure_blocks(s, s.num_computed + n);
    if (rem == 1)
      decodes.push_back(&s);  // fully prefix-cached prompt but one token: treat as decode
    else
      prefills.push_back({&s, s.num_computed, n});
    budget -= n;
  }

  // ---- 4. flatten
  int maxb = 0;
  for (auto& c : prefills) maxb = std::max(maxb, (int)c.s->blocks.size());
  for (auto* s : decodes) maxb = std::max(maxb, (int)s->blocks.size());
  b.max_blocks = std::max(maxb, 1);
  b.cu_q.push_back(0);
  for (auto& c : prefills) {
    Sequence& s = *c.s;
    for (int i = 0; i < c.n; ++i) {
      const int pos = c.start + i;
      b.token_ids.push_back(s.tokens[pos]);
      b.positions.push_back(pos);
      b.slots.push_back(s.blocks[pos / kBlockSize] * kBlockSize + pos % kBlockSize);
    }
    b.prefill_seq_ids.push_back(s.id);
    b.cu_q.push_back(b.cu_q.back() + c.n);
    b.prefill_ctx.push_back(c.start + c.n);
    b.prefill_qlen.push_back(c.n);
    b.prefill_samples.push_back(c.start + c.n == (int)s.tokens.size() ? 1 : 0);
    for (int j = 0; j < b.max_blocks; ++j)
      b.prefill_block_tables.push_back(j < (int)s.blocks.size() ? s.blocks[j] : 0);
    s.num_computed = c.start + c.n;
    commit_full_blocks(s);
  }
  b.num_prefill_tokens = (int)b.token_ids.size();
  for (auto* sp : decodes) {
    Sequence& s = *sp;
    const int pos = s.num_computed;
    b.token_ids.push_back(s.tokens[pos]);
    b.positions.push_back(pos);
    b.slots.push_back(s.blocks[pos / kBlockSize] * kBlockSize + pos % kBlockSize);
    b.decode_seq_ids.push_back(s.id);
    b.decode_ctx.push_back(pos + 1);
    for (int j = 0; j < b.max_blocks; ++j) b.decode_block_tables.push_back(j < (int)s.blocks.size() ? s.blocks[j] : 0);
    s.num_computed = pos + 1;
    commit_full_blocks(s);
  }
  return b;
}

bool Scheduler::reserve_decode(const std::vector<int64_t>& ids, int steps, std::vector<int32_t>& block_tables,
                               int& max_blocks) {
  if (steps < 1) throw std::runtime_error("reserve_decode: steps must be >= 1");
  int need = 0;
  for (int64_t id : ids) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) throw std::runtime_error("reserve_decode: unknown sequence");
    const Sequence& s = *it->second;
    const int upto = s.num_computed + steps - 1;
    if (upto > max_model_len_) return false;
    need += std::max(0, (upto + kBlockSize - 1) / kBlockSize - (int)s.blocks.size());
  }
  if (need > 0 && !bm_.can_allocate(need)) return false;
  max_blocks = 1;
  for (int64_t id : ids) {
    Sequence& s = *seqs_[id];
    ensure_blocks(s, s.num_computed + steps - 1);
    max_blocks = std::max(max_blocks, (int)s.blocks.size());
  }
  block_tables.assign(ids.size() * (size_t)max_blocks, 0);
  for (size_t i = 0; i < ids.size(); ++i) {
    const Sequence& s = *seqs_[ids[i]];
    std::copy(s.blocks.begin(), s.blocks.end(), block_tables.begin() + i * (size_t)max_blocks);
  }
  return true;
}

bool Scheduler::reserve_upto(const std::vector<int64_t>& ids, const std::vector<int>& upto,
                             std::vector<int32_t>& block_tables, int& max_blocks) {
  if (upto.size() != ids.size()) throw std::runtime_error("reserve_upto: size mismatch");
  int need = 0;
  for (size_t i = 0; i < ids.size(); ++i) {
    auto it = seqs_.find(ids[i]);
    if (it == seqs_.end()) throw std::runtime_error("reserve_upto: unknown sequence");
    if (upto[i] > max_model_len_) return false;
    need += std::max(0, (upto[i] + kBlockSize - 1) / kBlockSize - (int)it->second->blocks.size());
  }
  if (need > 0 && !bm_.can_allocate(need)) return false;
  max_blocks = 1;
  for (size_t i = 0; i < ids.size(); ++i) {
    Sequence& s = *seqs_[ids[i]];
    ensure_blocks(s, upto[i]);
    max_blocks = std::max(max_blocks, (int)s.blocks.size());
  }
  block_tables.assign(ids.size() * (size_t)max_blocks, 0);
  for (size_t i = 0; i < ids.size(); ++i) {
    const Sequence& s = *seqs_[ids[i]];
    std::copy(s.blocks.begin(), s.blocks.end(), block_tables.begin() + i * (size_t)max_blocks);
  }
  return true;
}

void Scheduler::advance_decode(const std::vector<int64_t>& ids, const std::vector<int>& toks, int steps, bool chained) {
  if (toks.size() != ids.size() * (size_t)steps) throw std::runtime_error("advance_decode: size mismatch");
  for (size_t i = 0; i < ids.size(); ++i) {
    auto it = seqs_.find(ids[i]);
    if (it == seqs_.end()) continue;  // finished / aborted during the run
    Sequence& s = *it->second;
    s.tokens.insert(s.tokens.end(), toks.begin() + i * steps, toks.begin() + (i + 1) * steps);
    s.num_computed += chained ? steps : steps - 1;
    if ((int)s.blocks.size() * kBlockSize < s.num_computed)
      throw std::runtime_error("advance_decode: sequence advanced past its reserved pages");
    commit_full_blocks(s);
  }
}

}  // namespace gai
