// Paged KV-cache block manager with hash-based prefix caching.
//
// Replaces the KV management inside the reference's external TRT-LLM/NIM
// containers. Blocks hold 16 tokens. A block that
// is completely filled by a sequence gets a content hash chained on its parent
// block's hash; later sequences whose prompt starts with the same tokens (the RAG
// system prompt, a shared retrieved context) reuse those blocks by reference
// count instead of recomputing them. Freed hashed blocks stay cached on an LRU list
// and are only reclaimed under memory pressure.
#pragma once

#include <cstdint>
#include <list>
#include <unordered_map>
#include <vector>

namespace gai {

constexpr int kBlockSize = 16;

struct BlockInfo {
  int ref = 0;
  uint64_t hash = 0;
  bool hashed = false;
  std::list<int>::iterator lru_it;
  bool in_lru = false;
};

class BlockManager {
 public:
  explicit BlockManager(int num_blocks, bool enable_prefix_cache = true);

  int num_blocks() const { return (int)blocks_.size(); }
  int num_free() const { return (int)free_.size() + (int)lru_.size(); }
  bool can_allocate(int n_blocks) const { return num_free() >= n_blocks; }

  // Allocate one fresh block (reclaims an LRU cached block if the free list is empty). -1 if none.
  int alloc();
  void incref(int b);
  void decref(int b);

  // Prefix caching: chained hashes of full blocks of `tokens`.
  static uint64_t chain_hash(uint64_t parent, const int* toks, int n);
  // Returns the longest run of cached full blocks matching the token prefix (refcounts taken).
  std::vector<int> match_prefix(const std::vector<int>& tokens, int max_blocks);
  // Registers block `b` (full) under `hash`.
  void commit(int b, uint64_t hash);

  int64_t hits() const { return hits_; }
  int64_t queries() const { return queries_; }

 private:
  std::vector<BlockInfo> blocks_;
  std::vector<int> free_;
  std::list<int> lru_;  // cached blocks with ref == 0 (front = oldest)
  std::unordered_map<uint64_t, int> by_hash_;
  bool prefix_cache_;
  int64_t hits_ = 0, queries_ = 0;
};

}  // namespace gai
