#include "block_manager.h"

#include <stdexcept>

namespace gai {

BlockManager::BlockManager(int num_blocks, bool enable_prefix_cache)
    : blocks_(num_blocks), prefix_cache_(enable_prefix_cache) {
  free_.reserve(num_blocks);
  for (int i = num_blocks - 1; i >= 0; --i) free_.push_back(i);
}

int BlockManager::alloc() {
  int b;
  if (!free_.empty()) {
    b = free_.back();
    free_.pop_back();
  } else if (!lru_.empty()) {
    b = lru_.front();
    lru_.pop_front();
    BlockInfo& bi = blocks_[b];
    bi.in_lru = false;
    if (bi.hashed) {
      auto it = by_hash_.find(bi.hash);
      if (it != by_hash_.end() && it->second == b) by_hash_.erase(it);
      bi.hashed = false;
    }
  } else {
    return -1;
  }
  blocks_[b].ref = 1;
  return b;
}

void BlockManager::incref(int b) {
  BlockInfo& bi = blocks_.at(b);
  if (bi.ref == 0 && bi.in_lru) {
    lru_.erase(bi.lru_it);
    bi.in_lru = false;
  }
  ++bi.ref;
}

void BlockManager::decref(int b) {
  BlockInfo& bi = blocks_.at(b);
  if (bi.ref <= 0) throw std::runtime_error("BlockManager: double free of block " + std::to_string(b));
  if (--bi.ref == 0) {
    if (bi.hashed && prefix_cache_) {
      lru_.push_back(b);
      bi.lru_it = std::prev(lru_.end());
      bi.in_lru = true;
    } else {
      bi.hashed = false;
      free_.push_back(b);
    }
  }
}

uint64_t BlockManager::chain_hash(uint64_t parent, const int* toks, int n) {
  // FNV-1a over (parent, tokens) followed by a splitmix finaliser
  uint64_t h = 1469598103934665603ull ^ (parent * 0x9E3779B97F4A7C15ull);
  for (int i = 0; i < n; ++i) {
    h ^= (uint64_t)(uint32_t)toks[i];
    h *= 1099511628211ull;
  }
  h ^= h >> 31;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 27;
  return h | 1ull;  // never 0
}

std::vector<int> BlockManager::match_prefix(const std::vector<int>& tokens, int max_blocks) {
  std::vector<int> out;
  if (!prefix_cache_) return out;
  ++queries_;
  uint64_t h = 0;
  const int nfull = (int)tokens.size() / kBlockSize;
  for (int i = 0; i < nfull && i < max_blocks; ++i) {
    h = chain_hash(h, tokens.data() + i * kBlockSize, kBlockSize);
    auto it = by_hash_.find(h);
    if (it == by_hash_.end()) break;
    incref(it->second);
    out.push_back(it->second);
  }
  if (!out.empty()) ++hits_;
  return out;
}

void BlockManager::commit(int b, uint64_t hash) {
  if (!prefix_cache_) return;
  BlockInfo& bi = blocks_.at(b);
  if (bi.hashed) return;
  auto it = by_hash_.find(hash);
  if (it != by_hash_.end()) return;  // identical content already cached elsewhere
  bi.hash = hash;
  bi.hashed = true;
  by_hash_[hash] = b;
}

}  // namespace gai
