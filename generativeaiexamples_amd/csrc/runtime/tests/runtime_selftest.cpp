// Randomised self-test of the native runtime (BlockManager + Scheduler), built with
// -fsanitize=address,undefined by tools/sanitize_runtime.sh (SURVEY §5.2 "ASan/UBSan on the C++ host
// runtime"). Drives thousands of add / schedule / append / finish / abort operations with random
// prompts (shared prefixes to exercise the prefix cache, tiny KV pools to force preemption) and
// checks the invariants after every step:
//   * no KV block is owned twice and every running sequence's blocks cover its computed tokens;
//   * the step's flat arrays are consistent (sizes, cu_q monotone, slots inside owned blocks);
//   * after everything finishes every block is free again (no leak).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <unordered_map>
#include <vector>

#include "../block_manager.h"
#include "../scheduler.h"

using namespace gai;

#define CHECK(c, ...)                                                  \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::fprintf(stderr, __VA_ARGS__);                               \
      std::fprintf(stderr, "\n");                                      \
      std::exit(1);                                                    \
    }                                                                  \
  } while (0)

static int run(uint32_t seed, int num_blocks, bool prefix, int chunk) {
  std::mt19937 rng(seed);
  const int max_seqs = 8, max_tokens = 256, max_len = 512;
  Scheduler s(num_blocks, max_seqs, max_tokens, max_len, prefix, chunk);
  std::vector<int> shared(96);
  for (auto& t : shared) t = rng() % 1000;
  std::unordered_map<int64_t, int> remaining;
  int64_t next = 1, steps = 0, finished = 0;
  for (int it = 0; it < 4000; ++it) {
    const int op = rng() % 10;
    if (op < 3 && remaining.size() < 24) {
      std::vector<int> p;
      if (rng() % 2) p.assign(shared.begin(), shared.begin() + 16 * (1 + rng() % 6));
      const int extra = 1 + rng() % 200;
      for (int i = 0; i < extra; ++i) p.push_back(rng() % 1000);
      if ((int)p.size() > max_len - 8) p.resize(max_len - 8);
      const int mx = 1 + rng() % 40;
      s.add(next, p, mx, 0);
      remaining[next++] = mx;
    } else if (op == 3 && !remaining.empty()) {
      auto itr = remaining.begin();
      std::advance(itr, rng() % remaining.size());
      s.abort(itr->first);
      remaining.erase(itr);
    } else {
      StepBatch b = s.schedule();
      ++steps;
      const size_t T = b.token_ids.size();
      CHECK(b.positions.size() == T && b.slots.size() == T, "flat array sizes");
      CHECK((int)T == b.num_prefill_tokens + (int)b.decode_seq_ids.size(), "token count");
      CHECK(b.cu_q.size() == b.prefill_seq_ids.size() + (b.prefill_seq_ids.empty() ? b.cu_q.size() : 1),
            "cu_q size");
      for (size_t i = 1; i < b.cu_q.size(); ++i) CHECK(b.cu_q[i] >= b.cu_q[i - 1], "cu_q monotone");
      std::set<int> slots;
      for (size_t i = 0; i < T; ++i) {
        CHECK(b.slots[i] >= 0 && b.slots[i] < num_blocks * kBlockSize, "slot range %d", b.slots[i]);
        CHECK(slots.insert(b.slots[i]).second, "slot %d written twice in one step", b.slots[i]);
      }
      for (size_t j = 0; j < b.decode_seq_ids.size(); ++j) {
        const int ctx = b.decode_ctx[j];
        const int nb = (ctx + kBlockSize - 1) / kBlockSize;
        CHECK(nb <= b.max_blocks, "decode block table too short");
        for (int k = 0; k < nb; ++k) {
          const int blk = b.decode_block_tables[j * b.max_blocks + k];
          CHECK(blk >= 0 && blk < num_blocks, "decode block %d", blk);
        }
      }
      // sample one token for every sequence that produced logits
      std::vector<int64_t> ids;
      std::vector<int> toks;
      for (size_t i = 0; i < b.prefill_seq_ids.size(); ++i)
        if (b.prefill_samples[i]) ids.push_back(b.prefill_seq_ids[i]);
      for (auto id : b.decode_seq_ids) ids.push_back(id);
      std::vector<int64_t> keep;
      for (auto id : ids) {
        auto r = remaining.find(id);
        if (r == remaining.end()) continue;
        if (--r->second <= 0 || rng() % 50 == 0) {
          s.finish(id);
          remaining.erase(r);
          ++finished;
        } else {
          keep.push_back(id);
          toks.push_back(rng() % 1000);
        }
      }
      s.append_tokens(keep, toks);
    }
  }
  // drain
  for (int guard = 0; s.has_work() && guard < 20000; ++guard) {
    StepBatch b = s.schedule();
    std::vector<int64_t> ids;
    for (size_t i = 0; i < b.prefill_seq_ids.size(); ++i)
      if (b.prefill_samples[i]) ids.push_back(b.prefill_seq_ids[i]);
    for (auto id : b.decode_seq_ids) ids.push_back(id);
    std::vector<int64_t> keep;
    std::vector<int> toks;
    for (auto id : ids) {
      auto r = remaining.find(id);
      if (r == remaining.end()) continue;
      if (--r->second <= 0) {
        s.finish(id);
        remaining.erase(r);
      } else {
        keep.push_back(id);
        toks.push_back(1);
      }
    }
    s.append_tokens(keep, toks);
  }
  CHECK(!s.has_work(), "scheduler did not drain");
  CHECK(s.num_free_blocks() == num_blocks, "block leak: %d of %d free", s.num_free_blocks(), num_blocks);
  std::printf("seed %u blocks %d prefix %d chunk %d: %lld steps, %lld finished, hit rate %.3f\n", seed, num_blocks,
              (int)prefix, chunk, (long long)steps, (long long)finished, s.prefix_hit_rate());
  return 0;
}

int main(int argc, char** argv) {
  const int seeds = argc > 1 ? std::atoi(argv[1]) : 8;
  for (int sd = 0; sd < seeds; ++sd) {
    run(1000 + sd, 48 + 16 * (sd % 4), sd % 2 == 0, sd % 3 == 0 ? 64 : 256);
  }
  std::printf("runtime selftest OK\n");
  return 0;
}
