// Randomized self-test of the constrained-decoding matcher (grammar.cpp), built with ASan/UBSan by
// tools/sanitize_runtime.sh: random walks over the allowed tokens of a byte vocabulary must always
// complete within their budget and end in a finished value.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "grammar.h"

using namespace gai;

static GNode obj(std::vector<std::string> keys, std::vector<int> props, std::vector<char> req) {
  GNode n;
  n.kind = G_OBJECT;
  n.keys = keys;
  n.props = props;
  n.required = req;
  return n;
}

int main(int argc, char** argv) {
  const int walks = argc > 1 ? std::atoi(argv[1]) * 50 : 400;
  std::vector<GNode> nodes(8);
  nodes[0].kind = G_STRING;
  nodes[0].max_len = 12;
  nodes[1].kind = G_INTEGER;
  nodes[2].kind = G_ARRAY;
  nodes[2].item = 0;
  nodes[2].max_items = 3;
  nodes[3].kind = G_ENUM;
  nodes[3].lits = {"\"admin\"", "\"user\"", "7", "null"};
  nodes[4].kind = G_NUMBER;
  nodes[5].kind = G_BOOLEAN;
  nodes[6].kind = G_ANYOF;
  nodes[6].alts = {0, 1};
  nodes[7] = obj({"\"name\"", "\"age\"", "\"tags\"", "\"role\"", "\"score\"", "\"ok\"", "\"x\""},
                 {0, 1, 2, 3, 4, 5, 6}, {1, 1, 0, 1, 0, 0, 0});
  std::vector<std::string> vocab(300);
  for (int b = 0; b < 256; ++b) vocab[b] = std::string(1, (char)b);
  vocab[256] = "\", \"";  // multi-byte tokens
  vocab[257] = "\":";
  vocab[258] = "true}";
  vocab[259] = "[\"";
  const int eos = 299;
  Grammar g(nodes, 7, vocab, {eos});
  std::mt19937 rng(1234);
  std::vector<uint32_t> mask((g.vocab_size() + 31) / 32);
  int ok = 0;
  for (int w = 0; w < walks; ++w) {
    Matcher m(&g);
    const int budget = 40 + (int)(rng() % 200);
    std::string out;
    for (int step = 0; step < budget; ++step) {
      m.fill_mask(budget - step, mask.data());
      std::vector<int> allowed;
      for (int t = 0; t < g.vocab_size(); ++t)
        if (mask[t >> 5] >> (t & 31) & 1) allowed.push_back(t);
      if (allowed.empty()) {
        std::fprintf(stderr, "walk %d: no allowed token after %s\n", w, out.c_str());
        return 1;
      }
      const int t = allowed[rng() % allowed.size()];
      if (t == eos) break;
      if (!m.advance(t)) {
        std::fprintf(stderr, "walk %d: advance rejected an allowed token\n", w);
        return 1;
      }
      out += vocab[t];
      if (m.done()) break;
    }
    if (!m.done() && !m.can_finish()) {
      std::fprintf(stderr, "walk %d: budget %d ran out before the value closed: %s\n", w, budget, out.c_str());
      return 1;
    }
    ++ok;
  }
  std::printf("grammar selftest: %d random walks completed\n", ok);
  return 0;
}
