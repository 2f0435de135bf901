// Constrained decoding: a character-level JSON / JSON-schema pushdown matcher and its token masks.
//
// The reference's notebooks rely on `with_structured_output` / `bind_tools` (OpenAI `response_format`
// json_schema and `tool_choice: required`, RAG/notebooks/langchain/Agent_use_tools_leveraging_NVIDIA_AI_
// endpoints.ipynb:271-272,325-326); here the generator itself is forced to emit text that parses and
// validates. The schema is compiled (engine/guided.py) into a node table; a Matcher walks the output
// one byte at a time on an explicit frame stack. Per decode step the allowed-token bitmask is computed
// by a depth-first walk of the vocabulary's byte trie from the current state (undo journal, no state
// copies), with the token budget enforced: a token is allowed only if the shortest completion of the
// state it leads to still fits in the tokens left, so every request ends in valid JSON. Masks of
// budget-independent states are cached per normalised stack (in-string states repeat constantly).
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace gai {

enum GNodeKind : int {
  G_ANY = 0,      // any JSON value (json_object mode: the root is G_OBJECT_ANY)
  G_OBJECT = 1,   // properties in declared order (required ones mandatory)
  G_ARRAY = 2,
  G_STRING = 3,
  G_NUMBER = 4,
  G_INTEGER = 5,
  G_BOOLEAN = 6,
  G_NULL = 7,
  G_ENUM = 8,     // JSON-encoded literals (strings keep their quotes)
  G_ANYOF = 9,    // alternatives told apart by their first character
  G_OBJECT_ANY = 10,  // any object (free keys, G_ANY values)
};

struct GNode {
  int kind = G_ANY;
  // object
  std::vector<std::string> keys;  // JSON-encoded with quotes
  std::vector<int> props;
  std::vector<char> required;
  int disc_prop = -1, dep_prop = -1;  // tagged union: enum value of keys[disc_prop] selects props[dep_prop]
  std::vector<int> dep_alts;
  // array
  int item = -1, min_items = 0, max_items = 1 << 20;
  // string
  int min_len = 0, max_len = 256;
  // enum
  std::vector<std::string> lits;
  // anyOf
  std::vector<int> alts;
};

struct GFrame {
  int16_t type = 0, sub = 0;
  int32_t node = 0;
  int32_t a = 0, b = 0;
  uint64_t m = 0;
};

constexpr int kGMaxDepth = 48;

struct GState {
  GFrame fr[kGMaxDepth];
  int depth = 0;
  int done = 0;
  int dead = 0;
};

class Grammar {
 public:
  // nodes: the compiled schema; root: its root node; vocab: bytes of every token id (empty = never
  // allowed); eos: token ids allowed once the value is complete
  Grammar(std::vector<GNode> nodes, int root, const std::vector<std::string>& vocab, std::vector<int> eos);

  int vocab_size() const { return vocab_size_; }
  int root() const { return root_; }
  const std::vector<GNode>& nodes() const { return nodes_; }
  const std::vector<int>& eos() const { return eos_; }
  int minlen(int node) const { return minlen_[node]; }
  int max_token_len() const { return max_tok_len_; }

  // trie of token byte strings
  struct TrieNode {
    int first_edge = 0, num_edges = 0;
    int first_tok = 0, num_toks = 0;
  };
  std::vector<TrieNode> trie;
  std::vector<uint8_t> edge_byte;
  std::vector<int> edge_child;
  std::vector<int> trie_toks;

  int lit_node_true_false = -1, lit_node_null = -1;  // internal literal sets
  int any_node = -1;                                  // free JSON value (items of free containers)
  const std::string& token_bytes(int id) const { return vocab_[id]; }

 private:
  std::vector<GNode> nodes_;
  std::vector<int> minlen_;
  std::vector<int> eos_;
  std::vector<std::string> vocab_;
  int root_ = 0, vocab_size_ = 0, max_tok_len_ = 1;
  int compute_minlen(int n, int depth);
};

class Matcher {
 public:
  explicit Matcher(const Grammar* g);

  // bit t of mask (uint32 words, vocab_size/32 rounded up) = token t allowed, given `budget` tokens
  // left including this one
  void fill_mask(int budget, uint32_t* mask);
  // consume a sampled token; false if it violates the grammar (the matcher is then dead)
  bool advance(int token);
  bool done() const { return st_.done != 0; }
  bool dead() const { return st_.dead != 0; }
  bool can_finish() const;
  int min_chars() const;
  bool feed_bytes(const std::string& s);  // test hook: advance by raw text
  size_t cache_size() const { return cache_.size(); }
  int vocab_size() const { return g_->vocab_size(); }

 private:
  const Grammar* g_;
  GState st_;
  struct JEntry {
    int16_t idx;  // frame index, -1: depth/done word
    GFrame f;
    int depth, done;
  };
  std::vector<JEntry> jr_;
  struct CacheEntry {
    std::vector<uint32_t> mask;  // allowed tokens with no budget
    int max_after;               // largest shortest-completion (chars) among them
  };
  std::unordered_map<std::string, CacheEntry> cache_;
  int max_after_ = 0;

  bool feed(GState& s, int c);
  void save(GState& s, int k);
  void undo(GState& s, size_t mark);
  void push(GState& s, const GFrame& f);
  void pop_complete(GState& s, int result);
  bool start_value(GState& s, int node, int c);
  bool start_key(GState& s, GFrame& obj);
  uint64_t key_candidates(const GFrame& obj) const;
  bool can_close(const GFrame& obj) const;
  int tail_after(const GFrame& obj, int k) const;
  int prop_node(const GFrame& obj, int k) const;
  int frame_rem(const GState& s, int i) const;
  int min_chars_of(const GState& s) const;
  bool can_finish_of(const GState& s) const;
  std::string cache_key(const GState& s) const;
  void dfs(GState& s, int tnode, int budget_after, uint32_t* mask);
};

}  // namespace gai
