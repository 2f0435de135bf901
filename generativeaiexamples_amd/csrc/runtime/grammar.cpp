// JSON / JSON-schema matcher and token masks (see grammar.h).
#include "grammar.h"

#include <algorithm>
#include <climits>
#include <cstring>
#include <map>

namespace gai {

namespace {

enum FrameType : int16_t { F_VALUE = 0, F_OBJ = 1, F_ARR = 2, F_STR = 3, F_NUM = 4, F_LIT = 5 };
// object sub-states
enum : int16_t { O_START, O_KEY, O_COLON, O_COLSP, O_VALSTART, O_VALUE, O_AFTER, O_COMMASP, O_KEYSTART };
// array sub-states
enum : int16_t { A_START, A_VALUE, A_AFTER, A_COMMASP, A_VALSTART };
// string sub-states (U1..U4: expecting the k-th hex digit of \uXXXX)
enum : int16_t { S_BODY, S_ESC, S_U1, S_U2, S_U3, S_U4 };
// number sub-states
enum : int16_t { N_START, N_MINUS, N_ZERO, N_INT, N_FRAC0, N_FRAC, N_EXP0, N_EXPS, N_EXP };

constexpr int kMaxDigits = 17;      // mantissa digits of a generated number (bounds the grammar)
constexpr int kMaxExpDigits = 3;    // exponent digits
constexpr int kMaxAnyDepth = 6;     // nesting of free-form (G_ANY) containers
constexpr int kKeyMaxLen = 64;      // free-form object keys
constexpr int kAnyStrMaxLen = 512;  // free-form strings

bool is_digit(int c) { return c >= '0' && c <= '9'; }
bool is_hex(int c) { return is_digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
bool num_accepting(int sub) { return sub == N_ZERO || sub == N_INT || sub == N_FRAC || sub == N_EXP; }

}  // namespace

// ------------------------------------------------------------------------------------------------ grammar
Grammar::Grammar(std::vector<GNode> nodes, int root, const std::vector<std::string>& vocab, std::vector<int> eos)
    : nodes_(std::move(nodes)), eos_(std::move(eos)), vocab_(vocab), root_(root), vocab_size_((int)vocab.size()) {
  GNode tf;
  tf.kind = G_ENUM;
  tf.lits = {"true", "false"};
  lit_node_true_false = (int)nodes_.size();
  nodes_.push_back(tf);
  GNode nl;
  nl.kind = G_ENUM;
  nl.lits = {"null"};
  lit_node_null = (int)nodes_.size();
  nodes_.push_back(nl);
  GNode an;
  an.kind = G_ANY;
  any_node = (int)nodes_.size();
  nodes_.push_back(an);
  for (auto& n : nodes_) {
    if (n.kind == G_ENUM && n.lits.size() > 64) n.lits.resize(64);
    if (n.kind == G_OBJECT && n.keys.size() > 64) {
      n.keys.resize(64);
      n.props.resize(64);
      n.required.resize(64);
    }
  }
  minlen_.assign(nodes_.size(), -1);
  for (int i = 0; i < (int)nodes_.size(); ++i) compute_minlen(i, 0);

  // byte trie over the vocabulary
  struct Tmp {
    std::map<uint8_t, int> ch;
    std::vector<int> toks;
  };
  std::vector<Tmp> t(1);
  for (int id = 0; id < vocab_size_; ++id) {
    const std::string& s = vocab[id];
    if (s.empty()) continue;
    max_tok_len_ = std::max(max_tok_len_, (int)s.size());
    int cur = 0;
    for (unsigned char c : s) {
      auto it = t[cur].ch.find(c);
      if (it == t[cur].ch.end()) {
        t.push_back(Tmp());
        const int nx = (int)t.size() - 1;
        t[cur].ch[c] = nx;
        cur = nx;
      } else {
        cur = it->second;
      }
    }
    t[cur].toks.push_back(id);
  }
  trie.resize(t.size());
  for (size_t i = 0; i < t.size(); ++i) {
    trie[i].first_edge = (int)edge_byte.size();
    trie[i].num_edges = (int)t[i].ch.size();
    for (auto& kv : t[i].ch) {
      edge_byte.push_back(kv.first);
      edge_child.push_back(kv.second);
    }
    trie[i].first_tok = (int)trie_toks.size();
    trie[i].num_toks = (int)t[i].toks.size();
    trie_toks.insert(trie_toks.end(), t[i].toks.begin(), t[i].toks.end());
  }
}

int Grammar::compute_minlen(int i, int depth) {
  if (minlen_[i] >= 0) return minlen_[i];
  if (depth > 64) return 1;
  const GNode& n = nodes_[i];
  int r = 1;
  switch (n.kind) {
    case G_ANY: r = 1; break;  // "0"
    case G_OBJECT_ANY: r = 2; break;
    case G_STRING: r = 2 + n.min_len; break;
    case G_NUMBER:
    case G_INTEGER: r = 1; break;
    case G_BOOLEAN: r = 4; break;
    case G_NULL: r = 4; break;
    case G_ENUM: {
      r = INT_MAX / 4;
      for (auto& l : n.lits) r = std::min(r, (int)l.size());
      if (n.lits.empty()) r = 1;
      break;
    }
    case G_ANYOF: {
      r = INT_MAX / 4;
      for (int a : n.alts) r = std::min(r, compute_minlen(a, depth + 1));
      if (n.alts.empty()) r = 1;
      break;
    }
    case G_ARRAY: {
      const int it = n.item >= 0 ? compute_minlen(n.item, depth + 1) : 1;
      r = 2 + n.min_items * it + std::max(0, n.min_items - 1);
      break;
    }
    case G_OBJECT: {
      r = 2;
      int cnt = 0;
      for (size_t k = 0; k < n.props.size(); ++k) {
        if (!n.required[k]) continue;
        int v = compute_minlen(n.props[k], depth + 1);
        if ((int)k == n.dep_prop && !n.dep_alts.empty()) {
          v = INT_MAX / 4;
          for (int a : n.dep_alts) v = std::min(v, compute_minlen(a, depth + 1));
        }
        r += (int)n.keys[k].size() + 1 + v;
        ++cnt;
      }
      r += std::max(0, cnt - 1);
      break;
    }
  }
  minlen_[i] = r;
  return r;
}

// ------------------------------------------------------------------------------------------------ matcher
Matcher::Matcher(const Grammar* g) : g_(g) {
  st_.depth = 1;
  st_.fr[0] = GFrame();
  st_.fr[0].type = F_VALUE;
  st_.fr[0].node = g->root();
}

void Matcher::save(GState& s, int k) {
  JEntry e;
  e.idx = (int16_t)k;
  e.depth = s.depth;
  e.done = s.done;
  if (k >= 0) e.f = s.fr[k];
  jr_.push_back(e);
}

void Matcher::undo(GState& s, size_t mark) {
  while (jr_.size() > mark) {
    const JEntry& e = jr_.back();
    s.depth = e.depth;
    s.done = e.done;
    if (e.idx >= 0) s.fr[e.idx] = e.f;
    jr_.pop_back();
  }
}

void Matcher::push(GState& s, const GFrame& f) {
  save(s, s.depth);
  s.fr[s.depth++] = f;
}

void Matcher::pop_complete(GState& s, int result) {
  save(s, -1);
  s.depth -= 1;
  if (s.depth == 0) {
    s.done = 1;
    return;
  }
  const int pi = s.depth - 1;
  save(s, pi);
  GFrame& p = s.fr[pi];
  if (p.type == F_OBJ) {
    if (p.sub == O_KEY) {
      if (g_->nodes()[p.node].kind == G_OBJECT) p.a = result;
      p.sub = O_COLON;
    } else if (p.sub == O_VALUE) {
      const GNode& n = g_->nodes()[p.node];
      if (n.kind == G_OBJECT && p.a == n.disc_prop) p.b = result;
      if (n.kind == G_OBJECT_ANY) p.a += 1;
      p.sub = O_AFTER;
    }
  } else if (p.type == F_ARR) {
    p.a += 1;
    p.sub = A_AFTER;
  }
}

uint64_t Matcher::key_candidates(const GFrame& obj) const {
  const GNode& n = g_->nodes()[obj.node];
  uint64_t m = 0;
  for (int k = obj.a + 1; k < (int)n.props.size(); ++k) {
    m |= 1ull << k;
    if (n.required[k]) break;
  }
  return m;
}

bool Matcher::can_close(const GFrame& obj) const {
  const GNode& n = g_->nodes()[obj.node];
  if (n.kind != G_OBJECT) return true;
  for (int k = obj.a + 1; k < (int)n.props.size(); ++k)
    if (n.required[k]) return false;
  return true;
}

int Matcher::prop_node(const GFrame& obj, int k) const {
  const GNode& n = g_->nodes()[obj.node];
  if (k == n.dep_prop && !n.dep_alts.empty()) {
    if (obj.b >= 0 && obj.b < (int)n.dep_alts.size()) return n.dep_alts[obj.b];
    return n.dep_alts[0];
  }
  return n.props[k];
}

bool Matcher::start_key(GState& s, GFrame& obj) {
  const GNode& n = g_->nodes()[obj.node];
  GFrame f;
  if (n.kind == G_OBJECT) {
    const uint64_t cand = key_candidates(obj);
    if (!cand) return false;
    f.type = F_LIT;
    f.node = obj.node;
    f.b = 1;  // literal set = the object's keys
    f.a = 1;  // the opening quote is consumed here
    f.m = cand;
  } else {
    f.type = F_STR;
    f.sub = S_BODY;
    f.node = -1;  // free key
  }
  obj.sub = O_KEY;
  push(s, f);
  return true;
}

bool Matcher::start_value(GState& s, int node, int c) {
  // the F_VALUE frame on top is replaced by the concrete frame
  const int ti = s.depth - 1;
  save(s, ti);
  GFrame& f = s.fr[ti];
  const GNode& n = g_->nodes()[node];
  int kind = n.kind;
  if (kind == G_ANYOF) {
    for (int alt : n.alts) {
      // first-character dispatch: the first alternative that accepts c
      const size_t mark = jr_.size();
      f.node = alt;
      f.type = F_VALUE;
      if (start_value(s, alt, c)) return true;
      undo(s, mark);
    }
    return false;
  }
  // nesting bound for free-form values
  int any_depth = 0;
  for (int i = 0; i < ti; ++i)
    if (s.fr[i].type == F_OBJ || s.fr[i].type == F_ARR) ++any_depth;
  const bool free = kind == G_ANY || kind == G_OBJECT_ANY;
  if ((kind == G_OBJECT || kind == G_OBJECT_ANY || kind == G_ANY) && c == '{') {
    if (free && any_depth >= kMaxAnyDepth) return false;
    f = GFrame();
    f.type = F_OBJ;
    f.sub = O_START;
    f.node = node;  // a G_ANY / G_OBJECT_ANY node makes a free object
    f.a = kind == G_OBJECT ? -1 : 0;
    f.b = -1;
    return true;
  }
  if ((kind == G_ARRAY || kind == G_ANY) && c == '[') {
    if (free && any_depth >= kMaxAnyDepth) return false;
    f = GFrame();
    f.type = F_ARR;
    f.sub = A_START;
    f.node = node;
    return true;
  }
  if ((kind == G_STRING || kind == G_ANY) && c == '"') {
    f = GFrame();
    f.type = F_STR;
    f.sub = S_BODY;
    f.node = node;
    return true;
  }
  if ((kind == G_NUMBER || kind == G_INTEGER || kind == G_ANY) && (c == '-' || is_digit(c))) {
    f = GFrame();
    f.type = F_NUM;
    f.node = node;
    f.sub = c == '-' ? N_MINUS : (c == '0' ? N_ZERO : N_INT);
    f.a = c == '-' ? 0 : 1;
    return true;
  }
  int lit = -1;
  if (kind == G_ENUM) lit = node;
  if ((kind == G_BOOLEAN || kind == G_ANY) && (c == 't' || c == 'f')) lit = g_->lit_node_true_false;
  if ((kind == G_NULL || kind == G_ANY) && c == 'n') lit = g_->lit_node_null;
  if (lit >= 0) {
    const GNode& ln = g_->nodes()[lit];
    uint64_t m = 0;
    for (size_t i = 0; i < ln.lits.size(); ++i)
      if (!ln.lits[i].empty() && (unsigned char)ln.lits[i][0] == c) m |= 1ull << i;
    if (!m) return false;
    f = GFrame();
    f.type = F_LIT;
    f.node = lit;
    f.b = 0;
    f.a = 1;
    f.m = m;
    // a one-character literal completes at once
    for (size_t i = 0; i < ln.lits.size(); ++i)
      if ((m >> i & 1) && ln.lits[i].size() == 1 && m == (1ull << i)) {
        pop_complete(s, (int)i);
        return true;
      }
    return true;
  }
  return false;
}

bool Matcher::feed(GState& s, int c) {
  for (int guard = 0; guard < 2 * kGMaxDepth; ++guard) {
    if (s.done || s.dead || s.depth == 0) return false;
    const int ti = s.depth - 1;
    GFrame cur = s.fr[ti];
    const std::vector<GNode>& nodes = g_->nodes();
    switch (cur.type) {
      case F_VALUE:
        return start_value(s, cur.node, c);
      case F_STR: {
        const int maxlen = cur.node < 0 ? kKeyMaxLen
                                        : (nodes[cur.node].kind == G_STRING ? nodes[cur.node].max_len : kAnyStrMaxLen);
        const int minlen = (cur.node >= 0 && nodes[cur.node].kind == G_STRING) ? nodes[cur.node].min_len : 0;
        save(s, ti);
        GFrame& f = s.fr[ti];
        if (f.sub == S_BODY) {
          if (f.b > 0) {  // inside a UTF-8 sequence: continuation byte in [m >> 8, m & 0xFF]
            if (c < (int)(f.m >> 8) || c > (int)(f.m & 0xFF)) return false;
            f.b -= 1;
            f.m = (0x80u << 8) | 0xBFu;
            return true;
          }
          if (c == '"') {
            if (f.a < minlen) return false;
            pop_complete(s, -1);
            return true;
          }
          if (c < 0x20 || f.a >= maxlen) return false;
          if (c == '\\') {
            f.sub = S_ESC;
            return true;
          }
          if (c >= 0x80) {  // UTF-8 lead byte: well-formed sequences only (no overlongs / surrogates)
            int lo = 0x80, hi = 0xBF, n;
            if (c >= 0xC2 && c <= 0xDF) n = 1;
            else if (c >= 0xE0 && c <= 0xEF) {
              n = 2;
              if (c == 0xE0) lo = 0xA0;
              if (c == 0xED) hi = 0x9F;
            } else if (c >= 0xF0 && c <= 0xF4) {
              n = 3;
              if (c == 0xF0) lo = 0x90;
              if (c == 0xF4) hi = 0x8F;
            } else {
              return false;
            }
            f.b = n;
            f.m = ((uint64_t)lo << 8) | (uint64_t)hi;
          }
          f.a += 1;
          return true;
        }
        if (f.sub == S_ESC) {
          if (c == 'u') {
            f.sub = S_U1;
            return true;
          }
          if (!std::strchr("\"\\/bfnrt", c) || c == 0) return false;
          f.sub = S_BODY;
          f.a += 1;
          return true;
        }
        if (!is_hex(c)) return false;
        if (f.sub == S_U4) {
          f.sub = S_BODY;
          f.a += 1;
        } else {
          f.sub += 1;
        }
        return true;
      }
      case F_NUM: {
        const bool integer = cur.node >= 0 && nodes[cur.node].kind == G_INTEGER;
        int nsub = -1;
        switch (cur.sub) {
          case N_MINUS:
            if (is_digit(c)) nsub = c == '0' ? N_ZERO : N_INT;
            break;
          case N_ZERO:
            if (c == '.' && !integer) nsub = N_FRAC0;
            else if ((c == 'e' || c == 'E') && !integer) nsub = N_EXP0;
            break;
          case N_INT:
            if (is_digit(c)) nsub = N_INT;
            else if (c == '.' && !integer) nsub = N_FRAC0;
            else if ((c == 'e' || c == 'E') && !integer) nsub = N_EXP0;
            break;
          case N_FRAC0:
          case N_FRAC:
            if (is_digit(c)) nsub = N_FRAC;
            else if (cur.sub == N_FRAC && (c == 'e' || c == 'E')) nsub = N_EXP0;
            break;
          case N_EXP0:
            if (c == '+' || c == '-') nsub = N_EXPS;
            else if (is_digit(c)) nsub = N_EXP;
            break;
          case N_EXPS:
          case N_EXP:
            if (is_digit(c)) nsub = N_EXP;
            break;
        }
        if (nsub >= 0) {
          // mantissa digits (a) and exponent digits (b) are bounded separately; '.' / 'e' need room for
          // the digit that must follow them
          const bool exp = nsub == N_EXP0 || nsub == N_EXPS || nsub == N_EXP;
          const int a = cur.a + (!exp && is_digit(c) ? 1 : 0);
          const int b = cur.b + (exp && is_digit(c) ? 1 : 0);
          if (a > kMaxDigits || b > kMaxExpDigits) return false;
          if (nsub == N_FRAC0 && a >= kMaxDigits) return false;
          save(s, ti);
          s.fr[ti].sub = (int16_t)nsub;
          s.fr[ti].a = a;
          s.fr[ti].b = b;
          return true;
        }
        if (!num_accepting(cur.sub)) return false;
        pop_complete(s, -1);
        continue;  // the character belongs to the enclosing frame
      }
      case F_LIT: {
        const GNode& ln = nodes[cur.node];
        const std::vector<std::string>& L = cur.b == 1 ? ln.keys : ln.lits;
        uint64_t nm = 0;
        int complete = -1;
        for (size_t i = 0; i < L.size(); ++i) {
          if (!(cur.m >> i & 1)) continue;
          if ((int)L[i].size() == cur.a) complete = (int)i;
          else if ((unsigned char)L[i][cur.a] == c) nm |= 1ull << i;
        }
        if (!nm) {
          if (complete < 0) return false;
          pop_complete(s, complete);
          continue;
        }
        save(s, ti);
        GFrame& f = s.fr[ti];
        f.m = nm;
        f.a += 1;
        // completed and unambiguous: close now
        int only = -1, longer = 0;
        for (size_t i = 0; i < L.size(); ++i) {
          if (!(nm >> i & 1)) continue;
          if ((int)L[i].size() == f.a) only = (int)i;
          else longer = 1;
        }
        if (only >= 0 && !longer) pop_complete(s, only);
        return true;
      }
      case F_OBJ: {
        const GNode& n = nodes[cur.node];
        const bool schema = n.kind == G_OBJECT;
        save(s, ti);
        GFrame& f = s.fr[ti];
        switch (f.sub) {
          case O_START:
            if (c == '"') return start_key(s, s.fr[ti]);
            if (c == '}' && can_close(f)) {
              pop_complete(s, -1);
              return true;
            }
            return false;
          case O_COLON:
            if (c != ':') return false;
            f.sub = O_COLSP;
            return true;
          case O_COLSP:
            if (c == ' ') {
              f.sub = O_VALSTART;
              return true;
            }
            [[fallthrough]];
          case O_VALSTART: {
            f.sub = O_VALUE;
            GFrame v;
            v.type = F_VALUE;
            v.node = schema ? prop_node(f, f.a) : g_->any_node;  // free objects hold free values
            push(s, v);
            continue;
          }
          case O_AFTER:
            if (c == ',') {
              if (schema && !key_candidates(f)) return false;
              f.sub = O_COMMASP;
              return true;
            }
            if (c == '}' && can_close(f)) {
              pop_complete(s, -1);
              return true;
            }
            return false;
          case O_COMMASP:
            if (c == ' ') {
              f.sub = O_KEYSTART;
              return true;
            }
            [[fallthrough]];
          case O_KEYSTART:
            if (c != '"') return false;
            return start_key(s, s.fr[ti]);
          default:
            return false;
        }
      }
      case F_ARR: {
        const GNode& n = nodes[cur.node];
        const int item = (n.kind == G_ARRAY && n.item >= 0) ? n.item : g_->any_node;  // free arrays: free values
        const int mn = n.kind == G_ARRAY ? n.min_items : 0;
        const int mx = n.kind == G_ARRAY ? n.max_items : (1 << 20);
        save(s, ti);
        GFrame& f = s.fr[ti];
        switch (f.sub) {
          case A_START:
            if (c == ']') {
              if (mn > 0) return false;
              pop_complete(s, -1);
              return true;
            }
            [[fallthrough]];
          case A_VALSTART: {
            if (f.a >= mx) return false;
            f.sub = A_VALUE;
            GFrame v;
            v.type = F_VALUE;
            v.node = item;
            push(s, v);
            continue;
          }
          case A_AFTER:
            if (c == ',' && f.a < mx) {
              f.sub = A_COMMASP;
              return true;
            }
            if (c == ']' && f.a >= mn) {
              pop_complete(s, -1);
              return true;
            }
            return false;
          case A_COMMASP:
            if (c == ' ') {
              f.sub = A_VALSTART;
              return true;
            }
            f.sub = A_VALSTART;
            continue;
          default:
            return false;
        }
      }
    }
    return false;
  }
  return false;
}

// ---- shortest completion (characters) of a state
int Matcher::tail_after(const GFrame& obj, int k) const {
  const GNode& n = g_->nodes()[obj.node];
  int r = 1;  // '}'
  for (int i = k + 1; i < (int)n.props.size(); ++i)
    if (n.required[i]) r += 1 + (int)n.keys[i].size() + 1 + g_->minlen(prop_node(obj, i));
  return r;
}

int Matcher::frame_rem(const GState& s, int i) const {
  const GFrame& f = s.fr[i];
  const std::vector<GNode>& nodes = g_->nodes();
  switch (f.type) {
    case F_VALUE:
      return g_->minlen(f.node);
    case F_STR: {
      const int minlen = (f.node >= 0 && nodes[f.node].kind == G_STRING) ? nodes[f.node].min_len : 0;
      const int need = std::max(0, minlen - f.a);
      if (f.sub == S_BODY) return f.b + need + 1;
      if (f.sub == S_ESC) return 1 + std::max(0, need - 1) + 1;
      return (S_U4 - f.sub + 1) + std::max(0, need - 1) + 1;
    }
    case F_NUM:
      return num_accepting(f.sub) ? 0 : 1;
    case F_LIT: {
      const GNode& ln = nodes[f.node];
      const std::vector<std::string>& L = f.b == 1 ? ln.keys : ln.lits;
      int r = INT_MAX / 4;
      for (size_t k = 0; k < L.size(); ++k) {
        if (!(f.m >> k & 1)) continue;
        int v = (int)L[k].size() - f.a;
        if (f.b == 1 && i > 0) {  // a key: the parent's remainder depends on which key
          const GFrame& p = s.fr[i - 1];
          v += 1 + g_->minlen(prop_node(p, (int)k)) + tail_after(p, (int)k);
        }
        r = std::min(r, v);
      }
      return r;
    }
    case F_OBJ: {
      const GNode& n = nodes[f.node];
      if (n.kind != G_OBJECT) {
        switch (f.sub) {
          case O_START: return 1;
          case O_KEY: return 3;  // ':' '0' '}' after the key string (its frame counts its own chars)
          case O_COLON: return 3;
          case O_COLSP:
          case O_VALSTART: return 2;
          case O_VALUE:
          case O_AFTER: return 1;
          default: return 5;  // '"' '"' ':' '0' '}'
        }
      }
      switch (f.sub) {
        case O_START: {
          int r = 1, cnt = 0;
          for (size_t k = 0; k < n.props.size(); ++k)
            if (n.required[k]) {
              r += (int)n.keys[k].size() + 1 + g_->minlen(prop_node(f, (int)k));
              ++cnt;
            }
          return r + std::max(0, cnt - 1);
        }
        case O_KEY:
          return 0;  // the key literal frame above accounts for the rest of this object
        case O_COLON:
          return 1 + g_->minlen(prop_node(f, f.a)) + tail_after(f, f.a);
        case O_COLSP:
        case O_VALSTART:
          return g_->minlen(prop_node(f, f.a)) + tail_after(f, f.a);
        case O_VALUE:
        case O_AFTER:
          return tail_after(f, f.a);
        default: {  // after ',': one more key is needed
          int r = INT_MAX / 4;
          const uint64_t cand = key_candidates(f);
          for (int k = 0; k < 64; ++k)
            if (cand >> k & 1)
              r = std::min(r, (int)n.keys[k].size() + 1 + g_->minlen(prop_node(f, k)) + tail_after(f, k));
          return r;
        }
      }
    }
    case F_ARR: {
      const GNode& n = nodes[f.node];
      const int mn = n.kind == G_ARRAY ? n.min_items : 0;
      const int it = (n.kind == G_ARRAY && n.item >= 0) ? g_->minlen(n.item) : 1;
      switch (f.sub) {
        case A_START: return mn == 0 ? 1 : mn * it + (mn - 1) + 1;
        case A_VALUE: return std::max(0, mn - (f.a + 1)) * (1 + it) + 1;
        case A_AFTER: return std::max(0, mn - f.a) * (1 + it) + 1;
        default: return it + std::max(0, mn - (f.a + 1)) * (1 + it) + 1;
      }
    }
  }
  return 0;
}

int Matcher::min_chars_of(const GState& s) const {
  if (s.done) return 0;
  int r = 0;
  for (int i = 0; i < s.depth; ++i) r += frame_rem(s, i);
  return r;
}

bool Matcher::can_finish_of(const GState& s) const {
  if (s.done) return true;
  if (s.depth != 1) return false;
  const GFrame& f = s.fr[0];
  if (f.type == F_NUM) return num_accepting(f.sub);
  if (f.type == F_LIT) {
    const GNode& ln = g_->nodes()[f.node];
    for (size_t k = 0; k < ln.lits.size(); ++k)
      if ((f.m >> k & 1) && (int)ln.lits[k].size() == f.a) return true;
  }
  return false;
}

int Matcher::min_chars() const { return min_chars_of(st_); }
bool Matcher::can_finish() const { return can_finish_of(st_); }

std::string Matcher::cache_key(const GState& s) const {
  // counters that cannot matter within one token are normalised so in-string / in-number states share
  // one entry
  const int T = g_->max_token_len();
  std::string k;
  k.reserve(s.depth * sizeof(GFrame) + 8);
  k.push_back((char)s.done);
  for (int i = 0; i < s.depth; ++i) {
    GFrame f = s.fr[i];
    const std::vector<GNode>& nodes = g_->nodes();
    if (f.type == F_STR) {
      const bool sch = f.node >= 0 && nodes[f.node].kind == G_STRING;
      const int maxlen = f.node < 0 ? kKeyMaxLen : (sch ? nodes[f.node].max_len : kAnyStrMaxLen);
      const int minlen = sch ? nodes[f.node].min_len : 0;
      if (f.a >= minlen && maxlen - f.a > T + 4) f.a = -1;
    } else if (f.type == F_NUM) {
      if (kMaxDigits - f.a > T + 1) f.a = -1;
      if (kMaxExpDigits - f.b > T + 1) f.b = -1;
    } else if (f.type == F_ARR) {
      const GNode& n = nodes[f.node];
      const int mn = n.kind == G_ARRAY ? n.min_items : 0;
      const int mx = n.kind == G_ARRAY ? n.max_items : (1 << 20);
      if (f.a >= mn && mx - f.a > T + 1) f.a = -1;
    } else if (f.type == F_OBJ && nodes[f.node].kind != G_OBJECT) {
      f.a = 0;
    }
    k.append(reinterpret_cast<const char*>(&f), sizeof(GFrame));
  }
  return k;
}

void Matcher::dfs(GState& s, int tn, int budget_after, uint32_t* mask) {
  const Grammar::TrieNode& node = g_->trie[tn];
  for (int e = 0; e < node.num_edges; ++e) {
    const int c = g_->edge_byte[node.first_edge + e];
    const int child = g_->edge_child[node.first_edge + e];
    const size_t mark = jr_.size();
    save(s, -1);
    if (feed(s, c)) {
      const Grammar::TrieNode& cn = g_->trie[child];
      const int mc = cn.num_toks ? min_chars_of(s) : 0;
      if (cn.num_toks && mc <= budget_after) {
        max_after_ = std::max(max_after_, mc);
        for (int t = 0; t < cn.num_toks; ++t) {
          const int id = g_->trie_toks[cn.first_tok + t];
          mask[id >> 5] |= 1u << (id & 31);
        }
      }
      if (cn.num_edges) dfs(s, child, budget_after, mask);
    }
    undo(s, mark);
  }
}

void Matcher::fill_mask(int budget, uint32_t* mask) {
  const int W = (g_->vocab_size() + 31) / 32;
  std::memset(mask, 0, sizeof(uint32_t) * W);
  if (st_.dead) return;
  if (can_finish_of(st_))
    for (int e : g_->eos()) mask[e >> 5] |= 1u << (e & 31);
  if (st_.done) return;
  const int budget_after = budget - 1;
  // A state's unconstrained mask is cached with the largest shortest-completion any of its tokens
  // leads to; while the budget covers that, the cached mask is exact, otherwise walk with the budget.
  const std::string key = cache_key(st_);
  auto it = cache_.find(key);
  if (it != cache_.end() && it->second.max_after <= budget_after) {
    for (int w = 0; w < W; ++w) mask[w] |= it->second.mask[w];
    return;
  }
  std::vector<uint32_t> m(W, 0);
  jr_.clear();
  GState s = st_;
  max_after_ = 0;
  const bool fresh = it == cache_.end();
  dfs(s, 0, fresh ? (1 << 29) : budget_after, m.data());
  if (fresh) {
    CacheEntry e{m, max_after_};
    if (max_after_ > budget_after) {  // the budget binds: redo the walk with it (the entry stays exact)
      std::fill(m.begin(), m.end(), 0u);
      jr_.clear();
      s = st_;
      dfs(s, 0, budget_after, m.data());
    }
    if (cache_.size() > 4096) cache_.clear();
    cache_.emplace(key, std::move(e));
  }
  for (int w = 0; w < W; ++w) mask[w] |= m[w];
}

bool Matcher::advance(int token) {
  if (st_.dead) return false;
  if (token < 0 || token >= g_->vocab_size()) {
    st_.dead = 1;
    return false;
  }
  for (int e : g_->eos())
    if (token == e) {
      if (!can_finish_of(st_)) st_.dead = 1;
      st_.done = 1;
      return !st_.dead;
    }
  const std::string& b = g_->token_bytes(token);
  if (b.empty()) {
    st_.dead = 1;
    return false;
  }
  return feed_bytes(b);
}

bool Matcher::feed_bytes(const std::string& str) {
  if (st_.dead) return false;
  jr_.clear();
  for (unsigned char c : str) {
    if (!feed(st_, c)) {
      st_.dead = 1;
      jr_.clear();
      return false;
    }
  }
  jr_.clear();
  return true;
}

}  // namespace gai
