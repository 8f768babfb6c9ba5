// K13 -- JSON / JSON-schema constrained decoding: host-side token masks.
//
// A byte-level pushdown automaton over a compiled schema (node table built by
// omnia_amd/engine/guided.py) decides which next bytes keep the output a valid
// prefix of a schema-conforming compact JSON document.  The token mask for a
// state is computed by walking a byte trie of the vocabulary with the
// automaton (pruning at the first rejected byte) and cached per automaton
// state, so the steady-state cost inside free-form strings is one hash lookup.
// The mask ([ceil(V/32)] uint32, bit = allowed) is applied to the logits on the
// GPU by omnia_apply_token_mask before the fused sampler.
//
// Output form: compact JSON (no insignificant whitespace); object keys in the
// schema's property order (optional keys may be skipped, required ones must
// appear); additionalProperties only for schemas without "properties".
// Reference parity: function-mode json_schema output
// (internal/runtime/response_format.go), where the reference can only ask the
// remote provider for JSON; here the engine enforces it.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

enum Kind : uint8_t { K_ANY = 0, K_OBJECT, K_ARRAY, K_STRING, K_NUMBER, K_INTEGER, K_LITERALS, K_UNION };

struct Prop {
  std::string key_lit;  // "\"name\"" (quoted JSON string)
  int child;
  bool required;
};

struct Node {
  Kind kind = K_ANY;
  std::vector<Prop> props;  // K_OBJECT (empty => free-form keys, values = `items`)
  int items = 0;            // K_ARRAY item node / free-form object value node
  int min_items = 0, max_items = -1;
  int min_len = 0, max_len = -1;  // K_STRING
  std::vector<std::string> literals;  // K_LITERALS (enum / const / true,false / null)
  std::vector<int> children;          // K_UNION
  // tagged object (tool-call union): props[0]'s value is an enum whose matched
  // literal i selects tag_children[i] as the value schema of props[1]
  std::vector<int> tag_children;
};

enum FK : uint8_t { F_VALUE = 0, F_OBJ, F_ARR, F_STR, F_NUM, F_LIT };
// object phases
enum : uint8_t { O_OPEN = 0, O_KEY, O_COLON, O_VAL, O_AFTER, O_NEXTKEY };
// array phases
enum : uint8_t { A_OPEN = 0, A_VAL, A_AFTER };
// string phases
enum : uint8_t { S_NORM = 0, S_ESC, S_U1, S_U2, S_U3, S_U4 };
// number states
enum : uint8_t { N_START = 0, N_MINUS, N_ZERO, N_INT, N_DOT, N_FRAC, N_E, N_ESIGN, N_EXP };

struct Frame {
  int32_t node;
  uint8_t kind;
  uint8_t phase;
  uint8_t is_key;    // F_STR used as a free-form object key / F_LIT matching keys
  uint8_t pad;
  int32_t a;         // obj: current prop index; arr: count; str: length; lit: position
  int32_t b;         // obj (keyed): matched prop; str: pending UTF-8 continuation bytes
  uint64_t alive;    // lit: candidate bitmask
};

constexpr int kMaxDepth = 48;

struct State {
  int n = 0;
  bool done = false;
  Frame f[kMaxDepth];
  std::string key() const {
    std::string k(reinterpret_cast<const char*>(f), sizeof(Frame) * n);
    k.push_back(done ? 1 : 0);
    return k;
  }
};

enum Step { ACCEPT, REJECT, END_RETRY, PUSHED };

struct Vocab {
  // byte trie: children as sorted (byte, node) lists in one arena
  struct TNode {
    int first_edge = -1, n_edges = 0;
    int tok_begin = 0, tok_count = 0;
  };
  std::vector<TNode> nodes;
  std::vector<std::pair<uint8_t, int>> edges;
  std::vector<int> toks;
  int vocab_size = 0;
  std::vector<int> eos;

  Vocab(const std::vector<py::bytes>& token_bytes, const std::vector<int>& eos_ids)
      : vocab_size((int)token_bytes.size()), eos(eos_ids) {
    // build a pointer trie first, then flatten breadth-first
    struct B { std::vector<std::pair<uint8_t, int>> ch; std::vector<int> t; };
    std::vector<B> tmp(1);
    for (int id = 0; id < vocab_size; ++id) {
      std::string s = token_bytes[id];
      if (s.empty()) continue;  // specials: never produced by the grammar
      int cur = 0;
      for (unsigned char c : s) {
        int nxt = -1;
        for (auto& e : tmp[cur].ch)
          if (e.first == c) { nxt = e.second; break; }
        if (nxt < 0) {
          nxt = (int)tmp.size();
          tmp[cur].ch.emplace_back(c, nxt);
          tmp.emplace_back();
        }
        cur = nxt;
      }
      tmp[cur].t.push_back(id);
    }
    nodes.resize(tmp.size());
    for (size_t i = 0; i < tmp.size(); ++i) {
      auto& ch = tmp[i].ch;
      std::sort(ch.begin(), ch.end());
      nodes[i].first_edge = (int)edges.size();
      nodes[i].n_edges = (int)ch.size();
      edges.insert(edges.end(), ch.begin(), ch.end());
      nodes[i].tok_begin = (int)toks.size();
      nodes[i].tok_count = (int)tmp[i].t.size();
      toks.insert(toks.end(), tmp[i].t.begin(), tmp[i].t.end());
    }
  }
  int words() const { return (vocab_size + 31) / 32; }
  size_t trie_nodes() const { return nodes.size(); }
};

class Grammar {
 public:
  std::vector<Node> nodes;
  int root = 0;
  std::shared_ptr<Vocab> vocab;
  std::unordered_map<std::string, std::vector<uint32_t>> cache;
  int64_t cache_hits = 0, cache_misses = 0;

  // ---------------------------------------------------------------- automaton
  static bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
  static bool is_hex(uint8_t c) {
    return is_digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
  }

  bool push(State& s, const Frame& fr) const {
    if (s.n >= kMaxDepth) return false;
    s.f[s.n++] = fr;
    return true;
  }
  static Frame mk(int node, uint8_t kind, uint8_t phase = 0) {
    Frame fr;
    std::memset(&fr, 0, sizeof(fr));
    fr.node = node;
    fr.kind = kind;
    fr.phase = phase;
    return fr;
  }

  // first required prop index >= from (or props.size())
  static int next_required(const Node& nd, int from) {
    for (int i = from; i < (int)nd.props.size(); ++i)
      if (nd.props[i].required) return i;
    return (int)nd.props.size();
  }

  // literal candidates of a keyed object's key slot starting at prop `from`
  static uint64_t key_candidates(const Node& nd, int from) {
    const int last = std::min(next_required(nd, from), (int)nd.props.size() - 1);
    uint64_t m = 0;
    for (int i = from; i <= last && i < 64; ++i) m |= (1ull << i);
    return m;
  }

  // a child frame completed: advance its parent (or finish the document)
  void complete_top(State& s) const {
    Frame done = s.f[s.n - 1];
    --s.n;
    if (s.n == 0) {
      s.done = true;
      return;
    }
    Frame& p = s.f[s.n - 1];
    if (p.kind == F_OBJ) {
      if (p.phase == O_KEY) {
        if (done.kind == F_LIT) {  // keyed object: which key matched
          const Node& nd = nodes[p.node];
          int idx = -1;
          for (int i = 0; i < (int)nd.props.size() && i < 64; ++i)
            if ((done.alive >> i) & 1) {
              if ((int)nd.props[i].key_lit.size() == done.a) { idx = i; break; }
            }
          p.b = idx;
        }
        p.phase = O_COLON;
      } else if (p.phase == O_VAL) {
        const Node& nd = nodes[p.node];
        if (!nd.tag_children.empty() && p.a == 0 && done.kind == F_LIT) {
          // remember which tag literal the discriminator matched (F_OBJ frames do
          // not use `alive` otherwise)
          const Node& ln = nodes[done.node];
          p.alive = 0;
          for (int i = 0; i < (int)ln.literals.size() && i < 64; ++i)
            if (((done.alive >> i) & 1) && (int)ln.literals[i].size() == done.a) {
              p.alive = (uint64_t)i;
              break;
            }
        }
        p.phase = O_AFTER;
      }
    } else if (p.kind == F_ARR) {
      if (p.phase == A_VAL) {
        p.phase = A_AFTER;
        p.a += 1;
      }
    }
  }

  bool can_end(const Frame& f) const {
    if (f.kind == F_NUM)
      return f.phase == N_ZERO || f.phase == N_INT || f.phase == N_FRAC || f.phase == N_EXP;
    if (f.kind == F_LIT) {
      const int n = nlits(f);
      for (int i = 0; i < n; ++i)
        if (((f.alive >> i) & 1) && (int)lit(f, i).size() == f.a) return true;
    }
    return false;
  }

  // literal list a F_LIT frame matches against (keys for keyed objects)
  const std::string& lit(const Frame& f, int i) const {
    const Node& nd = nodes[f.node];
    return f.is_key ? nd.props[i].key_lit : nd.literals[i];
  }
  int nlits(const Frame& f) const {
    const Node& nd = nodes[f.node];
    return std::min<int>(64, f.is_key ? (int)nd.props.size() : (int)nd.literals.size());
  }

  Step step(State& s, uint8_t c) const {
    Frame& f = s.f[s.n - 1];
    const Node& nd = nodes[f.node];
    switch (f.kind) {
      case F_VALUE: {
        Kind k = nd.kind;
        int node = f.node;
        if (k == K_UNION) {  // first child whose first byte fits
          int pick = -1;
          for (int ch : nd.children)
            if (first_ok(ch, c)) { pick = ch; break; }
          if (pick < 0) return REJECT;
          f.node = node = pick;
          return PUSHED;  // re-dispatch on the chosen branch (same frame)
        }
        if (k == K_ANY) {
          if (c == '{') { f = mk(node, F_OBJ, O_OPEN); return ACCEPT; }
          if (c == '[') { f = mk(node, F_ARR, A_OPEN); return ACCEPT; }
          if (c == '"') { f = mk(node, F_STR, S_NORM); return ACCEPT; }
          if (c == '-' || is_digit(c)) { f = mk(node, F_NUM, N_START); return PUSHED; }
          if (c == 't' || c == 'f' || c == 'n') {
            // ANY node carries the literals true/false/null
            f = mk(node, F_LIT);
            f.alive = (1ull << nd.literals.size()) - 1;
            return PUSHED;
          }
          return REJECT;
        }
        if (k == K_OBJECT) { if (c != '{') return REJECT; f = mk(node, F_OBJ, O_OPEN); return ACCEPT; }
        if (k == K_ARRAY) { if (c != '[') return REJECT; f = mk(node, F_ARR, A_OPEN); return ACCEPT; }
        if (k == K_STRING) { if (c != '"') return REJECT; f = mk(node, F_STR, S_NORM); return ACCEPT; }
        if (k == K_NUMBER || k == K_INTEGER) {
          if (c != '-' && !is_digit(c)) return REJECT;
          f = mk(node, F_NUM, N_START);
          return PUSHED;
        }
        if (k == K_LITERALS) {
          f = mk(node, F_LIT);
          f.alive = nd.literals.size() >= 64 ? ~0ull : ((1ull << nd.literals.size()) - 1);
          return PUSHED;
        }
        return REJECT;
      }
      case F_OBJ: {
        const bool keyed = nd.kind == K_OBJECT && !nd.props.empty();
        switch (f.phase) {
          case O_OPEN:
          case O_NEXTKEY: {
            const int from = f.phase == O_OPEN ? 0 : f.a + 1;
            if (c == '}' && f.phase == O_OPEN) {
              if (keyed && next_required(nd, 0) < (int)nd.props.size()) return REJECT;
              s.f[s.n - 1].phase = 0;
              complete_top(s);
              return ACCEPT;
            }
            if (c != '"') return REJECT;
            f.phase = O_KEY;
            if (keyed) {
              if (from >= (int)nd.props.size()) return REJECT;
              Frame k = mk(f.node, F_LIT);
              k.is_key = 1;
              k.alive = key_candidates(nd, from);
              if (!push(s, k)) return REJECT;
              return PUSHED;  // the key literal consumes the opening quote
            }
            Frame k = mk(0, F_STR, S_NORM);
            k.is_key = 1;
            if (!push(s, k)) return REJECT;
            return ACCEPT;
          }
          case O_COLON: {
            if (c != ':') return REJECT;
            f.phase = O_VAL;
            int child;
            if (keyed) {
              if (f.b < 0) return REJECT;
              f.a = f.b;
              child = nd.props[f.b].child;
              if (!nd.tag_children.empty() && f.b == 1) {
                if (f.alive >= nd.tag_children.size()) return REJECT;
                child = nd.tag_children[f.alive];
              }
            } else {
              child = nd.kind == K_OBJECT ? nd.items : 0;
            }
            if (!push(s, mk(child, F_VALUE))) return REJECT;
            return ACCEPT;
          }
          case O_AFTER: {
            if (c == '}') {
              if (keyed && next_required(nd, f.a + 1) < (int)nd.props.size()) return REJECT;
              complete_top(s);
              return ACCEPT;
            }
            if (c == ',') {
              if (keyed && f.a + 1 >= (int)nd.props.size()) return REJECT;
              f.phase = O_NEXTKEY;
              return ACCEPT;
            }
            return REJECT;
          }
          default:
            return REJECT;
        }
      }
      case F_ARR: {
        const int item = nd.kind == K_ARRAY ? nd.items : 0;
        const int mn = nd.kind == K_ARRAY ? nd.min_items : 0;
        const int mx = nd.kind == K_ARRAY ? nd.max_items : -1;
        if (f.phase == A_OPEN) {
          if (c == ']') {
            if (mn > 0) return REJECT;
            complete_top(s);
            return ACCEPT;
          }
          if (mx == 0) return REJECT;
          f.phase = A_VAL;
          if (!push(s, mk(item, F_VALUE))) return REJECT;
          return PUSHED;
        }
        if (f.phase == A_AFTER) {
          if (c == ']') {
            if (f.a < mn) return REJECT;
            complete_top(s);
            return ACCEPT;
          }
          if (c == ',') {
            if (mx >= 0 && f.a >= mx) return REJECT;
            f.phase = A_VAL;
            if (!push(s, mk(item, F_VALUE))) return REJECT;
            return ACCEPT;
          }
        }
        return REJECT;
      }
      case F_STR: {
        const int mn = (!f.is_key && nd.kind == K_STRING) ? nd.min_len : 0;
        const int mx = (!f.is_key && nd.kind == K_STRING) ? nd.max_len : -1;
        switch (f.phase) {
          case S_NORM:
            if (f.b > 0) {  // inside a multi-byte UTF-8 character
              if ((c & 0xC0) != 0x80) return REJECT;
              f.b -= 1;
              return ACCEPT;
            }
            if (c == '"') {
              if (f.a < mn) return REJECT;
              complete_top(s);
              return ACCEPT;
            }
            if (c < 0x20) return REJECT;
            if (c >= 0x80) {  // well-formed UTF-8 lead byte
              if (c >= 0xC2 && c <= 0xDF) f.b = 1;
              else if (c >= 0xE0 && c <= 0xEF) f.b = 2;
              else if (c >= 0xF0 && c <= 0xF4) f.b = 3;
              else return REJECT;
            }
            if (mx >= 0 && f.a >= mx) return REJECT;
            f.a += 1;
            if (c == '\\') f.phase = S_ESC;
            return ACCEPT;
          case S_ESC:
            if (c == 'u') { f.phase = S_U1; return ACCEPT; }
            if (c == '"' || c == '\\' || c == '/' || c == 'b' || c == 'f' || c == 'n' ||
                c == 'r' || c == 't') {
              f.phase = S_NORM;
              return ACCEPT;
            }
            return REJECT;
          default:  // \uXXXX
            if (!is_hex(c)) return REJECT;
            f.phase = f.phase == S_U4 ? S_NORM : f.phase + 1;
            return ACCEPT;
        }
      }
      case F_NUM: {
        const bool integer = nd.kind == K_INTEGER;
        switch (f.phase) {
          case N_START:
            if (c == '-') { f.phase = N_MINUS; return ACCEPT; }
            if (c == '0') { f.phase = N_ZERO; return ACCEPT; }
            if (is_digit(c)) { f.phase = N_INT; return ACCEPT; }
            return REJECT;
          case N_MINUS:
            if (c == '0') { f.phase = N_ZERO; return ACCEPT; }
            if (is_digit(c)) { f.phase = N_INT; return ACCEPT; }
            return REJECT;
          case N_ZERO:
          case N_INT:
            if (f.phase == N_INT && is_digit(c)) return ACCEPT;
            if (!integer && c == '.') { f.phase = N_DOT; return ACCEPT; }
            if (!integer && (c == 'e' || c == 'E')) { f.phase = N_E; return ACCEPT; }
            return END_RETRY;
          case N_DOT:
            if (is_digit(c)) { f.phase = N_FRAC; return ACCEPT; }
            return REJECT;
          case N_FRAC:
            if (is_digit(c)) return ACCEPT;
            if (c == 'e' || c == 'E') { f.phase = N_E; return ACCEPT; }
            return END_RETRY;
          case N_E:
            if (c == '+' || c == '-') { f.phase = N_ESIGN; return ACCEPT; }
            if (is_digit(c)) { f.phase = N_EXP; return ACCEPT; }
            return REJECT;
          case N_ESIGN:
            if (is_digit(c)) { f.phase = N_EXP; return ACCEPT; }
            return REJECT;
          case N_EXP:
            if (is_digit(c)) return ACCEPT;
            return END_RETRY;
        }
        return REJECT;
      }
      case F_LIT: {
        uint64_t nxt = 0;
        const int n = nlits(f);
        for (int i = 0; i < n; ++i) {
          if (!((f.alive >> i) & 1)) continue;
          const std::string& l = lit(f, i);
          if (f.a < (int)l.size() && (uint8_t)l[f.a] == c) nxt |= (1ull << i);
        }
        if (!nxt) return can_end(f) ? END_RETRY : REJECT;
        f.alive = nxt;
        f.a += 1;
        // complete when every surviving candidate is fully matched
        bool all_full = true;
        for (int i = 0; i < n; ++i)
          if (((nxt >> i) & 1) && (int)lit(f, i).size() != f.a) { all_full = false; break; }
        if (all_full) complete_top(s);
        return ACCEPT;
      }
    }
    return REJECT;
  }

  // can a value of `node` start with byte c
  bool first_ok(int node, uint8_t c) const {
    const Node& nd = nodes[node];
    switch (nd.kind) {
      case K_ANY:
        return c == '{' || c == '[' || c == '"' || c == '-' || is_digit(c) || c == 't' ||
               c == 'f' || c == 'n';
      case K_OBJECT: return c == '{';
      case K_ARRAY: return c == '[';
      case K_STRING: return c == '"';
      case K_NUMBER:
      case K_INTEGER: return c == '-' || is_digit(c);
      case K_LITERALS:
        for (auto& l : nd.literals)
          if (!l.empty() && (uint8_t)l[0] == c) return true;
        return false;
      case K_UNION:
        for (int ch : nd.children)
          if (first_ok(ch, c)) return true;
        return false;
    }
    return false;
  }

  bool feed(State& s, uint8_t c) const {
    for (int guard = 0; guard < 4 * kMaxDepth; ++guard) {
      if (s.n == 0) return false;  // document complete: only EOS
      Step r = step(s, c);
      if (r == ACCEPT) return true;
      if (r == REJECT) return false;
      if (r == END_RETRY) { complete_top(s); continue; }
      // PUSHED: feed the same byte to the (new / re-dispatched) top frame
    }
    return false;
  }

  bool accepts_eos(const State& s0) const {
    if (s0.done && s0.n == 0) return true;
    State s = s0;
    while (s.n > 0 && can_end(s.f[s.n - 1])) complete_top(s);
    return s.n == 0 && s.done;
  }

  // ---------------------------------------------------------------- masks
  void dfs(int tn, const State& st, uint32_t* mask) const {
    const Vocab& V = *vocab;
    const auto& node = V.nodes[tn];
    for (int e = 0; e < node.n_edges; ++e) {
      const auto& edge = V.edges[node.first_edge + e];
      State s2;
      s2.n = st.n;
      s2.done = st.done;
      std::memcpy(s2.f, st.f, sizeof(Frame) * st.n);
      if (!feed(s2, edge.first)) continue;
      const auto& ch = V.nodes[edge.second];
      for (int t = 0; t < ch.tok_count; ++t) {
        const int id = V.toks[ch.tok_begin + t];
        mask[id >> 5] |= (1u << (id & 31));
      }
      if (ch.n_edges) dfs(edge.second, s2, mask);
    }
  }

  const std::vector<uint32_t>& mask_for(const State& s) {
    std::string k = s.key();
    auto it = cache.find(k);
    if (it != cache.end()) {
      ++cache_hits;
      return it->second;
    }
    ++cache_misses;
    std::vector<uint32_t> m(vocab->words(), 0u);
    if (!(s.done && s.n == 0)) dfs(0, s, m.data());
    if (accepts_eos(s))
      for (int id : vocab->eos)
        if (id >= 0 && id < vocab->vocab_size) m[id >> 5] |= (1u << (id & 31));
    if (cache.size() > 200000) cache.clear();
    return cache.emplace(std::move(k), std::move(m)).first->second;
  }
};

class Matcher {
 public:
  std::shared_ptr<Grammar> g;
  State s;
  bool finished = false;
  std::vector<uint8_t> accepted;

  explicit Matcher(std::shared_ptr<Grammar> gr) : g(std::move(gr)) {
    s.f[0] = Grammar::mk(g->root, F_VALUE);
    s.n = 1;
  }

  bool accept_bytes(const std::string& b) {
    State t = s;
    for (unsigned char c : b)
      if (!g->feed(t, c)) return false;
    s = t;
    accepted.insert(accepted.end(), b.begin(), b.end());
    return true;
  }

  bool accept_token(int tid, const std::string& b) {
    for (int e : g->vocab->eos)
      if (e == tid) {
        if (!g->accepts_eos(s)) return false;
        finished = true;
        return true;
      }
    if (b.empty()) return false;
    return accept_bytes(b);
  }

  void fill_mask(py::buffer out) {
    py::buffer_info bi = out.request(true);
    if (bi.itemsize != 4 || bi.size < g->vocab->words())
      throw std::invalid_argument("mask buffer: need >= ceil(V/32) 32-bit words");
    auto* dst = static_cast<uint32_t*>(bi.ptr);
    if (finished) {
      std::memset(dst, 0, 4 * g->vocab->words());
      for (int id : g->vocab->eos) dst[id >> 5] |= (1u << (id & 31));
      return;
    }
    const auto& m = g->mask_for(s);
    std::memcpy(dst, m.data(), 4 * m.size());
  }

  bool is_complete() const { return g->accepts_eos(s); }
  bool can_continue() const { return !(s.done && s.n == 0); }
  py::bytes text() const { return py::bytes(reinterpret_cast<const char*>(accepted.data()), accepted.size()); }
};

std::shared_ptr<Grammar> make_grammar(std::shared_ptr<Vocab> v, const py::list& table, int root) {
  auto g = std::make_shared<Grammar>();
  g->vocab = std::move(v);
  g->root = root;
  for (auto item : table) {
    py::dict d = item.cast<py::dict>();
    Node n;
    n.kind = (Kind)d["kind"].cast<int>();
    if (d.contains("props"))
      for (auto p : d["props"].cast<py::list>()) {
        py::tuple t = p.cast<py::tuple>();
        n.props.push_back({t[0].cast<std::string>(), t[1].cast<int>(), t[2].cast<bool>()});
      }
    if (n.props.size() > 64) throw std::invalid_argument("at most 64 properties per object");
    if (d.contains("items")) n.items = d["items"].cast<int>();
    if (d.contains("min_items")) n.min_items = d["min_items"].cast<int>();
    if (d.contains("max_items")) n.max_items = d["max_items"].cast<int>();
    if (d.contains("min_len")) n.min_len = d["min_len"].cast<int>();
    if (d.contains("max_len")) n.max_len = d["max_len"].cast<int>();
    if (d.contains("literals")) n.literals = d["literals"].cast<std::vector<std::string>>();
    if (n.literals.size() > 64) throw std::invalid_argument("at most 64 enum values");
    if (d.contains("children")) n.children = d["children"].cast<std::vector<int>>();
    if (d.contains("tag_children")) {
      n.tag_children = d["tag_children"].cast<std::vector<int>>();
      if (n.props.size() < 2) throw std::invalid_argument("tagged object needs 2 properties");
    }
    g->nodes.push_back(std::move(n));
  }
  if (g->nodes.empty() || g->nodes[0].kind != K_ANY)
    throw std::invalid_argument("node 0 must be the ANY node");
  const int nn = (int)g->nodes.size();
  for (const Node& n : g->nodes) {  // every child reference in range
    auto bad = [nn](int i) { return i < 0 || i >= nn; };
    for (const Prop& p : n.props)
      if (bad(p.child)) throw std::invalid_argument("property child out of range");
    for (int c : n.children)
      if (bad(c)) throw std::invalid_argument("union child out of range");
    for (int c : n.tag_children)
      if (bad(c)) throw std::invalid_argument("tag child out of range");
    if (bad(n.items)) throw std::invalid_argument("items node out of range");
  }
  return g;
}

}  // namespace

void register_json_grammar(py::module_& m) {
  py::class_<Vocab, std::shared_ptr<Vocab>>(m, "GrammarVocab")
      .def(py::init<const std::vector<py::bytes>&, const std::vector<int>&>())
      .def_property_readonly("words", &Vocab::words)
      .def_property_readonly("trie_nodes", &Vocab::trie_nodes)
      .def_readonly("vocab_size", &Vocab::vocab_size);
  py::class_<Grammar, std::shared_ptr<Grammar>>(m, "JsonGrammar")
      .def(py::init(&make_grammar))
      .def_readonly("cache_hits", &Grammar::cache_hits)
      .def_readonly("cache_misses", &Grammar::cache_misses);
  py::class_<Matcher>(m, "JsonMatcher")
      .def(py::init<std::shared_ptr<Grammar>>())
      .def("accept_token", [](Matcher& mt, int tid, py::bytes b) {
        return mt.accept_token(tid, std::string(b));
      })
      .def("accept_bytes", [](Matcher& mt, py::bytes b) { return mt.accept_bytes(std::string(b)); })
      .def("fill_mask", &Matcher::fill_mask)
      .def("is_complete", &Matcher::is_complete)
      .def("can_continue", &Matcher::can_continue)
      .def_readonly("finished", &Matcher::finished)
      .def("text", &Matcher::text);
}
