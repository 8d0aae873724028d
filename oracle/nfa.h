// nfa.h — Thompson-NFA / Pike-VM membership simulator for ECMAScript
// regexes.  TEST INFRASTRUCTURE ONLY (oracle/): the long-input oracle of
// SURVEY.md §0.8 / §8(c).
//
// Why it exists: the reference engine behind HeaderMatcher regexes is
// libstdc++ std::regex with full-match semantics (ConfigUtility::matchHeaders
// called from envoy/cilium_network_policy.h:68-71; route.pb.go:2420-2430).
// Its backtracking executor is exponential on patterns like
// `(.{0,8}){1,8}foo` and overflows its stack on long subjects,
// so it cannot label BASELINE config 5.  For regular patterns regex_match's
// answer is language membership (the backtracker tries every alternative
// before it gives up; greedy / lazy only changes which match is reported),
// which this simulator computes in O(len x states) with no recursion.
//
// Independence: this parser does NOT share code with the product's regex
// front end (cilium_amd/csrc/regex_ecma.cc).  It follows the libstdc++
// ECMAScript grammar (GCC 11 bits/regex_scanner.tcc, regex_compiler.tcc) as
// probed in this container, and is pinned against std::regex_match by the
// differential fuzzer tests/cpp/fuzz_nfa.cc (tests/test_nfa_oracle_cpu.py):
//   * `.` excludes '\n' and '\r'; `\cX` is X; `\uHHHH` keeps the low byte;
//   * `[]` matches nothing, `[^]` everything; a leading ']' closes the class;
//   * ranges compare signed chars ([\x80-\xff] valid, [\x7f-\x80] not);
//     a class next to a range dash is an error ([\d-z], [a-\w]);
//   * `[[=x=]]` matches x in either case; `[[.x.]]` is the character x;
//   * stacked quantifiers (`a**`, `a{1}{2}`) and lazy markers parse;
//   * back-references and look-ahead throw Unsupported (regular subset only).
#pragma once
#include <bitset>
#include <cstdint>
#include <stdexcept>
#include <cstring>
#include <string>
#include <vector>

namespace nfa {

using ByteSet = std::bitset<256>;

struct SyntaxError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct Unsupported : std::runtime_error {
  using std::runtime_error::runtime_error;
};

enum Op : uint8_t { kByte, kSet, kSplit, kJmp, kBol, kEol, kWordB, kNotWordB, kMatch };
struct Inst {
  Op op;
  uint8_t ch;  // kByte
  uint32_t x;  // kSet: set id; kSplit / kJmp: target
  uint32_t y;  // kSplit: second target
};
struct Prog {
  std::vector<Inst> code;  // entry at 0; kByte / kSet / assertions fall through to pc + 1
  std::vector<ByteSet> sets;
  // Bytes every full match must start with (forced_prefix): a necessary
  // condition checked before the simulation, so a linear scan over many rules
  // rejects most of them with one compare.
  std::string prefix;
  bool exact = false;  // the pattern's language is {prefix} (a literal)
};

namespace detail {

inline bool is_digit(int c) { return c >= '0' && c <= '9'; }
inline bool is_xdigit(int c) { return is_digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
inline int hexv(int c) { return is_digit(c) ? c - '0' : (c | 0x20) - 'a' + 10; }

// classic-locale ctype classes over bytes 0..127 (bytes >= 0x80 belong to no class)
inline ByteSet cls(const std::string& name_in) {
  std::string n;
  for (char c : name_in) n.push_back(static_cast<char>(c >= 'A' && c <= 'Z' ? c + 32 : c));
  ByteSet s;
  for (int c = 0; c < 128; ++c) {
    const bool dig = is_digit(c), up = c >= 'A' && c <= 'Z', lo = c >= 'a' && c <= 'z';
    const bool alpha = up || lo, alnum = alpha || dig;
    const bool space = c == ' ' || (c >= 9 && c <= 13), cntrl = c < 32 || c == 127;
    const bool print = c >= 32 && c < 127, graph = c > 32 && c < 127;
    bool in;
    if (n == "d" || n == "digit") in = dig;
    else if (n == "w") in = alnum || c == '_';
    else if (n == "s" || n == "space") in = space;
    else if (n == "alnum") in = alnum;
    else if (n == "alpha") in = alpha;
    else if (n == "blank") in = c == ' ' || c == '\t';
    else if (n == "cntrl") in = cntrl;
    else if (n == "graph") in = graph;
    else if (n == "lower") in = lo;
    else if (n == "print") in = print;
    else if (n == "punct") in = graph && !alnum;
    else if (n == "upper") in = up;
    else if (n == "xdigit") in = is_xdigit(c);
    else throw SyntaxError("invalid character class");
    if (in) s.set(c);
  }
  return s;
}

// AST
struct Node {
  enum K { kSetN, kCat, kAlt, kRep, kAssert } k;
  ByteSet set;
  std::vector<int> kids;
  uint32_t lo = 0, hi = 0;  // kRep; hi == kInf: unbounded
  Op assert_op = kBol;
};
constexpr uint32_t kInf = 0xffffffffu;
constexpr uint32_t kMaxInsts = 4u << 20;  // expansion budget per pattern

class Parser {
 public:
  explicit Parser(const std::string& p) : p_(p) {}
  std::vector<Node> nodes;
  int parse() {
    const int r = disjunction();
    if (i_ != p_.size()) throw SyntaxError("mismatched ')'");
    return r;
  }

 private:
  const std::string& p_;
  size_t i_ = 0;
  int depth_ = 0;

  bool end() const { return i_ >= p_.size(); }
  int cur() const { return static_cast<unsigned char>(p_[i_]); }
  int add(Node n) {
    nodes.push_back(std::move(n));
    return static_cast<int>(nodes.size() - 1);
  }
  int set_node(const ByteSet& s) {
    Node n{Node::kSetN};
    n.set = s;
    return add(std::move(n));
  }
  static ByteSet one(int c) {
    ByteSet s;
    s.set(c & 0xff);
    return s;
  }

  int disjunction() {
    std::vector<int> alts{alternative()};
    while (!end() && cur() == '|') {
      ++i_;
      alts.push_back(alternative());
    }
    if (alts.size() == 1) return alts[0];
    Node n{Node::kAlt};
    n.kids = std::move(alts);
    return add(std::move(n));
  }
  int alternative() {
    Node n{Node::kCat};
    while (!end() && cur() != '|' && cur() != ')') n.kids.push_back(term());
    return add(std::move(n));
  }
  int term() {
    const int c = cur();
    if (c == '^' || c == '$') {  // assertions take no quantifier
      ++i_;
      Node n{Node::kAssert};
      n.assert_op = c == '^' ? kBol : kEol;
      return add(std::move(n));
    }
    if (c == '\\' && i_ + 1 < p_.size() && (p_[i_ + 1] == 'b' || p_[i_ + 1] == 'B')) {
      Node n{Node::kAssert};
      n.assert_op = p_[i_ + 1] == 'b' ? kWordB : kNotWordB;
      i_ += 2;
      return add(std::move(n));
    }
    int a = atom();
    for (;;) {  // stacked quantifiers apply in turn
      uint32_t lo, hi;
      if (end()) break;
      const int q = cur();
      if (q == '*') { lo = 0; hi = kInf; ++i_; }
      else if (q == '+') { lo = 1; hi = kInf; ++i_; }
      else if (q == '?') { lo = 0; hi = 1; ++i_; }
      else if (q == '{') { brace(&lo, &hi); }
      else break;
      if (!end() && cur() == '?') ++i_;  // non-greedy marker: same language
      Node n{Node::kRep};
      n.kids = {a};
      n.lo = lo;
      n.hi = hi;
      a = add(std::move(n));
    }
    return a;
  }
  uint32_t number() {
    if (end() || !is_digit(cur())) throw SyntaxError("brace: digit expected");
    uint64_t v = 0;
    while (!end() && is_digit(cur())) {
      v = v * 10 + static_cast<uint64_t>(cur() - '0');
      if (v > 100000) throw Unsupported("repeat count too large");
      ++i_;
    }
    return static_cast<uint32_t>(v);
  }
  void brace(uint32_t* lo, uint32_t* hi) {
    ++i_;  // '{'
    *lo = number();
    *hi = *lo;
    if (!end() && cur() == ',') {
      ++i_;
      *hi = (!end() && is_digit(cur())) ? number() : kInf;
    }
    if (end() || cur() != '}') throw SyntaxError("brace: '}' expected");
    ++i_;
    if (*hi != kInf && *hi < *lo) throw SyntaxError("brace: invalid range");
  }
  int atom() {
    if (end()) throw SyntaxError("atom expected");
    const int c = cur();
    switch (c) {
      case '*': case '+': case '?': case '{':
        throw SyntaxError("nothing to repeat");
      case ')': case '|':
        throw SyntaxError("unexpected token");
      case '.': {
        ++i_;
        ByteSet s;
        s.set();
        s.reset('\n');
        s.reset('\r');
        return set_node(s);
      }
      case '(': {
        ++i_;
        if (!end() && cur() == '?') {
          if (i_ + 1 < p_.size() && p_[i_ + 1] == ':') i_ += 2;
          else if (i_ + 1 < p_.size() && (p_[i_ + 1] == '=' || p_[i_ + 1] == '!')) throw Unsupported("look-ahead");
          else throw SyntaxError("invalid group");
        }
        if (++depth_ > 1000) throw Unsupported("nesting too deep");
        const int r = disjunction();
        --depth_;
        if (end() || cur() != ')') throw SyntaxError("parenthesis not closed");
        ++i_;
        return r;
      }
      case '[':
        ++i_;
        return set_node(bracket());
      case '\\':
        return set_node(escape(false));
      default:
        ++i_;
        return set_node(one(c));
    }
  }
  // After '\' (cur() == '\\').  In a bracket `\b` is backspace.
  ByteSet escape(bool in_bracket, bool* is_class = nullptr) {
    ++i_;
    if (end()) throw SyntaxError("trailing backslash");
    const int c = cur();
    ++i_;
    if (is_class) *is_class = false;
    switch (c) {
      case '0': return one(0);
      case 'b': return one(8);  // only reached inside brackets
      case 'f': return one('\f');
      case 'n': return one('\n');
      case 'r': return one('\r');
      case 't': return one('\t');
      case 'v': return one('\v');
      case 'd': case 'D': case 's': case 'S': case 'w': case 'W': {
        ByteSet s = cls(std::string(1, static_cast<char>(c)));
        if (c < 'a') s.flip();
        if (is_class) *is_class = true;
        return s;
      }
      case 'c':
        if (end()) throw SyntaxError("\\c at end");
        return one(p_[i_++]);
      case 'x': case 'u': {
        const int nd = c == 'x' ? 2 : 4;
        int v = 0;
        for (int k = 0; k < nd; ++k) {
          if (end() || !is_xdigit(cur())) throw SyntaxError("bad hex escape");
          v = v * 16 + hexv(cur());
          ++i_;
        }
        return one(v & 0xff);
      }
      default:
        if (is_digit(c)) throw Unsupported("back-reference");
        (void)in_bracket;
        return one(c);
    }
  }
  // Bracket expression after '[' (libstdc++ _M_expression_term, ECMAScript).
  ByteSet bracket() {
    bool neg = false;
    if (!end() && cur() == '^') {
      neg = true;
      ++i_;
    }
    ByteSet s;
    // pending single char (the possible start of a range) or a class
    enum { kNoLast, kChar, kClass } last = kNoLast;
    int lastc = 0;
    auto flush = [&]() {
      if (last == kChar) s.set(lastc & 0xff);
    };
    auto push_char = [&](int ch) {
      flush();
      last = kChar;
      lastc = ch;
    };
    auto push_class = [&](const ByteSet& cs) {
      flush();
      s |= cs;
      last = kClass;
    };
    // one "char" element: ordinary char, escape giving a char, [.x.]; returns false otherwise
    auto try_char = [&](int* out) -> bool {
      if (end()) return false;
      if (cur() == '\\') {
        const size_t save = i_;
        bool isc = false;
        ByteSet e = escape(true, &isc);
        if (isc) {
          i_ = save;
          return false;
        }
        for (int k = 0; k < 256; ++k)
          if (e.test(k)) *out = k;
        return true;
      }
      if (cur() == '[' && i_ + 1 < p_.size() && p_[i_ + 1] == '.') {
        const size_t close = p_.find(".]", i_ + 2);
        if (close == std::string::npos) throw SyntaxError("unterminated [.");
        const std::string name = p_.substr(i_ + 2, close - i_ - 2);
        if (name.size() != 1 || !((name[0] >= 'a' && name[0] <= 'z') || (name[0] >= 'A' && name[0] <= 'Z') ||
                                  is_digit(name[0])))
          throw Unsupported("collating element");
        *out = static_cast<unsigned char>(name[0]);
        i_ = close + 2;
        return true;
      }
      if (cur() == '[' && i_ + 1 < p_.size() && (p_[i_ + 1] == ':' || p_[i_ + 1] == '=')) return false;
      if (cur() == ']' || cur() == '-') return false;
      *out = cur();
      ++i_;
      return true;
    };
    for (;;) {
      if (end()) throw SyntaxError("bracket not closed");
      const int c = cur();
      if (c == ']') {  // ECMAScript: a leading ']' closes too ([] / [^])
        ++i_;
        break;
      }
      int ch;
      if (c == '[' && i_ + 1 < p_.size() && (p_[i_ + 1] == ':' || p_[i_ + 1] == '=')) {
        const char kind = p_[i_ + 1];
        const std::string term = std::string(1, kind) + "]";
        const size_t close = p_.find(term, i_ + 2);
        if (close == std::string::npos) throw SyntaxError("unterminated class name");
        const std::string name = p_.substr(i_ + 2, close - i_ - 2);
        i_ = close + 2;
        if (kind == ':') {
          push_class(cls(name));
        } else {  // [=x=]: equivalence class, transform_primary lower-cases
          if (name.size() != 1) throw Unsupported("equivalence class");
          ByteSet e;
          int x = static_cast<unsigned char>(name[0]);
          e.set(x);
          if (x >= 'A' && x <= 'Z') e.set(x + 32);
          if (x >= 'a' && x <= 'z') e.set(x - 32);
          push_class(e);
        }
        continue;
      }
      if (c == '\\') {
        const size_t save = i_;
        bool isc = false;
        ByteSet e = escape(true, &isc);
        if (isc) {
          push_class(e);
          continue;
        }
        i_ = save;
      }
      if (c == '-') {
        ++i_;
        if (!end() && cur() == ']') {  // "-]": literal dash
          push_char('-');
          continue;
        }
        if (last == kClass) throw SyntaxError("invalid start of range");
        if (last == kChar) {
          int hi;
          if (try_char(&hi)) {
          } else if (!end() && cur() == '-') {
            hi = '-';
            ++i_;
          } else {
            throw SyntaxError("invalid end of range");
          }
          const int a = static_cast<signed char>(lastc), b = static_cast<signed char>(hi);
          if (a > b) throw SyntaxError("invalid range");
          for (int k = a; k <= b; ++k) s.set(static_cast<unsigned char>(static_cast<signed char>(k)));
          last = kNoLast;
          continue;
        }
        push_char('-');  // a dash outside any range (ECMAScript)
        continue;
      }
      if (!try_char(&ch)) throw SyntaxError("unexpected character in bracket");
      push_char(ch);
    }
    flush();
    if (neg) s.flip();
    return s;
  }
};

class Compiler {
 public:
  Compiler(const std::vector<Node>& n, Prog* p) : n_(n), p_(p) {}
  void emit(int id) {
    const Node& nd = n_[id];
    switch (nd.k) {
      case Node::kSetN: {
        if (nd.set.count() == 1) {
          int c = 0;
          while (!nd.set.test(c)) ++c;
          put(Inst{kByte, static_cast<uint8_t>(c), 0, 0});
        } else {
          uint32_t sid = 0;
          while (sid < p_->sets.size() && p_->sets[sid] != nd.set) ++sid;
          if (sid == p_->sets.size()) p_->sets.push_back(nd.set);
          put(Inst{kSet, 0, sid, 0});
        }
        return;
      }
      case Node::kAssert:
        put(Inst{nd.assert_op, 0, 0, 0});
        return;
      case Node::kCat:
        for (int k : nd.kids) emit(k);
        return;
      case Node::kAlt: {
        std::vector<uint32_t> jumps;
        for (size_t k = 0; k < nd.kids.size(); ++k) {
          if (k + 1 < nd.kids.size()) {
            const uint32_t sp = put(Inst{kSplit, 0, 0, 0});
            p_->code[sp].x = pc();
            emit(nd.kids[k]);
            jumps.push_back(put(Inst{kJmp, 0, 0, 0}));
            p_->code[sp].y = pc();
          } else {
            emit(nd.kids[k]);
          }
        }
        for (uint32_t j : jumps) p_->code[j].x = pc();
        return;
      }
      case Node::kRep: {
        const int e = nd.kids[0];
        for (uint32_t k = 0; k < nd.lo; ++k) emit(e);
        if (nd.hi == kInf) {  // L: split body, out; body; jmp L
          const uint32_t sp = put(Inst{kSplit, 0, 0, 0});
          p_->code[sp].x = pc();
          emit(e);
          put(Inst{kJmp, 0, sp, 0});
          p_->code[sp].y = pc();
        } else {  // (hi - lo) nested optional copies, all exits to the end
          std::vector<uint32_t> outs;
          for (uint32_t k = nd.lo; k < nd.hi; ++k) {
            const uint32_t sp = put(Inst{kSplit, 0, 0, 0});
            p_->code[sp].x = pc();
            outs.push_back(sp);
            emit(e);
          }
          for (uint32_t sp : outs) p_->code[sp].y = pc();
        }
        return;
      }
    }
  }
  uint32_t pc() const { return static_cast<uint32_t>(p_->code.size()); }

 private:
  const std::vector<Node>& n_;
  Prog* p_;
  uint32_t put(const Inst& in) {
    if (p_->code.size() >= kMaxInsts) throw Unsupported("pattern expands past the instruction budget");
    p_->code.push_back(in);
    return static_cast<uint32_t>(p_->code.size() - 1);
  }
};

}  // namespace detail

// Parse + compile.  Throws SyntaxError where std::regex would throw, and
// Unsupported for constructs outside the regular subset.
inline Prog compile(const std::string& pattern) {
  detail::Parser ps(pattern);
  const int root = ps.parse();
  Prog p;
  detail::Compiler cc(ps.nodes, &p);
  cc.emit(root);
  p.code.push_back(Inst{kMatch, 0, 0, 0});
  // Forced prefix: from the current point, the epsilon closure taken with
  // every assertion passing (a superset of the real closure) holds exactly one
  // consuming instruction, a single byte, and no match: that byte must come
  // next.  Sound for full match, whatever the assertions decide.
  std::vector<uint32_t> stack, seen(p.code.size(), 0);
  uint32_t gen = 0, pc0 = 0;
  bool asserts = false;
  while (p.prefix.size() < 256) {
    ++gen;
    stack.assign(1, pc0);
    int consumers = 0;
    uint32_t only = 0;
    bool match = false;
    while (!stack.empty()) {
      const uint32_t pc = stack.back();
      stack.pop_back();
      if (seen[pc] == gen) continue;
      seen[pc] = gen;
      const Inst& in = p.code[pc];
      switch (in.op) {
        case kByte: case kSet: ++consumers; only = pc; break;
        case kMatch: match = true; break;
        case kJmp: stack.push_back(in.x); break;
        case kSplit: stack.push_back(in.y); stack.push_back(in.x); break;
        default: asserts = true; stack.push_back(pc + 1); break;  // assertions: assumed to pass
      }
    }
    if (match && consumers == 0 && !asserts) p.exact = true;
    if (match || consumers != 1) break;
    const Inst& in = p.code[only];
    int ch = in.op == kByte ? in.ch : -1;
    if (in.op == kSet && p.sets[in.x].count() == 1)
      for (int c = 0; c < 256; ++c)
        if (p.sets[in.x].test(c)) ch = c;
    if (ch < 0) break;
    p.prefix.push_back(static_cast<char>(ch));
    pc0 = only + 1;
  }
  return p;
}

// Pike-VM membership: full match (regex_match) or search (regex_search).
class Runner {
 public:
  bool run(const Prog& p, const uint8_t* s, size_t n, bool search) {
    if (!search && (n < p.prefix.size() || std::memcmp(s, p.prefix.data(), p.prefix.size()) != 0)) return false;
    if (!search && p.exact) return n == p.prefix.size();
    const size_t m = p.code.size();
    if (sparse_.size() < m) {
      sparse_.assign(m, 0);
      stamp_.assign(m, 0);
      cur_.reserve(m);
      nxt_.reserve(m);
    }
    cur_.clear();
    bool matched = false;
    add(p, s, n, 0, &cur_, &matched);
    for (size_t pos = 0;; ++pos) {
      if (search && matched) return true;
      if (pos == n) return matched;
      if (cur_.empty() && !search) return false;
      const uint8_t c = s[pos];
      nxt_.clear();
      matched = false;
      for (uint32_t pc : cur_) {
        const Inst& in = p.code[pc];
        const bool ok = in.op == kByte ? in.ch == c : in.op == kSet ? p.sets[in.x].test(c) : false;
        if (ok) add(p, s, n, pos + 1, &nxt_, &matched, pc + 1);
      }
      if (search) add(p, s, n, pos + 1, &nxt_, &matched);  // a new attempt at every position
      cur_.swap(nxt_);
    }
  }

 private:
  std::vector<uint32_t> sparse_, stamp_, cur_, nxt_, stack_;
  uint32_t gen_ = 0;

  static bool word(const uint8_t* s, size_t n, size_t i) {
    if (i >= n) return false;
    const int c = s[i];
    return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_';
  }
  // epsilon closure of pc at position pos into list (iterative, cycle-safe)
  void add(const Prog& p, const uint8_t* s, size_t n, size_t pos, std::vector<uint32_t>* list, bool* matched,
           uint32_t pc0 = 0) {
    if (list->empty()) {
      if (++gen_ == 0) {
        std::fill(stamp_.begin(), stamp_.end(), 0);
        gen_ = 1;
      }
    }
    stack_.clear();
    stack_.push_back(pc0);
    while (!stack_.empty()) {
      const uint32_t pc = stack_.back();
      stack_.pop_back();
      if (stamp_[pc] == gen_) continue;
      stamp_[pc] = gen_;
      const Inst& in = p.code[pc];
      switch (in.op) {
        case kByte: case kSet: list->push_back(pc); break;
        case kMatch: *matched = true; break;
        case kJmp: stack_.push_back(in.x); break;
        case kSplit: stack_.push_back(in.y); stack_.push_back(in.x); break;
        case kBol: if (pos == 0) stack_.push_back(pc + 1); break;
        case kEol: if (pos == n) stack_.push_back(pc + 1); break;
        case kWordB: case kNotWordB: {
          const bool b = (pos > 0 && word(s, n, pos - 1)) != word(s, n, pos);
          if (b == (in.op == kWordB)) stack_.push_back(pc + 1);
          break;
        }
      }
    }
  }
};

}  // namespace nfa
