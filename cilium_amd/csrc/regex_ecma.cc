// regex_ecma.cc — see regex_ecma.h.
//
// The grammar below follows the token rules of libstdc++'s std::regex
// ECMAScript scanner/compiler (GCC 11: bits/regex_scanner.tcc,
// bits/regex_compiler.tcc) because that is the engine Envoy links for
// HeaderMatcher regexes (reference: envoy/cilium_network_policy.h:52-71).
// Quirks reproduced on purpose (pinned against std::regex in this container
// by the differential fuzzer tests/cpp/fuzz_regex.cc, run from
// tests/test_http_cpu.py::test_regex_compiler_differential_fuzz):
//   * `\cX` is the character X (libstdc++ does not compute a control char);
//   * `\uHHHH` keeps only the low byte; `\0` is NUL and stops (no octal);
//   * `.` matches every byte except '\n' and '\r';
//   * `[]` matches nothing, `[^]` matches every byte;
//   * bracket ranges compare bytes as *signed* char ([\x80-\xff] is valid,
//     [\x7f-\x80] is not) and a class next to '-' ([\d-z]) is an error;
//   * `[[=x=]]` matches x in either case (transform_primary lower-cases);
//   * `a**`, `a{1}{2}` stack quantifiers; a '?' right after a quantifier is
//     its non-greedy marker (irrelevant for membership, relevant for parsing).
#include "regex_ecma.h"

#include <algorithm>
#include <functional>
#include <cstring>
#include <locale>
#include <map>
#include <unordered_map>
#include <unordered_set>

namespace l7m {
namespace re {
namespace {

// ---------------------------------------------------------------- classes --
const std::ctype<char>& classic_ctype() {
  static const std::ctype<char>& ct = std::use_facet<std::ctype<char>>(std::locale::classic());
  return ct;
}

ByteSet mask_set(std::ctype_base::mask m, bool under) {
  ByteSet s;
  const auto& ct = classic_ctype();
  for (int c = 0; c < 256; ++c) {
    char ch = static_cast<char>(c);
    if (ct.is(m, ch) || (under && ch == '_')) s.set(c);
  }
  return s;
}

// regex_traits<char>::lookup_classname (names compared after tolower).
bool lookup_class(const std::string& raw, ByteSet* out) {
  std::string n;
  for (char c : raw) n.push_back(static_cast<char>(classic_ctype().tolower(c)));
  using cb = std::ctype_base;
  if (n == "d" || n == "digit") { *out = mask_set(cb::digit, false); return true; }
  if (n == "w") { *out = mask_set(cb::alnum, true); return true; }
  if (n == "s" || n == "space") { *out = mask_set(cb::space, false); return true; }
  if (n == "alnum") { *out = mask_set(cb::alnum, false); return true; }
  if (n == "alpha") { *out = mask_set(cb::alpha, false); return true; }
  if (n == "blank") { *out = mask_set(cb::blank, false); return true; }
  if (n == "cntrl") { *out = mask_set(cb::cntrl, false); return true; }
  if (n == "graph") { *out = mask_set(cb::graph, false); return true; }
  if (n == "lower") { *out = mask_set(cb::lower, false); return true; }
  if (n == "print") { *out = mask_set(cb::print, false); return true; }
  if (n == "punct") { *out = mask_set(cb::punct, false); return true; }
  if (n == "upper") { *out = mask_set(cb::upper, false); return true; }
  if (n == "xdigit") { *out = mask_set(cb::xdigit, false); return true; }
  return false;
}

ByteSet any_but_newline() {
  ByteSet s;
  s.set();
  s.reset('\n');
  s.reset('\r');
  return s;
}

// ---------------------------------------------------------------- scanner --
enum Tok {
  T_EOF, T_ORD, T_HEX, T_BACKREF, T_QCLASS, T_WORDB, T_BOL, T_EOL, T_ANY, T_STAR, T_PLUS,
  T_OPT, T_OR, T_SUB, T_SUBNG, T_LOOKAHEAD, T_SUBEND, T_BRACK, T_BRACKNEG, T_BRACKEND,
  T_DASH, T_COLL, T_EQUIV, T_CLASSNAME, T_IBEGIN, T_IEND, T_DUP, T_COMMA,
};

struct ParseError {
  Status st;
  std::string msg;
};

class Parser {
 public:
  explicit Parser(const std::string& p) : p_(p) {}

  Ast run() {
    advance();
    int root = disjunction();
    if (tok_ != T_EOF) fail(Status::Syntax, "unexpected token");
    ast_.root = root;
    return std::move(ast_);
  }

 private:
  enum State { S_NORMAL, S_BRACKET, S_BRACE };

  [[noreturn]] void fail(Status st, const char* m) { throw ParseError{st, m}; }

  bool at_end() const { return i_ >= p_.size(); }
  unsigned char cur() const { return static_cast<unsigned char>(p_[i_]); }

  static bool is_digit(unsigned char c) { return c >= '0' && c <= '9'; }
  static bool is_xdigit(unsigned char c) {
    return is_digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
  }
  static int hexval(unsigned char c) {
    if (is_digit(c)) return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    return c - 'A' + 10;
  }

  // _M_eat_escape_ecma
  void eat_escape() {
    if (at_end()) fail(Status::Syntax, "trailing backslash");
    unsigned char c = p_[i_++];
    static const char tbl[][2] = {{'0', '\0'}, {'b', '\b'}, {'f', '\f'}, {'n', '\n'},
                                  {'r', '\r'}, {'t', '\t'}, {'v', '\v'}};
    const char* hit = nullptr;
    for (auto& e : tbl)
      if (static_cast<unsigned char>(e[0]) == c) hit = &e[1];
    if (hit && (c != 'b' || state_ == S_BRACKET)) {
      tok_ = T_ORD;
      val_ = static_cast<unsigned char>(*hit);
    } else if (c == 'b' || c == 'B') {
      tok_ = T_WORDB;
      val_ = c;
    } else if (c == 'd' || c == 'D' || c == 's' || c == 'S' || c == 'w' || c == 'W') {
      tok_ = T_QCLASS;
      val_ = c;
    } else if (c == 'c') {
      if (at_end()) fail(Status::Syntax, "\\c at end");
      tok_ = T_ORD;
      val_ = cur();
      ++i_;
    } else if (c == 'x' || c == 'u') {
      int n = c == 'x' ? 2 : 4;
      unsigned v = 0;
      for (int k = 0; k < n; ++k) {
        if (at_end() || !is_xdigit(cur())) fail(Status::Syntax, "bad hex escape");
        v = v * 16 + hexval(cur());
        ++i_;
      }
      tok_ = T_HEX;
      val_ = v & 0xff;  // _M_value.assign(1, int) narrows to char
    } else if (is_digit(c)) {
      unsigned long long v = c - '0';
      while (!at_end() && is_digit(cur())) {
        v = v * 10 + (cur() - '0');
        if (v > (1ull << 30)) v = 1ull << 30;
        ++i_;
      }
      tok_ = T_BACKREF;
      num_ = v;
    } else {
      tok_ = T_ORD;
      val_ = c;
    }
  }

  void eat_class(char close) {  // _M_eat_class: read until close + ']'
    str_.clear();
    while (i_ < p_.size() && p_[i_] != close) str_.push_back(p_[i_++]);
    if (i_ >= p_.size()) fail(Status::Syntax, "unterminated [: :]");
    ++i_;
    if (i_ >= p_.size() || p_[i_] != ']') fail(Status::Syntax, "unterminated [: :]");
    ++i_;
  }

  void advance() {
    if (at_end()) {
      if (state_ != S_NORMAL) fail(Status::Syntax, "unterminated bracket/brace");
      tok_ = T_EOF;
      return;
    }
    if (state_ == S_BRACE) {
      unsigned char c = p_[i_++];
      if (is_digit(c)) {
        unsigned long long v = c - '0';
        while (!at_end() && is_digit(cur())) {
          v = v * 10 + (cur() - '0');
          if (v > (1ull << 40)) v = 1ull << 40;
          ++i_;
        }
        tok_ = T_DUP;
        num_ = v;
      } else if (c == ',') {
        tok_ = T_COMMA;
      } else if (c == '}') {
        state_ = S_NORMAL;
        tok_ = T_IEND;
      } else {
        fail(Status::Syntax, "bad brace");
      }
      return;
    }
    if (state_ == S_BRACKET) {
      unsigned char c = p_[i_++];
      if (c == '-') {
        tok_ = T_DASH;
      } else if (c == '[') {
        if (at_end()) fail(Status::Syntax, "incomplete [[");
        unsigned char d = cur();
        if (d == '.') { ++i_; tok_ = T_COLL; eat_class('.'); }
        else if (d == ':') { ++i_; tok_ = T_CLASSNAME; eat_class(':'); }
        else if (d == '=') { ++i_; tok_ = T_EQUIV; eat_class('='); }
        else { tok_ = T_ORD; val_ = c; }
      } else if (c == ']') {
        tok_ = T_BRACKEND;
        state_ = S_NORMAL;
      } else if (c == '\\') {
        eat_escape();
      } else {
        tok_ = T_ORD;
        val_ = c;
      }
      return;
    }
    unsigned char c = p_[i_++];
    static const char* spec = "^$\\.*+?()[]{}|";
    if (c == 0 || std::strchr(spec, c) == nullptr) {
      if (c == 0) fail(Status::Unsupported, "NUL in pattern");
      tok_ = T_ORD;
      val_ = c;
      return;
    }
    switch (c) {
      case '\\': eat_escape(); return;
      case '(':
        if (!at_end() && cur() == '?') {
          ++i_;
          if (at_end()) fail(Status::Syntax, "(? at end");
          unsigned char d = p_[i_++];
          if (d == ':') tok_ = T_SUBNG;
          else if (d == '=' || d == '!') {
            tok_ = T_LOOKAHEAD;
            val_ = d;
          }
          else fail(Status::Syntax, "bad (?");
        } else {
          tok_ = T_SUB;
        }
        return;
      case ')': tok_ = T_SUBEND; return;
      case '[':
        state_ = S_BRACKET;
        if (!at_end() && cur() == '^') { tok_ = T_BRACKNEG; ++i_; }
        else tok_ = T_BRACK;
        return;
      case '{': state_ = S_BRACE; tok_ = T_IBEGIN; return;
      case ']': case '}': tok_ = T_ORD; val_ = c; return;
      case '^': tok_ = T_BOL; return;
      case '$': tok_ = T_EOL; return;
      case '.': tok_ = T_ANY; return;
      case '*': tok_ = T_STAR; return;
      case '+': tok_ = T_PLUS; return;
      case '?': tok_ = T_OPT; return;
      case '|': tok_ = T_OR; return;
    }
    fail(Status::Syntax, "scanner");
  }

  bool match(Tok t) {
    if (tok_ != t) return false;
    advance();
    return true;
  }

  int add(Node n) {
    ast_.nodes.push_back(std::move(n));
    return static_cast<int>(ast_.nodes.size()) - 1;
  }
  int mk_set(const ByteSet& s) {
    Node n;
    n.kind = Node::Set;
    n.set = s;
    return add(std::move(n));
  }
  int mk(Node::Kind k) {
    Node n;
    n.kind = k;
    return add(std::move(n));
  }

  int disjunction() {
    std::vector<int> alts{alternative()};
    while (match(T_OR)) alts.push_back(alternative());
    if (alts.size() == 1) return alts[0];
    Node n;
    n.kind = Node::Alt;
    n.kids = std::move(alts);
    return add(std::move(n));
  }

  int alternative() {
    std::vector<int> seq;
    for (;;) {
      int t = term();
      if (t < 0) break;
      seq.push_back(t);
    }
    if (seq.empty()) return mk(Node::Empty);
    if (seq.size() == 1) return seq[0];
    Node n;
    n.kind = Node::Cat;
    n.kids = std::move(seq);
    return add(std::move(n));
  }

  // _M_term: an assertion (^ $ \b \B (?=X) (?!X)) takes no quantifier.
  int term() {
    if (tok_ == T_BOL) { advance(); return mk(Node::Bol); }
    if (tok_ == T_EOL) { advance(); return mk(Node::Eol); }
    if (tok_ == T_WORDB) {
      const bool neg = val_ == 'B';
      advance();
      Node n;
      n.kind = Node::WordB;
      n.min = neg ? 1 : 0;
      return add(std::move(n));
    }
    if (tok_ == T_LOOKAHEAD) {
      const bool neg = val_ == '!';
      advance();
      const int r = disjunction();
      if (!match(T_SUBEND)) fail(Status::Syntax, "missing )");
      Node n;
      n.kind = Node::Look;
      n.min = neg ? 1 : 0;
      n.kids = {r};
      return add(std::move(n));
    }
    int a = atom();
    if (a < 0) return -1;
    for (;;) {
      int q = quantifier(a);
      if (q < 0) break;
      a = q;
    }
    return a;
  }

  int rep(int kid, int mn, int mx, bool lazy) {
    Node n;
    n.kind = Node::Rep;
    n.kids = {kid};
    n.min = mn;
    n.max = mx;
    n.lazy = lazy;
    return add(std::move(n));
  }

  int quantifier(int a) {
    if (match(T_STAR)) return rep(a, 0, -1, match(T_OPT));
    if (match(T_PLUS)) return rep(a, 1, -1, match(T_OPT));
    if (match(T_OPT)) return rep(a, 0, 1, match(T_OPT));
    if (match(T_IBEGIN)) {
      if (tok_ != T_DUP) fail(Status::Syntax, "bad brace");
      unsigned long long mn = num_;
      advance();
      long long mx = static_cast<long long>(mn);
      if (match(T_COMMA)) {
        if (tok_ == T_DUP) {
          mx = static_cast<long long>(num_);
          advance();
        } else {
          mx = -1;
        }
      }
      if (!match(T_IEND)) fail(Status::Syntax, "bad brace");
      const bool lazy = match(T_OPT);
      if (mx >= 0 && mx < static_cast<long long>(mn)) fail(Status::Syntax, "bad brace range");
      if (mn > 100000 || mx > 100000) fail(Status::TooBig, "repeat count");
      const int r = rep(a, static_cast<int>(mn), static_cast<int>(mx), lazy);
      ast_.nodes[r].brace = true;
      return r;
    }
    return -1;
  }

  bool try_char(unsigned* v) {
    if (tok_ == T_ORD || tok_ == T_HEX) {
      *v = val_;
      advance();
      return true;
    }
    return false;
  }

  int atom() {
    unsigned v;
    if (match(T_ANY)) return mk_set(any_but_newline());
    if (try_char(&v)) {
      ByteSet s;
      s.set(v);
      return mk_set(s);
    }
    if (tok_ == T_BACKREF) {
      const unsigned long long k = num_;
      advance();
      if (k < 1 || k >= static_cast<unsigned long long>(groups_)) fail(Status::Syntax, "back-reference");
      // _M_insert_backref: "referred to an opened sub-expression" (error_backref)
      for (int g : open_) if (static_cast<unsigned long long>(g) == k) fail(Status::Syntax, "back-reference to an open group");
      Node n;
      n.kind = Node::Backref;
      n.min = static_cast<int>(k);
      return add(std::move(n));
    }
    if (tok_ == T_QCLASS) {
      unsigned char c = static_cast<unsigned char>(val_);
      advance();
      ByteSet s;
      lookup_class(std::string(1, static_cast<char>(c)), &s);
      if (c >= 'A' && c <= 'Z') s.flip();
      return mk_set(s);
    }
    if (tok_ == T_SUBNG) {
      advance();
      int r = disjunction();
      if (!match(T_SUBEND)) fail(Status::Syntax, "missing )");
      return r;
    }
    if (tok_ == T_SUB) {  // capture group: numbered by its '(' (_M_insert_subexpr_begin)
      advance();
      const int idx = groups_++;
      open_.push_back(idx);
      int r = disjunction();
      if (!match(T_SUBEND)) fail(Status::Syntax, "missing )");
      open_.pop_back();
      Node n;
      n.kind = Node::Group;
      n.min = idx;
      n.kids = {r};
      return add(std::move(n));
    }
    if (tok_ == T_BRACK || tok_ == T_BRACKNEG) {
      bool neg = tok_ == T_BRACKNEG;
      advance();
      return bracket(neg);
    }
    return -1;
  }

  // --- bracket expressions (_M_insert_bracket_matcher / _M_expression_term)
  struct Last {
    enum { None, Char, Class } type = None;
    unsigned ch = 0;
  };
  struct Brk {
    ByteSet chars;                 // _M_char_set + _M_range_set + _M_class_set + equiv
    std::vector<ByteSet> negcls;   // _M_neg_class_set
  };

  void add_range(Brk& b, unsigned lo, unsigned hi) {
    int l = static_cast<signed char>(lo), h = static_cast<signed char>(hi);
    if (l > h) fail(Status::Syntax, "bad range");
    for (int c = 0; c < 256; ++c) {
      int sc = static_cast<signed char>(c);
      if (l <= sc && sc <= h) b.chars.set(c);
    }
  }

  bool expression_term(Last& last, Brk& b) {
    if (match(T_BRACKEND)) return false;
    auto push_char = [&](unsigned ch) {
      if (last.type == Last::Char) b.chars.set(last.ch);
      last.type = Last::Char;
      last.ch = ch;
    };
    auto push_class = [&]() {
      if (last.type == Last::Char) b.chars.set(last.ch);
      last.type = Last::Class;
    };
    unsigned v;
    if (tok_ == T_COLL) {
      std::string s = str_;
      advance();
      if (s.size() != 1) fail(Status::Unsupported, "multi-char collating element");
      push_char(static_cast<unsigned char>(s[0]));
    } else if (tok_ == T_EQUIV) {
      std::string s = str_;
      advance();
      if (s.size() != 1) fail(Status::Unsupported, "multi-char equivalence class");
      push_class();
      const auto& ct = classic_ctype();
      char want = ct.tolower(s[0]);
      for (int c = 0; c < 256; ++c)
        if (ct.tolower(static_cast<char>(c)) == want) b.chars.set(c);
    } else if (tok_ == T_CLASSNAME) {
      std::string s = str_;
      advance();
      push_class();
      ByteSet cs;
      if (!lookup_class(s, &cs)) fail(Status::Syntax, "unknown class name");
      b.chars |= cs;
    } else if (try_char(&v)) {
      push_char(v);
    } else if (match(T_DASH)) {
      if (match(T_BRACKEND)) {
        push_char('-');
        return false;
      } else if (last.type == Last::Class) {
        fail(Status::Syntax, "class as range start");
      } else if (last.type == Last::Char) {
        if (try_char(&v)) {
          add_range(b, last.ch, v);
          last.type = Last::None;
        } else if (match(T_DASH)) {
          add_range(b, last.ch, '-');
          last.type = Last::None;
        } else {
          fail(Status::Syntax, "bad range end");
        }
      } else {
        push_char('-');
      }
    } else if (tok_ == T_QCLASS) {
      unsigned char c = static_cast<unsigned char>(val_);
      advance();
      push_class();
      ByteSet cs;
      lookup_class(std::string(1, static_cast<char>(c)), &cs);
      if (c >= 'A' && c <= 'Z') b.negcls.push_back(cs);
      else b.chars |= cs;
    } else {
      fail(Status::Syntax, "unexpected token in bracket");
    }
    return true;
  }

  int bracket(bool neg) {
    Brk b;
    Last last;
    unsigned v;
    if (try_char(&v)) {
      last.type = Last::Char;
      last.ch = v;
    } else if (match(T_DASH)) {
      last.type = Last::Char;
      last.ch = '-';
    }
    while (expression_term(last, b)) {
    }
    if (last.type == Last::Char) b.chars.set(last.ch);
    ByteSet s = b.chars;
    for (const auto& nc : b.negcls) s |= ~nc;
    if (neg) s.flip();
    return mk_set(s);
  }

  const std::string& p_;
  size_t i_ = 0;
  State state_ = S_NORMAL;
  Tok tok_ = T_EOF;
  unsigned val_ = 0;
  unsigned long long num_ = 0;
  std::string str_;
  Ast ast_;
  int groups_ = 1;  // capture groups opened so far + 1 (group 0 = the whole match)
  std::vector<int> open_;  // capture groups whose ')' is still ahead (_M_paren_stack)
};

// ------------------------------------------------------------------- NFA --
struct NState {
  enum : uint8_t { CHR, SPLIT, EPS, BOL, EOL, MATCH, WORDB, LOOK } type;
  int out1 = -1, out2 = -1;
  int cs = -1;   // CHR: set id; LOOK: look-ahead automaton id
  int pat = -1;  // MATCH: pattern id; WORDB / LOOK: 1 = negated
};

// The automaton of a look-ahead (?=X) / (?!X): the DFA of X [\x00-\xff]*
// read as a full match of the rest of the subject -- libstdc++'s sub-executor
// (regex_executor.tcc _M_lookahead) runs X in prefix mode on [current, end)
// with current as its own begin, so '^' inside X holds at the look-ahead's
// position and '\b' there sees no character before it, exactly as for a
// subject that starts there.  `universal` marks the states from which every
// continuation is accepted at the end (the obligation is met, whatever follows).
struct LookDfa {
  Dfa dfa;
  std::vector<uint8_t> universal;
  bool neg = false;
};

struct Nfa {
  std::vector<NState> st;
  std::vector<ByteSet> sets;
  std::unordered_map<std::string, int> set_ids;
  std::vector<LookDfa> looks;
  bool ctx = false;  // has WORDB / LOOK states (context construction)
  DfaLimits lim;
  size_t limit = 8u << 20;

  int add(NState s) {
    if (st.size() >= limit) throw ParseError{Status::TooBig, "NFA too large"};
    st.push_back(s);
    return static_cast<int>(st.size()) - 1;
  }
  int set_id(const ByteSet& s) {
    std::string key = s.to_string();
    auto it = set_ids.find(key);
    if (it != set_ids.end()) return it->second;
    sets.push_back(s);
    int id = static_cast<int>(sets.size()) - 1;
    set_ids.emplace(std::move(key), id);
    return id;
  }

  int look_dfa(const Ast& a, int node, bool neg);

  // Thompson construction: returns the entry state of `node` continuing to `next`.
  int compile(const Ast& a, int node, int next) {
    const Node& n = a.nodes[node];
    switch (n.kind) {
      case Node::Empty:
        return next;
      case Node::Set: {
        NState s;
        s.type = NState::CHR;
        s.cs = set_id(n.set);
        s.out1 = next;
        return add(s);
      }
      case Node::Bol:
      case Node::Eol: {
        NState s;
        s.type = n.kind == Node::Bol ? NState::BOL : NState::EOL;
        s.out1 = next;
        return add(s);
      }
      case Node::WordB: {
        NState s;
        s.type = NState::WORDB;
        s.pat = n.min;
        s.out1 = next;
        ctx = true;
        return add(s);
      }
      case Node::Look: {
        NState s;
        s.type = NState::LOOK;
        s.pat = n.min;
        s.cs = look_dfa(a, n.kids[0], n.min != 0);
        s.out1 = next;
        ctx = true;
        return add(s);
      }
      case Node::Group:
        return compile(a, n.kids[0], next);
      case Node::Backref:
        throw ParseError{Status::Unsupported, "back-reference (lower_for_dfa first)"};
      case Node::Cat: {
        int cur = next;
        for (size_t k = n.kids.size(); k-- > 0;) cur = compile(a, n.kids[k], cur);
        return cur;
      }
      case Node::Alt: {
        int cur = compile(a, n.kids.back(), next);
        for (size_t k = n.kids.size() - 1; k-- > 0;) {
          int left = compile(a, n.kids[k], next);
          NState s;
          s.type = NState::SPLIT;
          s.out1 = left;
          s.out2 = cur;
          cur = add(s);
        }
        return cur;
      }
      case Node::Rep: {
        int kid = n.kids[0];
        int cur = next;
        if (n.max < 0) {
          NState s;
          s.type = NState::SPLIT;
          int loop = add(s);
          int body = compile(a, kid, loop);
          st[loop].out1 = body;
          st[loop].out2 = next;
          cur = loop;
        } else {
          for (int k = 0; k < n.max - n.min; ++k) {
            int body = compile(a, kid, cur);
            NState s;
            s.type = NState::SPLIT;
            s.out1 = body;
            s.out2 = next;
            cur = add(s);
          }
        }
        for (int k = 0; k < n.min; ++k) cur = compile(a, kid, cur);
        return cur;
      }
    }
    return next;
  }
};

struct VecHash {
  size_t operator()(const std::vector<int>& v) const {
    uint64_t h = 1469598103934665603ull;
    for (int x : v) {
      h ^= static_cast<uint32_t>(x);
      h *= 1099511628211ull;
    }
    return static_cast<size_t>(h ^ (h >> 29));
  }
};
struct U32VecHash {
  size_t operator()(const std::vector<uint32_t>& v) const {
    uint64_t h = 1469598103934665603ull;
    for (uint32_t x : v) {
      h ^= x;
      h *= 1099511628211ull;
    }
    return static_cast<size_t>(h ^ (h >> 29));
  }
};

class Closure {
 public:
  explicit Closure(const Nfa& n) : n_(n), mark_(n.st.size(), 0) {}
  // Kernel states reachable from `seed` through SPLIT/EPS (always), BOL (if
  // bol) and EOL (if eol).  Kernel = CHR, MATCH, and EOL when !eol.
  void run(const std::vector<int>& seed, bool bol, bool eol, std::vector<int>* out) {
    ++gen_;
    out->clear();
    stack_.assign(seed.begin(), seed.end());
    while (!stack_.empty()) {
      int s = stack_.back();
      stack_.pop_back();
      if (s < 0 || mark_[s] == gen_) continue;
      mark_[s] = gen_;
      const NState& x = n_.st[s];
      switch (x.type) {
        case NState::CHR:
        case NState::MATCH:
          out->push_back(s);
          break;
        case NState::SPLIT:
          stack_.push_back(x.out2);
          stack_.push_back(x.out1);
          break;
        case NState::EPS:
          stack_.push_back(x.out1);
          break;
        case NState::BOL:
          if (bol) stack_.push_back(x.out1);
          break;
        case NState::EOL:
          if (eol) stack_.push_back(x.out1);
          else out->push_back(s);
          break;
        default:  // WORDB / LOOK: build_ctx's closure
          break;
      }
    }
    std::sort(out->begin(), out->end());
  }

 private:
  const Nfa& n_;
  std::vector<uint32_t> mark_;
  uint32_t gen_ = 0;
  std::vector<int> stack_;
};

}  // namespace

Status parse_ecma(const std::string& pat, Ast* out, std::string* err) {
  try {
    Parser p(pat);
    *out = p.run();
    return Status::Ok;
  } catch (const ParseError& e) {
    if (err) *err = e.msg;
    return e.st;
  }
}

Ast literal_ast(const std::string& lit) {
  Ast a;
  Node cat;
  cat.kind = Node::Cat;
  for (unsigned char c : lit) {
    Node n;
    n.kind = Node::Set;
    n.set.set(c);
    a.nodes.push_back(n);
    cat.kids.push_back(static_cast<int>(a.nodes.size()) - 1);
  }
  a.nodes.push_back(cat);
  a.root = static_cast<int>(a.nodes.size()) - 1;
  return a;
}

void make_search_prefix(Ast* a) {
  Node any;
  any.kind = Node::Set;
  any.set.set();
  a->nodes.push_back(any);
  Node star;
  star.kind = Node::Rep;
  star.kids = {static_cast<int>(a->nodes.size()) - 1};
  star.min = 0;
  star.max = -1;
  a->nodes.push_back(star);
  Node cat;
  cat.kind = Node::Cat;
  cat.kids = {static_cast<int>(a->nodes.size()) - 1, a->root};
  a->nodes.push_back(cat);
  a->root = static_cast<int>(a->nodes.size()) - 1;
}

namespace {

// Moore minimisation (initial partition by end set and mid set) and BFS
// renumbering of an unminimised DFA (n0 states x ncls classes, state 0 dead).
Status finish_dfa(size_t n0, int ncls, const int* cls, const std::vector<uint32_t>& next,
                  const std::vector<uint32_t>& endset, const std::vector<uint32_t>& midset, int start_id,
                  std::vector<std::vector<uint32_t>>&& sets, const DfaLimits& lim, bool with_mid, Dfa* out) {
  // Moore minimisation: initial partition by end set (and mid set).
  std::vector<uint32_t> blk(n0);
  size_t nblk = 0;
  {
    // dense renumber
    std::unordered_map<uint64_t, uint32_t> rn;
    for (size_t s = 0; s < n0; ++s) {
      const uint64_t key = static_cast<uint64_t>(midset[s]) << 32 | endset[s];
      auto it = rn.find(key);
      if (it == rn.end()) it = rn.emplace(key, static_cast<uint32_t>(rn.size())).first;
      blk[s] = it->second;
    }
    nblk = rn.size();
  }
  std::vector<uint32_t> sig(static_cast<size_t>(ncls) + 1);
  for (;;) {
    std::unordered_map<std::vector<uint32_t>, uint32_t, U32VecHash> sigs;
    sigs.reserve(nblk * 2 + 16);
    std::vector<uint32_t> nb(n0);
    for (size_t s = 0; s < n0; ++s) {
      sig[0] = blk[s];
      for (int c = 0; c < ncls; ++c) sig[c + 1] = blk[next[s * ncls + c]];
      auto it = sigs.find(sig);
      if (it == sigs.end()) it = sigs.emplace(sig, static_cast<uint32_t>(sigs.size())).first;
      nb[s] = it->second;
    }
    size_t nn = sigs.size();
    blk.swap(nb);
    if (nn == nblk) break;
    nblk = nn;
  }

  // BFS renumbering over blocks; dead block -> 0.
  std::vector<int64_t> newid(nblk, -1);
  std::vector<size_t> rep(nblk, SIZE_MAX);
  for (size_t s = 0; s < n0; ++s)
    if (rep[blk[s]] == SIZE_MAX) rep[blk[s]] = s;
  newid[blk[0]] = 0;
  std::vector<uint32_t> order;  // block ids in new-id order
  order.push_back(blk[0]);
  size_t head = 0;
  if (newid[blk[start_id]] < 0) {
    newid[blk[start_id]] = static_cast<int64_t>(order.size());
    order.push_back(blk[start_id]);
  }
  head = 1;
  while (head < order.size()) {
    uint32_t b = order[head++];
    size_t s = rep[b];
    for (int c = 0; c < ncls; ++c) {
      uint32_t tb = blk[next[s * ncls + c]];
      if (newid[tb] < 0) {
        newid[tb] = static_cast<int64_t>(order.size());
        order.push_back(tb);
      }
    }
  }
  const size_t nst = order.size();
  if (nst > lim.max_states) return Status::TooBig;
  if (static_cast<uint64_t>(nst) * (ncls + 1) * 4 > lim.max_table_bytes) return Status::TooBig;

  Dfa d;
  d.ncls = ncls;
  for (int b = 0; b < 256; ++b) d.cmap[b] = static_cast<uint8_t>(cls[b]);
  d.nstates = static_cast<int>(nst);
  d.start = static_cast<int>(newid[blk[start_id]]);
  d.next.assign(nst * ncls, 0);
  d.endset.assign(nst, 0);
  if (with_mid) d.midset.assign(nst, 0);
  for (size_t i = 0; i < nst; ++i) {
    size_t s = rep[order[i]];
    for (int c = 0; c < ncls; ++c)
      d.next[i * ncls + c] = static_cast<uint32_t>(newid[blk[next[s * ncls + c]]]);
    d.endset[i] = endset[s];
    if (with_mid) d.midset[i] = midset[s];
  }
  d.sets = std::move(sets);
  *out = std::move(d);
  return Status::Ok;
}

}  // namespace

namespace {

ByteSet word_set() { return mask_set(std::ctype_base::alnum, true); }  // _M_is_word: lookup_classname("w")

int copy_subtree(const Ast& a, int node, Ast* dst) {
  Node m = a.nodes[node];
  for (int& k : m.kids) k = copy_subtree(a, k, dst);
  dst->nodes.push_back(std::move(m));
  return static_cast<int>(dst->nodes.size()) - 1;
}

// ---------------------------------------------- context construction ----
// Patterns with word boundaries or look-ahead.  A DFA state is a set of
// threads (NFA state + look-ahead obligations) plus the context the pending
// assertions need: whether this is the subject's start ('^') and whether the
// previous byte was a word character ('\b').  Assertions are resolved with
// the byte being consumed as their right context (or the end of the subject);
// a look-ahead at position i starts an obligation: its automaton (LookDfa)
// runs from i and must accept at the end of the subject ((?=X)) or must not
// ((?!X)); obligations whose automaton reaches the dead state or a universal
// state are decided early.
using Th = std::vector<int>;  // [nfa state, look id, look state, look id, look state, ...] (sorted pairs)

struct CtxIn {
  bool bol, eol, prev;
  int next;  // -1 unknown (assertions needing it stay pending), 0 non-word / end, 1 word
};

void th_add_obl(Th* t, int la, int q) {
  for (size_t k = 1; k < t->size(); k += 2)
    if ((*t)[k] == la && (*t)[k + 1] == q) return;
  t->push_back(la);
  t->push_back(q);
  std::vector<std::pair<int, int>> o;
  for (size_t k = 1; k < t->size(); k += 2) o.push_back({(*t)[k], (*t)[k + 1]});
  std::sort(o.begin(), o.end());
  for (size_t k = 0; k < o.size(); ++k) {
    (*t)[1 + 2 * k] = o[k].first;
    (*t)[2 + 2 * k] = o[k].second;
  }
}

struct ThHash {
  size_t operator()(const Th& v) const {
    uint64_t h = 1469598103934665603ull;
    for (int x : v) {
      h ^= static_cast<uint32_t>(x);
      h *= 1099511628211ull;
    }
    return static_cast<size_t>(h ^ (h >> 29));
  }
};

class CtxClosure {
 public:
  explicit CtxClosure(const Nfa& n) : n_(n) {}
  void run(const std::vector<Th>& seeds, const CtxIn& c, std::vector<Th>* out) {
    out->clear();
    seen_.clear();
    stack_ = seeds;
    while (!stack_.empty()) {
      Th t = std::move(stack_.back());
      stack_.pop_back();
      if (!seen_.insert(t).second) continue;
      const NState& x = n_.st[t[0]];
      auto go = [&](int to) {
        Th u = t;
        u[0] = to;
        stack_.push_back(std::move(u));
      };
      switch (x.type) {
        case NState::CHR:
        case NState::MATCH:
          out->push_back(t);
          break;
        case NState::SPLIT:
          go(x.out2);
          go(x.out1);
          break;
        case NState::EPS:
          go(x.out1);
          break;
        case NState::BOL:
          if (c.bol) go(x.out1);
          break;
        case NState::EOL:
          if (c.eol) go(x.out1);
          else out->push_back(t);
          break;
        case NState::WORDB:
          if (c.next < 0) out->push_back(t);
          else if ((c.prev != (c.next == 1)) == (x.pat == 0)) go(x.out1);
          break;
        case NState::LOOK: {
          const LookDfa& l = n_.looks[x.cs];
          const uint32_t q = static_cast<uint32_t>(l.dfa.start);
          if (c.eol) {
            if ((l.dfa.endset[q] != 0) != l.neg) go(x.out1);
          } else if (q == 0) {
            if (l.neg) go(x.out1);
          } else if (l.universal[q]) {
            if (!l.neg) go(x.out1);
          } else {
            Th u = t;
            u[0] = x.out1;
            th_add_obl(&u, x.cs, static_cast<int>(q));
            stack_.push_back(std::move(u));
          }
          break;
        }
      }
    }
    std::sort(out->begin(), out->end());
    out->erase(std::unique(out->begin(), out->end()), out->end());
  }
  // Consume byte b in every obligation of t; false if the thread dies.
  bool advance(Th* t, int b) const {
    Th u{(*t)[0]};
    for (size_t k = 1; k < t->size(); k += 2) {
      const LookDfa& l = n_.looks[(*t)[k]];
      const uint32_t q = l.dfa.next[static_cast<size_t>((*t)[k + 1]) * l.dfa.ncls + l.dfa.cmap[b]];
      if (q == 0) {
        if (!l.neg) return false;
        continue;  // (?!X): X can no longer match
      }
      if (l.universal[q]) {
        if (l.neg) return false;
        continue;  // (?=X): X has matched
      }
      th_add_obl(&u, (*t)[k], static_cast<int>(q));
    }
    *t = std::move(u);
    return true;
  }
  // At the end of the subject: do t's obligations hold?
  bool obligations_hold(const Th& t) const {
    for (size_t k = 1; k < t.size(); k += 2) {
      const LookDfa& l = n_.looks[t[k]];
      if ((l.dfa.endset[t[k + 1]] != 0) == l.neg) return false;
    }
    return true;
  }

 private:
  const Nfa& n_;
  std::unordered_set<Th, ThHash> seen_;
  std::vector<Th> stack_;
};

Status build_ctx(const Nfa& nfa, const std::vector<int>& starts, int ncls, const int* cls, const DfaLimits& lim,
                 Dfa* out) {
  std::vector<int> rep(ncls, -1);
  for (int b = 0; b < 256; ++b)
    if (rep[cls[b]] < 0) rep[cls[b]] = b;
  const ByteSet W = word_set();
  bool any_wb = false;
  for (const NState& x : nfa.st) any_wb |= x.type == NState::WORDB;
  struct St {
    std::vector<Th> th;
    bool start, prev;
  };
  std::vector<St> states(1);  // 0 = dead
  std::unordered_map<Th, int, ThHash> ids;
  std::vector<uint32_t> next(static_cast<size_t>(ncls), 0);
  auto intern = [&](std::vector<Th>&& th, bool start, bool prev) -> int {
    if (th.empty()) return 0;
    Th key{(start ? 1 : 0) | (prev ? 2 : 0)};
    for (const Th& t : th) {
      key.push_back(static_cast<int>(t.size()));
      key.insert(key.end(), t.begin(), t.end());
    }
    auto it = ids.find(key);
    if (it != ids.end()) return it->second;
    const int id = static_cast<int>(states.size());
    if (static_cast<size_t>(id) >= lim.max_states) throw ParseError{Status::TooBig, "context DFA too large"};
    ids.emplace(std::move(key), id);
    states.push_back(St{std::move(th), start, prev});
    next.resize(next.size() + ncls, 0);
    return id;
  };
  CtxClosure clo(nfa);
  std::vector<Th> seeds, k1, k2;
  int start_id;
  try {
    for (int s0 : starts) seeds.push_back(Th{s0});
    clo.run(seeds, CtxIn{true, false, false, -1}, &k1);
    start_id = intern(std::move(k1), true, false);
    for (size_t d = 1; d < states.size(); ++d) {
      for (int c = 0; c < ncls; ++c) {
        const int b = rep[c];
        const bool bw = W.test(b);
        clo.run(states[d].th, CtxIn{states[d].start, false, states[d].prev, bw ? 1 : 0}, &k1);
        seeds.clear();
        for (const Th& t : k1) {
          const NState& x = nfa.st[t[0]];
          if (x.type != NState::CHR || !nfa.sets[x.cs].test(b)) continue;
          Th u = t;
          u[0] = x.out1;
          if (clo.advance(&u, b)) seeds.push_back(std::move(u));
        }
        clo.run(seeds, CtxIn{false, false, bw, -1}, &k2);
        const int to = intern(std::move(k2), false, any_wb && bw);
        next[d * ncls + c] = static_cast<uint32_t>(to);
      }
    }
  } catch (const ParseError& e) {
    return e.st;
  }
  if (start_id == 0) {  // nothing can match: a one-state dead automaton with a start row
    start_id = static_cast<int>(states.size());
    states.push_back(St{{}, true, false});
    next.resize(next.size() + ncls, 0);
  }
  const size_t n0 = states.size();
  std::vector<std::vector<uint32_t>> sets{{}};
  std::unordered_map<std::vector<uint32_t>, uint32_t, U32VecHash> set_ids{{std::vector<uint32_t>{}, 0}};
  std::vector<uint32_t> endset(n0, 0), midset(n0, 0);
  for (size_t d = 1; d < n0; ++d) {
    clo.run(states[d].th, CtxIn{states[d].start, true, states[d].prev, 0}, &k1);
    std::vector<uint32_t> pats;
    for (const Th& t : k1)
      if (nfa.st[t[0]].type == NState::MATCH && clo.obligations_hold(t))
        pats.push_back(static_cast<uint32_t>(nfa.st[t[0]].pat));
    std::sort(pats.begin(), pats.end());
    pats.erase(std::unique(pats.begin(), pats.end()), pats.end());
    auto it = set_ids.find(pats);
    if (it == set_ids.end()) {
      it = set_ids.emplace(pats, static_cast<uint32_t>(sets.size())).first;
      sets.push_back(pats);
    }
    endset[d] = it->second;
  }
  states.clear();
  return finish_dfa(n0, ncls, cls, next, endset, midset, start_id, std::move(sets), lim, false, out);
}

}  // namespace

int Nfa::look_dfa(const Ast& a, int node, bool neg) {
  // X [\x00-\xff]*, determinised as a subject of its own (see LookDfa)
  Ast x;
  const int xr = copy_subtree(a, node, &x);
  Node any;
  any.kind = Node::Set;
  any.set.set();
  x.nodes.push_back(any);
  Node star;
  star.kind = Node::Rep;
  star.min = 0;
  star.max = -1;
  star.kids = {static_cast<int>(x.nodes.size()) - 1};
  x.nodes.push_back(star);
  Node cat;
  cat.kind = Node::Cat;
  cat.kids = {xr, static_cast<int>(x.nodes.size()) - 1};
  x.nodes.push_back(cat);
  x.root = static_cast<int>(x.nodes.size()) - 1;
  LookDfa l;
  l.neg = neg;
  const Status st = build_dfa({&x}, lim, &l.dfa);
  if (st != Status::Ok) throw ParseError{st, "look-ahead automaton"};
  const Dfa& d = l.dfa;
  l.universal.assign(d.nstates, 0);
  for (int q = 0; q < d.nstates; ++q) l.universal[q] = d.endset[q] != 0;
  for (bool changed = true; changed;) {
    changed = false;
    for (int q = 0; q < d.nstates; ++q) {
      if (!l.universal[q]) continue;
      for (int c = 0; c < d.ncls; ++c)
        if (!l.universal[d.next[static_cast<size_t>(q) * d.ncls + c]]) {
          l.universal[q] = 0;
          changed = true;
          break;
        }
    }
  }
  looks.push_back(std::move(l));
  return static_cast<int>(looks.size()) - 1;
}

bool has_node(const Ast& a, Node::Kind k) {
  for (const Node& n : a.nodes)
    if (n.kind == k) return true;
  return false;
}

namespace {
constexpr size_t kLowerBudget = 1u << 14;  // nodes of a lowered AST before references stop being copied

// in_ref: copying a group's pattern for a back-reference -- the reference
// compares text only, so the group's assertions (checked where the group
// matched) do not apply at the reference's position and are dropped.
int lower_node(const Ast& a, int node, Ast* dst, const std::vector<int>& gnode, bool* exact, bool drop_look,
               bool in_ref = false) {
  const Node& n = a.nodes[node];
  auto empty = [&]() {
    Node e;
    e.kind = Node::Empty;
    dst->nodes.push_back(e);
    return static_cast<int>(dst->nodes.size()) - 1;
  };
  switch (n.kind) {
    case Node::Group:
      return lower_node(a, n.kids[0], dst, gnode, exact, drop_look, in_ref);
    case Node::Backref: {
      // \k matches the text group k captured: a string of group k's language.
      // Chained references ((a)(\1\1)(\2\2)...) double the copy per level, so
      // past kLowerBudget nodes the copy is replaced by [\x00-\xff]* -- still a
      // superset, and the slow path decides the pattern exactly either way.
      *exact = false;
      const size_t mark = dst->nodes.size();
      if (mark < kLowerBudget) {
        const int r = lower_node(a, a.nodes[gnode[n.min]].kids[0], dst, gnode, exact, drop_look, true);
        if (dst->nodes.size() <= kLowerBudget) return r;
        dst->nodes.resize(mark);
      }
      Node any;
      any.kind = Node::Set;
      any.set.set();
      dst->nodes.push_back(any);
      Node star;
      star.kind = Node::Rep;
      star.kids = {static_cast<int>(dst->nodes.size()) - 1};
      star.min = 0;
      star.max = -1;
      dst->nodes.push_back(star);
      return static_cast<int>(dst->nodes.size()) - 1;
    }
    case Node::Look:
      if (drop_look || in_ref) {
        *exact = false;
        return empty();
      }
      break;
    case Node::WordB:
    case Node::Bol:
    case Node::Eol:
      if (in_ref) return empty();
      break;
    default:
      break;
  }
  Node m = n;
  for (int& k : m.kids) k = lower_node(a, k, dst, gnode, exact, drop_look, in_ref);
  dst->nodes.push_back(std::move(m));
  return static_cast<int>(dst->nodes.size()) - 1;
}

Ast lower(const Ast& a, bool* exact, bool drop_look) {
  std::vector<int> gnode;
  for (size_t i = 0; i < a.nodes.size(); ++i)
    if (a.nodes[i].kind == Node::Group) {
      if (gnode.size() <= static_cast<size_t>(a.nodes[i].min)) gnode.resize(a.nodes[i].min + 1, -1);
      gnode[a.nodes[i].min] = static_cast<int>(i);
    }
  Ast out;
  *exact = true;
  out.root = lower_node(a, a.root, &out, gnode, exact, drop_look);
  return out;
}
}  // namespace

Ast lower_for_dfa(const Ast& a, bool* exact) { return lower(a, exact, false); }

Ast drop_lookahead(const Ast& a) {
  bool exact;
  return lower(a, &exact, true);
}

Status build_dfa(const std::vector<const Ast*>& patterns, const DfaLimits& lim, Dfa* out, bool with_mid) {
  Nfa nfa;
  nfa.lim = lim;
  std::vector<int> starts;
  try {
    for (size_t p = 0; p < patterns.size(); ++p) {
      NState m;
      m.type = NState::MATCH;
      m.pat = static_cast<int>(p);
      int acc = nfa.add(m);
      starts.push_back(nfa.compile(*patterns[p], patterns[p]->root, acc));
    }
  } catch (const ParseError& e) {
    return e.st;
  }

  // Byte classes: refine the partition of 0..255 by every CHR set (and, for
  // the context construction, by \w and every look-ahead automaton's classes).
  std::vector<ByteSet> parts = nfa.sets;
  if (nfa.ctx) {
    parts.push_back(word_set());
    for (const LookDfa& l : nfa.looks)
      for (int c = 0; c < l.dfa.ncls; ++c) {
        ByteSet b;
        for (int x = 0; x < 256; ++x)
          if (l.dfa.cmap[x] == c) b.set(x);
        parts.push_back(b);
      }
  }
  int cls[256] = {0};
  int ncls = 1;
  for (const ByteSet& s : parts) {
    std::map<std::pair<int, int>, int> remap;
    int n2 = 0;
    int tmp[256];
    for (int b = 0; b < 256; ++b) {
      auto key = std::make_pair(cls[b], s.test(b) ? 1 : 0);
      auto it = remap.find(key);
      if (it == remap.end()) it = remap.emplace(key, n2++).first;
      tmp[b] = it->second;
    }
    std::memcpy(cls, tmp, sizeof cls);
    ncls = n2;
  }
  // Renumber classes by first byte occurrence for stable output.
  {
    int rn[256];
    std::fill(rn, rn + 256, -1);
    int k = 0;
    for (int b = 0; b < 256; ++b)
      if (rn[cls[b]] < 0) rn[cls[b]] = k++;
    for (int b = 0; b < 256; ++b) cls[b] = rn[cls[b]];
    ncls = k;
  }
  if (nfa.ctx) {
    if (with_mid) return Status::Unsupported;  // (search automata carry no assertions)
    return build_ctx(nfa, starts, ncls, cls, lim, out);
  }
  std::vector<std::vector<int>> set_classes(nfa.sets.size());
  for (size_t i = 0; i < nfa.sets.size(); ++i) {
    std::vector<char> seen(ncls, 0);
    for (int b = 0; b < 256; ++b)
      if (nfa.sets[i].test(b) && !seen[cls[b]]) {
        seen[cls[b]] = 1;
        set_classes[i].push_back(cls[b]);
      }
  }

  // Subset construction.  Key = kernel state list; the start state carries a
  // leading -1 marker because only it may pass '^' (and, at end, '^' after '$').
  Closure clo(nfa);
  std::unordered_map<std::vector<int>, int, VecHash> ids;
  std::vector<std::vector<int>> kern;
  std::vector<uint32_t> next;  // unminimised, states * ncls
  kern.push_back({});          // dead
  ids.emplace(std::vector<int>{}, 0);
  next.resize(static_cast<size_t>(ncls), 0);

  std::vector<int> tmpk;
  clo.run(starts, /*bol=*/true, /*eol=*/false, &tmpk);
  int start_id;
  {
    std::vector<int> key;
    key.push_back(-1);
    key.insert(key.end(), tmpk.begin(), tmpk.end());
    start_id = static_cast<int>(kern.size());
    ids.emplace(key, start_id);
    kern.push_back(std::move(key));
    next.resize(next.size() + ncls, 0);
  }
  std::vector<std::vector<int>> bucket(ncls);
  std::vector<int> used;
  for (size_t d = 1; d < kern.size(); ++d) {
    for (int c : used) bucket[c].clear();
    used.clear();
    for (int s : kern[d]) {
      if (s < 0) continue;
      const NState& x = nfa.st[s];
      if (x.type != NState::CHR) continue;
      for (int c : set_classes[x.cs]) {
        if (bucket[c].empty()) used.push_back(c);
        bucket[c].push_back(x.out1);
      }
    }
    for (int c : used) {
      clo.run(bucket[c], false, false, &tmpk);
      if (tmpk.empty()) continue;
      auto it = ids.find(tmpk);
      int id;
      if (it == ids.end()) {
        id = static_cast<int>(kern.size());
        if (static_cast<size_t>(id) >= lim.max_states) return Status::TooBig;
        ids.emplace(tmpk, id);
        kern.push_back(tmpk);
        next.resize(next.size() + ncls, 0);
      } else {
        id = it->second;
      }
      next[d * ncls + c] = static_cast<uint32_t>(id);
    }
  }
  const size_t n0 = kern.size();

  // End column: patterns matched when the input ends in this state.
  std::vector<std::vector<uint32_t>> sets;
  std::unordered_map<std::vector<uint32_t>, uint32_t, U32VecHash> set_ids;
  sets.push_back({});
  set_ids.emplace(std::vector<uint32_t>{}, 0);
  std::vector<uint32_t> endset(n0, 0), midset(n0, 0);
  std::vector<int> seed;
  auto set_of = [&](bool is_start, bool eol) -> uint32_t {
    clo.run(seed, is_start, eol, &tmpk);
    std::vector<uint32_t> pats;
    for (int s : tmpk)
      if (nfa.st[s].type == NState::MATCH) pats.push_back(static_cast<uint32_t>(nfa.st[s].pat));
    std::sort(pats.begin(), pats.end());
    pats.erase(std::unique(pats.begin(), pats.end()), pats.end());
    auto it = set_ids.find(pats);
    if (it != set_ids.end()) return it->second;
    const uint32_t sid = static_cast<uint32_t>(sets.size());
    set_ids.emplace(pats, sid);
    sets.push_back(pats);
    return sid;
  };
  for (size_t d = 1; d < n0; ++d) {
    bool is_start = !kern[d].empty() && kern[d][0] == -1;
    seed.clear();
    for (int s : kern[d])
      if (s >= 0) seed.push_back(s);
    endset[d] = set_of(is_start, true);
    if (with_mid) midset[d] = set_of(is_start, false);
  }
  kern.clear();
  kern.shrink_to_fit();
  return finish_dfa(n0, ncls, cls, next, endset, midset, start_id, std::move(sets), lim, with_mid, out);
}


// Back-references whose capture is forced (see regex_ecma.h DcapForm).
bool analyze_dcap(const Ast& a, DcapForm* out) {
  if (a.root < 0) return false;
  // exactly one back-reference, to a group that occurs once
  int nref = 0, ref = -1;
  for (const Node& n : a.nodes)
    if (n.kind == Node::Backref) {
      ++nref;
      ref = n.min;
    }
  if (nref != 1) return false;
  // the top-level concatenation, Cat nodes flattened
  std::vector<int> items;
  std::vector<int> stack{a.root};
  std::function<void(int)> flat = [&](int x) {
    if (a.nodes[x].kind == Node::Cat) {
      for (int k : a.nodes[x].kids) flat(k);
    } else {
      items.push_back(x);
    }
  };
  flat(a.root);
  int ig = -1, ib = -1;
  for (size_t i = 0; i < items.size(); ++i) {
    const Node& n = a.nodes[items[i]];
    if (n.kind == Node::Group && n.min == ref) ig = static_cast<int>(i);
    if (n.kind == Node::Backref) ib = static_cast<int>(i);
  }
  if (ig < 0 || ib < 0 || ib < ig + 2) return false;  // L2 non-empty: group, >= 1 literal, \k
  auto single = [&](int x, uint8_t* b) {
    const Node& n = a.nodes[x];
    if (n.kind != Node::Set || n.set.count() != 1) return false;
    for (int c = 0; c < 256; ++c)
      if (n.set.test(c)) *b = static_cast<uint8_t>(c);
    return true;
  };
  DcapForm f;
  for (int i = 0; i < ig; ++i) {  // P1: an optional leading '^', then literal bytes
    if (i == 0 && a.nodes[items[0]].kind == Node::Bol) continue;
    uint8_t b;
    if (!single(items[i], &b)) return false;
    f.p1.push_back(static_cast<char>(b));
  }
  // G: C, C*, C+, C{n}, C{n,}, C{n,m} of one byte class C
  const Node& g = a.nodes[items[ig]];
  if (g.kids.size() != 1) return false;
  const Node& gk = a.nodes[g.kids[0]];
  if (gk.kind == Node::Set) {
    f.cls = gk.set;
    f.min = f.max = 1;
  } else if (gk.kind == Node::Rep && gk.kids.size() == 1 && a.nodes[gk.kids[0]].kind == Node::Set) {
    f.cls = a.nodes[gk.kids[0]].set;
    f.min = gk.min;
    f.max = gk.max;
  } else {
    return false;
  }
  if (f.cls.none()) return false;
  for (int i = ig + 1; i < ib; ++i) {  // L2: literal bytes, the first outside C
    uint8_t b;
    if (!single(items[i], &b)) return false;
    if (i == ig + 1 && f.cls.test(b)) return false;
    f.l2.push_back(static_cast<char>(b));
  }
  // R: the rest, regular and context-free at its start (no ^, \b, \B,
  // look-ahead, groups referenced: the pattern's only reference is \k)
  Ast r;
  std::vector<int> rk;
  for (size_t i = ib + 1; i < items.size(); ++i) {
    const int x = items[i];
    std::vector<int> todo{x};
    while (!todo.empty()) {
      const Node& n = a.nodes[todo.back()];
      todo.pop_back();
      if (n.kind == Node::Bol || n.kind == Node::WordB || n.kind == Node::Look || n.kind == Node::Backref) return false;
      for (int k : n.kids) todo.push_back(k);
    }
    rk.push_back(copy_subtree(a, x, &r));
  }
  f.r_empty = rk.empty();
  if (!f.r_empty) {
    Node cat;
    cat.kind = Node::Cat;
    cat.kids = rk;
    r.nodes.push_back(cat);
    r.root = static_cast<int>(r.nodes.size()) - 1;
    bool exact = true;
    f.r = lower_for_dfa(r, &exact);
    if (!exact) return false;
  }
  *out = std::move(f);
  return true;
}

}  // namespace re
}  // namespace l7m
