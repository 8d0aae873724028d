// regex_re2.cc — parser for the L7M_DIALECT_RE2_SEARCH dialect: Go
// `regexp.MustCompile(p).MatchString(s)` (RE2 syntax, syntax.Perl flags:
// one-line ^/$, `.` excludes only '\n', negated classes include '\n'),
// evaluated byte-wise.  Exact for ASCII subjects; a subject byte >= 0x80 is
// one "character" here where Go would decode a UTF-8 rune (documented
// deviation).
//
// Accepted: literals (ASCII, or a whole UTF-8 rune as one atom), `.`, `^ $
// \A \z`, escapes \a \f \t \n \r \v, octal \0.. \1nn, \xHH \x{H..}, escaped
// punctuation, \Q...\E, Perl classes \d \D \s \S \w \W, bracket classes with
// ranges, Perl and [:posix:] classes, groups ( ) (?: ) (?P<n> ) (?<n> ),
// alternation, * + ? {n} {n,} {n,m} with the non-greedy `?`.  Rejected the
// way regexp.Compile rejects them (Status::Syntax -> L7M_EINVAL_REGEX):
// missing/unexpected parens, bad escapes, nested repetition (`a**`),
// repetition of nothing, repeat counts > 1000, reversed ranges, invalid
// UTF-8.  Valid RE2 outside the byte-exact subset (flag groups such as
// (?i), \b \B, \pN / \p{..}, non-ASCII inside classes) -> Unsupported.
#include <string>
#include <vector>

#include "regex_ecma.h"

namespace l7m {
namespace re {
namespace {

struct Re2Error {
  Status st;
  std::string msg;
};

class Re2Parser {
 public:
  explicit Re2Parser(const std::string& p) : p_(p) {}

  Ast run() {
    ast_.root = alternation(0);
    if (i_ < p_.size()) fail(Status::Syntax, "unexpected )");
    return std::move(ast_);
  }

 private:
  [[noreturn]] void fail(Status st, const std::string& m) { throw Re2Error{st, m}; }
  bool at_end() const { return i_ >= p_.size(); }
  unsigned char cur() const { return static_cast<unsigned char>(p_[i_]); }

  int add(Node n) {
    ast_.nodes.push_back(std::move(n));
    return static_cast<int>(ast_.nodes.size()) - 1;
  }
  int mk(Node::Kind k) {
    Node n;
    n.kind = k;
    return add(std::move(n));
  }
  int mk_set(const ByteSet& s) {
    Node n;
    n.kind = Node::Set;
    n.set = s;
    return add(std::move(n));
  }
  int mk_cat(std::vector<int> kids) {
    if (kids.empty()) return mk(Node::Empty);
    if (kids.size() == 1) return kids[0];
    Node n;
    n.kind = Node::Cat;
    n.kids = std::move(kids);
    return add(std::move(n));
  }
  int mk_byte(unsigned b) {
    ByteSet s;
    s.set(b);
    return mk_set(s);
  }
  // A code point as its UTF-8 bytes (one atom).
  int mk_rune(uint32_t r) {
    if (r < 0x80) return mk_byte(r);
    std::vector<int> bytes;
    if (r < 0x800) {
      bytes = {mk_byte(0xc0 | (r >> 6)), mk_byte(0x80 | (r & 0x3f))};
    } else if (r < 0x10000) {
      bytes = {mk_byte(0xe0 | (r >> 12)), mk_byte(0x80 | ((r >> 6) & 0x3f)), mk_byte(0x80 | (r & 0x3f))};
    } else {
      bytes = {mk_byte(0xf0 | (r >> 18)), mk_byte(0x80 | ((r >> 12) & 0x3f)), mk_byte(0x80 | ((r >> 6) & 0x3f)),
               mk_byte(0x80 | (r & 0x3f))};
    }
    return mk_cat(std::move(bytes));
  }

  // Decode one UTF-8 rune of the pattern at i_ (Go rejects invalid UTF-8).
  uint32_t next_rune() {
    const unsigned char c = cur();
    if (c < 0x80) {
      ++i_;
      return c;
    }
    int n = c >= 0xf0 && c <= 0xf4 ? 4 : c >= 0xe0 ? 3 : c >= 0xc2 && c <= 0xdf ? 2 : 0;
    if (!n || i_ + n > p_.size()) fail(Status::Syntax, "invalid UTF-8");
    uint32_t r = c & (0xff >> (n + 1));
    for (int k = 1; k < n; ++k) {
      const unsigned char b = static_cast<unsigned char>(p_[i_ + k]);
      if ((b & 0xc0) != 0x80) fail(Status::Syntax, "invalid UTF-8");
      r = (r << 6) | (b & 0x3f);
    }
    if ((n == 3 && (r < 0x800 || (r >= 0xd800 && r <= 0xdfff))) || (n == 4 && (r < 0x10000 || r > 0x10ffff)))
      fail(Status::Syntax, "invalid UTF-8");
    i_ += n;
    return r;
  }

  static ByteSet range(unsigned lo, unsigned hi) {
    ByteSet s;
    for (unsigned c = lo; c <= hi; ++c) s.set(c);
    return s;
  }
  // Perl classes (ASCII, regexp/syntax perl_groups.go).
  static bool perl_class(unsigned char c, ByteSet* out) {
    ByteSet s;
    switch (c | 0x20) {
      case 'd': s = range('0', '9'); break;
      case 's': s.set('\t'); s.set('\n'); s.set('\f'); s.set('\r'); s.set(' '); break;
      case 'w': s = range('0', '9') | range('A', 'Z') | range('a', 'z'); s.set('_'); break;
      default: return false;
    }
    if (c >= 'A' && c <= 'Z') s.flip();
    if (out) *out = s;
    return true;
  }
  // POSIX classes inside brackets (regexp/syntax posix_groups.go).
  static bool posix_class(const std::string& name, ByteSet* out) {
    ByteSet s;
    if (name == "alnum") s = range('0', '9') | range('A', 'Z') | range('a', 'z');
    else if (name == "alpha") s = range('A', 'Z') | range('a', 'z');
    else if (name == "ascii") s = range(0, 0x7f);
    else if (name == "blank") { s.set('\t'); s.set(' '); }
    else if (name == "cntrl") { s = range(0, 0x1f); s.set(0x7f); }
    else if (name == "digit") s = range('0', '9');
    else if (name == "graph") s = range('!', '~');
    else if (name == "lower") s = range('a', 'z');
    else if (name == "print") s = range(' ', '~');
    else if (name == "punct") s = range('!', '/') | range(':', '@') | range('[', '`') | range('{', '~');
    else if (name == "space") { s = range('\t', '\r'); s.set(' '); }
    else if (name == "upper") s = range('A', 'Z');
    else if (name == "word") { s = range('0', '9') | range('A', 'Z') | range('a', 'z'); s.set('_'); }
    else if (name == "xdigit") s = range('0', '9') | range('A', 'F') | range('a', 'f');
    else return false;
    *out = s;
    return true;
  }

  static bool is_octal(unsigned char c) { return c >= '0' && c <= '7'; }
  static int hexval(unsigned char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }

  // Escape after '\' yielding one code point (parseEscape); classes and
  // assertions are handled by the callers.
  uint32_t escape_rune() {
    if (at_end()) fail(Status::Syntax, "trailing backslash");
    const unsigned char c = cur();
    ++i_;
    switch (c) {
      case 'a': return 7;
      case 'f': return '\f';
      case 't': return '\t';
      case 'n': return '\n';
      case 'r': return '\r';
      case 'v': return '\v';
      case '1': case '2': case '3': case '4': case '5': case '6': case '7':
        if (at_end() || !is_octal(cur())) fail(Status::Syntax, "invalid escape (back-reference)");
        [[fallthrough]];
      case '0': {
        uint32_t r = c - '0';
        for (int k = 0; k < 2 && !at_end() && is_octal(cur()); ++k) r = r * 8 + (p_[i_++] - '0');
        return r;
      }
      case 'x': {
        if (at_end()) fail(Status::Syntax, "invalid escape");
        if (cur() == '{') {
          ++i_;
          uint32_t r = 0;
          int nd = 0;
          while (!at_end() && cur() != '}') {
            const int h = hexval(cur());
            if (h < 0) fail(Status::Syntax, "invalid escape");
            r = r * 16 + static_cast<uint32_t>(h);
            if (r > 0x10ffff) fail(Status::Syntax, "invalid escape");
            ++i_;
            ++nd;
          }
          if (at_end() || !nd) fail(Status::Syntax, "invalid escape");
          ++i_;
          return r;
        }
        if (i_ + 2 > p_.size() || hexval(p_[i_]) < 0 || hexval(p_[i_ + 1]) < 0) fail(Status::Syntax, "invalid escape");
        const uint32_t r = static_cast<uint32_t>(hexval(p_[i_]) * 16 + hexval(p_[i_ + 1]));
        i_ += 2;
        return r;
      }
      default:
        if (c < 0x80 && !((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')))
          return c;  // escaped punctuation
        fail(Status::Syntax, std::string("invalid escape \\") + static_cast<char>(c));
    }
  }

  int bracket() {  // after '['
    bool neg = false;
    if (!at_end() && cur() == '^') {
      neg = true;
      ++i_;
    }
    ByteSet s;
    bool first = true;
    for (;;) {
      if (at_end()) fail(Status::Syntax, "missing closing ]");
      if (cur() == ']' && !first) break;
      first = false;
      if (cur() == '[' && i_ + 1 < p_.size() && p_[i_ + 1] == ':') {
        const size_t e = p_.find(":]", i_ + 2);
        if (e != std::string::npos) {
          std::string name = p_.substr(i_ + 2, e - i_ - 2);
          bool pneg = !name.empty() && name[0] == '^';
          if (pneg) name = name.substr(1);
          ByteSet ps;
          if (!posix_class(name, &ps)) fail(Status::Syntax, "invalid character class range");
          s |= pneg ? ~ps : ps;
          i_ = e + 2;
          continue;
        }
      }
      uint32_t lo;
      if (cur() == '\\') {
        ++i_;
        if (at_end()) fail(Status::Syntax, "trailing backslash");
        ByteSet pc;
        if (perl_class(cur(), &pc)) {
          ++i_;
          s |= pc;
          continue;
        }
        if (cur() == 'p' || cur() == 'P') fail(Status::Unsupported, "\\p Unicode class");
        lo = escape_rune();
      } else {
        lo = next_rune();
      }
      uint32_t hi = lo;
      if (i_ + 1 < p_.size() && cur() == '-' && p_[i_ + 1] != ']') {
        ++i_;
        if (cur() == '\\') {
          ++i_;
          if (!at_end() && (perl_class(cur(), nullptr) || cur() == 'p' || cur() == 'P'))
            fail(Status::Syntax, "invalid character class range");
          hi = escape_rune();
        } else {
          hi = next_rune();
        }
        if (hi < lo) fail(Status::Syntax, "invalid character class range");
      }
      if (hi >= 0x80) fail(Status::Unsupported, "non-ASCII character class");
      s |= range(lo, hi);
    }
    ++i_;  // ']'
    if (neg) s.flip();
    return mk_set(s);
  }

  // Atom, or -1 at '|' / ')' / end.
  int atom(int depth) {
    if (at_end()) return -1;
    const unsigned char c = cur();
    switch (c) {
      case '|':
      case ')':
        return -1;
      case '*':
      case '+':
      case '?':
        fail(Status::Syntax, "missing argument to repetition operator");
      case '(': {
        ++i_;
        if (!at_end() && cur() == '?') {
          ++i_;
          if (!at_end() && cur() == ':') {
            ++i_;
          } else if (!at_end() && (cur() == 'P' || cur() == '<')) {
            if (cur() == 'P') {
              ++i_;
              if (at_end() || cur() != '<') fail(Status::Syntax, "invalid named capture");
            }
            const size_t e = p_.find('>', i_);
            if (e == std::string::npos || e == i_ + 1) fail(Status::Syntax, "invalid named capture");
            for (size_t k = i_ + 1; k < e; ++k) {
              const unsigned char ch = static_cast<unsigned char>(p_[k]);
              if (!((ch >= '0' && ch <= '9') || (ch >= 'a' && ch <= 'z') || (ch >= 'A' && ch <= 'Z') || ch == '_'))
                fail(Status::Syntax, "invalid named capture");
            }
            i_ = e + 1;
          } else {
            fail(Status::Unsupported, "flag group (?...)");
          }
        }
        const int r = alternation(depth + 1);
        if (at_end() || cur() != ')') fail(Status::Syntax, "missing closing )");
        ++i_;
        return r;
      }
      case '[':
        ++i_;
        return bracket();
      case '.': {
        ++i_;
        ByteSet s;
        s.set();
        s.reset('\n');
        return mk_set(s);
      }
      case '^':
        ++i_;
        return mk(Node::Bol);
      case '$':
        ++i_;
        return mk(Node::Eol);
      case '\\': {
        ++i_;
        if (at_end()) fail(Status::Syntax, "trailing backslash");
        const unsigned char e = cur();
        ByteSet pc;
        if (perl_class(e, &pc)) {
          ++i_;
          return mk_set(pc);
        }
        if (e == 'A') { ++i_; return mk(Node::Bol); }
        if (e == 'z') { ++i_; return mk(Node::Eol); }
        if (e == 'b' || e == 'B') fail(Status::Unsupported, "\\b / \\B word boundary");
        if (e == 'p' || e == 'P') fail(Status::Unsupported, "\\p Unicode class");
        if (e == 'Q') {
          ++i_;
          size_t end = p_.find("\\E", i_);
          std::string lit = p_.substr(i_, end == std::string::npos ? std::string::npos : end - i_);
          i_ = end == std::string::npos ? p_.size() : end + 2;
          std::vector<int> kids;
          for (unsigned char ch : lit) kids.push_back(mk_byte(ch));
          return mk_cat(std::move(kids));  // Go: a quantifier after \Q..\E binds the last char; see alternative()
        }
        return mk_rune(escape_rune());
      }
      default:
        return mk_rune(next_rune());
    }
  }

  // {n}, {n,}, {n,m} at i_ (after '{'); false (and i_ unchanged) if not a
  // valid repeat, in which case '{' is a literal.
  bool repeat_counts(int* mn, int* mx) {
    size_t k = i_ + 1;
    auto num = [&](int* v) {
      const size_t s = k;
      long long x = 0;
      while (k < p_.size() && p_[k] >= '0' && p_[k] <= '9') {
        x = x * 10 + (p_[k] - '0');
        if (x > 100000) x = 100000;
        ++k;
      }
      *v = static_cast<int>(x);
      return k > s;
    };
    if (!num(mn)) return false;
    *mx = *mn;
    if (k < p_.size() && p_[k] == ',') {
      ++k;
      if (!num(mx)) *mx = -1;
    }
    if (k >= p_.size() || p_[k] != '}') return false;
    i_ = k + 1;
    return true;
  }

  int alternative(int depth) {
    std::vector<int> seq;
    bool last_quantified = false;
    for (;;) {
      if (at_end() || cur() == '|' || cur() == ')') break;
      const unsigned char c = cur();
      int mn = -2, mx = 0;
      if (c == '*') { mn = 0; mx = -1; ++i_; }
      else if (c == '+') { mn = 1; mx = -1; ++i_; }
      else if (c == '?') { mn = 0; mx = 1; ++i_; }
      else if (c == '{') {
        int a, b;
        if (repeat_counts(&a, &b)) {
          if (a > 1000 || b > 1000 || (b >= 0 && b < a)) fail(Status::Syntax, "invalid repeat count");
          mn = a;
          mx = b;
        }
      }
      if (mn != -2) {
        if (seq.empty()) fail(Status::Syntax, "missing argument to repetition operator");
        if (last_quantified) fail(Status::Syntax, "invalid nested repetition operator");
        if (!at_end() && cur() == '?') ++i_;  // non-greedy
        Node n;
        n.kind = Node::Rep;
        n.kids = {seq.back()};
        n.min = mn;
        n.max = mx;
        // an operand of Bol/Eol/Empty repeats fine; keep it as is
        seq.back() = add(std::move(n));
        last_quantified = true;
        continue;
      }
      last_quantified = false;
      if (c == '{') {  // literal brace
        ++i_;
        seq.push_back(mk_byte('{'));
        continue;
      }
      const size_t at = i_;
      const int a = atom(depth);
      if (a < 0) break;
      // \Q..\E: a following quantifier applies to its last character only.
      if (p_.compare(at, 2, "\\Q") == 0 && ast_.nodes[a].kind == Node::Cat) {
        const std::vector<int> kids = ast_.nodes[a].kids;
        seq.insert(seq.end(), kids.begin(), kids.end());
      } else {
        seq.push_back(a);
      }
    }
    return mk_cat(std::move(seq));
  }

  int alternation(int depth) {
    if (depth > 1000) fail(Status::Syntax, "expression nests too deeply");
    std::vector<int> alts{alternative(depth)};
    while (!at_end() && cur() == '|') {
      ++i_;
      alts.push_back(alternative(depth));
    }
    if (alts.size() == 1) return alts[0];
    Node n;
    n.kind = Node::Alt;
    n.kids = std::move(alts);
    return add(std::move(n));
  }

  const std::string& p_;
  size_t i_ = 0;
  Ast ast_;
};

}  // namespace

Status parse_re2(const std::string& pat, Ast* out, std::string* err) {
  try {
    *out = Re2Parser(pat).run();
    return Status::Ok;
  } catch (const Re2Error& e) {
    if (err) *err = e.msg;
    return e.st;
  }
}

// MatchString is an unanchored search: the pattern may match any substring,
// i.e. the whole subject matches [\x00-\xff]* p [\x00-\xff]* (p's own ^ / $
// still assert the subject's ends).
// Search semantics make a pattern's trailing repetitions redundant: a
// subject contains p X{n,m} (or p X*) iff it contains p X{n} (p), so the
// trailing elements of the top-level concatenation are cut down to their
// minimum -- which keeps the per-pattern "inside the .* tail" states out of
// a search automaton's product (config 2's `/api/w/.*` family).  Nothing
// after them: a '$' keeps the pattern as it is.
void simplify_search(Ast* a) {
  std::vector<int> seq;
  const Node& r = a->nodes[a->root];
  if (r.kind == Node::Cat) seq = r.kids;
  else seq.push_back(a->root);
  while (!seq.empty()) {
    const Node& n = a->nodes[seq.back()];
    if (n.kind == Node::Rep && n.min == 0) {
      seq.pop_back();
      continue;
    }
    if (n.kind == Node::Rep && n.max != n.min) {
      Node m = n;
      m.max = m.min;
      a->nodes.push_back(m);
      seq.back() = static_cast<int>(a->nodes.size()) - 1;
    }
    break;
  }
  Node cat;
  cat.kind = Node::Cat;
  cat.kids = seq;
  a->nodes.push_back(cat);
  a->root = static_cast<int>(a->nodes.size()) - 1;
}

// Required literals: the maximal byte strings every match of the pattern
// contains (runs of single-byte atoms in a concatenation, a repeated exact
// atom's minimum, the exact string of a fully literal subexpression).
// Alternations and optional parts contribute nothing: the result is a set of
// necessary substrings, never a sufficient one.
namespace {
struct LitInfo {
  bool exact = false;          // the node matches exactly this one string
  std::string str;             // ... it
  std::vector<std::string> req;  // required substrings (non-exact nodes)
};
LitInfo lit_info(const Ast& a, int id, int depth) {
  const Node& n = a.nodes[id];
  LitInfo r;
  if (depth > 200) return r;  // deep nesting: nothing required (still a superset)
  switch (n.kind) {
    case Node::Empty:
    case Node::Bol:
    case Node::Eol:
    case Node::WordB:
    case Node::Look:
      r.exact = true;  // zero-width
      return r;
    case Node::Set:
      if (n.set.count() == 1) {
        for (int b = 0; b < 256; ++b)
          if (n.set.test(b)) r.str.push_back(static_cast<char>(b));
        r.exact = true;
      }
      return r;
    case Node::Group:
      return lit_info(a, n.kids[0], depth + 1);
    case Node::Cat: {
      std::string run;
      r.exact = true;
      for (int k : n.kids) {
        LitInfo c = lit_info(a, k, depth + 1);
        if (c.exact) {
          run += c.str;
          continue;
        }
        r.exact = false;
        if (!run.empty()) r.req.push_back(run);
        run.clear();
        for (auto& s : c.req) r.req.push_back(std::move(s));
      }
      if (r.exact) {
        r.str = run;
      } else if (!run.empty()) {
        r.req.push_back(run);
      }
      return r;
    }
    case Node::Rep: {
      LitInfo c = lit_info(a, n.kids[0], depth + 1);
      if (n.min == 0) return r;
      if (c.exact) {
        std::string s;
        for (int i = 0; i < n.min && s.size() < 64; ++i) s += c.str;
        if (n.max == n.min && s.size() < 64) {
          r.exact = true;
          r.str = s;
        } else if (!s.empty()) {
          r.req.push_back(s);
        }
        return r;
      }
      r.req = std::move(c.req);
      return r;
    }
    default:  // Alt, Backref: no required substring
      return r;
  }
}
}  // namespace

std::vector<std::string> required_literals(const Ast& a) {
  LitInfo r = lit_info(a, a.root, 0);
  if (r.exact) return r.str.empty() ? std::vector<std::string>{} : std::vector<std::string>{r.str};
  std::vector<std::string> out;
  for (auto& s : r.req)
    if (!s.empty()) out.push_back(std::move(s));
  return out;
}

namespace {
bool has_context_node(const Ast& a, int id, int depth) {
  const Node& n = a.nodes[id];
  if (depth > 400) return true;
  if (n.kind == Node::Bol || n.kind == Node::WordB || n.kind == Node::Look || n.kind == Node::Backref) return true;
  for (int k : n.kids)
    if (has_context_node(a, k, depth + 1)) return true;
  return false;
}
int copy_node(const Ast& a, int id, Ast* out) {
  Node m = a.nodes[id];
  for (int& k : m.kids) k = copy_node(a, k, out);
  out->nodes.push_back(std::move(m));
  return static_cast<int>(out->nodes.size()) - 1;
}
void key_of(const Ast& a, int id, std::string* k, int depth) {
  const Node& n = a.nodes[id];
  if (depth > 400) {
    k->append("?");
    return;
  }
  k->push_back(static_cast<char>('A' + n.kind));
  if (n.kind == Node::Set)
    for (int w = 0; w < 4; ++w) {
      uint64_t v = 0;
      for (int b = 0; b < 64; ++b)
        if (n.set.test(64 * w + b)) v |= 1ull << b;
      k->append(reinterpret_cast<const char*>(&v), 8);
    }
  if (n.kind == Node::Rep) k->append(std::to_string(n.min) + "," + std::to_string(n.max) + (n.lazy ? "l" : ""));
  k->push_back('(');
  for (int c : n.kids) key_of(a, c, k, depth + 1);
  k->push_back(')');
}
}  // namespace

bool split_literal_prefix(const Ast& a, std::string* lit, Ast* resid) {
  const Node& r = a.nodes[a.root];
  std::vector<int> kids;
  if (r.kind == Node::Cat) kids = r.kids;
  else kids.push_back(a.root);
  lit->clear();
  size_t i = 0;
  for (; i < kids.size(); ++i) {
    const Node& n = a.nodes[kids[i]];
    if (n.kind == Node::Empty) continue;
    if (n.kind != Node::Set || n.set.count() != 1) break;
    for (int b = 0; b < 256; ++b)
      if (n.set.test(b)) lit->push_back(static_cast<char>(b));
  }
  if (lit->size() < 4 || lit->size() > 255) return false;
  for (size_t j = i; j < kids.size(); ++j)
    if (has_context_node(a, kids[j], 0)) return false;
  // the residual R, followed by anything: the pattern matches at an
  // occurrence of L iff the bytes after it start with a match of R
  Ast out;
  Node cat;
  cat.kind = Node::Cat;
  for (size_t j = i; j < kids.size(); ++j) cat.kids.push_back(copy_node(a, kids[j], &out));
  Node any;
  any.kind = Node::Set;
  any.set.set();
  out.nodes.push_back(any);
  Node star;
  star.kind = Node::Rep;
  star.kids = {static_cast<int>(out.nodes.size()) - 1};
  star.min = 0;
  star.max = -1;
  out.nodes.push_back(star);
  cat.kids.push_back(static_cast<int>(out.nodes.size()) - 1);
  out.nodes.push_back(cat);
  out.root = static_cast<int>(out.nodes.size()) - 1;
  *resid = std::move(out);
  return true;
}

bool residual_is_empty(const Ast& resid) {
  const Node& r = resid.nodes[resid.root];
  for (size_t j = 0; j + 1 < r.kids.size(); ++j)
    if (resid.nodes[r.kids[j]].kind != Node::Empty) return false;
  return true;
}

std::string ast_key(const Ast& a) {
  std::string k;
  key_of(a, a.root, &k, 0);
  return k;
}

void make_search(Ast* a) {
  Node any;
  any.kind = Node::Set;
  any.set.set();
  a->nodes.push_back(any);
  const int any_id = static_cast<int>(a->nodes.size()) - 1;
  Node star;
  star.kind = Node::Rep;
  star.kids = {any_id};
  star.min = 0;
  star.max = -1;
  a->nodes.push_back(star);
  const int star_id = static_cast<int>(a->nodes.size()) - 1;
  Node cat;
  cat.kind = Node::Cat;
  cat.kids = {star_id, a->root, star_id};
  a->nodes.push_back(cat);
  a->root = static_cast<int>(a->nodes.size()) - 1;
}

}  // namespace re
}  // namespace l7m
