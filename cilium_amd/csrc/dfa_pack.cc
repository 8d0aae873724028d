// dfa_pack.cc — see dfa_pack.h.
#include "dfa_pack.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>

namespace l7m {
namespace {

constexpr uint32_t kNoPat = 0xffffffffu;
constexpr uint32_t kTail = 0x80000000u;  // product target flag: latched (tail) node id

// L7M_COMPILE_TRACE=1: per-phase compile times on stderr (development aid).
struct Trace {
  bool on = std::getenv("L7M_COMPILE_TRACE") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char* what, uint64_t n) {
    if (!on) return;
    auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[l7m compile] %-12s %10llu  %.3f s\n", what, static_cast<unsigned long long>(n),
                 std::chrono::duration<double>(now - t).count());
    t = now;
  }
};

// ---------------------------------------------------------------- split --
// A pattern = literal prefix (bytes every match starts with) + residual regex.
// The residual is determinised on its own and shared by every pattern with
// the same residual; the prefixes form the product's trie.
void flatten_cat(const re::Ast& a, int node, std::vector<int>* seq) {
  const re::Node& n = a.nodes[node];
  if (n.kind == re::Node::Cat) {
    for (int k : n.kids) flatten_cat(a, k, seq);
  } else {
    seq->push_back(node);
  }
}

// Assertions whose answer depends on where the residual starts: '^' (only at
// position 0) and '\b' / '\B' (the byte before); look-ahead is kept out of
// residuals too (its automaton is built with the residual's own start).
bool has_bol(const re::Ast& a, int node) {
  const re::Node& n = a.nodes[node];
  if (n.kind == re::Node::Bol || n.kind == re::Node::WordB || n.kind == re::Node::Look) return true;
  for (int k : n.kids)
    if (has_bol(a, k)) return true;
  return false;
}

int single_byte(const re::ByteSet& s) {
  if (s.count() != 1) return -1;
  for (int b = 0; b < 256; ++b)
    if (s.test(b)) return b;
  return -1;
}

void put32(std::string* k, uint32_t v) { k->append(reinterpret_cast<const char*>(&v), 4); }

// Deep copy of a subtree into dst, appending its canonical (self-delimiting)
// serialisation to key: equal keys = structurally equal residuals.
int copy_node(const re::Ast& src, int node, re::Ast* dst, std::string* key) {
  const re::Node& n = src.nodes[node];
  re::Node m;
  m.kind = n.kind;
  m.min = n.min;
  m.max = n.max;
  switch (n.kind) {
    case re::Node::Set: {
      const int b = single_byte(n.set);
      if (b >= 0) {
        key->push_back('c');
        key->push_back(static_cast<char>(b));
      } else {
        key->push_back('s');
        for (int w = 0; w < 32; ++w) {
          uint8_t x = 0;
          for (int k = 0; k < 8; ++k) x |= (n.set.test(8 * w + k) ? 1 : 0) << k;
          key->push_back(static_cast<char>(x));
        }
      }
      m.set = n.set;
      break;
    }
    case re::Node::Cat:
    case re::Node::Alt:
    case re::Node::Rep:
    case re::Node::Look:
      key->push_back(n.kind == re::Node::Cat ? 'C' : n.kind == re::Node::Alt ? 'A' : n.kind == re::Node::Rep ? 'R' : 'L');
      if (n.kind == re::Node::Rep || n.kind == re::Node::Look) {
        put32(key, static_cast<uint32_t>(n.min));
        put32(key, static_cast<uint32_t>(n.max));
      }
      put32(key, static_cast<uint32_t>(n.kids.size()));
      for (int k : n.kids) m.kids.push_back(copy_node(src, k, dst, key));
      break;
    case re::Node::Bol: key->push_back('^'); break;
    case re::Node::Eol: key->push_back('$'); break;
    case re::Node::Empty: key->push_back('e'); break;
    case re::Node::WordB: key->push_back(n.min ? 'B' : 'b'); break;
    case re::Node::Group:
    case re::Node::Backref:  // (removed by lower_for_dfa before any automaton is built)
      key->push_back('?');
      break;
  }
  dst->nodes.push_back(std::move(m));
  return static_cast<int>(dst->nodes.size()) - 1;
}

struct Split {
  std::string lit;
  re::Ast rest;
  std::string key;
};

void split_pattern(const re::Ast& a, Split* out) {
  std::vector<int> seq;
  flatten_cat(a, a.root, &seq);
  size_t k = 0;
  // Leading '^' always holds at position 0 (regex_match, no multiline).
  while (k < seq.size() && a.nodes[seq[k]].kind == re::Node::Bol) ++k;
  std::string lit;
  while (k < seq.size() && a.nodes[seq[k]].kind == re::Node::Set) {
    const int b = single_byte(a.nodes[seq[k]].set);
    if (b < 0) break;
    lit.push_back(static_cast<char>(b));
    ++k;
  }
  // The residual is determinised as if it started the subject: a '^' inside
  // it must stay at position 0, so such patterns are not split.
  for (size_t j = k; j < seq.size() && !lit.empty(); ++j)
    if (has_bol(a, seq[j])) {
      lit.clear();
      k = 0;
      break;
    }
  out->lit = lit;
  out->rest = re::Ast();
  out->key.clear();
  const size_t rem = seq.size() - k;
  if (rem == 0) {
    re::Node e;
    e.kind = re::Node::Empty;
    out->rest.nodes.push_back(e);
    out->rest.root = 0;
    out->key = "e";
  } else if (rem == 1) {
    out->rest.root = copy_node(a, seq[k], &out->rest, &out->key);
  } else {
    re::Node cat;
    cat.kind = re::Node::Cat;
    out->key.push_back('C');
    put32(&out->key, static_cast<uint32_t>(rem));
    for (size_t j = k; j < seq.size(); ++j) cat.kids.push_back(copy_node(a, seq[j], &out->rest, &out->key));
    out->rest.nodes.push_back(std::move(cat));
    out->rest.root = static_cast<int>(out->rest.nodes.size()) - 1;
  }
}

// ------------------------------------------------------------- residual --
// A determinised residual in sparse form: per state the non-dead
// transitions as (local class << 24 | target); state 0 is dead.
struct Residual {
  uint8_t cmap[256];
  uint32_t ncls = 0;
  uint32_t start = 0;
  uint32_t nstates = 0;
  std::vector<uint32_t> row;  // nstates + 1 offsets into tr
  std::vector<uint32_t> tr;
  std::vector<uint8_t> accept;
  std::vector<std::vector<uint8_t>> bytes;   // local class -> bytes
  std::vector<std::vector<uint16_t>> gcls;   // local class -> global classes
};

re::Status make_residual(const re::Ast& a, Residual* r) {
  re::Dfa d;
  re::DfaLimits lim;
  re::Status st = re::build_dfa({&a}, lim, &d);
  if (st != re::Status::Ok) return st;
  if (d.nstates >= (1 << 24) || d.ncls > 256) return re::Status::TooBig;
  std::memcpy(r->cmap, d.cmap, 256);
  r->ncls = static_cast<uint32_t>(d.ncls);
  r->start = static_cast<uint32_t>(d.start);
  r->nstates = static_cast<uint32_t>(d.nstates);
  r->row.assign(r->nstates + 1, 0);
  r->accept.assign(r->nstates, 0);
  for (uint32_t q = 0; q < r->nstates; ++q) {
    r->row[q] = static_cast<uint32_t>(r->tr.size());
    if (q != 0)
      for (uint32_t c = 0; c < r->ncls; ++c) {
        const uint32_t t = d.next[static_cast<size_t>(q) * d.ncls + c];
        if (t) r->tr.push_back(c << 24 | t);
      }
    r->accept[q] = d.endset[q] != 0 ? 1 : 0;
  }
  r->row[r->nstates] = static_cast<uint32_t>(r->tr.size());
  r->bytes.assign(r->ncls, {});
  for (int b = 0; b < 256; ++b) r->bytes[r->cmap[b]].push_back(static_cast<uint8_t>(b));
  return re::Status::Ok;
}

struct VecHash {
  size_t operator()(const std::vector<uint64_t>& v) const {
    uint64_t h = 1469598103934665603ull ^ v.size();
    for (uint64_t x : v) {
      h ^= x;
      h *= 1099511628211ull;
      h ^= h >> 31;
    }
    return static_cast<size_t>(h);
  }
};

// First-fit double-array placement over 24-bit bases.
class Packer {
 public:
  // Smallest base >= lo, not yet a base, whose slots base+b (b in bytes) are free.
  bool place(const uint8_t* bytes, size_t nb, uint32_t lo, uint32_t* out) {
    uint32_t base;
    if (nb == 0) {
      base = std::max(lo, empty_cursor_);
      while (base < taken_.size() && taken_[base]) ++base;
      empty_cursor_ = base;
    } else {
      const uint32_t b0 = bytes[0];
      // dense rows start near the end of the used range: first-fit from the
      // first free slot would re-scan the packed prefix for every one of them
      uint32_t f = std::max(lo + b0, std::max(first_free_, nb > 32 ? dense_cursor_ : 0u));
      uint32_t tries = 0;
      for (;; ++f) {
        if (f < used_.size() && used_[f]) continue;
        ++tries;
        base = f - b0;
        if (base > kMaxDaBase) return false;
        if (base < lo || (base < taken_.size() && taken_[base])) continue;
        bool ok = true;
        for (size_t k = 1; k < nb && ok; ++k) {
          const uint32_t s = base + bytes[k];
          ok = !(s < used_.size() && used_[s]);
        }
        if (ok) break;
      }
      // Holes no row could use (every label's base taken) would be re-scanned
      // by every later row: after a long search give up on the old ones.
      if (tries > 64 && f > 512) first_free_ = std::max(first_free_, f - 512);
    }
    if (base > kMaxDaBase) return false;
    if (taken_.size() <= base) taken_.resize(static_cast<size_t>(base) + 1, 0);
    taken_[base] = 1;
    for (size_t k = 0; k < nb; ++k) {
      const uint32_t s = base + bytes[k];
      if (used_.size() <= s) used_.resize(static_cast<size_t>(s) + 1, 0);
      used_[s] = 1;
    }
    while (first_free_ < used_.size() && used_[first_free_]) ++first_free_;
    if (nb > 32) dense_cursor_ = std::max(dense_cursor_, static_cast<uint32_t>(used_.size() > 256 ? used_.size() - 256 : 0));
    *out = base;
    return true;
  }
  // Next rows go at bases >= lo: first-fit cursors never look below it (the
  // holes left under a phase boundary would otherwise be re-scanned per row).
  void begin_phase(uint32_t lo) {
    first_free_ = std::max(first_free_, lo);
    while (first_free_ < used_.size() && used_[first_free_]) ++first_free_;
    dense_cursor_ = std::max(dense_cursor_, lo);
  }
  void reserve_base(uint32_t b) {
    if (taken_.size() <= b) taken_.resize(static_cast<size_t>(b) + 1, 0);
    taken_[b] = 1;
  }

 private:
  std::vector<char> used_, taken_;
  uint32_t first_free_ = 0, empty_cursor_ = 0, dense_cursor_ = 0;
};

}  // namespace

re::Status build_field_dfa(const std::vector<const re::Ast*>& patterns, const FieldDfaLimits& lim,
                           PackedDfa* out) {
  const uint32_t np = static_cast<uint32_t>(patterns.size());
  Trace tr;
  // 1. split patterns, determinise each distinct residual once
  std::vector<std::string> lit(np);
  std::vector<uint32_t> rid(np);
  std::vector<Residual> res;
  {
    std::unordered_map<std::string, uint32_t> rkey;
    std::vector<re::Ast> rast;  // distinct residuals
    Split sp;
    for (uint32_t p = 0; p < np; ++p) {
      split_pattern(*patterns[p], &sp);
      lit[p] = std::move(sp.lit);
      auto it = rkey.find(sp.key);
      if (it == rkey.end()) {
        it = rkey.emplace(sp.key, static_cast<uint32_t>(rast.size())).first;
        rast.push_back(std::move(sp.rest));
      }
      rid[p] = it->second;
    }
    // determinise the distinct residuals on the host's cores (independent)
    res.resize(rast.size());
    std::vector<re::Status> rst(rast.size(), re::Status::Ok);
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t i; (i = next.fetch_add(1)) < rast.size();) rst[i] = make_residual(rast[i], &res[i]);
    };
    const unsigned hw = std::thread::hardware_concurrency();
    const size_t nth = std::min<size_t>(rast.size() / 64 + 1, std::min<unsigned>(hw ? hw : 1, 16));
    std::vector<std::thread> th;
    for (size_t t = 1; t < nth; ++t) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
    for (re::Status st : rst)
      if (st != re::Status::Ok) return st;
  }
  const uint32_t nres = static_cast<uint32_t>(res.size());
  tr.mark("residuals", nres);

  // 2. field-wide byte partition: refines every residual's classes and makes
  // every literal-prefix byte a singleton
  uint16_t gc[256] = {0};
  uint32_t ng = 1;
  {
    std::vector<int> pairid(256 * 256, -1);
    std::vector<int> touched;
    auto refine = [&](const uint8_t* key) {
      uint16_t tmp[256];
      int n2 = 0;
      for (int b = 0; b < 256; ++b) {
        const int k = gc[b] * 256 + key[b];
        if (pairid[k] < 0) {
          pairid[k] = n2++;
          touched.push_back(k);
        }
        tmp[b] = static_cast<uint16_t>(pairid[k]);
      }
      for (int k : touched) pairid[k] = -1;
      touched.clear();
      std::memcpy(gc, tmp, sizeof gc);
      ng = static_cast<uint32_t>(n2);
    };
    uint8_t litkey[256] = {0};
    bool any_lit = false;
    for (uint32_t p = 0; p < np; ++p)
      for (unsigned char c : lit[p]) {
        litkey[c] = 1;
        any_lit = true;
      }
    if (any_lit) {
      uint8_t k2[256];
      for (int b = 0; b < 256; ++b) k2[b] = litkey[b] ? static_cast<uint8_t>(b) : 0;
      // k2 makes every literal byte but 0 a singleton; the mask itself then
      // separates a literal byte 0 from the non-literal bytes
      refine(k2);
      refine(litkey);
    }
    for (uint32_t r = 0; r < nres; ++r)
      if (res[r].ncls > 1) refine(res[r].cmap);
  }
  std::vector<std::vector<uint8_t>> gbytes(ng);
  std::vector<uint8_t> grep(ng, 0);
  for (int b = 255; b >= 0; --b) grep[gc[b]] = static_cast<uint8_t>(b);
  for (int b = 0; b < 256; ++b) gbytes[gc[b]].push_back(static_cast<uint8_t>(b));
  for (auto& r : res) {
    r.gcls.assign(r.ncls, {});
    for (uint32_t g = 0; g < ng; ++g) r.gcls[r.cmap[grep[g]]].push_back(static_cast<uint16_t>(g));
  }

  // 3. product of the per-pattern automata until one pattern remains live.
  // Item = pattern << 32 | pos: pos < |lit| is a literal position, else
  // residual state pos - |lit| (>= 1).
  std::unordered_map<std::vector<uint64_t>, uint32_t, VecHash> mid;
  std::vector<const std::vector<uint64_t>*> multi;  // id - 1 -> items
  struct MTr {
    uint16_t g;    // field byte class
    uint32_t tgt;  // multi id, or kTail | tail id
    uint32_t pat;  // tails: the one pattern still live
  };
  std::vector<std::vector<MTr>> mtr;  // product transitions
  std::vector<uint32_t> mset;                       // end set id per multi state
  std::vector<std::vector<uint32_t>> sets{{}};
  std::unordered_map<std::vector<uint64_t>, uint32_t, VecHash> set_ids;
  set_ids.emplace(std::vector<uint64_t>{}, 0);

  // tails (latched nodes): the states of each used residual, and literal
  // chain nodes hash-consed on (byte, next node) so that equal literal
  // suffixes before equal residuals are one chain (config 2: the 500
  // `/svc{i}/` rules share the "v" node in front of their common residual)
  constexpr uint32_t kDeadTail = 0xffffffffu;
  std::unordered_map<uint64_t, uint32_t> chain_id;  // byte << 32 | next -> tail id
  std::vector<uint64_t> chain_key;                   // chain index -> byte << 32 | next
  std::vector<uint32_t> rbase(nres, kNoPat);
  uint32_t ntail = 0;
  std::vector<uint8_t> tail_kind;  // 0 chain, 1 residual state (for rows)
  std::vector<uint32_t> tail_ref;  // chain: index into chain_key; residual: rid
  auto ensure_res = [&](uint32_t r) {
    if (rbase[r] != kNoPat) return;
    rbase[r] = ntail;
    const uint32_t k = res[r].nstates - 1;  // state q >= 1 -> tail rbase + q - 1
    ntail += k;
    tail_kind.insert(tail_kind.end(), k, 1);
    tail_ref.insert(tail_ref.end(), k, r);
  };
  auto tail_of = [&](uint64_t item) -> uint32_t {
    const uint32_t p = static_cast<uint32_t>(item >> 32), pos = static_cast<uint32_t>(item);
    const uint32_t L = static_cast<uint32_t>(lit[p].size());
    ensure_res(rid[p]);
    const Residual& R = res[rid[p]];
    if (pos >= L) return rbase[rid[p]] + (pos - L) - 1;
    uint32_t next = R.start ? rbase[rid[p]] + R.start - 1 : kDeadTail;
    for (uint32_t i = L; i-- > pos;) {
      const uint64_t key = static_cast<uint64_t>(static_cast<uint8_t>(lit[p][i])) << 32 | next;
      auto it = chain_id.find(key);
      if (it == chain_id.end()) {
        it = chain_id.emplace(key, ntail++).first;
        tail_kind.push_back(0);
        tail_ref.push_back(static_cast<uint32_t>(chain_key.size()));
        chain_key.push_back(key);
      }
      next = it->second;
    }
    return next;
  };
  std::vector<uint64_t> start_items;
  for (uint32_t p = 0; p < np; ++p) {
    if (!lit[p].empty()) start_items.push_back(static_cast<uint64_t>(p) << 32);
    else if (res[rid[p]].start) start_items.push_back(static_cast<uint64_t>(p) << 32 | res[rid[p]].start);
  }
  uint32_t start_row = 0;  // product node: 0 dead, m >= 1 multi, kTail | t
  uint32_t start_latch = kNoPat;
  auto intern_multi = [&](std::vector<uint64_t>&& items, bool* fresh) -> uint32_t {
    auto it = mid.find(items);
    if (it != mid.end()) {
      *fresh = false;
      return it->second;
    }
    const uint32_t id = static_cast<uint32_t>(multi.size()) + 1;
    it = mid.emplace(std::move(items), id).first;
    multi.push_back(&it->first);
    *fresh = true;
    return id;
  };
  if (start_items.size() == 1) {
    start_row = kTail | tail_of(start_items[0]);
    start_latch = static_cast<uint32_t>(start_items[0] >> 32);
  } else if (start_items.size() > 1) {
    bool fresh;
    start_row = intern_multi(std::move(start_items), &fresh);
  }
  {
    std::vector<std::vector<uint64_t>> bk(ng);
    std::vector<uint16_t> used;
    std::vector<uint64_t> acc;
    for (size_t m = 0; m < multi.size(); ++m) {
      if (multi.size() > lim.max_multi_states) return re::Status::TooBig;
      const std::vector<uint64_t>& S = *multi[m];
      for (uint16_t g : used) bk[g].clear();
      used.clear();
      acc.clear();
      auto push = [&](uint16_t g, uint64_t it) {
        if (bk[g].empty()) used.push_back(g);
        bk[g].push_back(it);
      };
      for (uint64_t item : S) {
        const uint32_t p = static_cast<uint32_t>(item >> 32), pos = static_cast<uint32_t>(item);
        const uint32_t L = static_cast<uint32_t>(lit[p].size());
        const Residual& R = res[rid[p]];
        const uint64_t hi = static_cast<uint64_t>(p) << 32;
        if (pos < L) {
          uint32_t nxt = pos + 1;
          if (nxt == L) {
            if (!R.start) continue;
            nxt = L + R.start;
          }
          push(gc[static_cast<unsigned char>(lit[p][pos])], hi | nxt);
        } else {
          const uint32_t q = pos - L;
          if (R.accept[q]) acc.push_back(p);
          for (uint32_t k = R.row[q]; k < R.row[q + 1]; ++k) {
            const uint32_t lc = R.tr[k] >> 24, t = R.tr[k] & 0xffffffu;
            for (uint16_t g : R.gcls[lc]) push(g, hi | (L + t));
          }
        }
      }
      std::sort(used.begin(), used.end());
      std::vector<MTr> trs;
      trs.reserve(used.size());
      for (uint16_t g : used) {
        std::vector<uint64_t>& S2 = bk[g];
        if (S2.size() == 1) {
          trs.push_back({g, kTail | tail_of(S2[0]), static_cast<uint32_t>(S2[0] >> 32)});
        } else {
          bool fresh;
          trs.push_back({g, intern_multi(std::vector<uint64_t>(S2), &fresh), kNoPat});
        }
      }
      mtr.push_back(std::move(trs));
      std::sort(acc.begin(), acc.end());
      auto si = set_ids.find(acc);
      uint32_t sid;
      if (si == set_ids.end()) {
        sid = static_cast<uint32_t>(sets.size());
        set_ids.emplace(acc, sid);
        sets.emplace_back(acc.begin(), acc.end());
      } else {
        sid = si->second;
      }
      mset.push_back(sid);
    }
  }
  const uint32_t nmulti = static_cast<uint32_t>(multi.size());
  tr.mark("product", nmulti);
  mid.clear();  // frees the item vectors
  multi.clear();

  // 4. rows: 0 dead, 1..nmulti product states, then tails
  const uint64_t nrows64 = 1ull + nmulti + ntail;
  if (nrows64 > kMaxDaBase) return re::Status::TooBig;
  const uint32_t nrows = static_cast<uint32_t>(nrows64);
  auto row_of = [&](uint32_t tgt) -> uint32_t { return (tgt & kTail) ? 1 + nmulti + (tgt & ~kTail) : tgt; };
  // explicit (byte, target row, latched pattern) list of a row
  struct RB {
    uint8_t b;
    uint32_t row;
    uint32_t pat;
    bool operator<(const RB& o) const { return b < o.b; }
  };
  std::vector<RB> rb;
  auto row_bytes = [&](uint32_t row) {
    rb.clear();
    if (row == 0) return;
    if (row <= nmulti) {
      for (const auto& tg : mtr[row - 1])
        for (uint8_t b : gbytes[tg.g]) rb.push_back({b, row_of(tg.tgt), tg.pat});
    } else {
      const uint32_t t = row - 1 - nmulti;
      if (tail_kind[t] == 0) {
        const uint64_t key = chain_key[tail_ref[t]];
        const uint32_t next = static_cast<uint32_t>(key);
        if (next != kDeadTail) rb.push_back({static_cast<uint8_t>(key >> 32), 1 + nmulti + next, kNoPat});
      } else {
        const uint32_t r = tail_ref[t];
        const Residual& R = res[r];
        const uint32_t q = t - rbase[r] + 1;
        for (uint32_t k = R.row[q]; k < R.row[q + 1]; ++k) {
          const uint32_t lc = R.tr[k] >> 24, tq = R.tr[k] & 0xffffffu;
          for (uint8_t b : R.bytes[lc]) rb.push_back({b, 1 + nmulti + rbase[r] + tq - 1, kNoPat});
        }
      }
    }
    std::sort(rb.begin(), rb.end());
  };
  auto row_accept = [&](uint32_t row) -> uint32_t {
    if (row == 0) return 0;
    if (row <= nmulti) return mset[row - 1];
    const uint32_t t = row - 1 - nmulti;
    if (tail_kind[t] == 0) return 0;  // a literal byte is still required
    const uint32_t r = tail_ref[t];
    return res[r].accept[t - rbase[r] + 1] ? kLatchedAccept : 0;
  };

  // 4b. skip rows (dfa_pack.h kSkipLoop / kSkipLit) among the tails: loop
  // rows, and literal runs of >= 2 bytes starting at a residual state or at a
  // chain node entered from >= 2 rows (the shared, hot ones: config 2's
  // `\.ns\.local` authority suffix, `(users|orders|items)/`); placed last so
  // that `base >= skip_lim` identifies them.
  std::vector<uint8_t> skind(nrows, 0);  // 1 loop, 2 one non-accepting transition to another row
  std::vector<uint32_t> snext(nrows, 0);
  std::vector<uint32_t> indeg(nrows, 0);
  for (uint32_t r = 1; r < nrows; ++r) {
    row_bytes(r);
    for (const auto& x : rb) ++indeg[x.row];
    if (r <= nmulti) continue;
    bool loop = true;
    for (const auto& x : rb) loop &= x.row == r;
    if (loop) skind[r] = 1;
    else if (rb.size() == 1 && row_accept(r) == 0) {
      skind[r] = 2;
      snext[r] = rb[0].row;
    }
  }
  std::vector<uint8_t> runlen(nrows, 0);  // literal run length from a kind-2 row (capped)
  for (uint32_t r = 1 + nmulti; r < nrows; ++r) {
    if (skind[r] != 2 || runlen[r]) continue;
    std::vector<uint32_t> path;
    uint32_t c = r;
    while (c && skind[c] == 2 && !runlen[c] && path.size() < 64) {
      runlen[c] = 0xff;  // on the current path (cycle guard)
      path.push_back(c);
      c = snext[c];
    }
    uint32_t tail_len = (c && skind[c] == 2 && runlen[c] != 0xff) ? runlen[c] : 0;
    for (size_t i = path.size(); i-- > 0;) {
      tail_len = tail_len + 1 > kSkipMaxLit ? kSkipMaxLit : tail_len + 1;
      runlen[path[i]] = static_cast<uint8_t>(tail_len);
    }
  }
  std::vector<uint8_t> has_skip(nrows, 0);
  {
    uint32_t nrows_skip = 0, pool = 0;
    for (uint32_t r = 1 + nmulti; r < nrows && nrows_skip < kSkipMaxRows; ++r)
      if (skind[r] == 1) {
        has_skip[r] = 1;
        ++nrows_skip;
      }
    // hot runs: rows of residual automata, chain nodes entered from >= 2 rows,
    // and every later row of a hot run (a block boundary can land anywhere in it)
    std::vector<uint8_t> hot(nrows, 0);
    for (uint32_t r = 1 + nmulti; r < nrows; ++r) {
      if (skind[r] != 2 || hot[r] || !(tail_kind[r - 1 - nmulti] == 1 || indeg[r] >= 2)) continue;
      for (uint32_t c = r, i = 0; c && skind[c] == 2 && !hot[c] && i < 64; c = snext[c], ++i) hot[c] = 1;
    }
    for (uint32_t r = 1 + nmulti; r < nrows && nrows_skip < kSkipMaxRows; ++r) {
      if (skind[r] != 2 || runlen[r] < 2) continue;
      if (!hot[r] || pool + runlen[r] > kSkipMaxPool) continue;
      has_skip[r] = 1;
      ++nrows_skip;
      pool += runlen[r];
    }
  }

  // 5. placement: product rows below `region`, tails at or above (skip rows
  // last); dense rows of each phase first
  std::vector<uint32_t> base(nrows, 0);
  std::vector<uint16_t> cnt(nrows, 0);
  uint64_t n_explicit = 0;
  for (uint32_t r = 1; r < nrows; ++r) {
    row_bytes(r);
    cnt[r] = static_cast<uint16_t>(rb.size());
    n_explicit += rb.size();
  }
  if (n_explicit > lim.max_slots) return re::Status::TooBig;
  Packer pk;
  pk.reserve_base(0);  // dead
  uint32_t max_base = 0;
  std::vector<uint8_t> bytes;
  auto place_phase = [&](uint32_t lo_row, uint32_t hi_row, uint32_t lo_base, int skip_sel) -> bool {
    pk.begin_phase(lo_base);
    std::vector<std::vector<uint32_t>> by(257);
    for (uint32_t r = lo_row; r < hi_row; ++r)
      if (skip_sel < 0 || has_skip[r] == skip_sel) by[cnt[r]].push_back(r);
    for (int c = 256; c >= 0; --c)
      for (uint32_t r : by[c]) {
        row_bytes(r);
        bytes.clear();
        for (const auto& x : rb) bytes.push_back(x.b);
        if (!pk.place(bytes.data(), bytes.size(), lo_base, &base[r])) return false;
        max_base = std::max(max_base, base[r]);
      }
    return true;
  };
  tr.mark("rows", nrows);
  if (!place_phase(1, 1 + nmulti, 1, -1)) return re::Status::TooBig;
  const uint32_t region = max_base + 1;
  if (!place_phase(1 + nmulti, nrows, region, 0)) return re::Status::TooBig;
  const uint32_t skip_lim = max_base + 1;
  bool any_skip = false;
  for (uint32_t r = 1 + nmulti; r < nrows; ++r) any_skip |= has_skip[r] != 0;
  if (any_skip && !place_phase(1 + nmulti, nrows, skip_lim, 1)) return re::Status::TooBig;
  tr.mark("placement", max_base);

  // 6. tables
  PackedDfa d;
  d.n_slots = max_base + 256 + 1;
  d.table.assign(d.n_slots, 0u);
  d.es.assign(d.n_slots, 0u);
  d.latch.assign(static_cast<size_t>(region) + 256, kNoPat);
  for (uint32_t r = 1; r < nrows; ++r) {
    row_bytes(r);
    const bool is_multi = r <= nmulti;
    for (const auto& x : rb) {
      const uint32_t slot = base[r] + x.b;
      d.table[slot] = base[x.row] << 8 | x.b;
      // entering the latched region: remember which pattern is still live
      if (is_multi && x.row > nmulti) d.latch[slot] = x.pat;
    }
    d.es[base[r]] = row_accept(r);
  }
  tr.mark("tables", d.n_slots);
  if (any_skip) {
    d.skip_lim = skip_lim;
    d.skip.assign(max_base + 1 - skip_lim, 0u);
    for (uint32_t r = 1 + nmulti; r < nrows; ++r) {
      if (!has_skip[r]) continue;
      uint32_t w = kSkipLoop;
      if (skind[r] == 2) {
        const uint32_t n = runlen[r], off = static_cast<uint32_t>(d.skip_lits.size());
        uint32_t c = r, tslot = 0;
        for (uint32_t i = 0; i < n; ++i) {  // the run's bytes; tslot = its last transition's slot
          row_bytes(c);
          d.skip_lits.push_back(rb[0].b);
          tslot = base[c] + rb[0].b;
          c = rb[0].row;
        }
        w = kSkipLit | n << 2 | off << 7 | tslot << 16;
        if (tslot >= (1u << 16)) w = 0;  // beyond an LDS table's reach: no skip
      }
      d.skip[base[r] - skip_lim] = w;
    }
  }
  d.start_base = start_row == 0 ? 0u : base[row_of(start_row)];
  d.start_latch = start_latch;
  d.region = region;
  d.nstates = nrows;
  d.n_explicit = n_explicit;
  d.n_multi = nmulti;
  d.n_residuals = nres;
  d.sets = std::move(sets);
  *out = std::move(d);
  return re::Status::Ok;
}

uint32_t packed_walk(const PackedDfa& p, const uint8_t* s, size_t n) {
  uint32_t base = p.start_base, last = kNoPat;
  for (size_t i = 0; i < n && base; ++i) {
    const uint32_t slot = base + s[i];
    const uint32_t e = p.table[slot];
    if (base < p.region) last = slot;
    base = (e & 0xffu) == s[i] ? e >> 8 : 0u;
  }
  if (!base) return 0;
  const uint32_t es = p.es[base];
  if (es == kLatchedAccept) return kLatchedAccept | (last == kNoPat ? p.start_latch : p.latch[last]);
  return es;
}

}  // namespace l7m
