// dfa_pack.cc — see dfa_pack.h.
#include "dfa_pack.h"

#include <algorithm>
#include <unordered_map>

namespace l7m {
namespace {

constexpr uint32_t kNoPat = 0xffffffffu;

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

struct Row {
  int orig;                   // representative original DFA state
  std::vector<uint8_t> bytes;  // explicit bytes (ascending)
  std::vector<uint32_t> tgt;   // new-state id per explicit byte
  uint32_t base = 0;
};

// First-fit double-array placement.
class Packer {
 public:
  // Smallest base >= lo, not yet a base, whose slots base+b (b in bytes) are free.
  bool place(const std::vector<uint8_t>& bytes, uint32_t lo, uint32_t* out) {
    uint32_t base;
    if (bytes.empty()) {
      base = std::max(lo, empty_cursor_);
      while (base < taken_.size() && taken_[base]) ++base;
      empty_cursor_ = base;
    } else {
      const uint32_t b0 = bytes[0];
      uint32_t f = std::max(lo + b0, first_free_);
      for (;; ++f) {
        if (f < used_.size() && used_[f]) continue;
        base = f - b0;
        if (base < lo || (base < taken_.size() && taken_[base])) continue;
        bool ok = true;
        for (size_t k = 1; k < bytes.size() && ok; ++k) {
          const uint32_t s = base + bytes[k];
          ok = !(s < used_.size() && used_[s]);
        }
        if (ok) break;
        if (base > kMaxDaBase) return false;
      }
    }
    if (base > kMaxDaBase) return false;
    if (taken_.size() <= base) taken_.resize(base + 1, 0);
    taken_[base] = 1;
    for (uint8_t b : bytes) {
      const uint32_t s = base + b;
      if (used_.size() <= s) used_.resize(s + 1, 0);
      used_[s] = 1;
    }
    while (first_free_ < used_.size() && used_[first_free_]) ++first_free_;
    *out = base;
    return true;
  }
  void reserve_base(uint32_t b) {
    if (taken_.size() <= b) taken_.resize(b + 1, 0);
    taken_[b] = 1;
  }

 private:
  std::vector<char> used_, taken_;
  uint32_t first_free_ = 0, empty_cursor_ = 0;
};

}  // namespace

re::Status pack_dfa(const re::Dfa& d, PackedDfa* out) {
  const int n = d.nstates, nc = d.ncls;
  auto nxt = [&](int s, int c) { return static_cast<int>(d.next[static_cast<size_t>(s) * nc + c]); };

  // 1. live patterns per state: count capped at 2 plus one representative.
  std::vector<uint8_t> cnt(n, 0);
  std::vector<uint32_t> rep(n, kNoPat);
  std::vector<std::vector<int>> rev(n);
  for (int s = 0; s < n; ++s) {
    for (int c = 0; c < nc; ++c) rev[nxt(s, c)].push_back(s);
    const auto& set = d.sets[d.endset[s]];
    if (set.size() >= 2) cnt[s] = 2;
    if (set.size() == 1) {
      cnt[s] = 1;
      rep[s] = set[0];
    }
  }
  std::vector<int> work;
  for (int s = 0; s < n; ++s) {
    auto& r = rev[s];
    std::sort(r.begin(), r.end());
    r.erase(std::unique(r.begin(), r.end()), r.end());
    if (cnt[s]) work.push_back(s);
  }
  while (!work.empty()) {
    const int t = work.back();
    work.pop_back();
    for (int s : rev[t]) {
      uint8_t c0 = cnt[s];
      uint32_t r0 = rep[s];
      if (c0 == 2) continue;
      if (cnt[t] == 2) {
        cnt[s] = 2;
      } else if (c0 == 0) {
        cnt[s] = 1;
        rep[s] = rep[t];
      } else if (rep[s] != rep[t]) {
        cnt[s] = 2;
      }
      if (cnt[s] != c0 || rep[s] != r0) work.push_back(s);
    }
  }

  // 2. minimise the latched (single-pattern) states with binary acceptance.
  // blk: -1 = not latched; dead (cnt 0) handled as a fixed block.
  std::vector<int> blk(n, -1);
  int nblk = 0;
  {
    bool any_acc = false, any_rej = false;
    for (int s = 0; s < n; ++s)
      if (cnt[s] == 1) (d.endset[s] ? any_acc : any_rej) = true;
    for (int s = 0; s < n; ++s)
      if (cnt[s] == 1) blk[s] = (d.endset[s] && any_rej) ? 1 : 0;
    nblk = (any_acc ? 1 : 0) + (any_rej ? 1 : 0);
    std::vector<uint32_t> sig(static_cast<size_t>(nc) + 1);
    for (;;) {
      std::unordered_map<std::vector<uint32_t>, int, U32VecHash> ids;
      std::vector<int> nb(n, -1);
      for (int s = 0; s < n; ++s) {
        if (blk[s] < 0) continue;
        sig[0] = static_cast<uint32_t>(blk[s]);
        for (int c = 0; c < nc; ++c) {
          const int t = nxt(s, c);
          // transitions out of a latched state stay latched or die
          sig[c + 1] = cnt[t] == 0 ? 0xffffffffu : static_cast<uint32_t>(blk[t]);
        }
        auto it = ids.find(sig);
        if (it == ids.end()) it = ids.emplace(sig, static_cast<int>(ids.size())).first;
        nb[s] = it->second;
      }
      const int nn = static_cast<int>(ids.size());
      blk.swap(nb);
      if (nn == nblk) break;
      nblk = nn;
    }
  }

  // 3. packed states: dead = 0, multi-pattern states, then latched blocks.
  std::vector<uint32_t> nid(n, 0);
  std::vector<Row> rows;  // rows[i] is packed state i + 1
  rows.reserve(n);
  for (int s = 0; s < n; ++s)
    if (cnt[s] == 2) {
      nid[s] = static_cast<uint32_t>(rows.size()) + 1;
      rows.push_back(Row{s});
    }
  const uint32_t n_multi = static_cast<uint32_t>(rows.size());
  {
    std::vector<int> first_of(nblk, -1);
    for (int s = 0; s < n; ++s)
      if (blk[s] >= 0 && first_of[blk[s]] < 0) first_of[blk[s]] = s;
    std::vector<uint32_t> bid(nblk, 0);
    std::vector<int> order;
    for (int b = 0; b < nblk; ++b)
      if (first_of[b] >= 0) order.push_back(b);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return first_of[a] < first_of[b]; });
    for (int b : order) {
      bid[b] = static_cast<uint32_t>(rows.size()) + 1;
      rows.push_back(Row{first_of[b]});
    }
    for (int s = 0; s < n; ++s)
      if (blk[s] >= 0) nid[s] = bid[blk[s]];
  }

  // 4. rows over raw bytes: every non-dead transition is explicit.
  uint64_t n_explicit = 0;
  for (uint32_t i = 0; i < rows.size(); ++i) {
    Row& r = rows[i];
    for (int b = 0; b < 256; ++b) {
      const uint32_t t = nid[nxt(r.orig, d.cmap[b])];
      if (t != 0) {
        r.bytes.push_back(static_cast<uint8_t>(b));
        r.tgt.push_back(t);
      }
    }
    n_explicit += r.bytes.size();
  }

  // 5. placement: multi-pattern rows below `region`, latched rows at or above.
  Packer pk;
  pk.reserve_base(0);  // dead
  uint32_t max_base = 0;
  for (uint32_t i = 0; i < n_multi; ++i) {
    if (!pk.place(rows[i].bytes, 1, &rows[i].base)) return re::Status::TooBig;
    max_base = std::max(max_base, rows[i].base);
  }
  const uint32_t region = max_base + 1;
  for (uint32_t i = n_multi; i < rows.size(); ++i) {
    if (!pk.place(rows[i].bytes, region, &rows[i].base)) return re::Status::TooBig;
    max_base = std::max(max_base, rows[i].base);
  }

  // 6. tables
  PackedDfa p;
  p.n_slots = max_base + 256 + 1;
  p.table.assign(p.n_slots, 0xffffu);
  p.es.assign(p.n_slots, 0);
  p.latch.assign(p.n_slots, kNoPat);
  auto base_of = [&](uint32_t id) -> uint32_t { return id == 0 ? 0u : rows[id - 1].base; };
  for (uint32_t i = 0; i < rows.size(); ++i) {
    const Row& r = rows[i];
    const bool multi = i < n_multi;
    for (size_t k = 0; k < r.bytes.size(); ++k) {
      const uint32_t slot = r.base + r.bytes[k];
      p.table[slot] = r.base | (base_of(r.tgt[k]) << 16);
      if (multi && r.tgt[k] > n_multi) {
        // entering the latched region: remember which pattern is still live
        p.latch[slot] = rep[nxt(r.orig, d.cmap[r.bytes[k]])];
      }
    }
    p.es[r.base] = multi ? d.endset[r.orig] : (d.endset[r.orig] ? kLatchedAccept : 0u);
  }
  const int s0 = d.start;
  if (cnt[s0] != 0) {
    p.start_base = base_of(nid[s0]);
    if (cnt[s0] == 1) p.start_latch = rep[s0];
  }
  p.region = region;
  p.nstates = static_cast<uint32_t>(rows.size()) + 1;
  p.n_explicit = static_cast<uint32_t>(n_explicit);
  p.sets = d.sets;
  *out = std::move(p);
  return re::Status::Ok;
}

uint32_t packed_walk(const PackedDfa& p, const uint8_t* s, size_t n) {
  uint32_t base = p.start_base, last = kNoPat;
  for (size_t i = 0; i < n && base; ++i) {
    const uint32_t slot = base + s[i];
    const uint32_t e = p.table[slot];
    if (base < p.region) last = slot;
    base = (e & 0xffffu) == base ? e >> 16 : 0u;
  }
  if (!base) return 0;
  const uint32_t es = p.es[base];
  if (es == kLatchedAccept) return kLatchedAccept | (last == kNoPat ? p.start_latch : p.latch[last]);
  return es;
}

}  // namespace l7m
