// regex_vm.cc — the slow path's program (regex_vm.h) from parse_ecma's AST,
// built the way libstdc++'s _Compiler builds its NFA (GCC 11
// bits/regex_compiler.tcc), state for state where the executor can tell:
//   _M_disjunction   a|b|c      left-nested alternatives (alt = left, next = right)
//   _M_quantifier    e*         repeat(alt = e) looping back from e's end
//                    e+         e, then repeat(alt = e)
//                    e?         repeat(alt = e), both to a dummy end
//                    e{n,m}     n copies of e, then m - n copies each behind a
//                               repeat whose next is the common end (the
//                               "switch _M_alt and _M_next" construction);
//                    e{n,}      n copies, then a copy looping through a repeat
//   _M_atom          (e)        subexpr begin / end around e (index = '(' order)
//   _M_assertion     (?=e)      look-ahead over e followed by accept
// and the whole pattern as subexpr 0 followed by accept.  Non-greedy
// quantifiers ('?' after them) set the repeat's lazy flag (_M_neg).
#include "regex_vm.h"

#include <cstring>
#include <string>
#include <vector>

#include "regex_ecma.h"

namespace l7m {
namespace {

struct Inst {
  uint32_t op, arg, next = kVmNone, alt = kVmNone, extra = 0;
};

struct Seq {
  uint32_t start, end;
};

class VmCompiler {
 public:
  explicit VmCompiler(const re::Ast& a) : a_(a) {}

  bool run(std::vector<uint32_t>* out, std::string* err) {
    uint32_t ncap = 1;
    for (const re::Node& n : a_.nodes)
      if (n.kind == re::Node::Group && static_cast<uint32_t>(n.min) + 1 > ncap) ncap = n.min + 1;
    Seq top{mk(kVmSubB, 0), 0};
    top.end = top.start;
    append(&top, compile(a_.root));
    append(&top, mk(kVmSubE, 0));
    append(&top, mk(kVmAccept, 0));
    if (too_big_) {
      *err = "slow-path program too large";
      return false;
    }
    const uint32_t n_inst = static_cast<uint32_t>(ins_.size());
    const uint32_t sets_off = kVmHeaderWords + 4 * n_inst;
    out->assign(sets_off + 8 * sets_.size(), 0);
    uint32_t* w = out->data();
    w[0] = kVmMagic;
    w[1] = n_inst;
    w[2] = ncap;
    w[3] = nrep_;
    w[4] = top.start;
    w[5] = sets_off;
    w[6] = static_cast<uint32_t>(out->size());
    for (uint32_t i = 0; i < n_inst; ++i) {
      const Inst& x = ins_[i];
      w[kVmHeaderWords + 4 * i] = x.op | x.arg << 8;
      w[kVmHeaderWords + 4 * i + 1] = x.next;
      w[kVmHeaderWords + 4 * i + 2] = x.alt;
      w[kVmHeaderWords + 4 * i + 3] = x.extra;
    }
    for (size_t k = 0; k < sets_.size(); ++k)
      for (int b = 0; b < 256; ++b)
        if (sets_[k].test(b)) w[sets_off + 8 * k + (b >> 5)] |= 1u << (b & 31);
    return true;
  }

 private:
  static constexpr size_t kMaxInst = 1u << 16;

  uint32_t mk(uint32_t op, uint32_t arg) {
    if (ins_.size() >= kMaxInst) {
      too_big_ = true;
      return 0;
    }
    Inst x;
    x.op = op;
    x.arg = arg;
    ins_.push_back(x);
    return static_cast<uint32_t>(ins_.size() - 1);
  }
  // _StateSeq::_M_append: the end state's next becomes id
  void append(Seq* s, uint32_t id) {
    ins_[s->end].next = id;
    s->end = id;
  }
  void append(Seq* s, const Seq& t) {
    ins_[s->end].next = t.start;
    s->end = t.end;
  }
  Seq one(uint32_t id) { return Seq{id, id}; }
  uint32_t set_id(const re::ByteSet& b) {
    for (size_t k = 0; k < sets_.size(); ++k)
      if (sets_[k] == b) return static_cast<uint32_t>(k);
    sets_.push_back(b);
    return static_cast<uint32_t>(sets_.size() - 1);
  }
  uint32_t rep(uint32_t alt, uint32_t next, bool lazy) {
    const uint32_t r = mk(kVmRep, nrep_++);
    ins_[r].alt = alt;
    ins_[r].next = next;
    ins_[r].extra = lazy ? 1u : 0u;
    return r;
  }

  Seq compile(int node) {
    if (too_big_) return one(0);
    const re::Node& n = a_.nodes[node];
    switch (n.kind) {
      case re::Node::Empty:
        return one(mk(kVmJmp, 0));
      case re::Node::Set:
        return one(mk(kVmMatch, set_id(n.set)));
      case re::Node::Cat: {
        Seq s = one(mk(kVmJmp, 0));
        for (int k : n.kids) append(&s, compile(k));
        return s;
      }
      case re::Node::Alt: {  // _M_disjunction: ((a|b)|c)
        Seq cur = compile(n.kids[0]);
        for (size_t j = 1; j < n.kids.size(); ++j) {
          Seq right = compile(n.kids[j]);
          const uint32_t end = mk(kVmJmp, 0);
          append(&cur, end);
          append(&right, end);
          const uint32_t alt = mk(kVmAlt, 0);
          ins_[alt].alt = cur.start;
          ins_[alt].next = right.start;
          cur = Seq{alt, end};
        }
        return cur;
      }
      case re::Node::Rep:
        return quant(n);
      case re::Node::Bol:
        return one(mk(kVmBol, 0));
      case re::Node::Eol:
        return one(mk(kVmEol, 0));
      case re::Node::WordB:
        return one(mk(kVmWordB, n.min ? 1u : 0u));
      case re::Node::Look: {
        Seq sub = compile(n.kids[0]);
        append(&sub, mk(kVmAccept, 0));
        const uint32_t l = mk(kVmLook, n.min ? 1u : 0u);
        ins_[l].alt = sub.start;
        return one(l);
      }
      case re::Node::Group: {
        Seq s = one(mk(kVmSubB, static_cast<uint32_t>(n.min)));
        append(&s, compile(n.kids[0]));
        append(&s, mk(kVmSubE, static_cast<uint32_t>(n.min)));
        return s;
      }
      case re::Node::Backref:
        return one(mk(kVmBackref, static_cast<uint32_t>(n.min)));
    }
    return one(mk(kVmJmp, 0));
  }

  Seq quant(const re::Node& n) {
    const int kid = n.kids[0];
    if (!n.brace) {
      if (n.min == 0 && n.max < 0) {  // e*
        Seq e = compile(kid);
        const uint32_t r = rep(e.start, kVmNone, n.lazy);
        append(&e, r);
        return one(r);
      }
      if (n.min == 1 && n.max < 0) {  // e+
        Seq e = compile(kid);
        append(&e, rep(e.start, kVmNone, n.lazy));
        return e;
      }
      // e?
      Seq e = compile(kid);
      const uint32_t end = mk(kVmJmp, 0);
      const uint32_t r = rep(e.start, end, n.lazy);
      append(&e, end);
      return Seq{r, end};
    }
    // e{n}, e{n,}, e{n,m}: copies of e (_StateSeq::_M_clone)
    if (static_cast<size_t>(n.min) + (n.max > n.min ? n.max - n.min : 1) > kMaxInst) {
      too_big_ = true;
      return one(0);
    }
    Seq s = one(mk(kVmJmp, 0));
    for (int k = 0; k < n.min; ++k) append(&s, compile(kid));
    if (n.max < 0) {
      Seq t = compile(kid);
      const uint32_t r = rep(t.start, kVmNone, n.lazy);
      append(&t, r);
      append(&s, r);
    } else {
      const uint32_t end = mk(kVmJmp, 0);
      for (int k = 0; k < n.max - n.min; ++k) {
        Seq t = compile(kid);
        const uint32_t r = rep(t.start, end, n.lazy);  // alt = one more copy, next = the end
        append(&s, Seq{r, t.end});
      }
      append(&s, end);
    }
    return s;
  }

  const re::Ast& a_;
  std::vector<Inst> ins_;
  std::vector<re::ByteSet> sets_;
  uint32_t nrep_ = 0;
  bool too_big_ = false;
};

}  // namespace

bool vm_compile(const re::Ast& full, std::vector<uint32_t>* out, std::string* err) {
  VmCompiler c(full);
  return c.run(out, err);
}

}  // namespace l7m
