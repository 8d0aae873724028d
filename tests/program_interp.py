"""Pure-Python interpreter of the compiled HTTP device program (TEST INFRA).

It walks the exact blob libl7match uploads to HBM (cilium_amd/csrc/program.h)
with the same algorithm as http_eval_kernel, so the rule COMPILER (regex ->
DFA groups, candidate lists, matcher tables) can be checked against the CPU
oracle without a GPU.  The kernel itself is checked on the GPU by the -m gpu
tests.  Small inputs only (pure-Python loops)."""
import struct

import numpy as np

from cilium_amd import l7match as L

KNONE = 0xFFFFFFFF
LATCHED = 0x80000000
HDR_FIELDS = ("magic n_rules n_fields n_dfas always_rule allow_no_l7 has_name_dfa off_dfas "
              "off_fields off_name_field off_sets off_cands off_rules off_matchers off_pool "
              "off_pcands lds_image_off lds_image_words total_words off_remotes any_remotes "
              "zero_off zero_len").split()
DFA_FIELDS = ("table_off lds_off start_desc region start_latch es_off latch_off n_slots set_base nsets "
              "pcand_base npats field nstates").split()


class HttpProgram:
    def __init__(self, prog: np.ndarray):
        self.w = prog.astype(np.uint64).astype(np.int64).tolist()
        self.h = dict(zip(HDR_FIELDS, self.w[:len(HDR_FIELDS)]))
        assert self.h["magic"] == 0x3248374C
        h = self.h
        ndt = h["n_dfas"] + h["has_name_dfa"]
        self.dfas = []
        for k in range(ndt):
            o = h["off_dfas"] + 16 * k
            d = dict(zip(DFA_FIELDS, self.w[o:o + len(DFA_FIELDS)]))
            if d["lds_off"] != KNONE:  # the LDS image is a copy of program words
                assert d["table_off"] == h["lds_image_off"] + d["lds_off"]
            self.dfas.append(d)
        self.fields = []
        for f in range(h["n_fields"]):
            o = h["off_fields"] + 4 * f
            self.fields.append(tuple(self.w[o:o + 4]))

    def span(self, off_words, idx):
        o = off_words + 2 * idx
        return self.w[o], self.w[o + 1]

    def pool(self, sp):
        o, n = sp
        b = self.h["off_pool"] + o
        return self.w[b:b + n]

    def walk(self, k, data: bytes):
        """Packed double-array walk (cilium_amd/csrc/dfa_pack.h): end code."""
        d = self.dfas[k]
        T = d["table_off"]
        desc = d["start_desc"]
        base = desc >> 1
        last = KNONE
        for b in data:
            if not desc:
                break
            slot = base + b
            e = self.w[T + slot]
            if base < d["region"]:
                last = slot
            if (e & 0xFFFF) == base:
                desc = e >> 16
            elif not desc & 1:
                desc = 0
            base = desc >> 1
        if not desc:
            return 0
        es = self.w[d["es_off"] + base]
        if es == LATCHED:
            return LATCHED | (d["start_latch"] if last == KNONE else self.w[d["latch_off"] + last])
        return es

    def eval_record(self, rec: bytes) -> int:
        h = self.h
        w0, remote, w2, w3, w4 = struct.unpack_from("<5I", rec, 0)
        flags = (w2 >> 16) & 0xFF
        nhdr = w2 >> 24
        mlen, plen, alen = w3 & 0xFFFF, w3 >> 16, w4 & 0xFFFF
        dirs = [struct.unpack_from("<I", rec, 20 + 4 * j)[0] for j in range(nhdr)]
        if 20 + 4 * nhdr + mlen + plen + alen + sum((e & 0xFFFF) + (e >> 16) for e in dirs) != w0:
            return L.VERDICT_PARSE_ERROR
        sids = [0] * h["n_dfas"]
        present = 0
        pos = 20 + 4 * nhdr

        def eval_field(f, data):
            first, nd, _po, _pl = self.fields[f]
            for k in range(first, first + nd):
                sids[k] = self.walk(k, data)

        for f, flag, ln in ((0, L.F_METHOD, mlen), (1, L.F_PATH, plen), (2, L.F_AUTHORITY, alen)):
            if flags & flag:
                present |= 1 << f
                eval_field(f, rec[pos:pos + ln])
            pos += ln
        if h["has_name_dfa"]:
            for e in dirs:
                nl, vl = e & 0xFFFF, e >> 16
                code = self.walk(h["n_dfas"], rec[pos:pos + nl])
                if code & LATCHED:
                    f = 3 + (code & ~LATCHED)
                else:
                    f = self.w[h["off_name_field"] + code] if code else KNONE
                if f != KNONE and not (present >> f) & 1:
                    present |= 1 << f
                    eval_field(f, rec[pos + nl:pos + nl + vl])
                pos += nl + vl
        best = h["always_rule"]

        def verify(rid):
            rr = self.pool(self.span(h["off_remotes"], rid))
            if rr and remote not in rr:
                return False
            mo, mn = self.span(h["off_rules"], rid)
            for j in range(mn):
                o = h["off_matchers"] + 4 * (mo + j)
                fld, kind, dfa, pat = self.w[o:o + 4]
                if not (present >> fld) & 1:
                    return False
                if kind == 0:
                    code = sids[dfa]
                    if code == 0:
                        return False
                    if code & LATCHED:
                        if code & ~LATCHED != pat:
                            return False
                    elif pat not in self.pool(self.span(h["off_sets"], self.dfas[dfa]["set_base"] + code)):
                        return False
            return True

        def scan(sp, best):
            for rid in self.pool(sp):
                if rid >= best:
                    break
                if verify(rid):
                    return rid
            return best

        for d in range(h["n_dfas"]):
            code = sids[d]
            if code & LATCHED:
                best = scan(self.span(h["off_pcands"], self.dfas[d]["pcand_base"] + (code & ~LATCHED)), best)
            elif code:
                best = scan(self.span(h["off_cands"], self.dfas[d]["set_base"] + code), best)
        for f in range(h["n_fields"]):
            if (present >> f) & 1:
                best = scan((self.fields[f][2], self.fields[f][3]), best)
        best = scan((h["zero_off"], h["zero_len"]), best)
        if h["allow_no_l7"]:
            return L.VERDICT_ALLOW_NO_L7
        return L.VERDICT_DENY if best == KNONE else best

    def eval(self, arena: np.ndarray, offsets: np.ndarray) -> np.ndarray:
        buf = arena.tobytes()
        out = np.empty(len(offsets), dtype=np.int32)
        for i, o in enumerate(offsets.tolist()):
            ln = struct.unpack_from("<I", buf, o)[0]
            out[i] = self.eval_record(buf[o:o + ((ln + 3) & ~3)])
        return out
