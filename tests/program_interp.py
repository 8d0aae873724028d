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
HDR_FIELDS = ("magic n_rules n_fields n_dfas always_rule allow_no_l7 has_name_dfa off_dfas "
              "off_fields off_name_field off_sets off_cands off_rules off_matchers off_pool "
              "off_tables table_words off_cmaps total_words off_remotes any_remotes zero_off zero_len").split()


class HttpProgram:
    def __init__(self, prog: np.ndarray):
        self.w = prog.astype(np.uint64).astype(np.int64).tolist()
        self.h = dict(zip(HDR_FIELDS, self.w[:len(HDR_FIELDS)]))
        assert self.h["magic"] == 0x5048374C
        h = self.h
        ndt = h["n_dfas"] + h["has_name_dfa"]
        self.dfas = []
        for k in range(ndt):
            o = h["off_dfas"] + 8 * k
            table_off, ncols, start, set_base, nsets, fld, nstates, cmi = self.w[o:o + 8]
            cm = prog.view(np.uint8)[4 * h["off_cmaps"] + 256 * cmi: 4 * h["off_cmaps"] + 256 * (cmi + 1)]
            self.dfas.append(dict(table_off=table_off, ncols=ncols, start=start, set_base=set_base,
                                  nsets=nsets, field=fld, cmap=cm.tolist()))
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
        d = self.dfas[k]
        tab = d["table_off"]
        s = d["start"]
        ncls = d["ncols"] - 1
        for b in data:
            s = self.w[tab + s + d["cmap"][b]]
            if s == 0:
                break
        return self.w[tab + s + ncls]

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
                sid = self.walk(h["n_dfas"], rec[pos:pos + nl])
                f = self.w[h["off_name_field"] + sid] if sid else KNONE
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
                    sid = sids[dfa]
                    if sid == 0:
                        return False
                    if pat not in self.pool(self.span(h["off_sets"], self.dfas[dfa]["set_base"] + sid)):
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
            if sids[d]:
                best = scan(self.span(h["off_cands"], self.dfas[d]["set_base"] + sids[d]), best)
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
