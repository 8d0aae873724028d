"""Pure-Python interpreter of the compiled HTTP device program (TEST INFRA).

It walks the exact blob libl7match uploads to HBM (cilium_amd/csrc/program.h)
with the same algorithm as http_eval_kernel, reading the LDS-image copies of
the tables where the kernel does (so the u16 end-code / latch images and the
LDS candidate tables are checked too).  This lets the rule COMPILER (regex ->
packed DFA groups, check records) be checked against the CPU oracle without a
GPU; the kernel itself is checked on the GPU by the -m gpu tests.  Small
inputs only (pure-Python loops)."""
import ctypes
import os
import struct

import numpy as np

from cilium_amd import l7match as L

_VM = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "bin", "libvmhost.so"))
_VM.vm_host_match.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
# regex_vm.h kVmScratchWords2 / kVmMaxSteps2: the slow pass's second tier (a
# request the first tier could not decide runs again with these), so the
# verdict is the one these limits give
VM_SCRATCH_WORDS, VM_MAX_STEPS = 262144, 1 << 25
VM_DEEP, VM_LIMIT = -2, -1
CR_SLOW = 0x40000000  # program.h kCrSlow

KNONE = 0xFFFFFFFF
LATCHED = 0x80000000
ES16_LATCHED = 0xFFFF
CR_REMOTE = 0x80000000
HDR_FIELDS = ("magic n_rules n_fields n_dfas always_rule allow_no_l7 has_name_dfa off_dfas off_fields "
              "off_name_field off_sets off_cr off_pool off_remotes any_remotes zero_off zero_len "
              "lds_image_off lds_image_words lds_dfas lds_fields lds_name_field total_words lds_name_tab "
              "name_tab_mask single_entry n_policies ent_tab_off lds_ent_tab ent_mask name_len_lo name_len_hi "
              "cand_dfas_lo cand_dfas_hi pres_fields_lo pres_fields_hi search lds_dcap off_slow n_slow").split()
DFA_FIELDS = ("table_off es_off latch_off ct_off lds_table lds_es lds_latch lds_ct lds_mask start_base region "
              "start_latch n_slots nsets npats set_base field nstates lds_ctmask ctmask_off start_es8 lit_tab "
              "lds_skip skip_lim kind acc_cmap_off acc_mid_off acc_ncls lds_search lds_mid").split()
ES_IN_ENTRY = 0xFFFFFFFE  # program.h kLdsEsInEntry
DFA_WORDS = 32  # sizeof(DfaDesc) / 4
DFA_SEARCH = 1  # program.h kDfaSearch
DFA_ALIT = 2    # program.h kDfaAlit
DCAP_SHIFT, PAT_MASK = 24, (1 << 24) - 1  # program.h kDcapShift / kPatMask
ALIT_BLOOM_BITS = 0  # program.h L7M_ALIT_BLOOM_BITS of the default build (prefilter off)


def gram_bucket(g):
    """program.h gram_bucket."""
    x = g ^ (g >> 15)
    return (((x & 0xFFFFFF) * 0x9E3779) & 0xFFFFFFFF) >> 10


def name_hash(data: bytes) -> int:
    """program.h name_hash_step / name_hash_final."""
    M = 0xFFFFFFFF
    h = 0
    for k in range((len(data) + 3) // 4):
        w = int.from_bytes(data[4 * k:4 * k + 4].ljust(4, b"\0"), "little")
        x = h ^ w
        h = ((x & 0xFFFFFF) * 0x9E3779 + (((x << 13) | (x >> 19)) & M)) & M
    h = ((h ^ len(data)) * 0x85EBCA6B) & M
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M
    h ^= h >> 16
    return h or 1


class HttpProgram:
    def __init__(self, prog: np.ndarray):
        self.prog = np.ascontiguousarray(prog, dtype=np.uint32)
        self.w = prog.astype(np.uint64).astype(np.int64).tolist()
        self.h = dict(zip(HDR_FIELDS, self.w[:len(HDR_FIELDS)]))
        h = self.h
        assert h["magic"] == 0x3448374C
        assert len(HDR_FIELDS) == 40  # program.h HttpHeader, 40 words
        io = h["lds_image_off"]
        self.img = self.w[io:io + h["lds_image_words"]]
        self.img16 = prog[io:io + h["lds_image_words"]].view(np.uint16).tolist()
        ndt = h["n_dfas"] + h["has_name_dfa"]
        # literal-anchored fields' residual automata follow the name DFA
        for f in range(h["n_fields"]):
            r = self.w[h["off_fields"] + 16 * f + 12]
            if r != KNONE:
                ndt = max(ndt, r + 1)
        # forced-capture patterns' R automata follow those (program.h DcapSpec)
        self.dcaps = []
        if h["lds_dcap"] != KNONE:
            dm = 0
            for f in range(h["n_fields"]):
                dm |= self.w[h["off_fields"] + 16 * f + 15]
            for k in range(dm.bit_length()):
                sp = self.img[h["lds_dcap"] + 16 * k: h["lds_dcap"] + 16 * k + 16]
                self.dcaps.append(sp)
                if sp[3] != KNONE:
                    ndt = max(ndt, sp[3] + 1)
        self.dfas = []
        for k in range(ndt):
            o = h["lds_dfas"] + DFA_WORDS * k  # the kernel reads the LDS copy
            d = dict(zip(DFA_FIELDS, self.img[o:o + len(DFA_FIELDS)]))
            g = h["off_dfas"] + DFA_WORDS * k
            assert self.w[g:g + DFA_WORDS] == self.img[o:o + DFA_WORDS]
            self.dfas.append(d)
        # program.h FieldDesc (16 words): dfa_first, ndfa, presence off/len,
        # gram_tab, gram_mask, always, search_first, n_search, alit_tab,
        # alit_mask, alit_pats, resid_dfa, alit_lds, alit_granules, dcap_mask
        self.fields = [tuple(self.img[h["lds_fields"] + 16 * f: h["lds_fields"] + 16 * f + 16])
                       for f in range(h["n_fields"])]
        self.prog_bytes = self.prog.tobytes()
        self.img_bytes = prog[io:io + h["lds_image_words"]].tobytes()

    def alit_scan(self, f, data: bytes, codes):
        """Literal-anchored RE2 patterns (program.h FieldDesc::alit_*): at
        every position whose 4-byte gram hits the table, compare the
        pattern's literal L at position - k and walk the residual automaton
        from the end of L; matched patterns set their bit in their kDfaAlit
        group's code."""
        fd = self.fields[f]
        tab, amask, pats, rdfa = fd[9], fd[10], fd[11], fd[12]
        for q in range(len(data) - 3):
            g = int.from_bytes(data[q:q + 4], "little")
            b = tab + 4 * (gram_bucket(g) & amask)
            e = self.img[b:b + 4]
            for eg, ep in ((e[0], e[1]), (e[2], e[3])):
                if not ep or eg != g:
                    continue
                # a build with the prefilter (program.h L7M_ALIT_BLOOM_BITS)
                # probes the bucket only where the gram's bit is set: no
                # table gram may lack it
                if ALIT_BLOOM_BITS:
                    bb = (gram_bucket(g) >> 8) & ((1 << ALIT_BLOOM_BITS) - 1)
                    assert (self.img[tab - (1 << ALIT_BLOOM_BITS) // 32 + (bb >> 5)] >> (bb & 31)) & 1, \
                        "alit prefilter misses a table gram"
                words, byts = (self.img, self.img_bytes) if fd[13] else (self.w, self.prog_bytes)  # alit_lds
                r = pats + 4 * (ep - 1)  # AlitRec: header granule, then L's bytes
                len_k, code, resid, _ = words[r:r + 4]
                ln, k = len_k & 0xFFFF, len_k >> 16
                s = q - k
                if s < 0 or s + ln > len(data) or data[s:s + ln] != byts[4 * (r + 4):4 * (r + 4) + ln]:
                    continue
                if resid != KNONE:
                    rc = self.walk(rdfa, data[s + ln:])
                    if not self.code_has(rdfa, rc, resid):
                        continue
                codes[code >> 8] |= 1 << (code & 31)

    def dcap_holds(self, k, data: bytes):
        """Forced-capture back-reference pattern k (program.h DcapSpec):
        P1, the maximal class run (length in [min, max]), L2, the run
        repeated, then R's automaton on the rest."""
        sp = self.dcaps[k]
        l1, l2 = sp[0] & 0xFFFF, sp[0] >> 16
        mn, mx, rdfa, cls = sp[1], sp[2], sp[3], sp[4:12]
        p1 = self.img_bytes[4 * sp[12]: 4 * sp[12] + l1]
        lit2 = self.img_bytes[4 * sp[13]: 4 * sp[13] + l2]
        if len(data) < l1 + l2 or data[:l1] != p1:
            return False
        e = l1
        while e < len(data) and (cls[data[e] >> 5] >> (data[e] & 31)) & 1:
            e += 1
        r = e - l1
        if r < mn or r > mx or e + l2 + r > len(data):
            return False
        if data[e:e + l2] != lit2 or data[e + l2:e + l2 + r] != data[l1:e]:
            return False
        t = e + l2 + r
        if rdfa == KNONE:
            return t == len(data)
        return self.code_has(rdfa, self.walk(rdfa, data[t:]), 0)

    def gram_select(self, f, data: bytes):
        """RE2-dialect gram filter (program.h FieldDesc::gram_tab): the mask
        of search groups (bit j % 32) a value must walk; None = walk all."""
        fd = self.fields[f]
        tab, gmask, always = fd[4], fd[5], fd[6]
        if tab == KNONE:
            return None
        m = always
        for i in range(len(data) - 3):
            g = int.from_bytes(data[i:i + 4], "little")
            b = tab + 4 * (gram_bucket(g) & gmask)
            e = self.img[b:b + 4]
            if e[0] == g:
                m |= e[1]
            if e[2] == g:
                m |= e[3]
        return m

    def name_tab_lookup(self, name: bytes):
        h = self.h
        hk = name_hash(name)
        at = hk & h["name_tab_mask"]
        while True:
            sl = self.img[h["lds_name_tab"] + 4 * at: h["lds_name_tab"] + 4 * at + 4]
            if sl[0] == 0:
                return KNONE
            if sl[0] == hk and sl[1] == len(name):
                words = self.img[sl[3]: sl[3] + (len(name) + 3) // 4]
                stored = b"".join(int(x).to_bytes(4, "little") for x in words)[:len(name)]
                if stored == name:
                    return sl[2]
            at = (at + 1) & h["name_tab_mask"]

    def walk_search(self, d, data: bytes):
        """Search automaton (program.h kDfaSearch): mask of the patterns
        matching some substring of data."""
        cm = b"".join(int(x).to_bytes(4, "little") for x in self.w[d["acc_cmap_off"]:d["acc_cmap_off"] + 64])
        ncls, T, mid = d["acc_ncls"], d["table_off"], d["acc_mid_off"]
        st, acc = d["start_base"], d["start_es8"]
        for b in data:
            e = self.w[T + st * ncls + cm[b]]
            st = e & 0xFFFFFF
            acc |= self.w[mid + (e >> 24)]
        return acc | self.w[d["es_off"] + st]

    def walk(self, k, data: bytes):
        """Packed double-array walk (cilium_amd/csrc/dfa_pack.h): end code."""
        d = self.dfas[k]
        if d["kind"] == DFA_SEARCH:
            return self.walk_search(d, data)
        lds = d["lds_table"] != KNONE
        base = d["start_base"]
        last = KNONE
        es8 = d["start_es8"]
        if lds:
            # LDS copy (program.h kLdsRowShift): e = (image row byte address
            # << 16) | es8 << 8 | label, 0 for dead transitions
            t0 = d["lds_table"]
            n = len(data)
            st = [base, es8, last]

            def step(c):
                bs = st[0]
                slot = bs + c
                e = self.img[t0 + slot]
                if bs < d["region"]:
                    st[2] = slot
                ok = (e & 0xFF) == c and (e >> 16) != 0  # row 0: the shared dead row
                st[0], st[1] = ((e >> 16) // 4 - t0, (e >> 8) & 0xFF) if ok else (0, 0)

            k = 0
            while k < n and st[0]:
                step(data[k])
                k += 1
            base, es8, last = st
        else:
            for b in data:
                if not base:
                    break
                slot = base + b
                e = self.w[d["table_off"] + slot]
                if base < d["region"]:
                    last = slot
                base = e >> 8 if (e & 0xFF) == b else 0
        if not base:
            return 0
        if lds and d["lds_es"] == ES_IN_ENTRY:
            if es8 != 0xFF:
                return es8
            return LATCHED | (d["start_latch"] if last == KNONE else self.img16[d["lds_latch"] + last])
        if lds and d["lds_es"] != KNONE:  # table-only LDS placement keeps end codes in the program
            es = self.img16[d["lds_es"] + base]
            if es != ES16_LATCHED:
                return es
            return LATCHED | (d["start_latch"] if last == KNONE else self.img16[d["lds_latch"] + last])
        es = self.w[d["es_off"] + base]
        if es != LATCHED:
            return es
        return LATCHED | (d["start_latch"] if last == KNONE else self.w[d["latch_off"] + last])

    def code_has(self, k, code, p):
        if code == 0:
            return False
        if self.dfas[k]["kind"] in (DFA_SEARCH, DFA_ALIT):
            return bool((code >> p) & 1)
        if code & LATCHED:
            return (code & ~LATCHED) == p
        d = self.dfas[k]
        if d["lds_mask"] != KNONE:
            lo, hi = self.img[d["lds_mask"] + 2 * code], self.img[d["lds_mask"] + 2 * code + 1]
            return bool(((hi << 32 | lo) >> p) & 1)
        so = self.h["off_sets"] + 2 * (d["set_base"] + code)
        po, pl = self.w[so], self.w[so + 1]
        return p in self.w[self.h["off_pool"] + po: self.h["off_pool"] + po + pl]

    def ct(self, k, idx):
        """Candidate list (pool offset, record count) of end-code index idx;
        checks the LDS presence bit and the inlined first record."""
        d = self.dfas[k]
        bit = (self.w[d["ctmask_off"] + (idx >> 5)] >> (idx & 31)) & 1
        if d["lds_ctmask"] != KNONE:
            assert bit == (self.img[d["lds_ctmask"] + (idx >> 5)] >> (idx & 31)) & 1
        if d["lds_ct"] != KNONE:
            e = self.img[d["lds_ct"] + 16 * idx: d["lds_ct"] + 16 * idx + 16]
        else:
            e = self.w[d["ct_off"] + 16 * idx: d["ct_off"] + 16 * idx + 16]
        n, off = e[0], e[1]
        assert bit == (1 if n else 0)
        if n:
            cr = self.h["off_cr"] + off
            nm = self.w[cr + 1] & 0xFF
            k_in = 2 + 2 * min(nm, 4)
            assert e[2:2 + k_in] == self.w[cr:cr + k_in]
        return off, n

    def ent_lookup(self, key):
        h = self.h
        if h["lds_ent_tab"] != KNONE:
            tab = self.img[h["lds_ent_tab"]: h["lds_ent_tab"] + 2 * (h["ent_mask"] + 1)]
            assert tab == self.w[h["ent_tab_off"]: h["ent_tab_off"] + 2 * (h["ent_mask"] + 1)]
        at = (((key * 0x9E3779B1) & 0xFFFFFFFF) >> 7) & h["ent_mask"]
        while True:
            k = self.w[h["ent_tab_off"] + 2 * at]
            if k == 0:
                return KNONE
            if k == key + 1:
                return self.w[h["ent_tab_off"] + 2 * at + 1]
            at = (at + 1) & h["ent_mask"]

    def slow_ok(self, rid, fvals):
        """The slow path (regex_vm.h, host build): every slow matcher of rule
        rid on its field's value; None when an evaluation hit its limits."""
        h = self.h
        so, sl = self.w[h["off_slow"] + 2 * rid: h["off_slow"] + 2 * rid + 2]
        for q in range(sl):
            f, off = self.w[h["off_pool"] + so + 2 * q], self.w[h["off_pool"] + so + 2 * q + 1]
            v = fvals.get(f)
            if v is None:
                return False
            r = _VM.vm_host_match(self.prog[off:].ctypes.data, v, len(v), VM_SCRATCH_WORDS, VM_MAX_STEPS)
            if r < 0:
                return None
            if r == 0:
                return False
        return True

    def eval_record(self, rec: bytes) -> int:
        """Both passes of the kernel: the first defers a request whose best
        candidate may be a slow-path rule (kCrSlow), the second
        (http_slow_kernel) evaluates those rules exactly."""
        v = self._eval(rec, False)
        return self._eval(rec, True) if v is None else v

    def _eval(self, rec: bytes, slow: bool):
        h = self.h
        w0, remote, w2, w3, w4 = struct.unpack_from("<5I", rec, 0)
        flags = (w2 >> 16) & 0xFF
        nhdr = w2 >> 24
        mlen, plen, alen = w3 & 0xFFFF, w3 >> 16, w4 & 0xFFFF
        dirs = [struct.unpack_from("<I", rec, 20 + 4 * j)[0] for j in range(nhdr)]
        if 20 + 4 * nhdr + mlen + plen + alen + sum((e & 0xFFFF) + (e >> 16) for e in dirs) != w0:
            return L.VERDICT_PARSE_ERROR
        # port entry selection (kernel: l7m_kernels.hip eval_record)
        pol, dport = w4 >> 16, w2 & 0xFFFF
        ex = e0 = 0
        h0 = True
        if h["single_entry"]:
            if pol != 0:
                return L.VERDICT_DENY
            if h["allow_no_l7"]:
                return L.VERDICT_ALLOW_NO_L7
        else:
            if pol >= h["n_policies"]:
                return L.VERDICT_DENY
            key0 = pol << 17 | (1 if flags & L.F_INGRESS else 0) << 16
            vx = self.ent_lookup(key0 | dport) if dport else KNONE
            v0 = self.ent_lookup(key0)
            if vx == KNONE and v0 == KNONE:
                return L.VERDICT_ALLOW_NO_PORT_POLICY
            first = vx if vx != KNONE else v0
            if not first & 0x80000000:
                return L.VERDICT_ALLOW_NO_L7
            ex = first & 0x7FFFFFFF
            both = vx != KNONE and v0 != KNONE
            e0 = (v0 & 0x7FFFFFFF) if both else ex
            h0 = bool(v0 & 0x80000000) if both else True

        def eligible(hd):
            e = (hd >> 8) & ((1 << 22) - 1)
            return e == ex or (h0 and e == e0)
        codes = [0] * h["n_dfas"]
        dmask = [0]  # forced-capture patterns that hold
        present = 0
        pos = 20 + 4 * nhdr
        fvals = {}

        def eval_field(f, data):
            fvals[f] = data
            first, nd = self.fields[f][0], self.fields[f][1]
            sf, ns = self.fields[f][7], self.fields[f][8]
            sel = self.gram_select(f, data)
            for k in range(first, first + nd):
                if self.dfas[k]["kind"] == DFA_ALIT:
                    codes[k] = 0  # set by the alit scan below
                    continue
                if sel is not None and sf <= k - first < sf + ns and not (sel >> ((k - first - sf) & 31)) & 1:
                    codes[k] = 0  # no chosen gram of the group's patterns: not walked
                    continue
                codes[k] = self.walk(k, data)
            if self.fields[f][9] != KNONE:
                self.alit_scan(f, data, codes)
            if h["lds_dcap"] != KNONE:
                m = self.fields[f][15]
                for k in range(32):
                    if (m >> k) & 1 and self.dcap_holds(k, data):
                        dmask[0] |= 1 << k

        for f, flag, ln in ((0, L.F_METHOD, mlen), (1, L.F_PATH, plen), (2, L.F_AUTHORITY, alen)):
            if flags & flag:
                present |= 1 << f
                eval_field(f, rec[pos:pos + ln])
            pos += ln
        if h["has_name_dfa"]:
            lmask = h["name_len_hi"] << 32 | h["name_len_lo"]
            for e in dirs:
                nl, vl = e & 0xFFFF, e >> 16
                if not (lmask >> min(nl, 63)) & 1:  # no referenced name has this length
                    pos += nl + vl
                    continue
                code = self.walk(h["n_dfas"], rec[pos:pos + nl])
                if code & LATCHED:
                    f = 3 + (code & ~LATCHED)
                else:
                    f = self.img[h["lds_name_field"] + code] if code else KNONE
                if h["lds_name_tab"] != KNONE:  # the kernel's table must agree with the DFA
                    assert self.name_tab_lookup(rec[pos:pos + nl]) == f
                if f != KNONE and not (present >> f) & 1:
                    present |= 1 << f
                    eval_field(f, rec[pos + nl:pos + nl + vl])
                pos += nl + vl
        best = h["always_rule"]
        cr = h["off_cr"]
        min_slow = [KNONE]
        limit = [KNONE]  # smallest rule whose slow evaluation hit its limits

        def remote_ok(rid):
            ro, rl = self.w[h["off_remotes"] + 2 * rid: h["off_remotes"] + 2 * rid + 2]
            return remote in self.w[h["off_pool"] + ro: h["off_pool"] + ro + rl]

        def scan(span, best):
            o, n = span
            for _ in range(n):
                rid, hd = self.w[cr + o], self.w[cr + o + 1]
                nm = hd & 0xFF
                if rid >= best:
                    break
                ok = eligible(hd) and (not (hd & CR_REMOTE) or remote_ok(rid))
                for q in range(nm):
                    if not ok:
                        break
                    a, pat = self.w[cr + o + 2 + 2 * q], self.w[cr + o + 3 + 2 * q]
                    if not (present >> (a & 0xFF)) & 1:
                        ok = False
                    elif not (a >> 8) & 1:
                        dk = pat >> DCAP_SHIFT
                        ok = self.code_has(a >> 9, codes[a >> 9], pat & PAT_MASK) and \
                            (dk == 0 or bool((dmask[0] >> (dk - 1)) & 1))
                if ok and hd & CR_SLOW:  # a superset automaton matched
                    if not slow:
                        min_slow[0] = min(min_slow[0], rid)
                        ok = False
                    else:
                        r = self.slow_ok(rid, fvals)
                        if r is None:
                            limit[0] = min(limit[0], rid)
                        ok = bool(r)
                if ok:
                    return rid
                o += 2 + 2 * nm
            return best

        for k in range(h["n_dfas"]):
            code = codes[k]
            if not code:
                continue
            if self.dfas[k]["kind"] in (DFA_SEARCH, DFA_ALIT):  # candidates of every matched pattern
                for p in range(32):
                    if (code >> p) & 1:
                        best = scan(self.ct(k, p), best)
                continue
            idx = self.dfas[k]["nsets"] + (code & ~LATCHED) if code & LATCHED else code
            best = scan(self.ct(k, idx), best)
        for f in range(h["n_fields"]):
            if (present >> f) & 1:
                best = scan((self.fields[f][2], self.fields[f][3]), best)
        best = scan((h["zero_off"], h["zero_len"]), best)
        if not slow and min_slow[0] < best:
            return None  # deferred to the slow pass
        if limit[0] < best:  # undecided: a rule before the first match hit the limits
            return L.VERDICT_UNSUPPORTED
        if best != KNONE:
            return best
        return L.VERDICT_DENY if h0 else L.VERDICT_ALLOW_NO_L7

    def eval(self, arena: np.ndarray, offsets: np.ndarray) -> np.ndarray:
        buf = arena.tobytes()
        out = np.empty(len(offsets), dtype=np.int32)
        for i, o in enumerate(offsets.tolist()):
            ln = struct.unpack_from("<I", buf, o)[0]
            out[i] = self.eval_record(buf[o:o + ((ln + 3) & ~3)])
        return out
