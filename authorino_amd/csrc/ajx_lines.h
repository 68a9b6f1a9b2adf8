// ajx_lines.h — the line engine: single-pass evaluation of one request per work-item,
// reading the document in 128-byte cache lines.
//
// Per line (one aligned 128-B line of the request's document, loaded as 8 x 16 B):
//   1. the line is written to the work-item's slot of a two-line LDS ring (the line
//      before stays resident, so keys and values that straddle a line boundary are
//      still readable) and the next line's loads are issued;
//   2. SWAR classification of the line in registers: quote and structural-byte planes
//      (128-bit masks); backslash escapes only when the line holds a backslash; the
//      string interior by a prefix-XOR of the unescaped quotes with the carry from the
//      previous line; tokens = structural bytes outside strings + closing quotes;
//   3. one token loop over the whole line: a JSON grammar automaton that follows every
//      selector of the ruleset at once through its trie, the same walk as the exact
//      scan's gjson.Get (first complete match in document order). The per-token step
//      is kept short: only containers on a selector path ("live": their trie node has
//      children) are tracked, each key of a live object is looked up once in the LDS
//      key table, and what the lookup found (child node, its selector, whether it is
//      live) is carried to the value that follows;
//   4. values that complete a selector (and the elements of captured arrays) are
//      queued and evaluated after the line's token loop, straight from the ring:
//      Pattern.Matches (pkg/jsonexp/expressions.go:59-96) for eq/neq/incl/excl against
//      the literal and `matches` on the LDS-resident DFA.
//
// Envelope: compact JSON (Go's encoding/json output, auth_pipeline.go:542-616) with an
// object or array root. Whitespace between tokens, a key with escapes on a selector
// path, nesting deeper than tracked, or anything that is not valid JSON ends the scan
// early: the request goes to the exact scan kernel (ajx_eval_scan), so results never
// depend on which path ran. So does a request with a selected value whose String() the
// engine does not produce (a \u escape outside ASCII, a number that FormatFloat would
// rewrite) or with non-ASCII bytes under `matches`: the engine carries no copy of the
// exact per-value code, which keeps the hot loop small. Values that began before the
// ring's older line are read back from global memory.
#pragma once
#include "ajx_fast.h"

namespace ajx {

constexpr uint32_t kLine = 128;

// queue entry kinds
enum : uint32_t { Q_VALUE = 0, Q_ELEM = 1, Q_ARRAY = 2 };
// String() source of a queued value: S_BYTES the span itself, S_ESC the span unescaped
// (a JSON string interior with escapes), S_TRUE / S_FALSE / S_NULL a literal
enum : uint32_t { S_BYTES = 0, S_TRUE = 1, S_FALSE = 2, S_NULL = 3, S_ESC = 4 };

// what a key lookup found, carried to the value after the key (and what the current
// live container is): node | selector << 8 (0xFF none) | live << 16 | indexed << 17
constexpr uint32_t kPendNone = 0x0000FFFFu;
AJX_HD uint32_t pend_of(const TrieNode* tn, uint32_t node) {
    if (node == kNoNode) return kPendNone;
    const TrieNode t = tn[node];
    const uint32_t sel = t.selector < 0 ? 0xFFu : (uint32_t)t.selector;
    return node | (sel << 8) | ((t.n_children ? 1u : 0u) << 16) | ((t.flags & 1u) << 17);
}

AJX_HD uint32_t ctz64(uint64_t x) { return (uint32_t)__builtin_ctzll(x); }
AJX_HD uint32_t hibit64(uint64_t x) { return 63u - (uint32_t)__builtin_clzll(x); }
AJX_HD uint64_t below64(uint32_t i) { return i >= 64 ? ~0ull : ((1ull << i) - 1ull); }

AJX_HD uint32_t align_bytes(uint32_t hi, uint32_t lo, uint32_t sh) {  // ({hi,lo} >> 8*sh) low 32
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
#else
    return sh ? (lo >> (8 * sh)) | (hi << (32 - 8 * sh)) : lo;
#endif
}

AJX_HD uint32_t haszero_bytes(uint32_t v) { return (v - 0x01010101u) & ~v & 0x80808080u; }
// 1 when x == y, else 0, computed without a comparison mask (a lane-mask boolean
// would put the flag logic on the scalar unit)
AJX_HD uint32_t eqf(uint32_t x, uint32_t y) {
    const uint32_t z = x ^ y;
    return ((z | (0u - z)) >> 31) ^ 1u;
}
// the low min(max(n, 0), 4) bytes of a word (n as a signed count)
AJX_HD uint32_t byte_mask(uint32_t n) {
    const int32_t k = (int32_t)n;
    return k >= 4 ? 0xFFFFFFFFu : k <= 0 ? 0u : (1u << (8u * (uint32_t)k)) - 1u;
}
// 0x80 in every byte that is not an ASCII digit
AJX_HD uint32_t non_digits(uint32_t w) {
    const uint32_t d = w ^ 0x30303030u;
    return ((d + 0x76767676u) | d) & 0x80808080u;
}

// the two-line ring of one work-item: line l lives in slot l & 1; chunk j (16 B) of a
// slot at ((slot * 8 + j) * lanes + lane) * 16, so a wave's 16-B accesses to one chunk
// index are contiguous (conflict-free ds_read_b128 / ds_write_b128)
struct Ring {
    uint8_t* base;    // LDS base of the wave's ring
    uint32_t lane16;  // lane * 16
    uint32_t cstride; // lanes * 16
    AJX_HD uint32_t off(uint32_t a) const { return ((a >> 4) & 15u) * cstride + lane16 + (a & 15u); }
    AJX_HD uint32_t u8(uint32_t a) const { return base[off(a)]; }
    AJX_HD uint32_t u32a(uint32_t a) const { return *reinterpret_cast<const uint32_t*>(base + off(a)); }  // a % 4 == 0
    AJX_HD uint32_t u32(uint32_t a) const {
        const uint32_t b = a & ~3u;
        return align_bytes(u32a(b + 4), u32a(b), a & 3u);
    }
    AJX_HD void put_line(uint32_t line, const Block16* r) {
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
#if defined(__HIP_DEVICE_COMPILE__)
            uint4* p = reinterpret_cast<uint4*>(base + (((line & 1u) * 8u + j) * cstride + lane16));
            *p = uint4{r[j].x, r[j].y, r[j].z, r[j].w};  // 16-B aligned: ds_write_b128
#else
            *reinterpret_cast<Block16*>(base + (((line & 1u) * 8u + j) * cstride + lane16)) = r[j];
#endif
        }
    }
};

AJX_HD uint32_t lds_u32(const uint8_t* p) {  // unaligned dword from a blob (LDS or global)
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);
    return align_bytes(q[1], q[0], sh);
}

struct LineScan {
    // ruleset tables (LDS copy of the blob when the batch shares one ruleset)
    const uint8_t* blob;
    const TrieNode* tn;
    const KeySlot* ks;
    const SelectorPatterns* sps;
    const uint16_t* plist;
    const Pattern* pats;
    const uint8_t* lits;
    uint32_t ks_log2;
    // request
    Ring ring;
    const uint8_t* d;  // document (global memory), d[k] = doc byte k
    uint32_t mis;      // document start within its first line; abs position = doc position + mis
    uint32_t end;      // abs end of the document
    uint32_t line;     // current line
    // classification carries
    uint32_t in_str, esc;
    uint32_t last_bs;       // abs position of the last backslash before the line (~0u none)
    uint64_t bs_lo, bs_hi;  // current line's backslashes
    uint64_t tk_lo, tk_hi;  // current line's tokens
    // grammar
    uint32_t st, depth, pp, bad;  // bad: sticky, the request goes to the exact scan
    uint32_t nbyte;               // the byte after pp (0x100: not known, read it from the ring)
    uint32_t is_arr;              // bit d: the container at depth d is an array (depth <= 31)
    // live containers: depths 1..ld are on selector paths; cur = pend_of(the one at
    // depth ld), stack = trie nodes of depths 1..ld-1 (8 bits each); pend = what the
    // last key's lookup found
    uint32_t ld, cur, pend;
    uint64_t stack, found;
    uint32_t arrn;        // element index in the current live indexed array (depth ld)
    uint32_t idx_bits;    // bit d: the live container at depth d is an array with index children
    uint64_t arrn_stack;  // element indexes of the enclosing live containers (8 bits each)
    uint32_t cap0, cap0_start, cap1, cap1_start, ncap;  // open container captures: sel | depth << 8
    uint32_t cap0_el, cap1_el;  // start of the current element of an open array capture
    // results
    uint64_t t0, t1, hit0, hit1;
    // per-line value queue, evaluated after the line's token loop:
    // a = abs start | kind << 24 | src << 26, b = len | sel << 24
    uint32_t qn, qa0, qb0, qa1, qb1, qa2, qb2, qa3, qb3, qa4, qb4, qa5, qb5, qa6, qb6, qa7, qb7;

    AJX_HD void init(const uint8_t* blob_, const uint8_t* doc, uint32_t n, uint32_t mis_) {
        blob = blob_;
        const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
        tn = reinterpret_cast<const TrieNode*>(blob + h->off_trie_nodes);
        ks = reinterpret_cast<const KeySlot*>(blob + h->off_key_slots);
        sps = reinterpret_cast<const SelectorPatterns*>(blob + h->off_sel_patterns);
        plist = reinterpret_cast<const uint16_t*>(blob + h->off_pattern_lists);
        pats = reinterpret_cast<const Pattern*>(blob + h->off_patterns);
        lits = blob + h->off_literals;
        ks_log2 = h->key_slots_log2;
        d = doc;
        mis = mis_;
        end = mis_ + n;
        line = 0;
        in_str = esc = 0;
        last_bs = ~0u;
        bs_lo = bs_hi = tk_lo = tk_hi = 0;
        st = X_ROOT;
        bad = 0;
        depth = 0;
        pp = mis_ - 1;  // the root container must be the first byte
        nbyte = 0x100u;
        is_arr = 0;
        ld = 0;
        cur = kPendNone;
        pend = pend_of(tn, 0);  // the root value is the trie root
        stack = 0;
        found = 0;
        arrn = 0;
        idx_bits = 0;
        arrn_stack = 0;
        cap0 = cap0_start = cap1 = cap1_start = ncap = 0;
        cap0_el = cap1_el = 0;
        t0 = t1 = hit0 = hit1 = 0;
        qn = qa0 = qb0 = qa1 = qb1 = qa2 = qb2 = qa3 = qb3 = qa4 = qb4 = qa5 = qb5 = qa6 = qb6 = qa7 = qb7 = 0;
    }

    // ---- byte access ----------------------------------------------------------------
    // a span that began before the ring's older line is no longer readable
    AJX_HD bool older(uint32_t a0) const { return a0 < (line ? (line - 1) * kLine : 0u); }
    AJX_HD uint32_t doc_u32(uint32_t a, bool) const { return ring.u32(a); }

    // ---- values ---------------------------------------------------------------------
    AJX_HD void push(uint32_t qa, uint32_t qb) {  // room: the token loop flushes at qn > 6
        const uint32_t k = qn;
        qa0 = k == 0 ? qa : qa0;
        qb0 = k == 0 ? qb : qb0;
        qa1 = k == 1 ? qa : qa1;
        qb1 = k == 1 ? qb : qb1;
        qa2 = k == 2 ? qa : qa2;
        qb2 = k == 2 ? qb : qb2;
        qa3 = k == 3 ? qa : qa3;
        qb3 = k == 3 ? qb : qb3;
        qa4 = k == 4 ? qa : qa4;
        qb4 = k == 4 ? qb : qb4;
        qa5 = k == 5 ? qa : qa5;
        qb5 = k == 5 ? qb : qb5;
        qa6 = k == 6 ? qa : qa6;
        qb6 = k == 6 ? qb : qb6;
        qa7 = k == 7 ? qa : qa7;
        qb7 = k == 7 ? qb : qb7;
        qn = k + 1;
    }
    // a value of selector s (or an element of its captured array) completed;
    // src S_BYTES / S_ESC: String() from abs bytes [a0, a1)
    AJX_HD void value(uint32_t kind, uint32_t s, uint32_t src, uint32_t a0, uint32_t a1) {
#ifdef AJX_ABLATE_NO_VALUES
        return;
#endif
        bad |= older(a0) ? 1u : 0u;  // a value longer than the ring holds: exact scan
        push(a0 | (kind << 24) | (src << 26), ((a1 - a0) & 0xFFFFFFu) | (s << 24));
    }

    // [a0, a0 + len) == the dword-aligned bytes at l, 16 B a step
    AJX_HD bool span_equals(uint32_t a0, uint32_t len, const uint8_t* l) const {
        const bool old = older(a0);
        for (uint32_t k = 0; k < len; k += 16) {
            uint32_t x = 0;
#pragma unroll
            for (uint32_t j = 0; j < 16; j += 4) {
                const uint32_t m =
                    k + j >= len ? 0u : len - k - j >= 4 ? 0xFFFFFFFFu : (1u << (8 * (len - k - j))) - 1u;
                x |= (doc_u32(a0 + k + j, old) ^ *reinterpret_cast<const uint32_t*>(l + k + j)) & m;
            }
            if (x) return false;
        }
        return true;
    }
    // Result.String() of an escaped string (gjson unescape, the StrSrc S_UNESC rules of
    // ajx_device.h) one byte at a time over the interior [*a, end): the byte, -1 at the
    // end, -2 for what the line engine leaves to the exact scan (a control byte, an
    // invalid escape, a \u escape outside ASCII)
    AJX_HD int unesc_next(uint32_t* a, uint32_t end_, bool old) const {
        if (*a >= end_) return -1;
        const uint32_t w = doc_u32(*a, old);
        const uint32_t c = w & 0xFFu;
        if (c < 0x20) return -2;
        if (c != '\\') { *a += 1; return (int)c; }
        if (*a + 1 >= end_) return -2;
        const uint32_t e = (w >> 8) & 0xFFu;
        int out;
        switch (e) {
            case '\\': out = '\\'; break;
            case '/': out = '/'; break;
            case '"': out = '"'; break;
            case 'b': out = '\b'; break;
            case 'f': out = '\f'; break;
            case 'n': out = '\n'; break;
            case 'r': out = '\r'; break;
            case 't': out = '\t'; break;
            case 'u': {
                if (*a + 6 > end_) return -2;
                const uint32_t hx = doc_u32(*a + 2, old);
                uint32_t v = 0;
                for (int k = 0; k < 4; k++) {
                    const uint32_t h = (hx >> (8 * k)) & 0xFFu;
                    uint32_t x;
                    if (h >= '0' && h <= '9') x = h - '0';
                    else if ((h | 0x20) >= 'a' && (h | 0x20) <= 'f') x = (h | 0x20) - 'a' + 10;
                    else return -2;
                    v = v * 16 + x;
                }
                if (v >= 0x80) return -2;
                *a += 6;
                return (int)v;
            }
            default: return -2;
        }
        *a += 2;
        return out;
    }
    // unescaped interior == literal: 1 / 0, or -1 (exact scan)
    AJX_HD int esc_equals(uint32_t a0, uint32_t len, const Pattern& pt) const {
        const uint8_t* l = lits + pt.lit_off;
        const bool old = older(a0);
        uint32_t a = a0, k = 0;
        bool eq = true;
        for (;;) {
            const int c = unesc_next(&a, a0 + len, old);
            if (c == -2) return -1;  // (even after a mismatch: the exact scan decides)
            if (c == -1) return (eq && k == pt.lit_len) ? 1 : 0;
            eq = eq && k < pt.lit_len && (uint32_t)c == l[k];
            k++;
        }
    }
    AJX_HD bool str_equals(uint32_t src, uint32_t a0, uint32_t len, const Pattern& pt) {
        if (src == S_BYTES) return len == pt.lit_len && span_equals(a0, len, lits + pt.lit_off);
#ifndef AJX_ABLATE_NO_ESC_DFA
        if (src == S_ESC) {
            const int r = esc_equals(a0, len, pt);
            if (r < 0) bad = 1;
            return r == 1;
        }
#endif
        const uint32_t f = src == S_TRUE ? kLitTrue : src == S_FALSE ? kLitFalse : kLitEmpty;
        return (pt.litf & f) != 0;
    }
    // Go regexp DFA over ASCII bytes; returns 0/1, or 2 when a byte >= 0x80 needs rune
    // decoding (the exact scan then evaluates the request)
    AJX_HD uint32_t dfa_span(uint32_t dfa_off, uint32_t a0, uint32_t len, bool esc_) const {
        const DfaHdr* h = reinterpret_cast<const DfaHdr*>(blob + dfa_off);
        const uint16_t* tr = reinterpret_cast<const uint16_t*>(blob + h->trans_off);
        const uint32_t nc = h->n_classes, ms = h->match_state;
        uint32_t st_ = h->start;
        if (st_ == ms) return 1;
        const bool old = older(a0);
        if (esc_) {
            uint32_t a = a0;
            for (;;) {
                const int b = unesc_next(&a, a0 + len, old);
                if (b == -1) break;
                if (b < 0 || b >= 0x80) return 2;
                st_ = tr[st_ * nc + h->ascii_class[b]];
                if (st_ == ms) return 1;
            }
            return blob[h->eot_off + st_] != 0;
        }
        for (uint32_t k = 0; k < len; k += 4) {
            const uint32_t w = doc_u32(a0 + k, old);
            const uint32_t m = len - k >= 4 ? 4u : len - k;
            for (uint32_t j = 0; j < m; j++) {
                const uint32_t b = (w >> (8 * j)) & 0xFFu;
                if (b >= 0x80) return 2;
                st_ = tr[st_ * nc + h->ascii_class[b]];
                if (st_ == ms) return 1;
            }
        }
        return blob[h->eot_off + st_] != 0;
    }

    // (both members written unconditionally: a store into one of two sibling members
    // chosen by a branch becomes a store through a selected address, which puts the
    // whole scanner state in scratch memory)
    AJX_HD void set_t(uint32_t p, bool v) {
        const uint64_t bit = 1ull << (p & 63);
        const uint64_t m0 = p < 64 ? bit : 0ull, m1 = p < 64 ? 0ull : bit;
        const uint64_t a = t0, b = t1;
        t0 = v ? a | m0 : a & ~m0;
        t1 = v ? b | m1 : b & ~m1;
    }
    AJX_HD void set_hit(uint32_t p) {
        const uint64_t bit = 1ull << (p & 63);
        const uint64_t a = hit0, b = hit1;
        hit0 = a | (p < 64 ? bit : 0ull);
        hit1 = b | (p < 64 ? 0ull : bit);
    }

    AJX_HD void eval_entry(uint32_t qa, uint32_t qb) {
        const uint32_t a0 = qa & 0xFFFFFFu, kind = (qa >> 24) & 3u, src = qa >> 26;
        const uint32_t len = qb & 0xFFFFFFu, s = qb >> 24;
        const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
        const SelectorPatterns sp = sps[s];
        if (kind == Q_VALUE && src == S_NULL) {  // a JSON null: String() "" and Array() [] as for Null
            t0 |= sp.mask[0] & h->null_true[0];
            t1 |= sp.mask[1] & h->null_true[1];
            return;
        }
#ifdef AJX_ABLATE_NO_EVAL
        for (uint32_t j = 0; j < sp.count; j++) set_t(plist[sp.begin + j], len > 3);
        return;
#endif
        for (uint32_t j = 0; j < sp.count; j++) {
            const uint32_t p = plist[sp.begin + j];
            const Pattern pt = pats[p];
            const uint64_t bit = 1ull << (p & 63);
            if (kind == Q_ELEM) {
                if ((pt.op == OP_INCL || pt.op == OP_EXCL) && str_equals(src, a0, len, pt)) set_hit(p);
                continue;
            }
            bool r;
            if (pt.op == OP_MATCHES) {
#ifdef AJX_ABLATE_NO_ESC_DFA
                bad = 1;
                return;
#endif
                const uint32_t m =
                    (src == S_BYTES || src == S_ESC) ? dfa_span(pt.dfa_off, a0, len, src == S_ESC) : 2u;
                if (m == 2) {  // true / false or non-ASCII bytes under a regex: exact scan
                    bad = 1;
                    return;
                }
                r = m != 0;
            } else if (kind == Q_ARRAY && (pt.op == OP_INCL || pt.op == OP_EXCL)) {
                const bool hit = ((p < 64 ? hit0 : hit1) & bit) != 0;
                r = hit == (pt.op == OP_INCL);
            } else {
                const bool eq = str_equals(src, a0, len, pt);
                r = eq == (pt.op == OP_EQ || pt.op == OP_INCL);
            }
            set_t(p, r);
        }
    }
    AJX_HD void flush() {
        for (uint32_t k = 0; k < qn && !bad; k++) {
            const uint32_t qa = k == 0 ? qa0 : k == 1 ? qa1 : k == 2 ? qa2 : k == 3 ? qa3 : k == 4 ? qa4 : k == 5 ? qa5 : k == 6 ? qa6 : qa7;
            const uint32_t qb = k == 0 ? qb0 : k == 1 ? qb1 : k == 2 ? qb2 : k == 3 ? qb3 : k == 4 ? qb4 : k == 5 ? qb5 : k == 6 ? qb6 : qb7;
            eval_entry(qa, qb);
        }
        qn = 0;
    }

    // ---- structure --------------------------------------------------------------------
    AJX_HD bool top_is_arr() const { return (is_arr >> depth) & 1u; }
    // selector of the open array capture whose direct element is a value completing at
    // the current depth (-1 none)
    AJX_HD int32_t elem_cap() const {
        if (!ncap || !top_is_arr()) return -1;
        const uint32_t c = ncap == 2 ? cap1 : cap0;
        return (c >> 8) == depth ? (int32_t)(c & 0xFF) : -1;
    }
    // what the value starting now is on the trie: after a key, what its lookup found;
    // in a live indexed array, the child for the element index
    AJX_HD uint32_t value_pend() const {
        if (!top_is_arr()) return (depth == 0 || depth == ld) ? pend : kPendNone;
        if (depth != ld || !(cur & (1u << 17))) return kPendNone;
        const TrieChild* tc = reinterpret_cast<const TrieChild*>(
            blob + reinterpret_cast<const RulesetHdr*>(blob)->off_trie_children);
        const uint32_t node = cur & 0xFFu;
        const uint32_t cb = tn[node].child_begin, nc = tn[node].n_children;
        for (uint32_t c = 0; c < nc; c++)
            if (tc[cb + c].array_index == (int32_t)arrn) return pend_of(tn, tc[cb + c].node);
        return kPendNone;
    }
    // the selector a value completes (-1 none): a leaf not matched before (first match
    // in document order wins)
    AJX_HD int32_t leaf(uint32_t pv) const {
        const uint32_t s = (pv >> 8) & 0xFFu;
        if (s == 0xFFu || ((found >> s) & 1)) return -1;
        return (int32_t)s;
    }
    AJX_HD void element_done() {  // a value completed at the current depth
        if (depth == ld && top_is_arr() && (cur & (1u << 17))) arrn++;
    }
    AJX_HD bool escaped_between(uint32_t o, uint32_t i) const {
        const uint64_t ml = bs_lo & below64(i), mh = i > 64 ? bs_hi & below64(i - 64) : 0ull;
        const uint32_t base = line * kLine;
        const uint32_t lb = mh ? base + 64 + hibit64(mh) : ml ? base + hibit64(ml) : last_bs;
        return lb != ~0u && lb > o;
    }
    // a key of a live object: [o + 1, a) with its quotes at o and a, line index i
    AJX_HD void key(uint32_t o, uint32_t a, uint32_t i, uint64_t before8) {
        pend = kPendNone;
#ifdef AJX_ABLATE_NO_KEYS
        return;
#endif
        if (escaped_between(o, i)) { st = X_SLOW; return; }  // escaped key on a live path
        const uint32_t parent = cur & 0xFFu;
        const uint32_t klen = a - o - 1;
        uint64_t sig;
        {
            const uint32_t have = a >= 8 ? 8u : a;  // bytes of before8 before the quote (fewer at the doc start)
            sig = have < 8 ? before8 << (8 * (8 - have)) : before8;
            if (klen < 8) sig = klen ? sig >> (8 * (8 - klen)) : 0ull;
        }
        const uint32_t want = (klen & 0xFFFFu) | (parent << 16), mask = (1u << ks_log2) - 1u;
        uint32_t at = key_slot_hash(sig, klen, parent, ks_log2);
        for (uint32_t probe = 0; probe <= mask; probe++, at = (at + 1) & mask) {
            const KeySlot slot = ks[at];
            if (slot.meta == kEmptySlot) return;
            if (slot.sig != sig || (slot.meta & 0xFFFFFFu) != want || klen > 0xFFFFu) continue;
            if (klen > 8) {
                if (older(o + 1)) { st = X_SLOW; return; }
                if (!span_equals(o + 1, klen - 8, lits + slot.key_off)) continue;
            }
            pend = pend_of(tn, slot.meta >> 24);
            return;
        }
    }
    // Result.String() of a number is its raw text when the raw text is -?[0-9]*
    // (gjson Result.String, string_of in ajx_device.h), or when the raw text already is
    // what strconv.FormatFloat(f, 'f', -1, 64) prints for it: -?(0|[1-9][0-9]*).[0-9]*[1-9]
    // with at most 15 significant digits and at most 24 bytes (such a decimal round-trips
    // through a normal float64, so no shorter decimal maps to the same value)
    AJX_HD bool number_is_canonical(uint32_t a0, uint32_t g, uint32_t c0) const {
        uint32_t dot = 0, nsig = 0, int_digits = 0, first = 0, lastc = 0;
        bool digits = true, lead = true;
        for (uint32_t j = c0 == '-' ? 1u : 0u; j < g; j++) {
            const uint32_t c = ring.u8(a0 + j);
            if (c == '.') {
                if (dot) { digits = false; break; }
                dot = 1;
                lastc = c;
                continue;
            }
            if (c < '0' || c > '9') { digits = false; break; }
            if (!dot) {
                if (int_digits == 0) first = c;
                int_digits++;
            }
            if (c != '0') lead = false;
            if (!lead) nsig++;
            lastc = c;
        }
        if (!digits) return false;
        if (!dot) return true;
        return g <= 24 && int_digits >= 1 && !(int_digits > 1 && first == '0') && lastc != '.' && lastc != '0' &&
               nsig <= 15;
    }
    // a scalar in [a0, a1) (abs) in a value position, followed directly by the token
    // at a1; false: not one the fast path accepts
    AJX_HD bool scalar(uint32_t a0, uint32_t a1) {
        const uint32_t g = a1 - a0;
        if (older(a0)) return false;  // longer than the ring holds
        const uint32_t w0 = ring.u32(a0);
        const uint32_t c0 = w0 & 0xFFu, c1 = (w0 >> 8) & 0xFFu;
        uint32_t src = S_BYTES;
        if (c0 == 't') {
            if (g != 4 || w0 != 0x65757274u) return false;
            src = S_TRUE;
        } else if (c0 == 'f') {
            if (g != 5 || w0 != 0x736C6166u || ring.u8(a0 + 4) != 'e') return false;
            src = S_FALSE;
        } else if (c0 == 'n' && c1 == 'u') {
            if (g != 4 || w0 != 0x6C6C756Eu) return false;
            src = S_NULL;
        } else if (!(c0 == '-' || c0 == '+' || (c0 >= '0' && c0 <= '9') || c0 == 'i' || c0 == 'I' || c0 == 'N' ||
                     c0 == 'n')) {
            return false;
        }
        // no whitespace (or control byte) inside the run
        for (uint32_t k = 0; k < g; k += 4) {
            const uint32_t w = ring.u32(a0 + k);
            const uint32_t m = g - k >= 4 ? 0xFFFFFFFFu : (1u << (8 * (g - k))) - 1u;
            if (le20_bytes(w) & m) return false;
        }
        const int32_t s = leaf(value_pend());
        const int32_t ec = elem_cap();
        if (s >= 0 || ec >= 0) {
            if (src == S_BYTES && !number_is_canonical(a0, g, c0)) return false;  // FormatFloat would rewrite it
            if (s >= 0) {
                found |= 1ull << s;
                value(Q_VALUE, (uint32_t)s, src, a0, a1);
            }
            if (ec >= 0) value(Q_ELEM, (uint32_t)ec, src, a0, a1);
        }
        element_done();
        return true;
    }
    // a string value closing at abs a (interior [o + 1, a)), line index i
    AJX_HD void string_value(uint32_t o, uint32_t a, uint32_t i) {
        const int32_t s = leaf(value_pend());
        const int32_t ec = elem_cap();
        if (s >= 0 || ec >= 0) {
            const uint32_t src = escaped_between(o, i) ? S_ESC : S_BYTES;
            if (s >= 0) {
                found |= 1ull << s;
                value(Q_VALUE, (uint32_t)s, src, o + 1, a);
            }
            if (ec >= 0) value(Q_ELEM, (uint32_t)ec, src, o + 1, a);
        }
        element_done();
    }
    AJX_HD bool open_container(bool arr, uint32_t a) {
        const uint32_t pv = value_pend();
        const int32_t s = leaf(pv);
        if (depth + 1 >= 32) return false;
        if (elem_cap() >= 0) {  // this container is an element of the innermost array capture
            const uint32_t e0 = cap0_el, e1 = cap1_el;
            cap0_el = ncap == 1 ? a : e0;
            cap1_el = ncap == 2 ? a : e1;
        }
        if ((pv >> 16) & 1u) {  // a live child: the new container is on a selector path
            if (ld >= kLinesMaxDepth || arrn > 0xFFu) return false;
            if (ld) {
                const uint32_t sh = 8 * (ld - 1);
                stack = (stack & ~(0xFFull << sh)) | ((uint64_t)(cur & 0xFFu) << sh);
                arrn_stack = (arrn_stack & ~(0xFFull << sh)) | ((uint64_t)arrn << sh);
            }
            ld = depth + 1;
            cur = pv;
            arrn = 0;
            const uint32_t bit = 1u << (depth + 1);
            idx_bits = (arr && (pv & (1u << 17))) ? idx_bits | bit : idx_bits & ~bit;
        }
        depth++;
        is_arr = arr ? is_arr | (1u << depth) : is_arr & ~(1u << depth);
        if (s >= 0) {
            found |= 1ull << s;
            if (ncap >= 2) return false;
            const uint32_t v = (uint32_t)s | (depth << 8), c0 = cap0, c1 = cap1, s0 = cap0_start, s1 = cap1_start;
            cap0 = ncap == 0 ? v : c0;
            cap0_start = ncap == 0 ? a : s0;
            cap1 = ncap == 1 ? v : c1;
            cap1_start = ncap == 1 ? a : s1;
            ncap++;
            const SelectorPatterns sp = sps[s];
            hit0 &= ~sp.mask[0];
            hit1 &= ~sp.mask[1];
        }
        return true;
    }
    AJX_HD void close_container(uint32_t a) {
        if (ncap) {
            const uint32_t cs = ncap == 2 ? cap1 : cap0;
            if ((cs >> 8) == depth) {
                const uint32_t start = ncap == 2 ? cap1_start : cap0_start;
                ncap--;
                value(top_is_arr() ? Q_ARRAY : Q_VALUE, cs & 0xFFu, S_BYTES, start, a + 1);
            }
        }
        if (depth == ld) {  // leaving a live container (its parent, if live, is at depth - 1)
            idx_bits &= ~(1u << depth);
            ld--;
            if (ld) {
                const uint32_t sh = 8 * (ld - 1);
                cur = pend_of(tn, (uint32_t)((stack >> sh) & 0xFFu));
                arrn = (uint32_t)((arrn_stack >> sh) & 0xFFu);
            } else {
                cur = kPendNone;
            }
        }
        depth--;
        // this container was an element of a captured array: its raw text
        const int32_t ec = elem_cap();
        if (ec >= 0) value(Q_ELEM, (uint32_t)ec, S_BYTES, ncap == 2 ? cap1_el : cap0_el, a + 1);
        element_done();
    }

    // classify line `line` (8 blocks in registers): token planes for token_loop()
    AJX_HD void classify(const Block16* r) {
        const uint32_t base = line * kLine;
        if (nbyte == 0x100u && pp + 1 == base) nbyte = r[0].x & 0xFFu;  // the previous token ended the line
        // valid bytes of the line
        uint64_t v_lo = ~0ull, v_hi = ~0ull;
        if (base < mis) {
            const uint32_t k = mis - base;  // < 128
            v_lo = k >= 64 ? 0ull : v_lo << k;
            v_hi = k > 64 ? v_hi << (k - 64) : v_hi;
        }
        if (base + kLine > end) {
            const uint32_t k = end - base;  // valid count, 1..127
            v_lo &= below64(k);
            v_hi &= k > 64 ? below64(k - 64) : 0ull;
        }
        uint64_t q_lo = 0, q_hi = 0, s_lo = 0, s_hi = 0;
        uint32_t bsany = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            uint32_t q16 = 0, s16 = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t x = k == 0 ? r[j].x : k == 1 ? r[j].y : k == 2 ? r[j].z : r[j].w;
                const uint32_t lx = x | 0x20202020u;
                q16 |= gather4(eq_bytes(x, 0x22222222u)) << (4 * k);
                s16 |= gather4(eq_bytes(lx, 0x7B7B7B7Bu) | eq_bytes(lx, 0x7D7D7D7Du) | eq_bytes(x, 0x3A3A3A3Au) |
                               eq_bytes(x, 0x2C2C2C2Cu))
                       << (4 * k);
                bsany |= haszero_bytes(x ^ 0x5C5C5C5Cu);
            }
            if (j < 4) {
                q_lo |= (uint64_t)q16 << (16 * j);
                s_lo |= (uint64_t)s16 << (16 * j);
            } else {
                q_hi |= (uint64_t)q16 << (16 * (j - 4));
                s_hi |= (uint64_t)s16 << (16 * (j - 4));
            }
        }
        q_lo &= v_lo;
        q_hi &= v_hi;
        s_lo &= v_lo;
        s_hi &= v_hi;
        uint64_t e_lo = 0, e_hi = 0;  // escaped bytes
        bs_lo = bs_hi = 0;
        if (bsany || esc) {
            // backslash planes, then the bytes escaped by odd backslash runs (carry esc)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                uint32_t b16 = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t x = k == 0 ? r[j].x : k == 1 ? r[j].y : k == 2 ? r[j].z : r[j].w;
                    b16 |= gather4(eq_bytes(x, 0x5C5C5C5Cu)) << (4 * k);
                }
                if (j < 4) bs_lo |= (uint64_t)b16 << (16 * j);
                else bs_hi |= (uint64_t)b16 << (16 * (j - 4));
            }
            bs_lo &= v_lo;
            bs_hi &= v_hi;
            // the branch-free odd-run rule on each 64-bit half
            {
                const uint64_t bs = bs_lo & ~(uint64_t)esc;
                const uint64_t follows = (bs << 1) | esc;
                const uint64_t even = 0x5555555555555555ull;
                const uint64_t odd_starts = bs & ~even & ~follows;
                const uint64_t seq = odd_starts + bs;
                const uint32_t carry = seq < bs ? 1u : 0u;
                e_lo = (even ^ (seq << 1)) & follows;
                esc = carry;
            }
            {
                const uint64_t bs = bs_hi & ~(uint64_t)esc;
                const uint64_t follows = (bs << 1) | esc;
                const uint64_t even = 0x5555555555555555ull;
                const uint64_t odd_starts = bs & ~even & ~follows;
                const uint64_t seq = odd_starts + bs;
                const uint32_t carry = seq < bs ? 1u : 0u;
                e_hi = (even ^ (seq << 1)) & follows;
                esc = carry;
            }
        }
        const uint64_t qu_lo = q_lo & ~e_lo, qu_hi = q_hi & ~e_hi;
        uint64_t x_lo = qu_lo, x_hi = qu_hi;
        x_lo ^= x_lo << 1; x_hi ^= x_hi << 1;
        x_lo ^= x_lo << 2; x_hi ^= x_hi << 2;
        x_lo ^= x_lo << 4; x_hi ^= x_hi << 4;
        x_lo ^= x_lo << 8; x_hi ^= x_hi << 8;
        x_lo ^= x_lo << 16; x_hi ^= x_hi << 16;
        x_lo ^= x_lo << 32; x_hi ^= x_hi << 32;
        if (in_str) x_lo = ~x_lo;
        if (x_lo >> 63) x_hi = ~x_hi;
        in_str = (uint32_t)(x_hi >> 63);
        const uint64_t out_lo = ~x_lo & ~qu_lo & v_lo, out_hi = ~x_hi & ~qu_hi & v_hi;
        tk_lo = (s_lo & out_lo) | (qu_lo & ~x_lo);
        tk_hi = (s_hi & out_hi) | (qu_hi & ~x_hi);
        if ((bs_lo & out_lo) | (bs_hi & out_hi)) st = X_SLOW;  // a backslash outside any string
    }

    // the grammar / selector walk over the current line's tokens, then its values
    AJX_HD void token_loop() {
        const uint32_t base = line * kLine;
        uint64_t tk_lo = this->tk_lo, tk_hi = this->tk_hi;
#ifdef AJX_ABLATE_WALK_ONLY
        {  // profiling: iterate the tokens, read each byte, nothing else
            uint32_t acc = 0;
            while (tk_lo | tk_hi) {
                const uint32_t i = tk_lo ? ctz64(tk_lo) : 64 + ctz64(tk_hi);
                if (i < 64) tk_lo &= tk_lo - 1;
                else tk_hi &= tk_hi - 1;
                acc += ring.u32(base + i);
            }
            pp ^= acc;
            if (line * kLine + kLine >= end) st = X_DONE;
            return;
        }
#endif
        // software-pipelined: the words of the next two tokens are read from the ring
        // while the current one is processed (the next token is one of them, depending
        // on whether the current token takes the ':' / ',' after it)
        bool have = (tk_lo | tk_hi) != 0;
        uint32_t i = tk_lo ? ctz64(tk_lo) : tk_hi ? 64 + ctz64(tk_hi) : 0u;
        if (i < 64) tk_lo &= tk_lo - 1;
        else tk_hi &= tk_hi - 1;
        uint32_t w = ring.u32(base + i);  // the token byte and the bytes after it
        while (have && st < X_DONE && !bad) {
            if (qn > 6) flush();  // (rare) a token queues at most two values
            const uint32_t a = base + i;
            const uint32_t n1 = tk_lo ? ctz64(tk_lo) : tk_hi ? 64 + ctz64(tk_hi) : 128u;
            uint32_t n2 = 128u;
            {
                const uint64_t l2 = n1 < 64 ? tk_lo & (tk_lo - 1) : tk_lo;
                const uint64_t h2 = n1 >= 64 && n1 < 128 ? tk_hi & (tk_hi - 1) : tk_hi;
                n2 = l2 ? ctz64(l2) : h2 ? 64 + ctz64(h2) : 128u;
            }
            const uint32_t w1 = ring.u32(base + (n1 & 127u)), w2 = ring.u32(base + (n2 & 127u));
            // the 8 bytes before the token (a key's signature)
            const uint32_t sx = a >= 8 ? a - 8 : 0u;
            const uint64_t before8 = (uint64_t)ring.u32(sx) | ((uint64_t)ring.u32(sx + 4) << 32);
            // the first 8 bytes after the previous token (a scalar's text)
            const uint32_t sw0 = ring.u32(pp + 1u), sw1 = ring.u32(pp + 5u);
            const uint32_t sw2 = ring.u32(pp + 9u), sw3 = ring.u32(pp + 13u);
            const uint32_t c = w & 0xFFu;
            // ---- the grammar on 0/1 integer flags (vector ALU; boolean && / || on lane
            // masks would run on the compute unit's one scalar ALU) ----
            const uint32_t cl = c | 0x20u;
            const uint32_t f_q = eqf(c, 0x22u), f_open = eqf(cl, 0x7Bu), f_close = eqf(cl, 0x7Du);
            const uint32_t f_colon = eqf(c, 0x3Au), f_comma = eqf(c, 0x2Cu);
            const uint32_t f_barr = ((c >> 5) & 1u) ^ 1u;  // '[' or ']'
            const uint32_t arr = (is_arr >> depth) & 1u;
            const uint32_t f_gap = (f_q ^ 1u) & (eqf(a, pp + 1) ^ 1u);  // a scalar before this token
            const uint32_t st1 = f_gap ? (uint32_t)X_COMMA_OR_CLOSE : st;
            const uint32_t in_val = (0x6u >> st1) & 1u, in_key = (0x18u >> st1) & 1u;  // {VALUE, VALUE_OR_CLOSE}, {KEY_OR_CLOSE, KEY}
            const uint32_t gap_ok = (f_gap ^ 1u) | (((0x6u >> st) & 1u) & (f_comma | f_close));
            const uint32_t f_ob = eqf(nbyte, 0x22u);  // compact JSON: a string opens right after the previous token
            const uint32_t key_ok = f_q & in_key & f_ob;
            const uint32_t sval_ok = f_q & in_val & f_ob;
            const uint32_t open_ok = f_open & ((0x7u >> st1) & 1u);  // {ROOT, VALUE, VALUE_OR_CLOSE}
            const uint32_t coc = eqf(st1, X_COMMA_OR_CLOSE);
            const uint32_t close_ok = f_close & ((eqf(st1, X_VALUE_OR_CLOSE) & f_barr) |
                                                 (eqf(st1, X_KEY_OR_CLOSE) & (f_barr ^ 1u)) | (coc & (arr ^ f_barr ^ 1u)));
            const uint32_t colon_ok = f_colon & eqf(st1, X_COLON);
            const uint32_t comma_ok = f_comma & coc;
            const uint32_t ok = gap_ok & (key_ok | sval_ok | open_ok | close_ok | colon_ok | comma_ok);
            const uint32_t live_here = eqf(depth, ld);  // the current container is on a selector path
            const uint32_t pv = (live_here & (arr ^ 1u)) ? pend : kPendNone;  // (indexed arrays are rare)
            const uint32_t pv_sel = (pv >> 8) & 0xFFu;
            const uint32_t pv_leaf = (eqf(pv_sel, 0xFFu) ^ 1u) & ((uint32_t)(found >> (pv_sel & 63u)) ^ 1u) & 1u;
            // the live container is an indexed array whose elements this token touches
            const uint32_t idx_arr = (cur >> 17) & (is_arr >> ld) & 1u;
            // ---- a scalar in [pp + 1, a) (f_gap): the fast path takes runs of up to 16 bytes ----
            const uint32_t g = a - pp - 1u;
            const uint32_t c0 = sw0 & 0xFFu, c1 = (sw0 >> 8) & 0xFFu;
            const uint32_t lit_t = eqf(c0, 't') & eqf(g, 4u) & eqf(sw0, 0x65757274u);
            const uint32_t lit_f = eqf(c0, 'f') & eqf(g, 5u) & eqf(sw0, 0x736C6166u) & eqf(sw1 & 0xFFu, 'e');
            const uint32_t nu = eqf(c0, 'n') & eqf(c1, 'u');
            const uint32_t lit_n = nu & eqf(g, 4u) & eqf(sw0, 0x6C6C756Eu);
            const uint32_t is_lit = lit_t | lit_f | lit_n;
            const uint32_t lit_start = eqf(c0, 't') | eqf(c0, 'f') | nu;  // must then be exactly the literal
            const uint32_t digit0 = ((9u - (c0 ^ 0x30u)) >> 31) ^ 1u;
            const uint32_t num_start = digit0 | eqf(c0, '-') | eqf(c0, '+') | eqf(c0, 'i') | eqf(c0, 'I') | eqf(c0, 'N') |
                                       (eqf(c0, 'n') & (nu ^ 1u));  // gjson parseNumber's first bytes
            const uint32_t m0 = byte_mask(g), m1 = byte_mask(g - 4u), m2 = byte_mask(g - 8u), m3 = byte_mask(g - 12u);
            const uint32_t ws = (le20_bytes(sw0) & m0) | (le20_bytes(sw1) & m1) | (le20_bytes(sw2) & m2) |
                                (le20_bytes(sw3) & m3);  // whitespace inside the run
            const uint32_t sc_ok = ((16u - g) >> 31 ^ 1u) & (lit_start ? is_lit : num_start) & eqf(ws, 0u);
            // Result.String() is the raw text: a literal, or -?[0-9]* (longer forms: general path)
            const uint32_t neg = eqf(c0, '-');
            const uint32_t nd = (non_digits(sw0) & m0 & (neg ? 0xFFFFFF00u : 0xFFFFFFFFu)) | (non_digits(sw1) & m1) |
                                (non_digits(sw2) & m2) | (non_digits(sw3) & m3);
            const uint32_t sc_raw = is_lit | eqf(nd, 0u);
            const uint32_t sc_src = lit_t ? (uint32_t)S_TRUE : lit_f ? (uint32_t)S_FALSE : lit_n ? (uint32_t)S_NULL : (uint32_t)S_BYTES;
            // ---- values this token completes ----
            const uint32_t has_cap = (ncap | (ncap >> 1)) & 1u;
            const uint32_t tcap = ncap == 2u ? cap1 : cap0;  // the innermost capture
            const uint32_t tcap_here = has_cap & eqf(tcap >> 8, depth);
            const uint32_t sv = f_gap | sval_ok;  // a scalar / string value ends here
            const uint32_t e_str = sval_ok & (escaped_between(pp + 1u, i) ? 1u : 0u);
            const uint32_t v_src = f_gap ? sc_src : e_str ? (uint32_t)S_ESC : (uint32_t)S_BYTES;
            const uint32_t v_a0 = pp + 1u + sval_ok;  // string interior / scalar start
            const uint32_t vd_leaf = sv & pv_leaf;              // completes selector pv_sel
            const uint32_t v_elem = sv & tcap_here & arr;       // an element of the innermost array capture
            const uint32_t cap_close = close_ok & tcap_here;    // the closing container is captured
            const uint32_t ncap2 = ncap - cap_close;
            const uint32_t tcap2 = cap_close ? cap0 : tcap;     // the innermost capture once it is closed
            const uint32_t c_elem = close_ok & ((ncap2 | (ncap2 >> 1)) & 1u) & eqf(tcap2 >> 8, depth - 1u) &
                                    (is_arr >> (depth - 1u)) & 1u;  // the closing container was an element
            const uint32_t el_start = (ncap2 == 2u) ? cap1_el : cap0_el;
            const uint32_t o_cap = open_ok & pv_leaf;           // a captured container opens
            const uint32_t o_elem = open_ok & tcap_here & arr;  // an element container of the innermost capture opens
            const uint32_t npush = vd_leaf + v_elem + cap_close + c_elem;
            // rare tokens take the general path
            uint32_t rare =
                ok & (((npush - 1u) >> 31 ^ 1u) & (npush != 1u ? 1u : 0u)  // two values at once
                      | (f_gap & (sc_ok ^ 1u))                                // a long / odd scalar
                      | (f_gap & ((vd_leaf | v_elem) & (sc_raw ^ 1u)))        // a number String() reformats
                      | (idx_arr & live_here) | (close_ok & (idx_bits >> (depth - 1u)) & 1u)
                      | (o_cap & (ncap >> 1)));                               // a third nested capture
#ifdef AJX_LINES_BRANCHY
            rare = ok;  // profiling: every token through the general (branchy) path
#endif
#ifdef AJX_COUNT_RARE
            if (rare) {
                extern uint64_t ajx_rare_counts[8];
                ajx_rare_counts[0]++;
                if ((npush - 1u) < 0x80000000u && npush != 1u) ajx_rare_counts[1]++;
                if (f_gap & (sc_ok ^ 1u)) ajx_rare_counts[2]++;
                if (f_gap & ((vd_leaf | v_elem) & (sc_raw ^ 1u))) ajx_rare_counts[3]++;
                if (idx_arr & live_here) ajx_rare_counts[4]++;
                if (close_ok & (idx_bits >> (depth - 1u)) & 1u) ajx_rare_counts[5]++;
                if (o_cap & (ncap >> 1)) ajx_rare_counts[6]++;
            }
            {
                extern uint64_t ajx_rare_counts[8];
                ajx_rare_counts[7]++;
            }
#endif
            if (rare) {
                if (f_gap) {
                    if (!scalar(pp + 1, a)) st = X_SLOW;
                    else st = X_COMMA_OR_CLOSE;
                }
                if (st != X_SLOW) {
                    if (key_ok) {
                        st = X_COLON;
                        if (live_here) key(pp + 1, a, i, before8);
                        else pend = kPendNone;
                    } else if (sval_ok) {
                        string_value(pp + 1, a, i);
                        st = X_COMMA_OR_CLOSE;
                    } else if (open_ok) {
                        if (!open_container(f_barr != 0, a)) st = X_SLOW;
                        else st = f_barr ? X_VALUE_OR_CLOSE : X_KEY_OR_CLOSE;
                    } else if (close_ok) {
                        close_container(a);
                        st = depth == 0 ? X_DONE : X_COMMA_OR_CLOSE;
                    } else {
                        st = (colon_ok | arr) ? (uint32_t)X_VALUE : (uint32_t)X_KEY;
                    }
                }
            } else {
                // ---- the common step (predicated) ----
                // the one value this token completes, if any
                const uint32_t q_kind = cap_close ? (arr ? (uint32_t)Q_ARRAY : (uint32_t)Q_VALUE)
                                       : (v_elem | c_elem) ? (uint32_t)Q_ELEM : (uint32_t)Q_VALUE;
                const uint32_t q_sel = vd_leaf ? pv_sel : (v_elem | cap_close) ? (tcap & 0xFFu) : (tcap2 & 0xFFu);
                const uint32_t q_src = (vd_leaf | v_elem) ? v_src : (uint32_t)S_BYTES;
                const uint32_t q_a0 = (vd_leaf | v_elem) ? v_a0
                                      : cap_close ? (ncap == 2u ? cap1_start : cap0_start) : el_start;
                const uint32_t q_a1 = (vd_leaf | v_elem) ? a : a + 1u;
                const uint32_t qa = q_a0 | (q_kind << 24) | (q_src << 26);
                const uint32_t qb = ((q_a1 - q_a0) & 0xFFFFFFu) | (q_sel << 24);
                const uint32_t k = npush ? qn : 8u;  // (no value: nothing is stored)
                qa0 = k == 0u ? qa : qa0;
                qb0 = k == 0u ? qb : qb0;
                qa1 = k == 1u ? qa : qa1;
                qb1 = k == 1u ? qb : qb1;
                qa2 = k == 2u ? qa : qa2;
                qb2 = k == 2u ? qb : qb2;
                qa3 = k == 3u ? qa : qa3;
                qb3 = k == 3u ? qb : qb3;
                qa4 = k == 4u ? qa : qa4;
                qb4 = k == 4u ? qb : qb4;
                qa5 = k == 5u ? qa : qa5;
                qb5 = k == 5u ? qb : qb5;
                qa6 = k == 6u ? qa : qa6;
                qb6 = k == 6u ? qb : qb6;
                qn += npush;
                bad |= npush & (older(q_a0) ? 1u : 0u);  // a value longer than the ring holds: exact scan
                // first match in document order: a selector completes once
                found |= (uint64_t)(vd_leaf | o_cap) << (pv_sel & 63u);
                // captures: a captured container opens (its incl/excl hits restart) / closes
                if (o_cap) {
                    const SelectorPatterns sp = sps[pv_sel];
                    hit0 &= ~sp.mask[0];
                    hit1 &= ~sp.mask[1];
                }
                const uint32_t cv = pv_sel | ((depth + 1u) << 8);
                cap0 = (o_cap & eqf(ncap, 0u)) ? cv : cap0;
                cap0_start = (o_cap & eqf(ncap, 0u)) ? a : cap0_start;
                cap1 = (o_cap & eqf(ncap, 1u)) ? cv : cap1;
                cap1_start = (o_cap & eqf(ncap, 1u)) ? a : cap1_start;
                cap0_el = (o_elem & eqf(ncap, 1u)) ? a : cap0_el;
                cap1_el = (o_elem & eqf(ncap, 2u)) ? a : cap1_el;
                ncap = ncap + o_cap - cap_close;
                // the live-container path
                const uint32_t push = open_ok & (pv >> 16) & 1u;
                const uint32_t pop = close_ok & live_here;
                const uint32_t has = eqf(ld, 0u) ^ 1u;  // ld != 0
                bad |= push & ((ld >= kLinesMaxDepth ? 1u : 0u) | (depth + 1 >= 32 ? 1u : 0u) | (arrn > 0xFFu ? 1u : 0u));
                const uint32_t sh = (8u * ((push ? ld : ld - 1u) - 1u)) & 63u;
                const uint64_t sm = 0xFFull << sh;
                const uint64_t stk = stack, ank = arrn_stack;
                const uint32_t wr = push & has;
                stack = wr ? (stk & ~sm) | ((uint64_t)(cur & 0xFFu) << sh) : stk;
                arrn_stack = wr ? (ank & ~sm) | ((uint64_t)(arrn & 0xFFu) << sh) : ank;
                const uint32_t popped = (uint32_t)(stk >> sh) & 0xFFu;
                const uint32_t popped_n = (uint32_t)(ank >> sh) & 0xFFu;
                const uint32_t nld = push ? depth + 1u : ld - pop;
                const uint32_t rd = pop & (eqf(nld, 0u) ^ 1u);
                const uint32_t restored = rd ? pend_of(tn, popped) : kPendNone;
                cur = push ? pv : pop ? restored : cur;
                arrn = push ? 0u : rd ? popped_n : arrn;
                ld = nld;
                const uint32_t nd = depth + open_ok - close_ok;
                const uint32_t ob_bit = open_ok << nd;
                is_arr = (is_arr & ~ob_bit) | (f_barr ? ob_bit : 0u);
                idx_bits = (idx_bits & ~(pop << depth) & ~(push << nd)) | ((push & f_barr & (pv >> 17)) << nd);
                depth = nd;
                const uint32_t ns =
                    key_ok ? (uint32_t)X_COLON
                    : sval_ok ? (uint32_t)X_COMMA_OR_CLOSE
                    : open_ok ? (f_barr ? (uint32_t)X_VALUE_OR_CLOSE : (uint32_t)X_KEY_OR_CLOSE)
                    : close_ok ? (eqf(nd, 0u) ? (uint32_t)X_DONE : (uint32_t)X_COMMA_OR_CLOSE)
                    : (colon_ok | arr) ? (uint32_t)X_VALUE : (uint32_t)X_KEY;
                st = ok ? ns : (uint32_t)X_SLOW;
                pend = key_ok ? kPendNone : pend;
                if (key_ok & live_here) key(pp + 1, a, i, before8);  // a key of a live object
            }
            pp = a;
            // compact JSON: the ':' after a key and the ',' after a value go with it
            const uint32_t c2 = (w >> 8) & 0xFFu;
            const uint32_t m_colon = eqf(st, X_COLON) & eqf(c2, 0x3Au);
            const uint32_t merge = eqf(n1, i + 1) & (n1 >> 7 ^ 1u) & (m_colon | (eqf(st, X_COMMA_OR_CLOSE) & eqf(c2, 0x2Cu)));
            st = merge ? ((m_colon | ((is_arr >> depth) & 1u)) ? (uint32_t)X_VALUE : (uint32_t)X_KEY) : st;
            pp = a + merge;
            // the byte after pp (from w when still in this line)
            nbyte = pp + 1 < base + kLine ? (w >> (8 * (pp + 1 - a))) & 0xFFu : 0x100u;
            // advance to the next token (its word was read above)
            const uint32_t nx = merge ? n2 : n1;
            {  // drop the lowest token (n1), and with a merge the next one (n2)
                const uint64_t l1 = tk_lo & (tk_lo - 1), h1 = tk_lo ? tk_hi : tk_hi & (tk_hi - 1);
                const uint64_t l2 = l1 & (l1 - 1), h2 = l1 ? h1 : h1 & (h1 - 1);
                tk_lo = merge ? l2 : l1;
                tk_hi = merge ? h2 : h1;
            }
            have = nx < 128;
            i = nx;
            w = merge ? w2 : w1;
        }
        if (bs_hi) last_bs = base + 64 + hibit64(bs_hi);
        else if (bs_lo) last_bs = base + hibit64(bs_lo);
    }
    AJX_HD void run_line(const Block16* r) {
        classify(r);
        token_loop();
        flush();
    }

    // after the last line: Null selectors; false when the request has to go to the
    // exact scan
    AJX_HD bool finish(uint64_t* t_0, uint64_t* t_1) {
        if (st != X_DONE || bad) return false;
        const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
        const uint32_t ns = h->n_selectors;
        for (uint32_t s = 0; s < ns; s++) {
            if ((found >> s) & 1) continue;
            t0 |= sps[s].mask[0] & h->null_true[0];
            t1 |= sps[s].mask[1] & h->null_true[1];
        }
        *t_0 = t0;
        *t_1 = t1;
        return true;
    }
};

}  // namespace ajx
