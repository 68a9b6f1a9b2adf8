// ajx_events.h — stage A of the single-pass kernel as an event automaton.
//
// One work-item per request, the document read once in 64-byte windows exactly as
// ajx_fast.h's Scan does (aligned dwordx4 loads, one SWAR classification per window,
// escapes by the odd-backslash-run rule, string interiors by a prefix-XOR). What differs
// is what the per-token loop sees. Go's encoding/json writes compact JSON (the
// Authorization JSON of pkg/service/auth_pipeline.go:542-616 is json.Marshal output), so
// the local grammar — what may stand next to ':' and ',' — is checked for the whole
// window at once with 64-bit masks, and ':' and ',' never enter the loop. Neither do the
// member values that are strings or scalars (an opening quote or a scalar right after a
// ':'): when such a value belongs to a selector, its span is found from the masks (the
// next closing quote / the next ',' '}' ']'), possibly windows later. The loop takes
// only EVENTS:
//   - brackets ('{' '[' '}' ']'): push / pop of the container stack, trie node per depth;
//   - strings opened after '{' '[' ',': object keys (followed by ':') and array elements;
//   - scalars started after '[' ',': array elements.
// A c2 document (1 KiB) has ~120 events against ~220 tokens, and each event runs one
// short body in which the key lookup is the only sizeable part, instead of a grammar
// state machine whose branches a wave pays for together.
//
// Accepted: compact, valid JSON with an object or array root (whitespace between tokens,
// a backslash or control byte outside strings, a bad literal, a key with escapes on a
// selector path, nesting past the trie's tracked depth all send the request to the
// exact scan, ajx_device.h gj_get). For such documents gjson v1.14.0 Get returns the
// first complete path match in document order — the span captured here (ajx_fast.h
// header; the trie, key table and container captures are Scan's).
#pragma once
#include "ajx_fast.h"

namespace ajx {

// event automaton states: before the root, right after '{', right after '[', after a
// key (its ':' and value follow), after a complete value, after the root closed
enum : uint32_t { E_ROOT = 0, E_OBJ = 1, E_ARR = 2, E_KEY = 3, E_VAL = 4, E_DONE = 5, E_BAD = 6 };

// classes of a window's last byte carried into the next window's predecessor masks
enum : uint32_t { PK_QC = 1, PK_V = 2, PK_BR = 4, PK_K = 8, PK_M = 16 };

struct EvScan : Scan {
    uint64_t mqc;    // closing quotes of the window
    uint64_t mdl;    // scalar delimiters of the window (',' and brackets outside strings)
    uint64_t ke;     // closing quotes of keys among the window's events
    uint32_t wfl;    // carried window flags: PK_* of the previous window's last byte | 32 (an
                     // event string is open at the window start)
    uint32_t est;    // E_*
    // the pending capture of a member value (or array element scalar) that is a string or
    // a scalar: selector + 1 (0: none), start, bit 0 string?, bit 1 backslash seen
    uint32_t pc_sel, pc_start, pc_fl;

    // document byte q (doc position): the window ring holds the current and the previous
    // window; older or later bytes come from the document in memory
    AJX_HD uint32_t byte_doc(uint32_t q) const {
        const int32_t rel = (int32_t)q - bpos;
        if (rel >= -64 && rel < 64) return ring.u8((uint32_t)((int32_t)wa + rel));
        return d[q];
    }

    // a pending member-value capture that ends in this window (at or after its start)
    AJX_HD void resolve_pending() {
        if (!pc_sel) return;
        const int32_t f = (int32_t)pc_start + 1 - bpos;
        if (f >= 64) return;
        const uint64_t live = f <= 0 ? ~0ull : ~below64f((uint32_t)f);
        const bool str = pc_fl & 1u;
        const uint64_t m = (str ? mqc : mdl) & live;
        const uint64_t bs = mbs & live;
        if (!m) {
            pc_fl |= bs != 0 ? 2u : 0u;
            return;
        }
        const uint32_t j = ctz64f(m);
        const uint32_t esc_ = ((pc_fl >> 1) & 1u) | ((bs & below64f(j)) != 0 ? 1u : 0u);
        uint32_t type = T_STRING;
        if (!str) {
            const uint32_t c0 = byte_doc(pc_start);
            type = c0 == 't' ? T_TRUE : c0 == 'f' ? T_FALSE : c0 == 'n' ? T_NULL : T_NUMBER;
        }
        record((int32_t)pc_sel - 1, pc_start, (uint32_t)(bpos + (int32_t)j) + (str ? 1u : 0u), type, str ? esc_ : 0u);
        pc_sel = 0;
    }

    // scalars: a number (a raw run gjson takes up to its delimiter) or exactly a literal
    AJX_HD bool scalar_ok(uint32_t p) const {
        const uint32_t c0 = byte_doc(p);
        if (c0 == '-' || (c0 >= '0' && c0 <= '9')) return true;
        const uint32_t L = c0 == 'f' ? 5u : 4u;
        if ((c0 != 't' && c0 != 'f' && c0 != 'n') || p + L >= n) return false;
        uint64_t w = 0;
        for (uint32_t j = 0; j <= L; j++) w |= (uint64_t)byte_doc(p + j) << (8 * j);
        const uint64_t lit = c0 == 't' ? 0x65757274ull : c0 == 'f' ? 0x65736C6166ull : 0x6C6C756Eull;
        const uint32_t nb = (uint32_t)(w >> (8 * L)) & 0xFFu;
        return (w & ((1ull << (8 * L)) - 1ull)) == lit && (nb == ',' || nb == '}' || nb == ']');
    }

    // one event at window bit i
    AJX_HD void event(uint32_t i) {
        const uint32_t p = (uint32_t)(bpos + (int32_t)i);
        const uint32_t c = byte_at(i);
        const uint32_t lc = c | 0x20u;
        const bool isQ = c == '"', isO = lc == '{', isC = lc == '}';
        const bool arrB = (c & 0x20u) == 0u;  // '[' ']'
        const bool isKey = ((ke >> i) & 1u) != 0;
        const uint32_t start = isQ ? open_before(i) : p;
        const uint32_t prevc = start ? byte_doc(start - 1) : 0u;
        const bool tarr = depth && top_is_arr();
        const bool member = isO && est == E_KEY && prevc == ':';
        // after a key, any event but its container value means the value (a string or a
        // scalar, not an event) is complete
        const uint32_t eff = est == E_KEY && !member ? E_VAL : est;
        const bool after_comma = eff == E_VAL && prevc == ',';
        const bool elem = tarr && ((eff == E_ARR && prevc == '[') || after_comma);
        const bool keyok = depth && !tarr && ((eff == E_OBJ && prevc == '{') || after_comma);
        const bool closeok = depth && tarr == arrB && prevc != ',' && prevc != ':' &&
                             (eff == E_VAL || eff == (arrB ? E_ARR : E_OBJ)) && (depth > 1 || p + 1 == n);
        const bool ok = isKey ? keyok : isO ? (member || elem || est == E_ROOT) : isC ? closeok : elem;
        if (!ok) {
            est = E_BAD;
            return;
        }
        if (isC) {
            close_container(p);
            est = depth ? E_VAL : E_DONE;
            return;
        }
        // the trie node of the key, or of the value that starts here (a member container:
        // its key's node; an array element: the index child; the root: node 0)
        uint32_t node;
        if (isKey) {
            st = X_ROOT;
            key_closed(p, i);
            if (st == X_SLOW) {  // an escaped key on a selector path
                est = E_BAD;
                return;
            }
            node = pending;
        } else {
            node = value_node();
        }
        const int32_t s = leaf_sel(node);
        if (isO) {
            if (!push(c, p, node, s)) {
                est = E_BAD;
                return;
            }
            est = arrB ? E_ARR : E_OBJ;
            return;
        }
        if (s >= 0) {
            // a string or a scalar value of selector s: the member value after this key
            // (a container value is captured by its own open event), or this element
            const uint32_t vs = isKey ? p + 2 : start;
            const uint32_t vb = isKey ? (vs < n ? byte_doc(vs) : 0u) : c;
            if (vb != '{' && vb != '[') {
                if (!isKey && isQ) {
                    const uint32_t lb = last_bs_before(i);
                    record(s, start, p + 1, T_STRING, (lb != ~0u && lb > start) ? 1u : 0u);
                } else {
                    found |= 1ull << s;  // (first match in document order)
                    pc_sel = (uint32_t)s + 1u;
                    pc_start = vs;
                    pc_fl = vb == '"' ? 1u : 0u;
                    resolve_pending();
                }
            }
        }
        if (!isKey) element_done();
        est = isKey ? E_KEY : E_VAL;
    }

    // Scan::open_container with the node and leaf selector already resolved
    AJX_HD bool push(uint32_t c, uint32_t p, uint32_t node, int32_t s) {
        if (depth + 1 >= 63) return false;
        depth++;
        const uint64_t bit = 1ull << depth;
        is_arr = c == '[' ? is_arr | bit : is_arr & ~bit;
        top_arr = c == '[' ? 1u : 0u;
        const uint32_t live = node != kNoNode && tn[node].n_children ? node : kNoNode;
        if (live != kNoNode && depth > kFastDepth) return false;
        set_node(depth, live);
        top_node = live;
        if (s >= 0) {
            found |= 1ull << s;  // first match in document order wins
            if (ncap >= 2) return false;
            const uint32_t v = (uint32_t)s | (depth << 8), c0 = cap0, c1 = cap1, s0 = cap0_start, s1 = cap1_start;
            cap0 = ncap == 0 ? v : c0;
            cap0_start = ncap == 0 ? p : s0;
            cap1 = ncap == 1 ? v : c1;
            cap1_start = ncap == 1 ? p : s1;
            ncap++;
        }
        if (c == '[' && live != kNoNode && (tn[live].flags & 1)) {
            if (narr >= 2) return false;
            const uint32_t a0 = arr0, a1 = arr1;
            arr0 = narr == 0 ? depth : a0;
            arr1 = narr == 1 ? depth : a1;
            narr++;
        }
        return true;
    }

    // the 64 document bytes of a window (ring position of byte 0 = a, a multiple of 64;
    // doc position of byte 0 = bp); nx0 = the next window's first byte (its ':' test)
    AJX_HD void window(const Block16* blk, uint32_t nx0, uint32_t a, int32_t bp) {
        wa = a;
        bpos = bp;
        uint64_t valid = ~0ull;
        if (bp < 0) valid &= ~below64f((uint32_t)(-bp));
        if (bp + 64 > (int32_t)n) valid &= below64f((uint32_t)((int32_t)n - bp));
        uint64_t mq = 0, mb = 0, mbr = 0, mkk = 0, mm = 0, mws = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const Block16 x4 = blk[j];
            ring.put(a + 16u * (uint32_t)j, x4);
            uint32_t q16 = 0, b16 = 0, r16 = 0, k16 = 0, m16 = 0, w16 = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t x = k == 0 ? x4.x : k == 1 ? x4.y : k == 2 ? x4.z : x4.w;
                const uint32_t lx = x | 0x20202020u;
                q16 |= gather4(eq_bytes(x, 0x22222222u)) << (4 * k);
                b16 |= gather4(eq_bytes(x, 0x5C5C5C5Cu)) << (4 * k);
                r16 |= gather4(eq_bytes(lx, 0x7B7B7B7Bu) | eq_bytes(lx, 0x7D7D7D7Du)) << (4 * k);
                k16 |= gather4(eq_bytes(x, 0x3A3A3A3Au)) << (4 * k);
                m16 |= gather4(eq_bytes(x, 0x2C2C2C2Cu)) << (4 * k);
                w16 |= gather4(le20_bytes(x)) << (4 * k);
            }
            mq |= (uint64_t)q16 << (16 * j);
            mb |= (uint64_t)b16 << (16 * j);
            mbr |= (uint64_t)r16 << (16 * j);
            mkk |= (uint64_t)k16 << (16 * j);
            mm |= (uint64_t)m16 << (16 * j);
            mws |= (uint64_t)w16 << (16 * j);
        }
        mq &= valid;
        mb &= valid;
        mbs = mb;
        // escaped bytes: the byte after an odd-length backslash run
        uint64_t escaped;
        {
            const uint64_t bs = mb & ~(uint64_t)esc;
            const uint64_t follows = (bs << 1) | esc;
            const uint64_t even = 0x5555555555555555ull;
            const uint64_t odd_starts = bs & ~even & ~follows;
            const uint64_t seq = odd_starts + bs;
            esc = seq < bs ? 1u : 0u;
            escaped = (even ^ (seq << 1)) & follows;
        }
        carry_bs = last_bs;
        if (mb) last_bs = (uint32_t)(bp + (int32_t)hibit64f(mb));
        const uint64_t qu = mq & ~escaped;
        uint64_t x = qu;
        x ^= x << 1;
        x ^= x << 2;
        x ^= x << 4;
        x ^= x << 8;
        x ^= x << 16;
        x ^= x << 32;
        const uint64_t instr = in_str ? ~x : x;  // inside a string after this byte
        in_str = (uint32_t)(instr >> 63);
        const uint64_t outside = ~instr & ~qu & valid;
        oq = qu & instr;
        carry_oq = last_oq;
        if (oq) last_oq = (uint32_t)(bp + (int32_t)hibit64f(oq));
        const uint64_t qc = qu & ~instr;
        const uint64_t K = mkk & outside, M = mm & outside, Br = mbr & outside;
        const uint64_t V = outside & ~(K | M | Br | mws | mb);
        mqc = qc;
        mdl = M | Br;
        // the compact-JSON rules around ':' ',' and value starts, for the whole window
        // (P(x): x at the preceding byte)
        const uint32_t pk = wfl;
        const uint64_t PQc = (qc << 1) | (pk & PK_QC ? 1u : 0u);
        const uint64_t PV = (V << 1) | (pk & PK_V ? 1u : 0u);
        const uint64_t PBr = (Br << 1) | (pk & PK_BR ? 1u : 0u);
        const uint64_t PK = (K << 1) | (pk & PK_K ? 1u : 0u);
        const uint64_t PM = (M << 1) | (pk & PK_M ? 1u : 0u);
        const uint64_t Vs = V & ~PV;  // scalar starts
        const uint64_t knext = nx0 == ':' && bp + 64 < (int32_t)n ? 1u : 0u;
        const uint64_t KC = qc & ((K >> 1) | (knext << 63));  // closing quotes of keys
        uint64_t bad = (mb | mws) & outside;
        bad |= K & ~PQc;
        bad |= M & ~(PQc | PV | PBr);
        bad |= (K | M) & (PK | PM);
        bad |= oq & (PQc | PV);
        bad |= Vs & PQc;
        // event strings: opened anywhere but right after ':' (the carry of the add moves
        // the mark from the opening quote along the string to its closing quote)
        const uint64_t SQ = oq & ~PK;
        const uint64_t s1 = instr + SQ;
        const uint64_t s2 = s1 + (uint64_t)((pk >> 5) & 1u);
        const uint64_t QcE = s2 & ~instr & qc;
        bad |= KC & ~QcE;  // a member value followed by ':'
        ke = KC;
        wfl = (uint32_t)(qc >> 63) * PK_QC | (uint32_t)(V >> 63) * PK_V | (uint32_t)(Br >> 63) * PK_BR |
              (uint32_t)(K >> 63) * PK_K | (uint32_t)(M >> 63) * PK_M | ((s1 < instr || s2 < s1) ? 32u : 0u);
        if (bad) {
            est = E_BAD;
            return;
        }
        // literals and number starts
        for (uint64_t t = Vs; t; t &= t - 1) {
            if (!scalar_ok((uint32_t)(bp + (int32_t)ctz64f(t)))) {
                est = E_BAD;
                return;
            }
        }
        resolve_pending();
        uint64_t ev = Br | QcE | (Vs & ~PK);
        while (ev) {
            const uint32_t i = ctz64f(ev);
            ev &= ev - 1;
            event(i);
            if (est == E_BAD) return;
        }
    }
};

// Stage A with the event automaton for one request; the same contract as scan_doc
// (ajx_fast.h): true when `row` holds the request's captures, false for the exact scan.
template <class LoadBlock>
AJX_HD bool scan_doc_ev(const uint8_t* blob, const Tables& tab, const uint8_t* d, uint32_t n, RowRef row,
                        const WinRing& ring, LoadBlock load) {
    const RulesetHdr* h = (const RulesetHdr*)blob;
    EvScan s;
    s.tn = tab.tn;
    s.tc = tab.tc;
    s.ks = tab.ks;
    s.ks_meta = h->key_slots_log2 | h->key_probes << 8;
    s.lits = blob + h->off_literals;
    s.d = d;
    s.row = row;
    s.n = n;
    s.ring = ring;
    s.wa = 0;
    s.bpos = 0;
    s.mbs = 0;
    s.carry_bs = ~0u;
    s.oq = 0;
    s.carry_oq = s.last_oq = 0;
    s.is_arr = 0;
    s.top_arr = 0;
    s.top_node = 0;  // (the root's node)
    s.nodes_lo = s.nodes_hi = ~0ull;
    s.found = 0;
    s.depth = 0;
    s.st = X_ROOT;
    s.pending = kNoNode;
    s.str_open = 0;
    s.gap_first = s.gap_last = s.gap_cnt = 0;
    s.last_bs = ~0u;
    s.in_str = s.esc = 0;
    s.cap0 = s.cap0_start = s.cap1 = s.cap1_start = s.ncap = 0;
    s.arr0 = s.arr1 = s.narr = 0;
    s.mqc = s.mdl = s.ke = 0;
    s.wfl = 0;
    s.est = E_ROOT;
    s.pc_sel = s.pc_start = s.pc_fl = 0;

    const uint32_t mis = (uint32_t)((uintptr_t)d & 15u);
    const uint32_t nblk = (n + mis + 15) / 16;
    Block16 cur[4], nxt[4];
#pragma unroll
    for (int j = 0; j < 4; j++) cur[j] = load((uint32_t)j, nblk);
#pragma unroll
    for (int j = 0; j < 4; j++) nxt[j] = load((uint32_t)(4 + j), nblk);
    for (uint32_t b0 = 0; b0 < nblk; b0 += 4) {
        s.window(cur, nxt[0].x & 0xFFu, b0 * 16, (int32_t)(b0 * 16) - (int32_t)mis);
        if (s.est == E_BAD) break;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            cur[j] = nxt[j];
            nxt[j] = load(b0 + 8 + (uint32_t)j, nblk);
        }
    }
    if (s.est != E_DONE || s.in_str || s.pc_sel) {
        row[0] = kRowSlow;
        return false;
    }
    row[0] = s.found;
    return true;
}

}  // namespace ajx
