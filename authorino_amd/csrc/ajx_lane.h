// ajx_lane.h — the lane kernel's per-request scanner: one work-item per request, the
// document read in 64-byte windows that the wavefront stages through LDS with coalesced
// loads (ajx_kernels.hip ajx_lane_eval: four 1 KiB wave loads bring the next window of
// all 64 requests of the wave, so each load instruction touches 16 documents, not 64).
//
// Per window, per request:
//   classify   SWAR byte classes -> 64-bit masks: '"', '\\', '{' '[', '}' ']', ':', ',',
//              whitespace
//   strings    odd-backslash-run escapes and a prefix-XOR of the unescaped quotes, with
//              string / escape state carried from window to window
//   grammar    every byte outside strings against the byte before it (compact JSON:
//              what may follow '{' '[' ':' ',' a closing quote, a scalar, a closing
//              bracket), literals exact
//   tokens     closing quotes (a key when ':' follows), scalar starts, '{' '[', '}' ']'
//              drive a small automaton: objects alternate key / value, arrays take
//              values, brackets match, one root. It follows every selector through the
//              trie (the key table of ajx_blob.h: signature, length, parent) and
//              captures the first value in document order on each selector's path —
//              gjson v1.14.0 Get's result for valid JSON.
// A request that is not provably valid compact JSON (or has a backslash in a key on a
// selector's path) goes to the exact scan (gj_get).
// Then the patterns and the fold run in the same work-item (ajx_fast.h stage B).
#pragma once
#include "ajx_fast.h"

namespace ajx {

// the staged windows are read through an LDS-typed pointer: a byte that may come from
// LDS or from the document would otherwise become one flat load through a selected pointer
#if defined(__HIP_DEVICE_COMPILE__)
#define AJX_LDS __attribute__((address_space(3)))
#else
#define AJX_LDS
#endif

constexpr uint32_t kLaneWin = 64;       // bytes per window and request
constexpr uint32_t kLaneSlot = 64 * kLaneWin;  // one staged window of a wavefront (64 requests)

AJX_HD uint64_t prefix_xor64(uint64_t x) {
    x ^= x << 1;
    x ^= x << 2;
    x ^= x << 4;
    x ^= x << 8;
    x ^= x << 16;
    x ^= x << 32;
    return x;
}

struct Classes64 {
    uint64_t q, bs, o, c, k, m, ws, sq;  // sq: '[' ']' among o / c
};
AJX_HD Classes64 classify64(const uint32_t (&x)[16]) {
    uint32_t q[2] = {0, 0}, bs[2] = {0, 0}, o[2] = {0, 0}, c[2] = {0, 0}, k[2] = {0, 0}, m[2] = {0, 0},
             ws[2] = {0, 0}, sq[2] = {0, 0};
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint32_t v = x[j], lx = v | 0x20202020u;
        const uint32_t sh = 4u * (uint32_t)(j & 7), h = (uint32_t)j >> 3;
        q[h] |= gather4(eq_bytes(v, 0x22222222u)) << sh;
        bs[h] |= gather4(eq_bytes(v, 0x5C5C5C5Cu)) << sh;
        o[h] |= gather4(eq_bytes(lx, 0x7B7B7B7Bu)) << sh;
        c[h] |= gather4(eq_bytes(lx, 0x7D7D7D7Du)) << sh;
        k[h] |= gather4(eq_bytes(v, 0x3A3A3A3Au)) << sh;
        m[h] |= gather4(eq_bytes(v, 0x2C2C2C2Cu)) << sh;
        ws[h] |= gather4(le20_bytes(v)) << sh;
        sq[h] |= gather4(~(v << 2) & 0x80808080u) << sh;  // bit 5 clear
    }
    auto w64 = [](const uint32_t (&p)[2]) { return (uint64_t)p[0] | ((uint64_t)p[1] << 32); };
    return Classes64{w64(q), w64(bs), w64(o), w64(c), w64(k), w64(m), w64(ws), w64(sq)};
}

// one request's scan state (registers); table pointers may point at an LDS copy
struct LaneScan {
    // tables
    const TrieNode* tn;
    const TrieChild* tc;
    const KeySlot* ks;
    const uint8_t* lits;
    uint32_t ks_log2;
    // document: aligned offset a = document position + mis; the staged windows w - 1, w,
    // w + 1 in LDS
    const AJX_LDS uint8_t* stage;  // the wavefront's 3 staging slots
    uint32_t lane_off;             // this request's 64 bytes inside a slot
    uint32_t mis, end;
    uint64_t* row;
    // lexer carries
    uint32_t in_str, esc, pin;  // pin: classes of the byte before the window (Qc K M O C V)
    uint32_t last_qo;           // aligned offset of the last opening quote
    uint32_t bs_in_str;         // a backslash inside the string open at the window start
    uint32_t w;                 // current window
    // automaton: container stack (is_arr bit per depth, trie node per depth up to
    // kFastDepth), cur = node of the innermost container (kNoNode: dead — no selector
    // reaches inside, only its brackets are followed)
    uint64_t is_arr, nodes_lo, nodes_hi, found;
    uint32_t depth, cur, expv, pend, done, bad;
    uint32_t sc, sc_start;      // pending scalar capture: selector + 1 | type << 8; start
    uint32_t cap0, cap0_start, cap1, cap1_start, ncap;  // open container captures
    uint32_t arr0, arr1, narr;  // live arrays with index children: depth | index << 8

    // byte / 8-byte word (a % 8 == 0) at aligned offset a of a staged window (w - 1, w
    // or w + 1; the scanner reads no other)
    AJX_HD uint32_t byte_at(uint32_t a) const {
        return stage[((a / kLaneWin) % 3) * kLaneSlot + lane_off + (a % kLaneWin)];
    }
    AJX_HD uint64_t word_at(uint32_t a) const {
        return *(const AJX_LDS uint64_t*)(stage + ((a / kLaneWin) % 3) * kLaneSlot + lane_off + (a % kLaneWin));
    }
    // the 8 bytes before aligned offset e, little-endian (e - 8 >= 64 (w - 1); bytes
    // before the document's first 16-byte block read as 0)
    AJX_HD uint64_t tail8(uint32_t e) const {
        const uint32_t e8 = e & ~7u, r = e & 7u;
        const uint64_t hi = r ? word_at(e8) : 0ull;
        const uint64_t lo = e8 >= 8 ? word_at(e8 - 8) : 0ull;
        return r ? (lo >> (8 * r)) | (hi << (64 - 8 * r)) : lo;
    }
    // child of `parent` by the key at aligned offsets [ka, e) (no backslash, ka + 56 >=
    // 64 w: every word read lies in a staged window): the key table (signature, length,
    // parent); kNoNode when no selector names it
    AJX_HD uint32_t key_node(uint32_t parent, uint32_t ka, uint32_t e) const {
        const uint32_t klen = e - ka, mask = (1u << ks_log2) - 1u;
        uint64_t sig = tail8(e);
        if (klen < 8) sig = klen ? sig >> (8 * (8 - klen)) : 0ull;
        const uint32_t want = klen | (parent << 16);
        uint32_t at = key_slot_hash(sig, klen, parent, ks_log2);
        for (uint32_t probe = 0; probe <= mask; probe++, at = (at + 1) & mask) {
            const KeySlot slot = ks[at];
            if (slot.meta == kEmptySlot) return kNoNode;
            if (slot.sig != sig || (slot.meta & 0xFFFFFFu) != want) continue;
            // the bytes before the signature, a word at a time (key literals are 8-byte
            // aligned in the pool)
            bool eq = true;
            const uint64_t* kl = (const uint64_t*)(lits + slot.key_off);
            for (uint32_t j = 0; j + 8 < klen; j += 8) {
                const uint32_t r = klen - 8 - j;
                const uint64_t m = r >= 8 ? ~0ull : (1ull << (8 * r)) - 1ull;
                if ((tail8(ka + j + 8) ^ kl[j / 8]) & m) { eq = false; break; }
            }
            if (eq) return slot.meta >> 24;
        }
        return kNoNode;
    }
    AJX_HD uint32_t node_at(uint32_t dd) const {
        if (dd == 0) return 0;
        if (dd > kFastDepth) return kNoNode;
        const uint32_t k = dd - 1;
        const uint64_t wv = k < 8 ? nodes_lo : nodes_hi;
        return (uint32_t)((wv >> ((k & 7) * 8)) & 0xFFu);
    }
    AJX_HD void set_node(uint32_t dd, uint32_t v) {
        if (dd == 0 || dd > kFastDepth) return;
        const uint32_t k = dd - 1;
        const uint64_t m = 0xFFull << ((k & 7) * 8);
        const uint64_t x = ((uint64_t)(v & 0xFF)) << ((k & 7) * 8);
        const uint64_t lo = nodes_lo, hi = nodes_hi;
        nodes_lo = k < 8 ? (lo & ~m) | x : lo;
        nodes_hi = k < 8 ? hi : (hi & ~m) | x;
    }
    AJX_HD bool top_is_arr() const { return (is_arr >> depth) & 1; }
    // node of the element about to start in the innermost (live array) container
    AJX_HD uint32_t elem_node() const {
        if (!narr || !(tn[cur].flags & 1)) return kNoNode;
        uint32_t h;
        if (narr >= 2 && (arr1 & 0xFF) == depth) h = arr1 >> 8;
        else if ((arr0 & 0xFF) == depth) h = arr0 >> 8;
        else return kNoNode;
        const uint32_t cb = tn[cur].child_begin, nc = tn[cur].n_children;
        for (uint32_t c = 0; c < nc; c++)
            if (tc[cb + c].array_index == (int32_t)h) return tc[cb + c].node;
        return kNoNode;
    }
    AJX_HD void element_done() {
        if (!narr || !top_is_arr()) return;
        const bool h1 = narr >= 2 && (arr1 & 0xFF) == depth;
        const bool h0 = !h1 && (arr0 & 0xFF) == depth;
        arr1 += h1 ? 0x100u : 0u;
        arr0 += h0 ? 0x100u : 0u;
    }
    AJX_HD int32_t leaf_sel(uint32_t node) const {
        if (node == kNoNode) return -1;
        const int32_t s = tn[node].selector;
        if (s < 0 || ((found >> s) & 1)) return -1;
        return s;
    }
    AJX_HD void record(int32_t s, uint32_t start, uint32_t stop, uint32_t type, uint32_t e) {
        found |= 1ull << s;
        row[1 + s] = (uint64_t)start | ((uint64_t)(((stop - start) & 0xFFFFFFu) | (type << 24) | (e << 27)) << 32);
    }
    AJX_HD void open(bool arr, uint32_t start, uint32_t node) {
        if (depth + 1 >= 63) { bad = 1; return; }
        depth++;
        const uint64_t bit = 1ull << depth;
        is_arr = arr ? is_arr | bit : is_arr & ~bit;
        expv = 0;
        cur = kNoNode;
        if (node == kNoNode) { set_node(depth, kNoNode); return; }
        const int32_t s = leaf_sel(node);
        const uint32_t live = tn[node].n_children ? node : kNoNode;
        if (live != kNoNode && depth > kFastDepth) { bad = 1; return; }
        set_node(depth, live);
        cur = live;
        if (s >= 0) {
            found |= 1ull << s;
            if (ncap >= 2) { bad = 1; return; }
            const uint32_t v = (uint32_t)s | (depth << 8);
            if (ncap == 0) { cap0 = v; cap0_start = start; }
            else { cap1 = v; cap1_start = start; }
            ncap++;
        }
        if (arr && live != kNoNode && (tn[live].flags & 1)) {
            if (narr >= 2) { bad = 1; return; }
            if (narr == 0) arr0 = depth;
            else arr1 = depth;
            narr++;
        }
    }
    AJX_HD void close(uint32_t pos) {
        if (ncap) {
            const uint32_t cs = ncap == 2 ? cap1 : cap0;
            if ((cs >> 8) == depth) {
                const uint32_t start = ncap == 2 ? cap1_start : cap0_start;
                row[1 + (cs & 0xFF)] =
                    (uint64_t)start | ((uint64_t)(((pos + 1 - start) & 0xFFFFFFu) | ((uint32_t)T_JSON << 24)) << 32);
                ncap--;
            }
        }
        if (narr) {
            const uint32_t at = narr == 2 ? arr1 : arr0;
            if ((at & 0xFF) == depth) narr--;
        }
        depth--;
        cur = node_at(depth);
        done = depth == 0;
        element_done();  // the container was an element of its parent array
    }

    AJX_HD void init(const uint8_t* blob, const Tables& tab, const uint8_t* doc, uint32_t len, uint64_t* r) {
        const RulesetHdr* h = (const RulesetHdr*)blob;
        tn = tab.tn;
        tc = tab.tc;
        ks = tab.ks;
        lits = blob + h->off_literals;
        ks_log2 = h->key_slots_log2;
        mis = (uint32_t)((uintptr_t)doc & 15u);
        end = mis + len;
        row = r;
        in_str = esc = pin = last_qo = bs_in_str = 0;
        w = 0;
        is_arr = 0;
        nodes_lo = nodes_hi = ~0ull;
        found = 0;
        depth = expv = done = bad = 0;
        cur = 0;
        pend = kNoNode;
        sc = sc_start = 0;
        cap0 = cap0_start = cap1 = cap1_start = ncap = 0;
        arr0 = arr1 = narr = 0;
    }

    // one 64-byte window (aligned offsets [64 w, 64 w + 64)) already staged.
    // ABL (profiling ablations, results meaningless): 2 no token walk, 3 no key lookups
    template <int ABL = 0>
    AJX_HD void window(const uint32_t (&x)[16], uint32_t win) {
        w = win;
        const uint32_t a0 = win * kLaneWin;
        uint64_t valid = ~0ull;
        if (a0 < mis) valid &= ~0ull << (mis - a0);
        if (a0 + kLaneWin > end) valid &= a0 >= end ? 0ull : (1ull << (end - a0)) - 1ull;
        const Classes64 k = classify64(x);
        const uint64_t BS = k.bs & valid;
        // escapes
        uint64_t E = 0;
        if (BS | esc) {
            const uint64_t bsx = BS & ~(uint64_t)esc;
            const uint64_t follows = (bsx << 1) | esc;
            const uint64_t even = 0x5555555555555555ull;
            const uint64_t odd_starts = bsx & ~even & ~follows;
            const uint64_t seq = odd_starts + bsx;
            esc = seq < bsx ? 1u : 0u;
            E = (even ^ (seq << 1)) & follows;
        }
        // strings
        const uint64_t QU = k.q & valid & ~E;
        const uint64_t instr = prefix_xor64(QU) ^ (in_str ? ~0ull : 0ull);
        const uint32_t in_str0 = in_str;
        in_str = (uint32_t)(instr >> 63);
        const uint64_t Qo = QU & instr, Qc = QU & ~instr;
        const uint64_t OUT = ~instr & ~QU & valid;
        const uint64_t Ko = k.k & OUT, Mo = k.m & OUT, Oo = k.o & OUT, Co = k.c & OUT;
        const uint64_t V = OUT & ~(Ko | Mo | Oo | Co | k.ws | BS);
        uint64_t lbad = (BS | k.ws) & OUT;
        // compact-JSON successor rules (what may follow each class)
        const uint64_t PQc = (Qc << 1) | (pin & 1u);
        const uint64_t PKM = ((Ko | Mo) << 1) | ((pin >> 1) & 1u);
        const uint64_t POo = (Oo << 1) | ((pin >> 3) & 1u);
        const uint64_t PCo = (Co << 1) | ((pin >> 4) & 1u);
        const uint64_t PV = (V << 1) | ((pin >> 5) & 1u);
        pin = (uint32_t)((Qc >> 63) | (((Ko | Mo) >> 63) << 1) | ((Oo >> 63) << 3) | ((Co >> 63) << 4) |
                         ((V >> 63) << 5));
        lbad |= PQc & ~(Ko | Mo | Co) & valid;
        lbad |= PKM & ~(Qo | Oo | V) & valid;
        lbad |= POo & ~(Qo | Oo | V | Co) & valid;
        lbad |= PCo & ~(Mo | Co) & valid;
        lbad |= PV & ~(V | Mo | Co) & valid;
        // the document starts with its root container and ends with its close
        if (a0 <= mis && mis < a0 + kLaneWin && !((Oo >> (mis - a0)) & 1u)) lbad |= 1;
        if (end - 1 >= a0 && end - 1 < a0 + kLaneWin && !((Co >> (end - 1 - a0)) & 1u)) lbad |= 1;
        if (lbad) bad = 1;
        const uint64_t Vst = V & ~PV;
        // scalars: a number (digit or '-') or exactly true / false / null, then , } ]
        {
            uint64_t lt = bad ? 0ull : Vst;
            while (lt) {
                const uint32_t t = ctz64f(lt);
                lt &= lt - 1;
                const uint32_t b = byte_at(a0 + t);
                if (b == '-' || (b >= '0' && b <= '9')) continue;
                uint32_t L;
                uint64_t want;
                if (b == 't') { L = 4; want = 0x65757274ull; }
                else if (b == 'f') { L = 5; want = 0x65736C6166ull; }
                else if (b == 'n') { L = 4; want = 0x6C6C756Eull; }
                else { bad = 1; break; }
                if (a0 + t + L >= end) { bad = 1; break; }
                uint64_t got = 0;
                for (uint32_t i = 0; i < L; i++) got |= (uint64_t)byte_at(a0 + t + i) << (8 * i);
                const uint32_t nb = byte_at(a0 + t + L);
                if (got != want || !(nb == ',' || nb == '}' || nb == ']')) { bad = 1; break; }
            }
        }
        // the carries of the next window (the token loop reads the current ones)
        uint32_t nlast_qo = last_qo, nbs = bs_in_str;
        if (Qo | Qc) {
            const uint32_t hq = hibit64f(Qo | Qc);
            if ((Qo >> hq) & 1u) {
                nlast_qo = a0 + hq;
                nbs = (BS >> hq) >> 1 ? 1u : 0u;
            }
        } else if (in_str0) {
            nbs |= BS ? 1u : 0u;
        }
        // tokens, kind coded in three masks: brackets A (B: close, C: square), else B
        // key (a closing quote followed by ':'), C string value, neither a scalar start
        const uint32_t nk = (Qc >> 63) && a0 + kLaneWin < end ? (byte_at(a0 + kLaneWin) == ':' ? 1u : 0u) : 0u;
        const uint64_t KC = Qc & ((Ko >> 1) | ((uint64_t)nk << 63));
        const uint64_t A = Oo | Co, B = Co | KC, C = (Qc & ~KC) | (A & k.sq);
        const uint64_t all = Qc | Vst | A;
        uint64_t tok = bad ? 0ull : (cur == kNoNode ? A : all);
        if constexpr (ABL == 2) {  // profiling: no token walk
            found += tok;
            tok = 0;
        }
        uint64_t skip = 0;
        while (tok) {
            const uint32_t t = ctz64f(tok);
            const uint64_t bit = 1ull << t;
            const uint32_t pos = a0 + t - mis;  // document position
            const bool brk = (A >> t) & 1, bb = (B >> t) & 1, cc = (C >> t) & 1;
            const bool quote = !brk && (bb || cc);  // a closing quote (key or string value)
            const uint64_t qb = Qo & (bit - 1);
            const uint32_t qo = qb ? a0 + hibit64f(qb) : last_qo;  // (quotes) opening quote, aligned
            // the next element's start (or the close) ends a pending scalar
            if (sc) {
                const uint32_t stop = (brk && bb) ? pos : (quote ? qo - mis : pos) - 1u;
                record((int32_t)(sc & 0xFF) - 1, sc_start, stop, sc >> 8, 0);
                sc = 0;
            }
            if (done) { bad = 1; break; }  // a token after the root closed
            const bool arr = top_is_arr();
            if (cur == kNoNode && depth > 0) {
                // inside a dead container: its brackets only (gjson skips the container
                // by bracket depth outside strings; the types must still match here)
                if (bb) {
                    if (cc != arr) { bad = 1; break; }
                    close(pos);
                } else {
                    open(cc, pos, kNoNode);
                }
            } else if (brk && bb) {  // '}' ']'
                if (depth == 0 || expv || cc != arr) { bad = 1; break; }
                close(pos);
            } else if (bb) {  // a key: the value comes next
                if (depth == 0 || arr || expv) { bad = 1; break; }
                expv = 1;
                pend = kNoNode;
                if (ABL != 3 && cur != kNoNode) {
                    // a backslash in a key on a live path: the exact scan
                    const uint64_t between = (bit - 1) & ~((qb ? (2ull << hibit64f(qb)) : 1ull) - 1);
                    if ((BS & between) || (!qb && bs_in_str)) { bad = 1; break; }
                    // (a key that began before the staged windows: the exact scan)
                    if (qo + 1 + 56 < a0) { bad = 1; break; }
                    pend = key_node(cur, qo + 1, a0 + t);
                }
                // a member no selector names whose value is a string or a scalar in this
                // window: the value token is consumed here (nothing to capture; the
                // grammar rules already hold for it)
                if (pend == kNoNode) {
                    const uint64_t nxt = all & ~((bit << 1) - 1ull);
                    const uint64_t vb = nxt & (0ull - nxt);
                    if (vb && !(A & vb)) {
                        expv = 0;
                        skip = vb;
                    }
                }
            } else {  // a value: container open, string or scalar
                uint32_t node;
                if (depth == 0) {
                    if (!brk || pos != 0) { bad = 1; break; }
                    node = 0;
                } else if (arr) {
                    node = elem_node();
                } else {
                    if (!expv) { bad = 1; break; }
                    node = pend;
                }
                expv = 0;
                if (brk) {
                    open(cc, pos, node);
                } else {
                    const int32_t s = leaf_sel(node);
                    if (s >= 0) {
                        if (cc) {
                            // a backslash between the opening and the closing quote
                            const uint64_t between = (bit - 1) & ~((qb ? (2ull << hibit64f(qb)) : 1ull) - 1);
                            const uint32_t e = (BS & between) || (!qb && bs_in_str) ? 1u : 0u;
                            record(s, qo - mis, pos + 1, T_STRING, e);
                        } else {
                            const uint32_t b = byte_at(a0 + t);
                            const uint32_t ty = b == 't' ? T_TRUE : b == 'f' ? T_FALSE : b == 'n' ? T_NULL : T_NUMBER;
                            sc = (uint32_t)(s + 1) | (ty << 8);
                            sc_start = pos;
                        }
                    }
                    element_done();
                }
            }
            if (bad) break;
            // next token: inside a dead container only its brackets
            const uint64_t above = ~((bit << 1) - 1ull);
            tok = (cur == kNoNode ? A : all) & above & ~skip;
            skip = 0;
        }
        last_qo = nlast_qo;
        bs_in_str = nbs;
    }

    // after the last window: true when the capture row is the gjson result
    AJX_HD bool finish() {
        if (bad || in_str || esc || !done) return false;
        row[0] = found;
        return true;
    }
};

}  // namespace ajx
