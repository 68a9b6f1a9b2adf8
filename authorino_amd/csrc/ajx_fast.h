// ajx_fast.h — single-pass evaluation of one request by one work-item.
//
// The document is read once, 16 bytes at a time (aligned dwordx4 loads, the next 64
// bytes prefetched). Each 16-byte block is classified with SWAR byte compares into
// bitmasks (quote, backslash, structural, whitespace); escapes are resolved with the
// branch-free odd-backslash-run rule and string interiors with a prefix-XOR of the
// unescaped quotes (carrying string / escape state from block to block). Only the
// tokens left (structural bytes outside strings, string delimiters, scalar runs) go
// through a JSON grammar automaton that
//   * follows every selector at once through the ruleset's trie (the path a gjson.Get
//     for each selector would take: for documents that are valid JSON, gjson v1.14.0
//     returns the first complete path match in document order, which is exactly the
//     first key (or element) reached here on a trie node that ends a selector), and
//   * evaluates a selector's patterns the moment its value is complete
//     (Pattern.Matches, pkg/jsonexp/expressions.go:59-96, via ajx_device.h).
// Anything the automaton can not prove equivalent to gjson's own scan (a document that
// is not valid JSON, a non-object/array root, a key with escapes on a selector path,
// nesting deeper than tracked) sets `slow`: such requests are re-evaluated by the
// exact per-selector gjson scan kernel (ajx_eval_scan).
#pragma once
#include "ajx_device.h"

namespace ajx {

// 0x80 in every byte equal to the byte replicated in c4
AJX_HD uint32_t eq_bytes(uint32_t w, uint32_t c4) {
    uint32_t t = w ^ c4;
    return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
}
// 0x80 in every byte <= 0x20
AJX_HD uint32_t le20_bytes(uint32_t w) {
    uint32_t t = (w & 0x7F7F7F7Fu) + 0x5F5F5F5Fu;
    return ~(t | w) & 0x80808080u;
}
// 0x80-per-byte flags -> 4-bit mask
AJX_HD uint32_t gather4(uint32_t f) {
    uint32_t x = f >> 7;
    return (x | (x >> 7) | (x >> 14) | (x >> 21)) & 0xFu;
}
AJX_HD uint32_t ctz32(uint32_t x) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_ctz(x);
#else
    return (uint32_t)__builtin_ctz(x);
#endif
}
AJX_HD uint32_t popc32(uint32_t x) { return (uint32_t)__builtin_popcount(x); }
AJX_HD uint32_t hibit32(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }

AJX_HD uint32_t byte_of(const uint32_t w[4], uint32_t i) { return (w[i >> 2] >> ((i & 3) * 8)) & 0xFFu; }

// grammar states
enum : uint8_t {
    X_ROOT = 0, X_VALUE, X_VALUE_OR_CLOSE, X_KEY_OR_CLOSE, X_KEY, X_COLON, X_COMMA_OR_CLOSE,
    X_IN_KEY, X_IN_VAL, X_DONE
};

constexpr int kFastDepth = 16;      // trie / element-index tracking depth
constexpr int kCapSlots = 4;        // simultaneously open container captures
constexpr int kArrSlots = 4;        // simultaneously open arrays on selector paths

struct FastOut {
    uint64_t t[2];   // pattern evaluated to T
    uint64_t u[2];   // pattern undecided
    bool slow;
};

// Read 4 bytes at doc position p (any alignment, within [0, n) or zero-filled).
struct DocReader {
    const uint8_t* d;
    uint32_t n;
    AJX_HD uint32_t byte(uint32_t p) const { return p < n ? d[p] : 0u; }
};

AJX_HD bool key_equals_child(const uint8_t* d, uint32_t ks, uint32_t klen, const TrieChild& c, const uint8_t* lits,
                             uint32_t prefix) {
    if (c.key_len != klen || c.prefix != prefix) return false;
    for (uint32_t k = 4; k < klen; k++)
        if (d[ks + k] != lits[c.key_off + k]) return false;
    return true;
}

// Evaluate every pattern on selector `sel` against value v.
AJX_HD void capture(const uint8_t* blob, const uint8_t* doc, uint32_t sel, const ValueRef& v, FastOut* o) {
    const RulesetHdr* h = (const RulesetHdr*)blob;
    const SelectorPatterns& sp = ((const SelectorPatterns*)(blob + h->off_sel_patterns))[sel];
    const uint16_t* pl = (const uint16_t*)(blob + h->off_pattern_lists);
    const Pattern* pats = (const Pattern*)(blob + h->off_patterns);
    for (uint32_t k = 0; k < sp.count; k++) {
        uint32_t p = pl[sp.begin + k];
        uint8_t r = eval_pattern(blob, pats[p], doc, v);
        uint64_t bit = 1ull << (p & 63);
        if (r == V_T) o->t[p >> 6] |= bit;
        else if (r == V_U) o->u[p >> 6] |= bit;
    }
}

// Full single-pass evaluation. `d` = document start, `n` = length. Returns with
// o->slow set when the request must be re-evaluated by the exact scan.
AJX_HD void fast_eval(const uint8_t* blob, const uint8_t* d, uint32_t n, FastOut* o) {
    const RulesetHdr* h = (const RulesetHdr*)blob;
    const TrieNode* tn = (const TrieNode*)(blob + h->off_trie_nodes);
    const TrieChild* tc = (const TrieChild*)(blob + h->off_trie_children);
    const SelectorPatterns* sp = (const SelectorPatterns*)(blob + h->off_sel_patterns);
    const uint8_t* lits = blob + h->off_literals;
    o->t[0] = o->t[1] = o->u[0] = o->u[1] = 0;
    o->slow = false;
    uint64_t found_sel = 0;    // selectors whose value has been captured
    uint64_t found_pat[2] = {0, 0};

    // container stack
    uint64_t is_arr = 0;       // bit d: container at depth d (1-based) is an array
    uint32_t depth = 0;
    uint64_t nodes_lo = ~0ull, nodes_hi = ~0ull;  // trie node per depth 1..16 (kNoNode = none)
    uint8_t st = X_ROOT;
    // pending: trie node the next value belongs to (from the key / element index)
    uint32_t pending = kNoNode;
    // key string
    uint32_t str_open = 0;
    // container captures: selector + depth + start
    uint32_t cap_sel[kCapSlots], cap_depth[kCapSlots], cap_start[kCapSlots];
    uint32_t ncap = 0;
    // live arrays: depth + next element index
    uint32_t arr_depth[kArrSlots], arr_h[kArrSlots];
    uint32_t narr = 0;
    // scalar gap (non-ws bytes outside strings since the last token)
    uint32_t gap_first = 0, gap_last = 0, gap_cnt = 0;
    uint32_t last_bs = 0xFFFFFFFFu;  // position of the last backslash seen (0xFFFFFFFF none)
    // string / escape carries
    uint32_t in_str = 0, esc = 0;

    auto node_at = [&](uint32_t dd) -> uint32_t {
        if (dd == 0) return 0;  // document root
        if (dd > (uint32_t)kFastDepth) return kNoNode;
        uint32_t k = dd - 1;
        uint64_t w = k < 8 ? nodes_lo : nodes_hi;
        return (uint32_t)((w >> ((k & 7) * 8)) & 0xFFu);
    };
    auto set_node = [&](uint32_t dd, uint32_t v) {
        if (dd == 0 || dd > (uint32_t)kFastDepth) return;
        uint32_t k = dd - 1;
        uint64_t m = 0xFFull << ((k & 7) * 8);
        uint64_t x = ((uint64_t)v & 0xFF) << ((k & 7) * 8);
        if (k < 8) nodes_lo = (nodes_lo & ~m) | x;
        else nodes_hi = (nodes_hi & ~m) | x;
    };
    // the value about to start: trie node from the key (objects) or element index (arrays)
    auto value_node = [&]() -> uint32_t {
        if (depth == 0) return 0;
        if (!((is_arr >> depth) & 1)) return pending;
        uint32_t parent = node_at(depth);
        if (parent == kNoNode || !(tn[parent].flags & 1)) return kNoNode;
        for (uint32_t s = 0; s < narr; s++) {
            if (arr_depth[s] != depth) continue;
            uint32_t hh = arr_h[s];
            const TrieNode& pn = tn[parent];
            for (uint32_t c = 0; c < pn.n_children; c++)
                if (tc[pn.child_begin + c].array_index == (int32_t)hh) return tc[pn.child_begin + c].node;
            return kNoNode;
        }
        return kNoNode;
    };
    auto leaf_sel = [&](uint32_t node) -> int32_t {
        if (node == kNoNode) return -1;
        int32_t s = tn[node].selector;
        if (s < 0 || ((found_sel >> s) & 1)) return -1;
        return s;
    };
    auto mark_found = [&](int32_t s) {
        found_sel |= 1ull << s;
        found_pat[0] |= sp[s].mask[0];
        found_pat[1] |= sp[s].mask[1];
    };
    auto open_container = [&](uint32_t c, uint32_t p) -> bool {
        uint32_t node = value_node();
        int32_t s = leaf_sel(node);
        if (depth + 1 >= 63) return false;
        depth++;
        if (c == '[') is_arr |= 1ull << depth;
        else is_arr &= ~(1ull << depth);
        uint32_t live = (node != kNoNode && tn[node].n_children) ? node : kNoNode;
        if (depth > (uint32_t)kFastDepth && live != kNoNode) return false;
        set_node(depth, live);
        if (s >= 0) {
            if (ncap >= (uint32_t)kCapSlots) return false;
            cap_sel[ncap] = (uint32_t)s; cap_depth[ncap] = depth; cap_start[ncap] = p;
            ncap++;
            mark_found(s);
        }
        if (c == '[' && live != kNoNode && (tn[live].flags & 1)) {
            if (narr >= (uint32_t)kArrSlots) return false;
            arr_depth[narr] = depth; arr_h[narr] = 0; narr++;
        }
        st = c == '[' ? X_VALUE_OR_CLOSE : X_KEY_OR_CLOSE;
        return true;
    };
    auto close_container = [&](uint32_t p) {
        if (ncap && cap_depth[ncap - 1] == depth) {
            ncap--;
            ValueRef v;
            v.start = cap_start[ncap]; v.end = p + 1; v.type = T_JSON; v.esc = 0;
            capture(blob, d, cap_sel[ncap], v, o);
        }
        if (narr && arr_depth[narr - 1] == depth) narr--;
        depth--;
        st = depth == 0 ? X_DONE : X_COMMA_OR_CLOSE;
        // the closed container was an element of its parent
        if (depth && ((is_arr >> depth) & 1) && narr && arr_depth[narr - 1] == depth) arr_h[narr - 1]++;
    };
    auto element_done = [&]() {
        // after a scalar / string value inside an array: advance its element index
        if (depth && ((is_arr >> depth) & 1) && narr && arr_depth[narr - 1] == depth) arr_h[narr - 1]++;
    };
    // a scalar occupying the gap [gap_first, gap_last] completed; st is X_VALUE*
    auto scalar_value = [&]() -> bool {
        if (gap_last + 1 - gap_first != gap_cnt) return false;  // ws inside the run
        uint32_t c0 = d[gap_first];
        ValueRef v;
        v.start = gap_first; v.end = gap_last + 1; v.esc = 0;
        bool lit_n = c0 == 'n' && gap_cnt >= 2 && d[gap_first + 1] == 'u';
        if (c0 == 't' || c0 == 'f' || lit_n) {
            // gjson parseLiteral consumes [a-z]*: require exactly the JSON literal
            if (c0 == 't') {
                if (gap_cnt != 4 || d[gap_first + 1] != 'r' || d[gap_first + 2] != 'u' || d[gap_first + 3] != 'e')
                    return false;
                v.type = T_TRUE;
            } else if (c0 == 'f') {
                if (gap_cnt != 5 || d[gap_first + 1] != 'a' || d[gap_first + 2] != 'l' || d[gap_first + 3] != 's' ||
                    d[gap_first + 4] != 'e')
                    return false;
                v.type = T_FALSE;
            } else {
                if (gap_cnt != 4 || d[gap_first + 2] != 'l' || d[gap_first + 3] != 'l') return false;
                v.type = T_NULL;
            }
        } else if (c0 == '-' || c0 == '+' || (c0 >= '0' && c0 <= '9') || c0 == 'i' || c0 == 'I' || c0 == 'N' ||
                   c0 == 'n') {
            v.type = T_NUMBER;  // gjson parseNumber: raw up to whitespace , ] }
        } else {
            return false;
        }
        int32_t s = leaf_sel(value_node());
        if (s >= 0) {
            mark_found(s);
            capture(blob, d, (uint32_t)s, v, o);
        }
        element_done();
        st = X_COMMA_OR_CLOSE;
        return true;
    };

    const uint32_t base_mis = (uint32_t)((uintptr_t)d & 15u);
    const uint32_t* aligned = (const uint32_t*)(d - base_mis);
    const uint32_t nblocks = (n + base_mis + 15) / 16;
    for (uint32_t b = 0; b < nblocks && st != X_DONE; b++) {
        uint32_t w[4];
        w[0] = aligned[b * 4 + 0];
        w[1] = aligned[b * 4 + 1];
        w[2] = aligned[b * 4 + 2];
        w[3] = aligned[b * 4 + 3];
        // valid bytes of this block: doc positions [0, n)
        const int32_t bpos = (int32_t)(b * 16) - (int32_t)base_mis;  // doc position of block byte 0
        uint32_t valid = 0xFFFFu;
        if (bpos < 0) valid &= 0xFFFFu << (uint32_t)(-bpos);
        if (bpos + 16 > (int32_t)n) valid &= 0xFFFFu >> (uint32_t)(bpos + 16 - (int32_t)n);
        uint32_t mq = 0, mbs = 0, mst = 0, mws = 0;
        for (int k = 0; k < 4; k++) {
            uint32_t x = w[k];
            uint32_t lx = x | 0x20202020u;
            mq |= gather4(eq_bytes(x, 0x22222222u)) << (4 * k);
            mbs |= gather4(eq_bytes(x, 0x5C5C5C5Cu)) << (4 * k);
            mst |= gather4(eq_bytes(lx, 0x7B7B7B7Bu) | eq_bytes(lx, 0x7D7D7D7Du) | eq_bytes(x, 0x3A3A3A3Au) |
                           eq_bytes(x, 0x2C2C2C2Cu))
                   << (4 * k);
            mws |= gather4(le20_bytes(x)) << (4 * k);
        }
        mq &= valid; mbs &= valid; mst &= valid; mws &= valid;
        // escapes (odd backslash runs); esc = first byte of this block is escaped
        uint32_t escaped;
        {
            uint32_t bs = mbs & ~esc;
            uint32_t follows = ((bs << 1) | esc) & 0xFFFFu;
            const uint32_t even = 0x5555u;
            uint32_t odd_starts = bs & ~even & ~follows;
            uint32_t seq = odd_starts + bs;
            uint32_t carry = (seq >> 16) & 1u;
            uint32_t inv = (seq << 1) & 0xFFFFu;
            escaped = (even ^ inv) & follows;
            esc = carry;
        }
        const uint32_t carry_bs = last_bs;  // last backslash before this block
        if (mbs) last_bs = (uint32_t)(bpos + (int32_t)hibit32(mbs));
        // last backslash strictly before block bit i
        auto bs_before = [&](uint32_t i) -> uint32_t {
            uint32_t m = mbs & ((1u << i) - 1u);
            return m ? (uint32_t)(bpos + (int32_t)hibit32(m)) : carry_bs;
        };
        const uint32_t qu = mq & ~escaped;
        uint32_t x = qu;
        x ^= x << 1; x ^= x << 2; x ^= x << 4; x ^= x << 8;
        x &= 0xFFFFu;
        const uint32_t instr = in_str ? (x ^ 0xFFFFu) : x;  // 1: inside a string after this byte
        in_str = (instr >> 15) & 1u;
        const uint32_t outside = ~instr & ~qu & valid;         // bytes outside strings (not quotes)
        if (mbs & outside) { o->slow = true; return; }         // backslash outside a string
        const uint32_t st_tok = mst & outside;
        const uint32_t ns = outside & ~mst & ~mws;             // scalar bytes
        uint32_t toks = (st_tok | qu) & 0xFFFFu;
        uint32_t prev_i = 0;  // bits below this already consumed
        while (toks) {
            const uint32_t i = ctz32(toks);
            toks &= toks - 1;
            const uint32_t p = (uint32_t)(bpos + (int32_t)i);
            // scalar bytes in the gap before this token
            const uint32_t g = ns & ((1u << i) - 1u) & ~((1u << prev_i) - 1u);
            if (g) {
                if (gap_cnt == 0) gap_first = (uint32_t)(bpos + (int32_t)ctz32(g));
                gap_last = (uint32_t)(bpos + (int32_t)hibit32(g));
                gap_cnt += popc32(g);
            }
            prev_i = i + 1;
            const uint32_t c = byte_of(w, i);
            if (gap_cnt) {
                if (st != X_VALUE && st != X_VALUE_OR_CLOSE) { o->slow = true; return; }
                if (!scalar_value()) { o->slow = true; return; }
                gap_cnt = 0;
                // a scalar must be followed by , ] } (gjson reads numbers up to them)
                if (c != ',' && c != ']' && c != '}') { o->slow = true; return; }
            }
            switch (st) {
                case X_ROOT:
                    if (c != '{' && c != '[') { o->slow = true; return; }
                    if (!open_container(c, p)) { o->slow = true; return; }
                    break;
                case X_KEY_OR_CLOSE:
                case X_KEY:
                    if (c == '"') { st = X_IN_KEY; str_open = p; break; }
                    if (c == '}' && st == X_KEY_OR_CLOSE) { close_container(p); break; }
                    o->slow = true;
                    return;
                case X_IN_KEY: {
                    // c is the closing quote
                    const uint32_t ks = str_open + 1, klen = p - ks;
                    pending = kNoNode;
                    const uint32_t parent = node_at(depth);
                    if (parent != kNoNode && tn[parent].n_children) {
                        const uint32_t lb = bs_before(i);
                        if (lb != 0xFFFFFFFFu && lb > str_open) { o->slow = true; return; }
                        uint32_t prefix = 0;
                        for (uint32_t k = 0; k < 4 && k < klen; k++) prefix |= (uint32_t)d[ks + k] << (8 * k);
                        const TrieNode& pn = tn[parent];
                        for (uint32_t k = 0; k < pn.n_children; k++) {
                            const TrieChild& ch = tc[pn.child_begin + k];
                            if (key_equals_child(d, ks, klen, ch, lits, prefix)) { pending = ch.node; break; }
                        }
                    }
                    st = X_COLON;
                    break;
                }
                case X_COLON:
                    if (c != ':') { o->slow = true; return; }
                    st = X_VALUE;
                    break;
                case X_VALUE:
                case X_VALUE_OR_CLOSE:
                    if (c == '"') { st = X_IN_VAL; str_open = p; break; }
                    if (c == '{' || c == '[') {
                        if (!open_container(c, p)) { o->slow = true; return; }
                        break;
                    }
                    if (c == ']' && st == X_VALUE_OR_CLOSE) { close_container(p); break; }
                    o->slow = true;
                    return;
                case X_IN_VAL: {
                    int32_t s = leaf_sel(value_node());
                    if (s >= 0) {
                        ValueRef v;
                        v.start = str_open; v.end = p + 1; v.type = T_STRING;
                        const uint32_t lb = bs_before(i);
                        v.esc = (lb != 0xFFFFFFFFu && lb > str_open) ? 1 : 0;
                        mark_found(s);
                        capture(blob, d, (uint32_t)s, v, o);
                    }
                    element_done();
                    st = X_COMMA_OR_CLOSE;
                    break;
                }
                case X_COMMA_OR_CLOSE:
                    if (c == ',') {
                        st = ((is_arr >> depth) & 1) ? X_VALUE : X_KEY;
                        break;
                    }
                    if ((c == '}' && !((is_arr >> depth) & 1)) || (c == ']' && ((is_arr >> depth) & 1))) {
                        close_container(p);
                        break;
                    }
                    o->slow = true;
                    return;
                default:
                    break;  // X_DONE: trailing bytes after the root are never read by gjson
            }
            if (st == X_DONE) break;
        }
        if (st == X_DONE) break;
        // scalar bytes after the last token of this block
        const uint32_t g = ns & ~((1u << prev_i) - 1u) & 0xFFFFu;
        if (g) {
            if (gap_cnt == 0) gap_first = (uint32_t)(bpos + (int32_t)ctz32(g));
            gap_last = (uint32_t)(bpos + (int32_t)hibit32(g));
            gap_cnt += popc32(g);
        }
        if (st == X_ROOT && gap_cnt) { o->slow = true; return; }  // scalar / junk root
    }
    if (st != X_DONE) { o->slow = true; return; }  // unterminated root
    // selectors that found nothing evaluate on Null
    for (int k = 0; k < 2; k++) {
        o->t[k] = (o->t[k] & found_pat[k]) | (h->null_true[k] & ~found_pat[k]);
        o->u[k] &= found_pat[k];
        o->u[k] |= h->unsupported[k];
    }
}

}  // namespace ajx
