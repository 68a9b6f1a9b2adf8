// ajx_fast.h — the single-pass structural scan (stage A) and the pattern stage (stage B).
//
// Stage A, one work-item per request: the document is read once in 64-byte windows of
// aligned dwordx4 loads (the next window prefetched while the current one is
// processed). Each 16-byte block is classified with SWAR byte compares into bitmasks
// (quote, backslash, structural, whitespace); escapes are resolved with the
// branch-free odd-backslash-run rule and string interiors with a prefix-XOR of the
// unescaped quotes, carrying string / escape state from block to block. Only the tokens
// (structural bytes outside strings, string delimiters, scalar runs) go through a JSON
// grammar automaton that follows every selector at once through the ruleset's trie.
// For documents that are valid JSON, gjson v1.14.0 Get returns the first complete path
// match in document order (its scan is a depth-first walk in document order that
// descends only into matching keys and stops at the first hit) — exactly the first key
// or element reached here on the trie node that ends the selector. The value span of
// each selector is written to the request's capture row.
// Anything the automaton can not prove equivalent to gjson's scan (not valid JSON, a
// non-object/array root, a key with escapes on a selector path, more nesting than
// tracked) marks the row `slow`; the exact per-selector scan (ajx_eval_scan) redoes it.
//
// Stage B, one work-item per request: Pattern.Matches (pkg/jsonexp/expressions.go:59-96)
// for every pattern on its selector's captured value (Null when not found), the T
// bitmap, and the And/Or fold (expressions.go:111-154).
#pragma once
#include "ajx_device.h"

namespace ajx {

// capture row: [0] = header (bit 63: slow, bits 0..62: selector found), then one
// 8-byte record per selector: low = start, high = len (24 bits) | type << 24 | esc << 27
constexpr uint64_t kRowSlow = 1ull << 63;

// A capture row in memory: word j at p[j * es]. es = 1: the row's words are contiguous
// (rows indexed by request); es = 64: the wave-interleaved layout of the fused kernels,
// where word j of the 64 work-items of a wave is one 512-B run, so a wave's record
// stores share cache lines and stage B's row reads are coalesced (wave_row).
struct RowRef {
    uint64_t* p;
    uint32_t es;
    AJX_HD RowRef() : p(nullptr), es(1) {}
    AJX_HD RowRef(uint64_t* q, uint32_t e = 1) : p(q), es(e) {}
    AJX_HD RowRef(const uint64_t* q, uint32_t e = 1) : p(const_cast<uint64_t*>(q)), es(e) {}  // (read-only uses)
    AJX_HD uint64_t& operator[](uint32_t j) const { return p[(size_t)j * es]; }
};
// work-item k's row in the wave-interleaved layout of (1 + n_selectors)-word rows
AJX_HD RowRef wave_row(uint64_t* rows, uint32_t row_stride, uint32_t k) {
    return RowRef(rows + (size_t)(k & ~63u) * row_stride + (k & 63u), 64u);
}

AJX_HD uint32_t eq_bytes(uint32_t w, uint32_t c4) {  // 0x80 in every byte equal to c
    uint32_t t = w ^ c4;
    return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
}
AJX_HD uint32_t le20_bytes(uint32_t w) {  // 0x80 in every byte <= 0x20
    uint32_t t = (w & 0x7F7F7F7Fu) + 0x5F5F5F5Fu;
    return ~(t | w) & 0x80808080u;
}
AJX_HD uint32_t gather4(uint32_t f) {  // 0x80-per-byte flags -> 4-bit mask
    uint32_t x = f >> 7;
    return (x | (x >> 7) | (x >> 14) | (x >> 21)) & 0xFu;
}
// the 0x80-per-byte flags of 16 bytes (f_i: bytes 4i..4i+3) -> 16-bit mask, bit 4i + j =
// byte j of f_i: the four dwords' flags are merged into one dword (byte j, bit i), its
// nibbles packed into a 4 x 4 bit matrix and transposed with two delta swaps
AJX_HD uint32_t gather16(uint32_t f0, uint32_t f1, uint32_t f2, uint32_t f3) {
    const uint32_t y = (f0 >> 7) | (f1 >> 6) | (f2 >> 5) | (f3 >> 4);
    const uint32_t t0 = (y | (y >> 4)) & 0x00FF00FFu;
    uint32_t z = (t0 | (t0 >> 8)) & 0xFFFFu;  // bit 4j + i
    uint32_t t = (z ^ (z >> 3)) & 0x0A0Au;
    z ^= t ^ (t << 3);
    t = (z ^ (z >> 6)) & 0x00CCu;
    z ^= t ^ (t << 6);
    return z;  // bit 4i + j
}
AJX_HD uint32_t ctz32(uint32_t x) { return (uint32_t)__builtin_ctz(x); }
AJX_HD uint32_t popc32(uint32_t x) { return (uint32_t)__builtin_popcount(x); }
AJX_HD uint32_t hibit32(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }

enum : uint32_t {
    X_ROOT = 0, X_VALUE, X_VALUE_OR_CLOSE, X_KEY_OR_CLOSE, X_KEY, X_COLON, X_COMMA_OR_CLOSE,
    X_IN_KEY, X_IN_VAL, X_DONE, X_SLOW
};

constexpr uint32_t kFastDepth = 16;  // trie tracking depth

struct Block16 {
    uint32_t x, y, z, w;
};

AJX_HD uint32_t ctz64f(uint64_t x) { return (uint32_t)__builtin_ctzll(x); }
AJX_HD uint32_t hibit64f(uint64_t x) { return 63u - (uint32_t)__builtin_clzll(x); }
AJX_HD uint32_t popc64f(uint64_t x) { return (uint32_t)__builtin_popcountll(x); }
AJX_HD uint64_t below64f(uint32_t i) { return i >= 64 ? ~0ull : ((1ull << i) - 1ull); }
AJX_HD uint64_t lt64(uint32_t i) { return (1ull << i) - 1ull; }  // bits below i, i < 64
AJX_HD uint64_t upto64(uint32_t i) { return ~0ull >> (63u - i); }  // bits 0..i, i < 64

// The document window ring of one work-item: the current and the previous 64-byte
// window. Chunk j (16 B) of the ring — j = (A >> 4) & 7 for the position A relative to
// the document's first aligned 16-B block — sits at j * cstride + lane16, so a wave's
// 16-B accesses to one chunk index are contiguous (conflict-free ds_write_b128).
struct WinRing {
    uint8_t* base;
    uint32_t lane16;   // lane * 16
    uint32_t cstride;  // lanes * 16
    AJX_HD uint32_t off(uint32_t a) const { return ((a >> 4) & 7u) * cstride + lane16 + (a & 15u); }
    AJX_HD uint32_t u8(uint32_t a) const { return base[off(a)]; }
    AJX_HD uint32_t u32a(uint32_t a) const { return *reinterpret_cast<const uint32_t*>(base + off(a)); }  // a % 4 == 0
    AJX_HD uint32_t u32(uint32_t a) const {  // the 4 bytes at a, little-endian
        const uint32_t q = a & ~3u, sh = a & 3u;
        const uint32_t w0 = u32a(q), w1 = u32a(q + 4);
#if defined(__HIP_DEVICE_COMPILE__)
        return __builtin_amdgcn_alignbyte(w1, w0, sh);
#else
        return sh ? (w0 >> (8 * sh)) | (w1 << (32 - 8 * sh)) : w0;
#endif
    }
    AJX_HD uint64_t u64(uint32_t a) const {  // the 8 bytes at a, little-endian
        const uint32_t q = a & ~3u, sh = a & 3u;
        const uint32_t w0 = u32a(q), w1 = u32a(q + 4), w2 = u32a(q + 8);
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh), hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
#else
        const uint32_t lo = sh ? (w0 >> (8 * sh)) | (w1 << (32 - 8 * sh)) : w0;
        const uint32_t hi = sh ? (w1 >> (8 * sh)) | (w2 << (32 - 8 * sh)) : w1;
#endif
        return (uint64_t)lo | ((uint64_t)hi << 32);
    }
    AJX_HD void put(uint32_t a, const Block16& b) {  // a % 16 == 0
#if defined(__HIP_DEVICE_COMPILE__)
        *reinterpret_cast<uint4*>(base + off(a)) = uint4{b.x, b.y, b.z, b.w};
#else
        *reinterpret_cast<Block16*>(base + off(a)) = b;
#endif
    }
};

// Stage-A scanner state (kept in registers; no dynamically indexed arrays). The trie
// tables are read through `tn`/`tc`, which the kernel points at an LDS copy when the
// whole batch uses one ruleset; document bytes a token needs (its byte, a key's last
// 8 bytes, a short scalar) come from the window ring, global memory only on rare paths.
// The document goes by in 64-byte windows: one classification per window and one token
// loop over its 64-bit token mask (a wave runs each loop as long as its busiest lane,
// so wider windows even out the lanes' token counts).
struct Scan {
    const TrieNode* tn;
    const TrieChild* tc;
    const KeySlot* ks;  // key table (1 << (ks_meta & 0xFF) slots)
    uint32_t ks_meta;   // log2 of the slot count | key_probes << 8 (one register for both)
    uint32_t ks_mult;   // key_slot_hash multiplier
    const uint8_t* lits;
    const uint8_t* d;
    RowRef row;     // capture row (header + records)
    uint32_t n;
    WinRing ring;

    uint32_t wa;        // ring position of the current window's byte 0
    int32_t bpos;       // doc position of the current window's byte 0
    uint64_t mbs;       // backslash bits of the current window
    uint32_t carry_bs;  // last backslash before the current window (~0u none)
    uint64_t oq;        // opening-quote bits of the current window
    uint32_t carry_oq;  // last opening quote before the current window
    uint32_t last_oq;

    uint64_t is_arr;    // bit k: container at depth k (1-based) is an array
    uint32_t top_arr;   // (is_arr >> depth) & 1, kept up to date at every push and pop
    uint32_t top_node;  // node_at(depth), kept likewise
    uint64_t nodes_lo;  // trie node per depth 1..8 (kNoNode = none)
    uint64_t nodes_hi;  // depths 9..16
    uint64_t found;     // selectors captured
    uint32_t depth, st, pending, str_open;
    uint32_t gap_first, gap_last, gap_cnt;
    uint32_t last_bs;   // last backslash position (~0u none)
    uint32_t in_str, esc;
    // open container captures (at most 2 nested): sel | depth << 8, start
    uint32_t cap0, cap0_start, cap1, cap1_start, ncap;
    // live arrays on selector paths (at most 2 nested): depth | h << 8
    uint32_t arr0, arr1, narr;

    // (values are selected after they are computed, never by member address: that keeps
    // the scanner state in registers)
    // the 8 document bytes ending just before window offset q (0..64), little-endian
    AJX_HD uint64_t tail8(uint32_t q) const {
        const int32_t a = (int32_t)(wa + q) - 8;
        if (a < 0) return ring.u64(0) << (8 * (uint32_t)(-a));  // (before the first block: zeros)
        return ring.u64((uint32_t)a);
    }
    // window byte i (< 64); wa is a multiple of 64, so its chunk is (wa's half of the
    // ring) | i / 16
    AJX_HD uint32_t byte_at(uint32_t i) const {
        return ring.base[(((wa >> 4) & 4u) | (i >> 4)) * ring.cstride + ring.lane16 + (i & 15u)];
    }
    // opening quote of the string whose closing quote is at window offset i
    AJX_HD uint32_t open_before(uint32_t i) const {
        const uint64_t ob = oq & lt64(i);  // (i < 64: a token's window offset)
        return ob ? (uint32_t)(bpos + (int32_t)hibit64f(ob)) : carry_oq;
    }
    AJX_HD uint32_t last_bs_before(uint32_t i) const {
        const uint64_t mb = mbs & lt64(i);
        return mb ? (uint32_t)(bpos + (int32_t)hibit64f(mb)) : carry_bs;
    }

    AJX_HD uint32_t node_at(uint32_t dd) const {
        if (dd == 0) return 0;
        if (dd > kFastDepth) return kNoNode;
        const uint32_t k = dd - 1;
        const uint64_t lo = nodes_lo, hi = nodes_hi;
        const uint64_t w = k < 8 ? lo : hi;
        return (uint32_t)((w >> ((k & 7) * 8)) & 0xFFu);
    }
    AJX_HD void set_node(uint32_t dd, uint32_t v) {
        if (dd == 0 || dd > kFastDepth) return;
        const uint32_t k = dd - 1;
        const uint64_t m = 0xFFull << ((k & 7) * 8);
        const uint64_t x = ((uint64_t)(v & 0xFF)) << ((k & 7) * 8);
        // (both members stored unconditionally: stores into sibling members from two
        // branches get merged into a store through a selected address, which would push
        // the scanner state out of registers)
        const uint64_t lo = nodes_lo, hi = nodes_hi;
        nodes_lo = k < 8 ? (lo & ~m) | x : lo;
        nodes_hi = k < 8 ? hi : (hi & ~m) | x;
    }
    AJX_HD bool top_is_arr() const { return top_arr != 0; }
    // trie node of the value about to start (key for objects, element index for arrays)
    AJX_HD uint32_t value_node() const {
        if (depth == 0) return 0;
        if (!top_is_arr()) return pending;
        if (!narr) return kNoNode;  // no live array open: the element is off every path
        const uint32_t parent = top_node;
        if (parent == kNoNode || !(tn[parent].flags & 1)) return kNoNode;
        uint32_t h;
        if (narr >= 2 && (arr1 & 0xFF) == depth) h = arr1 >> 8;
        else if (narr >= 1 && (arr0 & 0xFF) == depth) h = arr0 >> 8;
        else return kNoNode;
        const uint32_t cb = tn[parent].child_begin, nc = tn[parent].n_children;
        for (uint32_t c = 0; c < nc; c++)
            if (tc[cb + c].array_index == (int32_t)h) return tc[cb + c].node;
        return kNoNode;
    }
    AJX_HD int32_t leaf_sel(uint32_t node) const {
        if (node == kNoNode) return -1;
        const int32_t s = tn[node].selector;
        if (s < 0 || ((found >> s) & 1)) return -1;
        return s;
    }
    AJX_HD void record(int32_t s, uint32_t start, uint32_t end, uint32_t type, uint32_t esc_) {
        found |= 1ull << s;
        row[1 + s] = (uint64_t)start | ((uint64_t)(((end - start) & 0xFFFFFFu) | (type << 24) | (esc_ << 27)) << 32);
    }
    // a value (scalar, string or container) inside an array completed: next element
    AJX_HD void element_done() {
        if (!narr || !depth || !top_is_arr()) return;
        const uint32_t a0 = arr0, a1 = arr1;
        const bool h1 = narr >= 2 && (a1 & 0xFF) == depth;
        const bool h0 = !h1 && narr >= 1 && (a0 & 0xFF) == depth;
        arr1 = a1 + (h1 ? 0x100u : 0u);
        arr0 = a0 + (h0 ? 0x100u : 0u);
    }
    AJX_HD bool open_container(uint32_t c, uint32_t p) {
        const uint32_t node = value_node();
        if (depth + 1 >= 63) return false;
        depth++;
        const uint64_t bit = 1ull << depth;
        is_arr = c == '[' ? is_arr | bit : is_arr & ~bit;
        top_arr = c == '[' ? 1u : 0u;
        if (node == kNoNode) {  // off every selector path (the common case)
            set_node(depth, kNoNode);
            top_node = kNoNode;
            st = c == '[' ? X_VALUE_OR_CLOSE : X_KEY_OR_CLOSE;
            return true;
        }
        const int32_t s = leaf_sel(node);
        const uint32_t live = tn[node].n_children ? node : kNoNode;
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
        st = c == '[' ? X_VALUE_OR_CLOSE : X_KEY_OR_CLOSE;
        return true;
    }
    AJX_HD void close_container(uint32_t p) {
        // (copies first: a conditional over two lvalue members would select their
        // addresses and force the state out of registers)
        if (ncap) {
            const uint32_t c0 = cap0, c1 = cap1, s0 = cap0_start, s1 = cap1_start;
            const uint32_t cs = ncap == 2 ? c1 : c0;
            if ((cs >> 8) == depth) {
                const uint32_t start = ncap == 2 ? s1 : s0;
                row[1 + (cs & 0xFF)] =
                    (uint64_t)start | ((uint64_t)(((p + 1 - start) & 0xFFFFFFu) | ((uint32_t)T_JSON << 24)) << 32);
                ncap--;
            }
        }
        if (narr) {
            const uint32_t a0 = arr0, a1 = arr1;
            const uint32_t at = narr == 2 ? a1 : a0;
            if ((at & 0xFF) == depth) narr--;
        }
        depth--;
        top_arr = (uint32_t)(is_arr >> depth) & 1u;
        top_node = node_at(depth);
        st = depth == 0 ? X_DONE : X_COMMA_OR_CLOSE;
        element_done();  // the container was an element of its parent array
    }
    // a scalar occupying [gap_first, gap_last] completed in a value position
    AJX_HD bool scalar_value() {
        if (gap_last + 1 - gap_first != gap_cnt) return false;  // whitespace inside the run
        const int32_t qend = (int32_t)gap_last + 1 - bpos;
        const uint32_t m = gap_cnt < 8 ? gap_cnt : 8u;
        uint64_t t8 = 0;  // the scalar's last m bytes in the top m bytes
        if (qend >= 0) {
            t8 = tail8((uint32_t)qend);
        } else {  // trailing whitespace ran past a block boundary
            for (uint32_t j = 0; j < m; j++) t8 |= (uint64_t)d[gap_last + 1 - m + j] << (8 * (8 - m + j));
        }
        uint32_t c0, c1;
        if (gap_cnt <= 8) {
            c0 = (uint32_t)(t8 >> (8 * (8 - gap_cnt))) & 0xFFu;
            c1 = gap_cnt >= 2 ? (uint32_t)(t8 >> (8 * (9 - gap_cnt))) & 0xFFu : 0u;
        } else {
            const uint32_t a0 = gap_first + (wa - (uint32_t)bpos);  // ring position of the first byte
            if (a0 + 64u >= wa) {
                const uint32_t w = ring.u32(a0);
                c0 = w & 0xFFu;
                c1 = (w >> 8) & 0xFFu;
            } else {
                c0 = d[gap_first];
                c1 = d[gap_first + 1];
            }
        }
        uint32_t type;
        if (c0 == 't') {
            if (gap_cnt != 4 || (uint32_t)(t8 >> 32) != 0x65757274u) return false;  // "true"
            type = T_TRUE;
        } else if (c0 == 'f') {
            if (gap_cnt != 5 || (t8 >> 24) != 0x65736C6166ull) return false;  // "false"
            type = T_FALSE;
        } else if (c0 == 'n' && c1 == 'u') {
            if (gap_cnt != 4 || (uint32_t)(t8 >> 32) != 0x6C6C756Eu) return false;  // "null"
            type = T_NULL;
        } else if (c0 == '-' || c0 == '+' || (c0 >= '0' && c0 <= '9') || c0 == 'i' || c0 == 'I' || c0 == 'N' ||
                   c0 == 'n') {
            type = T_NUMBER;  // gjson parseNumber: raw runs to whitespace , ] }
        } else {
            return false;
        }
        const int32_t s = leaf_sel(value_node());
        if (s >= 0) record(s, gap_first, gap_last + 1, type, 0);
        element_done();
        st = X_COMMA_OR_CLOSE;
        return true;
    }
    // closing quote of a key at block offset i (doc position p)
    AJX_HD void key_closed(uint32_t p, uint32_t i) {
        pending = kNoNode;
        const uint32_t parent = top_node;
        if (parent == kNoNode) return;
        // (a live node always has children: open_container stores only those)
        str_open = open_before(i);
        const uint32_t lb = last_bs_before(i);
        if (lb != ~0u && lb > str_open) { st = X_SLOW; return; }  // escaped key on a live path
        const uint32_t k0 = str_open + 1, klen = p - k0;
        uint64_t sig = tail8(i);
        if (klen < 8) sig = klen ? sig >> (8 * (8 - klen)) : 0ull;
        if (klen >= kIndexKeyLen) return;
        const uint32_t log2 = ks_meta & 0xFFu, want = klen | (parent << 16), mask = (1u << log2) - 1u;
        const uint32_t at = key_slot_hash(sig, klen, parent, log2, ks_mult);
        // every key of the table sits within key_probes slots of its home (the compiler grows
        // the table for that), so the probe sequence is bounded by it, not by an empty slot
        uint32_t pos = at;
        for (uint32_t probe = 0; probe < (ks_meta >> 8); probe++, pos = (pos + 1) & mask) {
            const KeySlot slot = ks[pos];
            if (slot.meta == kEmptySlot) return;
            if (slot.sig != sig || (slot.meta & 0xFFFFFFu) != want) continue;
            if (klen <= 8 || key_rest_equal(k0, klen, (uint32_t)slot.key_off8 * 8u)) { pending = slot.meta >> 24; return; }
        }
    }
    // the bytes of a key [k0, k0 + klen) before its last 8 equal the literal at key_off
    AJX_HD bool key_rest_equal(uint32_t k0, uint32_t klen, uint32_t key_off) const {
        const uint8_t* kl = lits + key_off;
        const uint32_t a0 = k0 + (wa - (uint32_t)bpos);  // ring position of the key's first byte
        if (a0 + 64u >= wa) {  // the key began in the ring's windows: compare from LDS
            for (uint32_t k = 0; k + 8 < klen; k += 4) {
                const uint32_t r = klen - 8 - k;
                const uint32_t m = r >= 4 ? 0xFFFFFFFFu : (1u << (8 * r)) - 1u;
                if ((ring.u32(a0 + k) ^ load_u32_any(kl + k)) & m) return false;
            }
            return true;
        }
        for (uint32_t k = 0; k + 8 < klen; k++)
            if (d[k0 + k] != kl[k]) return false;
        return true;
    }

    // a string value closed at block offset i (state X_VALUE / X_VALUE_OR_CLOSE)
    AJX_HD void value_string(uint32_t i) {
        const int32_t s = leaf_sel(value_node());
        if (s >= 0) {
            const uint32_t so = open_before(i);
            const uint32_t lb = last_bs_before(i);
            record(s, so, (uint32_t)(bpos + (int32_t)i) + 1, T_STRING, (lb != ~0u && lb > so) ? 1u : 0u);
        }
        element_done();
        st = X_COMMA_OR_CLOSE;
    }

    // one token at block offset i (byte c). Strings arrive as one token, their closing
    // quote (nothing inside a string is a token, so the state before the opening quote
    // still holds there).
    AJX_HD void token(uint32_t c, uint32_t i) {
        const uint32_t p = (uint32_t)(bpos + (int32_t)i);
        if (gap_cnt) {
            if ((st != X_VALUE && st != X_VALUE_OR_CLOSE) || !scalar_value() || (c != ',' && c != ']' && c != '}')) {
                st = X_SLOW;
                return;
            }
            gap_cnt = 0;
        }
        switch (st) {
            case X_ROOT:
                if ((c != '{' && c != '[') || !open_container(c, p)) st = X_SLOW;
                return;
            case X_KEY_OR_CLOSE:
            case X_KEY:
                if (c == '"') {
                    st = X_COLON;
                    key_closed(p, i);
                    return;
                }
                if (c == '}' && st == X_KEY_OR_CLOSE) { close_container(p); return; }
                st = X_SLOW;
                return;
            case X_COLON:
                st = c == ':' ? X_VALUE : X_SLOW;
                return;
            case X_VALUE:
            case X_VALUE_OR_CLOSE:
                if (c == '"') {
                    value_string(i);
                    return;
                }
                if (c == '{' || c == '[') {
                    if (!open_container(c, p)) st = X_SLOW;
                    return;
                }
                if (c == ']' && st == X_VALUE_OR_CLOSE) { close_container(p); return; }
                st = X_SLOW;
                return;
            case X_COMMA_OR_CLOSE:
                if (c == ',') { st = top_is_arr() ? X_VALUE : X_KEY; return; }
                if ((c == '}' && !top_is_arr()) || (c == ']' && top_is_arr())) { close_container(p); return; }
                st = X_SLOW;
                return;
            default:
                return;
        }
    }

    // process the 64 document bytes of window `blk` (ring position of byte 0 = a, a
    // multiple of 64; doc position of byte 0 = bp)
    template <int MODE = 0>
    AJX_HD void window(const Block16* blk, uint32_t a, int32_t bp) {
        wa = a;
        bpos = bp;
        uint64_t valid = ~0ull;
        if (bp < 0) valid &= ~below64f((uint32_t)(-bp));
        if (bp + 64 > (int32_t)n) valid &= below64f((uint32_t)((int32_t)n - bp));
        uint64_t mq = 0, mst = 0, mws = 0, mb = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const Block16 x4 = blk[j];
            ring.put(a + 16u * (uint32_t)j, x4);
            uint32_t qf[4], bf[4], sf[4], wf[4];  // (0x80-per-byte flags; unrolled: registers)
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t x = k == 0 ? x4.x : k == 1 ? x4.y : k == 2 ? x4.z : x4.w;
                const uint32_t lx = x | 0x20202020u;
                qf[k] = eq_bytes(x, 0x22222222u);
                bf[k] = eq_bytes(x, 0x5C5C5C5Cu);
                sf[k] = eq_bytes(lx, 0x7B7B7B7Bu) | eq_bytes(lx, 0x7D7D7D7Du) | eq_bytes(x, 0x3A3A3A3Au) |
                        eq_bytes(x, 0x2C2C2C2Cu);
                wf[k] = le20_bytes(x);
            }
            const uint32_t q16 = gather16(qf[0], qf[1], qf[2], qf[3]), b16 = gather16(bf[0], bf[1], bf[2], bf[3]);
            const uint32_t s16 = gather16(sf[0], sf[1], sf[2], sf[3]), w16 = gather16(wf[0], wf[1], wf[2], wf[3]);
            mq |= (uint64_t)q16 << (16 * j);
            mb |= (uint64_t)b16 << (16 * j);
            mst |= (uint64_t)s16 << (16 * j);
            mws |= (uint64_t)w16 << (16 * j);
        }
        mq &= valid;
        mb &= valid;
        mst &= valid;
        mws &= valid;
        mbs = mb;
        // escaped bytes: the byte after an odd-length backslash run
        uint64_t escaped;
        {
            const uint64_t bs = mb & ~(uint64_t)esc;
            const uint64_t follows = (bs << 1) | esc;
            const uint64_t even = 0x5555555555555555ull;
            const uint64_t odd_starts = bs & ~even & ~follows;
            const uint64_t seq = odd_starts + bs;
            esc = seq < bs ? 1u : 0u;  // carry out of the window
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
        if (mb & outside) { st = X_SLOW; return; }  // backslash outside any string
        const uint64_t ns = outside & ~mst & ~mws;    // scalar bytes
        // tokens: structural bytes outside strings and closing quotes (an opening quote
        // is the quote after which the string is open)
        oq = qu & instr;
        carry_oq = last_oq;
        if (oq) last_oq = (uint32_t)(bp + (int32_t)hibit64f(oq));
        uint64_t toks = (mst & outside) | (qu & ~instr);
        if constexpr (MODE == 2) {  // ablation: classification only
            gap_cnt += popc64f(toks) + popc64f(ns);
            return;
        }
        uint64_t below = 0;  // bits already consumed
        while (toks) {
            const uint32_t i = ctz64f(toks);
            toks &= toks - 1;
            const uint64_t g = ns & lt64(i) & ~below;
            if (g) {
                if (gap_cnt == 0) gap_first = (uint32_t)(bp + (int32_t)ctz64f(g));
                gap_last = (uint32_t)(bp + (int32_t)hibit64f(g));
                gap_cnt += popc64f(g);
            }
            below = upto64(i);
            token(byte_at(i), i);
            if (st >= X_DONE) return;
            // compact JSON: the ':' right after a key and the ',' right after a value are
            // taken in the same iteration, and so is a member's string value that opens
            // right after its ':' ("key":"value", — one iteration per member)
            const uint32_t nb = i + 1;
            if (toks & (2ull << i)) {  // (a token at i + 1; none when i = 63)
                const uint32_t c2 = byte_at(nb);
                const bool colon = st == X_COLON && c2 == ':';
                const bool comma = st == X_COMMA_OR_CLOSE && c2 == ',';
                if (colon || comma) {
                    st = (colon || top_is_arr()) ? X_VALUE : X_KEY;
                    toks &= toks - 1;
                    below = upto64(nb);
                    // the opening quote right after the ':' and its closing quote in this
                    // window (nothing inside a string is a token: it is the next token)
                    if (colon && (oq & (4ull << i)) && toks) {
                        const uint32_t j = ctz64f(toks);
                        toks &= toks - 1;
                        below = upto64(j);
                        value_string(j);
                        const uint32_t nb2 = j + 1;
                        if ((toks & (2ull << j)) && byte_at(nb2) == ',') {
                            st = top_is_arr() ? X_VALUE : X_KEY;
                            toks &= toks - 1;
                            below = upto64(nb2);
                        }
                    }
                }
            }
        }
        const uint64_t g = ns & ~below;
        if (g) {
            if (gap_cnt == 0) gap_first = (uint32_t)(bp + (int32_t)ctz64f(g));
            gap_last = (uint32_t)(bp + (int32_t)hibit64f(g));
            gap_cnt += popc64f(g);
            if (st == X_ROOT) st = X_SLOW;  // a scalar (or junk) before the root container
        }
    }
};

// the single-pass path's lookup tables of a ruleset (the blob's own, or an LDS copy)
struct Tables {
    const TrieNode* tn;
    const TrieChild* tc;
    const KeySlot* ks;
};
AJX_HD Tables blob_tables(const uint8_t* blob) {
    const RulesetHdr* h = (const RulesetHdr*)blob;
    return Tables{(const TrieNode*)(blob + h->off_trie_nodes), (const TrieChild*)(blob + h->off_trie_children),
                  (const KeySlot*)(blob + h->off_key_slots)};
}

// Stage A for one request. `row` = capture row (1 + n_selectors u64); `ring` = the
// work-item's window ring (128 B). Returns true when the row is valid (false: the
// request needs the exact scan).
// MODE (profiling ablations only): 0 = full scan, 1 = loads only, 2 = loads + classification
template <int MODE = 0, class LoadBlock>
AJX_HD bool scan_doc(const uint8_t* blob, const Tables& tab, const uint8_t* d, uint32_t n, RowRef row,
                     const WinRing& ring, LoadBlock load) {
    const RulesetHdr* h = (const RulesetHdr*)blob;
    Scan s;
    s.tn = tab.tn;
    s.tc = tab.tc;
    s.ks = tab.ks;
    s.ks_meta = h->key_slots_log2 | h->key_probes << 8;
    s.ks_mult = h->key_mult;
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

    const uint32_t mis = (uint32_t)((uintptr_t)d & 15u);
    const uint32_t nblk = (n + mis + 15) / 16;
    Block16 cur[4], nxt[4];
#pragma unroll
    for (int j = 0; j < 4; j++) cur[j] = load((uint32_t)j, nblk);
#pragma unroll
    for (int j = 0; j < 4; j++) nxt[j] = load((uint32_t)(4 + j), nblk);
    for (uint32_t b0 = 0; b0 < nblk; b0 += 4) {
        if constexpr (MODE == 1) {
            s.found ^= (uint64_t)(cur[0].x ^ cur[1].y ^ cur[2].z ^ cur[3].w) << (b0 & 31);
        } else {
            s.window<MODE>(cur, b0 * 16, (int32_t)(b0 * 16) - (int32_t)mis);
        }
        if (s.st >= X_DONE) break;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            cur[j] = nxt[j];
            nxt[j] = load(b0 + 8 + (uint32_t)j, nblk);
        }
    }
    if constexpr (MODE != 0) {
        row[0] = s.found + s.gap_cnt;
        return true;
    }
    if (s.st != X_DONE) {
        row[0] = kRowSlow;
        return false;
    }
    row[0] = s.found;
    return true;
}

// the 4 bytes at p when only `avail` (>= 1) of them are readable: no aligned dword past
// the one holding p[avail - 1] is touched (bytes past it are garbage)
AJX_HD uint32_t load_u32_upto(const uint8_t* p, uint32_t avail) {
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t* q = (const uint32_t*)(p - sh);
    const uint32_t w0 = q[0];
    const uint32_t w1 = (sh && avail > 4u - sh) ? q[1] : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbyte(w1, w0, sh);
#else
    return sh ? (w0 >> (8 * sh)) | (w1 << (32 - 8 * sh)) : w0;
#endif
}

// A JSON number that is its own FormatFloat(f, 'f', -1, 64) (gjson Result.String() of a
// non-integer Number): (0|[1-9][0-9]*)\.[0-9]*[1-9] with at most 15 digits in all — a
// decimal of <= 15 significant digits is the only such decimal that parses to its double,
// so the shortest round-trip digits are its own (the sign is handled by the caller).
AJX_HD bool simple_decimal(const uint8_t* s, uint32_t n) {
    if (n < 3 || n > 16) return false;
    uint32_t i = 0, nd = 0;
    if (s[0] == '0') {
        i = 1;
        nd = 1;
    } else {
        while (i < n && s[i] >= '0' && s[i] <= '9') i++;
        nd = i;
        if (i == 0) return false;
    }
    if (i >= n || s[i] != '.') return false;
    const uint32_t f0 = ++i;
    while (i < n && s[i] >= '0' && s[i] <= '9') i++;
    if (i != n || i == f0 || s[n - 1] == '0') return false;
    return nd + (n - f0) <= 15;
}

struct RawVal {
    uint32_t a, n;  // span in the document
    uint32_t lit;   // 0 span, kLitTrue / kLitFalse / kLitEmpty for the literals
    bool ok;        // false: the general path formats it
};
AJX_HD RawVal raw_value(const uint8_t* doc, const ValueRef& v) {
    RawVal r{v.start, v.end - v.start, 0u, true};
    switch (v.type) {
        case T_STRING:
            r.a = v.start + 1;
            r.n = v.end - v.start - 2;
            r.ok = !v.esc;
            break;
        case T_NUMBER: {
            uint32_t k = v.start;
            if (k < v.end && doc[k] == '-') k++;
            const uint32_t k0 = k;
            for (; k < v.end; k += 4) {  // -?[0-9]* is its own String()
                const uint32_t w = load_u32_upto(doc + k, v.end - k);
                const uint32_t m = v.end - k >= 4 ? 0xFFFFFFFFu : (1u << (8 * (v.end - k))) - 1u;
                const uint32_t d = w ^ 0x30303030u;
                if ((((d + 0x76767676u) | d) & 0x80808080u) & m) { r.ok = false; break; }
            }
            if (!r.ok) r.ok = simple_decimal(doc + k0, v.end - k0);
            break;
        }
        case T_TRUE: r.lit = kLitTrue; r.n = 4; break;
        case T_FALSE: r.lit = kLitFalse; r.n = 5; break;
        case T_JSON: break;
        default: r.lit = kLitEmpty; r.n = 0; break;  // Null: ""
    }
    return r;
}

// `matches` on a raw span: ASCII four bytes at a time, utf8.DecodeRune otherwise (the
// S_RAW branch of dfa_match without a StrSrc)
AJX_HD bool dfa_match_span(const uint8_t* blob, uint32_t dfa_off, const uint8_t* p, uint32_t n) {
    const DfaHdr* h = (const DfaHdr*)(blob + dfa_off);
    const uint16_t* tr = (const uint16_t*)(blob + h->trans_off);
    const uint32_t nc = h->n_classes, ms = h->match_state;
    uint32_t st = h->start;
    if (st == ms) return true;
    uint32_t i = 0;
    // 16 ASCII bytes per step: the five aligned dwords that hold them are loaded together
    // (one memory latency per 16 bytes instead of one per dword: the span was read by stage
    // A long before and has left the caches); every dword loaded holds a byte of the span
    while (i + 16 <= n) {
        const uint32_t sh = (uint32_t)((uintptr_t)(p + i) & 3u);
        const uint32_t* q = (const uint32_t*)(p + i - sh);
        const uint32_t a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3], a4 = sh ? q[4] : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t w[4] = {__builtin_amdgcn_alignbyte(a1, a0, sh), __builtin_amdgcn_alignbyte(a2, a1, sh),
                               __builtin_amdgcn_alignbyte(a3, a2, sh), __builtin_amdgcn_alignbyte(a4, a3, sh)};
#else
        const uint64_t s8 = 8ull * sh;
        const uint32_t w[4] = {(uint32_t)((((uint64_t)a1 << 32) | a0) >> s8), (uint32_t)((((uint64_t)a2 << 32) | a1) >> s8),
                               (uint32_t)((((uint64_t)a3 << 32) | a2) >> s8), (uint32_t)((((uint64_t)a4 << 32) | a3) >> s8)};
#endif
        if ((w[0] | w[1] | w[2] | w[3]) & 0x80808080u) break;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            st = tr[st * nc + h->ascii_class[(w[k >> 2] >> (8 * (k & 3))) & 0x7Fu]];
            if (st == ms) return true;
        }
        i += 16;
    }
    while (i < n) {
        if (i + 4 <= n) {
            const uint32_t w = load_u32_any(p + i);
            if (!(w & 0x80808080u)) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    st = tr[st * nc + h->ascii_class[(w >> (8 * k)) & 0x7Fu]];
                    if (st == ms) return true;
                }
                i += 4;
                continue;
            }
        }
        const uint32_t b0 = p[i];
        int32_t r = (int32_t)b0;
        uint32_t sz = 1;
        if (b0 >= 0x80) {
            r = 0xFFFD;
            uint32_t need = 0, lo = 0x80, hi = 0xBF, v = 0;
            if (b0 >= 0xC2 && b0 <= 0xDF) { need = 2; v = b0 & 0x1F; }
            else if (b0 >= 0xE0 && b0 <= 0xEF) {
                need = 3; v = b0 & 0x0F;
                if (b0 == 0xE0) lo = 0xA0;
                if (b0 == 0xED) hi = 0x9F;
            } else if (b0 >= 0xF0 && b0 <= 0xF4) {
                need = 4; v = b0 & 0x07;
                if (b0 == 0xF0) lo = 0x90;
                if (b0 == 0xF4) hi = 0x8F;
            }
            if (need && n - i >= need && p[i + 1] >= lo && p[i + 1] <= hi) {
                bool good = true;
                v = (v << 6) | (p[i + 1] & 0x3Fu);
                for (uint32_t k = 2; k < need; k++) {
                    const uint32_t c = p[i + k];
                    if (c < 0x80 || c > 0xBF) { good = false; break; }
                    v = (v << 6) | (c & 0x3Fu);
                }
                if (good) { r = (int32_t)v; sz = need; }
            }
        }
        i += sz;
        st = tr[st * nc + rune_class(h, blob, r)];
        if (st == ms) return true;
    }
    return blob[h->eot_off + st] != 0;
}
// `matches` on a literal's text ("true" / "false" / ""), from registers
AJX_HD bool dfa_match_lit(const uint8_t* blob, uint32_t dfa_off, uint32_t lit) {
    const DfaHdr* h = (const DfaHdr*)(blob + dfa_off);
    const uint16_t* tr = (const uint16_t*)(blob + h->trans_off);
    const uint32_t nc = h->n_classes, ms = h->match_state;
    uint32_t st = h->start;
    if (st == ms) return true;
    const uint64_t text = lit == kLitTrue ? 0x65757274ull : lit == kLitFalse ? 0x65736C6166ull : 0ull;
    const uint32_t n = lit == kLitTrue ? 4u : lit == kLitFalse ? 5u : 0u;
    for (uint32_t k = 0; k < n; k++) {
        st = tr[st * nc + h->ascii_class[(text >> (8 * k)) & 0x7Fu]];
        if (st == ms) return true;
    }
    return blob[h->eot_off + st] != 0;
}

// The gjson unescape of a string's contents as a byte stream (StrSrc::S_UNESC) with
// every byte of state in registers: the UTF-8 bytes of a \u escape wait packed in `pend`.
struct UnescSrc {
    const uint8_t* p;
    uint32_t i, n;
    uint32_t pend, npend;
    bool done;
    AJX_HD void init(const uint8_t* s, uint32_t a, uint32_t b) {
        p = s;
        i = a;
        n = b;
        pend = npend = 0;
        done = false;
    }
    AJX_HD int next() {
        if (npend) {
            const int c = (int)(pend & 0xFFu);
            pend >>= 8;
            npend--;
            return c;
        }
        if (done || i >= n) return -1;
        const uint8_t c = p[i];
        if (c < ' ') { done = true; return -1; }
        if (c != '\\') { i++; return c; }
        i++;
        if (i >= n) { done = true; return -1; }
        const uint8_t e = p[i];
        uint8_t out;
        switch (e) {
            case '\\': out = '\\'; break;
            case '/': out = '/'; break;
            case 'b': out = '\b'; break;
            case 'f': out = '\f'; break;
            case 'n': out = '\n'; break;
            case 'r': out = '\r'; break;
            case 't': out = '\t'; break;
            case '"': out = '"'; break;
            case 'u': {
                if (i + 5 > n) { done = true; return -1; }
                uint32_t r = hexval4(p + i + 1);
                i += 5;
                if (r >= 0xD800 && r < 0xE000) {
                    if (n - i >= 6 && p[i] == '\\' && p[i + 1] == 'u') {
                        const uint32_t r2 = hexval4(p + i + 2);
                        if (r < 0xDC00 && r2 >= 0xDC00 && r2 < 0xE000)
                            r = (((r - 0xD800) << 10) | (r2 - 0xDC00)) + 0x10000;
                        else
                            r = 0xFFFD;
                        i += 6;
                    }
                }
                // utf8_put, packed low byte first
                if (r > 0x10FFFF || (r >= 0xD800 && r <= 0xDFFF)) r = 0xFFFD;
                uint32_t b;
                uint32_t k;
                if (r < 0x80) { b = r; k = 1; }
                else if (r < 0x800) { b = (0xC0 | (r >> 6)) | ((0x80 | (r & 0x3F)) << 8); k = 2; }
                else if (r < 0x10000) {
                    b = (0xE0 | (r >> 12)) | ((0x80 | ((r >> 6) & 0x3F)) << 8) | ((0x80 | (r & 0x3F)) << 16);
                    k = 3;
                } else {
                    b = (0xF0 | (r >> 18)) | ((0x80 | ((r >> 12) & 0x3F)) << 8) | ((0x80 | ((r >> 6) & 0x3F)) << 16) |
                        ((0x80 | (r & 0x3F)) << 24);
                    k = 4;
                }
                pend = b >> 8;
                npend = k - 1;
                return (int)(b & 0xFFu);
            }
            default: done = true; return -1;
        }
        i++;
        return out;
    }
};

// stream == literal (UnescSrc)
AJX_HD bool unesc_equals(UnescSrc* s, const uint8_t* lit, uint32_t len) {
    for (uint32_t k = 0; k < len; k++)
        if (s->next() != (int)lit[k]) return false;
    return s->next() < 0;
}

// `matches` over a UnescSrc: utf8.DecodeRune over the stream with the (up to 4) bytes
// of lookahead packed in a register (RuneReader, without its arrays)
AJX_HD bool dfa_match_unesc(const uint8_t* blob, uint32_t dfa_off, UnescSrc* s) {
    const DfaHdr* h = (const DfaHdr*)(blob + dfa_off);
    const uint16_t* tr = (const uint16_t*)(blob + h->trans_off);
    const uint32_t nc = h->n_classes, ms = h->match_state;
    uint32_t st = h->start;
    if (st == ms) return true;
    uint32_t la = 0, nla = 0;
    for (;;) {
        while (nla < 4) {
            const int c = s->next();
            if (c < 0) break;
            la |= (uint32_t)c << (8 * nla);
            nla++;
        }
        if (nla == 0) break;
        const uint32_t b0 = la & 0xFFu;
        uint32_t sz = 1;
        int32_t r = (int32_t)b0;
        if (b0 >= 0x80) {
            r = 0xFFFD;
            uint32_t need = 0, lo = 0x80, hi = 0xBF, v = 0;
            if (b0 >= 0xC2 && b0 <= 0xDF) { need = 2; v = b0 & 0x1F; }
            else if (b0 >= 0xE0 && b0 <= 0xEF) {
                need = 3; v = b0 & 0x0F;
                if (b0 == 0xE0) lo = 0xA0;
                if (b0 == 0xED) hi = 0x9F;
            } else if (b0 >= 0xF0 && b0 <= 0xF4) {
                need = 4; v = b0 & 0x07;
                if (b0 == 0xF0) lo = 0x90;
                if (b0 == 0xF4) hi = 0x8F;
            }
            const uint32_t b1 = (la >> 8) & 0xFFu;
            if (need && nla >= need && b1 >= lo && b1 <= hi) {
                bool good = true;
                v = (v << 6) | (b1 & 0x3Fu);
                for (uint32_t k = 2; k < need; k++) {
                    const uint32_t c = (la >> (8 * k)) & 0xFFu;
                    if (c < 0x80 || c > 0xBF) { good = false; break; }
                    v = (v << 6) | (c & 0x3Fu);
                }
                if (good) { r = (int32_t)v; sz = need; }
            }
        }
        la = sz == 4 ? 0u : la >> (8 * sz);
        nla -= sz;
        st = tr[st * nc + rune_class(h, blob, r)];
        if (st == ms) return true;
    }
    return blob[h->eot_off + st] != 0;
}

// eq on a raw value
AJX_HD bool raw_equals(const uint8_t* doc, const RawVal& r, const Pattern& pt, const uint8_t* lits) {
    if (r.lit) return (pt.litf & r.lit) != 0;
    return r.n == pt.lit_len && bytes_equal(doc + r.a, lits + pt.lit_off, r.n);
}

// incl / excl of every such pattern of one selector, the array walked once: bit j of the
// result = pattern j of the selector's list found among the elements. Compact arrays of
// unescaped strings / integers / literals only; false sends the selector to the general
// path (whitespace, escapes, nested containers, non-integer numbers, a non-array value).
AJX_HD bool incl_hits(const uint8_t* doc, const ValueRef& v, const Pattern* pats, const uint16_t* plist,
                      uint32_t begin, uint32_t cnt, const uint8_t* lits, uint32_t* hits) {
    uint32_t h = 0;
    if (v.type != T_JSON || v.end - v.start < 2 || doc[v.start] != '[') return false;
    uint32_t i = v.start + 1;
    const uint32_t end = v.end - 1;  // the ']'
    if (doc[end] != ']') return false;
    while (i < end) {
        ValueRef e;
        const uint32_t c = doc[i];
        e.start = i;
        e.esc = 0;
        if (c == '"') {  // the closing quote: the first '"' or '\\' after i
            uint32_t k = i + 1;
            for (;;) {
                if (k >= end) return false;
                const uint32_t w = load_u32_upto(doc + k, end + 1 - k);
                const uint32_t m = end - k >= 4 ? 0xFFFFFFFFu : (1u << (8 * (end - k))) - 1u;
                const uint32_t f = (eq_bytes(w, 0x22222222u) | eq_bytes(w, 0x5C5C5C5Cu)) & m;
                if (f) {
                    k += (uint32_t)__builtin_ctz(f) >> 3;
                    break;
                }
                k += 4;
            }
            if (doc[k] != '"') return false;  // an escape
            e.end = k + 1;
            e.type = T_STRING;
        } else if (c == 't' || c == 'f' || c == 'n') {
            const uint32_t w = load_u32_upto(doc + i, end + 1 - i);
            if (w == 0x65757274u) { e.end = i + 4; e.type = T_TRUE; }
            else if (w == 0x6C6C756Eu) { e.end = i + 4; e.type = T_NULL; }
            else if (w == 0x736C6166u && i + 4 < end && doc[i + 4] == 'e') { e.end = i + 5; e.type = T_FALSE; }
            else return false;
        } else if (c == '-' || (c >= '0' && c <= '9')) {
            uint32_t k = i + 1;
            while (k < end && doc[k] != ',') {
                if (doc[k] <= ' ') return false;  // (gjson's number ends there: the general path)
                k++;
            }
            e.end = k;
            e.type = T_NUMBER;
        } else {
            return false;
        }
        const RawVal r = raw_value(doc, e);
        if (!r.ok) return false;
        if (!r.lit && r.n <= 8) {
            // a short element (the common case: group / role names): its bytes are read
            // from the document once, into two masked dwords, and compared with each
            // literal's dwords (4-byte aligned in the pool, LDS when the blob is staged)
            const uint32_t n0 = r.n < 4 ? r.n : 4u, n1 = r.n - n0;
            const uint32_t m0 = n0 == 4 ? 0xFFFFFFFFu : (1u << (8 * n0)) - 1u;
            const uint32_t m1 = n1 == 4 ? 0xFFFFFFFFu : (1u << (8 * n1)) - 1u;
            const uint32_t w0 = n0 ? load_u32_upto(doc + r.a, n0) & m0 : 0u;
            const uint32_t w1 = n1 ? load_u32_upto(doc + r.a + 4, n1) & m1 : 0u;
            for (uint32_t j = 0; j < cnt; j++) {
                const Pattern pt = pats[plist[begin + j]];
                if ((pt.op != OP_INCL && pt.op != OP_EXCL) || pt.state != P_OK || pt.lit_len != r.n) continue;
                const uint32_t* lw = reinterpret_cast<const uint32_t*>(lits + pt.lit_off);
                if ((lw[0] & m0) == w0 && (n1 == 0 || (lw[1] & m1) == w1)) h |= 1u << j;
            }
        } else {
            for (uint32_t j = 0; j < cnt; j++) {
                const Pattern pt = pats[plist[begin + j]];
                if ((pt.op == OP_INCL || pt.op == OP_EXCL) && pt.state == P_OK && raw_equals(doc, r, pt, lits))
                    h |= 1u << j;
            }
        }
        i = e.end;
        if (i < end) {
            if (doc[i] != ',') return false;
            i++;
            if (i == end) return false;  // "[1,]"
        }
    }
    *hits = h;
    return true;
}

// The fold of a ruleset flagged kFlagFlatFold (one flat All / Any of patterns 0..n - 1 in
// order, n <= 64): the first pattern that is not the group's identity decides, read off the
// bitmaps (run_fold_bits' result, without interpreting the code)
AJX_HD uint8_t flat_fold(const RulesetHdr* h, const uint32_t* code, const uint64_t t[2], const uint64_t u[2],
                         const uint64_t se[2], int32_t* ep) {
    const bool any = (code[0] >> 24) == C_OPEN_OR;
    const uint32_t np = h->n_patterns;
    const uint64_t pm = np >= 64 ? ~0ull : (1ull << np) - 1ull;
    const uint64_t stick = pm & (se[0] | u[0] | (any ? t[0] : ~t[0]));  // (E and U are never the identity)
    *ep = -1;
    if (!stick) return any ? (uint8_t)V_F : (uint8_t)V_T;
    const uint32_t k = (uint32_t)__builtin_ctzll(stick);
    const uint8_t v = ((se[0] >> k) & 1u) ? (uint8_t)V_E : ((u[0] >> k) & 1u) ? (uint8_t)V_U
                    : ((t[0] >> k) & 1u) ? (uint8_t)V_T : (uint8_t)V_F;
    if (v == V_E || v == V_U) *ep = (int32_t)k;
    return v;
}

// The fold of a ruleset flagged kFlagGroupFold (one All / Any over patterns and groups of
// the other kind, patterns 0..n - 1 in code order). A child decides the outer group when
// its value is not the outer identity; a group's value is its first pattern that is not
// the group's identity (or the identity when there is none). The lone patterns that
// decide come off the bitmaps at once; the groups before the first of them are taken in
// order, one bitmap step each (run_fold_bits' result, without interpreting the code).
// (fold_masks: patterns 0..np - 1 of one tree's own bitmaps t0 / u0 / s0 and its group
// masks; *ep is the tree's pattern, from 0)
AJX_HD uint8_t fold_masks(bool any, uint32_t np, uint64_t g_any, uint64_t g_in, uint64_t g_start, uint64_t t0,
                          uint64_t u0, uint64_t s0, int32_t* ep) {
    const uint64_t pm = np >= 64 ? ~0ull : (1ull << np) - 1ull;
    const uint64_t se[1] = {s0}, u[1] = {u0};
    const uint64_t eu = s0 | u0;
    const uint64_t lone = pm & ~g_in & (eu | (any ? t0 : ~t0));   // lone patterns that decide
    const uint64_t inner = g_in & (eu | (g_any & t0) | (~g_any & ~t0));  // not their group's identity
    const uint32_t kl = lone ? (uint32_t)__builtin_ctzll(lone) : 64u;
    const uint8_t ident = any ? (uint8_t)V_F : (uint8_t)V_T;
    auto value = [&](uint32_t k) -> uint8_t {
        return ((se[0] >> k) & 1u) ? (uint8_t)V_E : ((u[0] >> k) & 1u) ? (uint8_t)V_U
             : ((t0 >> k) & 1u) ? (uint8_t)V_T : (uint8_t)V_F;
    };
    *ep = -1;
    uint64_t g = g_start;
    while (g) {
        const uint32_t lo = (uint32_t)__builtin_ctzll(g);
        if (lo > kl) break;
        g &= g - 1ull;
        // the group runs to the next group's first pattern or the next lone pattern
        const uint64_t above = lo >= 63 ? 0ull : ~0ull << (lo + 1);
        const uint64_t ends = (g | ~g_in) & above;
        const uint64_t range = (ends ? ((1ull << __builtin_ctzll(ends)) - 1ull) : ~0ull) & ~((1ull << lo) - 1ull);
        const uint64_t s = inner & range;
        if (!s) {  // the group's identity, the other kind's: it decides
            const uint8_t v = ((g_any >> lo) & 1u) ? (uint8_t)V_F : (uint8_t)V_T;
            if (v != ident) return v;
            continue;
        }
        const uint32_t k = (uint32_t)__builtin_ctzll(s);
        const uint8_t v = value(k);
        if (v != ident) {
            if (v == V_E || v == V_U) *ep = (int32_t)k;
            return v;
        }
    }
    if (kl == 64u) return ident;
    const uint8_t v = value(kl);
    if (v == V_E || v == V_U) *ep = (int32_t)kl;
    return v;
}
AJX_HD uint8_t group_fold(const RulesetHdr* h, const uint32_t* code, const uint64_t t[2], const uint64_t u[2],
                          const uint64_t se[2], int32_t* ep) {
    return fold_masks((code[0] >> 24) == C_OPEN_OR, h->n_patterns, h->fold_grp[0], h->fold_grp[1], h->fold_grp[2],
                      t[0], u[0], se[0], ep);
}
// bits base .. base + n - 1 of a 128-bit bitmap (n <= 64, base + n <= 128)
AJX_HD uint64_t bits_at(const uint64_t w[2], uint32_t base, uint32_t n) {
    const uint64_t lo = base >= 64 ? w[1] >> (base - 64u) : base ? (w[0] >> base) | (w[1] << (64u - base)) : w[0];
    return n >= 64 ? lo : lo & ((1ull << n) - 1ull);
}
// a forest's tree with a TreeFold shape: its fold off its own bits of the bitmaps
AJX_HD uint8_t tree_fold(const TreeFold& f, const uint64_t t[2], const uint64_t u[2], const uint64_t se[2],
                         int32_t* ep) {
    const uint8_t v = fold_masks(f.any != 0, f.n, f.g_any, f.g_in, f.g_start, bits_at(t, f.base, f.n),
                                 bits_at(u, f.base, f.n), bits_at(se, f.base, f.n), ep);
    if (*ep >= 0) *ep += (int32_t)f.base;
    return v;
}

// Stage B's values from LDS. In the lean kernel each lane's 128-byte share of the wave's
// ring is free once stage A is done (and no load of it is in flight), so stage B copies a
// captured value of up to kSpanMax bytes there and reads it from LDS: the value's aligned
// 16-byte blocks (at most eight) are loaded together, one memory latency per value, where
// walking it in memory costs one latency per dependent read (an array: about five per
// element; an escaped string: one per byte; a short literal compare: one per byte). The
// copy is contiguous, lane l's at l * kSpanStride in the wave's ring: 29 dwords, an odd
// count, so the lanes' reads at one offset fall in different banks.
constexpr uint32_t kSpanStride = 116;
constexpr uint32_t kSpanMax = 112;
// copy doc bytes [a, a + n) to buf (4-byte aligned): returns the offset in buf of byte a
// (a's offset in its dword; the dwords that hold the span are copied whole), or ~0u when
// they do not fit (more than kSpanStride bytes, or more than eight 16-byte blocks)
AJX_HD uint32_t stage_span(const uint8_t* src, uint32_t n, uint8_t* buf) {
    const uint32_t m16 = (uint32_t)((uintptr_t)src & 15u), sh = m16 & 3u;
    const uint32_t nb = (m16 + n + 15u) / 16u, nd = (sh + n + 3u) / 4u;
    if (nb > 8 || nd * 4u > kSpanStride || n == 0) return ~0u;
#if defined(__HIPCC__)
    using V16 = uint4;
#else
    using V16 = Block16;
#endif
    const V16* a4 = reinterpret_cast<const V16*>(src - m16);
    V16 blk[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; j++) blk[j] = a4[j < nb ? j : nb - 1u];
    // dword k of block j is the span's dword 4 j + k - m16 / 4
    uint32_t* bw = reinterpret_cast<uint32_t*>(buf);
#if !defined(__HIPCC__)
    // (host test builds: the bytes around the copy are poison, so that a read outside the
    // value's span shows as a wrong answer against the oracle)
    for (uint32_t k = 0; k < kSpanStride; k++) buf[k] = (k & 1u) ? 0x5Cu : 0x22u;
#endif
    const int32_t d0 = -(int32_t)(m16 >> 2);
#pragma unroll
    for (uint32_t j = 0; j < 8; j++) {
        const uint32_t x[4] = {blk[j].x, blk[j].y, blk[j].z, blk[j].w};
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const int32_t d = d0 + (int32_t)(4 * j + k);
            if (d >= 0 && d < (int32_t)nd) bw[d] = x[k];
        }
    }
    return sh;
}

// Stage B for one request: patterns on the captured values, bitmap, fold.
// res(p) values are V_T / V_F / V_E / V_U.
// (s0, sstep: the selectors s0, s0 + sstep, ... only — the lanes of a wave sharing one
// request's stage B; their t / u OR together)
// (ring: the lane's span buffer when the kernel has one free (the lean kernel's, see
// stage_span); nullptr: values are read in memory)
AJX_HD void patterns_from_row(const uint8_t* blob, const uint8_t* doc, RowRef row, uint64_t t[2],
                              uint64_t u[2], const uint64_t* dec = nullptr, uint32_t s0 = 0, uint32_t sstep = 1,
                              uint8_t* ring = nullptr) {
    // selector by selector: each captured value is decoded once for all its patterns;
    // when its String() is a byte span or a literal, eq/neq compare a dword at a time,
    // `matches` runs the DFA straight over the span and incl/excl walk a compact array
    // once for all of the selector's patterns; other values take eval_pattern
    const RulesetHdr* h = (const RulesetHdr*)blob;
    const Pattern* pats = (const Pattern*)(blob + h->off_patterns);
    const SelectorPatterns* sps = (const SelectorPatterns*)(blob + h->off_sel_patterns);
    const uint16_t* plist = (const uint16_t*)(blob + h->off_pattern_lists);
    const uint8_t* lits = blob + h->off_literals;
    const uint64_t found = row[0];
    uint64_t t0 = 0, t1 = 0, u0 = h->unsupported[0], u1 = h->unsupported[1];
    const uint64_t nt0 = h->null_true[0], nt1 = h->null_true[1];
    const uint32_t ns = h->n_selectors;
    // first the selectors decided without their record, then the others (needm) in order,
    // each one's record loaded while the one before it is decided (a row read is a memory
    // latency; `found` is one word, so selectors are < 64)
    uint64_t needm = 0;
    for (uint32_t s = s0; s < ns; s += sstep) {
        const uint32_t cnt = sps[s].count;
        if (!cnt) continue;
        if (!((found >> s) & 1)) {  // Null result
            t0 |= sps[s].mask[0] & nt0;
            t1 |= sps[s].mask[1] & nt1;
            continue;
        }
        if (dec && !(sps[s].mask[0] & ~dec[0]) && !sps[s].mask[1]) {  // decided while capturing
            t0 |= sps[s].mask[0] & dec[1];
            continue;
        }
        needm |= 1ull << s;
    }
    uint64_t rec_next = needm ? row[1 + ctz64f(needm)] : 0ull;
    while (needm) {
        const uint32_t s = ctz64f(needm);
        needm &= needm - 1ull;
        const uint64_t rec = rec_next;
        if (needm) rec_next = row[1 + ctz64f(needm)];
        const uint32_t cnt = sps[s].count;
        const uint32_t meta = (uint32_t)(rec >> 32);
        ValueRef v;
        v.start = (uint32_t)rec;
        v.end = v.start + (meta & 0xFFFFFFu);
        v.type = (uint8_t)((meta >> 24) & 7u);
        v.esc = (uint8_t)((meta >> 27) & 1u);
        // (vd: where the value's bytes are read, the document or the lane's copy in LDS)
        const uint8_t* vd = doc;
        if (ring && v.end - v.start <= kSpanMax) {
            const uint32_t at = stage_span(doc + v.start, v.end - v.start, ring);
            if (at != ~0u) {
                vd = ring;
                v.end = at + (v.end - v.start);
                v.start = at;
            }
        }
        const RawVal rv = raw_value(vd, v);
        const uint32_t begin = sps[s].begin;
        uint32_t hits = 0;
        const bool fast_incl = cnt <= 32 && incl_hits(vd, v, pats, plist, begin, cnt, lits, &hits);
        for (uint32_t j = 0; j < cnt; j++) {
            const uint32_t p = plist[begin + j];
            const Pattern pt = pats[p];
            uint8_t r;
            if (dec && p < 64 && ((dec[0] >> p) & 1u)) {
                r = ((dec[1] >> p) & 1u) ? V_T : V_F;
            } else if (pt.state != P_OK) {
                r = pt.state == P_STATIC_E ? V_E : V_U;
            } else if (rv.ok && (pt.op == OP_EQ || pt.op == OP_NEQ)) {
                r = raw_equals(vd, rv, pt, lits) == (pt.op == OP_EQ) ? V_T : V_F;
            } else if (rv.ok && pt.op == OP_MATCHES) {
                const bool m = rv.lit ? dfa_match_lit(blob, pt.dfa_off, rv.lit)
                                      : dfa_match_span(blob, pt.dfa_off, vd + rv.a, rv.n);
                r = m ? V_T : V_F;
            } else if (fast_incl && (pt.op == OP_INCL || pt.op == OP_EXCL)) {
                r = (((hits >> j) & 1u) != 0) == (pt.op == OP_INCL) ? V_T : V_F;
            } else {
                r = eval_pattern(blob, pt, vd, v);
            }
            const uint64_t bit = 1ull << (p & 63);
            if (r == V_T) {
                if (p < 64) t0 |= bit;
                else t1 |= bit;
            } else if (r == V_U) {
                if (p < 64) u0 |= bit;
                else u1 |= bit;
            }
        }
    }
    t[0] = t0;
    t[1] = t1;
    u[0] = u0;
    u[1] = u1;
}

}  // namespace ajx
