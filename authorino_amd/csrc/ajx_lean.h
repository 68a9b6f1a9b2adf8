// ajx_lean.h — stage A, the lean single-pass scan: one work-item per request (lane per
// document), written for a small executed-instruction count per document byte.
//
// The document goes by in 32-byte sub-windows (64-byte dwordx4 loads, the next window
// prefetched). Each sub-window is classified once:
//   * a byte LUT: three v_perm_b32 lookups on the byte's bit fields give an 8-bit class
//     (quote, backslash, { [, } ], :, ',', space / '!' / parens, control) per byte;
//   * one 32 x 8 bit transpose (two v_perm rounds, three delta-swap rounds) turns the
//     class bytes into eight 32-bit masks in byte order;
//   * escapes (odd backslash runs) and strings (prefix XOR of the unescaped quotes) as in
//     simdjson, with one-bit carries between sub-windows;
//   * the context-free grammar of compact JSON is checked for the whole sub-window at
//     once with mask shifts (which byte may follow which: an opening quote follows { [ : ,
//     a closing quote is followed by : , } ], a scalar run sits between { [ : , and , } ],
//     nothing but , } ] follows a close, ...); whitespace, backslashes, parens and control
//     bytes outside strings fail it. The first failing position is kept: a document is
//     proved only when nothing fails before its root's close.
// Only four kinds of bytes reach the per-token walker: closing quotes, { [, } ] and the
// scalar runs that start an array element. Colons and commas never do (the masks check
// them), and neither do object members' scalar values (they are looked at from their
// key). The walker keeps the context the masks can not see: the container stack (object
// or array, trie node), whether an object expects a key or a value, element indices of
// arrays on selector paths, and the captures.
//   * A key (a closing quote followed by ':') in an object on a selector path is looked up
//     once in the ruleset's key table (its last 8 bytes, length and parent node; longer
//     keys also compare their head), and its value is handled in the same iteration: a
//     string value's closing quote is taken from the masks, a container is opened, a
//     scalar is checked (gjson's value-start bytes) and captured when it ends a selector.
//   * A container off every selector path (gjson squashes it: parseSquash counts { [ ( and
//     } ] ) outside strings) is skipped by bracket counting: whole sub-windows at a time
//     when its depth can not reach zero in them, else bracket by bracket.
// For the documents it proves (valid compact JSON up to the root's close, with no parens
// anywhere), gjson v1.14.0 Get returns the first complete path match in document order —
// the first capture of each selector here. Anything else goes to the exact scan
// (ajx_eval_scan), as with the token scanner of ajx_fast.h.
//
// Output: the request's capture row in ajx_fast.h's format (stage B unchanged).
#pragma once
#include "ajx_lean_cls.h"

namespace ajx {
namespace lean {

#if !defined(__HIP_DEVICE_COMPILE__) && defined(AJX_LEAN_COUNT)
inline uint64_t g_lean_iters = 0, g_lean_subs = 0;  // (host test builds: walker iterations, sub-windows)
inline uint32_t* g_lean_trace = nullptr;  // (host test builds: sub-window << 8 | token kind per iteration)
inline uint32_t g_lean_trace_n = 0, g_lean_trace_cap = 0;
#define AJX_LEAN_TICK(x) (x)++
#define AJX_LEAN_TRACE(k) \
    (g_lean_trace && g_lean_trace_n < g_lean_trace_cap ? (void)(g_lean_trace[g_lean_trace_n++] = (uint32_t)(g_lean_subs << 8 | (k))) : (void)0)
#else
#define AJX_LEAN_TICK(x) ((void)0)
#define AJX_LEAN_TRACE(k) ((void)0)
#endif
// (token kinds of the trace: 0 squashed, 1 string element, 2 a key's string value from an
// earlier sub-window, 3 key + string, 4 key + container, 5 key + scalar, 6 root, 7 element
// container, 8 close, 9 scalar element)
// The ring: 8 chunks of 16 B per lane (a 128-byte window of the document: two 64-byte
// windows, the one being walked and the one before or after it), chunk-major across the
// wave: chunk j of lane l at j * kChunkStride + 16 l. That is the layout an LDS-DMA load
// (global_load_lds_dwordx4) writes, 1 KiB of 64 lanes per instruction, so the document
// goes from HBM to the ring without passing through registers; a wave's reads of one chunk
// index are contiguous too (conflict-free ds_read_b128 in classification).
constexpr uint32_t kRingStride = 128;  // ring bytes per lane
constexpr uint32_t kChunkStride = 64 * 16;
constexpr uint32_t kRingBytesPerWave = 64 * kRingStride;
constexpr uint32_t kMaxLive = 16;      // containers on selector paths nested (deeper: exact scan)
constexpr uint32_t kIdxKeyLen = kIndexKeyLen;

enum : uint32_t { S_RUN = 0, S_DONE = 1, S_SLOW = 2 };

// The walker of one document. ARR: the ruleset has array-index selectors (arrays on
// selector paths are walked element by element; without, every array is squashed: no
// selector can match inside one); CAPS: a selector's value can be a container the walk
// enters (a selector that is a prefix of another). The lean kernel takes the instance the
// ruleset needs (RulesetHdr::lean_feat, kLeanArr / kLeanCaps); the fewer features, the less
// state and code per iteration.
template <bool ARR = true, bool CAPS = true>
struct Walk {
    // tables
    const TrieNode* tn;
    const KeySlot* ks;
    const uint8_t* lits;
    uint32_t ks_mask, ks_probes, ks_mult, ks_shift;
    // document
    const uint8_t* a16;  // the document's first aligned 16-byte block (global: bytes the ring no longer holds)
    uint32_t mis;
    const uint8_t* ring;  // the lane's chunk 0 in the wave's ring (LDS on the device)
    RowRef row;
    // walker state
    uint32_t st, depth;
    uint32_t kinds;         // bit k: container at depth k is an array
    uint64_t nlo, nhi;      // trie node per depth 1..16
    uint32_t top, tarr;     // top container's node, is-array
    AJX_HD uint32_t ta() const { return ARR ? tarr : 0u; }
    uint32_t expk;          // top object expects a key (1) or its value (0)
    // (the fields the walk touches only at rarer tokens go packed, so the kernel keeps its
    // state in registers without spilling)
    uint32_t pend;          // a key's value pending over a sub-window boundary: start | node << 24
    uint32_t idx, asv, nasv;  // element index of the top array; saved indices of outer arrays (16 bits each)
    uint32_t skipw, skips;  // squash: depth (bits 0..23) | captured selector + 1 << 24; start (its open)
    uint32_t caps, cap0s, cap1s, ncap;  // open captured containers: sel | depth << 8 (16 bits each), starts
    uint32_t carry_oq;      // last opening quote before the sub-window being walked
    uint32_t lbs1;          // last backslash before it, + 1 (0 none)
    uint64_t found;
    // eager patterns (EagerSel, ajx_blob.h): decided (eD) and true (eT) bits of patterns < 64.
    // (Arrays are not compared element by element: an array value is squashed and stage B
    // decides its incl / excl patterns in one pass; comparing c2's two arrays in the walk
    // measured the same, 1.408 against 1.418 ms, and cost the walk a branch per token)
    const EagerSel* eg;
    uint64_t eT, eD;
    uint32_t keep;  // a caller reads the rows: the records of kEagerKeep selectors go to the row too

    AJX_HD uint32_t ro(uint32_t a) const { return ((a & 0x70u) << 6) | (a & 15u); }  // ring offset a (0..127)
    AJX_HD uint32_t rw(uint32_t q) const { return *reinterpret_cast<const uint32_t*>(ring + ro(q & 127u)); }
    AJX_HD uint32_t rb(uint32_t p) const { return ring[ro((p + mis) & 127u)]; }  // doc byte p (ring)
    AJX_HD uint32_t r32(uint32_t a) const {  // 4 ring bytes from ring offset a (0..127)
        const uint32_t q = a & ~3u, sh = a & 3u;
        const uint32_t w0 = rw(q), w1 = rw(q + 4);
#if defined(__HIP_DEVICE_COMPILE__)
        return __builtin_amdgcn_alignbyte(w1, w0, sh);
#else
        return sh ? (w0 >> (8 * sh)) | (w1 << (32 - 8 * sh)) : w0;
#endif
    }
    AJX_HD uint64_t r64(uint32_t a) const {
        const uint32_t q = a & ~3u, sh = a & 3u;
        const uint32_t w0 = rw(q), w1 = rw(q + 4), w2 = rw(q + 8);
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh), hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
#else
        const uint32_t lo = sh ? (w0 >> (8 * sh)) | (w1 << (32 - 8 * sh)) : w0;
        const uint32_t hi = sh ? (w1 >> (8 * sh)) | (w2 << (32 - 8 * sh)) : w1;
#endif
        return (uint64_t)lo | ((uint64_t)hi << 32);
    }
    AJX_HD uint32_t node_at(uint32_t dd) const {  // 1..16
        const uint32_t k = dd - 1;
        const uint64_t w = k < 8 ? nlo : nhi;
        return (uint32_t)(w >> ((k & 7) * 8)) & 0xFFu;
    }
    AJX_HD int32_t leaf_sel(uint32_t node) const {
        if (node == kNoNode) return -1;
        const int32_t s = tn[node].selector;
        if (s < 0 || ((found >> s) & 1)) return -1;
        return s;
    }
    // a captured value of selector s: doc [start, end), gjson type, has escapes. The
    // selector's eager patterns (EagerSel) are decided on an unescaped string's contents or
    // a literal's String() ("true", "false", ""); the capture record goes to the row unless
    // they were every pattern of the selector (and no caller reads it back: kEagerKeep)
    AJX_HD void record(int32_t s, uint32_t start, uint32_t end, uint32_t type, uint32_t esc) {
        found |= 1ull << s;
        bool dec = false;
        const bool lit = type == T_TRUE || type == T_FALSE || type == T_NULL;
        if (eg && ((type == T_STRING && !esc) || lit)) {
            const EagerSel e = eg[s];
            const uint32_t mt = lit ? lit_match(e, type) : eager_match(e, start + 1u, end - start - 2u);
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const uint32_t m = e.m[k], op = (m >> 8) & 0xFFu;
                const uint64_t bit = 1ull << (m & 63u);
                const bool yes = ((mt >> k) & 1u) == (op == OP_EQ || op == OP_INCL ? 1u : 0u);
                eD = (m & kEagerValid) ? eD | bit : eD;
                eT = (m & kEagerValid) && yes ? eT | bit : eT;
            }
            // (kept rows: every record a caller reads back, kEagerKeep)
            dec = (e.pad[0] & kEagerAll) != 0 && !(keep && (e.pad[0] & kEagerKeep));
        }
        if (!dec)
            row[1 + (uint32_t)s] =
                (uint64_t)start | ((uint64_t)(((end - start) & 0xFFFFFFu) | (type << 24) | (esc << 27)) << 32);
    }
    // bit k: entry k's literal equals a literal value's String() (EagerSel litf bits); null's
    // Value.Array() is empty, so incl / excl never find it
    AJX_HD static uint32_t lit_match(const EagerSel& e, uint32_t type) {
        const uint32_t litb = type == T_TRUE ? (uint32_t)kLitTrue : type == T_FALSE ? (uint32_t)kLitFalse
                                                                                    : (uint32_t)kLitEmpty;
        uint32_t r = 0;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const uint32_t m = e.m[k], op = (m >> 8) & 0xFFu;
            const bool arr = op == OP_INCL || op == OP_EXCL;
            r |= ((m >> 24) & litb) && !(type == T_NULL && arr) ? 1u << k : 0u;
        }
        return r;
    }
    // bit k: entry k's literal equals the string content [a, a + cl) (ring bytes; cl <= 16
    // for a match, and then the content lies in the ring's window)
    AJX_HD uint32_t eager_match(const EagerSel& e, uint32_t a, uint32_t cl) const {
        uint64_t c0 = 0, c1 = 0;
        if (cl <= 16) {
            c0 = r64((a + mis) & 127u);
            c1 = r64((a + 8u + mis) & 127u);
        }
        const uint64_t m0 = cl >= 8 ? ~0ull : ((1ull << (8 * cl)) - 1ull);
        const uint64_t m1 = cl >= 16 ? ~0ull : (cl > 8 ? ((1ull << (8 * (cl - 8))) - 1ull) : 0ull);
        uint32_t r = 0;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const uint64_t l0 = (uint64_t)e.lit[k][0] | ((uint64_t)e.lit[k][1] << 32);
            const uint64_t l1 = (uint64_t)e.lit[k][2] | ((uint64_t)e.lit[k][3] << 32);
            const bool eq = (e.m[k] & kEagerValid) && cl == ((e.m[k] >> 16) & 0xFFu) && ((c0 ^ l0) & m0) == 0 &&
                            ((c1 ^ l1) & m1) == 0;
            r |= eq ? 1u << k : 0u;
        }
        return r;
    }
    // the key table: (sig, len, parent) -> child node (kNoNode none). len = kIdxKeyLen:
    // sig is an array index. A hit on a key longer than 8 bytes also compares its head
    // (bytes [ks, len - 8) of the key, starting at doc position ks) from the ring: the walk
    // looks a key up in the sub-window holding its closing quote, and the ring still holds
    // the 32 bytes before that sub-window (ring_lo). A head that starts before that is read
    // from the document (a global load, which also waits for the ring's loads in flight:
    // rare, keys of 33 bytes and more).
    AJX_HD uint32_t lookup(uint64_t sig, uint32_t len, uint32_t parent, uint32_t kstart, int32_t ring_lo) const {
        const uint32_t want = len | (parent << 16);
        uint32_t h = (uint32_t)sig ^ (((uint32_t)(sig >> 32) << 13) | ((uint32_t)(sig >> 32) >> 19)) ^ (len << 24) ^
                     (parent << 16);
        h = (h * ks_mult) >> ks_shift;
        const bool longk = len > 8 && len != kIdxKeyLen;
        uint32_t node = kNoNode;
        for (uint32_t t = 0; t < ks_probes; t++) {
            const KeySlot sl = ks[(h + t) & ks_mask];
            bool hit = sl.meta != kEmptySlot && sl.sig == sig && (sl.meta & 0xFFFFFFu) == want;
            // (keys sharing their last 8 bytes, length and parent sit in later slots)
            if (hit && longk) {
                const uint8_t* kl = lits + (uint32_t)sl.key_off8 * 8u;
                hit = (int32_t)kstart >= ring_lo ? key_head_equal(kstart, len - 8, kl) : key_rest_equal(kstart, len - 8, kl);
            }
            node = hit ? sl.meta >> 24 : node;
        }
        return node;
    }
    // the key's bytes [k0, k0 + cnt) equal kl[0, cnt), 8 at a time from the ring
    AJX_HD bool key_head_equal(uint32_t k0, uint32_t cnt, const uint8_t* kl) const {
        bool eq = true;
        for (uint32_t k = 0; k < cnt; k += 8) {
            const uint32_t r = cnt - k;
            const uint64_t m = r >= 8 ? ~0ull : ((1ull << (8 * r)) - 1ull);
            const uint64_t b = (uint64_t)load_u32_any(kl + k) | ((uint64_t)load_u32_any(kl + k + 4) << 32);
            eq = eq && ((r64((k0 + k + mis) & 127u) ^ b) & m) == 0;
        }
        return eq;
    }
    AJX_COLD bool key_rest_equal(uint32_t k0, uint32_t cnt, const uint8_t* kl) const {
        for (uint32_t k = 0; k < cnt; k++)
            if (a16[mis + k0 + k] != kl[k]) return false;
        return true;
    }
    AJX_HD void close(uint32_t p) {
        if (CAPS && ncap) {
            const uint32_t cs = ncap == 2 ? caps >> 16 : caps & 0xFFFFu, start = ncap == 2 ? cap1s : cap0s;
            if ((cs >> 8) == depth) {
                row[1 + (cs & 0xFFu)] =
                    (uint64_t)start | ((uint64_t)(((p + 1 - start) & 0xFFFFFFu) | ((uint32_t)T_JSON << 24)) << 32);
                ncap--;
            }
        }
        depth--;
        if (depth == 0) {
            st = S_DONE;
            pend = p;  // (the root's close: no value is pending any more)
            return;
        }
        top = node_at(depth);
        tarr = ARR ? (kinds >> depth) & 1u : 0u;
        expk = 1;
        if (ARR && tarr) {
            idx = nasv == 2 ? asv >> 16 : asv & 0xFFFFu;
            nasv--;
        }
    }
    // a backslash in doc positions [a, b) (b inside sub-window c or the one after it)
    AJX_HD bool has_bs(uint32_t a, uint32_t b, const Sub& c, const Sub& l) const {
        if (lbs1 > a) return true;  // (a backslash before the sub-window, at or after a)
        const uint64_t bs = (uint64_t)c.bs | ((uint64_t)l.bs << 32);
        const int32_t ra = (int32_t)a - c.base, rbb = (int32_t)b - c.base;  // (rbb <= 64)
        uint64_t m = rbb >= 64 ? ~0ull : ((1ull << rbb) - 1ull);
        if (ra > 0) m &= ~((1ull << ra) - 1ull);
        return (bs & m) != 0;
    }

    // the trie node's facts (kNoNode: none): selector (-1 none) | n_children << 16 | flags << 24
    AJX_HD uint32_t node_facts(uint32_t node) const {
        if (node == kNoNode) return 0xFFFFu;
        const TrieNode t = tn[node];
        return (uint32_t)(uint16_t)t.selector | (uint32_t)t.n_children << 16 | (uint32_t)t.flags << 24;
    }
    // a container value at p ('{' or '['): node and its facts (node_facts)
    AJX_HD void open_f(uint32_t node, uint32_t nf, bool arr, uint32_t p) {
        int32_t s = (int32_t)(int16_t)(nf & 0xFFFFu);
        if (s >= 0 && ((found >> s) & 1)) s = -1;
        // squashed (captured when a leaf): off every selector path, and arrays whose node
        // has no array-index children (gjson matches no key inside an array)
        if (node == kNoNode || (nf >> 16 & 0xFFu) == 0 || (arr && !((nf >> 24) & 1u))) {
            skipw = 1u | ((s >= 0 ? (uint32_t)s + 1u : 0u) << 24);
            skips = p;
            return;
        }
        if (depth + 1 > kMaxLive) { st = S_SLOW; return; }
        if (ARR && tarr) {  // the outer array's element index comes back at its close
            if (nasv >= 2 || idx > 0xFFFFu) { st = S_SLOW; return; }
            asv = nasv == 1 ? (asv & 0xFFFFu) | (idx << 16) : nasv == 0 ? (asv & 0xFFFF0000u) | idx : asv;
            nasv++;
        }
        depth++;
        const uint32_t k = depth - 1;
        const uint64_t m = 0xFFull << ((k & 7) * 8), x = (uint64_t)node << ((k & 7) * 8);
        const uint64_t lo = nlo, hi = nhi;
        nlo = k < 8 ? (lo & ~m) | x : lo;
        nhi = k < 8 ? hi : (hi & ~m) | x;
        if (ARR) kinds = arr ? kinds | (1u << depth) : kinds & ~(1u << depth);
        top = node;
        tarr = ARR && arr ? 1u : 0u;
        expk = 1;
        idx = 0;
        if (CAPS && s >= 0) {
            found |= 1ull << s;  // (first match in document order)
            if (ncap >= 2) { st = S_SLOW; return; }
            const uint32_t v = (uint32_t)s | (depth << 8);  // (s < 64, depth <= 16)
            caps = ncap == 1 ? (caps & 0xFFFFu) | (v << 16) : ncap == 0 ? (caps & 0xFFFF0000u) | v : caps;
            cap1s = ncap == 1 ? p : cap1s;
            cap0s = ncap == 0 ? p : cap0s;
            ncap++;
        }
    }

    // Walk sub-window c (l: the one after it; its tokens may be taken here: l.tok updated).
    // One iteration takes one token of every lane, whatever its kind, through ONE copy of
    // each step: the token's kind decoded into flags, one key-table lookup (a key's last 8
    // bytes and length, or an element's index), one node read, the value's first byte, its
    // end (a string's closing quote from the masks, a scalar's next structural byte), one
    // capture record (with the eager patterns), one open and one close. The lanes of a wave
    // hold tokens of different kinds in most iterations, so a walker with a code path per
    // kind runs the union of the paths (round 5: ~460 wave instructions per iteration).
    // The same iteration also takes what follows the value: the run of closing brackets
    // after it (most closes: the last member of an object), and a container off every
    // selector path to its matching bracket when that lies in c (gjson's parseSquash: an
    // inner loop over c's bracket bits). Neither costs an iteration of its own then.
    AJX_HD void walk(const Sub& c, Sub& l) {
        uint32_t T;
        if (skipw) {  // squashing: only brackets (after the squash's own open) matter
            const int32_t rel = (int32_t)skips - c.base;
            const uint32_t ex = rel < 0 ? ~0u : above((uint32_t)rel);
            const uint32_t o = popc(c.op & ex), x = popc(c.cl & ex);
            if (x < (skipw & 0xFFFFFFu)) {  // the depth can not reach zero here
                skipw += o - x;
                T = 0;
            } else {  // it may end in c: to its matching bracket (the closes after it are tokens)
                uint32_t br = (c.op | c.cl) & ex, dep = skipw & 0xFFFFFFu, b = 0;
                while (dep && br) {
                    b = ctz(br);
                    br &= br - 1u;
                    dep = (c.op >> b) & 1u ? dep + 1u : dep - 1u;
                }
                if (dep) {  // (more opens than closes after all: on into the next sub-window)
                    skipw = (skipw & 0xFF000000u) | dep;
                    T = 0;
                } else {
                    if (skipw >> 24) record((int32_t)(skipw >> 24) - 1, skips, (uint32_t)c.base + b + 1u, T_JSON, 0);
                    skipw = 0;
                    T = c.tok & above(b);
                }
            }
        } else {
            T = c.tok;
        }
        const uint32_t cok = (c.co >> 1) | (l.co << 31);  // bit i: a colon at byte i + 1
        const uint32_t cb = (uint32_t)c.base;
        const uint64_t cl64 = (uint64_t)c.cl | ((uint64_t)l.cl << 32);
        constexpr uint32_t kNone = 0xFFFFFFFFu;
        AJX_LEAN_TICK(g_lean_subs);
        while (T) {
            AJX_LEAN_TICK(g_lean_iters);
            const uint32_t i = ctz(T);
            T &= T - 1u;
            const uint32_t p = cb + i;
            uint32_t after = kNone;  // the position after the value this iteration took
            bool bad = false;
            {
                const bool bq = (c.cq >> i) & 1u, bo = (c.op >> i) & 1u, bc = (c.cl >> i) & 1u, kq = (cok >> i) & 1u;
                const bool root = depth == 0;
                const bool key = bq && !ta() && expk;  // a key (its closing quote)
                const bool pv = bq && !ta() && !expk;  // the closing quote of a key's string value
                const bool el = ta() && !bc;           // an array element (string, container, scalar)
                // the grammar the masks can not see: a key where a key belongs, a value where
                // a value belongs, the root alone at depth 0
                bad = root ? !(bo && p == 0) : bq ? kq != key : bc ? false : !ta();
                // the string's opening quote (a key's, a string element's)
                const uint32_t oqb = c.oq & below(i);
                const uint32_t ss = oqb ? cb + hib(oqb) : carry_oq;
                const uint32_t k0 = ss + 1u, klen = p - k0;
                if (key && !bad) bad = klen >= kIdxKeyLen || has_bs(k0, p, c, l);
                // the key table: a key's (last 8 bytes, length, parent) or an element's index
                uint32_t node = kNoNode;
                const bool eidx = ARR && el && top != kNoNode && (tn[top].flags & 1);
                if ((key && !bad) || eidx) {
                    uint64_t sig = r64((p - 8u + mis) & 127u);
                    sig = klen >= 8 ? sig : (klen ? sig >> (8 * (8 - klen)) : 0ull);
                    node = lookup(key ? sig : (uint64_t)idx, key ? klen : kIdxKeyLen, top, k0, (int32_t)cb - 32);
                }
                idx += el ? 1u : 0u;
                node = pv ? pend >> 24 : root ? 0u : node;
                const uint32_t nf = node_facts(node);
                int32_t s = (int32_t)(int16_t)(nf & 0xFFFFu);
                if (s >= 0 && ((found >> s) & 1)) s = -1;
                // the value: start vs (a string's opening quote), first byte vb
                const uint32_t vs = key ? p + 2u : pv ? (pend & 0xFFFFFFu) : bq ? ss : p;
                const uint32_t vb = rb(key ? p + 2u : p);
                const bool vstr = bq && (!key || vb == '"');
                const bool vopen = key ? (vb == '{' || vb == '[') : bo;
                const bool vscal = !bq && !bo && !bc ? true : key && !vstr && !vopen;
                if (bc) bad |= root || ta() != (vb == ']' ? 1u : 0u) || (!ta() && !expk);
                // a key's string value: its closing quote from the masks (or pending)
                uint32_t e = p;
                bool ended = true;
                const uint32_t rv = vs - cb;  // (a key's value: 2..33)
                if (key && vstr) {
                    const uint64_t m = ((uint64_t)c.cq | ((uint64_t)l.cq << 32)) & (~0ull << (rv + 1));
                    if (m) {
                        const uint32_t j = (uint32_t)__builtin_ctzll(m);
                        if (j < 32) T &= ~(1u << j);
                        else l.tok &= ~(1u << (j - 32));
                        e = cb + j;
                    } else {
                        ended = false;
                        expk = 0;
                        pend = vs | (node << 24);  // (positions < 2^24)
                    }
                }
                if (pv) expk = 1;
                if (vstr && ended) after = e + 1u;
                // a scalar: gjson's value-start bytes, its end (the next structural byte), literals
                uint32_t type = T_STRING, end = e + 1u;
                if (vscal && !bad) {
                    const bool lit = vb == 't' || vb == 'f' || (vb == 'n' && rb(vs + 1) == 'u');
                    const uint32_t r = vs - cb;  // (< 64)
                    const uint64_t stm = (uint64_t)c.st | ((uint64_t)l.st << 32);
                    const uint64_t m = r >= 63 ? 0ull : stm & (~0ull << (r + 1));
                    end = cb + (uint32_t)__builtin_ctzll(m | (1ull << 63));
                    after = m ? end : kNone;
                    if (!scalar_start(vb)) {
                        bad = true;
                    } else if (s >= 0 || (el && lit)) {
                        const uint32_t len = end - vs;
                        type = T_NUMBER;
                        if (lit) {
                            const uint64_t w = r64((vs + mis) & 127u);
                            const bool ok = vb == 't' ? len == 4 && (uint32_t)w == 0x65757274u
                                          : vb == 'f' ? len == 5 && (w & 0xFFFFFFFFFFull) == 0x65736C6166ull
                                                      : len == 4 && (uint32_t)w == 0x6C6C756Eu;
                            type = vb == 't' ? T_TRUE : vb == 'f' ? T_FALSE : T_NULL;
                            bad |= !ok;
                        }
                        bad |= m == 0;  // (longer than the two sub-windows: exact scan)
                    }
                }
                // the capture record (one site for every kind of value)
                if (!bad && s >= 0 && ((vstr && ended) || vscal))
                    record(s, vs, end, type, vstr && has_bs(vs, e, c, l) ? 1u : 0u);
                // a container value
                if (!bad && vopen) {
                    if (key) {
                        if (rv < 32) T &= ~(1u << rv);
                        else l.tok &= ~(1u << (rv - 32));
                    }
                    open_f(node, nf, vb == '[', vs);
                    const uint32_t ip = key ? rv : i;
                    T = ip < 32 ? T & above(ip) : 0u;
                    after = vs + 1u;  // (an empty container closes right away)
                    if (skipw) {  // squashed: to its matching bracket, if that lies in c
                        bad |= root;  // (a ruleset whose root node is a leaf)
                        after = kNone;
                        if (ip < 32) {
                            uint32_t br = (c.op | c.cl) & above(ip), dep = 1;
                            while (br) {
                                const uint32_t b = ctz(br);
                                br &= br - 1u;
                                dep = (c.op >> b) & 1u ? dep + 1u : dep - 1u;
                                if (dep == 0) {
                                    if (skipw >> 24) record((int32_t)(skipw >> 24) - 1, skips, cb + b + 1u, T_JSON, 0);
                                    skipw = 0;
                                    T &= above(b);
                                    after = cb + b + 1u;
                                    break;
                                }
                            }
                            if (skipw) {  // (the rest of c lies inside it)
                                skipw = (skipw & 0xFF000000u) | dep;
                                T = 0;
                            }
                        }
                    }
                }
                if (!bad && bc) {
                    close(p);
                    after = p + 1u;
                }
                AJX_LEAN_TRACE(bc ? 8 : bo ? (root ? 6 : 7) : pv ? 2 : key ? (vstr ? 3 : vopen ? 4 : 5) : bq ? 1 : 9);
            }
            // the closing brackets that follow the value
            while (!bad && st == S_RUN && after != kNone) {
                const uint32_t r = after - cb;
                if (r >= 64 || !((cl64 >> r) & 1u)) break;
                bad = depth == 0 || ta() != (rb(after) == ']' ? 1u : 0u) || (!ta() && !expk);
                if (bad) break;
                if (r < 32) T &= ~(1u << r);
                else l.tok &= ~(1u << (r - 32));
                close(after);
                after++;
            }
            if (bad) st = S_SLOW;
            if (st != S_RUN) T = 0;
        }
        if (c.oq) carry_oq = (uint32_t)c.base + hib(c.oq);
        if (c.bs) lbs1 = (uint32_t)c.base + hib(c.bs) + 1u;
    }
};

// Stage A for one request with the lean scan.
//   ring: the lane's chunk 0 in the wave's ring (chunk-major: lane * 16 into the wave's
//         8 x kChunkStride bytes);
//   ld:   the document's loader: ld.issue(b, chunk) starts the copy of aligned 16-byte
//         block b of the document into ring chunk `chunk` (an LDS-DMA load on the device;
//         past the document's last block, that block again), ld.wait<K>() returns once at
//         most the last K issued loads are still in flight. n >= 1.
// Returns true when the capture row is valid (false: the exact scan decides the request);
// dec[0] / dec[1]: the patterns decided while capturing / those of them that are true.
// ABL (profiling ablations, kernel modes 15..18; the row then holds a checksum): 1 loads
// only, 2 + classification, 3 + the walk without eager patterns, 4 = stage A.
// keep: a caller reads the rows after the kernel (the records of kEagerKeep selectors go to
// the row as well as those stage B needs).
//
// Loads go by 32-byte halves of 64-byte windows, each into the ring chunks that the walk no
// longer needs: the next window's first half while the current window's first sub-window
// is walked (the ring keeps the 32 bytes before that sub-window), its second half while
// the second one is.
template <int ABL = 0, bool ARR = true, bool CAPS = true, class Loader>
AJX_HD bool scan_doc(const uint8_t* blob, uint32_t n, uint32_t mis, RowRef row, uint8_t* ring, Loader& ld,
                     uint64_t dec[2], uint32_t keep = 1) {
    const RulesetHdr* h = (const RulesetHdr*)blob;
    Walk<ARR, CAPS> w;
    // the tables as the blob pointer plus uniform offsets: the offsets go to scalar registers
    // and the pointers keep the blob's provenance, so that with the blob staged in LDS every
    // table read is a ds_read (a pointer made uniform through an integer would be generic:
    // flat loads, which wait for the document's loads in flight as well)
    w.tn = reinterpret_cast<const TrieNode*>(blob + uni(h->off_trie_nodes));
    w.ks = reinterpret_cast<const KeySlot*>(blob + uni(h->off_key_slots));
    w.lits = blob + uni(h->off_literals);
    w.ks_mask = uni((1u << h->key_slots_log2) - 1u);
    w.ks_probes = uni(h->key_probes);
    w.ks_mult = uni(h->key_mult);
    w.ks_shift = uni(32u - h->key_slots_log2);
    w.a16 = ld.base();
    w.mis = mis;
    w.ring = ring;
    w.row = row;
    w.st = S_RUN;
    w.depth = 0;
    w.kinds = 0;
    w.nlo = w.nhi = ~0ull;
    w.top = kNoNode;
    w.tarr = 0;
    w.expk = 1;
    w.pend = (uint32_t)kNoNode << 24;
    w.idx = w.asv = w.nasv = 0;
    w.skipw = w.skips = 0;
    w.caps = w.cap0s = w.cap1s = w.ncap = 0;
    w.carry_oq = 0;
    w.lbs1 = 0;
    w.found = 0;
    w.eg = ABL != 3 && uni(h->off_eager) ? reinterpret_cast<const EagerSel*>(blob + uni(h->off_eager)) : nullptr;
    w.eT = w.eD = 0;
    w.keep = keep;
    Carry cr;
    cr.f = 0;
    cr.bad = 0x7FFFFFFF;

    const uint32_t nblk = (n + mis + 15) / 16;
    const uint32_t nwin = (nblk + 3) / 4;  // 64-byte windows
    auto valid_of = [&](int32_t base) -> uint32_t {
        uint32_t v = ~0u;
        if (base < 0) v &= ~below((uint32_t)(-base));
        const int32_t hi = (int32_t)n - base;
        if (hi < 32) v &= hi <= 0 ? 0u : below((uint32_t)hi);
        return v;
    };
    // window win's half k (32 bytes) into chunks 4 (win & 1) + 2k, + 1
    auto issue_half = [&](uint32_t win, uint32_t k) {
        const uint32_t c = (win & 1u) * 4u + 2u * k;
        ld.issue(win * 4u + 2u * k, c);
        ld.issue(win * 4u + 2u * k + 1u, c + 1u);
    };
    // the 32 bytes of ring chunks c, c + 1 (c even)
    auto half_words = [&](uint32_t c, uint32_t x[8]) {
        const Block16 a = *reinterpret_cast<const Block16*>(ring + c * kChunkStride);
        const Block16 b = *reinterpret_cast<const Block16*>(ring + (c + 1u) * kChunkStride);
        x[0] = a.x, x[1] = a.y, x[2] = a.z, x[3] = a.w, x[4] = b.x, x[5] = b.y, x[6] = b.z, x[7] = b.w;
    };
    Sub s0, s1, s2;
    uint32_t ck = 0;  // (ablations: a checksum that keeps the skipped work's inputs live)
    issue_half(0, 0);
    issue_half(0, 1);
    ld.template wait<0>();
    {
        uint32_t x[8];
        half_words(0, x);
        if constexpr (ABL == 1) ck ^= x[0] ^ x[5];
        else classify(s0, x, -(int32_t)mis, valid_of(-(int32_t)mis), cr);
        half_words(2, x);
        if constexpr (ABL == 1) ck ^= x[2] ^ x[7];
        else classify(s1, x, 32 - (int32_t)mis, valid_of(32 - (int32_t)mis), cr);
    }
    for (uint32_t win = 0; win < nwin; win++) {
        const int32_t b0 = (int32_t)(win * 64u) - (int32_t)mis;
        const bool more = win + 1 < nwin;
        const uint32_t c2 = ((win + 1) & 1u) * 4u;  // the next window's first chunk
        if (more) issue_half(win + 1, 0);
        if constexpr (ABL != 1 && ABL != 2) {
            w.walk(s0, s1);
            if (w.st != S_RUN) break;
        }
        if (more) issue_half(win + 1, 1);
        if (more) {
            ld.template wait<2>();  // (the first half landed; the second may be in flight)
            uint32_t x[8];
            half_words(c2, x);
            if constexpr (ABL == 1) ck ^= x[1] ^ x[6];
            else classify(s2, x, b0 + 64, valid_of(b0 + 64), cr);
        } else {
            s2.base = b0 + 64;
            s2.tok = s2.cq = s2.oq = s2.op = s2.cl = s2.co = s2.st = s2.bs = 0;
        }
        if constexpr (ABL != 1 && ABL != 2) {
            w.walk(s1, s2);
            if (w.st != S_RUN) break;
        } else if constexpr (ABL == 2) {
            ck ^= s0.tok ^ s0.bs ^ s1.tok ^ s1.bs;
        }
        if (more) {
            ld.template wait<0>();
            uint32_t x[8];
            half_words(c2 + 2u, x);
            if constexpr (ABL == 1) ck ^= x[3] ^ x[4];
            else classify(s1, x, b0 + 96, valid_of(b0 + 96), cr);
        }
        s0 = s2;
    }
    if constexpr (ABL == 1 || ABL == 2) {
        row[0] = (uint64_t)ck ^ ((uint64_t)(uint32_t)cr.bad << 32) ^ s0.tok ^ s1.tok;
        dec[0] = dec[1] = 0;
        return true;
    }
    // (a walk that ended early may leave the next window's loads in flight: none may land in
    // the ring after this, stage B copies values there)
    ld.template wait<0>();
    if (w.st != S_DONE || cr.bad <= (int32_t)w.pend) {  // (pend: the root's close)
        row[0] = kRowSlow;
        return false;
    }
    row[0] = w.found;
    dec[0] = w.eD;
    dec[1] = w.eT;
    return true;
}

// The device loader of scan_doc: LDS-DMA loads of the document's aligned 16-byte blocks
// (a4: the document's first block; nblk: its block count) into the wave's ring (the wave's
// chunk 0: a uniform LDS address; each lane's 16 bytes land at 16 * lane past it).
#if defined(__HIPCC__)
// Every active lane issues every load, so that the wave's count of loads in flight is what
// wait<K> assumes: blocks past the document's last one load that block again (nblk >= 1:
// empty documents never reach the scan).
struct DmaLoader {
    const uint4* a4;
    uint32_t nblk;
    uint8_t* wave_ring;
    __device__ const uint8_t* base() const { return reinterpret_cast<const uint8_t*>(a4); }
    __device__ void issue(uint32_t b, uint32_t chunk) const {
        __builtin_amdgcn_global_load_lds(
                (const void*)(a4 + (b < nblk ? b : nblk - 1u)),
                (__attribute__((address_space(3))) void*)(wave_ring + chunk * kChunkStride), 16, 0, 0);
    }
    template <int K>
    __device__ void wait() const {
        // (also a compiler barrier: the ring reads after it stay after it)
        if constexpr (K == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
};
#endif
// the host builds' loader: a synchronous copy of the block (zeros past the document)
struct CopyLoader {
    const uint8_t* a16;  // the document's first aligned 16-byte block
    uint32_t nblk, avail;  // blocks of the document; blocks readable from a16
    uint8_t* lane_ring;
    AJX_HD const uint8_t* base() const { return a16; }
    AJX_HD void issue(uint32_t b, uint32_t chunk) const {
        const uint32_t bb = b < nblk ? b : nblk - 1u;  // (as the device: the last block again)
        uint8_t* dst = lane_ring + chunk * kChunkStride;
        for (uint32_t i = 0; i < 16; i++) dst[i] = bb < avail ? a16[16 * bb + i] : 0;
    }
    template <int K>
    AJX_HD void wait() const {}
};

}  // namespace lean
}  // namespace ajx
