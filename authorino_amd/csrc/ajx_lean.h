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
#include "ajx_fast.h"

namespace ajx {
namespace lean {

// ---------------------------------------------------------------- byte classes
enum : uint32_t { K_Q = 0, K_BS = 1, K_OPEN = 2, K_CLOSE = 3, K_COLON = 4, K_COMMA = 5, K_BAD1 = 6, K_CTRL = 7 };
// every class is a product set over the byte's fields h0 = b & 7, h1 = (b >> 3) & 7,
// h2 = b >> 6 (bitmask of the allowed values of each field, per class)
//                                   "      \\      { [      } ]      :      ,   sp ! ( )   0x00-0x1F
constexpr uint32_t kSetH0[8] = {1u << 2, 1u << 4, 1u << 3, 1u << 5, 1u << 2, 1u << 4, 0x03u, 0xFFu};
constexpr uint32_t kSetH1[8] = {1u << 4, 1u << 3, 0x88u, 0x88u, 1u << 7, 1u << 5, 0x30u, 0x0Fu};
constexpr uint32_t kSetH2[8] = {1u << 0, 1u << 1, 1u << 1, 1u << 1, 1u << 0, 1u << 0, 1u << 0, 1u << 0};
constexpr uint32_t lut_byte(const uint32_t* set, uint32_t v) {
    uint32_t r = 0;
    for (uint32_t c = 0; c < 8; c++) r |= ((set[c] >> v) & 1u) << c;
    return r;
}
constexpr uint32_t lut_word(const uint32_t* set, uint32_t v0) {
    return lut_byte(set, v0) | lut_byte(set, v0 + 1) << 8 | lut_byte(set, v0 + 2) << 16 | lut_byte(set, v0 + 3) << 24;
}
constexpr uint32_t kL0lo = lut_word(kSetH0, 0), kL0hi = lut_word(kSetH0, 4);
constexpr uint32_t kL1lo = lut_word(kSetH1, 0), kL1hi = lut_word(kSetH1, 4);
constexpr uint32_t kL2lo = lut_word(kSetH2, 0);
constexpr uint32_t class_ref(uint32_t b) {  // the classes by plain compares (the LUT's specification)
    return (b == '"' ? 1u << K_Q : 0u) | (b == '\\' ? 1u << K_BS : 0u) | (b == '{' || b == '[' ? 1u << K_OPEN : 0u) |
           (b == '}' || b == ']' ? 1u << K_CLOSE : 0u) | (b == ':' ? 1u << K_COLON : 0u) |
           (b == ',' ? 1u << K_COMMA : 0u) | (b == ' ' || b == '!' || b == '(' || b == ')' ? 1u << K_BAD1 : 0u) |
           (b < 0x20 ? 1u << K_CTRL : 0u);
}
constexpr bool lut_ok() {
    for (uint32_t b = 0; b < 256; b++)
        if ((lut_byte(kSetH0, b & 7) & lut_byte(kSetH1, (b >> 3) & 7) & lut_byte(kSetH2, b >> 6)) != class_ref(b))
            return false;
    return true;
}
static_assert(lut_ok(), "byte-class LUT");

// v_perm_b32: byte i of the result = byte sel_i of {lo (0..3), hi (4..7)}; 0x0C gives 0
AJX_HD uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    const uint64_t pool = (uint64_t)lo | ((uint64_t)hi << 32);
    uint32_t r = 0;
    for (int i = 0; i < 4; i++) {
        const uint32_t s = (sel >> (8 * i)) & 0xFFu;
        const uint32_t v = s < 8 ? (uint32_t)(pool >> (8 * s)) & 0xFFu : 0u;
        r |= v << (8 * i);
    }
    return r;
#endif
}
AJX_HD uint32_t classify4(uint32_t x) {
    const uint32_t a = perm(kL0hi, kL0lo, x & 0x07070707u);
    const uint32_t b = perm(kL1hi, kL1lo, (x >> 3) & 0x07070707u);
    const uint32_t c = perm(0u, kL2lo, (x >> 6) & 0x03030303u);
    return a & b & c;
}
// delta swap: A's bits at positions with bit q = 1 <-> B's bits at positions with q = 0
AJX_HD void dswap(uint32_t& a, uint32_t& b, uint32_t s, uint32_t m) {
    const uint32_t t = ((a >> s) ^ b) & m;
    b ^= t;
    a ^= t << s;
}
// 32 class bytes (d[j] byte b = byte 4j + b) -> eight 32-bit masks in byte order; class c
// ends in d[kClassReg[c]]
AJX_HD void transpose(uint32_t d[8]) {
#pragma unroll
    for (int j = 0; j < 4; j++) {  // register bit 2 <-> byte bit 1
        const uint32_t a = d[j], b = d[j + 4];
        d[j] = perm(b, a, 0x05040100u);
        d[j + 4] = perm(b, a, 0x07060302u);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {  // register bit 1 <-> byte bit 0
        if (j & 2) continue;
        const uint32_t a = d[j], b = d[j + 2];
        d[j] = perm(b, a, 0x06020400u);
        d[j + 2] = perm(b, a, 0x07030501u);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) dswap(d[j], d[j + 4], 2, 0x33333333u);  // register bit 2 <-> bit-in-byte 1
#pragma unroll
    for (int j = 0; j < 8; j++)
        if (!(j & 2)) dswap(d[j], d[j + 2], 1, 0x55555555u);  // register bit 1 <-> bit-in-byte 0
#pragma unroll
    for (int j = 0; j < 8; j += 2) dswap(d[j], d[j + 1], 4, 0x0F0F0F0Fu);  // register bit 0 <-> bit-in-byte 2
}
// register of class c after transpose(): (c1, c0, c2)
constexpr uint32_t creg(uint32_t c) { return ((c >> 1) & 1u) << 2 | (c & 1u) << 1 | (c >> 2); }

AJX_HD uint32_t ctz(uint32_t x) { return (uint32_t)__builtin_ctz(x); }
AJX_HD uint32_t hib(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }
AJX_HD uint32_t popc(uint32_t x) { return (uint32_t)__builtin_popcount(x); }
AJX_HD uint32_t below(uint32_t i) { return i >= 32 ? ~0u : (1u << i) - 1u; }  // bits < i
AJX_HD uint32_t above(uint32_t i) { return i >= 31 ? 0u : ~0u << (i + 1); }   // bits > i

// One sub-window's masks (outside-string classes unless noted).
struct Sub {
    int32_t base;   // doc position of byte 0
    uint32_t tok;   // walker tokens: closing quotes, { [, } ], array-position scalar starts
    uint32_t cq, oq;
    uint32_t op, cl, co;
    uint32_t st;    // structural bytes { [ } ] : ,
    uint32_t bs;    // backslashes (inside strings too)
};

// classification carries: escape (bit 0), inside a string (bit 1), and the previous
// sub-window's last byte: { [ (2), : , (3), : (4), closing quote (5), scalar (6), } ] (7)
struct Carry {
    uint32_t f;
    int32_t bad;  // first position failing a check (INT32_MAX none)
};

// Classify 32 bytes x[0..7] (doc positions base .. base + 31; `valid` marks the bytes of
// the document).
AJX_HD void classify(Sub& o, const uint32_t x[8], int32_t base, uint32_t valid, Carry& c) {
    uint32_t d[8];
#pragma unroll
    for (int j = 0; j < 8; j++) d[j] = classify4(x[j]);
    transpose(d);
    const uint32_t Q = d[creg(K_Q)] & valid, BS = d[creg(K_BS)] & valid;
    // escaped bytes: the byte after an odd-length backslash run
    const uint32_t esc_in = c.f & 1u;
    const uint32_t bsx = BS & ~esc_in;
    const uint32_t follows = (bsx << 1) | esc_in;
    const uint32_t even = 0x55555555u;
    const uint32_t odd_starts = bsx & ~even & ~follows;
    const uint64_t seq = (uint64_t)odd_starts + bsx;
    const uint32_t escaped = (even ^ ((uint32_t)seq << 1)) & follows;
    const uint32_t U = Q & ~escaped;
    uint32_t X = U;
    X ^= X << 1;
    X ^= X << 2;
    X ^= X << 4;
    X ^= X << 8;
    X ^= X << 16;
    X ^= (c.f & 2u) ? ~0u : 0u;  // inside a string at byte k (the opening quote included)
    const uint32_t OQ = U & X, CQ = U & ~X;
    const uint32_t outside = ~X & ~U & valid;
    const uint32_t OP = d[creg(K_OPEN)] & outside, CL = d[creg(K_CLOSE)] & outside;
    const uint32_t CO = d[creg(K_COLON)] & outside, CM = d[creg(K_COMMA)] & outside;
    const uint32_t badb = (d[creg(K_BAD1)] | d[creg(K_CTRL)] | BS) & outside;
    const uint32_t ST = OP | CL | CO | CM;
    const uint32_t SC = outside & ~ST & ~badb;
    // the previous byte's class (bit k: byte k - 1)
    const uint32_t f = c.f;
    const uint32_t nOP = (OP << 1) | ((f >> 2) & 1u), nCOCM = ((CO | CM) << 1) | ((f >> 3) & 1u);
    const uint32_t nCO = (CO << 1) | ((f >> 4) & 1u), nCQ = (CQ << 1) | ((f >> 5) & 1u);
    const uint32_t nSC = (SC << 1) | ((f >> 6) & 1u), nCL = (CL << 1) | ((f >> 7) & 1u);
    const uint32_t nSEP = nOP | nCOCM;
    const uint32_t SCS = SC & ~nSC;  // scalar run starts
    const uint32_t bad = badb | (OQ & ~nSEP) | (nCQ & ~(CO | CM | CL)) | (SCS & ~nSEP) | (nSC & ~(SC | CM | CL)) |
                         (nSEP & (CO | CM)) | (nCOCM & CL) | (nCL & ~(CM | CL));
    if (bad) {
        const int32_t bp = base + (int32_t)ctz(bad);
        c.bad = bp < c.bad ? bp : c.bad;
    }
    c.f = (uint32_t)(seq >> 32) | ((X >> 31) << 1) | ((OP >> 31) << 2) | (((CO | CM) >> 31) << 3) |
          ((CO >> 31) << 4) | ((CQ >> 31) << 5) | ((SC >> 31) << 6) | ((CL >> 31) << 7);
    o.base = base;
    o.cq = CQ;
    o.oq = OQ;
    o.op = OP;
    o.cl = CL;
    o.co = CO;
    o.st = ST;
    o.bs = BS;
    o.tok = CQ | OP | CL | (SCS & ~nCO);
}

// values every lane of the wave holds (the lean kernel runs one ruleset per batch): in
// scalar registers
AJX_HD uint32_t uni(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
#else
    return x;
#endif
}

// gjson's value-start bytes (parseObject / parseArray): " { [ n t f + - 0-9 i I N
AJX_HD bool scalar_start(uint32_t b) {
    return b == 't' || b == 'f' || b == 'n' || b == '-' || b == '+' || (b - '0') < 10u || b == 'i' || b == 'I' ||
           b == 'N';
}

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
// per lane: 4 slots of 32 B. 16-byte chunk k of a lane's ring sits at chunk k ^ (lane & 7)
// (ring_off), so that the 8 lanes of a ds_write_b128 lane group hit all 32 banks
constexpr uint32_t kRingStride = 128;
constexpr uint32_t kMaxLive = 16;      // containers on selector paths nested (deeper: exact scan)
constexpr uint32_t kIdxKeyLen = kIndexKeyLen;
constexpr uint32_t kRingKeyLen = 31;  // keys the walk compares from the ring (see Walk::lookup)

enum : uint32_t { S_RUN = 0, S_DONE = 1, S_SLOW = 2 };

// The walker of one document.
struct Walk {
    // tables
    const TrieNode* tn;
    const KeySlot* ks;
    const uint8_t* lits;
    uint32_t ks_mask, ks_probes, ks_mult, ks_shift;
    // document
    const uint8_t* d;  // (global: bytes the ring no longer holds)
    uint32_t n, mis;
    const uint8_t* ring;  // the lane's 128-byte ring (LDS on the device)
    uint32_t sw16;        // its chunk swizzle: (lane & 7) << 4
    RowRef row;
    // walker state
    uint32_t st, depth;
    uint32_t kinds;         // bit k: container at depth k is an array
    uint64_t nlo, nhi;      // trie node per depth 1..16
    uint32_t top, tarr;     // top container's node, is-array
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
    uint32_t keep;  // every capture record goes to the row (a caller reads the rows)

    AJX_HD uint32_t ro(uint32_t a) const { return ((a & 0x70u) ^ sw16) | (a & 15u); }  // ring offset a (0..127)
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
    // they were every pattern of the selector (and the caller keeps no rows)
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
            dec = (e.pad[0] & kEagerAll) != 0;
        }
        if (!dec || keep)
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
    // (bytes [ks, len - 8) of the key, starting at doc position ks).
    // Keys of up to kRingKeyLen bytes are read from the ring: the walk looks a key up in the
    // sub-window holding its closing quote, and the ring still holds the 32 bytes before
    // that sub-window (64 for the window's first one). Longer keys read the document (a
    // global load, which also waits for the next window's loads in flight: rare).
    AJX_HD uint32_t lookup(uint64_t sig, uint32_t len, uint32_t parent, uint32_t kstart) const {
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
            if (hit && longk) hit = key_head_equal(kstart, len - 8, lits + (uint32_t)sl.key_off8 * 8u);
            node = hit ? sl.meta >> 24 : node;
        }
        return node;
    }
    // the key's bytes [k0, k0 + cnt) equal kl[0, cnt), 8 at a time (ring) or byte by byte
    AJX_HD bool key_head_equal(uint32_t k0, uint32_t cnt, const uint8_t* kl) const {
        if (cnt + 8 > kRingKeyLen) return key_rest_equal(k0, cnt, kl);
        for (uint32_t k = 0; k < cnt; k += 8) {
            const uint32_t r = cnt - k;
            const uint64_t m = r >= 8 ? ~0ull : ((1ull << (8 * r)) - 1ull);
            const uint64_t b = (uint64_t)load_u32_any(kl + k) | ((uint64_t)load_u32_any(kl + k + 4) << 32);
            if ((r64((k0 + k + mis) & 127u) ^ b) & m) return false;
        }
        return true;
    }
    AJX_COLD bool key_rest_equal(uint32_t k0, uint32_t cnt, const uint8_t* kl) const {
        for (uint32_t k = 0; k < cnt; k++)
            if (d[k0 + k] != kl[k]) return false;
        return true;
    }
    // the node of the next element of the top array (its index, then the index moves on)
    AJX_HD uint32_t elem_node() {
        const uint32_t i = idx;
        idx = i + 1;
        if (top == kNoNode || !(tn[top].flags & 1)) return kNoNode;
        return lookup((uint64_t)i, kIdxKeyLen, top, 0);
    }
    // a container value at p ('{' or '['), node = its trie node
    AJX_HD void open(uint32_t node, bool arr, uint32_t p) {
        const int32_t s = leaf_sel(node);
        if (node == kNoNode || tn[node].n_children == 0) {  // squashed (captured when a leaf)
            skipw = 1u | ((s >= 0 ? (uint32_t)s + 1u : 0u) << 24);
            skips = p;
            return;
        }
        if (depth + 1 > kMaxLive) { st = S_SLOW; return; }
        if (tarr) {  // the outer array's element index comes back at its close
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
        kinds = arr ? kinds | (1u << depth) : kinds & ~(1u << depth);
        top = node;
        tarr = arr ? 1u : 0u;
        expk = 1;
        idx = 0;
        if (s >= 0) {
            found |= 1ull << s;  // (first match in document order)
            if (ncap >= 2) { st = S_SLOW; return; }
            const uint32_t v = (uint32_t)s | (depth << 8);  // (s < 64, depth <= 16)
            caps = ncap == 1 ? (caps & 0xFFFFu) | (v << 16) : ncap == 0 ? (caps & 0xFFFF0000u) | v : caps;
            cap1s = ncap == 1 ? p : cap1s;
            cap0s = ncap == 0 ? p : cap0s;
            ncap++;
        }
    }
    AJX_HD void close(uint32_t p) {
        if (ncap) {
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
        tarr = (kinds >> depth) & 1u;
        expk = 1;
        if (tarr) {
            idx = nasv == 2 ? asv >> 16 : asv & 0xFFFFu;
            nasv--;
        }
    }
    // a scalar value starting at p (first byte b): false when gjson would read it
    // differently (its value-start bytes; literals must be exact)
    AJX_HD bool scalar(uint32_t node, uint32_t p, uint32_t b, const Sub& c, const Sub& l, bool elem) {
        if (!scalar_start(b)) return false;
        const int32_t s = leaf_sel(node);
        const bool lit = b == 't' || b == 'f' || (b == 'n' && rb(p + 1) == 'u');
        if (s < 0 && !(elem && lit)) return true;
        // the run's end: the next structural byte
        const uint32_t r = p - (uint32_t)c.base;  // (< 64)
        const uint64_t stm = (uint64_t)c.st | ((uint64_t)l.st << 32);
        const uint64_t m = r >= 63 ? 0ull : stm & (~0ull << (r + 1));
        if (!m) return false;  // (longer than the two sub-windows: exact scan)
        const uint32_t end = (uint32_t)c.base + (uint32_t)__builtin_ctzll(m);
        const uint32_t len = end - p;
        uint32_t type = T_NUMBER;
        if (lit) {
            const uint64_t w = r64((p + mis) & 127u);
            if (b == 't') {
                if (len != 4 || (uint32_t)w != 0x65757274u) return false;
                type = T_TRUE;
            } else if (b == 'f') {
                if (len != 5 || (w & 0xFFFFFFFFFFull) != 0x65736C6166ull) return false;
                type = T_FALSE;
            } else {
                if (len != 4 || (uint32_t)w != 0x6C6C756Eu) return false;
                type = T_NULL;
            }
        }
        if (s >= 0) record(s, p, end, type, 0);
        return true;
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

    // walk sub-window c (l: the one after it; its tokens may be taken here: l.tok updated)
    AJX_HD void walk(const Sub& c, Sub& l) {
        uint32_t T;
        if (skipw) {  // squashing: only brackets (after the squash's own open) matter
            const int32_t rel = (int32_t)skips - c.base;
            const uint32_t ex = rel < 0 ? ~0u : above((uint32_t)rel);
            const uint32_t o = popc(c.op & ex), x = popc(c.cl & ex);
            if (x < (skipw & 0xFFFFFFu)) {  // the depth can not reach zero here
                skipw += o - x;
                T = 0;
            } else {
                T = (c.op | c.cl) & ex;
            }
        } else {
            T = c.tok;
        }
        const uint32_t cok = (c.co >> 1) | (l.co << 31);  // bit i: a colon at byte i + 1
        AJX_LEAN_TICK(g_lean_subs);
        while (T) {
            AJX_LEAN_TICK(g_lean_iters);
            const uint32_t i = ctz(T);
            T &= T - 1u;
            const uint32_t p = (uint32_t)(c.base + (int32_t)i);
            if (skipw) {
                AJX_LEAN_TRACE(0);
                if ((c.op >> i) & 1u) {
                    skipw++;
                } else if (((--skipw) & 0xFFFFFFu) == 0) {
                    if (skipw >> 24) record((int32_t)(skipw >> 24) - 1, skips, p + 1, T_JSON, 0);
                    skipw = 0;
                    T = c.tok & above(i);
                }
                continue;
            }
            if ((c.cq >> i) & 1u) {
                const bool kq = (cok >> i) & 1u;
                if (depth == 0 || (tarr && kq)) { st = S_SLOW; T = 0; break; }
                if (tarr) {  // a string element
                    AJX_LEAN_TRACE(1);
                    const uint32_t node = elem_node();
                    const int32_t s = leaf_sel(node);
                    if (s >= 0) {
                        const uint32_t so = (c.oq & below(i)) ? (uint32_t)c.base + hib(c.oq & below(i)) : carry_oq;
                        const bool esc = has_bs(so, p, c, l);
                        if (s >= 0) record(s, so, p + 1, T_STRING, esc ? 1u : 0u);
                    }
                    continue;
                }
                if (!expk) {  // the pending value string of a key
                    AJX_LEAN_TRACE(2);
                    if (kq) { st = S_SLOW; T = 0; break; }
                    const int32_t s = leaf_sel(pend >> 24);
                    const uint32_t ps = pend & 0xFFFFFFu;
                    if (s >= 0) record(s, ps, p + 1, T_STRING, has_bs(ps, p, c, l) ? 1u : 0u);
                    expk = 1;
                    continue;
                }
                if (!kq) { st = S_SLOW; T = 0; break; }  // a value where a key belongs
                // a key: [ks, p)
                const uint32_t ks0 = (c.oq & below(i)) ? (uint32_t)c.base + hib(c.oq & below(i)) : carry_oq;
                const uint32_t k0 = ks0 + 1, klen = p - k0;
                // (every object the walk is in has keys on selector paths: open() squashes
                // the others)
                if (klen >= kIdxKeyLen || has_bs(k0, p, c, l)) { st = S_SLOW; T = 0; break; }
                uint64_t sig = r64((p - 8u + mis) & 127u);
                sig = klen >= 8 ? sig : (klen ? sig >> (8 * (8 - klen)) : 0ull);
                const uint32_t node = lookup(sig, klen, top, k0);
                // its value at p + 2
                const uint32_t vs = p + 2, vb = rb(vs);
                const uint32_t rv = vs - (uint32_t)c.base;  // 2..33
                AJX_LEAN_TRACE(vb == '"' ? 3 : (vb == '{' || vb == '[') ? 4 : 5);
                if (vb == '"') {
                    const uint64_t cq = ((uint64_t)c.cq | ((uint64_t)l.cq << 32)) & (~0ull << (rv + 1));
                    if (cq) {
                        const uint32_t j = (uint32_t)__builtin_ctzll(cq);
                        if (j < 32) T &= ~(1u << j);
                        else l.tok &= ~(1u << (j - 32));
                        const int32_t s = leaf_sel(node);
                        const uint32_t e = (uint32_t)c.base + j;
                        if (s >= 0) record(s, vs, e + 1, T_STRING, has_bs(vs, e, c, l) ? 1u : 0u);
                    } else {
                        expk = 0;
                        pend = vs | (node << 24);  // (positions < 2^24)
                    }
                } else if (vb == '{' || vb == '[') {
                    if (rv < 32) T &= ~(1u << rv);
                    else l.tok &= ~(1u << (rv - 32));
                    open(node, vb == '[', vs);
                    if (skipw) T = rv < 32 ? T & (c.op | c.cl) & above(rv) : 0u;
                    else T = rv < 32 ? T & above(rv) : 0u;
                } else if (!scalar(node, vs, vb, c, l, false)) {
                    st = S_SLOW;
                    T = 0;
                    break;
                }
                continue;
            }
            if ((c.op >> i) & 1u) {
                AJX_LEAN_TRACE(depth == 0 ? 6 : 7);
                if (depth == 0) {  // the root
                    if (p != 0) { st = S_SLOW; T = 0; break; }
                    open(0, rb(p) == '[', p);
                    if (skipw) { st = S_SLOW; T = 0; break; }  // (a ruleset whose root node is a leaf)
                    continue;
                }
                if (!tarr) { st = S_SLOW; T = 0; break; }  // (a container where a key belongs)
                open(elem_node(), rb(p) == '[', p);
                if (skipw) T &= c.op | c.cl;
                continue;
            }
            if ((c.cl >> i) & 1u) {
                AJX_LEAN_TRACE(8);
                if (depth == 0 || tarr != (rb(p) == ']' ? 1u : 0u) || (!tarr && !expk)) { st = S_SLOW; T = 0; break; }
                close(p);
                if (st != S_RUN) { T = 0; break; }
                continue;
            }
            AJX_LEAN_TRACE(9);
            // an array element's scalar
            if (depth == 0 || !tarr) { st = S_SLOW; T = 0; break; }
            const uint32_t node = elem_node();
            if (!scalar(node, p, rb(p), c, l, true)) { st = S_SLOW; T = 0; break; }
        }
        if (c.oq) carry_oq = (uint32_t)c.base + hib(c.oq);
        if (c.bs) lbs1 = (uint32_t)c.base + hib(c.bs) + 1u;
    }
};

// Stage A for one request with the lean scan. `ring` = the work-item's 128-byte ring (lane:
// its lane in the wave, for the chunk swizzle),
// `load(b, nblk)` returns aligned 16-byte block b of the document (zeros past nblk). Returns
// true when the capture row is valid (false: the exact scan decides the request); dec[0] /
// dec[1]: the patterns decided while capturing / those of them that are true.
// ABL (profiling ablations, kernel modes 15..18; the row then holds a checksum): 1 loads and
// ring stores only, 2 + classification, 3 + the walk without eager patterns, 4 = stage A.
// keep: every capture goes to the row (a caller reads the rows after the kernel), else
// only those stage B needs.
template <int ABL = 0, class LoadBlock>
AJX_HD bool scan_doc(const uint8_t* blob, const Tables& tab, const uint8_t* d, uint32_t n, RowRef row, uint8_t* ring,
                     uint32_t lane, LoadBlock load, uint64_t dec[2], uint32_t keep = 1) {
    const RulesetHdr* h = (const RulesetHdr*)blob;
    Walk w;
    // the tables as the blob pointer plus uniform offsets: the offsets go to scalar registers
    // and the pointers keep the blob's provenance, so that with the blob staged in LDS every
    // table read is a ds_read (a pointer made uniform through an integer would be generic:
    // flat loads, which wait for the document's loads in flight as well)
    (void)tab;
    w.tn = reinterpret_cast<const TrieNode*>(blob + uni(h->off_trie_nodes));
    w.ks = reinterpret_cast<const KeySlot*>(blob + uni(h->off_key_slots));
    w.lits = blob + uni(h->off_literals);
    w.ks_mask = uni((1u << h->key_slots_log2) - 1u);
    w.ks_probes = uni(h->key_probes);
    w.ks_mult = uni(h->key_mult);
    w.ks_shift = uni(32u - h->key_slots_log2);
    w.d = d;
    w.n = n;
    w.mis = (uint32_t)((uintptr_t)d & 15u);
    w.ring = ring;
    w.sw16 = (lane & 7u) << 4;
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

    const uint32_t mis = w.mis;
    const uint32_t nblk = (n + mis + 15) / 16;
    const uint32_t nwin = (nblk + 3) / 4;  // 64-byte windows
    auto valid_of = [&](int32_t base) -> uint32_t {
        uint32_t v = ~0u;
        if (base < 0) v &= ~below((uint32_t)(-base));
        const int32_t hi = (int32_t)n - base;
        if (hi < 32) v &= hi <= 0 ? 0u : below((uint32_t)hi);
        return v;
    };
    auto put = [&](uint32_t slot0, const Block16* b) {  // a 64-byte window into ring slots slot0, slot0 + 1
#pragma unroll
        for (int q = 0; q < 4; q++)
            *reinterpret_cast<Block16*>(ring + w.ro(slot0 * 32u + 16u * (uint32_t)q)) = b[q];
    };
    // registers hold only the window on its way in (issued one sub-window's walk ahead of
    // its use); the halves classified later are read back from the ring
    Block16 nxt[4];
#pragma unroll
    for (int j = 0; j < 4; j++) nxt[j] = load((uint32_t)j, nblk);
    put(0, nxt);
    Sub s0, s1, s2;
    uint32_t ck = 0;  // (ablations: a checksum that keeps the skipped work's inputs live)
    {
        const uint32_t x0[8] = {nxt[0].x, nxt[0].y, nxt[0].z, nxt[0].w, nxt[1].x, nxt[1].y, nxt[1].z, nxt[1].w};
        classify(s0, x0, -(int32_t)mis, valid_of(-(int32_t)mis), cr);
        const uint32_t x1[8] = {nxt[2].x, nxt[2].y, nxt[2].z, nxt[2].w, nxt[3].x, nxt[3].y, nxt[3].z, nxt[3].w};
        classify(s1, x1, 32 - (int32_t)mis, valid_of(32 - (int32_t)mis), cr);
    }
    for (uint32_t win = 0; win < nwin; win++) {
        const int32_t b0 = (int32_t)(win * 64u) - (int32_t)mis;
        const bool more = win + 1 < nwin;
        if (more) {
#pragma unroll
            for (int j = 0; j < 4; j++) nxt[j] = load((win + 1) * 4u + (uint32_t)j, nblk);
        }
        if constexpr (ABL == 1) {
            if (more) {
                put(((win + 1) & 1u) * 2u, nxt);
                ck ^= nxt[0].x ^ nxt[1].y ^ nxt[2].z ^ nxt[3].w;
            }
            continue;
        }
        if constexpr (ABL == 2) {
            if (more) {
                const uint32_t slot2 = ((win + 1) & 1u) * 2u;
                put(slot2, nxt);
                const uint32_t x2[8] = {nxt[0].x, nxt[0].y, nxt[0].z, nxt[0].w, nxt[1].x, nxt[1].y, nxt[1].z, nxt[1].w};
                classify(s2, x2, b0 + 64, valid_of(b0 + 64), cr);
                const Block16 h0 = *reinterpret_cast<const Block16*>(ring + w.ro(slot2 * 32u + 32u));
                const Block16 h1 = *reinterpret_cast<const Block16*>(ring + w.ro(slot2 * 32u + 48u));
                const uint32_t x3[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
                classify(s1, x3, b0 + 96, valid_of(b0 + 96), cr);
                ck ^= s2.tok ^ s2.bs ^ s1.tok ^ s1.bs;
            }
            continue;
        }
        w.walk(s0, s1);
        if (w.st != S_RUN) break;
        // the next window into the ring (the slots of the sub-windows before this one)
        const uint32_t slot = ((win + 1) & 1u) * 2u;
        if (more) {
            put(slot, nxt);
            const uint32_t x2[8] = {nxt[0].x, nxt[0].y, nxt[0].z, nxt[0].w, nxt[1].x, nxt[1].y, nxt[1].z, nxt[1].w};
            classify(s2, x2, b0 + 64, valid_of(b0 + 64), cr);
        } else {
            s2.base = b0 + 64;
            s2.tok = s2.cq = s2.oq = s2.op = s2.cl = s2.co = s2.st = s2.bs = 0;
        }
        w.walk(s1, s2);
        if (w.st != S_RUN) break;
        if (more) {
            const Block16 h0 = *reinterpret_cast<const Block16*>(ring + w.ro(slot * 32u + 32u));
            const Block16 h1 = *reinterpret_cast<const Block16*>(ring + w.ro(slot * 32u + 48u));
            const uint32_t x3[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
            classify(s1, x3, b0 + 96, valid_of(b0 + 96), cr);
        }
        s0 = s2;
    }
    if constexpr (ABL == 1 || ABL == 2) {
        row[0] = (uint64_t)ck ^ ((uint64_t)(uint32_t)cr.bad << 32) ^ s0.tok ^ s1.tok;
        dec[0] = dec[1] = 0;
        return true;
    }
    if (w.st != S_DONE || cr.bad <= (int32_t)w.pend) {  // (pend: the root's close)
        row[0] = kRowSlow;
        return false;
    }
    row[0] = w.found;
    dec[0] = w.eD;
    dec[1] = w.eT;
    return true;
}

}  // namespace lean
}  // namespace ajx
