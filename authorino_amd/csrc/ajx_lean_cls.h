// ajx_lean_cls.h — the lean scan's per-lane classification of 32-byte sub-windows (byte
// classes by v_perm LUT, the 32 x 8 bit transpose, escapes, strings and the compact-JSON
// grammar on 32-bit masks), shared by the lean walker (ajx_lean.h) and the streaming
// kernel (ajx_stream.h). See ajx_lean.h for the scan it serves.
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

}  // namespace lean
}  // namespace ajx
