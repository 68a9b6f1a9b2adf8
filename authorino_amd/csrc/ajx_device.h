// ajx_device.h — per-document evaluation logic of the hot path, written once as
// __device__ code for the gfx950 kernels (ajx_kernels.hip).
//
//   gj_get          gjson.Get for a compiled selector (gjson v1.14.0 parseObject /
//                   parseArray scan, iterative with an explicit frame stack instead of
//                   recursion; same skipping/squashing rules, so the same value is found
//                   in every document, well-formed or not)
//   StrSrc          Result.String() as a byte stream (string unescape, number
//                   canonical form, literals, raw JSON spans) — never materialised
//   ArrIter         Result.Array() element walk (arrayOrMap rules)
//   eval_pattern    Pattern.Matches (pkg/jsonexp/expressions.go:59-96)
//   run_fold        And/Or evaluation (expressions.go:111-154) over pattern results
//
// AJX_HD expands to __device__ in the product build. The test-only host harness
// (tests/native) compiles this header for the CPU to debug it against the oracle; the
// product library contains no host copy of it.
#pragma once
#include <stdint.h>

#include "ajx_blob.h"
#include "ajx_float.h"

#ifndef AJX_HD
#define AJX_HD __device__ __forceinline__
#endif
#ifndef AJX_COLD
#if defined(__HIPCC__)
#define AJX_COLD __device__ __attribute__((noinline))  // rare paths kept out of line
#else
#define AJX_COLD inline
#endif
#endif

namespace ajx {

struct ValueRef {
    uint32_t start;  // raw span [start, end) in the document
    uint32_t end;
    uint8_t type;    // T_*
    uint8_t esc;     // string contains a backslash (needs unescape); kValCount: a count
};
// ValueRef::esc of a Number that is an array's element count (a "#" part, kArrCount):
// not a document span — the count is in `start` (start == end)
constexpr uint8_t kValCount = 2;
// ValueRef::esc of the array a "#." list part stopped at (kArrList): [start, end) is the
// array; the exact scan builds the list text from it (ajx_modifiers.h build_list)
constexpr uint8_t kValList = 3;

// ---------------------------------------------------------------------------------
// scanning primitives (gjson parseString / parseSquash / parseNumber / parseLiteral)
// ---------------------------------------------------------------------------------

// backslashes immediately before position q, not looking at index <= lo
AJX_HD bool quote_is_escaped(const uint8_t* d, uint32_t q, uint32_t lo) {
    if (d[q - 1] != '\\') return false;
    uint32_t nb = 0;
    for (int64_t j = (int64_t)q - 2; j > (int64_t)lo; j--) {
        if (d[j] != '\\') break;
        nb++;
    }
    return (nb & 1) == 0;
}

// i = index just past the opening quote. Returns index after the closing quote; *ok
// false when unterminated (then returns n). *esc: a backslash was seen.
AJX_HD uint32_t scan_string(const uint8_t* d, uint32_t n, uint32_t i, bool* esc, bool* ok) {
    *esc = false;
    for (; i < n; i++) {
        uint8_t c = d[i];
        if (c > '\\') continue;
        if (c == '"') { *ok = true; return i + 1; }
        if (c == '\\') {
            *esc = true;
            i++;
            for (; i < n; i++) {
                c = d[i];
                if (c > '\\') continue;
                if (c == '"') {
                    if (quote_is_escaped(d, i, 0)) continue;
                    *ok = true;
                    return i + 1;
                }
            }
            break;
        }
    }
    *ok = false;
    *esc = false;
    return n;
}

// d[i] in "{[(" ; returns index after the matching close (or n)
AJX_HD uint32_t squash(const uint8_t* d, uint32_t n, uint32_t i) {
    int depth = 1;
    i++;
    for (; i < n; i++) {
        uint8_t c = d[i];
        if (c < '"' || c > '}') continue;
        if (c == '"') {
            i++;
            uint32_t s2 = i;
            for (; i < n; i++) {
                uint8_t e = d[i];
                if (e > '\\') continue;
                if (e == '"') {
                    if (d[i - 1] == '\\') {
                        uint32_t nb = 0;
                        for (int64_t j = (int64_t)i - 2; j >= (int64_t)s2; j--) {
                            if (d[j] != '\\') break;
                            nb++;
                        }
                        if ((nb & 1) == 0) continue;
                    }
                    break;
                }
            }
        } else if (c == '{' || c == '[' || c == '(') {
            depth++;
        } else if (c == '}' || c == ']' || c == ')') {
            if (--depth == 0) return i + 1;
        }
    }
    return n;
}

AJX_HD uint32_t scan_number(const uint8_t* d, uint32_t n, uint32_t i) {
    for (i++; i < n; i++) {
        uint8_t c = d[i];
        if (c <= ' ' || c == ',' || c == ']' || c == '}') return i;
    }
    return n;
}

AJX_HD uint32_t scan_literal(const uint8_t* d, uint32_t n, uint32_t i) {
    for (i++; i < n; i++) {
        uint8_t c = d[i];
        if (c < 'a' || c > 'z') return i;
    }
    return n;
}

// ---------------------------------------------------------------------------------
// byte streams
// ---------------------------------------------------------------------------------
AJX_HD uint32_t hexval4(const uint8_t* s) {
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) {
        uint8_t c = s[k];
        uint32_t x;
        if (c >= '0' && c <= '9') x = c - '0';
        else if (c >= 'a' && c <= 'f') x = c - 'a' + 10;
        else if (c >= 'A' && c <= 'F') x = c - 'A' + 10;
        else return 0;  // ParseUint error ignored -> 0
        v = v * 16 + x;
    }
    return v;
}

// the same UTF-8 bytes packed low byte first into *w (register-resident: no byte array)
AJX_HD uint32_t utf8_put32(uint32_t r, uint32_t* w) {
    if (r > 0x10FFFF || (r >= 0xD800 && r <= 0xDFFF)) r = 0xFFFD;
    if (r < 0x80) { *w = r; return 1; }
    if (r < 0x800) { *w = (0xC0 | (r >> 6)) | ((0x80 | (r & 0x3F)) << 8); return 2; }
    if (r < 0x10000) {
        *w = (0xE0 | (r >> 12)) | ((0x80 | ((r >> 6) & 0x3F)) << 8) | ((0x80 | (r & 0x3F)) << 16);
        return 3;
    }
    *w = (0xF0 | (r >> 18)) | ((0x80 | ((r >> 12) & 0x3F)) << 8) | ((0x80 | ((r >> 6) & 0x3F)) << 16) |
         ((0x80 | (r & 0x3F)) << 24);
    return 4;
}
AJX_HD uint32_t utf8_put(uint32_t r, uint8_t* o) {
    if (r > 0x10FFFF || (r >= 0xD800 && r <= 0xDFFF)) r = 0xFFFD;
    if (r < 0x80) { o[0] = (uint8_t)r; return 1; }
    if (r < 0x800) { o[0] = (uint8_t)(0xC0 | (r >> 6)); o[1] = (uint8_t)(0x80 | (r & 0x3F)); return 2; }
    if (r < 0x10000) {
        o[0] = (uint8_t)(0xE0 | (r >> 12));
        o[1] = (uint8_t)(0x80 | ((r >> 6) & 0x3F));
        o[2] = (uint8_t)(0x80 | (r & 0x3F));
        return 3;
    }
    o[0] = (uint8_t)(0xF0 | (r >> 18));
    o[1] = (uint8_t)(0x80 | ((r >> 12) & 0x3F));
    o[2] = (uint8_t)(0x80 | ((r >> 6) & 0x3F));
    o[3] = (uint8_t)(0x80 | (r & 0x3F));
    return 4;
}

// Canonical number text for Result.String() when Raw is not -?[0-9]+:
// FormatFloat(ParseFloat(raw), 'f', -1, 64). num_canon: exact without float arithmetic
// for decimals with <= 15 significant digits in the normal range (the shortest
// round-trip digits of such a double are the decimal's own digits); K_HARD otherwise,
// which num_canon_exact decides (ajx_float.h). Hex mantissas and '_' separators (never
// in JSON a Go encoder writes) stay undecided.
struct NumCanon {
    enum : uint8_t { K_ZERO, K_DIGITS, K_PINF, K_NINF, K_NAN, K_UNDECIDED, K_HARD };
    uint8_t kind;
    uint8_t neg;
    uint8_t nd;     // significant digits (<= 17)
    int16_t dp;     // value = 0.D * 10^dp
    // the digits D, one nibble each (digit i at bits 4i of dlo, the 17th in dhi): registers,
    // where a byte array indexed by position would live in scratch memory
    uint64_t dlo;
    uint8_t dhi;
    AJX_HD void set_dig(int i, uint8_t c) {
        const uint64_t v = (uint64_t)(c - '0') & 0xFull;
        if (i < 16) dlo = (dlo & ~(0xFull << (4 * i))) | (v << (4 * i));
        else dhi = (uint8_t)v;
    }
    AJX_HD int dig_at(int i) const { return '0' + (int)(i < 16 ? (dlo >> (4 * i)) & 0xFull : dhi); }
};

AJX_HD uint8_t lower_c(uint8_t c) { return c | 0x20; }

AJX_HD void num_canon(const uint8_t* s, uint32_t n, NumCanon* o) {
    o->neg = 0;
    o->nd = 0;
    o->dp = 0;
    o->dlo = 0;
    o->dhi = 0;
    // strconv.special: [+-]inf / [+-]infinity / nan (case-insensitive), whole string
    {
        uint32_t i = 0;
        bool neg = false, sgn = false;
        if (n > 0 && (s[0] == '+' || s[0] == '-')) { sgn = true; neg = s[0] == '-'; i = 1; }
        const char* inf = "infinity";
        uint32_t k = 0;
        while (k < 8 && i + k < n && lower_c(s[i + k]) == (uint8_t)inf[k]) k++;
        if (k > 3 && k < 8) k = 3;
        if ((k == 3 || k == 8) && i + k == n) {
            o->kind = neg ? NumCanon::K_NINF : NumCanon::K_PINF;
            return;
        }
        if (!sgn && n == 3 && lower_c(s[0]) == 'n' && lower_c(s[1]) == 'a' && lower_c(s[2]) == 'n') {
            o->kind = NumCanon::K_NAN;
            return;
        }
    }
    uint32_t i = 0;
    bool neg = false;
    if (i < n && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; i++; }
    if (i + 2 < n && s[i] == '0' && lower_c(s[i + 1]) == 'x') { o->kind = NumCanon::K_UNDECIDED; return; }
    for (uint32_t k = 0; k < n; k++)
        if (s[k] == '_') { o->kind = NumCanon::K_UNDECIDED; return; }
    // mantissa: value = 0.D * 10^dp, D = significant digits
    bool sawdot = false, sawdig = false, seen = false;
    int dp = 0, nsig = 0, last_nz = 0;
    for (; i < n; i++) {
        uint8_t c = s[i];
        if (c == '.') {
            if (sawdot) break;
            sawdot = true;
            continue;
        }
        if (c < '0' || c > '9') break;
        sawdig = true;
        if (!seen && c == '0') {
            if (sawdot) dp--;
            continue;
        }
        seen = true;
        if (nsig < 16) o->set_dig(nsig, c);
        nsig++;
        if (c != '0') last_nz = nsig;
        if (!sawdot) dp++;
    }
    // ParseFloat syntax errors return 0 (positive zero)
    if (!sawdig) { o->kind = NumCanon::K_ZERO; return; }
    int64_t e = 0;
    if (i < n && lower_c(s[i]) == 'e') {
        i++;
        if (i >= n) { o->kind = NumCanon::K_ZERO; return; }
        int64_t esign = 1;
        if (s[i] == '+' || s[i] == '-') { esign = s[i] == '-' ? -1 : 1; i++; }
        if (i >= n || s[i] < '0' || s[i] > '9') { o->kind = NumCanon::K_ZERO; return; }
        for (; i < n && s[i] >= '0' && s[i] <= '9'; i++)
            if (e < 10000) e = e * 10 + (s[i] - '0');
        e *= esign;
    }
    if (i != n) { o->kind = NumCanon::K_ZERO; return; }
    if (!seen) { o->kind = NumCanon::K_ZERO; o->neg = neg; return; }  // +-0
    o->neg = neg;
    if (last_nz > 15) { o->kind = NumCanon::K_HARD; return; }
    int64_t ndp = (int64_t)dp + e;
    if (ndp >= 310) { o->kind = neg ? NumCanon::K_NINF : NumCanon::K_PINF; return; }
    if (ndp >= 309 || ndp < -306) { o->kind = NumCanon::K_HARD; return; }
    o->kind = NumCanon::K_DIGITS;
    o->neg = neg;
    o->nd = (uint8_t)last_nz;
    o->dp = (int16_t)ndp;
}

// num_canon for a K_HARD decimal s[0, n) (syntax already accepted by num_canon):
// ParseFloat exactly (the first 800 significant digits and a sticky bit, as Go's
// strconv/decimal keeps them), then the shortest round-trip digits (ajx_float.h).
AJX_COLD void num_canon_exact(const uint8_t* s, uint32_t n, NumCanon* o) {
    Big N, t, u;
    uint32_t i = 0;
    const bool neg = n > 0 && s[0] == '-';
    if (n > 0 && (s[0] == '+' || s[0] == '-')) i = 1;
    bool sawdot = false, seen = false, trunc = false;
    int dp = 0, nd = 0;
    uint64_t w19 = 0;
    uint32_t chunk = 0, cmul = 1;
    N.set(0);
    for (; i < n; i++) {
        const uint8_t c = s[i];
        if (c == '.') {
            sawdot = true;
            continue;
        }
        if (c < '0' || c > '9') break;
        if (!seen && c == '0') {
            if (sawdot) dp--;
            continue;
        }
        seen = true;
        if (!sawdot) dp++;
        if (nd >= 800) {
            trunc = trunc || c != '0';
            continue;
        }
        if (nd < 19) w19 = w19 * 10 + (uint64_t)(c - '0');
        nd++;
        chunk = chunk * 10 + (uint32_t)(c - '0');
        cmul *= 10;
        if (cmul == 1000000000u) {
            N.mul_add(cmul, chunk);
            if (N.n == 0 && chunk) N.set(chunk);
            chunk = 0;
            cmul = 1;
        }
    }
    if (cmul > 1) {
        N.mul_add(cmul, chunk);
        if (N.n == 0 && chunk) N.set(chunk);
    }
    int64_t e = 0;
    if (i < n && (s[i] | 0x20) == 'e') {
        i++;
        int64_t es = 1;
        if (s[i] == '+' || s[i] == '-') { es = s[i] == '-' ? -1 : 1; i++; }
        for (; i < n && s[i] >= '0' && s[i] <= '9'; i++)
            if (e < 100000) e = e * 10 + (s[i] - '0');
        e *= es;
    }
    o->neg = neg;
    const int64_t ndp = (int64_t)dp + e;
    double f;
    if (ndp > 400) f = f64_from(0x7FF0000000000000ull);
    else if (ndp < -400) f = 0.0;
    else f = dec_to_f64(N, nd, (int)ndp - nd, trunc, w19, t, u);
    const uint64_t fb = f64_bits(f);
    if (fb == 0) { o->kind = NumCanon::K_ZERO; return; }  // underflow: +-0
    if (fb >= 0x7FF0000000000000ull) { o->kind = neg ? NumCanon::K_NINF : NumCanon::K_PINF; return; }
    int ond, odp;
    uint8_t dg[18];  // (the exact path only)
    f64_shortest(f, dg, &ond, &odp, N, t, u);
    o->dlo = 0;
    o->dhi = 0;
    for (int i = 0; i < ond; i++) o->set_dig(i, dg[i]);
    o->kind = NumCanon::K_DIGITS;
    o->nd = (uint8_t)ond;
    o->dp = (int16_t)odp;
}

// Character stream of a Result.String()
struct StrSrc {
    enum : uint8_t { S_RAW, S_UNESC, S_NUM, S_CONST };
    const uint8_t* p;
    uint32_t i, n;
    uint8_t kind;
    uint8_t bn, bi;
    bool done;
    uint32_t bufw;  // an escape's UTF-8 bytes, low byte first
    NumCanon num;
    int32_t pos;  // S_NUM output position
    int32_t total;

    AJX_HD void init_raw(const uint8_t* s, uint32_t a, uint32_t b) {
        p = s; i = a; n = b; kind = S_RAW; bn = bi = 0; done = false;
    }
    AJX_HD void init_unesc(const uint8_t* s, uint32_t a, uint32_t b) {
        p = s; i = a; n = b; kind = S_UNESC; bn = bi = 0; done = false;
    }
    AJX_HD void init_const(const char* s, uint32_t len) {
        p = (const uint8_t*)s; i = 0; n = len; kind = S_RAW; bn = bi = 0; done = false;
    }
    // returns false if the number can not be formatted exactly (undecided). EXACT (the
    // exact scan): K_HARD numbers through num_canon_exact; otherwise they are undecided
    // here (the single-pass kernels hand such requests to the exact scan)
    template <bool EXACT = false>
    AJX_HD bool init_num(const uint8_t* s, uint32_t a, uint32_t b) {
        kind = S_NUM; bn = bi = 0; done = false; pos = 0;
        num_canon(s + a, b - a, &num);
        if (EXACT && num.kind == NumCanon::K_HARD) num_canon_exact(s + a, b - a, &num);
        switch (num.kind) {
            case NumCanon::K_UNDECIDED:
            case NumCanon::K_HARD: return false;
            case NumCanon::K_ZERO: init_const(num.neg ? "-0" : "0", num.neg ? 2 : 1); return true;
            case NumCanon::K_PINF: init_const("+Inf", 4); return true;
            case NumCanon::K_NINF: init_const("-Inf", 4); return true;
            case NumCanon::K_NAN: init_const("NaN", 3); return true;
            default: break;
        }
        // layout: [-] intpart [. frac]
        int nd = num.nd, dp = num.dp;
        int intlen = dp > 0 ? dp : 1;
        int frac = nd - dp > 0 ? nd - dp : 0;
        total = (num.neg ? 1 : 0) + intlen + (frac > 0 ? 1 + frac : 0);
        return true;
    }
    AJX_HD int num_char(int k) const {
        if (num.neg) {
            if (k == 0) return '-';
            k--;
        }
        int nd = num.nd, dp = num.dp;
        int intlen = dp > 0 ? dp : 1;
        if (k < intlen) {
            if (dp <= 0) return '0';
            return k < nd ? num.dig_at(k) : '0';
        }
        if (k == intlen) return '.';
        int j = dp + (k - intlen - 1);  // digit index in 0.D*10^dp coordinates
        if (j < 0 || j >= nd) return '0';
        return num.dig_at(j);
    }
    AJX_HD int next() {
        if (kind == S_RAW) return i < n ? p[i++] : -1;
        if (kind == S_NUM) return pos < total ? num_char(pos++) : -1;
        // S_UNESC (gjson unescape)
        if (bi < bn) return (int)((bufw >> (8u * bi++)) & 0xFFu);
        if (done || i >= n) return -1;
        uint8_t c = p[i];
        if (c < ' ') { done = true; return -1; }
        if (c != '\\') { i++; return c; }
        i++;
        if (i >= n) { done = true; return -1; }
        uint8_t e = p[i];
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
                        uint32_t r2 = hexval4(p + i + 2);
                        if (r < 0xDC00 && r2 >= 0xDC00 && r2 < 0xE000)
                            r = (((r - 0xD800) << 10) | (r2 - 0xDC00)) + 0x10000;
                        else
                            r = 0xFFFD;
                        i += 6;
                    }
                }
                bn = (uint8_t)utf8_put32(r, &bufw);
                bi = 1;
                return (int)(bufw & 0xFFu);
            }
            default: done = true; return -1;
        }
        i++;
        return out;
    }
};

// Result.String() stream for a value. Returns false when undecided.
template <bool EXACT = false>
AJX_HD bool string_of(const uint8_t* d, const ValueRef& v, StrSrc* s) {
    switch (v.type) {
        case T_STRING:
            if (v.esc) s->init_unesc(d, v.start + 1, v.end - 1);
            else s->init_raw(d, v.start + 1, v.end - 1);
            return true;
        case T_NUMBER: {
            if (v.esc == kValCount) {  // an element count: its decimal digits
                uint32_t x = v.start, nd = 0;
                for (uint32_t y = x; ; y /= 10u) { nd++; if (y < 10u) break; }
                s->kind = StrSrc::S_NUM; s->bn = s->bi = 0; s->done = false; s->pos = 0;
                s->num.kind = NumCanon::K_DIGITS; s->num.neg = 0; s->num.nd = (uint8_t)nd; s->num.dp = (int16_t)nd;
                s->num.dlo = 0; s->num.dhi = 0;
                for (int j = (int)nd - 1; j >= 0; j--, x /= 10u) s->num.set_dig(j, (uint8_t)('0' + x % 10u));
                s->total = (int32_t)nd;
                return true;
            }
            uint32_t k = v.start;
            if (k < v.end && d[k] == '-') k++;
            for (; k < v.end; k++)
                if (d[k] < '0' || d[k] > '9') break;
            if (k == v.end) { s->init_raw(d, v.start, v.end); return true; }
            return s->template init_num<EXACT>(d, v.start, v.end);
        }
        case T_TRUE: s->init_const("true", 4); return true;
        case T_FALSE: s->init_const("false", 5); return true;
        case T_JSON: s->init_raw(d, v.start, v.end); return true;
        default: s->init_const("", 0); return true;
    }
}

// the 4 bytes at p (any alignment) from the aligned dword(s) holding them; the second
// dword is read only when a byte lies in it. (Pointer arithmetic, not an integer cast,
// keeps the address space of an LDS pointer.)
AJX_HD uint32_t load_u32_any(const uint8_t* p) {
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t* q = (const uint32_t*)(p - sh);
    const uint32_t w0 = q[0];
    const uint32_t w1 = sh ? q[1] : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbyte(w1, w0, sh);
#else
    return sh ? (w0 >> (8 * sh)) | (w1 << (32 - 8 * sh)) : w0;
#endif
}

// a[0..len) == b[0..len), 16 bytes per step (their loads issued together: one memory
// latency per step on a document re-read in stage B), then a dword at a time
AJX_HD bool bytes_equal(const uint8_t* a, const uint8_t* b, uint32_t len) {
    uint32_t k = 0;
    for (; k + 16 <= len; k += 16) {
        const uint32_t x0 = load_u32_any(a + k), x1 = load_u32_any(a + k + 4), x2 = load_u32_any(a + k + 8),
                       x3 = load_u32_any(a + k + 12);
        const uint32_t y0 = load_u32_any(b + k), y1 = load_u32_any(b + k + 4), y2 = load_u32_any(b + k + 8),
                       y3 = load_u32_any(b + k + 12);
        if ((x0 ^ y0) | (x1 ^ y1) | (x2 ^ y2) | (x3 ^ y3)) return false;
    }
    for (; k + 4 <= len; k += 4)
        if (load_u32_any(a + k) != load_u32_any(b + k)) return false;
    for (; k < len; k++)
        if (a[k] != b[k]) return false;
    return true;
}

// stream == literal ?
AJX_HD bool stream_equals(StrSrc* s, const uint8_t* lit, uint32_t len) {
    if (s->kind == StrSrc::S_RAW) {
        if (s->n - s->i != len) return false;
        return bytes_equal(s->p + s->i, lit, len);
    }
    for (uint32_t k = 0; k < len; k++) {
        int c = s->next();
        if (c != (int)lit[k]) return false;
    }
    return s->next() < 0;
}

// ---------------------------------------------------------------------------------
// gjson.Get over a compiled selector
// ---------------------------------------------------------------------------------
AJX_HD bool key_matches(const uint8_t* d, uint32_t ks, uint32_t ke, bool kesc, const uint8_t* lit,
                        uint32_t len) {
    if (!kesc) {
        if (ke - ks != len) return false;
        for (uint32_t k = 0; k < len; k++)
            if (d[ks + k] != lit[k]) return false;
        return true;
    }
    StrSrc s;
    s.init_unesc(d, ks, ke);
    return stream_equals(&s, lit, len);
}

AJX_HD ValueRef gj_get(const uint8_t* d, uint32_t n, const Component* comps, uint32_t nc,
                       const uint8_t* lits) {
    ValueRef none;
    none.start = none.end = 0;
    none.type = T_NULL;
    none.esc = 0;
    uint32_t i = 0;
    while (i < n && d[i] != '{' && d[i] != '[') i++;
    if (i >= n || nc == 0) return none;
    uint8_t ftype[kMaxComponents];
    int32_t fh[kMaxComponents];
    uint32_t fs[kMaxComponents];  // the container's opening bracket
    int depth = 0;
    ftype[0] = d[i];
    fh[0] = 0;
    fs[0] = i;
    i++;
    for (;;) {
        const Component& c = comps[depth];
        const bool more = (uint32_t)depth + 1 < nc;
        bool pmatch;
        const bool is_arr = ftype[depth] == '[';
        if (!is_arr) {
            // key scan: next '"' starts a key, '}' ends the object
            bool ok = false, kesc = false, closed = false;
            uint32_t ks = 0, ke = 0;
            for (; i < n; i++) {
                if (d[i] == '"') {
                    ks = i + 1;
                    i = scan_string(d, n, i + 1, &kesc, &ok);
                    ke = i - 1;
                    break;
                }
                if (d[i] == '}') { closed = true; break; }
            }
            if (closed) {
                i++;
                if (depth == 0) return none;
                depth--;
                continue;  // parent resumes after this value
            }
            if (!ok) return none;
            pmatch = key_matches(d, ks, ke, kesc, lits + c.lit_off, c.lit_len);
        } else {
            pmatch = c.array_index == fh[depth];
            fh[depth]++;
        }
        const bool hit = pmatch && !more;
        // value scan
        bool popped = false, pushed = false;
        for (;; i++) {
            uint8_t ch;
            if (is_arr) {
                if (i > n) return none;
                ch = i == n ? (uint8_t)']' : d[i];
            } else {
                if (i >= n) return none;
                ch = d[i];
            }
            bool num = false;
            if (ch == '"') {
                bool esc, ok;
                uint32_t s0 = i;
                i = scan_string(d, n, i + 1, &esc, &ok);
                if (!ok) return none;
                if (hit) {
                    ValueRef v;
                    v.start = s0; v.end = i; v.type = T_STRING; v.esc = esc ? 1 : 0;
                    return v;
                }
                break;
            } else if (ch == '{' || ch == '[') {
                if (pmatch && !hit) {
                    depth++;
                    ftype[depth] = ch;
                    fh[depth] = 0;
                    fs[depth] = i;
                    i++;
                    pushed = true;
                    break;
                }
                uint32_t s0 = i;
                i = squash(d, n, i);
                if (hit) {
                    ValueRef v;
                    v.start = s0; v.end = i; v.type = T_JSON; v.esc = 0;
                    return v;
                }
                break;
            } else if (ch == 'n' && !(i + 1 < n && d[i + 1] != 'u')) {
                uint32_t s0 = i;
                i = scan_literal(d, n, i);
                if (hit) { ValueRef v; v.start = s0; v.end = i; v.type = T_NULL; v.esc = 0; return v; }
                break;
            } else if (ch == 't' || ch == 'f') {
                uint32_t s0 = i;
                i = scan_literal(d, n, i);
                if (hit) {
                    ValueRef v; v.start = s0; v.end = i; v.type = ch == 't' ? T_TRUE : T_FALSE; v.esc = 0;
                    return v;
                }
                break;
            } else if (ch == 'n' || ch == '+' || ch == '-' || (ch >= '0' && ch <= '9') || ch == 'i' ||
                       ch == 'I' || ch == 'N') {
                num = true;
            } else if (is_arr && ch == ']') {
                if (c.array_index == kArrCount && !more) {  // parseArray: Number(h - 1) at ']'
                    ValueRef v;
                    v.start = v.end = (uint32_t)(fh[depth] - 1);
                    v.type = T_NUMBER;
                    v.esc = kValCount;
                    return v;
                }
                if (c.array_index == kArrList) {  // parseArray alog: the list is built at ']'
                    ValueRef v;
                    v.start = fs[depth];
                    v.end = i + 1;
                    v.type = T_JSON;
                    v.esc = kValList;
                    return v;
                }
                i++;
                if (depth == 0) return none;
                depth--;
                popped = true;
                break;
            } else {
                continue;
            }
            if (num) {
                uint32_t s0 = i;
                i = scan_number(d, n, i);
                if (hit) { ValueRef v; v.start = s0; v.end = i; v.type = T_NUMBER; v.esc = 0; return v; }
                break;
            }
        }
        (void)popped;
        (void)pushed;
    }
}

// ---------------------------------------------------------------------------------
// Result.Array() (arrayOrMap '[' path)
// ---------------------------------------------------------------------------------
struct ArrIter {
    const uint8_t* d;
    uint32_t i, n;  // cursor within the raw array span
    bool single;    // non-array value: one element, itself
    bool done;
    ValueRef self;

    AJX_HD void init(const uint8_t* doc, const ValueRef& v) {
        d = doc;
        self = v;
        done = false;
        single = false;
        if (v.type == T_NULL) { done = true; return; }
        if (!(v.type == T_JSON && v.end > v.start && doc[v.start] == '[')) { single = true; return; }
        i = v.start;
        n = v.end;
        // skip to '[' (any byte > ' ' first ends it)
        for (; i < n; i++) {
            if (d[i] == '[') { i++; return; }
            if (d[i] > ' ') { done = true; return; }
        }
        done = true;
    }

    AJX_HD bool next(ValueRef* out) {
        if (done) return false;
        if (single) { *out = self; done = true; return true; }
        for (; i < n; i++) {
            uint8_t c = d[i];
            if (c <= ' ') continue;
            if (c == ']' || c == '}') { done = true; return false; }
            ValueRef v;
            v.start = i;
            v.esc = 0;
            if ((c >= '0' && c <= '9') || c == '-') {
                uint32_t k = i + 1;
                for (; k < n; k++) {
                    uint8_t e = d[k];
                    if (e <= ' ' || e == ',' || e == ']' || e == '}') break;
                }
                v.end = k;
                v.type = T_NUMBER;
            } else if (c == '{' || c == '[') {
                v.end = squash(d, n, i);
                v.type = T_JSON;
            } else if (c == 'n' || c == 't' || c == 'f') {
                v.end = scan_literal(d, n, i);
                v.type = c == 'n' ? T_NULL : c == 't' ? T_TRUE : T_FALSE;
            } else if (c == '"') {
                bool esc, ok;
                uint32_t e = scan_string(d, n, i + 1, &esc, &ok);
                v.type = T_STRING;
                if (ok) {
                    v.end = e;
                    v.esc = esc ? 1 : 0;
                } else {
                    // tostr on an unterminated string: contents run to the span end
                    v.end = n + 1;  // so that [start+1, end-1) = [start+1, n)
                    v.esc = 1;      // unescape() also stops at control bytes
                    // detect whether a backslash exists (tostr only unescapes then)
                    bool anybs = false;
                    for (uint32_t k = i + 1; k < n; k++)
                        if (d[k] == '\\') { anybs = true; break; }
                    v.esc = anybs ? 1 : 0;
                }
            } else {
                continue;
            }
            i = v.end > n ? n : v.end;
            *out = v;
            return true;
        }
        done = true;
        return false;
    }
};

// ---------------------------------------------------------------------------------
// Go regexp DFA over runes
// ---------------------------------------------------------------------------------
struct RuneReader {
    StrSrc* src;
    uint32_t law;  // the look-ahead bytes, low byte first (registers, not a byte array)
    int nla;
    AJX_HD void init(StrSrc* s) { src = s; nla = 0; law = 0; }
    AJX_HD uint32_t la(int k) const { return (law >> (8 * k)) & 0xFFu; }
    AJX_HD void fill() {
        while (nla < 4) {
            int c = src->next();
            if (c < 0) break;
            law |= (uint32_t)(c & 0xFF) << (8 * nla);
            nla++;
        }
    }
    // Go utf8.DecodeRune; returns -1 at end
    AJX_HD int32_t next() {
        fill();
        if (nla == 0) return -1;
        uint32_t b0 = la(0);
        int sz = 1;
        uint32_t r = 0xFFFD;
        if (b0 < 0x80) {
            r = b0;
        } else {
            int need = 0;
            uint32_t lo = 0x80, hi = 0xBF, v = 0;
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
            if (need && nla >= need && la(1) >= lo && la(1) <= hi) {
                bool good = true;
                v = (v << 6) | (la(1) & 0x3F);
                for (int k = 2; k < need; k++) {
                    if (la(k) < 0x80 || la(k) > 0xBF) { good = false; break; }
                    v = (v << 6) | (la(k) & 0x3F);
                }
                if (good) { r = v; sz = need; }
            }
        }
        law = sz >= 4 ? 0u : law >> (8 * sz);
        nla -= sz;
        return (int32_t)r;
    }
};

AJX_HD uint32_t rune_class(const DfaHdr* h, const uint8_t* blob, int32_t r) {
    if (r < 0x80) return h->ascii_class[r];
    const RuneRange* rg = (const RuneRange*)(blob + h->ranges_off);
    uint32_t lo = 0, hi = h->n_ranges;
    while (lo + 1 < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (rg[mid].lo <= (uint32_t)r) lo = mid;
        else hi = mid;
    }
    return rg[lo].cls;
}

AJX_HD bool dfa_match(const uint8_t* blob, uint32_t dfa_off, StrSrc* s) {
    const DfaHdr* h = (const DfaHdr*)(blob + dfa_off);
    const uint16_t* tr = (const uint16_t*)(blob + h->trans_off);
    const uint8_t* eot = blob + h->eot_off;
    uint32_t st = h->start;
    if (st == h->match_state) return true;
    const uint32_t nc = h->n_classes, ms = h->match_state;
    if (s->kind == StrSrc::S_RAW) {  // contiguous bytes: ASCII four at a time, utf8.DecodeRune otherwise
        const uint8_t* p = s->p;
        uint32_t i = s->i;
        const uint32_t n = s->n;
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
        return eot[st] != 0;
    }
    RuneReader rd;
    rd.init(s);
    for (;;) {
        int32_t r = rd.next();
        if (r < 0) break;
        st = tr[st * h->n_classes + rune_class(h, blob, r)];
        if (st == h->match_state) return true;
    }
    return eot[st] != 0;
}

// ---------------------------------------------------------------------------------
// Pattern.Matches on a resolved value
// ---------------------------------------------------------------------------------
// EXACT: the exact scan's instance (every number decided, ajx_float.h); the
// single-pass kernels' instance returns V_U for a number it leaves to the exact scan
template <bool EXACT = false>
AJX_HD uint8_t eval_pattern(const uint8_t* blob, const Pattern& p, const uint8_t* doc, const ValueRef& v) {
    if (p.state == P_STATIC_E) return V_E;
    if (p.state == P_UNSUPPORTED) return V_U;
    const RulesetHdr* hdr = (const RulesetHdr*)blob;
    const uint8_t* lit = blob + hdr->off_literals + p.lit_off;
    switch (p.op) {
        case OP_EQ:
        case OP_NEQ: {
            StrSrc s;
            if (!string_of<EXACT>(doc, v, &s)) return V_U;
            bool eq = stream_equals(&s, lit, p.lit_len);
            return (eq == (p.op == OP_EQ)) ? V_T : V_F;
        }
        case OP_INCL:
        case OP_EXCL: {
            ArrIter it;
            it.init(doc, v);
            ValueRef e;
            bool found = false, und = false;
            while (it.next(&e)) {
                StrSrc s;
                if (!string_of<EXACT>(doc, e, &s)) { und = true; continue; }
                if (stream_equals(&s, lit, p.lit_len)) { found = true; break; }
            }
            if (!found && und) return V_U;
            return (found == (p.op == OP_INCL)) ? V_T : V_F;
        }
        case OP_MATCHES: {
            StrSrc s;
            if (!string_of<EXACT>(doc, v, &s)) return V_U;
            return dfa_match(blob, p.dfa_off, &s) ? V_T : V_F;
        }
        default: return V_E;
    }
}

// ---------------------------------------------------------------------------------
// fold evaluation of the And/Or tree
// ---------------------------------------------------------------------------------
// result: low byte = tri-state, err pattern in *err (or -1)
template <typename ResFn>
AJX_HD uint8_t run_fold(const uint32_t* code, uint32_t n_code, ResFn res, int32_t* err) {
    uint8_t kind[kMaxDepth];
    uint8_t val[kMaxDepth];
    int32_t ep[kMaxDepth];
    int sp = 0;
    uint8_t out = V_T;
    int32_t out_ep = -1;
    for (uint32_t k = 0; k < n_code; k++) {
        uint32_t w = code[k];
        uint32_t op = w >> 24, arg = w & 0xFFFFFF;
        uint8_t v = V_T;
        int32_t e = -1;
        switch (op) {
            case C_OPEN_AND: kind[sp] = 0; val[sp] = V_T; ep[sp] = -1; sp++; continue;
            case C_OPEN_OR: kind[sp] = 1; val[sp] = V_F; ep[sp] = -1; sp++; continue;
            case C_CONST_T: v = V_T; break;
            case C_CONST_F: v = V_F; break;
            case C_PAT:
                v = res(arg);
                if (v == V_E || v == V_U) e = (int32_t)arg;
                break;
            case C_CLOSE:
                sp--;
                v = val[sp];
                e = ep[sp];
                break;
        }
        if (sp == 0) {
            out = v;
            out_ep = e;
        } else {
            const uint8_t ident = kind[sp - 1] == 0 ? V_T : V_F;
            if (val[sp - 1] == ident) {
                val[sp - 1] = v;
                ep[sp - 1] = e;
            }
        }
    }
    *err = (out == V_E || out == V_U) ? out_ep : -1;
    return out;
}

// run_fold for rulesets of at most 128 patterns whose results are bitmaps (T, undecided,
// static E): the same evaluation with the stack packed into registers — kind 1 bit,
// value 2 bits, error pattern + 1 in 8 bits per level — instead of indexed arrays
// (which would live in scratch memory).
AJX_HD uint64_t sel64(bool c, uint64_t a, uint64_t b) { return c ? a : b; }  // a value select

// fetch(k): code word k (run_fold_bits: from memory; a wave running one fold together can
// hand out words it holds in registers)
template <class Fetch>
AJX_HD uint8_t run_fold_bits_f(Fetch fetch, uint32_t n_code, const uint64_t t[2], const uint64_t u[2],
                               const uint64_t se[2], int32_t* err) {
    const uint64_t t0 = t[0], t1 = t[1], u0 = u[0], u1 = u[1], s0 = se[0], s1 = se[1];
    uint32_t kinds = 0, vals = 0;
    uint64_t ep_lo = 0, ep_hi = 0;  // levels 0..7 / 8..15
    uint32_t sp = 0;
    uint32_t out = V_T, out_e = 0;
    for (uint32_t k = 0; k < n_code; k++) {
        const uint32_t w = fetch(k);
        const uint32_t op = w >> 24, arg = w & 0xFFFFFFu;
        uint32_t v = V_T, e = 0;
        if (op == C_OPEN_AND || op == C_OPEN_OR) {
            const uint32_t sh = 2 * sp;
            kinds = (kinds & ~(1u << sp)) | ((op == C_OPEN_OR ? 1u : 0u) << sp);
            vals = (vals & ~(3u << sh)) | ((op == C_OPEN_OR ? (uint32_t)V_F : (uint32_t)V_T) << sh);
            const uint64_t m = ~(0xFFull << ((sp & 7) * 8));
            ep_lo = sel64(sp < 8, ep_lo & m, ep_lo);
            ep_hi = sel64(sp < 8, ep_hi, ep_hi & m);
            sp++;
            continue;
        }
        if (op == C_CONST_F) v = V_F;
        if (op == C_PAT) {
            const uint64_t bit = 1ull << (arg & 63);
            const uint32_t q = arg >> 6;
            const uint64_t tq = sel64(q != 0, t1, t0), uq = sel64(q != 0, u1, u0), sq = sel64(q != 0, s1, s0);
            v = (sq & bit) ? V_E : (uq & bit) ? V_U : (tq & bit) ? V_T : V_F;
            e = (v == V_E || v == V_U) ? arg + 1 : 0u;
        }
        if (op == C_CLOSE) {
            sp--;
            v = (vals >> (2 * sp)) & 3u;
            e = (uint32_t)((sel64(sp < 8, ep_lo, ep_hi) >> ((sp & 7) * 8)) & 0xFFu);
        }
        if (sp == 0) {
            out = v;
            out_e = e;
        } else {
            const uint32_t top = sp - 1;
            const uint32_t ident = ((kinds >> top) & 1u) ? (uint32_t)V_F : (uint32_t)V_T;
            if (((vals >> (2 * top)) & 3u) == ident) {
                vals = (vals & ~(3u << (2 * top))) | (v << (2 * top));
                const uint64_t m = 0xFFull << ((top & 7) * 8), x = (uint64_t)e << ((top & 7) * 8);
                ep_lo = sel64(top < 8, (ep_lo & ~m) | x, ep_lo);
                ep_hi = sel64(top < 8, ep_hi, (ep_hi & ~m) | x);
            }
        }
    }
    *err = (out == V_E || out == V_U) ? (int32_t)out_e - 1 : -1;
    return (uint8_t)out;
}
AJX_HD uint8_t run_fold_bits(const uint32_t* code, uint32_t n_code, const uint64_t t[2], const uint64_t u[2],
                             const uint64_t se[2], int32_t* err) {
    return run_fold_bits_f([&](uint32_t k) { return code[k]; }, n_code, t, u, se, err);
}

}  // namespace ajx
