// ajx_float.h — Go strconv's ParseFloat(s, 64) and FormatFloat(f, 'f', -1, 64) for the
// numbers whose gjson Result.String() the cheap canon (ajx_device.h num_canon: <= 15
// significant digits, normal range) can not decide: 16+ significant digits (Go's
// encoding/json writes up to 17, e.g. 0.30000000000000004), subnormals and the ends of
// the range. Exact integer arithmetic on a small bignum; no floating-point rounding is
// trusted except IEEE-correct single operations.
//
//   parse  the decimal N * 10^E (N = its first 800 significant digits, `trunc` = a
//          non-zero digit after them, as Go's strconv/decimal keeps them) rounded to the
//          nearest float64, ties to even: a double-arithmetic estimate, then exact
//          comparisons against the halfway points of the estimate's neighbours
//          (Go: strconv/atof.go atof64 -> eiselLemire64 / decimal.floatBits; the result is
//          the correctly rounded value either way)
//   format the shortest decimal that parses back to f, the closest to f among those,
//          ties to an even last digit (Go: ryuFtoaShortest): for p = 1..17 the two p-digit
//          neighbours of f's exact expansion are tested against f's rounding interval
//
// Used by the exact scan (ajx_kernels.hip eval_scan_one) only; the single-pass kernels
// hand a request with such a number over to it. Device code in a work-item: a Big is
// 528 bytes of scratch.
#pragma once
#include <stdint.h>

#ifndef AJX_HD
#define AJX_HD __device__ __forceinline__
#endif

namespace ajx {

constexpr int kBigWords = 132;  // 4224 bits: 800 decimal digits * 2^1075, 5^1124 * 2^54

struct Big {
    uint32_t w[kBigWords];  // little-endian 32-bit words
    int n;                  // words in use (w[n - 1] != 0 unless n == 0)

    AJX_HD void set(uint64_t v) {
        n = 0;
        while (v) {
            w[n++] = (uint32_t)v;
            v >>= 32;
        }
    }
    AJX_HD void copy(const Big& o) {
        n = o.n;
        for (int i = 0; i < n; i++) w[i] = o.w[i];
    }
    AJX_HD void mul_add(uint32_t m, uint32_t a) {  // this = this * m + a
        uint64_t c = a;
        for (int i = 0; i < n; i++) {
            c += (uint64_t)w[i] * m;
            w[i] = (uint32_t)c;
            c >>= 32;
        }
        if (c && n < kBigWords) w[n++] = (uint32_t)c;
    }
    AJX_HD void mul_pow5(int k) {
        const uint32_t p5[14] = {1u, 5u, 25u, 125u, 625u, 3125u, 15625u, 78125u, 390625u, 1953125u, 9765625u,
                                 48828125u, 244140625u, 1220703125u};
        for (; k >= 13; k -= 13) mul_add(p5[13], 0);
        if (k) mul_add(p5[k], 0);
    }
    AJX_HD void shl(int k) {
        if (n == 0 || k <= 0) return;
        const int ws = k / 32, bs = k % 32;
        int top = n + ws + 1;
        if (top > kBigWords) top = kBigWords;
        for (int i = top - 1; i >= 0; i--) {
            const int j = i - ws;
            uint32_t v = 0;
            if (j >= 0 && j < n) v = bs ? w[j] << bs : w[j];
            if (bs && j - 1 >= 0 && j - 1 < n) v |= w[j - 1] >> (32 - bs);
            w[i] = v;
        }
        n = top;
        while (n > 0 && w[n - 1] == 0) n--;
    }
    AJX_HD uint32_t divmod(uint32_t d) {  // this /= d, returns the remainder
        uint64_t r = 0;
        for (int i = n - 1; i >= 0; i--) {
            r = (r << 32) | w[i];
            w[i] = (uint32_t)(r / d);
            r %= d;
        }
        while (n > 0 && w[n - 1] == 0) n--;
        return (uint32_t)r;
    }
    AJX_HD bool below(uint64_t v) const {  // this < v
        if (n > 2) return false;
        const uint64_t x = n == 0 ? 0ull : n == 1 ? (uint64_t)w[0] : ((uint64_t)w[1] << 32) | w[0];
        return x < v;
    }
    AJX_HD uint64_t low64() const {
        return n == 0 ? 0ull : n == 1 ? (uint64_t)w[0] : ((uint64_t)w[1] << 32) | w[0];
    }
};

AJX_HD int big_cmp(const Big& a, const Big& b) {
    if (a.n != b.n) return a.n < b.n ? -1 : 1;
    for (int i = a.n - 1; i >= 0; i--)
        if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
    return 0;
}

// sign of N * 10^E - K * 2^q (N >= 0 as a Big, K >= 0); t and u are work space
AJX_HD int cmp_dec_dyadic(const Big& N, int E, uint64_t K, int q, Big& t, Big& u) {
    const int e5a = E > 0 ? E : 0, e5b = E < 0 ? -E : 0;
    int a2 = e5a + (q < 0 ? -q : 0), b2 = e5b + (q > 0 ? q : 0);
    const int c = a2 < b2 ? a2 : b2;
    a2 -= c;
    b2 -= c;
    t.copy(N);
    t.mul_pow5(e5a);
    t.shl(a2);
    u.set(K);
    u.mul_pow5(e5b);
    u.shl(b2);
    return big_cmp(t, u);
}

AJX_HD uint64_t f64_bits(double x) {
    union {
        double d;
        uint64_t u;
    } v;
    v.d = x;
    return v.u;
}
AJX_HD double f64_from(uint64_t b) {
    union {
        double d;
        uint64_t u;
    } v;
    v.u = b;
    return v.d;
}

// x = m * 2^e with m < 2^53 (x finite, >= 0)
AJX_HD void f64_split(double x, uint64_t* m, int* e) {
    const uint64_t b = f64_bits(x);
    const int be = (int)((b >> 52) & 0x7FF);
    const uint64_t frac = b & ((1ull << 52) - 1);
    if (be == 0) {
        *m = frac;
        *e = -1074;
    } else {
        *m = frac | (1ull << 52);
        *e = be - 1075;
    }
}

// The float64 nearest to N * 10^E (+ a positive amount below one unit of the last digit
// when trunc), ties to even; N has nd decimal digits and w19 holds its first
// min(nd, 19) digits. +Inf when it rounds past MaxFloat64. t, u: work space.
AJX_HD double dec_to_f64(const Big& N, int nd, int E, bool trunc, uint64_t w19, Big& t, Big& u) {
    if (N.n == 0) return 0.0;
    const int dexp = nd + E;  // N * 10^E in [10^(dexp-1), 10^dexp)
    if (dexp > 310) return f64_from(0x7FF0000000000000ull);
    if (dexp < -324) return 0.0;
    // estimate: the first 19 digits, scaled by exact powers of ten (each step one
    // correctly rounded operation; intermediates stay normal until the last steps)
    const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                            1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    double x = (double)w19;
    int e10 = E + (nd > 19 ? nd - 19 : 0);
    while (e10 > 0) {
        const int s = e10 > 22 ? 22 : e10;
        x *= p10[s];
        e10 -= s;
    }
    while (e10 < 0) {
        const int s = -e10 > 22 ? 22 : -e10;
        x /= p10[s];
        e10 += s;
    }
    const uint64_t kInf = 0x7FF0000000000000ull, kMax = 0x7FEFFFFFFFFFFFFFull;
    uint64_t xb = f64_bits(x);
    for (int iter = 0; iter < 64; iter++) {
        if (xb >= kInf) {  // +Inf: the value may still round to MaxFloat64
            // halfway above MaxFloat64 = (2 (2^53 - 1) + 1) * 2^970; a tie goes to the
            // even neighbour, 2^53 * 2^971 = overflow
            int c = cmp_dec_dyadic(N, E, (1ull << 54) - 1, 970, t, u);
            if (c == 0 && trunc) c = 1;
            if (c < 0) { xb = kMax; continue; }
            return f64_from(kInf);
        }
        uint64_t m;
        int e;
        f64_split(f64_from(xb), &m, &e);
        // above the upper halfway point (or on it with an odd mantissa): one up
        int c = cmp_dec_dyadic(N, E, 2 * m + 1, e - 1, t, u);
        if (c == 0 && trunc) c = 1;
        if (c > 0 || (c == 0 && (m & 1))) { xb++; continue; }
        if (m == 0) break;
        // below the lower halfway point (or on it with an odd mantissa): one down
        const bool pow2 = m == (1ull << 52) && e > -1074;
        c = pow2 ? cmp_dec_dyadic(N, E, 4 * m - 1, e - 2, t, u) : cmp_dec_dyadic(N, E, 2 * m - 1, e - 1, t, u);
        if (c == 0 && trunc) c = 1;
        if (c < 0 || (c == 0 && (m & 1))) { xb--; continue; }
        break;
    }
    return f64_from(xb);
}

// shortest round-trip digits of f > 0 finite: dig[0..nd) (no trailing zeros), value =
// 0.dig * 10^dp. T, t, u: work space.
AJX_HD void f64_shortest(double f, uint8_t* dig, int* ond, int* odp, Big& T, Big& t, Big& u) {
    uint64_t m;
    int e;
    f64_split(f, &m, &e);
    // exact expansion: X * 10^E10 with X an integer
    T.set(m);
    int E10 = 0;
    if (e >= 0) T.shl(e);
    else {
        T.mul_pow5(-e);
        E10 = e;
    }
    // keep its leading 17..18 digits: X = x * 10^cut + rest
    int cut = 0;
    while (!T.below(1000000000000000000ull)) {  // X >= 10^18
        if (T.n > 3) {  // X >= 2^96 > 10^28: nine digits can go
            T.divmod(1000000000u);
            cut += 9;
        } else {
            T.divmod(10u);
            cut++;
        }
    }
    const uint64_t x = T.low64();  // < 10^18
    char s[20];
    int L = 0;
    for (uint64_t y = x; y; y /= 10) s[L++] = (char)('0' + y % 10);
    for (int i = 0; i < L / 2; i++) {
        const char c = s[i];
        s[i] = s[L - 1 - i];
        s[L - 1 - i] = c;
    }
    const int dp = L + cut + E10;
    // f's rounding interval: halfway points below / above, inclusive for an even mantissa
    const bool pow2 = m == (1ull << 52) && e > -1074;
    const uint64_t Klo = pow2 ? 4 * m - 1 : 2 * m - 1;
    const int qlo = pow2 ? e - 2 : e - 1;
    const bool incl = (m & 1) == 0;
    uint64_t lo = 0;
    for (int p = 1; p <= 17; p++) {
        lo = lo * 10 + (uint64_t)(p <= L ? s[p - 1] - '0' : 0);
        const int E = dp - p;  // candidate = digits * 10^E
        Big& D = T;
        D.set(lo);
        int c = cmp_dec_dyadic(D, E, Klo, qlo, t, u);
        const bool lo_ok = c > 0 || (c == 0 && incl);  // (lo <= f < the upper point)
        D.set(lo + 1);
        c = cmp_dec_dyadic(D, E, 2 * m + 1, e - 1, t, u);
        bool hi_ok = c < 0 || (c == 0 && incl);
        if (hi_ok && lo_ok) {
            // both round-trip: the closer; the midpoint lo + 1/2 against f, ties even
            D.set(lo * 10 + 5);
            c = cmp_dec_dyadic(D, E - 1, m, e, t, u);  // mid - f
            if (c > 0) hi_ok = false;
            else if (c == 0 && (lo & 1) == 0) hi_ok = false;
        }
        if (lo_ok || hi_ok) {
            uint64_t v = hi_ok ? lo + 1 : lo;
            int vd = p, vdp = dp;
            // hi may carry into a new digit: 10^p -> "1", one more integer digit
            uint64_t lim = 1;
            for (int i = 0; i < p; i++) lim *= 10;
            if (v == lim) {
                v = 1;
                vd = 1;
                vdp = dp + 1;
            }
            char o[20];
            for (int i = vd - 1; i >= 0; i--) {
                o[i] = (char)('0' + v % 10);
                v /= 10;
            }
            while (vd > 1 && o[vd - 1] == '0') vd--;
            for (int i = 0; i < vd; i++) dig[i] = (uint8_t)o[i];
            *ond = vd;
            *odp = vdp;
            return;
        }
    }
    // (unreachable: 17 digits always round-trip)
    for (int i = 0; i < 17; i++) dig[i] = (uint8_t)(i < L ? s[i] : '0');
    *ond = 17;
    *odp = dp;
}

}  // namespace ajx
