/*
 * gofloat_ref.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restates the two Go 1.21 strconv routines gjson's Result.String() relies on for
 * numbers whose raw text is not -?[0-9]+ (gjson v1.14.0 Result.String, Number case):
 *   ParseFloat(raw, 64)            (value kept even on error: 0 / +-Inf)
 *   FormatFloat(num, 'f', -1, 64)  (shortest round-trip digits, fixed layout)
 * Syntax acceptance follows Go's readFloat / special / underscoreOK rules; the value is
 * then obtained from glibc strtod (correctly rounded, round-half-even like Go).
 * Shortest digits: for p = 1..17 the two p-digit neighbours of the exact binary value
 * are tried and the one that round-trips is kept (closest when both do).
 */
#include <ctype.h>
#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static int lower(int c) { return c | 0x20; }

static size_t prefix_ci(const char* s, size_t n, const char* pre) {
    size_t k = strlen(pre), i = 0;
    if (n < k) k = n;
    for (; i < k; i++)
        if (lower((unsigned char)s[i]) != pre[i]) break;
    return i;
}

/* strconv.special: returns consumed length (0 = no). */
static size_t go_special(const char* s, size_t n, double* f) {
    if (n == 0) return 0;
    int sign = 1;
    size_t nsign = 0;
    const char* t = s;
    size_t tn = n;
    switch (s[0]) {
        case '+': case '-':
            if (s[0] == '-') sign = -1;
            nsign = 1;
            t = s + 1;
            tn = n - 1;
            /* fallthrough */
        case 'i': case 'I': {
            size_t k = prefix_ci(t, tn, "infinity");
            if (3 < k && k < 8) k = 3;
            if (k == 3 || k == 8) { *f = sign > 0 ? INFINITY : -INFINITY; return nsign + k; }
            return 0;
        }
        case 'n': case 'N':
            if (prefix_ci(s, n, "nan") == 3) { *f = NAN; return 3; }
            return 0;
    }
    return 0;
}

static int underscore_ok(const char* s, size_t n) {
    char saw = '^';
    size_t i = 0;
    if (n >= 1 && (s[0] == '-' || s[0] == '+')) { s++; n--; }
    int hex = 0;
    if (n >= 2 && s[0] == '0' && (lower(s[1]) == 'b' || lower(s[1]) == 'o' || lower(s[1]) == 'x')) {
        i = 2;
        saw = '0';
        hex = lower(s[1]) == 'x';
    }
    for (; i < n; i++) {
        int c = (unsigned char)s[i];
        if ((c >= '0' && c <= '9') || (hex && lower(c) >= 'a' && lower(c) <= 'f')) { saw = '0'; continue; }
        if (c == '_') {
            if (saw != '0') return 0;
            saw = '_';
            continue;
        }
        if (saw == '_') return 0;
        saw = '!';
    }
    return saw != '_';
}

/* readFloat syntax check; returns consumed length or 0 on syntax failure. */
static size_t go_read_float(const char* s, size_t n, int* hex_out) {
    size_t i = 0;
    int underscores = 0, hex = 0;
    if (i >= n) return 0;
    if (s[i] == '+' || s[i] == '-') i++;
    int base = 10;
    char exp_char = 'e';
    if (i + 2 < n && s[i] == '0' && lower((unsigned char)s[i + 1]) == 'x') {
        base = 16;
        i += 2;
        exp_char = 'p';
        hex = 1;
    }
    int sawdot = 0, sawdigits = 0;
    for (; i < n; i++) {
        int c = (unsigned char)s[i];
        if (c == '_') { underscores = 1; continue; }
        if (c == '.') {
            if (sawdot) break;
            sawdot = 1;
            continue;
        }
        if (c >= '0' && c <= '9') { sawdigits = 1; continue; }
        if (base == 16 && lower(c) >= 'a' && lower(c) <= 'f') { sawdigits = 1; continue; }
        break;
    }
    if (!sawdigits) return 0;
    if (i < n && lower((unsigned char)s[i]) == exp_char) {
        i++;
        if (i >= n) return 0;
        if (s[i] == '+' || s[i] == '-') i++;
        if (i >= n || s[i] < '0' || s[i] > '9') return 0;
        for (; i < n && ((s[i] >= '0' && s[i] <= '9') || s[i] == '_'); i++)
            if (s[i] == '_') underscores = 1;
    } else if (base == 16) {
        return 0; /* hexadecimal mantissa requires a 'p' exponent */
    }
    if (underscores && !underscore_ok(s, i)) return 0;
    *hex_out = hex;
    return i;
}

int or_go_parse_float(const char* s, size_t n, double* out) {
    double f;
    size_t k = go_special(s, n, &f);
    if (k) {
        if (k == n) { *out = f; return 0; }
        *out = 0;
        return 1;
    }
    int hex = 0;
    k = go_read_float(s, n, &hex);
    if (k == 0 || k != n) { *out = 0; return 1; }
    char stack[128];
    char* tmp = n + 1 <= sizeof(stack) ? stack : (char*)malloc(n + 1);
    size_t m = 0;
    for (size_t i = 0; i < n; i++)
        if (s[i] != '_') tmp[m++] = s[i];
    tmp[m] = 0;
    errno = 0;
    f = strtod(tmp, NULL);
    int range = (errno == ERANGE) && isinf(f);
    if (tmp != stack) free(tmp);
    *out = f;
    return range ? 2 : 0;
}

/* ---- FormatFloat(f, 'f', -1, 64) ---------------------------------------- */
/* Exact decimal digits of |f| (scientific): digits[] and decimal exponent such that
 * value = 0.d1d2d3... * 10^dp. */
static void exact_digits(double f, char* digits, int* nd, int* dp) {
    char buf[1100];
    snprintf(buf, sizeof buf, "%.780e", f); /* exact: doubles have <= 767 sig digits */
    const char* p = buf;
    int k = 0;
    digits[k++] = *p++;
    if (*p == '.') p++;
    while (*p && *p != 'e') digits[k++] = *p++;
    int e = atoi(p + 1);
    while (k > 1 && digits[k - 1] == '0') k--;
    *nd = k;
    *dp = e + 1;
}

static double digits_to_double(const char* d, int nd, int dp) {
    char buf[64];
    int k = 0;
    buf[k++] = '0';
    buf[k++] = '.';
    for (int i = 0; i < nd; i++) buf[k++] = d[i];
    k += snprintf(buf + k, sizeof(buf) - k, "e%d", dp);
    return strtod(buf, NULL);
}

/* shortest digits for finite, non-zero |f| */
static void shortest_digits(double f, char* out, int* ond, int* odp) {
    static __thread char ex[1100];
    int nd, dp;
    exact_digits(f, ex, &nd, &dp);
    for (int p = 1; p <= 17; p++) {
        if (p >= nd) { memcpy(out, ex, nd); *ond = nd; *odp = dp; return; }
        char lo[20], hi[20];
        memcpy(lo, ex, p);
        int lodp = dp, hidp = dp;
        /* hi = lo + 1 unit in the p-th digit */
        memcpy(hi, ex, p);
        int j = p - 1;
        while (j >= 0 && hi[j] == '9') { hi[j] = '0'; j--; }
        int hnd = p;
        if (j < 0) { hi[0] = '1'; hnd = 1; hidp = dp + 1; }
        else hi[j]++;
        int lo_ok = digits_to_double(lo, p, lodp) == f;
        int hi_ok = digits_to_double(hi, hnd, hidp) == f;
        if (lo_ok && hi_ok) {
            /* closest; remainder digits ex[p..] vs one half */
            int cmp = 0;
            if (ex[p] > '5') cmp = 1;
            else if (ex[p] < '5') cmp = -1;
            else {
                cmp = 0;
                for (int q = p + 1; q < nd; q++) if (ex[q] != '0') { cmp = 1; break; }
                if (cmp == 0) cmp = ((lo[p - 1] - '0') & 1) ? 1 : -1; /* tie: even */
            }
            if (cmp > 0) lo_ok = 0; else hi_ok = 0;
        }
        if (lo_ok) {
            int k = p;
            while (k > 1 && lo[k - 1] == '0') k--;
            memcpy(out, lo, k); *ond = k; *odp = lodp; return;
        }
        if (hi_ok) {
            int k = hnd;
            while (k > 1 && hi[k - 1] == '0') k--;
            memcpy(out, hi, k); *ond = k; *odp = hidp; return;
        }
    }
    memcpy(out, ex, 17);
    *ond = 17;
    *odp = dp;
}

void or_go_format_float(double f, or_buf* out) {
    if (isnan(f)) { or_buf_push(out, "NaN", 3); return; }
    if (isinf(f)) { or_buf_push(out, f > 0 ? "+Inf" : "-Inf", 4); return; }
    if (signbit(f)) or_buf_push(out, "-", 1);
    if (f == 0) { or_buf_push(out, "0", 1); return; }
    char d[24];
    int nd, dp;
    shortest_digits(fabs(f), d, &nd, &dp);
    /* %f layout: integer part, then '.' and max(nd-dp,0) fraction digits */
    if (dp > 0) {
        int m = dp < nd ? dp : nd;
        or_buf_push(out, d, (size_t)m);
        for (int i = m; i < dp; i++) or_buf_push(out, "0", 1);
    } else {
        or_buf_push(out, "0", 1);
    }
    int frac = nd - dp;
    if (frac > 0) {
        or_buf_push(out, ".", 1);
        for (int i = 0; i < frac; i++) {
            int j = dp + i;
            char c = (j < 0 || j >= nd) ? '0' : d[j];
            or_buf_push(out, &c, 1);
        }
    }
}
