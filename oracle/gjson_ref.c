/*
 * gjson_ref.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restatement of github.com/tidwall/gjson v1.14.0 (go.mod:22, go.sum:530) Get / Result
 * String / Result Array, for the paths the reference's hot path uses
 * (pkg/jsonexp/expressions.go:61,65,68,71,79,91). The gjson source is absent from the
 * reference tree; behaviour follows the published v1.14.0 algorithm: a left-to-right
 * byte scan that descends only into the value whose key matches the current path
 * component and skips ("squashes") every other value by bracket depth. Every scanning
 * quirk that changes results on odd input (escaped-quote detection by counting
 * backslashes, numbers ending only at whitespace/,/]/}, literals ending at the first
 * byte outside a-z, parentheses counted by the squash) is kept.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

void or_buf_reset(or_buf* b) { b->n = 0; }
void or_buf_free(or_buf* b) {
    free(b->p);
    b->p = NULL;
    b->n = b->cap = 0;
}
void or_buf_push(or_buf* b, const char* s, size_t n) {
    if (b->n + n + 1 > b->cap) {
        size_t c = b->cap ? b->cap : 64;
        while (c < b->n + n + 1) c *= 2;
        b->p = (char*)realloc(b->p, c);
        b->cap = c;
    }
    if (n) memcpy(b->p + b->n, s, n);
    b->n += n;
    b->p[b->n] = 0;
}
static void buf_putc(or_buf* b, char c) { or_buf_push(b, &c, 1); }

void or_result_free(or_result* r) { or_buf_free(&r->own); }

static void result_clear(or_result* r) {
    or_buf own = r->own;
    memset(r, 0, sizeof(*r));
    r->own = own;
    or_buf_reset(&r->own);
}

/* ---- UTF-8 / UTF-16 helpers (Go unicode/utf8, unicode/utf16) ---------------- */
static size_t utf8_encode(unsigned r, char* o) {
    /* utf8.EncodeRune: invalid runes (surrogates, > 0x10FFFF) encode as U+FFFD */
    if (r > 0x10FFFF || (r >= 0xD800 && r <= 0xDFFF)) r = 0xFFFD;
    if (r < 0x80) { o[0] = (char)r; return 1; }
    if (r < 0x800) { o[0] = (char)(0xC0 | (r >> 6)); o[1] = (char)(0x80 | (r & 0x3F)); return 2; }
    if (r < 0x10000) {
        o[0] = (char)(0xE0 | (r >> 12)); o[1] = (char)(0x80 | ((r >> 6) & 0x3F));
        o[2] = (char)(0x80 | (r & 0x3F)); return 3;
    }
    o[0] = (char)(0xF0 | (r >> 18)); o[1] = (char)(0x80 | ((r >> 12) & 0x3F));
    o[2] = (char)(0x80 | ((r >> 6) & 0x3F)); o[3] = (char)(0x80 | (r & 0x3F));
    return 4;
}

/* gjson runeit(): strconv.ParseUint(s[:4], 16, 64) with the error ignored (-> 0). */
static unsigned runeit(const char* s) {
    unsigned v = 0;
    for (int i = 0; i < 4; i++) {
        char c = s[i];
        unsigned d;
        if (c >= '0' && c <= '9') d = (unsigned)(c - '0');
        else if (c >= 'a' && c <= 'f') d = (unsigned)(c - 'a' + 10);
        else if (c >= 'A' && c <= 'F') d = (unsigned)(c - 'A' + 10);
        else return 0; /* ParseUint error -> n == 0 */
        v = v * 16 + d;
    }
    return v;
}

/* gjson unescape(): restated. Stops (returns what it has) at a raw control byte
 * (< 0x20), at a trailing backslash and at an unknown escape letter. \uXXXX with a
 * surrogate consumes a following \uXXXX and combines them (utf16.DecodeRune,
 * U+FFFD when they do not form a pair); the rune is written with utf8.EncodeRune. */
void or_unescape(const char* s, size_t n, or_buf* out) {
    for (size_t i = 0; i < n; i++) {
        unsigned char c = (unsigned char)s[i];
        if (c < ' ') return;
        if (c != '\\') { buf_putc(out, (char)c); continue; }
        i++;
        if (i >= n) return;
        switch (s[i]) {
            case '\\': buf_putc(out, '\\'); break;
            case '/': buf_putc(out, '/'); break;
            case 'b': buf_putc(out, '\b'); break;
            case 'f': buf_putc(out, '\f'); break;
            case 'n': buf_putc(out, '\n'); break;
            case 'r': buf_putc(out, '\r'); break;
            case 't': buf_putc(out, '\t'); break;
            case '"': buf_putc(out, '"'); break;
            case 'u': {
                if (i + 5 > n) return;
                unsigned r = runeit(s + i + 1);
                i += 5;
                if (r >= 0xD800 && r < 0xE000) {
                    if (n - i >= 6 && s[i] == '\\' && s[i + 1] == 'u') {
                        unsigned r2 = runeit(s + i + 2);
                        /* utf16.DecodeRune */
                        if (r >= 0xD800 && r < 0xDC00 && r2 >= 0xDC00 && r2 < 0xE000)
                            r = (((r - 0xD800) << 10) | (r2 - 0xDC00)) + 0x10000;
                        else
                            r = 0xFFFD;
                        i += 6;
                    }
                }
                char tmp[4];
                size_t k = utf8_encode(r, tmp);
                or_buf_push(out, tmp, k);
                i--; /* backtrack by one: the loop increments */
                break;
            }
            default: return;
        }
    }
}

/* ---- scanning primitives ------------------------------------------------- */
typedef struct {
    const char* json;
    size_t len;
    or_result* value;
} pctx;

/* Is the quote at json[i] escaped? gjson counts the backslashes before it, looking
 * no further back than index lo+1 (parseString/tostr use lo=0; parseSquash uses
 * the string start). */
static int quote_escaped(const char* json, size_t i, size_t lo) {
    if (json[i - 1] != '\\') return 0;
    size_t nb = 0;
    for (size_t j = i - 2; j > lo && j < i; j--) {
        if (json[j] != '\\') break;
        nb++;
        if (j == 0) break;
    }
    return nb % 2 == 0;
}

/* parseString(json, i) with i just past the opening quote. Returns the index after
 * the string; [rs,re) = quoted span; *esc set when a backslash was seen;
 * *ok = 0 when the string is unterminated. */
static size_t parse_string(const char* json, size_t len, size_t i, size_t* rs, size_t* re, int* esc,
                           int* ok) {
    size_t s = i;
    for (; i < len; i++) {
        unsigned char c = (unsigned char)json[i];
        if (c > '\\') continue;
        if (c == '"') { *rs = s - 1; *re = i + 1; *esc = 0; *ok = 1; return i + 1; }
        if (c == '\\') {
            i++;
            for (; i < len; i++) {
                c = (unsigned char)json[i];
                if (c > '\\') continue;
                if (c == '"') {
                    if (quote_escaped(json, i, 0)) continue;
                    *rs = s - 1; *re = i + 1; *esc = 1; *ok = 1;
                    return i + 1;
                }
            }
            break;
        }
    }
    *rs = s - 1; *re = len; *esc = 0; *ok = 0;
    return i;
}

/* parseSquash: json[i] is '[' '{' or '('; skips the whole value. */
static size_t parse_squash(const char* json, size_t len, size_t i, size_t* end) {
    int depth = 1;
    i++;
    for (; i < len; i++) {
        unsigned char c = (unsigned char)json[i];
        if (c >= '"' && c <= '}') {
            switch (c) {
                case '"': {
                    i++;
                    size_t s2 = i;
                    for (; i < len; i++) {
                        unsigned char d = (unsigned char)json[i];
                        if (d > '\\') continue;
                        if (d == '"') {
                            if (json[i - 1] == '\\') {
                                size_t nb = 0;
                                for (size_t j = i - 2; j + 1 > s2 && j < i; j--) { /* j > s2-1 */
                                    if (json[j] != '\\') break;
                                    nb++;
                                    if (j == 0) break;
                                }
                                if (nb % 2 == 0) continue;
                            }
                            break;
                        }
                    }
                    break;
                }
                case '{': case '[': case '(': depth++; break;
                case '}': case ']': case ')':
                    depth--;
                    if (depth == 0) { *end = i + 1; return i + 1; }
                    break;
                default: break;
            }
        }
    }
    *end = len;
    return i;
}

static size_t parse_number(const char* json, size_t len, size_t i) {
    i++;
    for (; i < len; i++) {
        unsigned char c = (unsigned char)json[i];
        if (c <= ' ' || c == ',' || c == ']' || c == '}') return i;
    }
    return i;
}

static size_t parse_literal(const char* json, size_t len, size_t i) {
    i++;
    for (; i < len; i++) {
        unsigned char c = (unsigned char)json[i];
        if (c < 'a' || c > 'z') return i;
    }
    return i;
}

static void set_string_value(pctx* c, size_t rs, size_t re, int esc) {
    or_result* v = c->value;
    v->type = OR_STRING;
    v->raw = c->json + rs;
    v->raw_len = re - rs;
    if (esc) {
        or_buf_reset(&v->own);
        or_unescape(c->json + rs + 1, re - rs - 2, &v->own);
        or_buf_push(&v->own, "", 0);
        v->str = v->own.p;
        v->str_len = v->own.n;
    } else {
        v->str = c->json + rs + 1;
        v->str_len = re - rs - 2;
    }
}

static void set_number_value(pctx* c, size_t s, size_t e) {
    or_result* v = c->value;
    v->type = OR_NUMBER;
    v->raw = c->json + s;
    v->raw_len = e - s;
    double d = 0;
    or_go_parse_float(v->raw, v->raw_len, &d);
    v->num = d;
}

/* ---- path parsing (parseObjectPath / parseArrayPath) ---------------------- */
typedef struct {
    char* part; /* object part with escapes removed (malloc'd) */
    size_t part_len;
    const char* path; /* remainder after the separator */
    size_t path_len;
    int more, wild, piped;
} objpath;

static int is_dot_piper(const char* s, size_t n) {
    /* isDotPiperChar: '@' followed by a registered modifier name, '[' or '{'. The
     * oracle treats every '@' as a modifier (or_path_supported rejects them). */
    (void)n;
    return s[0] == '@' || s[0] == '[' || s[0] == '{';
}

static void parse_object_path(const char* path, size_t n, objpath* r) {
    memset(r, 0, sizeof(*r));
    for (size_t i = 0; i < n; i++) {
        char c = path[i];
        if (c == '|') {
            r->part = strndup(path, i);
            r->part_len = i;
            r->piped = 1;
            return;
        }
        if (c == '.') {
            r->part = strndup(path, i);
            r->part_len = i;
            if (i < n - 1 && is_dot_piper(path + i + 1, n - i - 1)) {
                r->piped = 1;
            } else {
                r->path = path + i + 1;
                r->path_len = n - i - 1;
                r->more = 1;
            }
            return;
        }
        if (c == '*' || c == '?') { r->wild = 1; continue; }
        if (c == '\\') {
            /* escape mode: strip the escape characters from the part */
            char* ep = (char*)malloc(n + 1);
            size_t k = i;
            memcpy(ep, path, i);
            i++;
            if (i < n) {
                ep[k++] = path[i];
                i++;
                for (; i < n; i++) {
                    if (path[i] == '\\') {
                        i++;
                        if (i < n) ep[k++] = path[i];
                        continue;
                    } else if (path[i] == '.') {
                        r->part = ep; r->part_len = k;
                        if (i < n - 1 && is_dot_piper(path + i + 1, n - i - 1)) {
                            r->piped = 1;
                        } else {
                            r->path = path + i + 1;
                            r->path_len = n - i - 1;
                            r->more = 1;
                        }
                        return;
                    } else if (path[i] == '|') {
                        r->part = ep; r->part_len = k; r->piped = 1;
                        return;
                    } else if (path[i] == '*' || path[i] == '?') {
                        r->wild = 1;
                    }
                    ep[k++] = path[i];
                }
            }
            r->part = ep;
            r->part_len = k;
            return;
        }
    }
    r->part = strndup(path, n);
    r->part_len = n;
}

typedef struct {
    const char* part;
    size_t part_len;
    const char* path;
    size_t path_len;
    int more, piped, arrch;
    int alogok;            /* "#.key": the list of each element's key */
    const char* alogkey;
    size_t alogkey_len;
} arrpath;

static void parse_array_path(const char* path, size_t n, arrpath* r) {
    memset(r, 0, sizeof(*r));
    for (size_t i = 0; i < n; i++) {
        if (path[i] == '|') {
            r->part = path; r->part_len = i; r->piped = 1;
            return;
        }
        if (path[i] == '.') {
            r->part = path; r->part_len = i;
            if (!r->arrch && i < n - 1 && is_dot_piper(path + i + 1, n - i - 1)) {
                r->piped = 1;
            } else {
                r->path = path + i + 1;
                r->path_len = n - i - 1;
                r->more = 1;
            }
            return;
        }
        if (path[i] == '#') {
            r->arrch = 1; /* ("#(" "#[" queries are rejected up front) */
            if (i == 0 && n > 1 && path[1] == '.') {
                r->alogok = 1;
                r->alogkey = path + 2;
                r->alogkey_len = n - 2;
            }
        }
    }
    r->part = path;
    r->part_len = n;
}

/* parseUint (gjson): digits only, non-empty; value wraps like uint64. */
static int parse_uint(const char* s, size_t n, uint64_t* v) {
    if (n == 0) return 0;
    uint64_t x = 0;
    for (size_t i = 0; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return 0;
        x = x * 10 + (uint64_t)(s[i] - '0');
    }
    *v = x;
    return 1;
}

static size_t parse_object(pctx* c, size_t i, const char* path, size_t plen, int* hit_out);

/* parseAny (hit): the extent [*s, *e) of the first value at or after json[i] */
static int any_span(const char* json, size_t len, size_t i, size_t* s, size_t* e) {
    for (; i < len; i++) {
        unsigned char ch = (unsigned char)json[i];
        if (ch <= ' ') continue;
        *s = i;
        if (ch == '"') {
            size_t rs, re; int esc, ok;
            size_t k = parse_string(json, len, i + 1, &rs, &re, &esc, &ok);
            *e = k;
            return ok;
        }
        if (ch == '{' || ch == '[') { parse_squash(json, len, i, e); return 1; }
        if (ch == 'n' && !(i + 1 < len && json[i + 1] != 'u')) { *e = parse_literal(json, len, i); return 1; }
        if (ch == 't' || ch == 'f') { *e = parse_literal(json, len, i); return 1; }
        if (ch == '-' || ch == '+' || (ch >= '0' && ch <= '9') || ch == 'i' || ch == 'I' || ch == 'N' || ch == 'n') {
            *e = parse_number(json, len, i);
            return 1;
        }
        /* (anything else, e.g. the ',' an element position starts at: skipped) */
    }
    return 0;
}

static size_t parse_array(pctx* c, size_t i, const char* path, size_t plen, int* hit_out) {
    arrpath rp;
    parse_array_path(path, plen, &rp);
    int64_t partidx = -1;
    uint64_t u;
    if (!rp.arrch && parse_uint(rp.part, rp.part_len, &u)) partidx = (int64_t)u;
    const char* json = c->json;
    size_t len = c->len;
    int64_t h = 0;
    size_t alog[4096];
    size_t nalog = 0;
    while (i < len + 1) {
        int pmatch = (partidx == h);
        int hit = pmatch && !rp.more;
        h++;
        if (rp.alogok && nalog < sizeof alog / sizeof alog[0]) alog[nalog++] = i;
        for (;; i++) {
            unsigned char ch;
            if (i > len) break;
            else if (i == len) ch = ']';
            else ch = (unsigned char)json[i];
            int num = 0;
            switch (ch) {
                default: continue;
                case '"': {
                    size_t rs, re; int esc, ok;
                    i = parse_string(json, len, i + 1, &rs, &re, &esc, &ok);
                    if (!ok) { *hit_out = 0; return i; }
                    if (hit) { set_string_value(c, rs, re, esc); *hit_out = 1; return i; }
                    break;
                }
                case '{': case '[': {
                    if (pmatch && !hit) {
                        int h2 = 0;
                        if (ch == '{') i = parse_object(c, i + 1, rp.path, rp.path_len, &h2);
                        else i = parse_array(c, i + 1, rp.path, rp.path_len, &h2);
                        if (h2) { *hit_out = 1; return i; }
                    } else {
                        size_t s = i, e;
                        i = parse_squash(json, len, i, &e);
                        if (hit) {
                            c->value->type = OR_JSON;
                            c->value->raw = json + s;
                            c->value->raw_len = e - s;
                            *hit_out = 1;
                            return i;
                        }
                    }
                    break;
                }
                case 'n':
                    if (i + 1 < len && json[i + 1] != 'u') { num = 1; break; }
                    /* fallthrough */
                case 't': case 'f': {
                    unsigned char vc = (unsigned char)json[i];
                    size_t s = i;
                    i = parse_literal(json, len, i);
                    if (hit) {
                        c->value->raw = json + s;
                        c->value->raw_len = i - s;
                        c->value->type = vc == 't' ? OR_TRUE : vc == 'f' ? OR_FALSE : OR_NULL;
                        *hit_out = 1;
                        return i;
                    }
                    break;
                }
                case '+': case '-': case '0': case '1': case '2': case '3': case '4':
                case '5': case '6': case '7': case '8': case '9': case 'i': case 'I': case 'N':
                    num = 1;
                    break;
                case ']':
                    if (rp.arrch && rp.part_len == 1 && rp.part[0] == '#' && rp.alogok) {
                        /* the list: Get(element, alogkey).Raw of each element where it exists */
                        or_buf lst = {0};
                        or_buf_push(&lst, "[", 1);
                        size_t k = 0;
                        for (size_t j = 0; j < nalog; j++) {
                            size_t idx = alog[j];
                            while (idx < len && (json[idx] == ' ' || json[idx] == '\t' || json[idx] == '\r' ||
                                                 json[idx] == '\n'))
                                idx++;
                            size_t es, ee;
                            if (idx < len && json[idx] != ']' && any_span(json, len, idx, &es, &ee)) {
                                or_result sub;
                                memset(&sub, 0, sizeof sub);
                                if (or_gjson_get(json + es, ee - es, rp.alogkey, rp.alogkey_len, &sub) == 0 &&
                                    sub.raw_len > 0) {
                                    if (k++) or_buf_push(&lst, ",", 1);
                                    or_buf_push(&lst, sub.raw, sub.raw_len);
                                }
                                or_result_free(&sub);
                            }
                        }
                        or_buf_push(&lst, "]", 1);
                        or_buf_reset(&c->value->own);
                        or_buf_push(&c->value->own, lst.p, lst.n);
                        or_buf_free(&lst);
                        c->value->type = OR_JSON;
                        c->value->raw = c->value->own.p;
                        c->value->raw_len = c->value->own.n;
                        *hit_out = 1;
                        return i + 1;
                    }
                    if (rp.arrch && rp.part_len == 1 && rp.part[0] == '#' && !rp.more) {
                        /* the element count: Number(h - 1), Raw = strconv.Itoa(h - 1) */
                        char dg[24];
                        int nd = snprintf(dg, sizeof dg, "%lld", (long long)(h - 1));
                        or_buf_reset(&c->value->own);
                        or_buf_push(&c->value->own, dg, (size_t)nd);
                        c->value->type = OR_NUMBER;
                        c->value->raw = c->value->own.p;
                        c->value->raw_len = (size_t)nd;
                        c->value->num = (double)(h - 1);
                        *hit_out = 1;
                        return i + 1;
                    }
                    *hit_out = 0;
                    return i + 1;
            }
            if (num) {
                size_t s = i;
                i = parse_number(json, len, i);
                if (hit) {
                    set_number_value(c, s, i);
                    *hit_out = 1;
                    return i;
                }
            }
            break;
        }
    }
    *hit_out = 0;
    return i;
}

static size_t parse_object(pctx* c, size_t i, const char* path, size_t plen, int* hit_out) {
    objpath rp;
    parse_object_path(path, plen, &rp);
    const char* json = c->json;
    size_t len = c->len;
    size_t ret = i;
    int found = 0;
    while (i < len) {
        size_t ks = 0, ke = 0;
        int kesc = 0, ok = 0;
        for (; i < len; i++) {
            if (json[i] == '"') {
                size_t rs, re;
                i = parse_string(json, len, i + 1, &rs, &re, &kesc, &ok);
                ks = rs + 1;
                ke = ok ? re - 1 : len;
                break;
            }
            if (json[i] == '}') { ret = i + 1; goto done; }
        }
        if (!ok) { ret = i; goto done; }
        int pmatch;
        if (kesc) {
            or_buf kb = {0};
            or_unescape(json + ks, ke - ks, &kb);
            pmatch = (kb.n == rp.part_len) && (kb.n == 0 || memcmp(kb.p, rp.part, kb.n) == 0);
            or_buf_free(&kb);
        } else {
            pmatch = (ke - ks == rp.part_len) && memcmp(json + ks, rp.part, rp.part_len) == 0;
        }
        int hit = pmatch && !rp.more;
        for (; i < len; i++) {
            unsigned char ch = (unsigned char)json[i];
            int num = 0;
            switch (ch) {
                default: continue;
                case '"': {
                    size_t rs, re; int esc, ok2;
                    i = parse_string(json, len, i + 1, &rs, &re, &esc, &ok2);
                    if (!ok2) { ret = i; goto done; }
                    if (hit) { set_string_value(c, rs, re, esc); found = 1; ret = i; goto done; }
                    break;
                }
                case '{': case '[': {
                    if (pmatch && !hit) {
                        int h2 = 0;
                        if (ch == '{') i = parse_object(c, i + 1, rp.path, rp.path_len, &h2);
                        else i = parse_array(c, i + 1, rp.path, rp.path_len, &h2);
                        if (h2) { found = 1; ret = i; goto done; }
                    } else {
                        size_t s = i, e;
                        i = parse_squash(json, len, i, &e);
                        if (hit) {
                            c->value->type = OR_JSON;
                            c->value->raw = json + s;
                            c->value->raw_len = e - s;
                            found = 1; ret = i; goto done;
                        }
                    }
                    break;
                }
                case 'n':
                    if (i + 1 < len && json[i + 1] != 'u') { num = 1; break; }
                    /* fallthrough */
                case 't': case 'f': {
                    unsigned char vc = (unsigned char)json[i];
                    size_t s = i;
                    i = parse_literal(json, len, i);
                    if (hit) {
                        c->value->raw = json + s;
                        c->value->raw_len = i - s;
                        c->value->type = vc == 't' ? OR_TRUE : vc == 'f' ? OR_FALSE : OR_NULL;
                        found = 1; ret = i; goto done;
                    }
                    break;
                }
                case '+': case '-': case '0': case '1': case '2': case '3': case '4':
                case '5': case '6': case '7': case '8': case '9': case 'i': case 'I': case 'N':
                    num = 1;
                    break;
            }
            if (num) {
                size_t s = i;
                i = parse_number(json, len, i);
                if (hit) { set_number_value(c, s, i); found = 1; ret = i; goto done; }
            }
            break;
        }
        ret = i;
    }
    ret = i;
done:
    free(rp.part);
    *hit_out = found;
    return ret;
}

int or_path_supported(const char* p, size_t n) {
    if (n == 0) return 0;
    if (n > 1 && (p[0] == '@' || p[0] == '!' || p[0] == '[' || p[0] == '{')) return -1;
    if (n >= 2 && p[0] == '.' && p[1] == '.') return -1;
    for (size_t i = 0; i < n; i++) {
        char c = p[i];
        if (c == '\\') { i++; if (i < n && (p[i] == '|' || p[i] == '#')) return -1; continue; }
        if (c == '|' || c == '*' || c == '?') return -1;
        /* '#' array forms: "#(" "#[" queries are not restated; a part "#" on an array
         * is its element count, "#.key" the list of the elements' keys (no further '#'
         * in that key path) */
        if (c == '#' && i + 1 < n && (p[i + 1] == '(' || p[i + 1] == '[')) return -1;
        if (c == '#' && i + 1 < n && p[i + 1] == '.' && (i == 0 || p[i - 1] == '.') &&
            memchr(p + i + 1, '#', n - i - 1))
            return -1;
        if (c == '.' && i + 1 < n && (p[i + 1] == '@' || p[i + 1] == '[' || p[i + 1] == '{')) return -1;
    }
    return 0;
}

int or_gjson_get(const char* json, size_t jlen, const char* path, size_t plen, or_result* r) {
    result_clear(r);
    if (or_path_supported(path, plen) != 0) return -1;
    pctx c = {json, jlen, r};
    for (size_t i = 0; i < jlen; i++) {
        int hit = 0;
        if (json[i] == '{') { parse_object(&c, i + 1, path, plen, &hit); break; }
        if (json[i] == '[') { parse_array(&c, i + 1, path, plen, &hit); break; }
    }
    return 0;
}

/* ---- Result.String ------------------------------------------------------- */
void or_result_string(const or_result* r, or_buf* out) {
    switch (r->type) {
        default: return; /* Null */
        case OR_FALSE: or_buf_push(out, "false", 5); return;
        case OR_TRUE: or_buf_push(out, "true", 4); return;
        case OR_STRING: or_buf_push(out, r->str, r->str_len); return;
        case OR_JSON: or_buf_push(out, r->raw, r->raw_len); return;
        case OR_NUMBER: {
            size_t i = 0;
            if (r->raw_len == 0) { or_go_format_float(r->num, out); return; }
            if (r->raw[0] == '-') i++;
            for (; i < r->raw_len; i++) {
                if (r->raw[i] < '0' || r->raw[i] > '9') { or_go_format_float(r->num, out); return; }
            }
            or_buf_push(out, r->raw, r->raw_len);
            return;
        }
    }
}

/* ---- Result.Array (arrayOrMap with vc='[') -------------------------------- */
/* tonum / tolit / tostr / squash as used by arrayOrMap. */
static size_t tonum_len(const char* s, size_t n) {
    for (size_t i = 1; i < n; i++) {
        unsigned char c = (unsigned char)s[i];
        if (c <= '-') {
            if (c <= ' ' || c == ',') return i;
        } else if (c == ']' || c == '}') {
            return i;
        }
    }
    return n;
}
static size_t tolit_len(const char* s, size_t n) {
    for (size_t i = 1; i < n; i++) {
        unsigned char c = (unsigned char)s[i];
        if (c < 'a' || c > 'z') return i;
    }
    return n;
}
/* tostr: returns raw length; *esc / str span for the contents. */
static size_t tostr_len(const char* s, size_t n, int* esc, size_t* str_end) {
    for (size_t i = 1; i < n; i++) {
        unsigned char c = (unsigned char)s[i];
        if (c > '\\') continue;
        if (c == '"') { *esc = 0; *str_end = i; return i + 1; }
        if (c == '\\') {
            i++;
            for (; i < n; i++) {
                c = (unsigned char)s[i];
                if (c > '\\') continue;
                if (c == '"') {
                    if (s[i - 1] == '\\') {
                        size_t nb = 0;
                        for (size_t j = i - 2; j > 0 && j < i; j--) {
                            if (s[j] != '\\') break;
                            nb++;
                        }
                        if (nb % 2 == 0) continue;
                    }
                    *esc = 1; *str_end = i;
                    return i + 1;
                }
            }
            *esc = 1;
            *str_end = i;
            return (i + 1 < n) ? i + 1 : i;
        }
    }
    *esc = 0;
    *str_end = n; /* json[1:] */
    return n;
}
static size_t squash_len(const char* s, size_t n) {
    size_t e;
    parse_squash(s, n, 0, &e);
    return e;
}

int or_result_array_next(const or_result* r, size_t* cursor, or_result* item) {
    result_clear(item);
    if (r->type == OR_NULL) return 0;
    int is_array = r->type == OR_JSON && r->raw_len > 0 && r->raw[0] == '[';
    if (!is_array) {
        if (*cursor != 0) return 0;
        *cursor = 1;
        item->type = r->type;
        item->raw = r->raw;
        item->raw_len = r->raw_len;
        item->num = r->num;
        if (r->type == OR_STRING) {
            or_buf_push(&item->own, r->str, r->str_len);
            item->str = item->own.p;
            item->str_len = r->str_len;
        }
        return 1;
    }
    const char* json = r->raw;
    size_t n = r->raw_len;
    size_t i = *cursor;
    if (i == 0) {
        /* skip to the opening '[' (anything > ' ' first ends the scan: no items) */
        for (; i < n; i++) {
            if (json[i] == '[') { i++; break; }
            if ((unsigned char)json[i] > ' ') { *cursor = n; return 0; }
        }
    }
    for (; i < n; i++) {
        unsigned char c = (unsigned char)json[i];
        if (c <= ' ') continue;
        if (c == ']' || c == '}') { *cursor = n; return 0; }
        size_t vl;
        switch (c) {
            default:
                if ((c >= '0' && c <= '9') || c == '-') {
                    vl = tonum_len(json + i, n - i);
                    item->type = OR_NUMBER;
                    item->raw = json + i;
                    item->raw_len = vl;
                    or_go_parse_float(item->raw, vl, &item->num);
                } else {
                    continue;
                }
                break;
            case '{': case '[':
                vl = squash_len(json + i, n - i);
                item->type = OR_JSON; item->raw = json + i; item->raw_len = vl;
                break;
            case 'n':
                vl = tolit_len(json + i, n - i);
                item->type = OR_NULL; item->raw = json + i; item->raw_len = vl;
                break;
            case 't':
                vl = tolit_len(json + i, n - i);
                item->type = OR_TRUE; item->raw = json + i; item->raw_len = vl;
                break;
            case 'f':
                vl = tolit_len(json + i, n - i);
                item->type = OR_FALSE; item->raw = json + i; item->raw_len = vl;
                break;
            case '"': {
                int esc; size_t se;
                vl = tostr_len(json + i, n - i, &esc, &se);
                item->type = OR_STRING; item->raw = json + i; item->raw_len = vl;
                if (esc) {
                    or_unescape(json + i + 1, se - 1, &item->own);
                } else {
                    or_buf_push(&item->own, json + i + 1, se - 1);
                }
                or_buf_push(&item->own, "", 0);
                item->str = item->own.p;
                item->str_len = item->own.n;
                break;
            }
        }
        /* i += len(value.Raw) - 1, then the loop's i++ */
        *cursor = i + vl;
        return 1;
    }
    *cursor = n;
    return 0;
}
