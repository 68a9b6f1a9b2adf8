/*
 * gjson_mods_ref.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restates the reference's custom gjson modifiers (pkg/json/json.go:161-264: extractJSONStr
 * :161-185, replaceJSONStr :187-206, caseJSONStr :208-216, base64JSONStr :218-238,
 * stripJSONstr :240-249, wrap/escapeQuotes :251-257, registration :258-264) and the parts
 * of gjson v1.14.0 that run them: execModifier (name, JSON argument by squash or plain
 * argument up to '|'), the pipe into the modifier after a found value, Result.ForEach of
 * the argument, and Parse of each output; plus Go's encoding/base64 Std / RawStd decoding
 * (partial output on a CorruptInputError) and strings.Split / ReplaceAll.
 * ToUpper / ToLower and unicode.IsPrint are restated for ASCII text; a non-ASCII text
 * there is reported undecided, as the device does. gjson's own @fromstr (modFromStr:
 * Parse(json).String() when Valid(json), else "") and a path after a modifier (Get:
 * execModifier, then Get(rjson, path[1:])) are restated too, with gjson's recursive
 * validator (validpayload, validany, validobject, validarray, validstring, validnumber).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static int is_ws(char c) { return (unsigned char)c <= ' '; }

/* gjson squash of a JSON value starting at s[i]: end offset, or 0 when unbalanced */
static size_t squash_end(const char* s, size_t n, size_t i) {
    if (s[i] == '"') {
        for (size_t k = i + 1; k < n; k++) {
            if (s[k] == '\\') { k++; continue; }
            if (s[k] == '"') return k + 1;
        }
        return 0;
    }
    int depth = 0;
    for (size_t k = i; k < n; k++) {
        char c = s[k];
        if (c == '"') {
            k++;
            while (k < n && s[k] != '"') { if (s[k] == '\\') k++; k++; }
            if (k >= n) return 0;
            continue;
        }
        if (c == '{' || c == '[' || c == '(') depth++;
        else if (c == '}' || c == ']' || c == ')') { if (--depth == 0) return k + 1; }
    }
    return 0;
}

/* a JSON string literal at s[*i]: its unescaped text in out (gjson Result.String of it) */
static int arg_string(const char* s, size_t n, size_t* i, or_buf* out) {
    size_t k = *i + 1, start = k;
    int esc = 0;
    for (; k < n; k++) {
        if (s[k] == '\\') { esc = 1; k++; continue; }
        if (s[k] == '"') break;
    }
    if (k >= n) return 0;
    or_buf_reset(out);
    if (esc) or_unescape(s + start, k - start, out);
    else or_buf_push(out, s + start, k - start);
    *i = k + 1;
    return 1;
}

/* ForEach over an object argument: sep / pos (extract), old / new (replace); the last
 * occurrence of a key wins. Returns 0 when the argument has another shape than the one
 * restated (non-string sep/old/new, a pos that is not a non-negative number). */
static int parse_arg_object(const char* a, size_t n, int want_extract, or_mod* m) {
    size_t i = 0;
    or_buf key, val;
    memset(&key, 0, sizeof key);
    memset(&val, 0, sizeof val);
    int ok = 0;
    while (i < n && is_ws(a[i])) i++;
    if (i >= n || a[i] != '{') goto out;
    i++;
    for (;;) {
        while (i < n && is_ws(a[i])) i++;
        if (i < n && a[i] == '}') { ok = 1; break; }
        if (i >= n || a[i] != '"' || !arg_string(a, n, &i, &key)) break;
        while (i < n && is_ws(a[i])) i++;
        if (i >= n || a[i] != ':') break;
        i++;
        while (i < n && is_ws(a[i])) i++;
        if (i >= n) break;
        int is_str = a[i] == '"';
        size_t vs = i;
        if (is_str) {
            if (!arg_string(a, n, &i, &val)) break;
        } else if (a[i] == '{' || a[i] == '[') {
            size_t e = squash_end(a, n, i);
            if (!e) break;
            i = e;
        } else {
            while (i < n && a[i] != ',' && a[i] != '}' && !is_ws(a[i])) i++;
        }
        const char* kp = key.p ? key.p : "";
        if (want_extract && key.n == 3 && !memcmp(kp, "sep", 3)) {
            if (!is_str) goto out;
            free(m->a);
            m->a = (char*)malloc(val.n + 1);
            memcpy(m->a, val.p ? val.p : "", val.n);
            m->a_len = val.n;
        } else if (want_extract && key.n == 3 && !memcmp(kp, "pos", 3)) {
            if (is_str) goto out;
            char tmp[64];
            size_t L = i - vs < 63 ? i - vs : 63;
            memcpy(tmp, a + vs, L);
            tmp[L] = 0;
            char* endp;
            double v = strtod(tmp, &endp);
            if (*endp || !(v >= 0) || v > 9007199254740991.0) goto out;
            m->pos = (uint64_t)trunc(v);
        } else if (!want_extract && key.n == 3 && !memcmp(kp, "old", 3)) {
            if (!is_str) goto out;
            free(m->a);
            m->a = (char*)malloc(val.n + 1);
            memcpy(m->a, val.p ? val.p : "", val.n);
            m->a_len = val.n;
            m->has_old = 1;
        } else if (!want_extract && key.n == 3 && !memcmp(kp, "new", 3)) {
            if (!is_str) goto out;
            free(m->b);
            m->b = (char*)malloc(val.n + 1);
            memcpy(m->b, val.p ? val.p : "", val.n);
            m->b_len = val.n;
        }
        while (i < n && is_ws(a[i])) i++;
        if (i < n && a[i] == ',') { i++; continue; }
        if (i < n && a[i] == '}') { ok = 1; break; }
        break;
    }
out:
    or_buf_free(&key);
    or_buf_free(&val);
    return ok;
}

void or_mods_free(or_mod* mods, int n) {
    for (int k = 0; k < n; k++) {
        free(mods[k].a);
        free(mods[k].b);
        mods[k].a = mods[k].b = NULL;
    }
}

int or_mod_split(const char* p, size_t n, size_t* base_len, or_mod* mods, int max_mods, int* n_mods) {
    *n_mods = 0;
    size_t cut = 0;
    int found = 0;
    for (size_t i = 0; i + 1 < n; i++) {
        if (p[i] == '\\') { i++; continue; }
        if (p[i] == '|' || (p[i] == '.' && p[i + 1] == '@')) { cut = i; found = 1; break; }
    }
    if (!found || cut == 0) return 0;
    *base_len = cut;
    size_t i = cut + 1;
    while (i < n) {
        if (*n_mods >= max_mods) return -1;
        if (p[i] != '@') {  /* a path after a modifier, up to the next '|@' / '.@' */
            size_t e = i;
            while (e < n) {
                if (p[e] == '\\') { e += 2; continue; }
                if (p[e] == '|' || (p[e] == '.' && e + 1 < n && p[e + 1] == '@')) break;
                e++;
            }
            if (e > n) e = n;
            or_mod* m = &mods[*n_mods];
            memset(m, 0, sizeof *m);
            (*n_mods)++;
            m->kind = OR_MOD_PATH;
            m->a = (char*)malloc(e - i + 1);
            memcpy(m->a, p + i, e - i);
            m->a_len = e - i;
            if (e >= n) break;
            i = e + 1;
            continue;
        }
        size_t k = i + 1;
        while (k < n && p[k] != ':' && p[k] != '|' && p[k] != '.') k++;
        const char* name = p + i + 1;
        size_t name_len = k - i - 1;
        const char* arg = "";
        size_t arg_len = 0, next = k;
        int has_args = 0;
        if (k < n && p[k] == ':') {
            size_t a = k + 1;
            has_args = a < n;
            if (has_args && (p[a] == '{' || p[a] == '[' || p[a] == '"')) {
                size_t e = squash_end(p, n, a);
                if (!e) return -1;
                arg = p + a;
                arg_len = e - a;
                next = e;
            } else {
                size_t e = a;
                while (e < n && p[e] != '|') e++;
                arg = p + a;
                arg_len = e - a;
                next = e;
            }
        }
        or_mod* m = &mods[*n_mods];
        memset(m, 0, sizeof *m);
        (*n_mods)++;
#define NAME_IS(s) (name_len == strlen(s) && !memcmp(name, s, name_len))
#define ARG_IS(s) (arg_len == strlen(s) && !memcmp(arg, s, arg_len))
        if (NAME_IS("extract")) {
            m->kind = OR_MOD_EXTRACT;
            m->a = (char*)malloc(2);
            m->a[0] = ' ';
            m->a_len = 1;
            if (has_args && arg_len && arg[0] == '{') {
                if (!parse_arg_object(arg, arg_len, 1, m)) return -1;
            } else if (has_args && arg_len && (arg[0] == '[' || arg[0] == '"')) {
                return -1;
            }
            if (m->a_len == 0) return -1;
        } else if (NAME_IS("replace")) {
            m->kind = OR_MOD_REPLACE;
            if (has_args && arg_len) {
                if (arg[0] != '{' || !parse_arg_object(arg, arg_len, 0, m)) return -1;
                if (!m->has_old || m->a_len == 0) return -1;
                m->variant = 1;
            }
        } else if (NAME_IS("case")) {
            m->kind = OR_MOD_CASE;
            m->variant = ARG_IS("upper") ? 1 : ARG_IS("lower") ? 2 : 0;
        } else if (NAME_IS("base64")) {
            m->kind = OR_MOD_BASE64;
            m->variant = ARG_IS("encode") ? 1 : ARG_IS("decode") ? 2 : 0;
        } else if (NAME_IS("strip")) {
            m->kind = OR_MOD_STRIP;
        } else if (NAME_IS("fromstr")) {
            m->kind = OR_MOD_FROMSTR;
        } else {
            return -1;
        }
#undef NAME_IS
#undef ARG_IS
        if (next >= n) break;
        if (p[next] != '|' && p[next] != '.') return -1;
        i = next + 1;
        if (i >= n) return -1;
    }
    return *n_mods ? 1 : -1;
}

/* gjson.Parse(text): result fields point into text / r->own */
int or_parse(const char* s, size_t n, or_result* r) {
    or_buf_reset(&r->own);
    r->type = OR_NULL;
    r->raw = s;
    r->raw_len = 0;
    r->str = NULL;
    r->str_len = 0;
    r->num = 0;
    size_t i = 0;
    while (i < n && is_ws(s[i])) i++;
    if (i >= n) return 0;
    char c = s[i];
    if (c == '{' || c == '[') {
        r->type = OR_JSON;
        r->raw = s + i;
        r->raw_len = n - i;
        return 0;
    }
    if (c == '"') {
        /* tostr */
        size_t k = i + 1, close = n;
        int esc = 0, term = 0;
        for (; k < n; k++) {
            if ((unsigned char)s[k] > '\\') continue;
            if (s[k] == '"') { close = k; term = 1; break; }
            if (s[k] == '\\') {
                esc = 1;
                for (; k < n; k++) {
                    if ((unsigned char)s[k] > '\\') continue;
                    if (s[k] == '"') {
                        if (s[k - 1] == '\\') {
                            size_t nb = 0;
                            for (size_t q = k - 2; q > i && q < k; q--) {
                                if (s[q] != '\\') break;
                                nb++;
                            }
                            if (nb % 2 == 0) continue;
                        }
                        close = k;
                        term = 1;
                        break;
                    }
                }
                break;
            }
        }
        r->type = OR_STRING;
        r->raw = s + i;
        r->raw_len = (term ? close + 1 : n) - i;
        if (esc) {
            or_unescape(s + i + 1, close - i - 1, &r->own);
            r->str = r->own.p ? r->own.p : "";
            r->str_len = r->own.n;
        } else {
            r->str = s + i + 1;
            r->str_len = close - i - 1;
        }
        return 0;
    }
    if (c == '-' || (c >= '0' && c <= '9')) {
        size_t k = i + 1;
        for (; k < n; k++) {
            unsigned char d = (unsigned char)s[k];
            if (d <= '-') { if (d <= ' ' || d == ',') break; }
            else if (d == ']' || d == '}') break;
        }
        r->type = OR_NUMBER;
        r->raw = s + i;
        r->raw_len = k - i;
        or_go_parse_float(r->raw, r->raw_len, &r->num);
        return 0;
    }
    if (c == 't' || c == 'f' || (c == 'n' && (i + 1 >= n || s[i + 1] == 'u'))) {
        size_t k = i + 1;
        while (k < n && s[k] >= 'a' && s[k] <= 'z') k++;
        r->type = c == 't' ? OR_TRUE : c == 'f' ? OR_FALSE : OR_NULL;
        r->raw = s + i;
        r->raw_len = k - i;
        return 0;
    }
    return -1; /* '+' 'i' 'I' 'N', NaN-like 'n...': not restated */
}

/* gjson.Parse(text).String() appended to out; -1 undecided */
static int parse_string_of(const char* s, size_t n, or_buf* out) {
    or_result r;
    memset(&r, 0, sizeof r);
    int rc = or_parse(s, n, &r);
    if (rc == 0) or_result_string(&r, out);
    or_result_free(&r);
    return rc;
}

static int b64v(unsigned char c) {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    return -1;
}

/* encoding/base64 (Encoding).Decode, not strict: decodeQuantum by decodeQuantum; bytes of
 * complete quanta before an error are kept. padded: StdEncoding, else RawStdEncoding.
 * Returns 1 when err == nil. */
static int go_b64_decode(const unsigned char* src, size_t n, int padded, or_buf* out) {
    size_t si = 0;
    for (;;) {
        int dbuf[4] = {0, 0, 0, 0};
        int dlen = 4, j;
        int err = 0, fin = 0;
        for (j = 0; j < 4; j++) {
            if (si == n) {
                if (j == 0) return 1;
                if (j == 1 || padded) return 0;
                dlen = j;
                fin = 1;
                break;
            }
            unsigned char in = src[si++];
            int v = b64v(in);
            if (v >= 0) { dbuf[j] = v; continue; }
            if (in == '\n' || in == '\r') { j--; continue; }
            if (!padded || in != '=') return 0;
            if (j == 0 || j == 1) return 0;
            if (j == 2) {
                while (si < n && (src[si] == '\n' || src[si] == '\r')) si++;
                if (si == n) return 0;
                if (src[si] != '=') return 0;
                si++;
            }
            while (si < n && (src[si] == '\n' || src[si] == '\r')) si++;
            if (si < n) err = 1;
            dlen = j;
            fin = 1;
            break;
        }
        unsigned val = (unsigned)dbuf[0] << 18 | (unsigned)dbuf[1] << 12 | (unsigned)dbuf[2] << 6 | (unsigned)dbuf[3];
        char b3[3] = {(char)(val >> 16), (char)(val >> 8), (char)val};
        or_buf_push(out, b3, (size_t)(dlen - 1));
        if (err) return 0;
        if (fin) return 1;
    }
}

static void go_b64_encode(const unsigned char* s, size_t n, or_buf* out) {
    static const char al[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    size_t i = 0;
    char q[4];
    for (; i + 3 <= n; i += 3) {
        unsigned v = (unsigned)s[i] << 16 | (unsigned)s[i + 1] << 8 | s[i + 2];
        q[0] = al[v >> 18 & 63]; q[1] = al[v >> 12 & 63]; q[2] = al[v >> 6 & 63]; q[3] = al[v & 63];
        or_buf_push(out, q, 4);
    }
    if (n - i == 1) {
        unsigned v = (unsigned)s[i] << 16;
        q[0] = al[v >> 18 & 63]; q[1] = al[v >> 12 & 63]; q[2] = '='; q[3] = '=';
        or_buf_push(out, q, 4);
    } else if (n - i == 2) {
        unsigned v = (unsigned)s[i] << 16 | (unsigned)s[i + 1] << 8;
        q[0] = al[v >> 18 & 63]; q[1] = al[v >> 12 & 63]; q[2] = al[v >> 6 & 63]; q[3] = '=';
        or_buf_push(out, q, 4);
    }
}

/* gjson v1.14.0 validator, recursive as gjson's: each returns the index after the value
 * and sets *ok */
static size_t v_any(const char* s, size_t n, size_t i, int* ok);
static int v_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
static size_t v_string(const char* s, size_t n, size_t i, int* ok) { /* i after the quote */
    for (; i < n; i++) {
        unsigned char c = (unsigned char)s[i];
        if (c < ' ') { *ok = 0; return i; }
        if (c == '\\') {
            if (++i == n) { *ok = 0; return i; }
            switch (s[i]) {
                case '"': case '\\': case '/': case 'b': case 'f': case 'n': case 'r': case 't': break;
                case 'u':
                    for (int j = 0; j < 4; j++) {
                        i++;
                        if (i >= n || !((s[i] >= '0' && s[i] <= '9') || (s[i] >= 'a' && s[i] <= 'f') ||
                                        (s[i] >= 'A' && s[i] <= 'F'))) { *ok = 0; return i; }
                    }
                    break;
                default: *ok = 0; return i;
            }
        } else if (c == '"') {
            *ok = 1;
            return i + 1;
        }
    }
    *ok = 0;
    return i;
}
static size_t v_number(const char* s, size_t n, size_t i, int* ok) { /* i after the first char */
    i--;
#define DIG(k) ((k) < n && s[k] >= '0' && s[k] <= '9')
    *ok = 0;
    if (s[i] == '-') { i++; if (!DIG(i)) return i; }
    if (s[i] == '0') i++;
    else while (DIG(i)) i++;
    if (i < n && s[i] == '.') { i++; if (!DIG(i)) return i; while (DIG(i)) i++; }
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
        i++;
        if (i < n && (s[i] == '+' || s[i] == '-')) i++;
        if (!DIG(i)) return i;
        while (DIG(i)) i++;
    }
#undef DIG
    *ok = 1;
    return i;
}
static size_t v_comma(const char* s, size_t n, size_t i, char end, int* ok) {
    for (; i < n; i++) {
        if (v_ws(s[i])) continue;
        *ok = s[i] == ',' || s[i] == end;
        return i;
    }
    *ok = 0;
    return i;
}
static size_t v_array(const char* s, size_t n, size_t i, int* ok) { /* after '[' */
    for (; i < n; i++) {
        if (v_ws(s[i])) continue;
        if (s[i] == ']') { *ok = 1; return i + 1; }
        for (;;) {
            i = v_any(s, n, i, ok);
            if (!*ok) return i;
            i = v_comma(s, n, i, ']', ok);
            if (!*ok) return i;
            if (s[i] == ']') return i + 1;
            i++;
        }
    }
    *ok = 0;
    return i;
}
static size_t v_object(const char* s, size_t n, size_t i, int* ok) { /* after '{' */
    for (; i < n; i++) {
        if (v_ws(s[i])) continue;
        if (s[i] == '}') { *ok = 1; return i + 1; }
        if (s[i] != '"') { *ok = 0; return i; }
        for (;;) {  /* at a key's quote */
            i = v_string(s, n, i + 1, ok);
            if (!*ok) return i;
            while (i < n && v_ws(s[i])) i++;
            if (i >= n || s[i] != ':') { *ok = 0; return i; }
            i = v_any(s, n, i + 1, ok);
            if (!*ok) return i;
            i = v_comma(s, n, i, '}', ok);
            if (!*ok) return i;
            if (s[i] == '}') return i + 1;
            i++;
            while (i < n && v_ws(s[i])) i++;
            if (i >= n || s[i] != '"') { *ok = 0; return i; }
        }
    }
    *ok = 0;
    return i;
}
static size_t v_word(const char* s, size_t n, size_t i, const char* rest, int* ok) {
    size_t L = strlen(rest);
    *ok = i + L <= n && !memcmp(s + i, rest, L);
    return *ok ? i + L : i;
}
static size_t v_any(const char* s, size_t n, size_t i, int* ok) {
    for (; i < n; i++) {
        switch (s[i]) {
            case ' ': case '\t': case '\n': case '\r': continue;
            case '{': return v_object(s, n, i + 1, ok);
            case '[': return v_array(s, n, i + 1, ok);
            case '"': return v_string(s, n, i + 1, ok);
            case '-': case '0': case '1': case '2': case '3': case '4': case '5': case '6': case '7': case '8':
            case '9': return v_number(s, n, i + 1, ok);
            case 't': return v_word(s, n, i + 1, "rue", ok);
            case 'f': return v_word(s, n, i + 1, "alse", ok);
            case 'n': return v_word(s, n, i + 1, "ull", ok);
            default: *ok = 0; return i;
        }
    }
    *ok = 0;
    return i;
}
int or_valid(const char* s, size_t n) {
    int ok = 0;
    size_t i = v_any(s, n, 0, &ok);
    if (!ok) return 0;
    for (; i < n; i++)
        if (!v_ws(s[i])) return 0;
    return 1;
}

static void wrap_into(const char* s, size_t n, or_buf* out) {
    or_buf_push(out, "\"", 1);
    or_buf_push(out, s, n);
    or_buf_push(out, "\"", 1);
}

int or_mod_apply(const or_mod* mods, int n_mods, const char* raw, size_t raw_len, or_buf* text) {
    or_buf cur, nxt, tmp;
    memset(&cur, 0, sizeof cur);
    memset(&nxt, 0, sizeof nxt);
    memset(&tmp, 0, sizeof tmp);
    or_buf_push(&cur, raw, raw_len);
    int rc = 0;
    for (int k = 0; k < n_mods && rc == 0; k++) {
        const or_mod* m = &mods[k];
        const char* in = cur.p ? cur.p : "";
        size_t in_n = cur.n;
        or_buf_reset(&nxt);
        or_buf_reset(&tmp);
        switch (m->kind) {
            case OR_MOD_EXTRACT: {
                if (parse_string_of(in, in_n, &tmp) != 0) { rc = -1; break; }
                const char* t = tmp.p ? tmp.p : "";
                uint64_t part = 0;
                size_t ps = 0, i = 0;
                int done = 0;
                for (;;) {
                    const char* hit = NULL;
                    for (size_t e = i; e + m->a_len <= tmp.n; e++)
                        if (!memcmp(t + e, m->a, m->a_len)) { hit = t + e; break; }
                    size_t e = hit ? (size_t)(hit - t) : tmp.n;
                    if (part == m->pos) { wrap_into(t + ps, e - ps, &nxt); done = 1; break; }
                    if (!hit) break;
                    part++;
                    i = e + m->a_len;
                    ps = i;
                }
                if (!done) or_buf_push(&nxt, "n", 1);
                break;
            }
            case OR_MOD_REPLACE: {
                if (!m->variant) { or_buf_push(&nxt, in, in_n); break; }
                if (parse_string_of(in, in_n, &tmp) != 0) { rc = -1; break; }
                const char* t = tmp.p ? tmp.p : "";
                or_buf_push(&nxt, "\"", 1);
                for (size_t i = 0; i < tmp.n;) {
                    if (i + m->a_len <= tmp.n && !memcmp(t + i, m->a, m->a_len)) {
                        or_buf_push(&nxt, m->b ? m->b : "", m->b_len);
                        i += m->a_len;
                    } else {
                        or_buf_push(&nxt, t + i, 1);
                        i++;
                    }
                }
                or_buf_push(&nxt, "\"", 1);
                break;
            }
            case OR_MOD_CASE: {
                for (size_t i = 0; i < in_n; i++) {
                    char c = in[i];
                    if ((unsigned char)c >= 0x80 && m->variant) { rc = -1; break; }
                    if (m->variant == 1 && c >= 'a' && c <= 'z') c = (char)(c - 'a' + 'A');
                    if (m->variant == 2 && c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
                    or_buf_push(&nxt, &c, 1);
                }
                break;
            }
            case OR_MOD_BASE64: {
                if (!m->variant) { or_buf_push(&nxt, in, in_n); break; }
                if (parse_string_of(in, in_n, &tmp) != 0) { rc = -1; break; }
                const unsigned char* t = (const unsigned char*)(tmp.p ? tmp.p : "");
                if (m->variant == 1) {
                    or_buf enc;
                    memset(&enc, 0, sizeof enc);
                    go_b64_encode(t, tmp.n, &enc);
                    wrap_into(enc.p ? enc.p : "", enc.n, &nxt);
                    or_buf_free(&enc);
                    break;
                }
                or_buf dec;
                memset(&dec, 0, sizeof dec);
                int ok = 0;
                if (tmp.n % 4 == 0) ok = go_b64_decode(t, tmp.n, 1, &dec);
                if (!ok) {
                    or_buf_reset(&dec);
                    go_b64_decode(t, tmp.n, 0, &dec);
                }
                /* wrap(escapeQuotes(decoded)) */
                or_buf_push(&nxt, "\"", 1);
                for (size_t i = 0; i < dec.n; i++) {
                    if (dec.p[i] == '"') or_buf_push(&nxt, "\\", 1);
                    or_buf_push(&nxt, dec.p + i, 1);
                }
                or_buf_push(&nxt, "\"", 1);
                or_buf_free(&dec);
                break;
            }
            case OR_MOD_STRIP: {
                for (size_t i = 0; i < in_n; i++) {
                    unsigned char c = (unsigned char)in[i];
                    if (c >= 0x80) { rc = -1; break; }
                    if (c >= 0x20 && c != 0x7F) or_buf_push(&nxt, (const char*)&c, 1);
                }
                break;
            }
            case OR_MOD_FROMSTR: {
                if (!or_valid(in, in_n)) break; /* "" */
                if (parse_string_of(in, in_n, &nxt) != 0) rc = -1;
                break;
            }
            case OR_MOD_PATH: {
                or_result r;
                memset(&r, 0, sizeof r);
                if (or_gjson_get(in, in_n, m->a, m->a_len, &r) != 0) { rc = -1; or_result_free(&r); break; }
                if (r.raw_len == 0) { /* not found: the Result is Null, the chain ends */
                    or_result_free(&r);
                    or_buf_reset(&cur);
                    k = n_mods;
                    goto done;
                }
                or_buf_push(&nxt, r.raw, r.raw_len);
                or_result_free(&r);
                break;
            }
            default: rc = -1;
        }
        or_buf t = cur;
        cur = nxt;
        nxt = t;
    }
done:
    if (rc == 0) {
        or_buf_reset(text);
        or_buf_push(text, cur.p ? cur.p : "", cur.n);
    }
    or_buf_free(&cur);
    or_buf_free(&nxt);
    or_buf_free(&tmp);
    return rc;
}

int or_gjson_get_mods(const char* json, size_t jlen, const char* path, size_t plen, or_result* r, or_buf* text) {
    or_mod mods[8];
    int nm = 0;
    size_t base = plen;
    int mr = or_mod_split(path, plen, &base, mods, 8, &nm);
    if (mr < 0) {
        or_mods_free(mods, nm);
        return -1;
    }
    if (mr == 0) return or_gjson_get(json, jlen, path, plen, r);
    int rc = or_gjson_get(json, jlen, path, base, r);
    if (rc == 0 && r->raw_len > 0) {
        if (or_mod_apply(mods, nm, r->raw, r->raw_len, text) != 0 || or_parse(text->p ? text->p : "", text->n, r) != 0)
            rc = -2;
    }
    or_mods_free(mods, nm);
    return rc;
}
