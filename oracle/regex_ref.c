/*
 * regex_ref.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restatement of Go 1.21 regexp.Compile / (*Regexp).MatchString as used by the
 * reference's `matches` operator (pkg/jsonexp/expressions.go:87-91). Go's regexp is
 * stdlib and absent from the reference tree; this follows its published behaviour:
 *   - regexp/syntax Parse with the Perl flag set (ClassNL|OneLine|PerlX|UnicodeGroups):
 *     the operator-stack parser, its error rules (missing/unexpected paren, missing
 *     repeat argument, nested repetition `**`, repeat bounds > 1000 and the nested
 *     repeat product limit, class / escape / flag-group errors), (?flags) scoping,
 *     (?P<name>..) (Go 1.21 has no (?<name>..)), \Q..\E, octal / \x escapes, Perl
 *     classes \d\s\w (ASCII), POSIX [[:name:]] classes, ClassNL negated classes.
 *   - MatchString = unanchored boolean search over the UTF-8-decoded runes of the
 *     subject (invalid bytes decode to U+FFFD, width 1), with empty-width assertions
 *     evaluated from (previous rune, next rune) exactly like syntax.EmptyOpContext.
 * The matcher is a Pike-VM (Thompson NFA simulation) — independent of the product's
 * DFA construction. \p{..} Unicode groups and (?i) folding of non-ASCII runes are not
 * restated: such patterns report *unsupported instead of a result.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define MAX_RUNE 0x10FFFF

/* ---------- rune ranges ---------- */
typedef struct {
    unsigned lo, hi;
} rr;
typedef struct {
    rr* r;
    int n, cap;
} rclass;

static void rc_add(rclass* c, unsigned lo, unsigned hi) {
    if (c->n == c->cap) {
        c->cap = c->cap ? c->cap * 2 : 8;
        c->r = (rr*)realloc(c->r, (size_t)c->cap * sizeof(rr));
    }
    c->r[c->n].lo = lo;
    c->r[c->n].hi = hi;
    c->n++;
}
static int rr_cmp(const void* a, const void* b) {
    const rr* x = (const rr*)a;
    const rr* y = (const rr*)b;
    if (x->lo != y->lo) return x->lo < y->lo ? -1 : 1;
    return x->hi < y->hi ? -1 : x->hi > y->hi;
}
static void rc_clean(rclass* c) {
    if (c->n == 0) return;
    qsort(c->r, (size_t)c->n, sizeof(rr), rr_cmp);
    int w = 0;
    for (int i = 1; i < c->n; i++) {
        if (c->r[i].lo <= c->r[w].hi + 1) {
            if (c->r[i].hi > c->r[w].hi) c->r[w].hi = c->r[i].hi;
        } else {
            c->r[++w] = c->r[i];
        }
    }
    c->n = w + 1;
}
static void rc_negate(rclass* c) {
    rc_clean(c);
    rclass o = {0};
    unsigned next = 0;
    for (int i = 0; i < c->n; i++) {
        if (c->r[i].lo > next) rc_add(&o, next, c->r[i].lo - 1);
        next = c->r[i].hi + 1;
    }
    if (next <= MAX_RUNE) rc_add(&o, next, MAX_RUNE);
    free(c->r);
    *c = o;
}
static int rc_has(const rclass* c, unsigned r) {
    for (int i = 0; i < c->n; i++)
        if (r >= c->r[i].lo && r <= c->r[i].hi) return 1;
    return 0;
}

/* ---------- AST ---------- */
enum {
    N_CLASS,   /* literal runes or class */
    N_EMPTY,   /* empty match */
    N_ASSERT,  /* empty-width */
    N_STAR, N_PLUS, N_QUEST, N_REPEAT,
    N_CONCAT, N_ALT, N_CAP,
    P_LPAREN, P_VBAR /* pseudo ops */
};
/* assertion bits (syntax.EmptyOp) */
enum { E_BOL = 1, E_EOL = 2, E_BOT = 4, E_EOT = 8, E_WB = 16, E_NWB = 32 };
/* parser flags */
enum { F_FOLD = 1, F_DOTNL = 2, F_ONELINE = 4, F_NONGREEDY = 8 };

typedef struct node {
    int op;
    int flags;
    rclass cls;
    int assert_bits;
    struct node** sub;
    int nsub;
    int min, max;
    int cap;
} node;

typedef struct {
    node** st;
    int n, cap;
    int flags;
    int ncap;
    int unsupported;
    char* err;
    size_t errcap;
    int failed;
    const char* whole;
    size_t wlen;
    node** all; /* every node allocated, for freeing */
    int nall, capall;
} parser;

static node* new_node(parser* p, int op) {
    node* n = (node*)calloc(1, sizeof(node));
    n->op = op;
    n->flags = p->flags;
    if (p->nall == p->capall) {
        p->capall = p->capall ? p->capall * 2 : 32;
        p->all = (node**)realloc(p->all, (size_t)p->capall * sizeof(node*));
    }
    p->all[p->nall++] = n;
    return n;
}
static void push(parser* p, node* n) {
    if (p->n == p->cap) {
        p->cap = p->cap ? p->cap * 2 : 16;
        p->st = (node**)realloc(p->st, (size_t)p->cap * sizeof(node*));
    }
    p->st[p->n++] = n;
}
static void add_sub(node* n, node* s) {
    n->sub = (node**)realloc(n->sub, (size_t)(n->nsub + 1) * sizeof(node*));
    n->sub[n->nsub++] = s;
}

static int fail(parser* p, const char* code, const char* expr, size_t elen) {
    if (!p->failed) {
        p->failed = 1;
        snprintf(p->err, p->errcap, "error parsing regexp: %s: `%.*s`", code, (int)elen, expr);
    }
    return -1;
}

/* ---------- UTF-8 (Go utf8.DecodeRune) ---------- */
static int decode_rune(const unsigned char* s, size_t n, unsigned* r) {
    if (n == 0) { *r = 0xFFFD; return 0; }
    unsigned b0 = s[0];
    if (b0 < 0x80) { *r = b0; return 1; }
    int sz;
    unsigned lo = 0x80, hi = 0xBF, v;
    if (b0 >= 0xC2 && b0 <= 0xDF) { sz = 2; v = b0 & 0x1F; }
    else if (b0 >= 0xE0 && b0 <= 0xEF) {
        sz = 3; v = b0 & 0x0F;
        if (b0 == 0xE0) lo = 0xA0;
        if (b0 == 0xED) hi = 0x9F;
    } else if (b0 >= 0xF0 && b0 <= 0xF4) {
        sz = 4; v = b0 & 0x07;
        if (b0 == 0xF0) lo = 0x90;
        if (b0 == 0xF4) hi = 0x8F;
    } else { *r = 0xFFFD; return 1; }
    if (n < (size_t)sz) { *r = 0xFFFD; return 1; }
    if (s[1] < lo || s[1] > hi) { *r = 0xFFFD; return 1; }
    v = (v << 6) | (s[1] & 0x3F);
    for (int i = 2; i < sz; i++) {
        if (s[i] < 0x80 || s[i] > 0xBF) { *r = 0xFFFD; return 1; }
        v = (v << 6) | (s[i] & 0x3F);
    }
    *r = v;
    return sz;
}

/* nextRune: error on invalid UTF-8 in the pattern */
static int next_rune(parser* p, const char* t, size_t n, unsigned* r) {
    if (n == 0) { *r = 0xFFFD; return 0; }
    int k = decode_rune((const unsigned char*)t, n, r);
    if (*r == 0xFFFD && k == 1) { /* utf8.RuneError with size 1 = invalid byte */
        fail(p, "invalid UTF-8", t, n);
        return -1;
    }
    return k;
}

/* ---------- case folding (ASCII orbits only) ---------- */
static void fold_add(parser* p, rclass* c, unsigned lo, unsigned hi) {
    /* appendFoldedRange: full-coverage shortcut, else fold each rune's orbit */
    if (lo <= 0x41 && hi >= 0x1E943) { rc_add(c, lo, hi); return; }
    rc_add(c, lo, hi);
    for (unsigned r = lo; r <= hi && r < 0x80; r++) {
        if (r >= 'a' && r <= 'z') rc_add(c, r - 32, r - 32);
        if (r >= 'A' && r <= 'Z') rc_add(c, r + 32, r + 32);
        if (r == 'k' || r == 'K') rc_add(c, 0x212A, 0x212A);
        if (r == 's' || r == 'S') rc_add(c, 0x17F, 0x17F);
    }
    if (hi >= 0x80) {
        /* non-ASCII runes with case orbits: not restated by this oracle */
        unsigned a = lo < 0x80 ? 0x80 : lo;
        if (a <= hi && a <= 0x1E943) p->unsupported = 1;
    }
}

static void class_add(parser* p, rclass* c, unsigned lo, unsigned hi) {
    if (p->flags & F_FOLD) fold_add(p, c, lo, hi);
    else rc_add(c, lo, hi);
}

static void literal(parser* p, unsigned r) {
    node* n = new_node(p, N_CLASS);
    class_add(p, &n->cls, r, r);
    push(p, n);
}

/* Perl / POSIX groups (ASCII). sign = +1 or -1 */
typedef struct {
    const char* name;
    const char* ranges; /* pairs */
} group;
static const group perl_groups[] = {
    {"\\d", "09"}, {"\\s", "\t\n\f\r  "}, {"\\w", "09AZ__az"},
};
static const group posix_groups[] = {
    {"[:alnum:]", "09AZaz"}, {"[:alpha:]", "AZaz"}, {"[:ascii:]", "\x01\x7f"},
    {"[:blank:]", "\t\t  "}, {"[:cntrl:]", "\x01\x1f\x7f\x7f"}, {"[:digit:]", "09"},
    {"[:graph:]", "!~"}, {"[:lower:]", "az"}, {"[:print:]", " ~"},
    {"[:punct:]", "!/:@[`{~"}, {"[:space:]", "\t\r  "}, {"[:upper:]", "AZ"},
    {"[:word:]", "09AZ__az"}, {"[:xdigit:]", "09AFaf"},
};

static void add_group(parser* p, rclass* c, const char* ranges, int sign, int ascii_has_nul) {
    rclass g = {0};
    size_t L = strlen(ranges);
    if (ascii_has_nul) rc_add(&g, 0, 0);
    for (size_t i = 0; i + 1 < L; i += 2) {
        unsigned lo = (unsigned char)ranges[i], hi = (unsigned char)ranges[i + 1];
        if (p->flags & F_FOLD) fold_add(p, &g, lo, hi);
        else rc_add(&g, lo, hi);
    }
    if (sign < 0) rc_negate(&g);
    for (int i = 0; i < g.n; i++) rc_add(c, g.r[i].lo, g.r[i].hi);
    free(g.r);
}

/* \d \D \s \S \w \W ; returns consumed bytes or 0 */
static size_t perl_class(parser* p, const char* t, size_t n, rclass* c) {
    if (n < 2 || t[0] != '\\') return 0;
    char k = t[1];
    int sign = 1;
    char lk = k;
    if (k == 'D' || k == 'S' || k == 'W') { sign = -1; lk = (char)(k + 32); }
    const char* rg = NULL;
    if (lk == 'd') rg = perl_groups[0].ranges;
    else if (lk == 's') rg = perl_groups[1].ranges;
    else if (lk == 'w') rg = perl_groups[2].ranges;
    if (!rg) return 0;
    add_group(p, c, rg, sign, 0);
    return 2;
}

/* [:name:] inside a class. returns consumed, 0 if not a named class, -1 error */
static long named_class(parser* p, const char* t, size_t n, rclass* c) {
    if (n < 2 || t[0] != '[' || t[1] != ':') return 0;
    const char* e = NULL;
    for (size_t i = 2; i + 1 < n; i++)
        if (t[i] == ':' && t[i + 1] == ']') { e = t + i; break; }
    if (!e) return 0;
    size_t nl = (size_t)(e - t) + 2;
    int sign = 1;
    char name[32];
    if (nl >= sizeof name) return fail(p, "invalid character class range", t, nl);
    memcpy(name, t, nl);
    name[nl] = 0;
    if (name[2] == '^') {
        sign = -1;
        memmove(name + 2, name + 3, nl - 2);
    }
    for (size_t i = 0; i < sizeof posix_groups / sizeof posix_groups[0]; i++) {
        if (strcmp(posix_groups[i].name, name) == 0) {
            int nul = strcmp(name, "[:ascii:]") == 0 || strcmp(name, "[:cntrl:]") == 0;
            add_group(p, c, posix_groups[i].ranges, sign, nul);
            return (long)nl;
        }
    }
    return fail(p, "invalid character class range", t, nl);
}

static int unhex(unsigned c) {
    if (c >= '0' && c <= '9') return (int)(c - '0');
    if (c >= 'a' && c <= 'f') return (int)(c - 'a' + 10);
    if (c >= 'A' && c <= 'F') return (int)(c - 'A' + 10);
    return -1;
}
static int isalnum_ascii(unsigned c) {
    return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
}

/* parseEscape: t points at '\'. returns consumed (>0) or -1 */
static long parse_escape(parser* p, const char* t, size_t n, unsigned* out) {
    if (n < 2) return fail(p, "trailing backslash at end of expression", "", 0);
    unsigned c;
    int k = next_rune(p, t + 1, n - 1, &c);
    if (k < 0) return -1;
    size_t pos = 1 + (size_t)k;
    switch (c) {
        default:
            if (c < 0x80 && !isalnum_ascii(c)) { *out = c; return (long)pos; }
            break;
        case '1': case '2': case '3': case '4': case '5': case '6': case '7':
            if (pos >= n || t[pos] < '0' || t[pos] > '7') break;
            /* fallthrough */
        case '0': {
            unsigned r = c - '0';
            for (int i = 1; i < 3; i++) {
                if (pos >= n || t[pos] < '0' || t[pos] > '7') break;
                r = r * 8 + (unsigned)(t[pos] - '0');
                pos++;
            }
            *out = r;
            return (long)pos;
        }
        case 'x': {
            if (pos >= n) break;
            unsigned d;
            k = next_rune(p, t + pos, n - pos, &d);
            if (k < 0) return -1;
            pos += (size_t)k;
            if (d == '{') {
                int nhex = 0;
                unsigned r = 0;
                for (;;) {
                    if (pos >= n) goto bad;
                    k = next_rune(p, t + pos, n - pos, &d);
                    if (k < 0) return -1;
                    pos += (size_t)k;
                    if (d == '}') break;
                    int v = unhex(d);
                    if (v < 0) goto bad;
                    r = r * 16 + (unsigned)v;
                    if (r > MAX_RUNE) goto bad;
                    nhex++;
                }
                if (nhex == 0) goto bad;
                *out = r;
                return (long)pos;
            }
            int x = unhex(d);
            unsigned e = 0xFFFD;
            if (pos < n) {
                k = next_rune(p, t + pos, n - pos, &e);
                if (k < 0) return -1;
                pos += (size_t)k;
            }
            int y = unhex(e);
            if (x < 0 || y < 0) break;
            *out = (unsigned)(x * 16 + y);
            return (long)pos;
        }
        case 'a': *out = 7; return (long)pos;
        case 'f': *out = 12; return (long)pos;
        case 'n': *out = 10; return (long)pos;
        case 'r': *out = 13; return (long)pos;
        case 't': *out = 9; return (long)pos;
        case 'v': *out = 11; return (long)pos;
    }
bad:
    return fail(p, "invalid escape sequence", t, pos);
}

/* parseClass: t points at '['. returns consumed or -1 */
static long parse_class(parser* p, const char* s, size_t n) {
    size_t i = 1;
    node* nd = new_node(p, N_CLASS);
    rclass* c = &nd->cls;
    int sign = 1;
    if (i < n && s[i] == '^') {
        sign = -1;
        i++;
        /* ClassNL is set under Perl flags: nothing added */
    }
    int first = 1;
    while (i >= n || s[i] != ']' || first) {
        /* PerlX: '-' is fine anywhere */
        first = 0;
        if (i < n && n - i > 2 && s[i] == '[' && s[i + 1] == ':') {
            long k = named_class(p, s + i, n - i, c);
            if (k < 0) return -1;
            if (k > 0) { i += (size_t)k; continue; }
        }
        if (i + 1 < n && s[i] == '\\' && (s[i + 1] == 'p' || s[i + 1] == 'P')) {
            p->unsupported = 1;
            return fail(p, "unsupported \\p class", s + i, 2);
        }
        size_t k = perl_class(p, s + i, n - i, c);
        if (k) { i += k; continue; }
        size_t rng = i;
        unsigned lo, hi;
        if (i >= n) return fail(p, "missing closing ]", s, n);
        if (s[i] == '\\') {
            long e = parse_escape(p, s + i, n - i, &lo);
            if (e < 0) return -1;
            i += (size_t)e;
        } else {
            int kk = next_rune(p, s + i, n - i, &lo);
            if (kk < 0) return -1;
            i += (size_t)kk;
        }
        hi = lo;
        if (n - i >= 2 && s[i] == '-' && s[i + 1] != ']') {
            i++;
            if (i >= n) return fail(p, "missing closing ]", s, n);
            if (s[i] == '\\') {
                long e = parse_escape(p, s + i, n - i, &hi);
                if (e < 0) return -1;
                i += (size_t)e;
            } else {
                int kk = next_rune(p, s + i, n - i, &hi);
                if (kk < 0) return -1;
                i += (size_t)kk;
            }
            if (hi < lo) return fail(p, "invalid character class range", s + rng, i - rng);
        }
        class_add(p, c, lo, hi);
    }
    i++; /* ] */
    rc_clean(c);
    if (sign < 0) rc_negate(c);
    push(p, nd);
    return (long)i;
}

/* ---------- stack collapse ---------- */
static void concat(parser* p) {
    int i = p->n;
    while (i > 0 && p->st[i - 1]->op < P_LPAREN) i--;
    int cnt = p->n - i;
    node* r;
    if (cnt == 0) r = new_node(p, N_EMPTY);
    else if (cnt == 1) r = p->st[i];
    else {
        r = new_node(p, N_CONCAT);
        for (int k = i; k < p->n; k++) add_sub(r, p->st[k]);
    }
    p->n = i;
    push(p, r);
}

/* collapse [x, VBAR, y, VBAR, z] above the nearest LPAREN (or bottom) into ALT */
static void alternate(parser* p) {
    int i = p->n;
    while (i > 0 && p->st[i - 1]->op != P_LPAREN) i--;
    node* r = NULL;
    int nalt = 0;
    for (int k = i; k < p->n; k++)
        if (p->st[k]->op != P_VBAR) nalt++;
    if (nalt == 1) {
        for (int k = i; k < p->n; k++)
            if (p->st[k]->op != P_VBAR) r = p->st[k];
    } else {
        r = new_node(p, N_ALT);
        for (int k = i; k < p->n; k++)
            if (p->st[k]->op != P_VBAR) add_sub(r, p->st[k]);
    }
    p->n = i;
    push(p, r);
}

/* repeatIsValid (regexp/syntax) */
static int repeat_valid(node* re, int n) {
    if (re->op == N_REPEAT) {
        int m = re->max;
        if (m == 0) return 1;
        if (m < 0) m = re->min;
        if (m > n) return 0;
        if (m > 0) n /= m;
    }
    for (int i = 0; i < re->nsub; i++)
        if (!repeat_valid(re->sub[i], n)) return 0;
    return 1;
}

/* parseInt for {n,m}: no leading zeros; >= 1e8 -> -1 */
static int parse_int(const char* s, size_t n, size_t* i, int* v) {
    size_t k = *i;
    if (k >= n || s[k] < '0' || s[k] > '9') return 0;
    if (n - k >= 2 && s[k] == '0' && s[k + 1] >= '0' && s[k + 1] <= '9') return 0;
    size_t st = k;
    while (k < n && s[k] >= '0' && s[k] <= '9') k++;
    int x = 0;
    for (size_t j = st; j < k; j++) {
        if (x >= 100000000) { x = -1; break; }
        x = x * 10 + (s[j] - '0');
    }
    *v = x;
    *i = k;
    return 1;
}

static int parse_repeat(const char* s, size_t n, int* min, int* max, size_t* len) {
    size_t i = 1;
    if (!parse_int(s, n, &i, min)) return 0;
    if (i >= n) return 0;
    if (s[i] != ',') {
        *max = *min;
    } else {
        i++;
        if (i >= n) return 0;
        if (s[i] == '}') *max = -1;
        else {
            if (!parse_int(s, n, &i, max)) return 0;
            if (*max < 0) *min = -1;
        }
    }
    if (i >= n || s[i] != '}') return 0;
    *len = i + 1;
    return 1;
}

static int is_word_name(const char* s, size_t n) {
    if (n == 0) return 0;
    for (size_t i = 0; i < n; i++) {
        char c = s[i];
        if (!(c == '_' || isalnum_ascii((unsigned char)c))) return 0;
    }
    return 1;
}

/* (?...) ; t points at '('. returns consumed or -1 */
static long parse_perl_flags(parser* p, const char* t, size_t n) {
    if (n > 4 && t[2] == 'P' && t[3] == '<') {
        const char* e = memchr(t, '>', n);
        if (!e) return fail(p, "invalid named capture", t, n);
        size_t end = (size_t)(e - t);
        if (!is_word_name(t + 4, end - 4)) return fail(p, "invalid named capture", t, end + 1);
        p->ncap++;
        node* lp = new_node(p, P_LPAREN);
        lp->cap = p->ncap;
        push(p, lp);
        return (long)end + 1;
    }
    size_t i = 2;
    int flags = p->flags;
    int sign = 1, saw = 0;
    while (i < n) {
        unsigned c;
        int k = next_rune(p, t + i, n - i, &c);
        if (k < 0) return -1;
        i += (size_t)k;
        switch (c) {
            default: goto bad;
            case 'i': flags |= F_FOLD; saw = 1; break;
            case 'm': flags &= ~F_ONELINE; saw = 1; break;
            case 's': flags |= F_DOTNL; saw = 1; break;
            case 'U': flags |= F_NONGREEDY; saw = 1; break;
            case '-':
                if (sign < 0) goto bad;
                sign = -1;
                flags = ~flags;
                saw = 0;
                break;
            case ':': case ')':
                if (sign < 0) {
                    if (!saw) goto bad;
                    flags = ~flags;
                }
                if (c == ':') {
                    node* lp = new_node(p, P_LPAREN);
                    push(p, lp);
                }
                p->flags = flags;
                return (long)i;
        }
    }
bad:
    return fail(p, "invalid or unsupported Perl syntax", t, i);
}

static node* parse(parser* p, const char* s, size_t n) {
    p->flags = F_ONELINE;
    p->whole = s;
    p->wlen = n;
    size_t i = 0;
    int last_repeat = 0;
    while (i < n) {
        int repeat = 0;
        char c = s[i];
        switch (c) {
            default: {
                unsigned r;
                int k = next_rune(p, s + i, n - i, &r);
                if (k < 0) return NULL;
                literal(p, r);
                i += (size_t)k;
                break;
            }
            case '(':
                if (n - i >= 2 && s[i + 1] == '?') {
                    long k = parse_perl_flags(p, s + i, n - i);
                    if (k < 0) return NULL;
                    i += (size_t)k;
                    break;
                }
                p->ncap++;
                {
                    node* lp = new_node(p, P_LPAREN);
                    lp->cap = p->ncap;
                    push(p, lp);
                }
                i++;
                break;
            case '|':
                concat(p);
                push(p, new_node(p, P_VBAR));
                i++;
                break;
            case ')': {
                concat(p);
                alternate(p);
                if (p->n < 2 || p->st[p->n - 2]->op != P_LPAREN) {
                    fail(p, "unexpected )", s, n);
                    return NULL;
                }
                node* body = p->st[p->n - 1];
                node* lp = p->st[p->n - 2];
                p->n -= 2;
                p->flags = lp->flags;
                if (lp->cap == 0) push(p, body);
                else {
                    node* cn = new_node(p, N_CAP);
                    add_sub(cn, body);
                    push(p, cn);
                }
                i++;
                break;
            }
            case '^': {
                node* a = new_node(p, N_ASSERT);
                a->assert_bits = (p->flags & F_ONELINE) ? E_BOT : E_BOL;
                push(p, a);
                i++;
                break;
            }
            case '$': {
                node* a = new_node(p, N_ASSERT);
                a->assert_bits = (p->flags & F_ONELINE) ? E_EOT : E_EOL;
                push(p, a);
                i++;
                break;
            }
            case '.': {
                node* d = new_node(p, N_CLASS);
                if (p->flags & F_DOTNL) rc_add(&d->cls, 0, MAX_RUNE);
                else { rc_add(&d->cls, 0, 9); rc_add(&d->cls, 11, MAX_RUNE); }
                push(p, d);
                i++;
                break;
            }
            case '[': {
                long k = parse_class(p, s + i, n - i);
                if (k < 0) return NULL;
                i += (size_t)k;
                break;
            }
            case '*': case '+': case '?': case '{': {
                int op, min = 0, max = 0;
                size_t tl = 1;
                if (c == '{') {
                    if (!parse_repeat(s + i, n - i, &min, &max, &tl)) {
                        literal(p, '{');
                        i++;
                        break;
                    }
                    op = N_REPEAT;
                    if (min < 0 || min > 1000 || max > 1000 || (max >= 0 && min > max)) {
                        fail(p, "invalid repeat count", s + i, tl);
                        return NULL;
                    }
                } else {
                    op = c == '*' ? N_STAR : c == '+' ? N_PLUS : N_QUEST;
                }
                size_t after = i + tl;
                if (after < n && s[after] == '?') after++;
                if (last_repeat) {
                    fail(p, "invalid nested repetition operator", s + i, after - i);
                    return NULL;
                }
                if (p->n == 0 || p->st[p->n - 1]->op >= P_LPAREN) {
                    fail(p, "missing argument to repetition operator", s + i, after - i);
                    return NULL;
                }
                node* sub = p->st[p->n - 1];
                node* r = new_node(p, op);
                r->min = min;
                r->max = max;
                add_sub(r, sub);
                p->st[p->n - 1] = r;
                if (op == N_REPEAT && (min >= 2 || max >= 2) && !repeat_valid(r, 1000)) {
                    fail(p, "invalid repeat count", s + i, after - i);
                    return NULL;
                }
                repeat = 1;
                i = after;
                break;
            }
            case '\\': {
                if (n - i >= 2) {
                    char k = s[i + 1];
                    int a = 0;
                    if (k == 'A') a = E_BOT;
                    else if (k == 'b') a = E_WB;
                    else if (k == 'B') a = E_NWB;
                    else if (k == 'z') a = E_EOT;
                    if (a) {
                        node* an = new_node(p, N_ASSERT);
                        an->assert_bits = a;
                        push(p, an);
                        i += 2;
                        break;
                    }
                    if (k == 'C') { fail(p, "invalid escape sequence", s + i, 2); return NULL; }
                    if (k == 'Q') {
                        size_t j = i + 2;
                        size_t e = n;
                        for (size_t q = j; q + 1 < n; q++)
                            if (s[q] == '\\' && s[q + 1] == 'E') { e = q; break; }
                        while (j < e) {
                            unsigned r;
                            int kk = next_rune(p, s + j, e - j, &r);
                            if (kk < 0) return NULL;
                            literal(p, r);
                            j += (size_t)kk;
                        }
                        i = e < n ? e + 2 : n;
                        break;
                    }
                    if (k == 'p' || k == 'P') {
                        p->unsupported = 1;
                        fail(p, "unsupported \\p group", s + i, 2);
                        return NULL;
                    }
                }
                node* cn = new_node(p, N_CLASS);
                size_t k = perl_class(p, s + i, n - i, &cn->cls);
                if (k) {
                    push(p, cn);
                    i += k;
                    break;
                }
                unsigned r;
                long e = parse_escape(p, s + i, n - i, &r);
                if (e < 0) return NULL;
                literal(p, r);
                i += (size_t)e;
                break;
            }
        }
        last_repeat = repeat;
    }
    concat(p);
    alternate(p);
    if (p->n != 1) {
        fail(p, "missing closing )", s, n);
        return NULL;
    }
    return p->st[0];
}

/* ---------- NFA ---------- */
enum { I_RUNE, I_EMPTY, I_SPLIT, I_JMP, I_MATCH, I_NOP };
typedef struct {
    int op;
    int x, y;
    int bits;
    rclass* cls;
} inst;

struct or_regex {
    inst* prog;
    int n, cap;
    int start;
    rclass* classes; /* owned copies */
    int ncls;
    int too_big;
};

static int emit(or_regex* re, int op) {
    if (re->n == re->cap) {
        re->cap = re->cap ? re->cap * 2 : 64;
        re->prog = (inst*)realloc(re->prog, (size_t)re->cap * sizeof(inst));
    }
    memset(&re->prog[re->n], 0, sizeof(inst));
    re->prog[re->n].op = op;
    re->prog[re->n].x = re->prog[re->n].y = -1;
    if (re->n > 200000) re->too_big = 1;
    return re->n++;
}

/* fragment: start pc and list of dangling out-slots (encoded pc*2+which) */
typedef struct {
    int start;
    int* out;
    int nout;
} frag;

static void patch(or_regex* re, frag* f, int to) {
    for (int i = 0; i < f->nout; i++) {
        int pc = f->out[i] >> 1;
        if (f->out[i] & 1) re->prog[pc].y = to;
        else re->prog[pc].x = to;
    }
    free(f->out);
    f->out = NULL;
    f->nout = 0;
}
static void outs_add(frag* f, int slot) {
    f->out = (int*)realloc(f->out, (size_t)(f->nout + 1) * sizeof(int));
    f->out[f->nout++] = slot;
}
static void outs_merge(frag* a, frag* b) {
    for (int i = 0; i < b->nout; i++) outs_add(a, b->out[i]);
    free(b->out);
    b->out = NULL;
    b->nout = 0;
}

static frag comp(or_regex* re, node* n);

static frag comp_empty(or_regex* re) {
    frag f = {0};
    f.start = emit(re, I_NOP);
    outs_add(&f, f.start * 2);
    return f;
}

static frag comp_star(or_regex* re, frag s) {
    frag f = {0};
    int sp = emit(re, I_SPLIT);
    re->prog[sp].x = s.start;
    patch(re, &s, sp);
    f.start = sp;
    outs_add(&f, sp * 2 + 1);
    return f;
}

static frag comp(or_regex* re, node* n) {
    frag f = {0};
    if (re->too_big) return comp_empty(re);
    switch (n->op) {
        case N_CLASS: {
            int pc = emit(re, I_RUNE);
            re->prog[pc].cls = &n->cls;
            f.start = pc;
            outs_add(&f, pc * 2);
            return f;
        }
        case N_EMPTY: return comp_empty(re);
        case N_ASSERT: {
            int pc = emit(re, I_EMPTY);
            re->prog[pc].bits = n->assert_bits;
            f.start = pc;
            outs_add(&f, pc * 2);
            return f;
        }
        case N_CAP: return comp(re, n->sub[0]);
        case N_CONCAT: {
            f = comp(re, n->sub[0]);
            for (int i = 1; i < n->nsub; i++) {
                frag g = comp(re, n->sub[i]);
                patch(re, &f, g.start);
                f.out = g.out;
                f.nout = g.nout;
            }
            return f;
        }
        case N_ALT: {
            frag acc = comp(re, n->sub[n->nsub - 1]);
            for (int i = n->nsub - 2; i >= 0; i--) {
                frag g = comp(re, n->sub[i]);
                int sp = emit(re, I_SPLIT);
                re->prog[sp].x = g.start;
                re->prog[sp].y = acc.start;
                outs_merge(&g, &acc);
                g.start = sp;
                acc = g;
            }
            return acc;
        }
        case N_STAR: return comp_star(re, comp(re, n->sub[0]));
        case N_PLUS: {
            frag s = comp(re, n->sub[0]);
            int sp = emit(re, I_SPLIT);
            re->prog[sp].x = s.start;
            patch(re, &s, sp);
            f.start = s.start;
            outs_add(&f, sp * 2 + 1);
            return f;
        }
        case N_QUEST: {
            frag s = comp(re, n->sub[0]);
            int sp = emit(re, I_SPLIT);
            re->prog[sp].x = s.start;
            f.start = sp;
            outs_merge(&f, &s);
            outs_add(&f, sp * 2 + 1);
            return f;
        }
        case N_REPEAT: {
            int min = n->min, max = n->max;
            if (max == 0) return comp_empty(re);
            frag acc = {0};
            int have = 0;
            for (int i = 0; i < min; i++) {
                frag g = comp(re, n->sub[0]);
                if (!have) { acc = g; have = 1; }
                else { patch(re, &acc, g.start); acc.out = g.out; acc.nout = g.nout; }
            }
            if (max < 0) {
                frag g = comp_star(re, comp(re, n->sub[0]));
                if (!have) return g;
                patch(re, &acc, g.start);
                acc.out = g.out;
                acc.nout = g.nout;
                return acc;
            }
            /* (x(x(x)?)?)? for the optional copies */
            int opt = max - min;
            frag tail = {0};
            int have_tail = 0;
            for (int i = 0; i < opt; i++) {
                frag g = comp(re, n->sub[0]);
                if (have_tail) {
                    patch(re, &g, tail.start);
                    outs_merge(&g, &tail);
                }
                int sp = emit(re, I_SPLIT);
                re->prog[sp].x = g.start;
                frag q = {0};
                q.start = sp;
                outs_merge(&q, &g);
                outs_add(&q, sp * 2 + 1);
                tail = q;
                have_tail = 1;
            }
            if (!have_tail) return acc; /* x{n}: no optional copies */
            if (!have) return tail;
            patch(re, &acc, tail.start);
            acc.out = tail.out;
            acc.nout = tail.nout;
            return acc;
        }
    }
    return comp_empty(re);
}

/* deep-copy the classes the program points at so the AST can be freed */
static void own_classes(or_regex* re) {
    int cnt = 0;
    for (int i = 0; i < re->n; i++)
        if (re->prog[i].op == I_RUNE) cnt++;
    re->classes = (rclass*)calloc((size_t)(cnt ? cnt : 1), sizeof(rclass));
    re->ncls = 0;
    for (int i = 0; i < re->n; i++) {
        if (re->prog[i].op != I_RUNE) continue;
        rclass* src = re->prog[i].cls;
        rclass* dst = &re->classes[re->ncls++];
        dst->n = dst->cap = src->n;
        dst->r = (rr*)malloc((size_t)(src->n ? src->n : 1) * sizeof(rr));
        memcpy(dst->r, src->r, (size_t)src->n * sizeof(rr));
        re->prog[i].cls = dst;
    }
}

or_regex* or_regex_compile(const char* pat, size_t n, char* errbuf, size_t errcap, int* unsupported) {
    parser p;
    memset(&p, 0, sizeof p);
    p.err = errbuf;
    p.errcap = errcap;
    if (errcap) errbuf[0] = 0;
    *unsupported = 0;
    node* root = parse(&p, pat, n);
    or_regex* re = NULL;
    if (root && !p.unsupported) {
        re = (or_regex*)calloc(1, sizeof(or_regex));
        frag f = comp(re, root);
        int m = emit(re, I_MATCH);
        patch(re, &f, m);
        re->start = f.start;
        own_classes(re);
        if (re->too_big) {
            or_regex_free(re);
            re = NULL;
            p.unsupported = 1;
        }
    }
    if (p.unsupported) {
        *unsupported = 1;
        if (errcap) snprintf(errbuf, errcap, "regex syntax not restated by the oracle");
        if (re) { or_regex_free(re); re = NULL; }
    }
    for (int i = 0; i < p.nall; i++) {
        free(p.all[i]->cls.r);
        free(p.all[i]->sub);
        free(p.all[i]);
    }
    free(p.all);
    free(p.st);
    return re;
}

void or_regex_free(or_regex* re) {
    if (!re) return;
    for (int i = 0; i < re->ncls; i++) free(re->classes[i].r);
    free(re->classes);
    free(re->prog);
    free(re);
}

/* ---------- Pike VM ---------- */
static int is_word(long r) {
    return r >= 0 && r < 0x80 && (isalnum_ascii((unsigned)r) || r == '_');
}
/* syntax.EmptyOpContext(r1, r2) */
static int empty_ctx(long r1, long r2) {
    int op = E_NWB;
    int boundary = 0;
    if (is_word(r1)) boundary = 1;
    else if (r1 == '\n') op |= E_BOL;
    else if (r1 < 0) op |= E_BOT | E_BOL;
    if (is_word(r2)) boundary ^= 1;
    else if (r2 == '\n') op |= E_EOL;
    else if (r2 < 0) op |= E_EOT | E_EOL;
    if (boundary) op ^= (E_WB | E_NWB);
    return op;
}

typedef struct {
    int* pcs;
    int n;
    unsigned char* on;
} tlist;

/* add pc and its epsilon closure under context ctx; returns 1 if MATCH reached */
static int addthread(const or_regex* re, tlist* l, int pc, int ctx, int* stack) {
    int sp = 0;
    stack[sp++] = pc;
    int matched = 0;
    while (sp) {
        int q = stack[--sp];
        if (q < 0 || l->on[q]) continue;
        l->on[q] = 1;
        const inst* in = &re->prog[q];
        switch (in->op) {
            case I_MATCH: matched = 1; break;
            case I_RUNE: l->pcs[l->n++] = q; break;
            case I_NOP: case I_JMP: stack[sp++] = in->x; break;
            case I_SPLIT: stack[sp++] = in->y; stack[sp++] = in->x; break;
            case I_EMPTY:
                if ((in->bits & ~ctx) == 0) stack[sp++] = in->x;
                break;
        }
    }
    return matched;
}

int or_regex_match(const or_regex* re, const char* s, size_t n) {
    int np = re->n;
    tlist a, b;
    a.pcs = (int*)malloc((size_t)np * sizeof(int));
    b.pcs = (int*)malloc((size_t)np * sizeof(int));
    a.on = (unsigned char*)calloc((size_t)np, 1);
    b.on = (unsigned char*)calloc((size_t)np, 1);
    int* stack = (int*)malloc((size_t)(2 * np + 4) * sizeof(int));
    a.n = b.n = 0;
    tlist* cur = &a;
    tlist* nxt = &b;
    const unsigned char* u = (const unsigned char*)s;
    size_t pos = 0;
    long prev = -1;
    int result = 0;
    for (;;) {
        unsigned r = 0;
        int w = 0;
        long next = -1;
        if (pos < n) {
            w = decode_rune(u + pos, n - pos, &r);
            next = (long)r;
        }
        int ctx = empty_ctx(prev, next);
        /* re-closure of the carried threads is not needed: carried pcs are the targets of
         * rune instructions, already expanded below with this position's context. */
        if (addthread(re, cur, re->start, ctx, stack)) { result = 1; break; }
        if (pos >= n) break;
        /* step */
        memset(nxt->on, 0, (size_t)np);
        nxt->n = 0;
        unsigned r2 = 0;
        long after = -1;
        if (pos + (size_t)w < n) {
            decode_rune(u + pos + w, n - pos - w, &r2);
            after = (long)r2;
        }
        int ctx2 = empty_ctx(next, after);
        int hit = 0;
        for (int i = 0; i < cur->n; i++) {
            const inst* in = &re->prog[cur->pcs[i]];
            if (rc_has(in->cls, r)) {
                if (addthread(re, nxt, in->x, ctx2, stack)) { hit = 1; break; }
            }
        }
        if (hit) { result = 1; break; }
        tlist* t = cur;
        cur = nxt;
        nxt = t;
        pos += (size_t)w;
        prev = next;
    }
    free(a.pcs); free(b.pcs); free(a.on); free(b.on); free(stack);
    return result;
}
