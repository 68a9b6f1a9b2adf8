/*
 * jsonexp_ref.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restatement of pkg/jsonexp/expressions.go:
 *   Pattern.Matches  :59-96   gjson.Get, then eq/neq on String(), incl/excl over
 *                             Array() items' String(), matches = regexp.Compile (per
 *                             call in the reference; its error is static so it is
 *                             compiled once here) + MatchString, unknown op -> error
 *   And.Matches      :111-125 nil side skipped; left err/false returned first
 *   Or.Matches       :136-154 left err returned even if right would be true
 *   All / Any        :160-178 right-nested chains ending in empty And{} / Or{}
 * plus the per-batch driver used as the CPU baseline (std threads over requests).
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
    or_pattern p;
    or_regex* re;     /* matches: compiled once */
    int static_state; /* -1 none, OR_E = static error, OR_UNSUPPORTED */
    char err[256];
    size_t base_len;  /* the selector's plain path (before a modifier chain) */
    or_mod mods[8];   /* pkg/json/json.go modifiers applied to the path's value */
    int n_mods;
} pat_entry;

struct or_ruleset {
    pat_entry* pats;
    uint32_t n_pats;
    or_node* nodes;
    uint32_t n_nodes;
    int32_t root;
};

or_ruleset* or_ruleset_new(const or_pattern* patterns, uint32_t n_patterns, const or_node* nodes,
                           uint32_t n_nodes, int32_t root) {
    or_ruleset* rs = (or_ruleset*)calloc(1, sizeof(*rs));
    rs->pats = (pat_entry*)calloc(n_patterns ? n_patterns : 1, sizeof(pat_entry));
    rs->n_pats = n_patterns;
    rs->nodes = (or_node*)calloc(n_nodes ? n_nodes : 1, sizeof(or_node));
    memcpy(rs->nodes, nodes, n_nodes * sizeof(or_node));
    rs->n_nodes = n_nodes;
    rs->root = root;
    for (uint32_t i = 0; i < n_patterns; i++) {
        pat_entry* e = &rs->pats[i];
        e->p = patterns[i];
        e->static_state = -1;
        e->base_len = e->p.selector_len;
        int mr = or_mod_split(e->p.selector, e->p.selector_len, &e->base_len, e->mods, 8, &e->n_mods);
        if (mr <= 0) {
            or_mods_free(e->mods, e->n_mods);
            e->n_mods = 0;
            e->base_len = e->p.selector_len;
        }
        if (mr < 0 || or_path_supported(e->p.selector, e->base_len) != 0) {
            e->static_state = OR_UNSUPPORTED;
            snprintf(e->err, sizeof e->err, "unsupported selector syntax");
            continue;
        }
        switch (e->p.op) {
            case OR_OP_EQ: case OR_OP_NEQ: case OR_OP_INCL: case OR_OP_EXCL: break;
            case OR_OP_MATCHES: {
                int unsup = 0;
                e->re = or_regex_compile(e->p.value, e->p.value_len, e->err, sizeof e->err, &unsup);
                if (!e->re) e->static_state = unsup ? OR_UNSUPPORTED : OR_E;
                break;
            }
            default:
                e->static_state = OR_E;
                snprintf(e->err, sizeof e->err, "unsupported operator for json authorization");
        }
    }
    return rs;
}

void or_ruleset_free(or_ruleset* rs) {
    if (!rs) return;
    for (uint32_t i = 0; i < rs->n_pats; i++) {
        if (rs->pats[i].re) or_regex_free(rs->pats[i].re);
        or_mods_free(rs->pats[i].mods, rs->pats[i].n_mods);
    }
    free(rs->pats);
    free(rs->nodes);
    free(rs);
}

const char* or_pattern_error(or_ruleset* rs, uint32_t i) { return rs->pats[i].err; }

typedef struct {
    or_result v, item;
    or_buf s;
    or_buf mt; /* modifier chain output text (v points into it) */
} scratch;

static int str_eq(const or_buf* b, const char* v, uint32_t n) {
    return b->n == n && (n == 0 || memcmp(b->p, v, n) == 0);
}

static int pattern_matches(or_ruleset* rs, uint32_t i, const char* json, size_t jlen, scratch* sc) {
    pat_entry* e = &rs->pats[i];
    if (e->static_state >= 0) return e->static_state;
    or_gjson_get(json, jlen, e->p.selector, e->base_len, &sc->v);
    /* gjson pipes a found value (raw JSON) through the modifiers and Parses the output */
    if (e->n_mods && sc->v.raw_len > 0) {
        if (or_mod_apply(e->mods, e->n_mods, sc->v.raw, sc->v.raw_len, &sc->mt) != 0) return OR_UNSUPPORTED;
        if (or_parse(sc->mt.p ? sc->mt.p : "", sc->mt.n, &sc->v) != 0) return OR_UNSUPPORTED;
    }
    switch (e->p.op) {
        case OR_OP_EQ:
        case OR_OP_NEQ: {
            or_buf_reset(&sc->s);
            or_result_string(&sc->v, &sc->s);
            int eq = str_eq(&sc->s, e->p.value, e->p.value_len);
            return (e->p.op == OR_OP_EQ) == eq ? OR_T : OR_F;
        }
        case OR_OP_INCL:
        case OR_OP_EXCL: {
            size_t cur = 0;
            int found = 0;
            while (or_result_array_next(&sc->v, &cur, &sc->item)) {
                or_buf_reset(&sc->s);
                or_result_string(&sc->item, &sc->s);
                if (str_eq(&sc->s, e->p.value, e->p.value_len)) { found = 1; break; }
            }
            return (e->p.op == OR_OP_INCL) == found ? OR_T : OR_F;
        }
        case OR_OP_MATCHES: {
            or_buf_reset(&sc->s);
            or_result_string(&sc->v, &sc->s);
            return or_regex_match(e->re, sc->s.p ? sc->s.p : "", sc->s.n) ? OR_T : OR_F;
        }
    }
    return OR_E;
}

int or_pattern_matches(or_ruleset* rs, uint32_t i, const char* json, size_t jlen) {
    scratch sc;
    memset(&sc, 0, sizeof sc);
    int r = pattern_matches(rs, i, json, jlen, &sc);
    or_result_free(&sc.v);
    or_result_free(&sc.item);
    or_buf_free(&sc.s);
    or_buf_free(&sc.mt);
    return r;
}

/* Recursive Matches with the reference's short-circuit order. Result T/F/E/UNSUPPORTED;
 * *errp = pattern index whose error decided. res (may be NULL): every pattern's result
 * already evaluated once (the batch driver's bitmap pass), read instead of re-evaluating. */
static int node_matches_r(or_ruleset* rs, int32_t n, const char* json, size_t jlen, scratch* sc,
                          int32_t* errp, const uint8_t* res) {
    const or_node* nd = &rs->nodes[n];
    if (nd->kind == OR_NODE_PATTERN) {
        int r = res ? res[nd->pattern] : pattern_matches(rs, (uint32_t)nd->pattern, json, jlen, sc);
        if (r == OR_E || r == OR_UNSUPPORTED) *errp = nd->pattern;
        return r;
    }
    if (nd->kind == OR_NODE_AND) {
        if (nd->left >= 0) {
            int l = node_matches_r(rs, nd->left, json, jlen, sc, errp, res);
            if (l != OR_T) return l;
        }
        if (nd->right >= 0) {
            int r = node_matches_r(rs, nd->right, json, jlen, sc, errp, res);
            if (r != OR_T) return r;
        }
        return OR_T;
    }
    /* Or */
    if (nd->left >= 0) {
        int l = node_matches_r(rs, nd->left, json, jlen, sc, errp, res);
        if (l == OR_E || l == OR_UNSUPPORTED) return l;
        if (l == OR_T) return OR_T;
    }
    if (nd->right >= 0) return node_matches_r(rs, nd->right, json, jlen, sc, errp, res);
    return OR_F;
}

static int node_matches(or_ruleset* rs, int32_t n, const char* json, size_t jlen, scratch* sc,
                        int32_t* errp) {
    return node_matches_r(rs, n, json, jlen, sc, errp, NULL);
}

int or_expression_matches(or_ruleset* rs, const char* json, size_t jlen, int32_t* err_pattern) {
    *err_pattern = -1;
    if (rs->root < 0) return OR_T;
    scratch sc;
    memset(&sc, 0, sizeof sc);
    int r = node_matches(rs, rs->root, json, jlen, &sc, err_pattern);
    or_result_free(&sc.v);
    or_result_free(&sc.item);
    or_buf_free(&sc.s);
    or_buf_free(&sc.mt);
    if (r != OR_E && r != OR_UNSUPPORTED) *err_pattern = -1;
    return r;
}

/* ---- batch driver (cpu_baseline) ------------------------------------------ */
typedef struct {
    or_ruleset* const* sets;
    const uint32_t* set_of_req;
    const uint8_t* arena;
    const uint64_t* offs;
    const uint32_t* lens;
    uint8_t* out_tristate;
    int32_t* out_err_idx;
    uint64_t* out_bitmap;
    uint32_t stride;
    uint32_t lo, hi;
} job;

static void* run_job(void* arg) {
    job* j = (job*)arg;
    scratch sc;
    memset(&sc, 0, sizeof sc);
    uint8_t* res = NULL;
    uint32_t res_cap = 0;
    for (uint32_t r = j->lo; r < j->hi; r++) {
        or_ruleset* rs = j->sets[j->set_of_req ? j->set_of_req[r] : 0];
        const char* doc = (const char*)j->arena + j->offs[r];
        size_t len = j->lens[r];
        const uint8_t* cached = NULL;
        if (j->out_bitmap) {
            /* every pattern once: the bitmap, then the tree walk reads these results */
            if (rs->n_pats > res_cap) {
                res_cap = rs->n_pats;
                res = (uint8_t*)realloc(res, res_cap);
            }
            uint64_t* row = j->out_bitmap + (size_t)r * j->stride;
            memset(row, 0, j->stride * sizeof(uint64_t));
            for (uint32_t p = 0; p < rs->n_pats; p++) {
                res[p] = (uint8_t)pattern_matches(rs, p, doc, len, &sc);
                if (res[p] == OR_T) row[p >> 6] |= 1ull << (p & 63);
            }
            cached = res;
        }
        int32_t ep = -1;
        int t = OR_T;
        if (rs->root >= 0) t = node_matches_r(rs, rs->root, doc, len, &sc, &ep, cached);
        if (t != OR_E && t != OR_UNSUPPORTED) ep = -1;
        j->out_tristate[r] = (uint8_t)t;
        if (j->out_err_idx) j->out_err_idx[r] = ep;
    }
    or_result_free(&sc.v);
    or_result_free(&sc.item);
    or_buf_free(&sc.s);
    or_buf_free(&sc.mt);
    free(res);
    return NULL;
}

void or_eval_batch(or_ruleset* const* sets, const uint32_t* set_of_req, const uint8_t* arena,
                   const uint64_t* offs, const uint32_t* lens, uint32_t n, uint8_t* out_tristate,
                   int32_t* out_err_idx, uint64_t* out_bitmap, uint32_t bitmap_stride_words,
                   int nthreads) {
    if (nthreads < 1) nthreads = 1;
    job* jobs = (job*)calloc((size_t)nthreads, sizeof(job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        job* j = &jobs[t];
        j->sets = sets; j->set_of_req = set_of_req; j->arena = arena; j->offs = offs; j->lens = lens;
        j->out_tristate = out_tristate; j->out_err_idx = out_err_idx; j->out_bitmap = out_bitmap;
        j->stride = bitmap_stride_words;
        j->lo = (uint32_t)((uint64_t)n * t / nthreads);
        j->hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
        if (nthreads == 1) run_job(j);
        else pthread_create(&th[t], NULL, run_job, j);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
}
