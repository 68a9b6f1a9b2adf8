/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's pattern-matching hot path, used solely as the
 * checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg. The
 * product (authorino_amd/, libauthjx.so) never links or calls anything in oracle/.
 *
 * What it restates (reference = /root/reference, modassarrana89/authorino @ 2024-08-07):
 *   - pkg/jsonexp/expressions.go:10-178   Operator, Pattern.Matches, And/Or/All/Any
 *   - pkg/evaluators/authorization/json.go:15-27   JSONPatternMatching.Call
 *   - pkg/service/auth_pipeline.go:378-388   evaluateConditions
 *   - third-party github.com/tidwall/gjson v1.14.0 (go.mod:22; source NOT in the
 *     reference tree): Get / Result.String / Result.Array for simple paths
 *   - Go 1.21 strconv ParseFloat / FormatFloat(f,'f',-1,64) (used by gjson String())
 *   - Go 1.21 regexp (RE2 syntax) Compile / MatchString (regex_ref.c)
 *
 * Pinning: tests/test_oracle_golden.py checks this oracle against every known-answer
 * vector the reference's own tests hold for this path (pkg/jsonexp/expressions_test.go,
 * pkg/evaluators/authorization/json_test.go, pkg/json/json_test.go selector cases,
 * pkg/service/auth_pipeline_test.go `when` cases). Behaviour not covered by any
 * reference test (see SURVEY.md §8c "Parity unpinned") is restated from the published
 * gjson / Go algorithms and documented as unpinned in DESIGN.md.
 */
#ifndef AUTHJX_ORACLE_H
#define AUTHJX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* gjson.Type (gjson v1.14.0): Null=0, False, Number, String, True, JSON */
enum { OR_NULL = 0, OR_FALSE = 1, OR_NUMBER = 2, OR_STRING = 3, OR_TRUE = 4, OR_JSON = 5 };

/* Growable byte buffer (oracle-private scratch). */
typedef struct {
    char* p;
    size_t n, cap;
} or_buf;

void or_buf_reset(or_buf* b);
void or_buf_free(or_buf* b);
void or_buf_push(or_buf* b, const char* s, size_t n);

/* gjson.Result. raw/str point into the document or into `own`. */
typedef struct {
    int type;
    const char* raw;
    size_t raw_len;
    const char* str; /* String(): for OR_STRING the (possibly unescaped) contents */
    size_t str_len;
    double num;
    or_buf own; /* backing store for unescaped strings */
} or_result;

void or_result_free(or_result* r);

/* Path classification: 0 = simple (restated here), -1 = uses gjson syntax this
 * oracle does not restate (modifiers, wildcards, queries, multipaths, '#'). */
int or_path_supported(const char* path, size_t plen);

/* gjson.Get(json, path). Returns 0, or -1 for an unsupported path (r = Null). */
int or_gjson_get(const char* json, size_t jlen, const char* path, size_t plen, or_result* r);

/* Result.String() appended to out. */
void or_result_string(const or_result* r, or_buf* out);

/* Result.Array(): iterate; returns 1 and fills item while elements remain.
 * *cursor must start at 0. item must be freed with or_result_free by the caller
 * (it is reset on every call). */
int or_result_array_next(const or_result* r, size_t* cursor, or_result* item);

/* ---- the reference's gjson modifiers (pkg/json/json.go:161-264; gjson_mods_ref.c) ---- */
enum { OR_MOD_EXTRACT = 1, OR_MOD_REPLACE = 2, OR_MOD_CASE = 3, OR_MOD_BASE64 = 4, OR_MOD_STRIP = 5,
       OR_MOD_FROMSTR = 6 /* gjson's own @fromstr */, OR_MOD_PATH = 7 /* a path Get after a modifier (a) */ };
/* gjson Valid (validpayload): 1 when s[0..n) is one JSON value with surrounding whitespace */
int or_valid(const char* s, size_t n);
typedef struct {
    int kind, variant, has_old;
    char* a; /* extract: sep; replace: old */
    size_t a_len;
    char* b; /* replace: new */
    size_t b_len;
    uint64_t pos; /* extract */
} or_mod;
/* Split path into a plain base (path[0 .. *base_len)) and a modifier chain: 0 none, 1 ok,
 * -1 a form not restated. Free the chain with or_mods_free. */
int or_mod_split(const char* path, size_t n, size_t* base_len, or_mod* mods, int max_mods, int* n_mods);
void or_mods_free(or_mod* mods, int n);
/* Run the chain on a found value's raw JSON: the last output text (0), or -1 undecided
 * (non-ASCII text under @case / @strip, a Parse the oracle does not restate). */
int or_mod_apply(const or_mod* mods, int n_mods, const char* raw, size_t raw_len, or_buf* text);
/* gjson.Parse(text) (0; -1 for a leading '+' 'i' 'I' 'N' or NaN-like 'n'). */
int or_parse(const char* text, size_t n, or_result* r);
/* gjson.Get with a modifier chain (text: the chain's output, r points into it): 0, -1
 * unsupported path, -2 undecided. */
int or_gjson_get_mods(const char* json, size_t jlen, const char* path, size_t plen, or_result* r, or_buf* text);

/* gjson's unescape(): JSON string escapes -> bytes (exact quirks restated). */
void or_unescape(const char* s, size_t n, or_buf* out);

/* Go strconv.ParseFloat(s, 64): returns 0 ok, 1 syntax error (*out=0), 2 range error (*out=+-Inf). */
int or_go_parse_float(const char* s, size_t n, double* out);
/* Go strconv.FormatFloat(f, 'f', -1, 64) appended to out. */
void or_go_format_float(double f, or_buf* out);

/* ---- jsonexp ---------------------------------------------------------- */
/* Operator (pkg/jsonexp/expressions.go:12-19) */
enum { OR_OP_UNKNOWN = 0, OR_OP_EQ = 1, OR_OP_NEQ = 2, OR_OP_INCL = 3, OR_OP_EXCL = 4, OR_OP_MATCHES = 5 };
/* Tri-state result of Matches(): (false,nil)=F, (true,nil)=T, (false,err)=E */
enum { OR_F = 0, OR_T = 1, OR_E = 2, OR_UNSUPPORTED = 3 };

typedef struct {
    const char* selector;
    uint32_t selector_len;
    int32_t op;
    const char* value;
    uint32_t value_len;
} or_pattern;

/* Node kinds of an expression tree: a Pattern leaf, an And{Left,Right} or Or{Left,Right}
 * (children are node indices, -1 = nil). */
enum { OR_NODE_PATTERN = 0, OR_NODE_AND = 1, OR_NODE_OR = 2 };
typedef struct {
    int32_t kind;
    int32_t left, right;
    int32_t pattern;
} or_node;

typedef struct or_ruleset or_ruleset;

/* Build a checker for one expression tree (root index; -1 = nil expression). */
or_ruleset* or_ruleset_new(const or_pattern* patterns, uint32_t n_patterns, const or_node* nodes,
                           uint32_t n_nodes, int32_t root);
void or_ruleset_free(or_ruleset* rs);
/* Pattern.Matches for pattern i of the set: OR_T / OR_F / OR_E / OR_UNSUPPORTED. */
int or_pattern_matches(or_ruleset* rs, uint32_t i, const char* json, size_t jlen);
/* Expression.Matches for the root; *err_pattern receives the pattern whose error
 * decided the result (or -1). nil root -> T (matches JSONPatternMatching Rules==nil). */
int or_expression_matches(or_ruleset* rs, const char* json, size_t jlen, int32_t* err_pattern);
/* Error text Go would produce for pattern i when it evaluates to E (static). */
const char* or_pattern_error(or_ruleset* rs, uint32_t i);

/* Batch evaluation over a packed arena with nthreads host threads (cpu_baseline). */
void or_eval_batch(or_ruleset* const* sets, const uint32_t* set_of_req, const uint8_t* arena,
                   const uint64_t* offs, const uint32_t* lens, uint32_t n, uint8_t* out_tristate,
                   int32_t* out_err_idx, uint64_t* out_bitmap, uint32_t bitmap_stride_words,
                   int nthreads);

/* ---- Go regexp (regex_ref.c) ---------------------------------------- */
typedef struct or_regex or_regex;
/* Compile with Go 1.21 regexp.Compile semantics. Returns NULL on error and writes
 * the Go error text ("error parsing regexp: ...") into errbuf.
 * *unsupported is set when the pattern uses syntax this oracle does not restate
 * (\p{..} Unicode groups, non-ASCII case folding). */
or_regex* or_regex_compile(const char* pat, size_t n, char* errbuf, size_t errcap, int* unsupported);
int or_regex_match(const or_regex* re, const char* s, size_t n);
void or_regex_free(or_regex* re);

#ifdef __cplusplus
}
#endif
#endif
