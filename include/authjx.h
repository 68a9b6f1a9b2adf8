/*
 * authjx.h — C-ABI of libauthjx.so, the MI355X-native batched evaluator for Authorino's
 * pattern-matching authorization hot path.
 *
 * Plain C types only (pointers, sizes, integers); no torch / HIP types in signatures
 * (`stream` is an opaque hipStream_t passed as void*).
 *
 * Concurrency: every function may be called from any thread. Compiled rulesets are
 * immutable after authjx_compile and may be shared by any number of threads and
 * contexts of their device (the reference shares expression trees across goroutines:
 * pkg/service/auth.go:300 copies AuthConfig by value, sharing its trees). A context
 * keeps one workspace (set table, capture rows, exact-scan list, request order) per
 * stream it is called with: batches on different streams of one context run
 * concurrently without sharing scratch; calls on one stream are serialised (their
 * kernels are ordered by the stream). authjx_free waits for the last batch of every
 * stream that used the ruleset, nothing else. The host-buffer entry points
 * (authjx_eval_batch, authjx_select_batch) use the context's own stream, one call at a
 * time. For many concurrent callers with one request each, use the micro-batcher
 * (authjx_batcher_*), which forms the batches.
 *
 * Interface each entry point replaces (reference = modassarrana89/authorino):
 *   authjx_compile          controllers/auth_config_controller.go:805-852
 *                           buildJSONExpression / buildJSONExpressionPattern(s): the
 *                           reconcile-time construction of a jsonexp tree. Here the tree
 *                           (flattened, see authjx_tree) is compiled once into
 *                           device-resident tables (selector paths, literal pool,
 *                           fold bytecode, regex DFAs).
 *   authjx_compile_forest   the same compile point for every expression of one
 *                           AuthConfig's authorization phase at once (one document scan
 *                           per request for all of them).
 *   authjx_free             pkg/auth/auth.go:30-33 AuthConfigCleaner.Clean (called from
 *                           pkg/evaluators/config.go:42-68 before re-translate/delete).
 *   authjx_eval_batch[_device]
 *                           pkg/jsonexp/expressions.go:102-104 Expression.Matches(json)
 *                           (Pattern.Matches :59-96, And :111-125, Or :136-154) for a
 *                           micro-batch of Authorization-JSON documents; its callers are
 *                           pkg/evaluators/authorization/json.go:19 (JSON rules) and
 *                           pkg/service/auth_pipeline.go:382 (every `when` gate).
 *   authjx_select_batch[_device]
 *                           pkg/json/json.go:41-53 JSONValue.ResolveFor's
 *                           gjson.Get(authJSON, pattern) (and the per-placeholder Get of
 *                           ReplaceJSONPlaceholders, :96-151) for a micro-batch: the
 *                           selector values behind response headers
 *                           (pkg/evaluators/response.go:150-174), returned as spans of
 *                           the document that the host formats (Value()/String()).
 *   authjx_pattern_error    the static error a pattern yields (regexp.Compile's
 *                           "error parsing regexp: ..." or expressions.go:94
 *                           "unsupported operator for json authorization").
 */
#ifndef AUTHJX_H
#define AUTHJX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AUTHJX_ABI_VERSION 1

/* return codes */
#define AUTHJX_OK 0
#define AUTHJX_EINVAL (-1)
#define AUTHJX_ENOMEM (-2)
#define AUTHJX_EDEVICE (-3)
#define AUTHJX_ELIMIT (-4)
#define AUTHJX_ETIMEDOUT (-5) /* micro-batcher: the deadline passed before evaluation */
#define AUTHJX_ECLOSED (-6)   /* micro-batcher: destroyed while the request waited for room */
#define AUTHJX_EEXIST (-7)    /* index: the key is taken and override was not asked for */

/* jsonexp.Operator (pkg/jsonexp/expressions.go:12-19) */
#define AUTHJX_OP_UNKNOWN 0
#define AUTHJX_OP_EQ 1
#define AUTHJX_OP_NEQ 2
#define AUTHJX_OP_INCL 3
#define AUTHJX_OP_EXCL 4
#define AUTHJX_OP_MATCHES 5

/* tree node kinds: jsonexp.Pattern, *jsonexp.And, *jsonexp.Or */
#define AUTHJX_NODE_PATTERN 0
#define AUTHJX_NODE_AND 1
#define AUTHJX_NODE_OR 2

/* Tri-state result of Expression.Matches: (false,nil)=F, (true,nil)=T, (false,err)=E.
 * UNDECIDED: the result depends on a pattern compiled as AUTHJX_PAT_UNSUPPORTED, or on
 * a hex mantissa / '_'-separated number literal (never valid JSON); the caller must not
 * take a decision from it and routes that request to its own evaluator. Every JSON
 * number is decided: Go ParseFloat + FormatFloat(f, 'f', -1, 64) run exactly on the
 * device (ajx_float.h). */
#define AUTHJX_F 0
#define AUTHJX_T 1
#define AUTHJX_E 2
#define AUTHJX_UNDECIDED 3

/* per-pattern compile status */
#define AUTHJX_PAT_OK 0
#define AUTHJX_PAT_STATIC_ERROR 1 /* Matches always returns (false, err): bad regex / op */
#define AUTHJX_PAT_UNSUPPORTED 2  /* selector / regex syntax not compiled for the device */

typedef struct authjx_ctx authjx_ctx;
typedef struct authjx_ruleset authjx_ruleset;

typedef struct {
    const char* selector; /* gjson path (jsonexp.Pattern.Selector) */
    uint32_t selector_len;
    int32_t op; /* AUTHJX_OP_* */
    const char* value; /* jsonexp.Pattern.Value */
    uint32_t value_len;
} authjx_pattern;

typedef struct {
    int32_t kind;  /* AUTHJX_NODE_* */
    int32_t left;  /* node index or -1 (nil) */
    int32_t right; /* node index or -1 (nil) */
    int32_t pattern; /* pattern index for AUTHJX_NODE_PATTERN */
} authjx_node;

/* One jsonexp.Expression, flattened. root = -1 means a nil Expression. */
typedef struct {
    const authjx_pattern* patterns;
    uint32_t n_patterns;
    const authjx_node* nodes;
    uint32_t n_nodes;
    int32_t root;
} authjx_tree;

/* Device context: one per GPU (device ordinal). authjx_shutdown first destroys every
 * micro-batcher still alive on the context (authjx_batcher_destroy: queued requests are
 * evaluated); their handles are invalid afterwards. */
int authjx_init(int device, authjx_ctx** out);
void authjx_shutdown(authjx_ctx* ctx);
/* Release the per-stream workspace (capture rows, slow list, order, set table) the
 * context keeps for `stream` since its first device call on it: for callers that use
 * short-lived streams. Not the context's own stream. The workspace is reference-counted:
 * a call still running on that stream, or an authjx_last_* reader, keeps it until that
 * call returns, and whichever thread drops the last reference (this one, or that call's)
 * waits for the stream's last batch before freeing it, so this call may return before
 * that batch has ended. Only authjx_shutdown must not race the context's calls. */
int authjx_release_stream(authjx_ctx* ctx, void* stream);
// The sha256 (first 32 hex digits) of the sources the library was built from
// (authorino_amd/build.py source_hash); the Python runtime refuses a stale binary.
const char* authjx_build_hash(void);
int authjx_device_count(void);

/* Compile one tree into a device-resident ruleset. pattern_status (n_patterns entries,
 * may be NULL) receives AUTHJX_PAT_*. A ruleset that contains UNSUPPORTED patterns is
 * still created; evaluating it yields AUTHJX_UNDECIDED for requests whose result
 * depends on them. errbuf (may be NULL) receives a diagnostic. */
int authjx_compile(authjx_ctx* ctx, const authjx_tree* tree, authjx_ruleset** out,
                   int32_t* pattern_status, char* errbuf, size_t errcap);
/* Compile several trees that read the same documents into ONE ruleset, so that one
 * scan of a document evaluates all of them (an authorization phase: the AuthConfig-level
 * `when`, each evaluator's `when` and rules — pkg/service/auth_pipeline.go:120-125,
 * :287-322, :454-457). Patterns are numbered across the trees in order (tree k's
 * pattern i is pattern sum_{j<k} n_patterns_j + i; pattern_status has that many
 * entries); selectors shared by several trees are scanned once. Evaluating it writes
 * one result per tree: d_out_tristate[r * n_trees + k] and d_out_err_idx[r * n_trees + k]
 * (the error index in the forest's numbering). Every ruleset of one batch must have the
 * same tree count. */
int authjx_compile_forest(authjx_ctx* ctx, const authjx_tree* trees, uint32_t n_trees, authjx_ruleset** out,
                          int32_t* pattern_status, char* errbuf, size_t errcap);
/* Results per request of the ruleset (1 for authjx_compile). */
uint32_t authjx_ruleset_trees(const authjx_ruleset* rs);
void authjx_free(authjx_ruleset* rs);
uint32_t authjx_ruleset_patterns(const authjx_ruleset* rs);
uint32_t authjx_ruleset_selectors(const authjx_ruleset* rs);
/* Copies the static error text of pattern i ("" when it has none); returns its length. */
size_t authjx_pattern_error(const authjx_ruleset* rs, uint32_t i, char* buf, size_t cap);

/* Evaluate a batch whose documents are already in device memory (HBM).
 *   sets[n_sets]      rulesets; request r uses sets[set_of_req ? set_of_req[r] : 0]
 *   d_set_of_req      device u32[n] (entries < n_sets) or NULL; ignored when n_sets == 1
 *   d_arena           device bytes; document r = d_arena[d_offs[r] .. + d_lens[r]). The
 *                     kernels read whole aligned 32-byte blocks (the streaming kernel's
 *                     unit; the others read 16): every block holding a document byte must
 *                     be readable (device allocations are; an arena carved from a larger
 *                     buffer needs 31 readable bytes after its end)
 *   d_out_tristate    device u8[n * n_trees]  (AUTHJX_F/T/E/UNDECIDED; n_trees = 1 unless
 *                     the rulesets come from authjx_compile_forest)
 *   d_out_err_idx     device i32[n * n_trees] pattern whose error decided an E, else -1
 *                     (may be NULL)
 *   d_out_bitmap      device u64[n * bitmap_stride_words]: bit p = pattern p evaluated to T
 *                     (every pattern evaluated, no short-circuit), may be NULL
 *   stream            hipStream_t (NULL = the context's stream). Asynchronous. */
int authjx_eval_batch_device(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                             const uint32_t* d_set_of_req, const uint8_t* d_arena,
                             const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n,
                             uint8_t* d_out_tristate, int32_t* d_out_err_idx,
                             uint64_t* d_out_bitmap, uint32_t bitmap_stride_words, void* stream);

/* Same, from host buffers: copies to the device, evaluates, copies back; synchronous.
 * This is the entry point a cgo shim's micro-batcher calls. */
int authjx_eval_batch(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                      const uint32_t* set_of_req, const uint8_t* arena, uint64_t arena_len,
                      const uint64_t* offs, const uint32_t* lens, uint32_t n,
                      uint8_t* out_tristate, int32_t* out_err_idx, uint64_t* out_bitmap,
                      uint32_t bitmap_stride_words);

/* gjson.Get(doc, selector) as a span of the document. type is gjson.Type
 * (AUTHJX_JSON_*); start is relative to the document; for strings the span includes the
 * quotes and esc = 1 when the contents hold a backslash escape. A missing path is
 * {0, 0, AUTHJX_JSON_NULL}. AUTHJX_JSON_UNSUPPORTED: the selector uses gjson syntax the
 * device does not compile (its pattern_status is AUTHJX_PAT_UNSUPPORTED). */
#define AUTHJX_JSON_NULL 0
#define AUTHJX_JSON_FALSE 1
#define AUTHJX_JSON_NUMBER 2
#define AUTHJX_JSON_STRING 3
#define AUTHJX_JSON_TRUE 4
#define AUTHJX_JSON_JSON 5
#define AUTHJX_JSON_UNSUPPORTED 255
#define AUTHJX_VALUE_COUNT 2 /* authjx_value.esc: `start` is an array's element count (a
                              * last path part "#", gjson parseArray), len 0: no span */
#define AUTHJX_VALUE_TEXT 4  /* authjx_value.esc flag (with 1 = escapes): the value is built
                              * text — the Result of a modifier chain or a "#." list — at
                              * [start, start + len) of the request's text slot
                              * (authjx_select_text_batch[_device]) */
typedef struct {
    uint32_t start;
    uint32_t len;
    uint8_t type;
    uint8_t esc; /* 1: a string with escapes (gjson unescape applies); AUTHJX_VALUE_COUNT */
    uint16_t reserved;
} authjx_value;

/* Resolve the selector of every pattern of `sets[set_of_req[r]]` (operators and values
 * are ignored; compile the selectors as a tree of AUTHJX_OP_EQ patterns with root -1)
 * for every request: d_out_values[r * values_stride + p], values_stride >= the largest
 * n_patterns. Device buffers, asynchronous on `stream` (NULL = the context's stream). */
int authjx_select_batch_device(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                               const uint32_t* d_set_of_req, const uint8_t* d_arena, const uint64_t* d_offs,
                               const uint32_t* d_lens, uint32_t n, authjx_value* d_out_values,
                               uint32_t values_stride, void* stream);
/* The values of patterns [first_pattern, first_pattern + values_stride) of `rs` from the
 * capture rows the last authjx_eval_batch_device call on this context wrote: that call
 * must have evaluated `rs` alone over the same d_arena / d_offs / d_lens (n requests),
 * without authjx_set_exact_scan, and `rs` must come from authjx_compile_forest (the
 * default kernel keeps capture rows for forests only). For a phase compiled with authjx_compile_forest whose
 * last tree holds the response selectors (AUTHJX_OP_EQ patterns, root -1), this resolves
 * them without a second document scan: the gjson.Get of JSONValue.ResolveFor
 * (pkg/json/json.go:41-53) after the rules of the same request. The patterns must belong
 * to root-less trees of the forest (the kernel writes capture records only for those and
 * for the values its stage B reads). AUTHJX_EINVAL when the rows are not that
 * evaluation's, or a pattern's record is not kept. Asynchronous on `stream`; order it
 * after the eval. */
int authjx_select_from_eval_device(authjx_ctx* ctx, const authjx_ruleset* rs, uint32_t first_pattern,
                                   const uint8_t* d_arena, const uint64_t* d_offs, const uint32_t* d_lens,
                                   uint32_t n, authjx_value* d_out_values, uint32_t values_stride, void* stream);
/* Same from host buffers; synchronous. */
int authjx_select_batch(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                        const uint32_t* set_of_req, const uint8_t* arena, uint64_t arena_len,
                        const uint64_t* offs, const uint32_t* lens, uint32_t n, authjx_value* out_values,
                        uint32_t values_stride);
/* authjx_select_batch[_device] for selectors with gjson modifiers (`a.b|@case:upper`,
 * `@extract:{...}`, ...) and "#." lists: their values are built text, not document spans
 * — the response / denyWith / cache-key templates of pkg/json/json.go:96-151 and
 * pkg/evaluators/authorization.go:56-66. Request r's text slot is
 * out_text[r * text_stride, (r + 1) * text_stride); a value esc has AUTHJX_VALUE_TEXT and
 * start / len within that slot. A value that does not fit, or that the device leaves
 * undecided (@case / @strip on a code point its Unicode tables do not vouch for), is
 * AUTHJX_JSON_UNSUPPORTED. Plain selectors are document spans as above. */
int authjx_select_text_batch_device(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                                    const uint32_t* d_set_of_req, const uint8_t* d_arena, const uint64_t* d_offs,
                                    const uint32_t* d_lens, uint32_t n, authjx_value* d_out_values,
                                    uint32_t values_stride, uint8_t* d_out_text, uint32_t text_stride, void* stream);
int authjx_select_text_batch(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                             const uint32_t* set_of_req, const uint8_t* arena, uint64_t arena_len,
                             const uint64_t* offs, const uint32_t* lens, uint32_t n, authjx_value* out_values,
                             uint32_t values_stride, uint8_t* out_text, uint32_t text_stride);

/* Route every request through the exact per-selector scan kernel instead of the
 * single-pass kernel (results are identical; used to cross-check the two paths). */
int authjx_set_exact_scan(authjx_ctx* ctx, int force);
/* Number of requests of the last batch the single-pass kernel handed to the exact scan
 * (documents it could not prove gjson-equivalent, e.g. not valid JSON). Synchronises. */
int64_t authjx_last_exact_count(authjx_ctx* ctx);

/* Kernel-only timing of the last device call on the context (its stream's events
 * around the launches, ms). */
float authjx_last_kernel_ms(authjx_ctx* ctx);

/* ---- micro-batcher --------------------------------------------------------------
 * Replaces the per-request evaluation made from each request's own goroutine
 * (pkg/service/auth_pipeline.go:150-164 evaluator goroutines; main.go:69,451 up to 10k
 * concurrent streams): callers submit one request each and block; a worker thread
 * flushes a batch when max_batch requests are queued or the oldest has waited
 * window_us, drops requests whose deadline passed (AUTHJX_ETIMEDOUT, not evaluated),
 * orders the rest by ruleset (AuthConfig buckets) and evaluates them with one launch on
 * the batcher's own stream (rulesets of one batch share n_trees; others wait for the
 * next batch). The queue holds at most queue_cap requests (0: 4 * max_batch); a caller
 * waits for room up to its deadline. */
typedef struct authjx_batcher authjx_batcher;
int authjx_batcher_create(authjx_ctx* ctx, uint32_t max_batch, uint32_t window_us, uint32_t queue_cap,
                          authjx_batcher** out);
/* Evaluates what is queued, then stops the worker (callers still waiting for room get
 * AUTHJX_ECLOSED). */
void authjx_batcher_destroy(authjx_batcher* b);
/* Blocking: Expression.Matches of `rs` on one document (copied at batch time; the
 * buffer must stay valid until return). timeout_us: 0 = no deadline. out_tristate /
 * out_err_idx (may be NULL): n_trees entries, as authjx_eval_batch writes them. */
int authjx_batcher_eval(authjx_batcher* b, const authjx_ruleset* rs, const uint8_t* doc, size_t len,
                        uint64_t timeout_us, uint8_t* out_tristate, int32_t* out_err_idx);
int authjx_batcher_stats(authjx_batcher* b, uint64_t* batches, uint64_t* requests, uint64_t* expired,
                         uint64_t* max_batch_seen);

/* ---- AuthConfig index (host) ----------------------------------------------------
 * pkg/index/index.go's authConfigTree (:37-243), native, for the micro-batcher's
 * per-request AuthConfig selection (config C4). Keys are hostnames ('*' labels are
 * wildcards); entries are ruleset ids (the `set_of_req` values of authjx_eval_batch).
 * Set = index.go:67-80 (AUTHJX_EEXIST: "authconfig already exists in the index" when the
 * key is taken and override is 0); DeleteKey = :93-98 (the key's entry is removed only
 * when it is this id's). Lookups take a shared lock, Set/DeleteKey an exclusive one
 * (the reference's RWMutex, :51). */
typedef struct authjx_index authjx_index;
int authjx_index_new(authjx_index** out);
void authjx_index_free(authjx_index* ix);
int authjx_index_set(authjx_index* ix, const char* key, uint32_t key_len, int32_t set_id, int override_);
int authjx_index_delete_key(authjx_index* ix, const char* key, uint32_t key_len, int32_t set_id);
/* Index.Get (index.go:56-65) with the ':port' retry of pkg/service/auth.go:270-280:
 * *out_set = the host's ruleset id, -1 when none (the reference answers NOT_FOUND,
 * auth.go:282-287). */
int authjx_index_get(const authjx_index* ix, const char* host, uint32_t host_len, int32_t* out_set);
/* The same for a micro-batch of hosts (host r = hosts[offs[r] .. offs[r] + lens[r])) on
 * n_threads host threads (0: all cores), each distinct host walked once per thread. */
int authjx_index_lookup_batch(const authjx_index* ix, const uint8_t* hosts, const uint64_t* offs,
                              const uint32_t* lens, uint32_t n, int32_t* out_sets, uint32_t n_threads);

/* ---- Authorization JSON packing (host) -------------------------------------------
 * The producer's output stage (pkg/service/auth_pipeline.go:542-616 GetAuthorizationJSON,
 * json.Marshal per evaluator call in the reference): each request's values, walked once
 * by the caller into a TAPE, are encoded with encoding/json's rules (HTML-safe string
 * escapes, U+2028/U+2029, invalid UTF-8 as \ufffd, map keys sorted by bytes, float64 'f'
 * or 'e' by magnitude) straight into the batch arena that authjx_eval_batch reads.
 * Tape (little-endian), one value:
 *   AUTHJX_TAPE_NULL / TRUE / FALSE
 *   AUTHJX_TAPE_F64 <8 B double>      float64 (NaN / Inf: the request fails, as Marshal does)
 *   AUTHJX_TAPE_I64 <8 B int64>       integer types
 *   AUTHJX_TAPE_STRING <u32 len><bytes>
 *   AUTHJX_TAPE_RAW <u32 len><bytes>  pre-encoded JSON (json.RawMessage), copied
 *   AUTHJX_TAPE_ARRAY <u32 n><n values>
 *   AUTHJX_TAPE_OBJECT <u32 n><n x (<u32 len><key bytes> value)>  a struct: member order kept
 *   AUTHJX_TAPE_MAP <u32 n><same>     a map: members written sorted by key bytes */
#define AUTHJX_TAPE_NULL 1
#define AUTHJX_TAPE_TRUE 2
#define AUTHJX_TAPE_FALSE 3
#define AUTHJX_TAPE_F64 4
#define AUTHJX_TAPE_I64 5
#define AUTHJX_TAPE_STRING 6
#define AUTHJX_TAPE_RAW 7
#define AUTHJX_TAPE_ARRAY 8
#define AUTHJX_TAPE_OBJECT 9
#define AUTHJX_TAPE_MAP 10
/* Request r's tape is tapes[tape_offs[r] .. + tape_lens[r]); its document goes to
 * arena[out_offs[r] .. + out_lens[r]), the documents back to back in request order, on
 * n_threads host threads (0: all cores). *out_total = the bytes the batch needs:
 * AUTHJX_ELIMIT (nothing written) when that exceeds arena_cap; AUTHJX_EINVAL when a
 * tape is malformed or holds a NaN / Inf (that request: out_offs = ~0, out_lens = 0). */
int authjx_pack_json(const uint8_t* tapes, const uint64_t* tape_offs, const uint32_t* tape_lens, uint32_t n,
                     uint8_t* arena, uint64_t arena_cap, uint64_t* out_offs, uint32_t* out_lens,
                     uint64_t* out_total, uint32_t n_threads);

#ifdef __cplusplus
}
#endif
#endif
