// ajx_api.cpp — the C-ABI (include/authjx.h): device contexts, reconcile-time compile
// into HBM-resident rulesets, batch evaluation.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/authjx.h"
#include "ajx_compiler.h"
#include "ajx_blob.h"
#include "ajx_kernels.h"

struct authjx_ruleset {
    int device = 0;
    uint8_t* d_blob = nullptr;
    ajx::CompiledRuleset c;
};

struct authjx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::mutex mu;        // serialises device-side calls on this context (set table)
    std::mutex batch_mu;  // serialises authjx_eval_batch (owns the staging buffer)
    // device set table: pointers to ruleset blobs
    const uint8_t** d_sets = nullptr;
    uint32_t sets_cap = 0;
    std::vector<const uint8_t*> last_sets;
    const uint8_t** h_sets_pinned = nullptr;
    // staging for authjx_eval_batch (host buffers)
    uint8_t* d_stage = nullptr;
    size_t stage_cap = 0;
    // requests the fast kernel hands to the exact scan
    uint32_t* d_slow = nullptr;  // [0] = count, [1..] = ids
    uint32_t slow_cap = 0;
    uint64_t* d_rows = nullptr;  // stage-A capture rows
    size_t rows_cap = 0;         // in u64
    uint32_t* d_perm = nullptr;  // length-bucketed request order (+ 2 x 1024 + 1 u32 histogram)
    uint32_t perm_cap = 0;
    int len_sort = 1;            // order requests by length class before the single-pass kernel
    int no_tenant_stage = 0;     // profiling: multi-tenant batches read tables from global memory
    // the capture rows in d_rows: written by the last single-ruleset, single-pass
    // evaluation of rows_rs over rows_n requests (nullptr: none usable)
    const authjx_ruleset* rows_rs = nullptr;
    uint32_t rows_n = 0, rows_stride = 0;
    int force_scan = 0;
    int ablate = 0;  // profiling only: 1/2/3 reduced single-pass variants, 20 the lane kernel,
                     // 21..24 its ablations (ajx_kernels.hip ajx_lane_eval)
    float last_ms = 0.f;
};

namespace {

#define HIP_OK(x)                                   \
    do {                                            \
        hipError_t e_ = (x);                        \
        if (e_ != hipSuccess) return AUTHJX_EDEVICE; \
    } while (0)

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

int ensure_sets(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets, hipStream_t stream) {
    std::vector<const uint8_t*> ptrs(n_sets);
    for (uint32_t i = 0; i < n_sets; i++) {
        if (!sets[i] || sets[i]->device != ctx->device) return AUTHJX_EINVAL;
        ptrs[i] = sets[i]->d_blob;
    }
    if (ptrs == ctx->last_sets) return AUTHJX_OK;
    if (n_sets > ctx->sets_cap) {
        if (ctx->d_sets) (void)hipFree(ctx->d_sets);
        if (ctx->h_sets_pinned) (void)hipHostFree(ctx->h_sets_pinned);
        ctx->d_sets = nullptr;
        ctx->h_sets_pinned = nullptr;
        uint32_t cap = n_sets < 64 ? 64 : n_sets;
        HIP_OK(hipMalloc(&ctx->d_sets, cap * sizeof(uint8_t*)));
        HIP_OK(hipHostMalloc(&ctx->h_sets_pinned, cap * sizeof(uint8_t*), hipHostMallocDefault));
        ctx->sets_cap = cap;
    }
    // the pinned table may still be read by an in-flight copy of the previous batch
    HIP_OK(hipStreamSynchronize(stream));
    std::memcpy(ctx->h_sets_pinned, ptrs.data(), n_sets * sizeof(uint8_t*));
    HIP_OK(hipMemcpyAsync(ctx->d_sets, ctx->h_sets_pinned, n_sets * sizeof(uint8_t*), hipMemcpyHostToDevice, stream));
    ctx->last_sets = ptrs;
    return AUTHJX_OK;
}

// capture rows, slow list and request order for a batch of n on stream s (grown when
// needed: no batch in flight on this context may still use the old buffers)
int ensure_work(authjx_ctx* ctx, uint32_t n, uint32_t row_stride, hipStream_t s) {
    if (n <= ctx->slow_cap && n <= ctx->perm_cap && (size_t)n * row_stride <= ctx->rows_cap) return AUTHJX_OK;
    HIP_OK(hipStreamSynchronize(s));
    if (n > ctx->slow_cap) {
        if (ctx->d_slow) (void)hipFree(ctx->d_slow);
        ctx->d_slow = nullptr;
        ctx->slow_cap = 0;
        HIP_OK(hipMalloc(&ctx->d_slow, ((size_t)n + 1) * sizeof(uint32_t)));
        ctx->slow_cap = n;
    }
    if (n > ctx->perm_cap) {
        if (ctx->d_perm) (void)hipFree(ctx->d_perm);
        ctx->d_perm = nullptr;
        ctx->perm_cap = 0;
        HIP_OK(hipMalloc(&ctx->d_perm, ((size_t)n + 4096) * sizeof(uint32_t)));
        ctx->perm_cap = n;
    }
    if ((size_t)n * row_stride > ctx->rows_cap) {
        if (ctx->d_rows) (void)hipFree(ctx->d_rows);
        ctx->d_rows = nullptr;
        ctx->rows_cap = 0;
        HIP_OK(hipMalloc(&ctx->d_rows, (size_t)n * row_stride * sizeof(uint64_t)));
        ctx->rows_cap = (size_t)n * row_stride;
    }
    return AUTHJX_OK;
}

}  // namespace

extern "C" {

int authjx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int authjx_init(int device, authjx_ctx** out) {
    if (!out) return AUTHJX_EINVAL;
    *out = nullptr;
    int n = authjx_device_count();
    if (device < 0 || device >= n) return AUTHJX_EDEVICE;
    HIP_OK(hipSetDevice(device));
    authjx_ctx* c = new authjx_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        delete c;
        return AUTHJX_EDEVICE;
    }
    *out = c;
    return AUTHJX_OK;
}

void authjx_shutdown(authjx_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->d_sets) (void)hipFree(ctx->d_sets);
    if (ctx->h_sets_pinned) (void)hipHostFree(ctx->h_sets_pinned);
    if (ctx->d_stage) (void)hipFree(ctx->d_stage);
    if (ctx->d_slow) (void)hipFree(ctx->d_slow);
    if (ctx->d_rows) (void)hipFree(ctx->d_rows);
    if (ctx->d_perm) (void)hipFree(ctx->d_perm);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

namespace {
int finish_compile(authjx_ctx* ctx, authjx_ruleset* rs, int rc, const std::string& err, authjx_ruleset** out,
                   int32_t* pattern_status, char* errbuf, size_t errcap);
}

int authjx_compile(authjx_ctx* ctx, const authjx_tree* tree, authjx_ruleset** out, int32_t* pattern_status,
                   char* errbuf, size_t errcap) {
    if (!ctx || !tree || !out) return AUTHJX_EINVAL;
    *out = nullptr;
    authjx_ruleset* rs = new authjx_ruleset();
    std::string err;
    int rc = ajx::compile_tree(tree, &rs->c, &err);
    return finish_compile(ctx, rs, rc, err, out, pattern_status, errbuf, errcap);
}

int authjx_compile_forest(authjx_ctx* ctx, const authjx_tree* trees, uint32_t n_trees, authjx_ruleset** out,
                          int32_t* pattern_status, char* errbuf, size_t errcap) {
    if (!ctx || !trees || !n_trees || !out) return AUTHJX_EINVAL;
    *out = nullptr;
    authjx_ruleset* rs = new authjx_ruleset();
    std::string err;
    int rc = ajx::compile_forest(trees, n_trees, &rs->c, &err);
    return finish_compile(ctx, rs, rc, err, out, pattern_status, errbuf, errcap);
}

uint32_t authjx_ruleset_trees(const authjx_ruleset* rs) { return rs ? rs->c.n_trees : 0; }

namespace {
int finish_compile(authjx_ctx* ctx, authjx_ruleset* rs, int rc, const std::string& err, authjx_ruleset** out,
                   int32_t* pattern_status, char* errbuf, size_t errcap) {
    if (errbuf && errcap) std::snprintf(errbuf, errcap, "%s", err.c_str());
    if (rc != AUTHJX_OK) {
        delete rs;
        return rc;
    }
    if (pattern_status)
        for (uint32_t i = 0; i < rs->c.n_patterns; i++) pattern_status[i] = rs->c.pattern_status[i];
    rs->device = ctx->device;
    if (hipSetDevice(ctx->device) != hipSuccess ||
        hipMalloc(&rs->d_blob, rs->c.blob.size()) != hipSuccess ||
        hipMemcpy(rs->d_blob, rs->c.blob.data(), rs->c.blob.size(), hipMemcpyHostToDevice) != hipSuccess) {
        if (rs->d_blob) (void)hipFree(rs->d_blob);
        delete rs;
        return AUTHJX_EDEVICE;
    }
    *out = rs;
    return AUTHJX_OK;
}
}  // namespace

void authjx_free(authjx_ruleset* rs) {
    if (!rs) return;
    if (rs->d_blob) {
        (void)hipSetDevice(rs->device);
        (void)hipDeviceSynchronize();  // no batch may still read the blob
        (void)hipFree(rs->d_blob);
    }
    delete rs;
}

uint32_t authjx_ruleset_patterns(const authjx_ruleset* rs) { return rs ? rs->c.n_patterns : 0; }
uint32_t authjx_ruleset_selectors(const authjx_ruleset* rs) { return rs ? rs->c.n_selectors : 0; }

size_t authjx_pattern_error(const authjx_ruleset* rs, uint32_t i, char* buf, size_t cap) {
    if (!rs || i >= rs->c.n_patterns) return 0;
    const std::string& e = rs->c.pattern_error[i];
    if (buf && cap) std::snprintf(buf, cap, "%s", e.c_str());
    return e.size();
}

int authjx_eval_batch_device(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                             const uint32_t* d_set_of_req, const uint8_t* d_arena, const uint64_t* d_offs,
                             const uint32_t* d_lens, uint32_t n, uint8_t* d_out_tristate, int32_t* d_out_err_idx,
                             uint64_t* d_out_bitmap, uint32_t bitmap_stride_words, void* stream) {
    if (!ctx || !sets || n_sets == 0 || (n && (!d_arena || !d_offs || !d_lens || !d_out_tristate)))
        return AUTHJX_EINVAL;
    if (n_sets > 1 && !d_set_of_req) return AUTHJX_EINVAL;
    if (n_sets == 1) d_set_of_req = nullptr;  // every request uses sets[0] (uniform-ruleset kernels)
    uint32_t need_words = 0, max_sel = 0;
    for (uint32_t i = 0; i < n_sets; i++) {
        if (!sets[i] || sets[i]->c.n_trees != sets[0]->c.n_trees) return AUTHJX_EINVAL;
        uint32_t w = (sets[i]->c.n_patterns + 63) / 64;
        if (w > need_words) need_words = w;
        if (sets[i]->c.n_selectors > max_sel) max_sel = sets[i]->c.n_selectors;
    }
    const uint32_t row_stride = 1 + max_sel;
    if (d_out_bitmap && bitmap_stride_words < need_words) return AUTHJX_EINVAL;
    std::lock_guard<std::mutex> lock(ctx->mu);
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    HIP_OK(hipSetDevice(ctx->device));
    int rc = ensure_sets(ctx, sets, n_sets, s);
    if (rc != AUTHJX_OK) return rc;
    if (!ctx->force_scan) {
        rc = ensure_work(ctx, n, row_stride, s);
        if (rc != AUTHJX_OK) return rc;
    }
    HIP_OK(hipEventRecord(ctx->ev0, s));
    // kernel: the single-pass kernel (default; ajx_scan_fused); ablate 20 the lane
    // kernel (21..24 its ablations), 1..3 single-pass ablations
    bool fast_tables = !ctx->force_scan;
    for (uint32_t i = 0; i < n_sets && fast_tables; i++)
        fast_tables = (reinterpret_cast<const ajx::RulesetHdr*>(sets[i]->c.blob.data())->flags & ajx::kFlagFastOk) != 0;
    const bool lane = fast_tables && ctx->ablate >= 20;
    // capture rows kept for authjx_select_from_eval_device: one ruleset, a full kernel
    const bool full = ctx->ablate == 0 || ctx->ablate == 20;
    const bool keep_rows = !ctx->force_scan && n_sets == 1 && full;
    ctx->rows_rs = keep_rows ? sets[0] : nullptr;
    ctx->rows_n = n;
    ctx->rows_stride = row_stride;
    size_t max_blob = 0;
    for (uint32_t i = 0; i < n_sets; i++) max_blob = std::max(max_blob, sets[i]->c.blob.size());
    if (ctx->force_scan) {
        HIP_OK(ajx::launch_eval_scan(ctx->d_sets, d_set_of_req, d_arena, d_offs, d_lens, n, d_out_tristate,
                                     d_out_err_idx, d_out_bitmap, bitmap_stride_words, s));
    } else {
        // length-bucketed order: one ruleset for the batch (multi-tenant batches keep the
        // caller's bucketing by AuthConfig), a full kernel, batches worth sorting
        const uint32_t* perm = nullptr;
        if (ctx->len_sort && (n_sets == 1 || ctx->len_sort > 1) && full && n >= 4096) {
            HIP_OK(ajx::launch_len_order(d_lens, n, ctx->d_perm + n, ctx->d_perm, s));
            perm = ctx->d_perm;
        }
        if (lane) {
            const uint32_t stage_bytes =
                n_sets == 1 && max_blob <= ajx::kMaxSharedBlobBytes ? (uint32_t)max_blob : 0u;
            HIP_OK(ajx::launch_eval_lane(ctx->d_sets, d_set_of_req, stage_bytes, d_arena, d_offs, d_lens, n,
                                         d_out_tristate, d_out_err_idx, d_out_bitmap, bitmap_stride_words,
                                         ctx->d_rows, row_stride, ctx->d_slow, ctx->d_slow + 1, s,
                                         ctx->ablate - 20, perm));
        } else {
            // uniform batch: the blob staged once per workgroup; multi-tenant batch: the
            // largest blob, for workgroups whose requests share one ruleset
            // (ajx_scan_fused_tenant)
            const uint32_t stage_bytes =
                n_sets == 1 ? (max_blob <= ajx::kMaxSharedBlobBytes ? (uint32_t)max_blob : 0u)
                            : (!ctx->no_tenant_stage && max_blob <= ajx::kMaxTenantStageBytes ? (uint32_t)max_blob
                                                                                              : 0u);
            HIP_OK(ajx::launch_eval_fast(ctx->d_sets, d_set_of_req, stage_bytes, d_arena, d_offs, d_lens, n,
                                         d_out_tristate, d_out_err_idx, d_out_bitmap, bitmap_stride_words,
                                         ctx->d_rows, row_stride, ctx->d_slow, ctx->d_slow + 1, s,
                                         ctx->ablate < 20 ? ctx->ablate : 0, perm));
        }
    }
    HIP_OK(hipEventRecord(ctx->ev1, s));
    return AUTHJX_OK;
}

static_assert(sizeof(authjx_value) == 12, "authjx_value is three u32 words on the device");

int authjx_select_batch_device(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                               const uint32_t* d_set_of_req, const uint8_t* d_arena, const uint64_t* d_offs,
                               const uint32_t* d_lens, uint32_t n, authjx_value* d_out_values,
                               uint32_t values_stride, void* stream) {
    if (!ctx || !sets || n_sets == 0 || (n && (!d_arena || !d_offs || !d_lens || !d_out_values)))
        return AUTHJX_EINVAL;
    if (n_sets > 1 && !d_set_of_req) return AUTHJX_EINVAL;
    if (n_sets == 1) d_set_of_req = nullptr;
    uint32_t max_sel = 0;
    for (uint32_t i = 0; i < n_sets; i++) {
        if (!sets[i] || sets[i]->c.n_patterns > values_stride) return AUTHJX_EINVAL;
        if (sets[i]->c.n_selectors > max_sel) max_sel = sets[i]->c.n_selectors;
    }
    const uint32_t row_stride = 1 + max_sel;
    std::lock_guard<std::mutex> lock(ctx->mu);
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    HIP_OK(hipSetDevice(ctx->device));
    int rc = ensure_sets(ctx, sets, n_sets, s);
    if (rc != AUTHJX_OK) return rc;
    const bool exact = ctx->force_scan != 0;  // the exact Get per selector (cross-check)
    ctx->rows_rs = nullptr;  // (the rows are rewritten for this ruleset)
    if (!exact && (rc = ensure_work(ctx, n, row_stride, s)) != AUTHJX_OK) return rc;
    const uint32_t* perm = nullptr;
    if (!exact && ctx->len_sort && n_sets == 1 && n >= 4096) {
        HIP_OK(ajx::launch_len_order(d_lens, n, ctx->d_perm + n, ctx->d_perm, s));
        perm = ctx->d_perm;
    }
    const uint32_t shared_bytes =
        (n_sets == 1 && sets[0]->c.blob.size() <= ajx::kMaxSharedBlobBytes) ? (uint32_t)sets[0]->c.blob.size() : 0u;
    HIP_OK(ajx::launch_select(ctx->d_sets, d_set_of_req, shared_bytes, d_arena, d_offs, d_lens, n,
                              reinterpret_cast<uint32_t*>(d_out_values), values_stride,
                              exact ? nullptr : ctx->d_rows, row_stride, ctx->d_slow, ctx->d_slow + 1, perm, s));
    return AUTHJX_OK;
}

int authjx_select_from_eval_device(authjx_ctx* ctx, const authjx_ruleset* rs, uint32_t first_pattern,
                                   const uint8_t* d_arena, const uint64_t* d_offs, const uint32_t* d_lens,
                                   uint32_t n, authjx_value* d_out_values, uint32_t values_stride, void* stream) {
    if (!ctx || !rs || values_stride == 0 || (n && (!d_arena || !d_offs || !d_lens || !d_out_values)))
        return AUTHJX_EINVAL;
    if (first_pattern + values_stride > rs->c.n_patterns) return AUTHJX_EINVAL;
    std::lock_guard<std::mutex> lock(ctx->mu);
    // the rows must be the last evaluation's, of this ruleset, over this many requests
    if (ctx->rows_rs != rs || ctx->rows_n != n) return AUTHJX_EINVAL;
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    HIP_OK(hipSetDevice(ctx->device));
    const authjx_ruleset* one[1] = {rs};
    int rc = ensure_sets(ctx, one, 1, s);
    if (rc != AUTHJX_OK) return rc;
    HIP_OK(ajx::launch_select_rows(ctx->d_sets, d_arena, d_offs, d_lens, n, reinterpret_cast<uint32_t*>(d_out_values),
                                   values_stride, ctx->d_rows, ctx->rows_stride, first_pattern, s));
    return AUTHJX_OK;
}

int authjx_select_batch(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                        const uint32_t* set_of_req, const uint8_t* arena, uint64_t arena_len,
                        const uint64_t* offs, const uint32_t* lens, uint32_t n, authjx_value* out_values,
                        uint32_t values_stride) {
    if (!ctx || (n && (!arena || !offs || !lens || !out_values))) return AUTHJX_EINVAL;
    for (uint32_t r = 0; r < n; r++)
        if (offs[r] + lens[r] > arena_len) return AUTHJX_EINVAL;
    const bool with_sor = set_of_req != nullptr;
    const size_t o_offs = round_up(arena_len, 256);
    const size_t o_lens = round_up(o_offs + (size_t)n * 8, 256);
    const size_t o_sor = round_up(o_lens + (size_t)n * 4, 256);
    const size_t o_out = round_up(o_sor + (with_sor ? (size_t)n * 4 : 0), 256);
    const size_t out_bytes = (size_t)n * values_stride * sizeof(authjx_value);
    const size_t total = round_up(o_out + out_bytes, 256);
    std::lock_guard<std::mutex> batch_lock(ctx->batch_mu);
    {
        std::lock_guard<std::mutex> lock(ctx->mu);
        HIP_OK(hipSetDevice(ctx->device));
        if (total > ctx->stage_cap) {
            HIP_OK(hipStreamSynchronize(ctx->stream));
            if (ctx->d_stage) (void)hipFree(ctx->d_stage);
            ctx->d_stage = nullptr;
            ctx->stage_cap = 0;
            HIP_OK(hipMalloc(&ctx->d_stage, total));
            ctx->stage_cap = total;
        }
        uint8_t* b = ctx->d_stage;
        hipStream_t s = ctx->stream;
        HIP_OK(hipMemcpyAsync(b, arena, arena_len, hipMemcpyHostToDevice, s));
        HIP_OK(hipMemcpyAsync(b + o_offs, offs, (size_t)n * 8, hipMemcpyHostToDevice, s));
        HIP_OK(hipMemcpyAsync(b + o_lens, lens, (size_t)n * 4, hipMemcpyHostToDevice, s));
        if (with_sor) HIP_OK(hipMemcpyAsync(b + o_sor, set_of_req, (size_t)n * 4, hipMemcpyHostToDevice, s));
    }
    uint8_t* b = ctx->d_stage;
    int rc = authjx_select_batch_device(ctx, sets, n_sets, with_sor ? (const uint32_t*)(b + o_sor) : nullptr, b,
                                        (const uint64_t*)(b + o_offs), (const uint32_t*)(b + o_lens), n,
                                        (authjx_value*)(b + o_out), values_stride, nullptr);
    if (rc != AUTHJX_OK) return rc;
    std::lock_guard<std::mutex> lock(ctx->mu);
    HIP_OK(hipMemcpyAsync(out_values, b + o_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
    return AUTHJX_OK;
}

// Profiling only (not in authjx.h): replace stage A by a reduced variant whose outputs
// are meaningless, to price its parts (loads, classification) on the hardware.
int authjx_debug_ablate(authjx_ctx* ctx, int mode) {
    if (!ctx) return AUTHJX_EINVAL;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->ablate = mode;
    return AUTHJX_OK;
}


// Profiling only (not in authjx.h): the length-bucketed request order off (0), for
// single-ruleset batches (1, default) or for every batch (2).
int authjx_debug_len_sort(authjx_ctx* ctx, int on) {
    if (!ctx) return AUTHJX_EINVAL;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->len_sort = on;  // 0 off, 1 single-ruleset batches, 2 also multi-tenant batches
    return AUTHJX_OK;
}

// Profiling only (not in authjx.h): workgroup-uniform LDS staging of multi-tenant
// rulesets on (1, default) or off (0: every table read from global memory).
int authjx_debug_tenant_stage(authjx_ctx* ctx, int on) {
    if (!ctx) return AUTHJX_EINVAL;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->no_tenant_stage = on ? 0 : 1;
    return AUTHJX_OK;
}

int authjx_set_exact_scan(authjx_ctx* ctx, int force) {
    if (!ctx) return AUTHJX_EINVAL;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->force_scan = force ? 1 : 0;
    return AUTHJX_OK;
}

int64_t authjx_last_exact_count(authjx_ctx* ctx) {
    if (!ctx) return AUTHJX_EINVAL;
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (ctx->force_scan || !ctx->d_slow) return -1;
    uint32_t c = 0;
    if (hipSetDevice(ctx->device) != hipSuccess || hipEventSynchronize(ctx->ev1) != hipSuccess ||
        hipMemcpy(&c, ctx->d_slow, sizeof c, hipMemcpyDeviceToHost) != hipSuccess)
        return AUTHJX_EDEVICE;
    return (int64_t)c;
}

float authjx_last_kernel_ms(authjx_ctx* ctx) {
    if (!ctx) return 0.f;
    float ms = 0.f;
    if (hipEventSynchronize(ctx->ev1) != hipSuccess) return 0.f;
    if (hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) != hipSuccess) return 0.f;
    return ms;
}

int authjx_eval_batch(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                      const uint32_t* set_of_req, const uint8_t* arena, uint64_t arena_len, const uint64_t* offs,
                      const uint32_t* lens, uint32_t n, uint8_t* out_tristate, int32_t* out_err_idx,
                      uint64_t* out_bitmap, uint32_t bitmap_stride_words) {
    if (!ctx || (n && (!arena || !offs || !lens || !out_tristate))) return AUTHJX_EINVAL;
    for (uint32_t r = 0; r < n; r++)
        if (offs[r] + lens[r] > arena_len) return AUTHJX_EINVAL;
    const bool with_sor = set_of_req != nullptr;
    if (!sets || n_sets == 0 || !sets[0]) return AUTHJX_EINVAL;
    const size_t nt = sets[0]->c.n_trees;  // results per request
    size_t o_arena = 0;
    size_t o_offs = round_up(o_arena + arena_len, 256);
    size_t o_lens = round_up(o_offs + (size_t)n * 8, 256);
    size_t o_sor = round_up(o_lens + (size_t)n * 4, 256);
    size_t o_tri = round_up(o_sor + (with_sor ? (size_t)n * 4 : 0), 256);
    size_t o_err = round_up(o_tri + (size_t)n * nt, 256);
    size_t o_bm = round_up(o_err + (size_t)n * nt * 4, 256);
    size_t total = round_up(o_bm + (out_bitmap ? (size_t)n * bitmap_stride_words * 8 : 0), 256);
    std::lock_guard<std::mutex> batch_lock(ctx->batch_mu);
    {
        std::lock_guard<std::mutex> lock(ctx->mu);
        HIP_OK(hipSetDevice(ctx->device));
        if (total > ctx->stage_cap) {
            if (ctx->d_stage) (void)hipFree(ctx->d_stage);
            ctx->d_stage = nullptr;
            ctx->stage_cap = 0;
            HIP_OK(hipMalloc(&ctx->d_stage, total));
            ctx->stage_cap = total;
        }
        uint8_t* b = ctx->d_stage;
        hipStream_t s = ctx->stream;
        HIP_OK(hipMemcpyAsync(b + o_arena, arena, arena_len, hipMemcpyHostToDevice, s));
        HIP_OK(hipMemcpyAsync(b + o_offs, offs, (size_t)n * 8, hipMemcpyHostToDevice, s));
        HIP_OK(hipMemcpyAsync(b + o_lens, lens, (size_t)n * 4, hipMemcpyHostToDevice, s));
        if (with_sor) HIP_OK(hipMemcpyAsync(b + o_sor, set_of_req, (size_t)n * 4, hipMemcpyHostToDevice, s));
    }
    uint8_t* b = ctx->d_stage;
    int rc = authjx_eval_batch_device(ctx, sets, n_sets, with_sor ? (const uint32_t*)(b + o_sor) : nullptr,
                                      b + o_arena, (const uint64_t*)(b + o_offs), (const uint32_t*)(b + o_lens), n,
                                      b + o_tri, out_err_idx ? (int32_t*)(b + o_err) : nullptr,
                                      out_bitmap ? (uint64_t*)(b + o_bm) : nullptr, bitmap_stride_words, nullptr);
    if (rc != AUTHJX_OK) return rc;
    std::lock_guard<std::mutex> lock(ctx->mu);
    hipStream_t s = ctx->stream;
    HIP_OK(hipMemcpyAsync(out_tristate, b + o_tri, (size_t)n * nt, hipMemcpyDeviceToHost, s));
    if (out_err_idx) HIP_OK(hipMemcpyAsync(out_err_idx, b + o_err, (size_t)n * nt * 4, hipMemcpyDeviceToHost, s));
    if (out_bitmap)
        HIP_OK(hipMemcpyAsync(out_bitmap, b + o_bm, (size_t)n * bitmap_stride_words * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return AUTHJX_OK;
}

}  // extern "C"
