// ajx_api.cpp — the C-ABI (include/authjx.h): device contexts, reconcile-time compile
// into HBM-resident rulesets, batch evaluation.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/authjx.h"
#include "ajx_compiler.h"
#include "ajx_blob.h"
#include "ajx_kernels.h"
#include "ajx_batcher.h"

struct authjx_ruleset {
    int device = 0;
    uint8_t* d_blob = nullptr;
    ajx::CompiledRuleset c;
    bool stream_ok = false;  // the streaming kernel takes it (ajx::stream_eligible)
    uint32_t stream_rec = 0;  // its capture records there (ajx::stream_records)
    // workspaces (by registry id) whose stream has run a batch over this ruleset:
    // authjx_free waits for their last batch instead of the whole device
    std::mutex mu;
    std::vector<uint64_t> users;
    void note_use(uint64_t ws_id) {
        std::lock_guard<std::mutex> lock(mu);
        if (std::find(users.begin(), users.end(), ws_id) == users.end()) users.push_back(ws_id);
    }
};

// The end-of-batch event of a workspace, shared with the registry (authjx_free waits on
// it outside any lock): destroyed when the last holder lets go.
struct EndEvent {
    hipEvent_t ev = nullptr;
    ~EndEvent() {
        if (ev) (void)hipEventDestroy(ev);
    }
};

// Per-stream scratch of a context: every distinct stream a context is called with gets
// its own set table, slow list, capture rows and request order, so batches on two
// streams of one context never share a buffer; calls on one stream take its mutex
// (their kernels are ordered by the stream anyway).
//
// Lifetime: every user (a call through WsLock, the last_* readers) holds a reference,
// taken and dropped under ctx->mu. Releasing the stream (authjx_release_stream, a
// batcher's private streams) retires the workspace: it leaves ctx->ws and ctx->last_ws at
// once, and whoever drops the last reference destroys it.
struct Workspace {
    hipStream_t stream = nullptr;
    uint64_t id = 0;  // registry id (ruleset users)
    uint32_t refs = 0;     // (ctx->mu)
    bool retired = false;  // (ctx->mu)
    std::mutex mu;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;  // ev1: end of the last batch on this stream
    std::shared_ptr<EndEvent> end;            // owns ev1
    // the ruleset pointer table the kernels index by set_of_req: two slots (device + pinned
    // source each), so a batch over another ruleset list fills the slot the batch before
    // the last one used (its event, not a stream synchronize, guards the reuse)
    const uint8_t** d_sets = nullptr;  // the current slot's device table
    const uint8_t** d_sets_base = nullptr;
    const uint8_t** h_sets_base = nullptr;
    uint32_t sets_cap = 0;  // entries per slot
    uint32_t sets_slot = 0;
    hipEvent_t sets_ev[2] = {nullptr, nullptr};
    bool sets_ev_rec[2] = {false, false};
    std::vector<const uint8_t*> last_sets;
    // [0] = count, [1..] = ids: requests for the exact scan (the streaming kernel: [1] its
    // stage-B count, [2] its finished waves, ids from [3])
    uint32_t* d_slow = nullptr;
    uint32_t slow_cap = 0;
    // the streaming kernel's small-batch instance (FIN) leaves [0..2] zero for the next launch
    // on this stream (no fill) and publishes its exact-path count at [3]
    bool cnt_zero = false, exact3 = false;
    uint64_t* d_rows = nullptr;  // stage-A capture rows
    size_t rows_cap = 0;         // in u64
    // length-bucketed request order: perm [n] | histogram (2 x 1024 + 1 u32, in 4096) |
    // pos_of [n] (each request's work-item)
    uint32_t* d_perm = nullptr;
    uint32_t perm_cap = 0;
    uint8_t* d_tout = nullptr;  // the lean kernel's outputs in work-item order (tout_bytes)
    size_t tout_cap = 0;
    // the capture rows in d_rows: written by the last single-ruleset, full evaluation of
    // rows_rs over rows_n requests on this stream (nullptr: none usable)
    const authjx_ruleset* rows_rs = nullptr;
    uint32_t rows_n = 0, rows_stride = 0;
    const uint32_t* rows_perm = nullptr;  // that evaluation's work-item order (d_perm or none)
    bool rows_wave = false;               // rows in the fused kernels' wave-interleaved layout
    bool ran = false;  // ev0 / ev1 recorded
};

namespace {
// live workspaces: id -> end-of-last-batch event; authjx_free looks its ruleset's users
// up here (an id that is gone belongs to a workspace already destroyed)
std::mutex g_reg_mu;
std::vector<std::pair<uint64_t, std::shared_ptr<EndEvent>>> g_reg;
uint64_t g_next_ws = 1;
}  // namespace

struct authjx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;  // the context's own stream (host-buffer entry points)
    std::mutex mu;                 // workspace list and settings
    std::mutex batch_mu;           // serialises the host-buffer entry points (staging buffer)
    std::vector<Workspace*> ws;
    Workspace* last_ws = nullptr;  // of the last device call (last_kernel_ms / last_exact_count)
    std::vector<authjx_batcher*> batchers;  // alive on this context (shutdown destroys them first)
    // staging for the host-buffer entry points
    uint8_t* d_stage = nullptr;
    size_t stage_cap = 0;
    int len_sort = 1;         // order requests by length class before the single-pass kernel
    int no_tenant_stage = 0;  // profiling: multi-tenant batches read tables from global memory
    int force_scan = 0;
    // batches of up to this many requests go to the streaming kernel (latency: several
    // waves per document span), larger ones to the lean / multi-tenant kernels
    uint32_t stream_max_n = 4096;
    int ablate = 0;  // profiling / comparison only: 41 the lean single-pass kernel where the
                     // streaming kernel would run, 52 the streaming kernel for a one-ruleset
                     // batch of any size, 50 / 51 its structural pass alone / without its
                     // fold, 53 its small-batch phase clocks (over the bitmap), 1..3 /
                     // 10..12 token-scanner ablations and workgroup sizes
};

namespace {

// the last HIP error an entry point returned AUTHJX_EDEVICE for, on this thread
// (authjx_debug_last_error); the runtime's own last-error slot is cleared, so the caller's
// next HIP call does not report it again
thread_local hipError_t t_last_hip = hipSuccess;
thread_local int t_last_line = 0;

#define HIP_OK(x)                  \
    do {                           \
        hipError_t e_ = (x);       \
        if (e_ != hipSuccess) {    \
            t_last_hip = e_;       \
            t_last_line = __LINE__; \
            (void)hipGetLastError(); \
            return AUTHJX_EDEVICE; \
        }                          \
    } while (0)

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// the workspace of stream s (created on first use); ctx->mu held by the caller
Workspace* workspace_of(authjx_ctx* ctx, hipStream_t s) {
    for (Workspace* w : ctx->ws)
        if (w->stream == s) return w;
    Workspace* w = new Workspace();
    w->stream = s;
    w->end = std::make_shared<EndEvent>();
    if (hipEventCreate(&w->ev0) != hipSuccess || hipEventCreate(&w->end->ev) != hipSuccess) {
        if (w->ev0) (void)hipEventDestroy(w->ev0);
        delete w;
        return nullptr;
    }
    w->ev1 = w->end->ev;
    {
        std::lock_guard<std::mutex> lock(g_reg_mu);
        w->id = g_next_ws++;
        g_reg.push_back({w->id, w->end});
    }
    ctx->ws.push_back(w);
    return w;
}

void destroy_workspace(Workspace* w) {
    if (w->ran) (void)hipEventSynchronize(w->ev1);
    {
        std::lock_guard<std::mutex> lock(g_reg_mu);
        for (size_t i = 0; i < g_reg.size(); i++)
            if (g_reg[i].first == w->id) {
                g_reg.erase(g_reg.begin() + (long)i);
                break;
            }
    }
    if (w->d_sets_base) (void)hipFree(w->d_sets_base);
    if (w->h_sets_base) (void)hipHostFree(w->h_sets_base);
    for (int k = 0; k < 2; k++)
        if (w->sets_ev[k]) (void)hipEventDestroy(w->sets_ev[k]);
    if (w->d_slow) (void)hipFree(w->d_slow);
    if (w->d_rows) (void)hipFree(w->d_rows);
    if (w->d_perm) (void)hipFree(w->d_perm);
    if (w->d_tout) (void)hipFree(w->d_tout);
    if (w->ev0) (void)hipEventDestroy(w->ev0);
    delete w;  // (ev1 goes with the last holder of w->end)
}

// a reference to w (ctx->mu held by the caller)
Workspace* ws_ref(Workspace* w) {
    if (w) w->refs++;
    return w;
}
// drops a reference; the last one of a retired workspace destroys it
void ws_unref(authjx_ctx* ctx, Workspace* w) {
    bool dead;
    {
        std::lock_guard<std::mutex> g(ctx->mu);
        dead = --w->refs == 0 && w->retired;
    }
    if (dead) destroy_workspace(w);  // (waits for the stream's last batch)
}

// retires the workspace of stream s (the caller holds no lock)
void retire_stream(authjx_ctx* ctx, hipStream_t s) {
    Workspace* w = nullptr;
    bool dead = false;
    {
        std::lock_guard<std::mutex> g(ctx->mu);
        for (size_t i = 0; i < ctx->ws.size(); i++)
            if (ctx->ws[i]->stream == s) {
                w = ctx->ws[i];
                ctx->ws.erase(ctx->ws.begin() + (long)i);
                if (ctx->last_ws == w) ctx->last_ws = nullptr;
                w->retired = true;
                dead = w->refs == 0;
                break;
            }
    }
    if (dead) destroy_workspace(w);  // (else the call still on that stream does, when it ends)
}

// d_pre: the caller's device copy of the blob pointers (the micro-batcher's staging buffer,
// one copy with the documents), used as is
int ensure_sets(Workspace* w, int device, const authjx_ruleset* const* sets, uint32_t n_sets,
                const uint8_t* const* d_pre = nullptr) {
    std::vector<const uint8_t*> ptrs(n_sets);
    for (uint32_t i = 0; i < n_sets; i++) {
        if (!sets[i] || sets[i]->device != device) return AUTHJX_EINVAL;
        ptrs[i] = sets[i]->d_blob;
    }
    if (d_pre) {
        w->d_sets = const_cast<const uint8_t**>(d_pre);
        w->last_sets.clear();  // (the next call without one copies its table again)
        return AUTHJX_OK;
    }
    if (ptrs == w->last_sets) return AUTHJX_OK;
    if (n_sets > w->sets_cap) {  // (grows: the stream's previous batches may read the old table)
        HIP_OK(hipStreamSynchronize(w->stream));
        if (w->d_sets_base) (void)hipFree(w->d_sets_base);
        if (w->h_sets_base) (void)hipHostFree(w->h_sets_base);
        w->d_sets_base = nullptr;
        w->h_sets_base = nullptr;
        w->d_sets = nullptr;
        w->sets_cap = 0;
        w->sets_ev_rec[0] = w->sets_ev_rec[1] = false;
        uint32_t cap = n_sets < 64 ? 64 : n_sets;
        HIP_OK(hipMalloc(&w->d_sets_base, 2 * cap * sizeof(uint8_t*)));
        HIP_OK(hipHostMalloc(&w->h_sets_base, 2 * cap * sizeof(uint8_t*), hipHostMallocDefault));
        for (int k = 0; k < 2; k++)
            if (!w->sets_ev[k]) HIP_OK(hipEventCreateWithFlags(&w->sets_ev[k], hipEventDisableTiming));
        w->sets_cap = cap;
    }
    // the other slot: free once the last batch that used it has finished
    const uint32_t k = w->d_sets ? 1u - w->sets_slot : 0u;
    if (w->sets_ev_rec[k]) HIP_OK(hipEventSynchronize(w->sets_ev[k]));
    const uint8_t** h = w->h_sets_base + (size_t)k * w->sets_cap;
    const uint8_t** dv = w->d_sets_base + (size_t)k * w->sets_cap;
    std::memcpy(h, ptrs.data(), n_sets * sizeof(uint8_t*));
    HIP_OK(hipMemcpyAsync(dv, h, n_sets * sizeof(uint8_t*), hipMemcpyHostToDevice, w->stream));
    w->sets_slot = k;
    w->d_sets = dv;
    w->last_sets = ptrs;
    return AUTHJX_OK;
}

// capture rows, slow list and request order for a batch of n (grown when needed, after
// this stream's earlier batches are done with the old buffers)
int ensure_work(Workspace* w, uint32_t n, uint32_t row_stride) {
    // (rows for whole waves: the fused kernels' wave-interleaved layout)
    const size_t rows_need = (size_t)((n + 63u) & ~63u) * row_stride;
    if (n <= w->slow_cap && n <= w->perm_cap && rows_need <= w->rows_cap) return AUTHJX_OK;
    HIP_OK(hipStreamSynchronize(w->stream));
    w->rows_rs = nullptr;
    if (n > w->slow_cap) {
        if (w->d_slow) (void)hipFree(w->d_slow);
        w->d_slow = nullptr;
        w->slow_cap = 0;
        HIP_OK(hipMalloc(&w->d_slow, ((size_t)n + 4) * sizeof(uint32_t)));
        w->slow_cap = n;
        w->cnt_zero = w->exact3 = false;
    }
    if (n > w->perm_cap) {
        if (w->d_perm) (void)hipFree(w->d_perm);
        w->d_perm = nullptr;
        w->perm_cap = 0;
        HIP_OK(hipMalloc(&w->d_perm, (2 * (size_t)n + 4096) * sizeof(uint32_t)));
        w->perm_cap = n;
    }
    if (rows_need > w->rows_cap) {
        if (w->d_rows) (void)hipFree(w->d_rows);
        w->d_rows = nullptr;
        w->rows_cap = 0;
        HIP_OK(hipMalloc(&w->d_rows, rows_need * sizeof(uint64_t)));
        w->rows_cap = rows_need;
    }
    return AUTHJX_OK;
}

// room for the lean kernel's work-item-ordered outputs (grown as ensure_work grows)
int ensure_tout(Workspace* w, size_t bytes) {
    if (bytes <= w->tout_cap) return AUTHJX_OK;
    HIP_OK(hipStreamSynchronize(w->stream));
    if (w->d_tout) (void)hipFree(w->d_tout);
    w->d_tout = nullptr;
    w->tout_cap = 0;
    HIP_OK(hipMalloc(&w->d_tout, bytes));
    w->tout_cap = bytes;
    return AUTHJX_OK;
}

// a device call's workspace, locked: ctx->mu only while the workspace is looked up, not
// while waiting for a busy stream's workspace (calls on the context's other streams, the
// batcher's workers among them, go on meanwhile). The reference taken with the lookup keeps
// the workspace alive while this call waits for its mutex, even if its stream is released
// meanwhile. Lock order: w->mu before ctx->mu.
struct WsLock {
    authjx_ctx* ctx;
    Workspace* w = nullptr;
    std::unique_lock<std::mutex> lock;
    WsLock(authjx_ctx* c, void* stream) : ctx(c) {
        {
            std::lock_guard<std::mutex> g(ctx->mu);
            w = ws_ref(workspace_of(ctx, stream ? (hipStream_t)stream : ctx->stream));
        }
        if (w) {
            lock = std::unique_lock<std::mutex>(w->mu);
            std::lock_guard<std::mutex> g(ctx->mu);
            if (!w->retired) ctx->last_ws = w;
        }
    }
    ~WsLock() {
        if (!w) return;
        lock.unlock();
        ws_unref(ctx, w);
    }
    WsLock(const WsLock&) = delete;
    WsLock& operator=(const WsLock&) = delete;
};

// ctx->last_ws with a reference (the last_* readers)
struct LastWs {
    authjx_ctx* ctx;
    Workspace* w = nullptr;
    int force_scan = 0;
    explicit LastWs(authjx_ctx* c) : ctx(c) {
        std::lock_guard<std::mutex> g(ctx->mu);
        w = ws_ref(ctx->last_ws);
        force_scan = ctx->force_scan;
    }
    ~LastWs() {
        if (w) ws_unref(ctx, w);
    }
    LastWs(const LastWs&) = delete;
    LastWs& operator=(const LastWs&) = delete;
};

// after the launches of a batch: ev1 marks its end on the stream; the rulesets record
// this workspace as a user
int batch_done(Workspace* w, const authjx_ruleset* const* sets, uint32_t n_sets) {
    HIP_OK(hipEventRecord(w->ev1, w->stream));
    if (w->sets_ev[w->sets_slot]) {  // (the end of the last batch that read this set-table slot)
        HIP_OK(hipEventRecord(w->sets_ev[w->sets_slot], w->stream));
        w->sets_ev_rec[w->sets_slot] = true;
    }
    w->ran = true;
    for (uint32_t i = 0; i < n_sets; i++) const_cast<authjx_ruleset*>(sets[i])->note_use(w->id);
    return AUTHJX_OK;
}

}  // namespace

extern "C" {

#ifndef AJX_SRC_HASH
#define AJX_SRC_HASH "unknown"
#endif
const char* authjx_build_hash(void) { return AJX_SRC_HASH; }

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
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return AUTHJX_EDEVICE;
    }
    *out = c;
    return AUTHJX_OK;
}

void authjx_shutdown(authjx_ctx* ctx) {
    if (!ctx) return;
    // batchers still alive: closed (their queued requests evaluated, workers joined) before
    // the workspaces they use go away
    std::vector<authjx_batcher*> live;
    {
        std::lock_guard<std::mutex> g(ctx->mu);
        live = ctx->batchers;
    }
    for (authjx_batcher* b : live) authjx_batcher_destroy(b);
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (Workspace* w : ctx->ws) destroy_workspace(w);  // (no call may run during shutdown)
    if (ctx->d_stage) (void)hipFree(ctx->d_stage);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int authjx_release_stream(authjx_ctx* ctx, void* stream) {
    if (!ctx || !stream || (hipStream_t)stream == ctx->stream) return AUTHJX_EINVAL;
    (void)hipSetDevice(ctx->device);
    retire_stream(ctx, (hipStream_t)stream);
    return AUTHJX_OK;
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
    rs->stream_ok = ajx::stream_eligible(rs->c.blob.data(), (uint32_t)rs->c.blob.size());
    rs->stream_rec = ajx::stream_records(rs->c.blob.data());
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
        // wait for the last batch of every stream that used this ruleset (not the device:
        // other streams' batches and other work go on); the events are collected under the
        // registry lock and waited on outside it
        std::vector<std::shared_ptr<EndEvent>> evs;
        {
            std::lock_guard<std::mutex> lock(rs->mu);
            std::lock_guard<std::mutex> reg(g_reg_mu);
            for (uint64_t id : rs->users)
                for (const auto& e : g_reg)
                    if (e.first == id) evs.push_back(e.second);
        }
        for (const auto& e : evs) (void)hipEventSynchronize(e->ev);
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

// authjx_eval_batch_device; d_sets_pre: the blob pointers already on the device (the
// micro-batcher's one staging copy), else this stream's table is filled from sets
static int eval_device(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                       const uint32_t* d_set_of_req, const uint8_t* d_arena, const uint64_t* d_offs,
                       const uint32_t* d_lens, uint32_t n, uint8_t* d_out_tristate, int32_t* d_out_err_idx,
                       uint64_t* d_out_bitmap, uint32_t bitmap_stride_words, void* stream,
                       const uint8_t* const* d_sets_pre) {
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
    int force_scan, ablate, len_sort, no_tenant_stage;
    uint32_t stream_max_n;
    {
        std::lock_guard<std::mutex> g(ctx->mu);
        force_scan = ctx->force_scan;
        ablate = ctx->ablate;
        len_sort = ctx->len_sort;
        no_tenant_stage = ctx->no_tenant_stage;
        stream_max_n = ctx->stream_max_n;
    }
    WsLock wl(ctx, stream);
    Workspace* w = wl.w;
    if (!w) return AUTHJX_EDEVICE;
    hipStream_t s = w->stream;
    HIP_OK(hipSetDevice(ctx->device));
    int rc = ensure_sets(w, ctx->device, sets, n_sets, d_sets_pre);
    if (rc != AUTHJX_OK) return rc;
    // the streaming kernel: small batches (latency; one request per wave for a multi-tenant
    // batch) whose rulesets all have stream tables; any one-ruleset batch under kernel
    // mode 50..52 (its rows carry 4 more words: the eager decisions stage B reads)
    bool all_stream = true;
    for (uint32_t i = 0; i < n_sets; i++) all_stream = all_stream && sets[i]->stream_ok;
    const bool small = n <= stream_max_n;
    const bool use_stream = !force_scan && all_stream &&
                            (((ablate == 0 || ablate == 53) && small) || (n_sets == 1 && ablate >= 50 && ablate <= 52));
    // requests per wave: 32 for throughput, fewer for a small batch (more waves share it)
    uint32_t per = ajx::kStreamSpan;
    if (n_sets > 1)
        per = 1;
    else if (ablate == 0 || ablate == 53)
        per = std::max<uint32_t>(1u, std::min<uint32_t>(ajx::kStreamSpan, (n + 2047u) / 2048u));
    uint32_t max_rec = 0;
    for (uint32_t i = 0; i < n_sets; i++) max_rec = std::max(max_rec, sets[i]->stream_rec);
    const uint32_t rows_stride = use_stream ? std::max(row_stride, 1u + max_rec) + 4u : row_stride;
    if (!force_scan) {
        rc = ensure_work(w, n, rows_stride);
        if (rc != AUTHJX_OK) return rc;
    }
    HIP_OK(hipEventRecord(w->ev0, s));
    // kernel: the streaming kernel (ajx_stream.h) for a one-ruleset batch whose ruleset it
    // takes, else the lean single-pass kernel (ajx_lean.h) or the multi-tenant kernel; the
    // exact scan for what they hand over
    bool mods = false;  // modifier chains: the exact scan's instance with text buffers
    for (uint32_t i = 0; i < n_sets; i++)
        mods = mods || reinterpret_cast<const ajx::RulesetHdr*>(sets[i]->c.blob.data())->n_modifiers != 0 ||
               (reinterpret_cast<const ajx::RulesetHdr*>(sets[i]->c.blob.data())->flags & ajx::kFlagBufs) != 0;
    // capture rows kept for authjx_select_from_eval_device: one forest ruleset
    // (authjx_compile_forest), a full kernel
    const bool full = ablate == 0 || ablate == 41 || ablate == 52 || (ablate >= 10 && ablate <= 12) ||
                      (ablate >= 15 && ablate <= 18);  // (15..18: lean ablations, length order kept)
    const auto* h0 = reinterpret_cast<const ajx::RulesetHdr*>(sets[0]->c.blob.data());
    // (not under the lean ablations 15..18: their rows hold checksums)
    const bool keep_rows = !force_scan && n_sets == 1 && full && !(ablate >= 15 && ablate <= 18) && h0->pad1[0] != 0;
    w->rows_rs = keep_rows ? sets[0] : nullptr;
    w->rows_n = n;
    w->rows_stride = row_stride;
    w->rows_perm = nullptr;
    w->rows_wave = true;
    size_t max_blob = 0;
    for (uint32_t i = 0; i < n_sets; i++) max_blob = std::max(max_blob, sets[i]->c.blob.size());
    // (the counters are zero only after a FIN launch: every other launch fills them itself)
    bool cnt_zero = w->cnt_zero;
    w->cnt_zero = w->exact3 = false;
    if (force_scan) {
        HIP_OK(ajx::launch_eval_scan(w->d_sets, d_set_of_req, d_arena, d_offs, d_lens, n, d_out_tristate,
                                     d_out_err_idx, d_out_bitmap, bitmap_stride_words, s, mods));
    } else if (use_stream) {
        // the streaming kernel (ajx_stream.h; ablate 50: its structural pass alone, 51: no
        // fold), its stage B over the d_perm buffer as the stage-B list
        w->rows_stride = rows_stride;
        HIP_OK(ajx::launch_eval_stream(w->d_sets, d_set_of_req, (uint32_t)max_blob, max_rec, d_arena,
                                       d_offs, d_lens, n, d_out_tristate, d_out_err_idx, d_out_bitmap,
                                       bitmap_stride_words, w->d_rows, rows_stride, keep_rows, w->d_perm, w->d_slow,
                                       w->d_slow + 3, s, ablate == 50 ? 1 : ablate == 51 ? 2 : ablate == 53 ? 3 : 0, mods,
                                       per, &cnt_zero));
        w->cnt_zero = w->exact3 = cnt_zero;
    } else {
        // length-bucketed order: one ruleset for the batch (multi-tenant batches keep the
        // caller's bucketing by AuthConfig), a full kernel, batches worth sorting
        const uint32_t* perm = nullptr;
        uint32_t* pos_of = nullptr;
        const uint32_t n_out = n_sets == 1 && h0->pad1[0] ? h0->pad1[0] : 1u;
        if (len_sort && (n_sets == 1 || len_sort > 1) && full && n >= 4096) {
            // (one ruleset: its outputs in work-item order, gathered back by pos_of)
            // (forests, several results per request, keep writing at the request: the
            // gather's strided byte copies cost more than the scattered stores, c5 12.0 → 12.4 ms)
            if (n_sets == 1 && n_out == 1) {
                rc = ensure_tout(w, ajx::tout_bytes(n, n_out, d_out_bitmap ? bitmap_stride_words : 0u));
                if (rc != AUTHJX_OK) return rc;
                pos_of = w->d_perm + (size_t)n + 4096;
            }
            HIP_OK(ajx::launch_len_order(d_lens, n, w->d_perm + n, w->d_perm, s, pos_of));
            perm = w->d_perm;
        }
        w->rows_perm = perm;
        // uniform batch: the blob staged once per workgroup; multi-tenant batch: nonzero
        // turns on the per-workgroup staging of its runs' rulesets (ajx_scan_fused_tenant)
        const uint32_t stage_bytes =
            n_sets == 1 ? (max_blob <= ajx::kMaxSharedBlobBytes ? (uint32_t)max_blob : 0u)
                        : (!no_tenant_stage ? (uint32_t)std::min<size_t>(max_blob, ajx::kMaxTenantStageBytes) : 0u);
        HIP_OK(ajx::launch_eval_fast(w->d_sets, d_set_of_req, stage_bytes, d_arena, d_offs, d_lens, n,
                                     d_out_tristate, d_out_err_idx, d_out_bitmap, bitmap_stride_words,
                                     w->d_rows, row_stride, w->d_slow, w->d_slow + 1, s,
                                     ablate < 20 ? ablate : 0, perm, mods, keep_rows, n_sets == 1 ? h0->lean_feat : 3u,
                                     pos_of, pos_of ? w->d_tout : nullptr, n_out));
    }
    return batch_done(w, sets, n_sets);
}

int authjx_eval_batch_device(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                             const uint32_t* d_set_of_req, const uint8_t* d_arena, const uint64_t* d_offs,
                             const uint32_t* d_lens, uint32_t n, uint8_t* d_out_tristate, int32_t* d_out_err_idx,
                             uint64_t* d_out_bitmap, uint32_t bitmap_stride_words, void* stream) {
    return eval_device(ctx, sets, n_sets, d_set_of_req, d_arena, d_offs, d_lens, n, d_out_tristate, d_out_err_idx,
                       d_out_bitmap, bitmap_stride_words, stream, nullptr);
}

static_assert(sizeof(authjx_value) == 12, "authjx_value is three u32 words on the device");

int authjx_select_batch_device(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                               const uint32_t* d_set_of_req, const uint8_t* d_arena, const uint64_t* d_offs,
                               const uint32_t* d_lens, uint32_t n, authjx_value* d_out_values,
                               uint32_t values_stride, void* stream) {
    return authjx_select_text_batch_device(ctx, sets, n_sets, d_set_of_req, d_arena, d_offs, d_lens, n, d_out_values,
                                           values_stride, nullptr, 0, stream);
}

int authjx_select_text_batch_device(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                                    const uint32_t* d_set_of_req, const uint8_t* d_arena, const uint64_t* d_offs,
                                    const uint32_t* d_lens, uint32_t n, authjx_value* d_out_values,
                                    uint32_t values_stride, uint8_t* d_out_text, uint32_t text_stride, void* stream) {
    if (!ctx || !sets || n_sets == 0 || (n && (!d_arena || !d_offs || !d_lens || !d_out_values)))
        return AUTHJX_EINVAL;
    if (d_out_text && text_stride == 0) return AUTHJX_EINVAL;
    if (n_sets > 1 && !d_set_of_req) return AUTHJX_EINVAL;
    if (n_sets == 1) d_set_of_req = nullptr;
    uint32_t max_sel = 0;
    for (uint32_t i = 0; i < n_sets; i++) {
        if (!sets[i] || sets[i]->c.n_patterns > values_stride) return AUTHJX_EINVAL;
        if (sets[i]->c.n_selectors > max_sel) max_sel = sets[i]->c.n_selectors;
    }
    const uint32_t row_stride = 1 + max_sel;
    int force_scan, len_sort;
    {
        std::lock_guard<std::mutex> g(ctx->mu);
        force_scan = ctx->force_scan;
        len_sort = ctx->len_sort;
    }
    WsLock wl(ctx, stream);
    Workspace* w = wl.w;
    if (!w) return AUTHJX_EDEVICE;
    hipStream_t s = w->stream;
    HIP_OK(hipSetDevice(ctx->device));
    int rc = ensure_sets(w, ctx->device, sets, n_sets);
    if (rc != AUTHJX_OK) return rc;
    const bool exact = force_scan != 0;  // the exact Get per selector (cross-check)
    w->rows_rs = nullptr;  // (the rows are rewritten for this ruleset)
    w->cnt_zero = w->exact3 = false;  // (its slow count is filled and left nonzero)
    if (!exact && (rc = ensure_work(w, n, row_stride)) != AUTHJX_OK) return rc;
    const uint32_t* perm = nullptr;
    if (!exact && len_sort && n_sets == 1 && n >= 4096) {
        HIP_OK(ajx::launch_len_order(d_lens, n, w->d_perm + n, w->d_perm, s));
        perm = w->d_perm;
    }
    const uint32_t shared_bytes =
        (n_sets == 1 && sets[0]->c.blob.size() <= ajx::kMaxSharedBlobBytes) ? (uint32_t)sets[0]->c.blob.size() : 0u;
    HIP_OK(ajx::launch_select(w->d_sets, d_set_of_req, shared_bytes, d_arena, d_offs, d_lens, n,
                              reinterpret_cast<uint32_t*>(d_out_values), values_stride,
                              exact ? nullptr : w->d_rows, row_stride, w->d_slow, w->d_slow + 1, perm, d_out_text,
                              text_stride, s));
    return batch_done(w, sets, n_sets);
}

int authjx_select_from_eval_device(authjx_ctx* ctx, const authjx_ruleset* rs, uint32_t first_pattern,
                                   const uint8_t* d_arena, const uint64_t* d_offs, const uint32_t* d_lens,
                                   uint32_t n, authjx_value* d_out_values, uint32_t values_stride, void* stream) {
    if (!ctx || !rs || values_stride == 0 || (n && (!d_arena || !d_offs || !d_lens || !d_out_values)))
        return AUTHJX_EINVAL;
    if (first_pattern + values_stride > rs->c.n_patterns) return AUTHJX_EINVAL;
    WsLock wl(ctx, stream);
    Workspace* w = wl.w;
    if (!w) return AUTHJX_EDEVICE;
    // the rows must be this stream's last evaluation's, of this ruleset, over this many
    // requests, and hold these patterns' records: a selector the scan decides eagerly has a
    // record only when it belongs to a root-less tree of the forest (kEagerKeep)
    if (w->rows_rs != rs || w->rows_n != n) return AUTHJX_EINVAL;
    {
        const auto* h = reinterpret_cast<const ajx::RulesetHdr*>(rs->c.blob.data());
        const auto* pats = reinterpret_cast<const ajx::Pattern*>(rs->c.blob.data() + h->off_patterns);
        const auto* eg = h->off_eager ? reinterpret_cast<const ajx::EagerSel*>(rs->c.blob.data() + h->off_eager)
                                      : nullptr;
        for (uint32_t p = first_pattern; eg && p < first_pattern + values_stride; p++) {
            const uint32_t f = eg[pats[p].selector].pad[0];
            if ((f & ajx::kEagerAll) && !(f & ajx::kEagerKeep)) return AUTHJX_EINVAL;
        }
    }
    hipStream_t s = w->stream;
    HIP_OK(hipSetDevice(ctx->device));
    const authjx_ruleset* one[1] = {rs};
    int rc = ensure_sets(w, ctx->device, one, 1);
    if (rc != AUTHJX_OK) return rc;
    HIP_OK(ajx::launch_select_rows(w->d_sets, d_arena, d_offs, d_lens, n, reinterpret_cast<uint32_t*>(d_out_values),
                                   values_stride, w->d_rows, w->rows_stride, first_pattern, w->rows_perm,
                                   w->rows_wave, s));
    return batch_done(w, one, 1);
}

int authjx_select_batch(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                        const uint32_t* set_of_req, const uint8_t* arena, uint64_t arena_len,
                        const uint64_t* offs, const uint32_t* lens, uint32_t n, authjx_value* out_values,
                        uint32_t values_stride) {
    return authjx_select_text_batch(ctx, sets, n_sets, set_of_req, arena, arena_len, offs, lens, n, out_values,
                                    values_stride, nullptr, 0);
}

int authjx_select_text_batch(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                             const uint32_t* set_of_req, const uint8_t* arena, uint64_t arena_len,
                             const uint64_t* offs, const uint32_t* lens, uint32_t n, authjx_value* out_values,
                             uint32_t values_stride, uint8_t* out_text, uint32_t text_stride) {
    if (!ctx || (n && (!arena || !offs || !lens || !out_values))) return AUTHJX_EINVAL;
    if (out_text && text_stride == 0) return AUTHJX_EINVAL;
    for (uint32_t r = 0; r < n; r++)
        if (offs[r] + lens[r] > arena_len || (set_of_req && set_of_req[r] >= n_sets)) return AUTHJX_EINVAL;
    const bool with_sor = set_of_req != nullptr;
    const size_t o_offs = round_up(arena_len, 256);
    const size_t o_lens = round_up(o_offs + (size_t)n * 8, 256);
    const size_t o_sor = round_up(o_lens + (size_t)n * 4, 256);
    const size_t o_out = round_up(o_sor + (with_sor ? (size_t)n * 4 : 0), 256);
    const size_t out_bytes = (size_t)n * values_stride * sizeof(authjx_value);
    const size_t o_text = round_up(o_out + out_bytes, 256);
    const size_t text_bytes = out_text ? (size_t)n * text_stride : 0;
    const size_t total = round_up(o_text + text_bytes, 256);
    std::lock_guard<std::mutex> batch_lock(ctx->batch_mu);
    {
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
    int rc = authjx_select_text_batch_device(ctx, sets, n_sets, with_sor ? (const uint32_t*)(b + o_sor) : nullptr,
                                             b, (const uint64_t*)(b + o_offs), (const uint32_t*)(b + o_lens), n,
                                             (authjx_value*)(b + o_out), values_stride,
                                             out_text ? b + o_text : nullptr, text_stride, nullptr);
    if (rc != AUTHJX_OK) return rc;
    HIP_OK(hipMemcpyAsync(out_values, b + o_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
    if (out_text) HIP_OK(hipMemcpyAsync(out_text, b + o_text, text_bytes, hipMemcpyDeviceToHost, ctx->stream));
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


// Profiling only (not in authjx.h): batches of up to n requests take the streaming kernel
// (default 4096; 0: never)
int authjx_debug_stream_max(authjx_ctx* ctx, uint32_t n) {
    if (!ctx) return AUTHJX_EINVAL;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->stream_max_n = n;
    return AUTHJX_OK;
}

// Diagnostics (not in authjx.h): the HIP error behind this thread's last AUTHJX_EDEVICE and
// the ajx_api.cpp line that saw it ("" when none)
const char* authjx_debug_last_error(void) {
    static thread_local char buf[160];
    if (t_last_hip == hipSuccess) return "";
    std::snprintf(buf, sizeof buf, "%s (ajx_api.cpp:%d)", hipGetErrorString(t_last_hip), t_last_line);
    return buf;
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

// profiling: a compiled ruleset's device blob size in bytes (what the kernels stage in LDS)
uint32_t authjx_debug_blob_bytes(const authjx_ruleset* rs) { return rs ? (uint32_t)rs->c.blob.size() : 0u; }

int authjx_set_exact_scan(authjx_ctx* ctx, int force) {
    if (!ctx) return AUTHJX_EINVAL;
    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->force_scan = force ? 1 : 0;
    return AUTHJX_OK;
}

int64_t authjx_last_exact_count(authjx_ctx* ctx) {
    if (!ctx) return AUTHJX_EINVAL;
    LastWs ref(ctx);
    Workspace* w = ref.w;
    if (ref.force_scan || !w) return -1;
    std::lock_guard<std::mutex> lock(w->mu);
    if (!w->d_slow || !w->ran) return -1;
    uint32_t c = 0;
    if (hipSetDevice(ctx->device) != hipSuccess || hipEventSynchronize(w->ev1) != hipSuccess ||
        hipMemcpy(&c, w->d_slow + (w->exact3 ? 3 : 0), sizeof c, hipMemcpyDeviceToHost) != hipSuccess)
        return AUTHJX_EDEVICE;
    return (int64_t)c;
}

float authjx_last_kernel_ms(authjx_ctx* ctx) {
    if (!ctx) return 0.f;
    LastWs ref(ctx);
    Workspace* w = ref.w;
    if (!w) return 0.f;
    std::lock_guard<std::mutex> lock(w->mu);
    float ms = 0.f;
    if (!w->ran || hipEventSynchronize(w->ev1) != hipSuccess) return 0.f;
    if (hipEventElapsedTime(&ms, w->ev0, w->ev1) != hipSuccess) return 0.f;
    return ms;
}

int authjx_eval_batch(authjx_ctx* ctx, const authjx_ruleset* const* sets, uint32_t n_sets,
                      const uint32_t* set_of_req, const uint8_t* arena, uint64_t arena_len, const uint64_t* offs,
                      const uint32_t* lens, uint32_t n, uint8_t* out_tristate, int32_t* out_err_idx,
                      uint64_t* out_bitmap, uint32_t bitmap_stride_words) {
    if (!ctx || (n && (!arena || !offs || !lens || !out_tristate))) return AUTHJX_EINVAL;
    for (uint32_t r = 0; r < n; r++)
        if (offs[r] + lens[r] > arena_len || (set_of_req && set_of_req[r] >= n_sets)) return AUTHJX_EINVAL;
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
    hipStream_t s = ctx->stream;
    HIP_OK(hipMemcpyAsync(out_tristate, b + o_tri, (size_t)n * nt, hipMemcpyDeviceToHost, s));
    if (out_err_idx) HIP_OK(hipMemcpyAsync(out_err_idx, b + o_err, (size_t)n * nt * 4, hipMemcpyDeviceToHost, s));
    if (out_bitmap)
        HIP_OK(hipMemcpyAsync(out_bitmap, b + o_bm, (size_t)n * bitmap_stride_words * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return AUTHJX_OK;
}

// ---- micro-batcher ------------------------------------------------------------------

}  // extern "C"

constexpr uint32_t kBatcherMaxWorkers = 8;
// workers per batcher: 2 by default (one packs and launches while the other's batch runs);
// authjx_debug_batcher_workers changes it for batchers created afterwards
std::atomic<uint32_t> g_batcher_workers{2};
// profiling knobs (authjx_debug_batcher_modes), read when a batcher is created: how callers
// are woken (0: one condition variable each, 1: one broadcast per batch, 2: one futex word
// each, 3: as 2, in a binary tree where each woken caller wakes two more), how a worker waits
// for its batch (0: hipStreamSynchronize, 1: polling hipStreamQuery), where the kernel reads
// the batch (0: one copy into device memory, 1: the pinned staging buffer itself)
// (zero-copy is the default: measured p50 3-15 µs lower at 64 producers, the same or more
// decisions/s at 256)
std::atomic<uint32_t> g_batcher_wake{0}, g_batcher_sync{0}, g_batcher_zcopy{1};

struct authjx_batcher {
    authjx_ctx* ctx = nullptr;
    // per worker: its own stream (its own workspace in ctx) and staging buffers
    struct Lane {
        hipStream_t stream = nullptr;
        uint8_t* h_buf = nullptr;  // pinned staging: arena | offs | lens | set_of_req | sets | outputs
        uint8_t* h_dev = nullptr;  // its device address (the kernel writes the outputs there)
        size_t h_cap = 0;
        uint8_t* d_buf = nullptr;
        size_t d_cap = 0;
    } lanes[kBatcherMaxWorkers];
    uint32_t n_lanes = 2;
    uint32_t sync_mode = 0, zcopy = 0;
    ajx::BatchCore* core = nullptr;
    // profiling sums (ns): packing the staging buffer, launch calls, the wait for the device
    std::atomic<uint64_t> pack_ns{0}, launch_ns{0}, sync_ns{0};

    // one batch (ordered by ruleset): pack, one launch (worker `wid` only). The pinned
    // staging buffer carries the documents, offsets, lengths, each request's ruleset index
    // and the rulesets' blob pointers; the kernel reads them from it (mapped host memory;
    // with zero-copy off, one copy into device memory first) and writes the results into
    // it, so a small batch is one kernel (its counters left zero by the last one on this
    // stream) and a synchronize.
    int evaluate(std::vector<ajx::BatchReq*>& reqs, uint32_t wid) {
        Lane& L = lanes[wid];
        hipStream_t stream = L.stream;
        uint8_t*& h_buf = L.h_buf;
        size_t& h_cap = L.h_cap;
        uint8_t*& d_buf = L.d_buf;
        size_t& d_cap = L.d_cap;
        const uint32_t n = (uint32_t)reqs.size(), nt = reqs[0]->n_out;
        std::vector<const authjx_ruleset*> sets;
        std::vector<uint32_t> sor(n);
        size_t arena_len = 0;
        for (uint32_t i = 0; i < n; i++) {
            const authjx_ruleset* rs = (const authjx_ruleset*)reqs[i]->rs;
            if (sets.empty() || sets.back() != rs) sets.push_back(rs);
            sor[i] = (uint32_t)sets.size() - 1;
            arena_len += reqs[i]->len;
        }
        const size_t o_offs = round_up(arena_len + 1, 256);
        const size_t o_lens = round_up(o_offs + (size_t)n * 8, 256);
        const size_t o_sor = round_up(o_lens + (size_t)n * 4, 256);
        const size_t o_sets = round_up(o_sor + (size_t)n * 4, 256);
        const size_t o_in_end = round_up(o_sets + sets.size() * sizeof(uint8_t*), 256);
        const size_t o_tri = o_in_end;  // (host side only: written by the kernel)
        const size_t o_err = round_up(o_tri + (size_t)n * nt, 256);
        const size_t total = round_up(o_err + (size_t)n * nt * 4, 256);
        HIP_OK(hipSetDevice(ctx->device));
        if (total > h_cap) {
            if (h_buf) (void)hipHostFree(h_buf);
            h_buf = nullptr;
            h_cap = 0;
            L.h_dev = nullptr;
            HIP_OK(hipHostMalloc(&h_buf, total, hipHostMallocDefault));
            h_cap = total;
            void* dp = nullptr;
            HIP_OK(hipHostGetDevicePointer(&dp, h_buf, 0));
            L.h_dev = (uint8_t*)dp;
        }
        if (o_in_end > d_cap) {
            if (d_buf) (void)hipFree(d_buf);
            d_buf = nullptr;
            d_cap = 0;
            HIP_OK(hipMalloc(&d_buf, o_in_end));
            d_cap = o_in_end;
        }
        const uint64_t t0 = ajx::mono_ns();
        uint64_t* offs = (uint64_t*)(h_buf + o_offs);
        uint32_t* lens = (uint32_t*)(h_buf + o_lens);
        size_t at = 0;
        for (uint32_t i = 0; i < n; i++) {
            if (reqs[i]->len) std::memcpy(h_buf + at, reqs[i]->doc, reqs[i]->len);
            offs[i] = at;
            lens[i] = (uint32_t)reqs[i]->len;
            at += reqs[i]->len;
        }
        h_buf[at] = 0;
        std::memcpy(h_buf + o_sor, sor.data(), (size_t)n * 4);
        const uint8_t** hs = (const uint8_t**)(h_buf + o_sets);
        for (size_t k = 0; k < sets.size(); k++) hs[k] = sets[k] ? sets[k]->d_blob : nullptr;
        const uint64_t t1 = ajx::mono_ns();
        // (zero-copy: the kernel reads the batch from the mapped staging buffer over PCIe)
        const uint8_t* in = zcopy ? L.h_dev : d_buf;
        if (!zcopy) HIP_OK(hipMemcpyAsync(d_buf, h_buf, o_in_end, hipMemcpyHostToDevice, stream));
        const int rc = eval_device(ctx, sets.data(), (uint32_t)sets.size(), (const uint32_t*)(in + o_sor), in,
                                   (const uint64_t*)(in + o_offs), (const uint32_t*)(in + o_lens), n,
                                   L.h_dev + o_tri, (int32_t*)(L.h_dev + o_err), nullptr, 0, stream,
                                   (const uint8_t* const*)(in + o_sets));
        if (rc != AUTHJX_OK) return rc;
        const uint64_t t2 = ajx::mono_ns();
        if (sync_mode == 1) {
            for (;;) {
                const hipError_t q = hipStreamQuery(stream);
                if (q == hipSuccess) break;
                if (q != hipErrorNotReady) HIP_OK(q);
            }
        } else {
            HIP_OK(hipStreamSynchronize(stream));
        }
        const uint64_t t3 = ajx::mono_ns();
        pack_ns.fetch_add(t1 - t0, std::memory_order_relaxed);
        launch_ns.fetch_add(t2 - t1, std::memory_order_relaxed);
        sync_ns.fetch_add(t3 - t2, std::memory_order_relaxed);
        const uint8_t* tri = h_buf + o_tri;
        const int32_t* err = (const int32_t*)(h_buf + o_err);
        for (uint32_t i = 0; i < n; i++) {
            for (uint32_t k = 0; k < nt; k++) {
                reqs[i]->out_tri[k] = tri[(size_t)i * nt + k];
                if (reqs[i]->out_err) reqs[i]->out_err[k] = err[(size_t)i * nt + k];
            }
        }
        return AUTHJX_OK;
    }
};

extern "C" {

int authjx_batcher_create(authjx_ctx* ctx, uint32_t max_batch, uint32_t window_us, uint32_t queue_cap,
                          authjx_batcher** out) {
    if (!ctx || !out || max_batch == 0) return AUTHJX_EINVAL;
    *out = nullptr;
    HIP_OK(hipSetDevice(ctx->device));
    authjx_batcher* b = new authjx_batcher();
    b->ctx = ctx;
    b->n_lanes = std::min<uint32_t>(std::max<uint32_t>(g_batcher_workers.load(), 1u), kBatcherMaxWorkers);
    b->sync_mode = g_batcher_sync.load();
    b->zcopy = g_batcher_zcopy.load();
    for (uint32_t k = 0; k < b->n_lanes; k++)
        if (hipStreamCreateWithFlags(&b->lanes[k].stream, hipStreamNonBlocking) != hipSuccess) {
            for (auto& M : b->lanes)
                if (M.stream) (void)hipStreamDestroy(M.stream);
            delete b;
            return AUTHJX_EDEVICE;
        }
    b->core = new ajx::BatchCore(
        max_batch, (uint64_t)window_us * 1000ull, queue_cap ? queue_cap : 4 * max_batch,
        [b](std::vector<ajx::BatchReq*>& reqs, uint32_t wid) { return b->evaluate(reqs, wid); }, b->n_lanes,
        g_batcher_wake.load());
    {
        std::lock_guard<std::mutex> g(ctx->mu);
        ctx->batchers.push_back(b);
    }
    *out = b;
    return AUTHJX_OK;
}

// Profiling only (not in authjx.h): worker threads (each with its own stream) of the
// batchers created after this call (1..8; default 2). n = 0 returns the current count.
int authjx_debug_batcher_workers(uint32_t n) {
    if (n == 0) return (int)g_batcher_workers.load();
    if (n > kBatcherMaxWorkers) return AUTHJX_EINVAL;
    g_batcher_workers.store(n);
    return AUTHJX_OK;
}

// Profiling only (not in authjx.h): the knobs of g_batcher_wake (0..3) / _sync / _zcopy
// (0 or 1) for the batchers created after this call.
int authjx_debug_batcher_modes(uint32_t wake, uint32_t sync, uint32_t zcopy) {
    if (wake > 3 || sync > 1 || zcopy > 1) return AUTHJX_EINVAL;
    g_batcher_wake.store(wake);
    g_batcher_sync.store(sync);
    g_batcher_zcopy.store(zcopy);
    return AUTHJX_OK;
}

// Profiling only (not in authjx.h): out[0..8] = batches, requests, and the sums in ns of the
// queue wait (per request), evaluation, waking callers, callers' resume (per request),
// packing, launch calls and the device wait (per batch).
int authjx_debug_batcher_profile(authjx_batcher* b, uint64_t* out) {
    if (!b || !out) return AUTHJX_EINVAL;
    const ajx::BatchStats st = b->core->stats();
    const uint64_t v[9] = {st.batches, st.requests, st.wait_ns, st.eval_ns, st.wake_ns, st.resume_ns,
                           b->pack_ns.load(), b->launch_ns.load(), b->sync_ns.load()};
    std::memcpy(out, v, sizeof(v));
    return AUTHJX_OK;
}

void authjx_batcher_destroy(authjx_batcher* b) {
    if (!b) return;
    {
        std::lock_guard<std::mutex> g(b->ctx->mu);
        auto& v = b->ctx->batchers;
        v.erase(std::remove(v.begin(), v.end(), b), v.end());
    }
    delete b->core;  // evaluates what is queued, joins the workers
    (void)hipSetDevice(b->ctx->device);
    for (auto& L : b->lanes) {
        if (L.stream) (void)hipStreamSynchronize(L.stream);
        if (L.h_buf) (void)hipHostFree(L.h_buf);
        if (L.d_buf) (void)hipFree(L.d_buf);
        if (L.stream) retire_stream(b->ctx, L.stream);  // (only the joined workers used it)
        if (L.stream) (void)hipStreamDestroy(L.stream);
    }
    delete b;
}

int authjx_batcher_eval(authjx_batcher* b, const authjx_ruleset* rs, const uint8_t* doc, size_t len,
                        uint64_t timeout_us, uint8_t* out_tristate, int32_t* out_err_idx) {
    if (!b || !rs || (!doc && len) || !out_tristate || len >= (1ull << 32)) return AUTHJX_EINVAL;
    if (rs->device != b->ctx->device) return AUTHJX_EINVAL;
    ajx::BatchReq r;
    r.rs = rs;
    r.n_out = rs->c.n_trees;
    r.doc = doc;
    r.len = len;
    r.deadline_ns = timeout_us ? ajx::mono_ns() + timeout_us * 1000ull : 0;
    r.out_tri = out_tristate;
    r.out_err = out_err_idx;
    return b->core->submit(r);
}

// Profiling only (not in authjx.h): the serving path under load. `threads` producer threads
// each submit their share of the n requests (request i: sets[sor[i]] on arena[offs[i] ..
// offs[i] + lens[i]); thread t takes i = t, t + threads, ...) one at a time through the
// batcher (authjx_batcher_eval, blocking, as a serving goroutine would); lat_ns[i] = that
// call's latency, out_tri[i] its first result; *wall_ns = the whole run.
int authjx_debug_loadgen(authjx_batcher* b, const authjx_ruleset* const* sets, const uint32_t* sor,
                         const uint8_t* arena, const uint64_t* offs, const uint32_t* lens, uint32_t n,
                         uint32_t threads, uint64_t* lat_ns, uint8_t* out_tri, uint64_t* wall_ns) {
    if (!b || !sets || !sor || !arena || !offs || !lens || !lat_ns || !out_tri || !wall_ns || threads == 0)
        return AUTHJX_EINVAL;
    std::atomic<int> first_rc{AUTHJX_OK};
    const uint64_t t0 = ajx::mono_ns();
    std::vector<std::thread> ts;
    for (uint32_t t = 0; t < threads; t++)
        ts.emplace_back([&, t] {
            uint8_t tri[64];
            for (uint32_t i = t; i < n; i += threads) {
                const authjx_ruleset* rs = sets[sor[i]];
                if (rs->c.n_trees > 64) {
                    first_rc.store(AUTHJX_EINVAL);
                    return;
                }
                const uint64_t a = ajx::mono_ns();
                const int rc = authjx_batcher_eval(b, rs, arena + offs[i], lens[i], 0, tri, nullptr);
                lat_ns[i] = ajx::mono_ns() - a;
                out_tri[i] = tri[0];
                if (rc != AUTHJX_OK) {
                    int ok = AUTHJX_OK;
                    first_rc.compare_exchange_strong(ok, rc);
                }
            }
        });
    for (auto& th : ts) th.join();
    *wall_ns = ajx::mono_ns() - t0;
    return first_rc.load();
}

int authjx_batcher_stats(authjx_batcher* b, uint64_t* batches, uint64_t* requests, uint64_t* expired,
                         uint64_t* max_batch_seen) {
    if (!b) return AUTHJX_EINVAL;
    const ajx::BatchStats st = b->core->stats();
    if (batches) *batches = st.batches;
    if (requests) *requests = st.requests;
    if (expired) *expired = st.expired;
    if (max_batch_seen) *max_batch_seen = st.max_batch_seen;
    return AUTHJX_OK;
}

}  // extern "C"
