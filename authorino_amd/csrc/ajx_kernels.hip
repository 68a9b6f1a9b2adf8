// ajx_kernels.hip — gfx950 kernels of the batched evaluator.
//
// ajx_scan_fast  stage A, one work-item per request: single pass over the document,
//                all selectors followed at once through the ruleset trie; writes each
//                selector's value span to the request's capture row (ajx_fast.h).
//                Requests it can not prove gjson-equivalent go to a slow list.
// ajx_patterns   stage B, one work-item per request: patterns on the captured values,
//                T bitmap, And/Or fold.
// ajx_eval_scan  one work-item per request on the slow list (or on every request when
//                forced): for each selector an exact gjson.Get scan (ajx_device.h gj_get),
//                then the patterns and the fold. Exact for arbitrary input bytes.
#include <hip/hip_runtime.h>

#include "ajx_fast.h"
#include "ajx_kernels.h"

namespace ajx {

constexpr int kSelCache = 32;  // resolved selector values kept per request
constexpr int kPatCache = 64;  // pattern results kept per request for the fold

__device__ __forceinline__ void eval_scan_one(uint32_t r, const uint8_t* const* __restrict__ sets,
                                              const uint32_t* __restrict__ set_of_req,
                                              const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                                              const uint32_t* __restrict__ lens, uint8_t* __restrict__ out_tri,
                                              int32_t* __restrict__ out_err, uint64_t* __restrict__ out_bm,
                                              uint32_t stride) {
    const uint8_t* blob = sets[set_of_req ? set_of_req[r] : 0];
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
    const Selector* sels = reinterpret_cast<const Selector*>(blob + h->off_selectors);
    const Component* comps = reinterpret_cast<const Component*>(blob + h->off_components);
    const Pattern* pats = reinterpret_cast<const Pattern*>(blob + h->off_patterns);
    const uint32_t* code = reinterpret_cast<const uint32_t*>(blob + h->off_code);
    const uint8_t* lits = blob + h->off_literals;
    const uint8_t* doc = arena + offs[r];
    const uint32_t len = lens[r];

    const uint32_t ns = h->n_selectors, np = h->n_patterns;
    ValueRef vals[kSelCache];
    const bool cache_sel = ns <= (uint32_t)kSelCache;
    if (cache_sel)
        for (uint32_t s = 0; s < ns; s++)
            vals[s] = gj_get(doc, len, comps + sels[s].comp_begin, sels[s].comp_count, lits);

    auto value_of = [&](uint32_t p) -> ValueRef {
        if (cache_sel) return vals[pats[p].selector];
        const Selector& s = sels[pats[p].selector];
        return gj_get(doc, len, comps + s.comp_begin, s.comp_count, lits);
    };
    auto eval = [&](uint32_t p) -> uint8_t {
        const Pattern& pt = pats[p];
        if (pt.state != P_OK) return eval_pattern(blob, pt, doc, ValueRef{0, 0, T_NULL, 0});
        return eval_pattern(blob, pt, doc, value_of(p));
    };

    uint8_t res[kPatCache];
    const bool cache_pat = np <= (uint32_t)kPatCache;
    if (out_bm) {
        uint64_t* row = out_bm + (size_t)r * stride;
        for (uint32_t w = 0; w < stride; w++) {
            uint64_t word = 0;
            for (uint32_t b = 0; b < 64; b++) {
                uint32_t p = w * 64 + b;
                if (p >= np) break;
                uint8_t v = eval(p);
                if (cache_pat) res[p] = v;
                if (v == V_T) word |= 1ull << b;
            }
            row[w] = word;
        }
    }
    int32_t ep;
    uint8_t t;
    if (cache_pat) {
        if (!out_bm)
            for (uint32_t p = 0; p < np; p++) res[p] = eval(p);
        t = run_fold(code, h->n_code, [&](uint32_t p) { return res[p]; }, &ep);
    } else {
        t = run_fold(code, h->n_code, eval, &ep);
    }
    out_tri[r] = t;
    if (out_err) out_err[r] = ep;
}

__global__ __launch_bounds__(256) void ajx_eval_scan(const uint8_t* const* __restrict__ sets,
                                                     const uint32_t* __restrict__ set_of_req,
                                                     const uint8_t* __restrict__ arena,
                                                     const uint64_t* __restrict__ offs,
                                                     const uint32_t* __restrict__ lens, uint32_t n,
                                                     uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err,
                                                     uint64_t* __restrict__ out_bm, uint32_t stride) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    eval_scan_one(r, sets, set_of_req, arena, offs, lens, out_tri, out_err, out_bm, stride);
}

// the slow list: grid-stride over the ids the fast kernel appended
__global__ __launch_bounds__(256) void ajx_eval_scan_list(const uint8_t* const* __restrict__ sets,
                                                          const uint32_t* __restrict__ set_of_req,
                                                          const uint8_t* __restrict__ arena,
                                                          const uint64_t* __restrict__ offs,
                                                          const uint32_t* __restrict__ lens,
                                                          const uint32_t* __restrict__ slow_count,
                                                          const uint32_t* __restrict__ slow_ids,
                                                          uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err,
                                                          uint64_t* __restrict__ out_bm, uint32_t stride) {
    const uint32_t cnt = *slow_count;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x)
        eval_scan_one(slow_ids[i], sets, set_of_req, arena, offs, lens, out_tri, out_err, out_bm, stride);
}

// LDS image of a ruleset's single-pass tables (SHARED kernels): trie nodes, trie
// children, key slots, each region sized for the compile limits.
constexpr uint32_t kLdsNodeWords = kFastMaxNodes * sizeof(TrieNode) / 4;
constexpr uint32_t kLdsChildWords = kFastMaxNodes * sizeof(TrieChild) / 4;
constexpr uint32_t kLdsSlotWords = (1u << kMaxKeySlotsLog2) * sizeof(KeySlot) / 4;
constexpr uint32_t kLdsTabWords = kLdsNodeWords + kLdsChildWords + kLdsSlotWords;
static_assert((kLdsNodeWords * 4) % 8 == 0 && ((kLdsNodeWords + kLdsChildWords) * 4) % 8 == 0, "LDS table alignment");

// SHARED: the whole batch uses one ruleset; its tables are copied to LDS once per
// workgroup (every thread reaches the barrier) and the scan reads them with ds_read.
template <bool SHARED>
__device__ __forceinline__ Tables stage_tables(const uint8_t* blob, uint32_t* s_tab, bool fast_ok) {
    Tables t = blob_tables(blob);
    if constexpr (SHARED) {
        const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
        if (fast_ok) {  // uniform over the workgroup
            const uint32_t nn = h->n_trie_nodes;
            const uint32_t wn = nn * (sizeof(TrieNode) / 4), wc = (nn - 1) * (sizeof(TrieChild) / 4);
            const uint32_t wk = (1u << h->key_slots_log2) * (sizeof(KeySlot) / 4);
            const uint32_t* gn = reinterpret_cast<const uint32_t*>(t.tn);
            const uint32_t* gc = reinterpret_cast<const uint32_t*>(t.tc);
            const uint32_t* gk = reinterpret_cast<const uint32_t*>(t.ks);
            for (uint32_t i = threadIdx.x; i < wn; i += blockDim.x) s_tab[i] = gn[i];
            for (uint32_t i = threadIdx.x; i < wc; i += blockDim.x) s_tab[kLdsNodeWords + i] = gc[i];
            for (uint32_t i = threadIdx.x; i < wk; i += blockDim.x) s_tab[kLdsNodeWords + kLdsChildWords + i] = gk[i];
        }
        __syncthreads();
        t.tn = reinterpret_cast<const TrieNode*>(s_tab);  // unconditionally LDS: ds_read in the scan
        t.tc = reinterpret_cast<const TrieChild*>(s_tab + kLdsNodeWords);
        t.ks = reinterpret_cast<const KeySlot*>(s_tab + kLdsNodeWords + kLdsChildWords);
    }
    return t;
}

// Stage A: structural scan -> capture rows (requests it can not handle -> slow list).
// SHARED: the whole batch uses sets[0]; its trie tables are copied to LDS once per
// workgroup so the token loop never touches global memory for them.
template <int MODE, bool SHARED>
__global__ __launch_bounds__(256) void ajx_scan_fast(const uint8_t* const* __restrict__ sets,
                                                     const uint32_t* __restrict__ set_of_req,
                                                     const uint8_t* __restrict__ arena,
                                                     const uint64_t* __restrict__ offs,
                                                     const uint32_t* __restrict__ lens, uint32_t n,
                                                     uint64_t* __restrict__ rows, uint32_t row_stride,
                                                     uint32_t* __restrict__ slow_count,
                                                     uint32_t* __restrict__ slow_ids) {
    __shared__ uint32_t s_tab[SHARED ? kLdsTabWords : 1];
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    const uint8_t* blob = sets[SHARED || !set_of_req ? 0 : (r < n ? set_of_req[r] : 0)];
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
    const bool fast_ok = (h->flags & kFlagFastOk) != 0;
    const Tables tab = stage_tables<SHARED>(blob, s_tab, fast_ok);
    if (r >= n) return;
    uint64_t* row = rows + (size_t)r * row_stride;
    const uint8_t* d = arena + offs[r];
    const uint32_t len = lens[r];
    bool ok = false;
    if (fast_ok && len < (1u << 24)) {
        const uint4* a4 = reinterpret_cast<const uint4*>(d - ((uintptr_t)d & 15u));
        ok = scan_doc<MODE>(blob, tab, d, len, row, [&](uint32_t b, uint32_t nblk) -> Block16 {
            if (b < nblk) {
                const uint4 v = a4[b];
                return Block16{v.x, v.y, v.z, v.w};
            }
            return Block16{0u, 0u, 0u, 0u};
        });
    } else {
        row[0] = kRowSlow;
    }
    if (!ok) slow_ids[atomicAdd(slow_count, 1u)] = r;
}

// Stages A+B fused: the patterns run right after the scan, while the request's value
// bytes are still in L2 / MALL (stage B alone re-reads them from HBM).
template <bool SHARED>
__global__ __launch_bounds__(256) void ajx_scan_fused(const uint8_t* const* __restrict__ sets,
                                                      const uint32_t* __restrict__ set_of_req,
                                                      const uint8_t* __restrict__ arena,
                                                      const uint64_t* __restrict__ offs,
                                                      const uint32_t* __restrict__ lens, uint32_t n,
                                                      uint64_t* __restrict__ rows, uint32_t row_stride,
                                                      uint32_t* __restrict__ slow_count,
                                                      uint32_t* __restrict__ slow_ids, uint8_t* __restrict__ out_tri,
                                                      int32_t* __restrict__ out_err, uint64_t* __restrict__ out_bm,
                                                      uint32_t stride) {
    __shared__ uint32_t s_tab[SHARED ? kLdsTabWords : 1];
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    const uint8_t* blob = sets[SHARED || !set_of_req ? 0 : (r < n ? set_of_req[r] : 0)];
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
    const bool fast_ok = (h->flags & kFlagFastOk) != 0;
    const Tables tab = stage_tables<SHARED>(blob, s_tab, fast_ok);
    if (r >= n) return;
    uint64_t* row = rows + (size_t)r * row_stride;
    const uint8_t* d = arena + offs[r];
    const uint32_t len = lens[r];
    bool ok = false;
    if (fast_ok && len < (1u << 24)) {
        const uint4* a4 = reinterpret_cast<const uint4*>(d - ((uintptr_t)d & 15u));
        ok = scan_doc<0>(blob, tab, d, len, row, [&](uint32_t b, uint32_t nblk) -> Block16 {
            if (b < nblk) {
                const uint4 v = a4[b];
                return Block16{v.x, v.y, v.z, v.w};
            }
            return Block16{0u, 0u, 0u, 0u};
        });
    }
    if (!ok) {
        slow_ids[atomicAdd(slow_count, 1u)] = r;
        return;
    }
    uint64_t t[2], u[2];
    patterns_from_row(blob, d, row, t, u);
    if (out_bm) {
        uint64_t* orow = out_bm + (size_t)r * stride;
        for (uint32_t w = 0; w < stride; w++) orow[w] = w < 2 ? t[w] : 0ull;
    }
    const uint32_t* code = reinterpret_cast<const uint32_t*>(blob + h->off_code);
    int32_t ep;
    const uint8_t tri = run_fold(code, h->n_code,
                                 [&](uint32_t p) -> uint8_t {
                                     const uint64_t bit = 1ull << (p & 63);
                                     const uint32_t k = p >> 6;
                                     if (h->static_error[k] & bit) return V_E;
                                     if (u[k] & bit) return V_U;
                                     return (t[k] & bit) ? V_T : V_F;
                                 },
                                 &ep);
    out_tri[r] = tri;
    if (out_err) out_err[r] = ep;
}

// Stage B: patterns on the captured values, T bitmap, And/Or fold
__global__ __launch_bounds__(256) void ajx_patterns(const uint8_t* const* __restrict__ sets,
                                                    const uint32_t* __restrict__ set_of_req,
                                                    const uint8_t* __restrict__ arena,
                                                    const uint64_t* __restrict__ offs, uint32_t n,
                                                    const uint64_t* __restrict__ rows, uint32_t row_stride,
                                                    uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err,
                                                    uint64_t* __restrict__ out_bm, uint32_t stride) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint64_t* row = rows + (size_t)r * row_stride;
    if (row[0] & kRowSlow) return;
    const uint8_t* blob = sets[set_of_req ? set_of_req[r] : 0];
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
    uint64_t t[2], u[2];
    patterns_from_row(blob, arena + offs[r], row, t, u);
    if (out_bm) {
        uint64_t* orow = out_bm + (size_t)r * stride;
        for (uint32_t w = 0; w < stride; w++) orow[w] = w < 2 ? t[w] : 0ull;
    }
    const uint32_t* code = reinterpret_cast<const uint32_t*>(blob + h->off_code);
    int32_t ep;
    const uint8_t tri = run_fold(code, h->n_code,
                                 [&](uint32_t p) -> uint8_t {
                                     const uint64_t bit = 1ull << (p & 63);
                                     const uint32_t k = p >> 6;
                                     if (h->static_error[k] & bit) return V_E;
                                     if (u[k] & bit) return V_U;
                                     return (t[k] & bit) ? V_T : V_F;
                                 },
                                 &ep);
    out_tri[r] = tri;
    if (out_err) out_err[r] = ep;
}

hipError_t launch_eval_scan(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, const uint8_t* d_arena,
                            const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n, uint8_t* d_tri,
                            int32_t* d_err, uint64_t* d_bm, uint32_t stride, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t block = 256;
    const uint32_t grid = (n + block - 1) / block;
    hipLaunchKernelGGL(ajx_eval_scan, dim3(grid), dim3(block), 0, stream, d_sets, d_set_of_req, d_arena, d_offs,
                       d_lens, n, d_tri, d_err, d_bm, stride);
    return hipGetLastError();
}

hipError_t launch_eval_fast(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, const uint8_t* d_arena,
                            const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n, uint8_t* d_tri,
                            int32_t* d_err, uint64_t* d_bm, uint32_t stride, uint64_t* d_rows, uint32_t row_stride,
                            uint32_t* d_slow_count, uint32_t* d_slow_ids, hipStream_t stream, int ablate) {
    if (n == 0) return hipSuccess;
    const uint32_t block = 256;
    const uint32_t grid = (n + block - 1) / block;
    hipError_t e = hipMemsetAsync(d_slow_count, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    const bool shared = d_set_of_req == nullptr;
#define AJX_SCAN(M, S)                                                                                      \
    hipLaunchKernelGGL((ajx_scan_fast<M, S>), dim3(grid), dim3(block), 0, stream, d_sets, d_set_of_req, d_arena, \
                       d_offs, d_lens, n, d_rows, row_stride, d_slow_count, d_slow_ids)
    if (ablate == 3 || ablate == 4) {
    } else if (ablate == 1) AJX_SCAN(1, true);
    else if (ablate == 2) AJX_SCAN(2, true);
    else if (shared) AJX_SCAN(0, true);
    else AJX_SCAN(0, false);
#undef AJX_SCAN
    if (ablate == 3 || ablate == 4) {  // fused A+B (4: per-request ruleset table)
        if (ablate == 3)
            hipLaunchKernelGGL((ajx_scan_fused<true>), dim3(grid), dim3(block), 0, stream, d_sets, d_set_of_req,
                               d_arena, d_offs, d_lens, n, d_rows, row_stride, d_slow_count, d_slow_ids, d_tri, d_err,
                               d_bm, stride);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        const uint32_t sgrid = grid < 2048 ? grid : 2048;
        hipLaunchKernelGGL(ajx_eval_scan_list, dim3(sgrid), dim3(block), 0, stream, d_sets, d_set_of_req, d_arena,
                           d_offs, d_lens, d_slow_count, d_slow_ids, d_tri, d_err, d_bm, stride);
        return hipGetLastError();
    }
    if (ablate) return hipGetLastError();  // profiling ablation: stage A only
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(ajx_patterns, dim3(grid), dim3(block), 0, stream, d_sets, d_set_of_req, d_arena, d_offs, n,
                       d_rows, row_stride, d_tri, d_err, d_bm, stride);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const uint32_t sgrid = grid < 2048 ? grid : 2048;
    hipLaunchKernelGGL(ajx_eval_scan_list, dim3(sgrid), dim3(block), 0, stream, d_sets, d_set_of_req, d_arena,
                       d_offs, d_lens, d_slow_count, d_slow_ids, d_tri, d_err, d_bm, stride);
    return hipGetLastError();
}

}  // namespace ajx
