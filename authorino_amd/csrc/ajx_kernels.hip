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

#include <atomic>

#include "ajx_fast.h"
#include "ajx_modifiers.h"
#include "ajx_stream.h"
#include "ajx_kernels.h"
#include "ajx_kcommon.h"

namespace ajx {


constexpr int kSelCache = 32;  // resolved selector values kept per request
constexpr int kPatCache = 64;  // pattern results kept per request for the fold

// MODS: the rulesets of the batch have modifier chains (ajx_modifiers.h; mb: the
// work-item's three text buffers, the caller's scratch)
template <bool MODS>
__device__ __forceinline__ void eval_scan_one(uint32_t r, const uint8_t* const* __restrict__ sets,
                                              const uint32_t* __restrict__ set_of_req,
                                              const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                                              const uint32_t* __restrict__ lens, uint8_t* __restrict__ out_tri,
                                              int32_t* __restrict__ out_err, uint64_t* __restrict__ out_bm,
                                              uint32_t stride, [[maybe_unused]] ModBufs* mb) {
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
        if (pt.state != P_OK) return eval_pattern<true>(blob, pt, doc, ValueRef{0, 0, T_NULL, 0});
        if constexpr (MODS) {
            const Selector& sl = sels[pt.selector];
            const ValueRef v = value_of(p);
            if (v.esc == kValList) {  // a "#." list (no modifier chain after it)
                const uint8_t* rd;
                ValueRef rv;
                if (!build_list(blob, sl, doc, v, *mb, &rd, &rv)) return V_U;
                return eval_pattern<true>(blob, pt, rd, rv);
            }
            if (sl.mod_count) {
                const uint8_t* rd;
                ValueRef rv;
                if (!apply_modifiers(blob, sl, doc, value_of(p), *mb, &rd, &rv)) return V_U;
                return eval_pattern<true>(blob, pt, rd, rv);
            }
        }
        return eval_pattern<true>(blob, pt, doc, value_of(p));
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
    if (cache_pat && !out_bm)
        for (uint32_t p = 0; p < np; p++) res[p] = eval(p);
    // one fold program per tree (a forest ruleset writes n_trees results per request)
    const uint32_t nt = h->pad1[0] ? h->pad1[0] : 1u;
    const uint32_t* rc = h->pad1[0] ? reinterpret_cast<const uint32_t*>(blob + h->pad1[1]) : nullptr;
    for (uint32_t k = 0; k < nt; k++) {
        const uint32_t* c = rc ? code + rc[2 * k] : code;
        const uint32_t len = rc ? rc[2 * k + 1] : h->n_code;
        int32_t ep;
        uint8_t t;
        if (cache_pat)
            t = run_fold(c, len, [&](uint32_t p) { return res[p]; }, &ep);
        else
            t = run_fold(c, len, eval, &ep);
        out_tri[(size_t)r * nt + k] = t;
        if (out_err) out_err[(size_t)r * nt + k] = ep;
    }
}

template <bool MODS>
__global__ __launch_bounds__(256) void ajx_eval_scan(const uint8_t* const* __restrict__ sets,
                                                     const uint32_t* __restrict__ set_of_req,
                                                     const uint8_t* __restrict__ arena,
                                                     const uint64_t* __restrict__ offs,
                                                     const uint32_t* __restrict__ lens, uint32_t n,
                                                     uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err,
                                                     uint64_t* __restrict__ out_bm, uint32_t stride) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    if constexpr (MODS) {
        ModBufs mb;
        eval_scan_one<true>(r, sets, set_of_req, arena, offs, lens, out_tri, out_err, out_bm, stride, &mb);
    } else {
        eval_scan_one<false>(r, sets, set_of_req, arena, offs, lens, out_tri, out_err, out_bm, stride, nullptr);
    }
}

// the slow list: grid-stride over the ids the fast kernel appended
template <bool MODS>
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
    if constexpr (MODS) {
        ModBufs mb;
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x)
            eval_scan_one<true>(slow_ids[i], sets, set_of_req, arena, offs, lens, out_tri, out_err, out_bm, stride,
                                &mb);
    } else {
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x)
            eval_scan_one<false>(slow_ids[i], sets, set_of_req, arena, offs, lens, out_tri, out_err, out_bm, stride,
                                 nullptr);
    }
}

// the exact scan over the slow list; the instance with modifier buffers when the batch's
// rulesets have modifier chains
static void launch_slow_list(bool mods, uint32_t sgrid, hipStream_t stream, const uint8_t* const* d_sets,
                             const uint32_t* d_set_of_req, const uint8_t* d_arena, const uint64_t* d_offs,
                             const uint32_t* d_lens, const uint32_t* d_slow_count, const uint32_t* d_slow_ids,
                             uint8_t* d_tri, int32_t* d_err, uint64_t* d_bm, uint32_t stride) {
    if (mods)
        hipLaunchKernelGGL(ajx_eval_scan_list<true>, dim3(sgrid), dim3(256), 0, stream, d_sets, d_set_of_req, d_arena,
                           d_offs, d_lens, d_slow_count, d_slow_ids, d_tri, d_err, d_bm, stride);
    else
        hipLaunchKernelGGL(ajx_eval_scan_list<false>, dim3(sgrid), dim3(256), 0, stream, d_sets, d_set_of_req, d_arena,
                           d_offs, d_lens, d_slow_count, d_slow_ids, d_tri, d_err, d_bm, stride);
}




// Stage A alone (profiling split / ablations): structural scan -> capture rows.
// MODE 1/2 are the loads-only / loads+classification ablations.
template <int MODE, bool SHARED>
__global__ __launch_bounds__(kFastMaxBlock, AJX_FAST_WAVES) void ajx_scan_fast(const uint8_t* const* __restrict__ sets,
                                                     const uint32_t* __restrict__ set_of_req,
                                                     const uint8_t* __restrict__ arena,
                                                     const uint64_t* __restrict__ offs,
                                                     const uint32_t* __restrict__ lens, uint32_t n,
                                                     uint64_t* __restrict__ rows, uint32_t row_stride,
                                                     uint32_t* __restrict__ slow_count,
                                                     uint32_t* __restrict__ slow_ids, uint32_t ring_off,
                                                     const uint32_t* __restrict__ perm) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t r = k < n ? (perm ? perm[k] : k) : 0u;
    const uint8_t* blob = stage_blob<SHARED>(sets[SHARED || !set_of_req ? 0 : set_of_req[r]]);
    if (k >= n) return;
    if (!scan_request<MODE>(blob, arena + offs[r], lens[r], rows + (size_t)r * row_stride, lane_ring(ring_off)))
        slow_ids[atomicAdd(slow_count, 1u)] = r;
}

// Stage B alone (profiling split): patterns on the captured values, bitmap, fold
template <bool SHARED>
__global__ __launch_bounds__(kFastMaxBlock) void ajx_patterns(const uint8_t* const* __restrict__ sets,
                                                    const uint32_t* __restrict__ set_of_req,
                                                    const uint8_t* __restrict__ arena,
                                                    const uint64_t* __restrict__ offs, uint32_t n,
                                                    const uint64_t* __restrict__ rows, uint32_t row_stride,
                                                    uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err,
                                                    uint64_t* __restrict__ out_bm, uint32_t stride) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    const uint8_t* blob = stage_blob<SHARED>(sets[SHARED || !set_of_req ? 0 : (r < n ? set_of_req[r] : 0)]);
    if (r >= n) return;
    const uint64_t* row = rows + (size_t)r * row_stride;
    if (row[0] & kRowSlow) return;
    (void)finish_request(r, blob, arena + offs[r], row, out_tri, out_err, out_bm, stride);  // (profiling split)
}

// The token-scanner single-pass kernel for multi-tenant batches without staging: stage A
// then stage B in the same work-item, every table read from global memory through the
// request's own ruleset. Requests stage A can not prove gjson-equivalent go to the slow list.
__global__ __launch_bounds__(kFastMaxBlock, AJX_FAST_WAVES) void ajx_scan_fused(const uint8_t* const* __restrict__ sets,
                                                      const uint32_t* __restrict__ set_of_req,
                                                      const uint8_t* __restrict__ arena,
                                                      const uint64_t* __restrict__ offs,
                                                      const uint32_t* __restrict__ lens, uint32_t n,
                                                      uint64_t* __restrict__ rows, uint32_t row_stride,
                                                      uint32_t* __restrict__ slow_count,
                                                      uint32_t* __restrict__ slow_ids, uint8_t* __restrict__ out_tri,
                                                      int32_t* __restrict__ out_err, uint64_t* __restrict__ out_bm,
                                                      uint32_t stride, uint32_t ring_off,
                                                      const uint32_t* __restrict__ perm) {
    // work-item k takes request perm[k] (length-bucketed order, see ajx_len_scatter) or k;
    // its capture row is row k of the wave-interleaved layout (wave_row)
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t r = k < n ? (perm ? perm[k] : k) : 0u;
    const uint8_t* blob = sets[set_of_req ? set_of_req[r] : 0];
    if (k >= n) return;
    const RowRef row = wave_row(rows, row_stride, k);
    const uint8_t* d = arena + offs[r];
    if (!scan_request<0>(blob, d, lens[r], row, lane_ring(ring_off))) {
        slow_ids[atomicAdd(slow_count, 1u)] = r;
        return;
    }
    if (!finish_request(r, blob, d, row, out_tri, out_err, out_bm, stride)) {
        row[0] = kRowSlow;
        slow_ids[atomicAdd(slow_count, 1u)] = r;
    }
}



// a stage-B list entry the stream could not prove (merge_slow): the exact scan decides it
constexpr uint32_t kStageExact = 1u << 31;

// The streaming kernel (ajx_stream.h): each wave takes a span of stream::kSpan requests in
// arena order and reads their bytes as one coalesced stream; a lane per request then folds
// the patterns the stream decided. Requests with a pattern left (a value to parse or
// unescape, a regex, a long value) go with their row (found word, records, the 4 eager
// words: row_stride >= 5 + n_rec, StreamHdr) to ajx_stream_finish through the stage-B list;
// requests it can not prove go to the slow list (the exact scan). keep_rows (forest
// rulesets, for authjx_select_from_eval_device): every request's row is written (slow
// ones: kRowSlow), those with an open record through stage B. Rows: the wave-interleaved
// layout at work-item r. Profiling: MODE 1 the structural pass only, 2 no fold.
// Dynamic LDS: [blob copy] [per wave: WaveLds, capture rows, eager decisions].
// MT (multi-tenant latency batches): one request per wave (per = 1) under its own
// ruleset sets[set_of_req[r]], its tables read from global memory (L2), no blob copy.
// LAT (small batches, no kept rows): a span that fit one step has its documents in LDS
// still, and its lanes run stage B there (finish_full on the ring); what that leaves goes
// to the exact scan through the stage-B list.
template <int MODE, bool MT = false, bool LAT = false>
__device__ __forceinline__ void stream_body(const uint8_t* const* __restrict__ sets,
                                                       const uint32_t* __restrict__ set_of_req,
                                                       const uint8_t* __restrict__ arena,
                                                       const uint64_t* __restrict__ offs,
                                                       const uint32_t* __restrict__ lens, uint32_t n,
                                                       uint32_t* __restrict__ slow_count,
                                                       uint32_t* __restrict__ slow_ids, uint32_t* __restrict__ stage_ids,
                                                       uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err,
                                                       uint64_t* __restrict__ out_bm, uint32_t stride, uint32_t wave_off,
                                                       uint32_t wave_bytes, uint64_t* __restrict__ rows_out,
                                                       uint32_t row_stride, uint32_t keep_rows, uint32_t per,
                                                       uint32_t merge_slow) {
    extern __shared__ uint4 s_stream_dyn[];
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
    const uint32_t span = blockIdx.x * (blockDim.x >> 6) + w;
    // (profiling, keep_rows bit 1: lane 0 of a one-request wave writes its phases' clock
    // counts over the request's bitmap word: blob copy | stream | stage B, 21 bits each, x16)
    const bool timing = (keep_rows & 2u) != 0;
    keep_rows &= 1u;
    const uint64_t c0 = timing ? __builtin_readcyclecounter() : 0ull;
    uint64_t c1 = 0, c2 = 0;
    const uint8_t* blob;
    uint8_t* base;
    if constexpr (MT) {
        // per wave: [its ruleset's blob, when it fits wave_off bytes] [WaveLds, rows]
        if (span >= n) return;  // (wave-uniform; per = 1)
        const uint8_t* g = sets[set_of_req[span]];
        uint8_t* wb = reinterpret_cast<uint8_t*>(s_stream_dyn) + w * wave_bytes;
        const uint32_t tb = lean::uni(reinterpret_cast<const RulesetHdr*>(g)->total_bytes);  // (x16)
        if (tb <= wave_off) {
            copy_words_reg(reinterpret_cast<uint4*>(wb), reinterpret_cast<const uint4*>(g), tb / 16u, l, 64u);
            wave::sync();
            blob = wb;
        } else {
            blob = g;
        }
        base = wb + wave_off;
    } else {
        blob = stage_blob<true>(sets[0]);
        base = reinterpret_cast<uint8_t*>(s_stream_dyn) + wave_off + w * wave_bytes;
    }
    stream::WaveLds& L = *reinterpret_cast<stream::WaveLds*>(base);
    uint64_t* rows = reinterpret_cast<uint64_t*>(base + sizeof(stream::WaveLds));
    if (span * per >= n) return;  // (wave-uniform)
    if (timing) c1 = __builtin_readcyclecounter();
    const uint64_t *rowp = nullptr, *dwp = nullptr;
    const uint8_t* lds_doc = nullptr;
    uint64_t* ck = L.clk;  // (timing: the step's and stage B's phase clocks)
    if (timing) {
        if (l < 9) ck[l] = 0;
        wave::sync();
    }
    const uint32_t res = stream::scan_span<MODE>(L, rows, blob, arena, offs, lens, n, span, per, l, out_tri, out_err,
                                                 out_bm, stride, &rowp, &dwp, LAT ? &lds_doc : nullptr,
                                                 timing ? ck : nullptr);
    const uint32_t r = span * per + l;
    if (timing) c2 = __builtin_readcyclecounter();
    auto times = [&](uint32_t rq) {
        if (!timing || l != 0 || !out_bm) return;
        const uint64_t c3 = __builtin_readcyclecounter();
        auto f = [](uint64_t a, uint64_t b) { return ((b - a) >> 4) & 0x1FFFFFull; };
        uint64_t* o = out_bm + (size_t)rq * stride;
        o[0] = f(c0, c1) | (f(c1, c2) << 21) | (f(c2, c3) << 42);
        if (stride >= 4 && ck[0] && ck[8]) {  // (the sub-phases: step 0..3, stage B 5..8)
            o[1] = f(c1, ck[0]) | (f(ck[0], ck[1]) << 21) | (f(ck[1], ck[2]) << 42);
            o[2] = f(ck[2], ck[3]) | (f(ck[3], c2) << 21) | (f(c2, ck[5]) << 42);
            o[3] = f(ck[5], ck[6]) | (f(ck[6], ck[7]) << 21) | (f(ck[7], ck[8]) << 42);
        }
    };
    if constexpr (LAT) {
        // one request per wave: every lane takes part in its stage B (finish_full<true>)
        if (per == 1 && wave::readlane(res == stream::R_STAGE_B && lds_doc ? 1u : 0u, 0) != 0) {
            auto bcast = [](const void* q) {  // lane 0's pointer
                const uint64_t v = (uint64_t)(uintptr_t)q;
                return (uintptr_t)((uint64_t)wave::readlane((uint32_t)v, 0) |
                                   ((uint64_t)wave::readlane((uint32_t)(v >> 32), 0) << 32));
            };
            const uint8_t* d0 = reinterpret_cast<const uint8_t*>(bcast(lds_doc));
            const uint64_t* row0 = reinterpret_cast<const uint64_t*>(bcast(rowp));
            const uint64_t* dw0 = reinterpret_cast<const uint64_t*>(bcast(dwp));
            const uint32_t r0 = span;
            const bool ok = stream::finish_full<true>(r0, blob, d0, lens[r0], RowRef(row0), out_tri, out_err, out_bm,
                                                      stride, dw0, timing ? ck : nullptr);
            if (!ok && l == 0) {
                atomicAdd(slow_count, 1u);
                stage_ids[atomicAdd(slow_count + 1, 1u)] = r0 | kStageExact;
            }
            times(r0);
            return;
        }
    }
    if (l >= per || r >= n || MODE != 0) return;
    if constexpr (LAT) {
        if (res == stream::R_STAGE_B && lds_doc) {
            if (!stream::finish_full(r, blob, lds_doc, lens[r], RowRef(rowp), out_tri, out_err, out_bm, stride,
                                     dwp)) {
                atomicAdd(slow_count, 1u);
                stage_ids[atomicAdd(slow_count + 1, 1u)] = r | kStageExact;
            }
            return;
        }
    }
    const RowRef o = wave_row(rows_out, row_stride, r);
    if (res == stream::R_SLOW) {
        // (merge_slow: the stage-B kernel runs its exact scan, flagged on the stage-B list)
        if (merge_slow) {
            atomicAdd(slow_count, 1u);
            stage_ids[atomicAdd(slow_count + 1, 1u)] = r | kStageExact;
        } else {
            slow_ids[atomicAdd(slow_count, 1u)] = r;
        }
        if (keep_rows) o[0] = kRowSlow;
        return;
    }
    // (the records: the selectors', then exact selectors' prefixes')
    const RulesetHdr* hb = reinterpret_cast<const RulesetHdr*>(blob);
    const uint32_t ns = reinterpret_cast<const StreamHdr*>(blob + hb->off_stream)->n_rec;
    bool open = false;
    if (keep_rows)
        for (uint32_t s = 0; s < ns; s++) open = open || ((rowp[1u + s] >> 32) & stream::kOpenEnd);
    if (res == stream::R_STAGE_B || open) {
        for (uint32_t s = 0; s <= ns; s++) o[s] = rowp[s];
        for (uint32_t k = 0; k < 4; k++) o[1u + ns + k] = dwp[k];
        stage_ids[atomicAdd(slow_count + 1, 1u)] = r;  // (the stage-B count follows the slow count)
    } else if (keep_rows) {
        for (uint32_t s = 0; s <= ns; s++) o[s] = rowp[s];
    }
}

// The stage-B list of a small batch, run by the wave that finished last: a call, not
// inlined, so that the exact scan's registers stay out of the walk's own allocation (the
// inlined list took the kernel to 256 VGPRs, AGPR spills and ~1,400 SGPR spills)
template <bool MT>
__device__ __noinline__ void stream_fin_list(const uint8_t* const* __restrict__ sets,
                                             const uint32_t* __restrict__ set_of_req,
                                             const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                                             const uint32_t* __restrict__ lens, uint32_t cnt,
                                             uint32_t* __restrict__ slow_count, const uint32_t* __restrict__ stage_ids,
                                             uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err,
                                             uint64_t* __restrict__ out_bm, uint32_t stride,
                                             uint64_t* __restrict__ rows_out, uint32_t row_stride, uint32_t l) {
    for (uint32_t i = l; i < cnt; i += 64u) {
        const uint32_t e = stage_ids[i];
        const uint32_t r = e & ~kStageExact;
        const uint8_t* blob = sets[MT ? set_of_req[r] : 0];
        bool ok = false;
        if (!(e & kStageExact)) {
            ok = stream::finish_full(r, blob, arena + offs[r], lens[r], wave_row(rows_out, row_stride, r), out_tri,
                                     out_err, out_bm, stride);
            if (!ok) atomicAdd(slow_count, 1u);
        }
        if (!ok)
            eval_scan_one<false>(r, sets, MT ? set_of_req : nullptr, arena, offs, lens, out_tri, out_err, out_bm,
                                 stride, nullptr);
    }
}

// The kernel: the span's walk (stream_body), then, with FIN (a small batch without
// modifier chains), the stage-B list in the wave that finishes last: the requests left to
// the exact scan and those whose stage B could not run on the LDS copy — no second launch.
// slow_count[2] counts the finished waves.
template <int MODE, bool MT = false, bool LAT = false, bool FIN = false>
__global__ __launch_bounds__(256) void ajx_scan_stream(const uint8_t* const* __restrict__ sets,
                                                       const uint32_t* __restrict__ set_of_req,
                                                       const uint8_t* __restrict__ arena,
                                                       const uint64_t* __restrict__ offs,
                                                       const uint32_t* __restrict__ lens, uint32_t n,
                                                       uint32_t* __restrict__ slow_count,
                                                       uint32_t* __restrict__ slow_ids, uint32_t* __restrict__ stage_ids,
                                                       uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err,
                                                       uint64_t* __restrict__ out_bm, uint32_t stride, uint32_t wave_off,
                                                       uint32_t wave_bytes, uint64_t* __restrict__ rows_out,
                                                       uint32_t row_stride, uint32_t keep_rows, uint32_t per,
                                                       uint32_t merge_slow) {
    stream_body<MODE, MT, LAT>(sets, set_of_req, arena, offs, lens, n, slow_count, slow_ids, stage_ids, out_tri,
                               out_err, out_bm, stride, wave_off, wave_bytes, rows_out, row_stride, keep_rows, per,
                               merge_slow);
    if constexpr (FIN) {
        const uint32_t l = threadIdx.x & 63u;
        __threadfence();  // (this wave's stage-B list entries and rows, before its count)
        uint32_t last = 0;
        if (l == 0) last = atomicAdd(slow_count + 2, 1u) + 1u == gridDim.x * (blockDim.x >> 6) ? 1u : 0u;
        if (!wave::readlane(last, 0)) return;
        __threadfence();
        const uint32_t cnt = __hip_atomic_load(slow_count + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cnt)
            stream_fin_list<MT>(sets, set_of_req, arena, offs, lens, cnt, slow_count, stage_ids, out_tri, out_err,
                                out_bm, stride, rows_out, row_stride, l);
        // every other wave is done with the counters: back to zero for the next launch on
        // this stream (no fill before it), the slow count kept at [3] for the host
        __threadfence();
        if (l == 0) {
            slow_count[3] = __hip_atomic_load(slow_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            slow_count[0] = 0;
            slow_count[1] = 0;
            slow_count[2] = 0;
        }
    }
}

// Stage B of the streaming kernel: one work-item per request on the stage-B list, on its
// row in HBM (stream::finish_full); what it can not decide goes to the slow list. MT: each
// request's own ruleset, read from global memory. EXACT (small batches, one launch fewer):
// the exact scan runs here, for the requests the stream flagged (kStageExact) and for those
// stage B can not decide; 1 without, 2 with modifier buffers.
template <bool MT = false, int EXACT = 0>
__global__ __launch_bounds__(256) void ajx_stream_finish(const uint8_t* const* __restrict__ sets,
                                                         const uint32_t* __restrict__ set_of_req,
                                                         const uint8_t* __restrict__ arena,
                                                         const uint64_t* __restrict__ offs,
                                                         const uint32_t* __restrict__ lens,
                                                         const uint32_t* __restrict__ stage_ids,
                                                         uint64_t* __restrict__ rows, uint32_t row_stride,
                                                         uint32_t* __restrict__ slow_count,
                                                         uint32_t* __restrict__ slow_ids, uint8_t* __restrict__ out_tri,
                                                         int32_t* __restrict__ out_err, uint64_t* __restrict__ out_bm,
                                                         uint32_t stride) {
    const uint8_t* blob0 = MT ? nullptr : stage_blob<true>(sets[0]);
    const uint32_t cnt = slow_count[1];  // (the stage-B count)
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
        const uint32_t e = stage_ids[i];
        const uint32_t r = e & ~kStageExact;
        const uint8_t* blob = MT ? sets[set_of_req[r]] : blob0;
        bool ok = false;
        if (!(e & kStageExact))
            ok = stream::finish_full(r, blob, arena + offs[r], lens[r], wave_row(rows, row_stride, r), out_tri,
                                     out_err, out_bm, stride);
        if (ok) continue;
        if constexpr (EXACT == 0) {
            slow_ids[atomicAdd(slow_count, 1u)] = r;
        } else {
            if (!(e & kStageExact)) atomicAdd(slow_count, 1u);
            if constexpr (EXACT == 2) {
                ModBufs mb;
                eval_scan_one<true>(r, sets, set_of_req, arena, offs, lens, out_tri, out_err, out_bm, stride, &mb);
            } else {
                eval_scan_one<false>(r, sets, set_of_req, arena, offs, lens, out_tri, out_err, out_bm, stride,
                                     nullptr);
            }
        }
    }
}

bool stream_eligible(const uint8_t* host_blob, uint32_t blob_bytes) {
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(host_blob);
    return h->off_stream != 0 && blob_bytes <= kMaxSharedBlobBytes && (h->flags & kFlagFastOk) &&
           h->n_selectors <= kFastMaxSelectors;
}

uint32_t stream_records(const uint8_t* host_blob) {
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(host_blob);
    return h->off_stream ? reinterpret_cast<const StreamHdr*>(host_blob + h->off_stream)->n_rec : h->n_selectors;
}

static_assert(kStreamSpan == stream::kSpan, "requests per wave");

// 4-wave workgroups (the kernel's launch bounds), each with its own blob copy
constexpr uint32_t kStreamBlock = 256;
// the largest batch whose stage-B list the last wave runs itself (FIN): at most 8 list
// entries per lane
constexpr uint32_t kFinMaxN = 512;

hipError_t launch_eval_stream(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, uint32_t blob_bytes,
                              uint32_t n_rec, const uint8_t* d_arena, const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n,
                              uint8_t* d_tri, int32_t* d_err, uint64_t* d_bm, uint32_t stride, uint64_t* d_rows,
                              uint32_t row_stride, bool keep_rows, uint32_t* d_stage_ids, uint32_t* d_slow_count,
                              uint32_t* d_slow_ids, hipStream_t stream, int mode, bool mods, uint32_t per,
                              bool* counters_zero) {
    const bool was_zero = counters_zero && *counters_zero;
    if (counters_zero) *counters_zero = false;
    if (n == 0) return hipSuccess;
    if (row_stride < 5u + n_rec) return hipErrorInvalidValue;
    const bool mt = d_set_of_req != nullptr;
    const bool timing = mode == 3;  // (profiling: the LAT instance's phase clocks, §ajx_scan_stream)
    if (timing) mode = 0;
    if (mt) {
        if (mode != 0) return hipErrorInvalidValue;
        per = 1;
    }
    uint32_t wave_off = (blob_bytes + 15u) & ~15u;
    uint32_t wave_bytes = (stream::lds_bytes(n_rec) + 15u) & ~15u;
    if (mt) {
        // each wave copies its own ruleset's blob next to its LDS when it fits (blob_bytes:
        // the batch's largest), else reads it from global memory: wave_off is that room
        const uint32_t room = 160u * 1024u / (kStreamBlock / 64u);
        uint32_t cap = wave_off;
        if (cap + wave_bytes > room) cap = room > wave_bytes ? (room - wave_bytes) & ~15u : 0u;
        if (cap < 1024u) cap = 0;
        wave_off = cap;
        wave_bytes += cap;
    }
    const uint32_t block = kStreamBlock;
    const uint32_t lds = (mt ? 0u : wave_off) + (block / 64) * wave_bytes;
    if (lds > 160u * 1024u) return hipErrorInvalidValue;
    if (per == 0 || per > stream::kSpan) per = stream::kSpan;
    // a small batch (fewer requests per wave, or one per wave under its own ruleset): stage B
    // runs the exact scan too (one launch fewer on the latency path)
    const bool merge = mt || per < stream::kSpan;
    const uint32_t spans = (n + per - 1) / per;
    const uint32_t grid = (spans + block / 64 - 1) / (block / 64);
    // (one fill: the slow count, the stage-B count and the finished-wave count after it;
    // none after a FIN launch on this stream, whose last wave cleared them)
    hipError_t e = hipSuccess;
    if (!was_zero && (e = hipMemsetAsync(d_slow_count, 0, 3 * sizeof(uint32_t), stream)) != hipSuccess) return e;
    static std::atomic<uint64_t> attr_done{0};
    e = attr_once(attr_done, [] {
        for (const void* k : {reinterpret_cast<const void*>(&ajx_scan_stream<0>),
                              reinterpret_cast<const void*>(&ajx_scan_stream<1>),
                              reinterpret_cast<const void*>(&ajx_scan_stream<2>),
                              reinterpret_cast<const void*>(&ajx_scan_stream<0, true>),
                              reinterpret_cast<const void*>(&ajx_scan_stream<0, false, true>),
                              reinterpret_cast<const void*>(&ajx_scan_stream<0, true, true>),
                              reinterpret_cast<const void*>(&ajx_scan_stream<0, false, true, true>),
                              reinterpret_cast<const void*>(&ajx_scan_stream<0, true, true, true>),
                              reinterpret_cast<const void*>(&ajx_stream_finish<false>),
                              reinterpret_cast<const void*>(&ajx_stream_finish<false, 1>),
                              reinterpret_cast<const void*>(&ajx_stream_finish<false, 2>),
                              reinterpret_cast<const void*>(&ajx_stream_finish<true, 1>),
                              reinterpret_cast<const void*>(&ajx_stream_finish<true, 2>)}) {
            // (the dynamic ceiling is what the kernel's static LDS leaves of the CU's 160 KiB:
            // stage B's per-thread buffers are static)
            hipFuncAttributes fa;
            hipError_t r = hipFuncGetAttributes(&fa, k);
            if (r != hipSuccess) return r;
            r = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    160 * 1024 - (int)fa.sharedSizeBytes);
            if (r != hipSuccess) return r;
        }
        return hipSuccess;
    });
    if (e != hipSuccess) return e;
#define AJX_STREAM_LAUNCH(M, T, LT, F)                                                                        \
    hipLaunchKernelGGL((ajx_scan_stream<M, T, LT, F>), dim3(grid), dim3(block), lds, stream, d_sets, d_set_of_req,  \
                       d_arena, \
                       d_offs, d_lens, n, \
                       d_slow_count, d_slow_ids, d_stage_ids, d_tri, d_err, d_bm, stride, wave_off, wave_bytes,       \
                       d_rows, row_stride, (keep_rows ? 1u : 0u) | (timing ? 2u : 0u), per, merge ? 1u : 0u)
    const bool lat = merge && !keep_rows;
    // (stage B and the exact scan in the last wave: no second launch). Only for batches of at
    // most kFinMaxN requests: that wave walks the list 64 entries at a time, so a large batch
    // of requests the stream cannot finish (long or deeply nested documents) would put
    // thousands of exact scans behind one wave; larger batches take the grid-stride
    // ajx_stream_finish launch
    const bool fin = lat && !mods && n <= kFinMaxN;
    if (mt && fin)
        AJX_STREAM_LAUNCH(0, true, true, true);
    else if (mt && lat)
        AJX_STREAM_LAUNCH(0, true, true, false);
    else if (mt)
        AJX_STREAM_LAUNCH(0, true, false, false);
    else if (mode == 1)
        AJX_STREAM_LAUNCH(1, false, false, false);
    else if (mode == 2)
        AJX_STREAM_LAUNCH(2, false, false, false);
    else if (fin)
        AJX_STREAM_LAUNCH(0, false, true, true);
    else if (lat)
        AJX_STREAM_LAUNCH(0, false, true, false);
    else
        AJX_STREAM_LAUNCH(0, false, false, false);
#undef AJX_STREAM_LAUNCH
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (counters_zero) *counters_zero = fin && (mt || (mode != 1 && mode != 2));
    if (mode != 0 || fin) return hipSuccess;
    // stage B and the exact scan over their lists (grid-stride: the lists' lengths are on the device)
    const uint32_t fgrid = n < 2048u * 256u ? (n + 255) / 256 : 4096;
#define AJX_FINISH_LAUNCH(T, X, LDS)                                                                              \
    hipLaunchKernelGGL((ajx_stream_finish<T, X>), dim3(fgrid), dim3(256), LDS, stream, d_sets,                    \
                       T ? d_set_of_req : nullptr, d_arena, d_offs, d_lens, d_stage_ids, d_rows, row_stride,      \
                       d_slow_count, d_slow_ids, d_tri, d_err, d_bm, stride)
    if (mt && mods)
        AJX_FINISH_LAUNCH(true, 2, 0);
    else if (mt)
        AJX_FINISH_LAUNCH(true, 1, 0);
    else if (merge && mods)
        AJX_FINISH_LAUNCH(false, 2, wave_off);
    else if (merge)
        AJX_FINISH_LAUNCH(false, 1, wave_off);
    else
        AJX_FINISH_LAUNCH(false, 0, wave_off);
#undef AJX_FINISH_LAUNCH
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (merge) return hipSuccess;
    const uint32_t sgrid = n < 1024u * 128u ? 2 * ((n + 255) / 256) : 4096;
    launch_slow_list(mods, sgrid, stream, d_sets, d_set_of_req, d_arena, d_offs, d_lens, d_slow_count, d_slow_ids, d_tri,
                     d_err, d_bm, stride);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// Length bucketing: a wave of the single-pass kernel runs each window's token loop as
// long as its busiest lane, and the whole document loop as long as its longest
// document, so the 64 requests of a wave should have similar lengths. A counting sort
// by 8-byte length class (longest first; documents over 8 KiB share the last class)
// gives the order work-items take requests in; outputs still go to each request's own
// index. Three small launches over lens[] (4 B
// per request each).
// ---------------------------------------------------------------------------------
constexpr uint32_t kLenBuckets = 1024;

__device__ __forceinline__ uint32_t len_bucket(uint32_t len) {
    const uint32_t b = len >> 3;
    return kLenBuckets - 1u - (b < kLenBuckets ? b : kLenBuckets - 1u);
}

__global__ __launch_bounds__(kLenBuckets) void ajx_len_hist(const uint32_t* __restrict__ lens, uint32_t n,
                                                            uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kLenBuckets];
    h[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        atomicAdd(&h[len_bucket(lens[i])], 1u);
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

// exclusive scan of the histogram into per-class cursors (one workgroup).
// cursor[kLenBuckets] = 1 when the lengths span fewer than kLenSpreadMin classes: the
// order would not even out the waves (and scatters the outputs), so the scatter writes
// the identity instead.
constexpr uint32_t kLenSpreadMin = 32;  // 256 bytes
__global__ __launch_bounds__(kLenBuckets) void ajx_len_scan(const uint32_t* __restrict__ hist,
                                                            uint32_t* __restrict__ cursor) {
    __shared__ uint32_t s[kLenBuckets];
    __shared__ uint32_t lo, hi;
    const uint32_t t = threadIdx.x;
    const uint32_t own = hist[t];
    if (t == 0) {
        lo = kLenBuckets;
        hi = 0;
    }
    s[t] = own;
    __syncthreads();
    if (own) {
        atomicMin(&lo, t);
        atomicMax(&hi, t);
    }
    for (uint32_t o = 1; o < kLenBuckets; o <<= 1) {
        const uint32_t v = t >= o ? s[t - o] : 0u;
        __syncthreads();
        s[t] += v;
        __syncthreads();
    }
    cursor[t] = s[t] - own;
    if (t == 0) cursor[kLenBuckets] = (hi < lo || hi - lo < kLenSpreadMin) ? 1u : 0u;
}

// perm[cursor[class] + rank] = request; one global atomic per (workgroup, class).
// pos_of (optional): pos_of[request] = its work-item, written in request order (coalesced),
// for the gather that puts work-item-ordered outputs back in request order (ajx_unpermute)
__global__ __launch_bounds__(kLenBuckets) void ajx_len_scatter(const uint32_t* __restrict__ lens, uint32_t n,
                                                               uint32_t* __restrict__ cursor,
                                                               uint32_t* __restrict__ perm,
                                                               uint32_t* __restrict__ pos_of) {
    __shared__ uint32_t cnt[kLenBuckets];
    __shared__ uint32_t base[kLenBuckets];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (cursor[kLenBuckets]) {  // narrow length spread: keep the caller's order
        if (i < n) {
            perm[i] = i;
            if (pos_of) pos_of[i] = i;
        }
        return;
    }
    cnt[threadIdx.x] = 0;
    __syncthreads();
    uint32_t b = 0, rank = 0;
    if (i < n) {
        b = len_bucket(lens[i]);
        rank = atomicAdd(&cnt[b], 1u);
    }
    __syncthreads();
    if (cnt[threadIdx.x]) base[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], cnt[threadIdx.x]);
    __syncthreads();
    if (i < n) {
        perm[base[b] + rank] = i;
        if (pos_of) pos_of[i] = base[b] + rank;
    }
}

// outputs written in work-item order (t_*) back to request order: request i's results are
// work-item pos_of[i]'s. One thread per request, so the stores are coalesced; the loads are
// a gather over the work-item-ordered copies (n x (n_out x 5 + stride x 8) bytes, mostly
// still in L2 / MALL behind the kernel that wrote them).
__global__ __launch_bounds__(256) void ajx_unpermute(const uint32_t* __restrict__ pos_of, uint32_t n, uint32_t n_out,
                                                     uint32_t stride, const uint8_t* __restrict__ t_tri,
                                                     const int32_t* __restrict__ t_err,
                                                     const uint64_t* __restrict__ t_bm, uint8_t* __restrict__ tri,
                                                     int32_t* __restrict__ err, uint64_t* __restrict__ bm) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const size_t j = pos_of[i];
    for (uint32_t q = 0; q < n_out; q++) {
        tri[(size_t)i * n_out + q] = t_tri[j * n_out + q];
        if (err) err[(size_t)i * n_out + q] = t_err[j * n_out + q];
    }
    if (bm)
        for (uint32_t w = 0; w < stride; w++) bm[(size_t)i * stride + w] = t_bm[j * stride + w];
}

hipError_t launch_len_order(const uint32_t* d_lens, uint32_t n, uint32_t* d_hist, uint32_t* d_perm,
                            hipStream_t stream, uint32_t* d_pos_of) {
    hipError_t e = hipMemsetAsync(d_hist, 0, (2 * kLenBuckets + 1) * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    const uint32_t blocks = (n + kLenBuckets - 1) / kLenBuckets;
    hipLaunchKernelGGL(ajx_len_hist, dim3(blocks < 512 ? blocks : 512), dim3(kLenBuckets), 0, stream, d_lens, n,
                       d_hist);
    hipLaunchKernelGGL(ajx_len_scan, dim3(1), dim3(kLenBuckets), 0, stream, d_hist, d_hist + kLenBuckets);
    hipLaunchKernelGGL(ajx_len_scatter, dim3(blocks), dim3(kLenBuckets), 0, stream, d_lens, n, d_hist + kLenBuckets,
                       d_perm, d_pos_of);
    return hipGetLastError();
}

// gjson.Get per pattern selector (the response / header selectors of SURVEY.md §8 a14):
// one work-item per request, the exact device Get (gj_get) for each of the ruleset's
// patterns; out[r * stride + p] = {start (relative to the document), len, type, esc}.
// An UNSUPPORTED selector reports type 0xFF. TEXT: a selector with modifiers and a "#."
// list resolve to built text, copied into the request's slot text[r * text_stride ...]
// (select_value, ajx_modifiers.h; 0xFF when it does not fit); without TEXT they report
// 0xFF (the capture-row path of select_from_eval).
template <bool TEXT>
__global__ __launch_bounds__(256) void ajx_select_values(const uint8_t* const* __restrict__ sets,
                                                         const uint32_t* __restrict__ set_of_req,
                                                         const uint8_t* __restrict__ arena,
                                                         const uint64_t* __restrict__ offs,
                                                         const uint32_t* __restrict__ lens, uint32_t n,
                                                         uint32_t* __restrict__ out, uint32_t stride,
                                                         const uint64_t* __restrict__ rows, uint32_t row_stride,
                                                         uint32_t p0, const uint32_t* __restrict__ perm,
                                                         uint32_t wave_rows, uint8_t* __restrict__ text,
                                                         uint32_t text_stride) {
    // work-item k: request perm[k] (the order the rows were written in) or k; its row is
    // row k of the wave-interleaved layout (wave_rows: the fused kernels') or row r
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t r = perm ? perm[k] : k;
    // the single-pass scan's capture row when it has one (not on the slow list)
    const RowRef row = !rows ? RowRef() : wave_rows ? wave_row(const_cast<uint64_t*>(rows), row_stride, k)
                                                    : RowRef(rows + (size_t)r * row_stride);
    const uint64_t found = rows ? row[0] : kRowSlow;
    const uint8_t* blob = sets[set_of_req ? set_of_req[r] : 0];
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
    const Selector* sels = reinterpret_cast<const Selector*>(blob + h->off_selectors);
    const Component* comps = reinterpret_cast<const Component*>(blob + h->off_components);
    const Pattern* pats = reinterpret_cast<const Pattern*>(blob + h->off_patterns);
    const uint8_t* lits = blob + h->off_literals;
    const uint8_t* doc = arena + offs[r];
    const uint32_t len = lens[r];
    // patterns [p0, p0 + stride): the whole ruleset (p0 = 0) or, after a forest
    // evaluation, the response selectors compiled as its last tree
    const uint32_t avail = h->n_patterns > p0 ? h->n_patterns - p0 : 0u;
    const uint32_t np = avail < stride ? avail : stride;
    [[maybe_unused]] uint32_t used = 0;  // (TEXT: bytes of the request's text slot taken)
    for (uint32_t q = 0; q < np; q++) {
        const uint32_t p = p0 + q;
        uint32_t* o = out + ((size_t)r * stride + q) * 3;
        const uint32_t si = pats[p].selector;
        if (pats[p].state == P_UNSUPPORTED || (!TEXT && sels[si].mod_count)) {
            o[0] = 0;
            o[1] = 0;
            o[2] = 0xFFu;
            continue;
        }
        if constexpr (TEXT) {
            if (sels[si].mod_count) {
                ModBufs mb;
                if (!select_value(blob, sels[si], doc, len, mb, text + (size_t)r * text_stride, text_stride, &used, o))
                    o[0] = 0, o[1] = 0, o[2] = 0xFFu;
                continue;
            }
        }
        if (!(found & kRowSlow)) {
            if ((found >> si) & 1u) {
                const uint64_t rec = row[1 + si];
                const uint32_t meta = (uint32_t)(rec >> 32);
                o[0] = (uint32_t)rec;
                o[1] = meta & 0xFFFFFFu;
                o[2] = ((meta >> 24) & 7u) | (((meta >> 27) & 1u) << 8);
            } else {
                o[0] = 0;
                o[1] = 0;
                o[2] = T_NULL;
            }
            continue;
        }
        const Selector& sl = sels[si];
        const ValueRef v = gj_get(doc, len, comps + sl.comp_begin, sl.comp_count, lits);
        o[0] = v.start;
        o[1] = v.end - v.start;
        o[2] = (uint32_t)v.type | ((uint32_t)v.esc << 8);
        if (v.esc == kValList) {  // a "#." list: built text (without TEXT: not selectable)
            o[2] = 0xFFu;
            if constexpr (TEXT) {
                ModBufs mb;
                if (!select_value(blob, sl, doc, len, mb, text + (size_t)r * text_stride, text_stride, &used, o))
                    o[0] = 0, o[1] = 0, o[2] = 0xFFu;
            }
        }
    }
}

hipError_t launch_select(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, uint32_t shared_blob_bytes,
                         const uint8_t* d_arena, const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n,
                         uint32_t* d_out, uint32_t stride, uint64_t* d_rows, uint32_t row_stride,
                         uint32_t* d_slow_count, uint32_t* d_slow_ids, const uint32_t* d_perm, uint8_t* d_text,
                         uint32_t text_stride, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (d_rows) {  // stage A of the single-pass kernel captures every selector's span
        const bool shared = shared_blob_bytes != 0 && d_set_of_req == nullptr;
        const uint32_t fblock = shared ? fast_block(shared_blob_bytes) : kFastBlock;
        const uint32_t fgrid = (n + fblock - 1) / fblock;
        const uint32_t ring_off = shared ? (shared_blob_bytes + 15u) & ~15u : 0u;
        const uint32_t lds = ring_off + (fblock / 64) * kWinRingBytesPerWave;
        hipError_t e = hipMemsetAsync(d_slow_count, 0, sizeof(uint32_t), stream);
        if (e != hipSuccess) return e;
        static std::atomic<uint64_t> attr_done{0};
        e = attr_once(attr_done, [] {
            const void* ks[] = {reinterpret_cast<const void*>(&ajx_scan_fast<0, true>),
                                reinterpret_cast<const void*>(&ajx_scan_fast<0, false>)};
            for (const void* k : ks) {
                const hipError_t r = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                if (r != hipSuccess) return r;
            }
            return hipSuccess;
        });
        if (e != hipSuccess) return e;
        if (shared)
            hipLaunchKernelGGL((ajx_scan_fast<0, true>), dim3(fgrid), dim3(fblock), lds, stream, d_sets, d_set_of_req,
                               d_arena, d_offs, d_lens, n, d_rows, row_stride, d_slow_count, d_slow_ids, ring_off,
                               d_perm);
        else
            hipLaunchKernelGGL((ajx_scan_fast<0, false>), dim3(fgrid), dim3(fblock), lds, stream, d_sets,
                               d_set_of_req, d_arena, d_offs, d_lens, n, d_rows, row_stride, d_slow_count, d_slow_ids,
                               ring_off, d_perm);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const uint32_t block = 256;
    const uint32_t grid = (n + block - 1) / block;
    if (d_text)
        hipLaunchKernelGGL(ajx_select_values<true>, dim3(grid), dim3(block), 0, stream, d_sets, d_set_of_req, d_arena,
                           d_offs, d_lens, n, d_out, stride, d_rows, row_stride, 0u, nullptr, 0u, d_text, text_stride);
    else
        hipLaunchKernelGGL(ajx_select_values<false>, dim3(grid), dim3(block), 0, stream, d_sets, d_set_of_req, d_arena,
                           d_offs, d_lens, n, d_out, stride, d_rows, row_stride, 0u, nullptr, 0u, nullptr, 0u);
    return hipGetLastError();
}

hipError_t launch_select_rows(const uint8_t* const* d_sets, const uint8_t* d_arena, const uint64_t* d_offs,
                              const uint32_t* d_lens, uint32_t n, uint32_t* d_out, uint32_t stride,
                              const uint64_t* d_rows, uint32_t row_stride, uint32_t p0, const uint32_t* d_perm,
                              bool wave_rows, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t block = 256;
    const uint32_t grid = (n + block - 1) / block;
    hipLaunchKernelGGL(ajx_select_values<false>, dim3(grid), dim3(block), 0, stream, d_sets, nullptr, d_arena, d_offs,
                       d_lens, n, d_out, stride, d_rows, row_stride, p0, d_perm, wave_rows ? 1u : 0u, nullptr, 0u);
    return hipGetLastError();
}

hipError_t launch_eval_scan(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, const uint8_t* d_arena,
                            const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n, uint8_t* d_tri,
                            int32_t* d_err, uint64_t* d_bm, uint32_t stride, hipStream_t stream, bool mods) {
    if (n == 0) return hipSuccess;
    const uint32_t block = 256;
    const uint32_t grid = (n + block - 1) / block;
    if (mods)
        hipLaunchKernelGGL(ajx_eval_scan<true>, dim3(grid), dim3(block), 0, stream, d_sets, d_set_of_req, d_arena,
                           d_offs, d_lens, n, d_tri, d_err, d_bm, stride);
    else
        hipLaunchKernelGGL(ajx_eval_scan<false>, dim3(grid), dim3(block), 0, stream, d_sets, d_set_of_req, d_arena,
                           d_offs, d_lens, n, d_tri, d_err, d_bm, stride);
    return hipGetLastError();
}

hipError_t launch_eval_fast(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, uint32_t shared_blob_bytes,
                            const uint8_t* d_arena, const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n,
                            uint8_t* d_tri, int32_t* d_err, uint64_t* d_bm, uint32_t stride, uint64_t* d_rows,
                            uint32_t row_stride, uint32_t* d_slow_count, uint32_t* d_slow_ids, hipStream_t stream,
                            int mode, const uint32_t* d_perm, bool mods, bool keep_rows, uint32_t lean_feat,
                            const uint32_t* d_pos_of, uint8_t* d_tout, uint32_t n_out) {
    if (n == 0) return hipSuccess;
    const bool shared = shared_blob_bytes != 0 && d_set_of_req == nullptr;
    // workgroup size by the waves a CU holds (each workgroup stages its own blob copy)
    uint32_t block = shared ? fast_block(shared_blob_bytes) : kFastBlock;
    if (mode >= 10 && mode <= 12) {  // profiling: the default kernel at a forced workgroup size
        block = 256u << (mode - 10);
        mode = 0;
        if (((shared ? (shared_blob_bytes + 15u) & ~15u : 0u) + (block / 64) * kWinRingBytesPerWave) > 160u * 1024u)
            return hipErrorInvalidValue;
    }
    const uint32_t grid = (n + block - 1) / block;
    // dynamic LDS of the single-pass kernels: [blob copy (shared)] [window rings]
    const uint32_t ring_off = shared ? (shared_blob_bytes + 15u) & ~15u : 0u;
    const uint32_t lds = ring_off + (block / 64) * kWinRingBytesPerWave;
    hipError_t e = hipMemsetAsync(d_slow_count, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    static std::atomic<uint64_t> attr_done{0};
    e = attr_once(attr_done, [] {
        const void* ks[] = {reinterpret_cast<const void*>(&ajx_scan_fast<0, true>),
                            reinterpret_cast<const void*>(&ajx_scan_fast<0, false>),
                            reinterpret_cast<const void*>(&ajx_scan_fast<1, true>),
                            reinterpret_cast<const void*>(&ajx_scan_fast<2, true>),
                            reinterpret_cast<const void*>(&ajx_scan_fused)};
        for (const void* k : ks) {
            const hipError_t r = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (r != hipSuccess) return r;
        }
        return hipSuccess;
    });
    if (e != hipSuccess) return e;
    if (mode == 1 || mode == 2) {  // profiling ablations of stage A (uniform ruleset only)
        if (!shared) return hipErrorInvalidValue;
        if (mode == 1)
            hipLaunchKernelGGL((ajx_scan_fast<1, true>), dim3(grid), dim3(block), lds, stream, d_sets, d_set_of_req,
                               d_arena, d_offs, d_lens, n, d_rows, row_stride, d_slow_count, d_slow_ids, ring_off, nullptr);
        else
            hipLaunchKernelGGL((ajx_scan_fast<2, true>), dim3(grid), dim3(block), lds, stream, d_sets, d_set_of_req,
                               d_arena, d_offs, d_lens, n, d_rows, row_stride, d_slow_count, d_slow_ids, ring_off, nullptr);
        return hipGetLastError();
    }
    if (mode == 3) {  // profiling split: stage A and stage B as two launches
        if (shared) {
            hipLaunchKernelGGL((ajx_scan_fast<0, true>), dim3(grid), dim3(block), lds, stream, d_sets, d_set_of_req,
                               d_arena, d_offs, d_lens, n, d_rows, row_stride, d_slow_count, d_slow_ids, ring_off, nullptr);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            hipLaunchKernelGGL((ajx_patterns<true>), dim3(grid), dim3(block), ring_off, stream, d_sets, d_set_of_req,
                               d_arena, d_offs, n, d_rows, row_stride, d_tri, d_err, d_bm, stride);
        } else {
            hipLaunchKernelGGL((ajx_scan_fast<0, false>), dim3(grid), dim3(block), lds, stream, d_sets, d_set_of_req,
                               d_arena, d_offs, d_lens, n, d_rows, row_stride, d_slow_count, d_slow_ids, ring_off, nullptr);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            hipLaunchKernelGGL((ajx_patterns<false>), dim3(grid), dim3(block), 0, stream, d_sets, d_set_of_req,
                               d_arena, d_offs, n, d_rows, row_stride, d_tri, d_err, d_bm, stride);
        }
    } else if ((mode >= 15 && mode <= 18) || !d_set_of_req) {
        // the lean single-pass kernel (one ruleset; ajx_lean.hip), or its profiling ablations
        // (multi-tenant batches: the staged tenant scanner below. Measured on c4, the lean
        // scan with per-lane table parameters took 6.39 ms and one pass per ruleset of a
        // wave 7.3-7.8 ms, against 5.38 ms for the tenant kernel's LDS-staged tables)
        if (mode >= 15 && !shared) return hipErrorInvalidValue;
        // in length order, the outputs go to d_tout in work-item order and are gathered back
        // (ajx_unpermute) before the exact scan writes its requests' own
        const bool out_k = d_perm && d_pos_of && d_tout && mode < 15;
        const size_t o_err = ((size_t)n * n_out + 255u) & ~(size_t)255u;
        const size_t o_bm = o_err + (((size_t)n * n_out * 4u + 255u) & ~(size_t)255u);
        uint8_t* k_tri = out_k ? d_tout : d_tri;
        int32_t* k_err = out_k ? (d_err ? reinterpret_cast<int32_t*>(d_tout + o_err) : nullptr) : d_err;
        uint64_t* k_bm = out_k ? (d_bm ? reinterpret_cast<uint64_t*>(d_tout + o_bm) : nullptr) : d_bm;
        e = launch_lean(d_sets, shared ? shared_blob_bytes : 0u, d_arena, d_offs, d_lens, n, d_rows, row_stride,
                        d_slow_count, d_slow_ids, k_tri, k_err, k_bm, stride, stream, mode >= 15 ? mode - 14 : 0,
                        d_perm, keep_rows, lean_feat, out_k);
        if (e != hipSuccess || mode >= 15) return e;
        if (out_k) {
            hipLaunchKernelGGL(ajx_unpermute, dim3((n + 255u) / 256u), dim3(256), 0, stream, d_pos_of, n, n_out,
                               stride, k_tri, k_err, k_bm, d_tri, d_err, d_bm);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
    } else if (shared_blob_bytes) {
        // multi-tenant batch (shared_blob_bytes != 0: staging on): each workgroup stages its
        // runs' rulesets, those that fit (ajx_scan_fused_tenant);
        // 4-wave workgroups, so more of them fall inside one AuthConfig's bucket
        // (staging region: the tenant budget less room for the kernel's static LDS, so
        // four groups still fit a CU)
        e = launch_tenant(d_sets, d_set_of_req, d_arena, d_offs, d_lens, n, d_rows, row_stride, d_slow_count,
                          d_slow_ids, d_tri, d_err, d_bm, stride, stream, d_perm);
        if (e != hipSuccess) return e;
    } else {
        hipLaunchKernelGGL(ajx_scan_fused, dim3(grid), dim3(block), lds, stream, d_sets, d_set_of_req,
                           d_arena, d_offs, d_lens, n, d_rows, row_stride, d_slow_count, d_slow_ids, d_tri, d_err, d_bm,
                           stride, ring_off, d_perm);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const uint32_t sgrid = grid < 2048 ? 2 * grid : 4096;
    launch_slow_list(mods, sgrid, stream, d_sets, d_set_of_req, d_arena, d_offs, d_lens, d_slow_count, d_slow_ids,
                     d_tri, d_err, d_bm, stride);
    return hipGetLastError();
}

}  // namespace ajx
