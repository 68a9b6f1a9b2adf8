// ajx_lean.hip — the lean single-pass kernel (ajx_lean.h) in its own translation unit, so
// that the walker's code is compiled (and tuned) without the rest of the kernels.
#include <hip/hip_runtime.h>

#include "ajx_kcommon.h"
#include "ajx_kernels.h"
#include "ajx_lean.h"


namespace ajx {

static_assert(64 * kSpanStride <= lean::kRingBytesPerWave, "stage B's span buffers lie in the wave's ring");
constexpr uint32_t kLeanMaxBlock = 1024;
#ifndef AJX_LEAN_MAXBLOCK
#define AJX_LEAN_MAXBLOCK kLeanMaxBlock
#endif

// The lean single-pass kernel (ajx_lean.h): stage A with the lean scan, then stage B in the
// same work-item. Dynamic LDS: [blob copy (SHARED)] [per wave: 64 lanes x 144-B rings].
#ifndef AJX_LEAN_WAVES
#define AJX_LEAN_WAVES AJX_FAST_WAVES  // waves per SIMD the lean kernel's registers are set for
#endif
#ifndef AJX_LEAN_MAXBLOCK
#define AJX_LEAN_MAXBLOCK kLeanMaxBlock
#endif
// ABL: profiling ablations (kernel modes 15..18, lean::scan_doc): stage A cut short, no stage B.
// FEAT: the walker features the ruleset needs (RulesetHdr::lean_feat: kLeanArr | kLeanCaps)
template <bool SHARED, int ABL = 0, int FEAT = 3>
__global__ __launch_bounds__(AJX_LEAN_MAXBLOCK, AJX_LEAN_WAVES) void ajx_scan_lean(
    const uint8_t* const* __restrict__ sets, const uint32_t* __restrict__ set_of_req,
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs, const uint32_t* __restrict__ lens, uint32_t n,
    uint64_t* __restrict__ rows, uint32_t row_stride, uint32_t* __restrict__ slow_count,
    uint32_t* __restrict__ slow_ids, uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err,
    uint64_t* __restrict__ out_bm, uint32_t stride, uint32_t ring_off, const uint32_t* __restrict__ perm,
    uint32_t keep_rows) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t r = k < n ? (perm ? perm[k] : k) : 0u;
    // keep_rows bit 1: the outputs in work-item order (gathered back by ajx_unpermute)
    const uint32_t o = (keep_rows & 2u) ? k : r;
    keep_rows &= 1u;
    const uint8_t* blob = stage_blob<SHARED>(sets[SHARED || !set_of_req ? 0 : set_of_req[r]]);
    if (k >= n) return;
    extern __shared__ uint4 s_lean_dyn[];
    uint8_t* wring = reinterpret_cast<uint8_t*>(s_lean_dyn) + ring_off + (threadIdx.x >> 6) * lean::kRingBytesPerWave;
    const RowRef row = wave_row(rows, row_stride, k);
    const uint8_t* d = arena + offs[r];
    const uint32_t len = lens[r];
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
    bool ok = (h->flags & kFlagFastOk) && len > 0 && len < (1u << 24);  // (empty: the exact scan)
    uint64_t dec[2] = {0ull, 0ull};
    if (ok) {
        const uint32_t mis = (uint32_t)((uintptr_t)d & 15u);
        lean::DmaLoader ld{reinterpret_cast<const uint4*>(d - mis), (len + mis + 15u) / 16u, wring};
        ok = lean::scan_doc<ABL, (FEAT & kLeanArr) != 0, (FEAT & kLeanCaps) != 0>(
            blob, len, mis, row, wring + (threadIdx.x & 63u) * 16u, ld, dec, keep_rows);
    } else {
        row[0] = kRowSlow;
    }
    if constexpr (ABL != 0) {
        if (dec[0] ^ dec[1]) row[0] ^= dec[0] ^ dec[1];
        return;
    }
    if (!ok) {
        slow_ids[atomicAdd(slow_count, 1u)] = r;
        return;
    }
    // (stage B reads short values from a copy in the lane's share of the ring, stage_span:
    // scan_doc left no load in flight)
    if (!finish_request(o, blob, d, row, out_tri, out_err, out_bm, stride, dec, wring + (threadIdx.x & 63u) * kSpanStride)) {
        row[0] = kRowSlow;
        slow_ids[atomicAdd(slow_count, 1u)] = r;
    }
}
// workgroup size for the lean kernel with a staged blob of `blob_bytes` (as fast_block)
static uint32_t lean_block(uint32_t blob_bytes) {
    const uint32_t stage = (blob_bytes + 15u) & ~15u;
    uint32_t best = 0, best_w = 0;
    for (uint32_t b = 256; b <= AJX_LEAN_MAXBLOCK; b *= 2) {
        const uint32_t lds = stage + (b / 64) * lean::kRingBytesPerWave;
        uint32_t w = lds <= 160u * 1024u ? (160u * 1024u / lds) * (b / 64) : 0u;
        if (w > 4u * AJX_LEAN_WAVES) w = 4u * AJX_LEAN_WAVES;
        if (w > best_w) best = b, best_w = w;
    }
    return best ? best : 256u;
}

#define AJX_LEAN_K(SH, A, F) reinterpret_cast<const void*>(&ajx_scan_lean<SH, A, F>)
hipError_t launch_lean(const uint8_t* const* d_sets, uint32_t shared_blob_bytes, const uint8_t* d_arena,
                       const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n, uint64_t* d_rows,
                       uint32_t row_stride, uint32_t* d_slow_count, uint32_t* d_slow_ids, uint8_t* d_tri,
                       int32_t* d_err, uint64_t* d_bm, uint32_t stride, hipStream_t stream, int abl,
                       const uint32_t* d_perm, bool keep_rows, uint32_t lean_feat, bool out_k) {
    if (n == 0) return hipSuccess;
    const bool shared = shared_blob_bytes != 0;
    static std::atomic<uint64_t> attr_done{0};
    hipError_t e = attr_once(attr_done, [] {
        const void* ks[] = {AJX_LEAN_K(true, 0, 2), AJX_LEAN_K(true, 0, 3), AJX_LEAN_K(false, 0, 3),
#if defined(AJX_LEAN_ABLATIONS)
                            AJX_LEAN_K(true, 1, 2), AJX_LEAN_K(true, 2, 2), AJX_LEAN_K(true, 3, 2), AJX_LEAN_K(true, 4, 2),
                            AJX_LEAN_K(true, 1, 3), AJX_LEAN_K(true, 2, 3), AJX_LEAN_K(true, 3, 3), AJX_LEAN_K(true, 4, 3)
#endif
        };
        for (const void* k : ks) {
            const hipError_t r = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (r != hipSuccess) return r;
        }
        return hipSuccess;
    });
    if (e != hipSuccess) return e;
    const uint32_t ring_off = shared ? (shared_blob_bytes + 15u) & ~15u : 0u;
    const uint32_t lblock = shared ? lean_block(shared_blob_bytes) : 256u;
    const uint32_t lgrid = (n + lblock - 1) / lblock;
    const uint32_t llds = ring_off + (lblock / 64) * lean::kRingBytesPerWave;
    const uint32_t keep = (keep_rows ? 1u : 0u) | (out_k && d_perm ? 2u : 0u);
    // (two instances: without and with array walking. The capture-free instances cost
    // the walk loop scratch reloads of spilled scalar registers, which wait behind the
    // ring's loads in flight: measured slower, c2 1.39 against 1.27 ms)
    const uint32_t feat = (lean_feat & kLeanArr) ? 3u : 2u;
    using K = void (*)(const uint8_t* const*, const uint32_t*, const uint8_t*, const uint64_t*, const uint32_t*,
                       uint32_t, uint64_t*, uint32_t, uint32_t*, uint32_t*, uint8_t*, int32_t*, uint64_t*, uint32_t,
                       uint32_t, const uint32_t*, uint32_t);
    K k = nullptr;
    if (abl) {
#if defined(AJX_LEAN_ABLATIONS)
        if (!shared || abl > 4) return hipErrorInvalidValue;
        const bool f2 = feat == 2;
        k = abl == 1 ? (f2 ? &ajx_scan_lean<true, 1, 2> : &ajx_scan_lean<true, 1, 3>)
          : abl == 2 ? (f2 ? &ajx_scan_lean<true, 2, 2> : &ajx_scan_lean<true, 2, 3>)
          : abl == 3 ? (f2 ? &ajx_scan_lean<true, 3, 2> : &ajx_scan_lean<true, 3, 3>)
                     : (f2 ? &ajx_scan_lean<true, 4, 2> : &ajx_scan_lean<true, 4, 3>);
#else
        return hipErrorInvalidValue;  // (a profiling build: scripts/build_variant.sh NAME -DAJX_LEAN_ABLATIONS)
#endif
    } else if (!shared) {
        k = &ajx_scan_lean<false, 0, 3>;
    } else {
        k = feat == 2 ? &ajx_scan_lean<true, 0, 2> : &ajx_scan_lean<true, 0, 3>;
    }
    hipLaunchKernelGGL(k, dim3(lgrid), dim3(lblock), llds, stream, d_sets, nullptr, d_arena, d_offs, d_lens, n,
                       d_rows, row_stride, d_slow_count, d_slow_ids, d_tri, d_err, d_bm, stride, ring_off, d_perm,
                       keep);
    return hipGetLastError();
}
#undef AJX_LEAN_K

// The single-pass kernel for multi-tenant batches (one ruleset per request through
// set_of_req; the caller buckets requests by AuthConfig, so a workgroup's requests form a
// few runs of one ruleset each). The workgroup finds its runs (a run starts where the
// ruleset differs from the previous work-item's) and copies the blobs of its first runs
// into LDS — each blob's hot prefix, [0, hot_bytes), which holds every table this kernel
// reads — as many as fit the staging region; a wave whose requests all fall in staged
// runs reads every table from LDS (each lane from its own run's copy), any other wave
// reads them from global memory. Dynamic LDS: [staging region (ring_off bytes)] [rings].
constexpr uint32_t kTenantRuns = 16;  // runs a workgroup may stage
static_assert(lean::kRingBytesPerWave == kWinRingBytesPerWave, "the tenant kernel's rings serve both scans");
__global__ __launch_bounds__(kFastBlock, AJX_FAST_WAVES) void ajx_scan_fused_tenant(
    const uint8_t* const* __restrict__ sets, const uint32_t* __restrict__ set_of_req,
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs, const uint32_t* __restrict__ lens, uint32_t n,
    uint64_t* __restrict__ rows, uint32_t row_stride, uint32_t* __restrict__ slow_count,
    uint32_t* __restrict__ slow_ids, uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err,
    uint64_t* __restrict__ out_bm, uint32_t stride, uint32_t ring_off, const uint32_t* __restrict__ perm) {
    extern __shared__ uint4 s_stage[];
    __shared__ uint32_t s_wcnt[kFastBlock / 64];
    __shared__ uint32_t s_rsid[kTenantRuns];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6, nw = blockDim.x >> 6;
    const uint32_t k = blockIdx.x * blockDim.x + t;  // (the grid covers n: n > 0 here)
    const uint32_t kc = k < n ? k : n - 1u;           // (tail threads: the last request's run)
    const uint32_t r = perm ? perm[kc] : kc;
    const uint32_t sid = set_of_req[r];
    bool start = t == 0;
    if (!start) {
        const uint32_t kp = (k - 1u) < n ? k - 1u : n - 1u;
        start = set_of_req[perm ? perm[kp] : kp] != sid;
    }
    // run index of every work-item: starts before it in the workgroup, minus one
    const uint64_t m = __ballot(start);
    if (lane == 0) s_wcnt[wv] = (uint32_t)__builtin_popcountll(m);
    __syncthreads();
    uint32_t base = 0, nrun = 0;
    for (uint32_t i = 0; i < nw; i++) {
        const uint32_t c = s_wcnt[i];
        base += i < wv ? c : 0u;
        nrun += c;
    }
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    const uint32_t ridx = base + (uint32_t)__builtin_popcountll(m & upto) - 1u;
    if (start && ridx < kTenantRuns) s_rsid[ridx] = sid;
    __syncthreads();
    // stage the leading runs' blobs while they fit (every thread walks the same list)
    uint32_t nst = 0, off = 0, my_off = 0;
    const uint32_t nr = nrun < kTenantRuns ? nrun : kTenantRuns;
    for (uint32_t j = 0; j < nr; j++) {
        const uint8_t* g = sets[s_rsid[j]];
        const uint32_t bytes = reinterpret_cast<const RulesetHdr*>(g)->hot_bytes;  // (a multiple of 16)
        if (off + bytes > ring_off) break;
        const uint4* src = reinterpret_cast<const uint4*>(g);
        for (uint32_t i = t; i < bytes / 16u; i += blockDim.x) s_stage[off / 16u + i] = src[i];
        if (j == ridx) my_off = off;
        off += bytes;
        nst++;
    }
    __syncthreads();
    const RowRef row = wave_row(rows, row_stride, k);
    const uint8_t* d = arena + offs[r];
    // (wave-uniform: the whole wave takes the LDS tables or the global ones)
    if (__all(ridx < nst)) {
        // a wave whose requests all use one staged ruleset (the caller's bucketing makes most
        // waves so: 84 % of c4's) runs the lean scan on that copy (ajx_scan_lean's
        // per-request body); a wave of several rulesets, the token scanner with each lane's
        // own copy. (As two kernels, one per kind of wave, each with its own registers: c4
        // 5.57 ms against 4.85 ms for this one.)
        const uint32_t off0 = lean::uni(my_off);
        if (__all(my_off == off0)) {
            const uint8_t* blob = reinterpret_cast<const uint8_t*>(s_stage) + off0;
            if (k >= n) return;
            const uint32_t len = lens[r];
            const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
            uint64_t dec[2] = {0ull, 0ull};
            bool ok = (h->flags & kFlagFastOk) && len > 0 && len < (1u << 24);
            if (ok) {
                uint8_t* wring = reinterpret_cast<uint8_t*>(s_stage) + ring_off + wv * lean::kRingBytesPerWave;
                const uint32_t mis = (uint32_t)((uintptr_t)d & 15u);
                lean::DmaLoader ld{reinterpret_cast<const uint4*>(d - mis), (len + mis + 15u) / 16u, wring};
                ok = lean::scan_doc(blob, len, mis, row, wring + lane * 16u, ld, dec, 0u) &&
                     finish_request(r, blob, d, row, out_tri, out_err, out_bm, stride, dec, wring + lane * kSpanStride);
            }
            if (!ok) {
                row[0] = kRowSlow;
                slow_ids[atomicAdd(slow_count, 1u)] = r;
            }
            return;
        }
    }
    // a wave of several rulesets, or of rulesets not staged: the token scanner, each lane on
    // its own ruleset (its staged copy or the global blob: one generic pointer, one copy of
    // the scanner and of stage B in the kernel, which keeps the lean path's registers)
    const uint8_t* blob = ridx < nst ? reinterpret_cast<const uint8_t*>(s_stage) + my_off : sets[sid];
    if (k >= n) return;
    if (!scan_request<0>(blob, d, lens[r], row, lane_ring(ring_off)) ||
        !finish_request(r, blob, d, row, out_tri, out_err, out_bm, stride)) {
        row[0] = kRowSlow;
        slow_ids[atomicAdd(slow_count, 1u)] = r;
    }
}

hipError_t launch_tenant(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, const uint8_t* d_arena,
                         const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n, uint64_t* d_rows,
                         uint32_t row_stride, uint32_t* d_slow_count, uint32_t* d_slow_ids, uint8_t* d_tri,
                         int32_t* d_err, uint64_t* d_bm, uint32_t stride, hipStream_t stream, const uint32_t* d_perm) {
    if (n == 0) return hipSuccess;
    static std::atomic<uint64_t> attr_done{0};
    hipError_t e = attr_once(attr_done, [] {
        // (the kernel also holds static LDS for its run table: ask only for what its launch
        // uses, the staging region + four window rings)
        return hipFuncSetAttribute(reinterpret_cast<const void*>(&ajx_scan_fused_tenant),
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   kMaxTenantStageBytes + (kTenantBlock / 64) * kWinRingBytesPerWave);
    });
    if (e != hipSuccess) return e;
    // (staging region: the tenant budget less room for the kernel's static LDS, so two
    // groups still fit a CU)
    const uint32_t tblock = kTenantBlock, tgrid = (n + tblock - 1) / tblock;
    const uint32_t toff = kMaxTenantStageBytes - 256u;
    hipLaunchKernelGGL(ajx_scan_fused_tenant, dim3(tgrid), dim3(tblock), toff + (tblock / 64) * kWinRingBytesPerWave,
                       stream, d_sets, d_set_of_req, d_arena, d_offs, d_lens, n, d_rows, row_stride, d_slow_count,
                       d_slow_ids, d_tri, d_err, d_bm, stride, toff, d_perm);
    return hipGetLastError();
}

}  // namespace ajx
