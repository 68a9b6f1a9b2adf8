// ajx_kcommon.h — device helpers shared by the kernel translation units (ajx_kernels.hip,
// ajx_lean.hip): per-device attribute guards, the LDS staging of a ruleset blob, and stage
// B's outputs (the T bitmap and the And/Or fold of every tree).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>

#include "ajx_fast.h"

#ifndef AJX_FAST_WAVES
#define AJX_FAST_WAVES 4  // waves per SIMD the single-pass kernels' register budget is set for
#endif

namespace ajx {

// The dynamic-LDS ceiling of a group of kernels is set once per device (the attribute
// belongs to that device's code object); any thread may launch first, so the per-device
// bits are atomic (setting an attribute twice is harmless).
template <class F>
static hipError_t attr_once(std::atomic<uint64_t>& done, F set) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = dev >= 0 && dev < 64 ? 1ull << dev : 0ull;
    if (bit && (done.load(std::memory_order_acquire) & bit)) return hipSuccess;
    if ((e = set()) != hipSuccess) return e;
    done.fetch_or(bit, std::memory_order_acq_rel);
    return hipSuccess;
}

// SHARED kernels: the whole batch uses sets[0], and the ruleset blob (trie, key table,
// patterns, literals, DFA tables, fold code — h->total_bytes, a multiple of 16) is
// copied into dynamic LDS once per workgroup; every thread reaches the barrier. All
// table reads of the scan and the patterns are then ds_reads.
// copies nq 16-byte words, four loads in flight per thread before their stores. The source
// is read as global memory (a blob pointer loaded from the set table is generic: flat
// loads otherwise), every load unconditional (a clamped index past the end), so that
// nothing goes to scratch.
__device__ __forceinline__ void copy_words(uint4* __restrict__ dst, const uint4* __restrict__ src, uint32_t nq,
                                           uint32_t t, uint32_t nt) {
#if defined(__HIP_DEVICE_COMPILE__)
    const __attribute__((address_space(1))) uint4* g = (const __attribute__((address_space(1))) uint4*)src;
#else
    const uint4* g = src;  // (host pass of the kernel source: never run)
#endif
    const uint32_t last = nq - 1u;
    for (uint32_t b = t; b < nq; b += 4u * nt) {
        const uint32_t k1 = b + nt, k2 = b + 2u * nt, k3 = b + 3u * nt;
        const uint4 v0 = g[b];
        const uint4 v1 = g[k1 < nq ? k1 : last];
        const uint4 v2 = g[k2 < nq ? k2 : last];
        const uint4 v3 = g[k3 < nq ? k3 : last];
        dst[b] = v0;
        if (k1 < nq) dst[k1] = v1;
        if (k2 < nq) dst[k2] = v2;
        if (k3 < nq) dst[k3] = v3;
    }
}

// copy_words with every load unconditional (past the end, word b again): the array stays
// in registers (the streaming kernel's per-wave blob copy: c4 serving 7.8 k -> 4.0 k clocks)
__device__ __forceinline__ void copy_words_reg(uint4* __restrict__ dst, const uint4* __restrict__ src, uint32_t nq,
                                               uint32_t t, uint32_t nt) {
    for (uint32_t b = t; b < nq; b += 8u * nt) {
        uint4 v[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t k = b + j * nt;
            v[j] = src[k < nq ? k : b];
        }
#pragma unroll
        for (uint32_t j = 0; j < 8; j++)
            if (b + j * nt < nq) dst[b + j * nt] = v[j];
    }
}

template <bool SHARED>
__device__ __forceinline__ const uint8_t* stage_blob(const uint8_t* gblob) {
    if constexpr (SHARED) {
        extern __shared__ uint4 s_blob[];
        const uint32_t nq = reinterpret_cast<const RulesetHdr*>(gblob)->total_bytes / 16;
        copy_words(s_blob, reinterpret_cast<const uint4*>(gblob), nq, threadIdx.x, blockDim.x);
        __syncthreads();
        return reinterpret_cast<const uint8_t*>(s_blob);
    } else {
        return gblob;
    }
}

// the And/Or fold of every tree of the ruleset on the pattern bitmaps; a forest ruleset
// (authjx_compile_forest) writes its n_trees results at r * n_trees + k
__device__ __forceinline__ void fold_outputs(uint32_t r, const uint8_t* blob, const RulesetHdr* h, const uint64_t t[2],
                                             const uint64_t u[2], const uint64_t se[2],
                                             uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err) {
    const uint32_t* code = reinterpret_cast<const uint32_t*>(blob + h->off_code);
    const uint32_t nt = h->pad1[0];
    if (h->flags & kFlagFlatFold) {  // (one tree, [open, pattern 0, ..., pattern n - 1, close])
        int32_t ep;
        out_tri[r] = flat_fold(h, code, t, u, se, &ep);
        if (out_err) out_err[r] = ep;
        return;
    }
    if (h->flags & kFlagGroupFold) {  // (one tree: groups of patterns under one All / Any)
        int32_t ep;
        out_tri[r] = group_fold(h, code, t, u, se, &ep);
        if (out_err) out_err[r] = ep;
        return;
    }
    if (nt == 0) {
        int32_t ep;
        out_tri[r] = run_fold_bits(code, h->n_code, t, u, se, &ep);
        if (out_err) out_err[r] = ep;
        return;
    }
    const uint32_t* rc = reinterpret_cast<const uint32_t*>(blob + h->pad1[1]);
    const TreeFold* tf = h->pad1[2] ? reinterpret_cast<const TreeFold*>(blob + h->pad1[2]) : nullptr;
    for (uint32_t k = 0; k < nt; k++) {
        int32_t ep;
        out_tri[(size_t)r * nt + k] = tf && tf[k].shape ? tree_fold(tf[k], t, u, se, &ep)
                                                        : run_fold_bits(code + rc[2 * k], rc[2 * k + 1], t, u, se, &ep);
        if (out_err) out_err[(size_t)r * nt + k] = ep;
    }
}

// stage B for request r on its capture row: patterns, T bitmap, And/Or fold, outputs.
// false (nothing written): a value needs the exact scan (a number only ajx_float.h
// decides), the caller hands the request over
__device__ __forceinline__ bool finish_request(uint32_t r, const uint8_t* blob, const uint8_t* d, RowRef row,
                                               uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err,
                                               uint64_t* __restrict__ out_bm, uint32_t stride,
                                               const uint64_t* dec = nullptr, uint8_t* ring = nullptr) {
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
    uint64_t t[2], u[2];
    patterns_from_row(blob, d, row, t, u, dec, 0, 1, ring);
    if ((u[0] & ~h->unsupported[0]) | (u[1] & ~h->unsupported[1])) return false;
    if (out_bm) {
        uint64_t* orow = out_bm + (size_t)r * stride;
        orow[0] = t[0];
        if (stride > 1) orow[1] = t[1];
        for (uint32_t w = 2; w < stride; w++) orow[w] = 0ull;
    }
    const uint64_t se[2] = {h->static_error[0], h->static_error[1]};
    fold_outputs(r, blob, h, t, u, se, out_tri, out_err);
    return true;
}

// the work-item's 128-B window ring in dynamic LDS: [blob copy (SHARED)] [ring: per wave
// 8 chunks x 64 lanes x 16 B]
constexpr uint32_t kWinRingBytesPerWave = 8 * 64 * 16;
// single-pass workgroups of 4, 8 or 16 waves (fast_block): one LDS copy of the ruleset
// blob per workgroup next to its waves' rings, so 16 waves per CU fit the 160 KiB for
// blobs up to ~8 KiB in 4-wave groups, ~16 KiB in 8-wave groups, ~32 KiB in one 16-wave
// group (4 waves/SIMD by registers either way)
constexpr uint32_t kFastBlock = 512;
constexpr uint32_t kFastMaxBlock = 1024;
#ifndef AJX_FAST_WAVES
#define AJX_FAST_WAVES 4  // waves per SIMD the single-pass kernels' register budget is set for
#endif
// the workgroup size that fits the most waves per CU for a staged blob of `blob_bytes`
// (0: nothing staged); the smallest such size on a tie: a workgroup retires as a unit, so
// smaller ones leave fewer idle waves behind the longest document (measured: c2 4-wave
// 2.03 ms vs 8-wave 2.11; c3 at 16 waves/CU 2 x 8-wave 3.78 vs 1 x 16-wave 4.03)
static uint32_t fast_block(uint32_t blob_bytes) {
    const uint32_t stage = (blob_bytes + 15u) & ~15u;
    uint32_t best = 0, best_w = 0;
    for (uint32_t b = 256; b <= kFastMaxBlock; b *= 2) {
        const uint32_t lds = stage + (b / 64) * kWinRingBytesPerWave;
        uint32_t w = lds <= 160u * 1024u ? (160u * 1024u / lds) * (b / 64) : 0u;
        if (w > 4u * AJX_FAST_WAVES) w = 4u * AJX_FAST_WAVES;
        if (w > best_w) best = b, best_w = w;
    }
    return best ? best : 256u;
}
__device__ __forceinline__ WinRing lane_ring(uint32_t ring_off) {
    extern __shared__ uint4 s_dyn_ring[];
    WinRing r;
    r.base = reinterpret_cast<uint8_t*>(s_dyn_ring) + ring_off + (threadIdx.x >> 6) * kWinRingBytesPerWave;
    r.lane16 = (threadIdx.x & 63u) * 16u;
    r.cstride = 64u * 16u;
    return r;
}

// stage A for request r: single-pass scan into its capture row (false: slow list)
template <int MODE>
__device__ __forceinline__ bool scan_request(const uint8_t* blob, const uint8_t* d, uint32_t len, RowRef row,
                                             const WinRing& ring) {
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
    if (!(h->flags & kFlagFastOk) || len >= (1u << 24)) {
        row[0] = kRowSlow;
        return false;
    }
    const uint4* a4 = reinterpret_cast<const uint4*>(d - ((uintptr_t)d & 15u));
    auto load = [&](uint32_t b, uint32_t nblk) -> Block16 {
        if (b < nblk) {
            const uint4 v = a4[b];
            return Block16{v.x, v.y, v.z, v.w};
        }
        return Block16{0u, 0u, 0u, 0u};
    };
    return scan_doc<MODE>(blob, blob_tables(blob), d, len, row, ring, load);
}

}  // namespace ajx
