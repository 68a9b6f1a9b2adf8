// ajx_rowk.hip — the row kernel's stage A launch (ajx_row.h): four documents per
// wavefront, 16 lanes each. Workgroups of 4 waves stage the ruleset blob in LDS next to
// each wave's row buffers, then every wave walks groups of four requests (grid-stride;
// the requests of a group are consecutive in the length-bucketed order, so their lengths
// are alike). A tier takes the documents that fit its row buffers (maxb); longer ones go
// to the next tier's list (the last tier's "next" is the exact scan's list), as do the
// ones the row scan can not prove. Output: each request's capture row (row r, header
// kRowSlow when handed over).
#include <hip/hip_runtime.h>

#include <atomic>

#include "ajx_fast.h"
#include "ajx_kernels.h"
#include "ajx_row.h"

namespace ajx {

constexpr uint32_t kRowBlock = 256;

__global__ __launch_bounds__(kRowBlock) void ajx_row_scan(
    const uint8_t* const* __restrict__ sets, const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
    const uint32_t* __restrict__ lens, uint32_t n, const uint32_t* __restrict__ perm,
    const uint32_t* __restrict__ in_count, const uint32_t* __restrict__ in_ids, uint64_t* __restrict__ rows,
    uint32_t row_stride, uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err, uint64_t* __restrict__ out_bm,
    uint32_t bm_stride, uint32_t* __restrict__ slow_count, uint32_t* __restrict__ slow_ids,
    uint32_t* __restrict__ next_count, uint32_t* __restrict__ next_ids, w::RowLayout L, uint32_t blob_region,
    uint32_t stop) {
    using namespace w;
    extern __shared__ uint4 s_row[];
    const uint8_t* gblob = sets[0];
    {
        const uint32_t nq = reinterpret_cast<const RulesetHdr*>(gblob)->total_bytes / 16;
        const uint4* g = reinterpret_cast<const uint4*>(gblob);
        for (uint32_t i = threadIdx.x; i < nq; i += blockDim.x) s_row[i] = g[i];
        __syncthreads();
    }
    Lds lds = (Lds)(uint8_t*)s_row;  // (an address-space cast: ds_ instructions for the row buffers)
    const uint8_t* blob = reinterpret_cast<const uint8_t*>(s_row);  // (generic: stage B's scalar code)
    const RowTabs T = row_tabs(gblob, lds);
    const uint32_t wv = threadIdx.x >> 6;
    Lds wl = lds + blob_region + wv * L.bytes;
    const V ln = lane(), row = ln >> 4, rl = ln & 15u;
    const uint32_t count = in_ids ? *in_count : n;
    const uint32_t ngroups = (count + 3u) >> 2;
    const uint32_t wpb = blockDim.x >> 6;  // waves per workgroup
    const uint32_t gstep = gridDim.x * wpb;
    // the request of each row of group gg (every lane of a row holds its row's)
    struct Req {
        V r, len, mis;
        M live, toolong;
        uint64_t off;
    };
    auto req_of = [&](uint32_t gg) -> Req {
        Req q;
        const V k = gg * 4u + row;
        q.live = gg < ngroups && k < count;
        q.r = q.live ? (in_ids ? in_ids[k] : (perm ? perm[k] : k)) : 0u;
        q.len = q.live ? lens[q.r] : 0u;
        q.off = q.live ? offs[q.r] : 0ull;
        q.mis = (V)(q.off & 15u);
        const V nblk = (q.len + q.mis + 15u) >> 4;
        q.toolong = q.live & (q.len != 0u) & (nblk * 16u > L.maxb);
        return q;
    };
    // the aligned blocks of the group's documents into the document rows at `docoff`: one
    // LDS-DMA instruction per KiB of a document (64 lanes x 16 B, contiguous)
    auto dma_group = [&](const Req& q, uint32_t docoff) {
        for (uint32_t rr = 0; rr < 4; rr++) {
            const uint32_t lv = 16u * rr;
            if (!readlane((q.live & !q.toolong) ? 1u : 0u, lv)) continue;
            const uint32_t len = readlane(q.len, lv);
            const uint64_t off = ((uint64_t)readlane((V)(q.off >> 32), lv) << 32) | readlane((V)q.off, lv);
            const uint32_t mis = (uint32_t)(off & 15u);
            const uint32_t nblk = (len + mis + 15u) >> 4;
            const uint8_t* base = arena + (off - mis);
            for (uint32_t c = 0; c * 64u < nblk; c++) {
                const V blk = c * 64u + ln;
                dma16(base + blk * 16u, wl + docoff + rr * L.doc_stride + 16u + c * 1024u, blk < nblk);
            }
        }
    };
    uint32_t g = blockIdx.x * wpb + wv;
    Req q = req_of(g);
    uint32_t cur = L.doc, other = L.doc2;
    if (g < ngroups) dma_group(q, cur);
    for (; g < ngroups; g += gstep) {
        const Req qn = req_of(g + gstep);
        wait_vm();  // this group's documents are in its document rows
        if (g + gstep < ngroups) dma_group(qn, other);  // (lands while this group is scanned)
        const V r = q.r, len = q.len, mis = q.mis;
        if (q.toolong & (rl == 0u)) next_ids[atomicAdd(next_count, 1u)] = r;
        const M mine = q.live & !q.toolong;
        auto load = [&](V, M) -> G16 { return G16{0u, 0u, 0u, 0u}; };
        M ok = row_scan<true>(T, wl, L, mine, len, mis, load, stop, cur);
        if (stop && stop <= 2) {  // (profiling ablations: outputs meaningless)
            if (mine & (rl == 0u)) out_tri[r] = ok ? 1 : 0;
        } else {
            uint64_t* orow = rows ? rows + (size_t)r * row_stride : nullptr;
            V hlo, hhi;
            ok = row_finish(
                T, wl, L, ok, mis, hlo, hhi,
                [&](V s, M m, M found, V start, V vlen, V type, V esc) {
                    if (orow && (m & found))
                        orow[1 + s] =
                            (uint64_t)start | ((uint64_t)((vlen & 0xFFFFFFu) | (type << 24) | (esc << 27)) << 32);
                },
                cur);
            if (stop == 3) {
                if (mine & (rl == 0u)) out_tri[r] = ok ? 1 : 0;
            } else {
                ok = row_patterns(
                    blob, wl, L, ok, mis, r,
                    [&](uint32_t rr, uint32_t kk, uint32_t nt, uint8_t t, int32_t e) {
                        out_tri[(size_t)rr * nt + kk] = t;
                        if (out_err) out_err[(size_t)rr * nt + kk] = e;
                    },
                    [&](uint32_t rr, uint32_t kk, uint64_t word) { out_bm[(size_t)rr * bm_stride + kk] = word; },
                    out_bm ? bm_stride : 0u, cur);
                if (mine & (rl == 0u)) {
                    if (orow) orow[0] = ok ? ((uint64_t)hlo | ((uint64_t)hhi << 32)) : kRowSlow;
                    if (!ok) slow_ids[atomicAdd(slow_count, 1u)] = r;
                }
            }
        }
        q = qn;
        const uint32_t t = cur;
        cur = other;
        other = t;
    }
}

static int row_cu_count() {
    static std::atomic<int> cached{0};
    int c = cached.load();
    if (c) return c;
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
        v = 256;
    cached.store(v);
    return v;
}

// tiers of the row kernel: row buffers for documents up to 1.5 KiB, 4.5 KiB, 8 KiB; each
// wave holds two sets of four document rows (the group being scanned and the next one,
// landing by LDS-DMA), so the longer tiers run in 2- and 1-wave workgroups (~48 / ~82 KiB
// of LDS a wave)
constexpr uint32_t kRowTiers = 3;
constexpr uint32_t kRowTierMaxb[kRowTiers] = {1536, 4608, 8192};
constexpr uint32_t kRowTierBlock[kRowTiers] = {256, 128, 64};

bool row_kernel_fits(uint32_t blob_bytes) {
    const uint32_t blob_region = (blob_bytes + 15u) & ~15u;
    for (uint32_t t = 0; t < kRowTiers; t++) {
        const w::RowLayout L = w::row_layout(kRowTierMaxb[t], kRowTierMaxb[t] / 4, true);
        if (blob_region + (kRowTierBlock[t] / 64) * L.bytes > 160u * 1024u) return false;
    }
    return true;
}

hipError_t launch_row_scan(const uint8_t* const* d_sets, uint32_t blob_bytes, const uint8_t* d_arena,
                           const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n, uint64_t* d_rows,
                           uint32_t row_stride, uint8_t* d_tri, int32_t* d_err, uint64_t* d_bm, uint32_t stride,
                           uint32_t* d_slow, uint32_t* d_tier, hipStream_t stream, const uint32_t* d_perm,
                           uint32_t stop) {
    if (n == 0) return hipSuccess;
    const uint32_t blob_region = (blob_bytes + 15u) & ~15u;
    // (the dynamic-LDS ceiling is a per-device attribute of the code object)
    static std::atomic<uint64_t> attr_done{0};
    {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        const uint64_t bit = dev >= 0 && dev < 64 ? 1ull << dev : 0ull;
        if (!bit || !(attr_done.load() & bit)) {
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(&ajx_row_scan),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) return e;
            attr_done.fetch_or(bit);
        }
    }
    hipError_t e;
    // counters: slow list [0], tier lists A/B at d_tier[0] / d_tier[n + 1]
    if ((e = hipMemsetAsync(d_slow, 0, sizeof(uint32_t), stream)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(d_tier, 0, sizeof(uint32_t), stream)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(d_tier + n + 1, 0, sizeof(uint32_t), stream)) != hipSuccess) return e;
    const uint32_t cus = (uint32_t)row_cu_count();
    uint32_t* lists[2] = {d_tier, d_tier + n + 1};
    for (uint32_t t = 0; t < kRowTiers; t++) {
        const w::RowLayout L = w::row_layout(kRowTierMaxb[t], kRowTierMaxb[t] / 4, true);
        const uint32_t block = kRowTierBlock[t];
        const uint32_t lds = blob_region + (block / 64) * L.bytes;
        if (lds > 160u * 1024u) return hipErrorInvalidValue;
        const uint32_t per_cu = (160u * 1024u) / lds;
        uint32_t grid = cus * (per_cu ? per_cu : 1u) * 2u;
        if (t == 0) {
            const uint32_t need = (n + (block / 16) - 1) / (block / 16);
            if (grid > need) grid = need;
        }
        const bool last = t + 1 == kRowTiers;
        uint32_t* in = t == 0 ? nullptr : lists[(t - 1) & 1];
        uint32_t* nxt = last ? d_slow : lists[t & 1];
        if (t >= 2 && !last && (e = hipMemsetAsync(lists[t & 1], 0, sizeof(uint32_t), stream)) != hipSuccess) return e;
        hipLaunchKernelGGL(ajx_row_scan, dim3(grid), dim3(block), lds, stream, d_sets, d_arena, d_offs, d_lens, n,
                           t == 0 ? d_perm : nullptr, in, in ? in + 1 : nullptr, d_rows, row_stride, d_tri, d_err,
                           d_bm, stride, d_slow, d_slow + 1, nxt, nxt + 1, L, blob_region, stop);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace ajx
