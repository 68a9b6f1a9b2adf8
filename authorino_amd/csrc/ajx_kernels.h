// ajx_kernels.h — host-side launch wrappers for the gfx950 kernels (ajx_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ajx {

hipError_t launch_eval_scan(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, const uint8_t* d_arena,
                            const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n, uint8_t* d_tri,
                            int32_t* d_err, uint64_t* d_bm, uint32_t stride, hipStream_t stream, bool mods = false);

// gjson.Get of every pattern's selector: d_out = u32[n][stride][3] {start, len, type | esc << 8}.
// With d_rows: the single-pass stage A captures all spans in one scan per document (rows of
// 1 + n_selectors u64, requests it can not prove go through the exact Get); without, the
// exact Get per selector.
hipError_t launch_select(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, uint32_t shared_blob_bytes,
                         const uint8_t* d_arena, const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n,
                         uint32_t* d_out, uint32_t stride, uint64_t* d_rows, uint32_t row_stride,
                         uint32_t* d_slow_count, uint32_t* d_slow_ids, const uint32_t* d_perm, uint8_t* d_text,
                         uint32_t text_stride, hipStream_t stream);

// The values of patterns [p0, p0 + stride) of sets[0] from capture rows an earlier
// single-pass evaluation of that ruleset wrote (no document scan; slow rows: exact Get).
// d_perm: that evaluation's work-item order (nullptr: identity); wave_rows: the rows are in
// the fused kernels' wave-interleaved layout (indexed by work-item), else one per request.
hipError_t launch_select_rows(const uint8_t* const* d_sets, const uint8_t* d_arena, const uint64_t* d_offs,
                              const uint32_t* d_lens, uint32_t n, uint32_t* d_out, uint32_t stride,
                              const uint64_t* d_rows, uint32_t row_stride, uint32_t p0, const uint32_t* d_perm,
                              bool wave_rows, hipStream_t stream);

}  // namespace ajx

namespace ajx {

// Largest ruleset blob the kernels stage into LDS (a batch over one ruleset).
constexpr uint32_t kMaxSharedBlobBytes = 48 * 1024;
// multi-tenant batches: the LDS an 8-wave workgroup stages its runs' blobs in, next to its
// window rings (16 KiB + 8 x 8 KiB rings per group keeps 2 groups = 4 waves/SIMD per CU;
// c4: 83 % of the waves on one staged ruleset, against 80 % for 4-wave groups with 8 KiB)
constexpr uint32_t kMaxTenantStageBytes = 16 * 1024;
constexpr uint32_t kTenantBlock = 512;

// `mods` (every launcher): a ruleset of the batch has modifier chains (RulesetHdr
// n_modifiers); the exact scan then runs its instance with modifier buffers.
// single-pass kernel + exact scan of the requests it hands over (d_slow_count is zeroed
// on the stream first; d_slow_ids needs room for n entries). shared_blob_bytes: the
// blob size of sets[0] when every request uses it and it fits kMaxSharedBlobBytes,
// else 0. mode: 0 the single-pass kernel (default, ajx_fast.h); profiling only: 1
// stage-A loads only, 2 stage-A loads + classification, 3 stage A and stage B as
// separate launches.
hipError_t launch_eval_fast(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, uint32_t shared_blob_bytes,
                            const uint8_t* d_arena, const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n,
                            uint8_t* d_tri, int32_t* d_err, uint64_t* d_bm, uint32_t stride, uint64_t* d_rows,
                            uint32_t row_stride, uint32_t* d_slow_count, uint32_t* d_slow_ids, hipStream_t stream,
                            int mode = 0, const uint32_t* d_perm = nullptr, bool mods = false,
                            bool keep_rows = true, uint32_t lean_feat = 3, const uint32_t* d_pos_of = nullptr,
                            uint8_t* d_tout = nullptr, uint32_t n_out = 1);
// (d_pos_of, d_tout: with d_perm, the lean kernel writes its outputs to d_tout in work-item
// order, tri-states | error indices | bitmaps at 256-byte aligned offsets
// (tout_bytes), and ajx_unpermute gathers them to request order by d_pos_of
// (launch_len_order); n_out: results per request)
inline size_t tout_bytes(uint32_t n, uint32_t n_out, uint32_t stride) {
    const size_t a = ((size_t)n * n_out + 255u) & ~(size_t)255u;
    const size_t b = ((size_t)n * n_out * 4u + 255u) & ~(size_t)255u;
    return a + b + (size_t)n * stride * 8u;
}

// The lean single-pass kernel (ajx_lean.hip, one ruleset for the batch): stage A with the
// lean scan and stage B per work-item; requests it can not prove go to d_slow_ids (the
// caller zeroes d_slow_count first and runs the exact scan after). shared_blob_bytes: the
// blob of sets[0] is staged into LDS (0: read from global memory). abl (profiling builds
// with AJX_LEAN_ABLATIONS, kernel modes 15..18): 1..4 the stage-A ablations, no stage B.
// lean_feat: RulesetHdr::lean_feat of sets[0] (the walker instance; 3 takes every ruleset).
hipError_t launch_lean(const uint8_t* const* d_sets, uint32_t shared_blob_bytes, const uint8_t* d_arena,
                       const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n, uint64_t* d_rows,
                       uint32_t row_stride, uint32_t* d_slow_count, uint32_t* d_slow_ids, uint8_t* d_tri,
                       int32_t* d_err, uint64_t* d_bm, uint32_t stride, hipStream_t stream, int abl,
                       const uint32_t* d_perm, bool keep_rows, uint32_t lean_feat, bool out_k = false);

// The multi-tenant single-pass kernel (ajx_lean.hip): each workgroup stages its runs'
// rulesets in LDS; waves of one staged ruleset run the lean scan, others the token scanner.
hipError_t launch_tenant(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, const uint8_t* d_arena,
                         const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n, uint64_t* d_rows,
                         uint32_t row_stride, uint32_t* d_slow_count, uint32_t* d_slow_ids, uint8_t* d_tri,
                         int32_t* d_err, uint64_t* d_bm, uint32_t stride, hipStream_t stream, const uint32_t* d_perm);

// The streaming kernel (ajx_stream.h), its stage B (ajx_stream_finish) and the exact scan of
// what they hand over: one ruleset for the batch (sets[0], staged in LDS); stream_eligible
// says whether it can take the ruleset. d_rows: rows of row_stride >= 5 + n_rec
// words for n requests (wave layout, work-item = request): the rows stage B reads, and with
// keep_rows every request's row for authjx_select_from_eval_device. d_stage_ids: n u32;
// d_slow_count[1] (the stage-B count) and [2] (finished waves) follow the slow count;
// counters_zero (in): [0..2] are zero already, no fill; (out): this launch leaves them zero
// (the small-batch instance: its last wave clears them, the slow count moved to [3]). mode (profiling): 1 the structural pass alone, 2 no fold. per: requests per wave
// (1..32, 0 = 32): fewer for small batches, so more waves share the walk. d_set_of_req
// (a multi-tenant batch, every ruleset stream-eligible): one request per wave under its
// own ruleset, tables from global memory; n_rec then the largest of the batch.
bool stream_eligible(const uint8_t* host_blob, uint32_t blob_bytes);
// capture records of the streaming kernel's rows (n_selectors + exact selectors' prefixes)
uint32_t stream_records(const uint8_t* host_blob);
constexpr uint32_t kStreamSpan = 32;  // requests per wave at most (stream::kSpan)
hipError_t launch_eval_stream(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, uint32_t blob_bytes,
                              uint32_t n_rec, const uint8_t* d_arena, const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n,
                              uint8_t* d_tri, int32_t* d_err, uint64_t* d_bm, uint32_t stride, uint64_t* d_rows,
                              uint32_t row_stride, bool keep_rows, uint32_t* d_stage_ids, uint32_t* d_slow_count,
                              uint32_t* d_slow_ids, hipStream_t stream, int mode = 0, bool mods = false,
                              uint32_t per = 0, bool* counters_zero = nullptr);

// Length-bucketed request order for the single-pass kernel: d_perm[n] = request ids,
// longest 8-byte length class first; d_hist needs 2 * 1024 + 1 u32 of scratch.
// d_pos_of (optional): n u32, the inverse (work-item of each request).
hipError_t launch_len_order(const uint32_t* d_lens, uint32_t n, uint32_t* d_hist, uint32_t* d_perm,
                            hipStream_t stream, uint32_t* d_pos_of = nullptr);

}  // namespace ajx
