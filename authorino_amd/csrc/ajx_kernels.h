// ajx_kernels.h — host-side launch wrappers for the gfx950 kernels (ajx_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ajx {

hipError_t launch_eval_scan(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, const uint8_t* d_arena,
                            const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n, uint8_t* d_tri,
                            int32_t* d_err, uint64_t* d_bm, uint32_t stride, hipStream_t stream);

}  // namespace ajx

namespace ajx {

// single-pass fast kernel + exact scan of the requests it hands over (d_slow_count is
// zeroed on the stream first; d_slow_ids needs room for n entries)
hipError_t launch_eval_fast(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, const uint8_t* d_arena,
                            const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n, uint8_t* d_tri,
                            int32_t* d_err, uint64_t* d_bm, uint32_t stride, uint64_t* d_rows, uint32_t row_stride,
                            uint32_t* d_slow_count, uint32_t* d_slow_ids, hipStream_t stream, int ablate = 0);

}  // namespace ajx
