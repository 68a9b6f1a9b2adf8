// ajx_kernels.h — host-side launch wrappers for the gfx950 kernels (ajx_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ajx {

hipError_t launch_eval_scan(const uint8_t* const* d_sets, const uint32_t* d_set_of_req, const uint8_t* d_arena,
                            const uint64_t* d_offs, const uint32_t* d_lens, uint32_t n, uint8_t* d_tri,
                            int32_t* d_err, uint64_t* d_bm, uint32_t stride, hipStream_t stream);

}  // namespace ajx
