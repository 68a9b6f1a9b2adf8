// TEST-ONLY: host implementation of hipstub/hip/hip_runtime.h (see there) and of the kernel
// launchers ajx_api.cpp calls (ajx_kernels.h): every launch writes the outputs the real
// kernels write (slow-list count, capture rows, results) from the calling thread, so the
// ThreadSanitizer run sees the same host-side accesses to a workspace's buffers.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstring>

#include "../../authorino_amd/csrc/ajx_kernels.h"

struct ihipStream_t {
    int flags;
};
struct ihipEvent_t {
    std::atomic<uint64_t> stamp{0};
};
static std::atomic<uint64_t> g_clock{1};

hipError_t hipSetDevice(int d) { return d == 0 ? hipSuccess : hipErrorNoDevice; }
hipError_t hipGetDevice(int* d) {
    *d = 0;
    return hipSuccess;
}
hipError_t hipGetDeviceCount(int* n) {
    *n = 1;
    return hipSuccess;
}
hipError_t hipMallocRaw(void** p, size_t n) {
    *p = std::calloc(1, n ? n : 1);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p) {
    std::free(p);
    return hipSuccess;
}
hipError_t hipHostMallocRaw(void** p, size_t n, unsigned) { return hipMallocRaw(p, n); }
hipError_t hipHostFree(void* p) { return hipFree(p); }
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned) {
    *d = h;
    return hipSuccess;
}
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) {
    if (n) std::memmove(d, s, n);
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind k, hipStream_t) { return hipMemcpy(d, s, n, k); }
hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t) {
    std::memset(d, v, n);
    return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned f) {
    *s = new ihipStream_t{(int)f};
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
    delete s;
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamQuery(hipStream_t) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t* e) {
    *e = new ihipEvent_t();
    return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { return hipEventCreate(e); }
hipError_t hipEventDestroy(hipEvent_t e) {
    delete e;
    return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t) {
    e->stamp.store(g_clock.fetch_add(1), std::memory_order_release);
    return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t e) {
    (void)e->stamp.load(std::memory_order_acquire);
    return hipSuccess;
}
hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b) {
    *ms = (float)(b->stamp.load(std::memory_order_acquire) - a->stamp.load(std::memory_order_acquire)) * 1e-3f;
    return hipSuccess;
}
hipError_t hipGetLastError() { return hipSuccess; }
const char* hipGetErrorString(hipError_t e) { return e == hipSuccess ? "hipSuccess" : "hip stub error"; }

namespace ajx {

static void results(uint32_t n, uint8_t* tri, int32_t* err, uint64_t* bm, uint32_t stride) {
    for (uint32_t r = 0; r < n; r++) {
        tri[r] = 1;
        if (err) err[r] = -1;
        if (bm)
            for (uint32_t w = 0; w < stride; w++) bm[(size_t)r * stride + w] = 1;
    }
}

hipError_t launch_eval_scan(const uint8_t* const*, const uint32_t*, const uint8_t*, const uint64_t*, const uint32_t*,
                            uint32_t n, uint8_t* tri, int32_t* err, uint64_t* bm, uint32_t stride, hipStream_t, bool) {
    results(n, tri, err, bm, stride);
    return hipSuccess;
}
hipError_t launch_select(const uint8_t* const*, const uint32_t*, uint32_t, const uint8_t*, const uint64_t*,
                         const uint32_t*, uint32_t n, uint32_t* out, uint32_t stride, uint64_t* rows,
                         uint32_t row_stride, uint32_t* slow_count, uint32_t*, const uint32_t*, uint8_t*, uint32_t,
                         hipStream_t) {
    if (rows) {
        *slow_count = 0;
        for (uint32_t r = 0; r < n; r++) rows[(size_t)r * row_stride] = r;
    }
    std::memset(out, 0, (size_t)n * stride * 12);
    return hipSuccess;
}
hipError_t launch_select_rows(const uint8_t* const*, const uint8_t*, const uint64_t*, const uint32_t*, uint32_t n,
                              uint32_t* out, uint32_t stride, const uint64_t* rows, uint32_t row_stride, uint32_t,
                              const uint32_t*, bool, hipStream_t) {
    for (uint32_t r = 0; r < n; r++) out[(size_t)r * stride * 3] = (uint32_t)rows[(size_t)r * row_stride];
    return hipSuccess;
}
hipError_t launch_eval_fast(const uint8_t* const*, const uint32_t*, uint32_t, const uint8_t*, const uint64_t*,
                            const uint32_t*, uint32_t n, uint8_t* tri, int32_t* err, uint64_t* bm, uint32_t stride,
                            uint64_t* rows, uint32_t row_stride, uint32_t* slow_count, uint32_t*, hipStream_t, int,
                            const uint32_t*, bool, bool, uint32_t, const uint32_t*, uint8_t*, uint32_t) {
    *slow_count = n / 7;
    for (uint32_t r = 0; r < n; r++) rows[(size_t)r * row_stride] = r;
    results(n, tri, err, bm, stride);
    return hipSuccess;
}
bool stream_eligible(const uint8_t*, uint32_t) { return true; }
uint32_t stream_records(const uint8_t*) { return 1; }
hipError_t launch_eval_stream(const uint8_t* const*, const uint32_t*, uint32_t, uint32_t, const uint8_t*,
                              const uint64_t*, const uint32_t*, uint32_t n, uint8_t* tri, int32_t* err, uint64_t* bm,
                              uint32_t stride, uint64_t* rows, uint32_t row_stride, bool keep_rows,
                              uint32_t* stage_ids, uint32_t* slow_count, uint32_t*, hipStream_t, int, bool,
                              uint32_t, bool* zero) {
    // (as the small-batch instance: the counters left zero, the slow count at [3])
    slow_count[3] = n / 5;
    slow_count[0] = slow_count[1] = slow_count[2] = 0;
    if (zero) *zero = !keep_rows;
    if (keep_rows) slow_count[0] = n / 5;
    (void)stage_ids;
    if (keep_rows)
        for (uint32_t r = 0; r < n; r++) rows[(size_t)r * row_stride] = r;
    results(n, tri, err, bm, stride);
    return hipSuccess;
}
hipError_t launch_len_order(const uint32_t*, uint32_t n, uint32_t* hist, uint32_t* perm, hipStream_t,
                            uint32_t* pos_of) {
    hist[0] = n;
    for (uint32_t r = 0; r < n; r++) perm[r] = r;
    if (pos_of)
        for (uint32_t r = 0; r < n; r++) pos_of[r] = r;
    return hipSuccess;
}

}  // namespace ajx
