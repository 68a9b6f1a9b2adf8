// TEST-ONLY: a host stand-in for the few HIP runtime entry points ajx_api.cpp calls, so the
// C-ABI's host logic (workspaces, registry, locks) builds with g++ under ThreadSanitizer
// (tests/native/tsan_api.cpp). The "device" is host memory and every operation completes
// before it returns (hip_stub.cpp); kernels are the launchers' stubs there.
#pragma once
#include <stddef.h>
#include <stdint.h>

enum hipError_t { hipSuccess = 0, hipErrorInvalidValue = 1, hipErrorOutOfMemory = 2, hipErrorNoDevice = 100, hipErrorNotReady = 600 };
enum hipMemcpyKind { hipMemcpyHostToHost = 0, hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2,
                     hipMemcpyDeviceToDevice = 3, hipMemcpyDefault = 4 };
struct ihipStream_t;
struct ihipEvent_t;
typedef ihipStream_t* hipStream_t;
typedef ihipEvent_t* hipEvent_t;
constexpr unsigned hipStreamNonBlocking = 1;
constexpr unsigned hipEventDisableTiming = 2;
constexpr unsigned hipHostMallocDefault = 0;

hipError_t hipSetDevice(int);
hipError_t hipGetDevice(int*);
hipError_t hipGetDeviceCount(int*);
hipError_t hipMallocRaw(void**, size_t);
hipError_t hipFree(void*);
hipError_t hipHostMallocRaw(void**, size_t, unsigned);
hipError_t hipHostFree(void*);
hipError_t hipHostGetDevicePointer(void**, void*, unsigned);
hipError_t hipMemcpy(void*, const void*, size_t, hipMemcpyKind);
hipError_t hipMemcpyAsync(void*, const void*, size_t, hipMemcpyKind, hipStream_t);
hipError_t hipMemsetAsync(void*, int, size_t, hipStream_t);
hipError_t hipStreamCreateWithFlags(hipStream_t*, unsigned);
hipError_t hipStreamDestroy(hipStream_t);
hipError_t hipStreamSynchronize(hipStream_t);
hipError_t hipStreamQuery(hipStream_t);
hipError_t hipEventCreate(hipEvent_t*);
hipError_t hipEventCreateWithFlags(hipEvent_t*, unsigned);
hipError_t hipEventDestroy(hipEvent_t);
hipError_t hipEventRecord(hipEvent_t, hipStream_t);
hipError_t hipEventSynchronize(hipEvent_t);
hipError_t hipEventElapsedTime(float*, hipEvent_t, hipEvent_t);
hipError_t hipGetLastError();
const char* hipGetErrorString(hipError_t);

template <class T>
hipError_t hipMalloc(T** p, size_t n) {
    return hipMallocRaw(reinterpret_cast<void**>(p), n);
}
template <class T>
hipError_t hipHostMalloc(T** p, size_t n, unsigned f) {
    return hipHostMallocRaw(reinterpret_cast<void**>(p), n, f);
}
