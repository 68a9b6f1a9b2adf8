// Micro-benchmark (profiling only, not product code): read throughput of the document
// arena under the access shapes of a row-per-document scan, where G consecutive lanes
// (a "row") read one document 16 B per lane, G x 16 B per step, and stage it in LDS.
//   R<G>   rows of G lanes, 64/G documents per wave at a time, one step prefetched
//   R<G>p2 the same with two steps in flight
//   D      perfectly coalesced grid-stride stream over the whole arena (the ceiling)
// Each wave takes 64 consecutive documents (the request order a length-sorted batch
// gives it) and walks them 64/G at a time.
// build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_wave_loads.hip -o /tmp/ubw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

constexpr uint32_t kDocBuf = 2048;  // LDS bytes per row (documents up to ~2 KiB here)

template <int G, int AHEAD>
__global__ __launch_bounds__(256) void rowload(const uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                                               uint32_t n, uint32_t* out) {
    constexpr int R = 64 / G;
    __shared__ uint4 buf[4][R][kDocBuf / 16];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, row = lane / G, rl = lane % G;
    const uint32_t wave = blockIdx.x * 4 + wv;
    uint32_t acc = 0;
    for (uint32_t g = 0; g < 64 / R; g++) {
        const uint32_t r = wave * 64 + g * R + row;
        const bool live = r < n;
        const uint8_t* d = arena + (live ? offs[r] : 0);
        const uint32_t len = live ? lens[r] : 0;
        const uint32_t mis = (uint32_t)((uintptr_t)d & 15u);
        const uint4* a4 = (const uint4*)(d - mis);
        const uint32_t nblk = len ? (len + mis + 15) / 16 : 0;
        uint32_t nstep = (nblk + G - 1) / G;
        for (int o = 32; o >= 1; o >>= 1) nstep = max(nstep, (uint32_t)__shfl_xor((int)nstep, o));
        uint4 pf[AHEAD + 1];
#pragma unroll
        for (int k = 0; k < AHEAD; k++) {
            const uint32_t b = k * G + rl;
            pf[k] = b < nblk ? a4[b] : make_uint4(0, 0, 0, 0);
        }
        for (uint32_t s = 0; s < nstep; s++) {
            const uint32_t b = (s + AHEAD) * G + rl;
            pf[AHEAD] = b < nblk ? a4[b] : make_uint4(0, 0, 0, 0);
            const uint4 v = pf[0];
            const uint32_t bb = s * G + rl;
            if (bb < kDocBuf / 16) buf[wv][row][bb] = v;
            acc ^= v.x + v.y * 3 + v.z * 5 + v.w * 7;
#pragma unroll
            for (int k = 0; k < AHEAD; k++) pf[k] = pf[k + 1];
        }
        __builtin_amdgcn_wave_barrier();
        acc += ((const uint32_t*)buf[wv][row])[rl];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void varD(const uint4* a, uint64_t n16, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        uint4 v0 = a[i], v1 = a[i + stride], v2 = a[i + 2 * stride], v3 = a[i + 3 * stride];
        acc ^= v0.x + v1.y * 3 + v2.z * 5 + v3.w * 7;
    }
    for (; i < n16; i += stride) acc ^= a[i].x;
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : (1u << 20);
    const uint32_t lo = argc > 2 ? atoi(argv[2]) : 768, hi = argc > 3 ? atoi(argv[3]) : 1280;
    std::mt19937 g(2);
    std::vector<uint32_t> lens(n);
    std::vector<uint64_t> offs(n);
    uint64_t tot = 0;
    for (uint32_t i = 0; i < n; i++) {
        lens[i] = lo + g() % (hi - lo + 1);
        offs[i] = tot;
        tot += lens[i];
    }
    uint8_t* da;
    uint64_t* doffs;
    uint32_t *dlens, *dout;
    CK(hipMalloc(&da, tot + 256));
    CK(hipMemset(da, 0x41, tot + 256));
    CK(hipMalloc(&doffs, n * 8));
    CK(hipMalloc(&dlens, n * 4));
    CK(hipMalloc(&dout, (size_t)(n + 4096) * 256));
    CK(hipMemcpy(doffs, offs.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlens, lens.data(), n * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t waves = (n + 63) / 64, blocks = (waves + 3) / 4;
    const char* names[] = {"R16", "R16p2", "R16p4", "R8", "R8p2", "R32", "R64", "D_coalesced"};
    const int nv = sizeof(names) / sizeof(names[0]);
    for (int rep = 0; rep < 3; rep++)
        for (int v = 0; v < nv; v++) {
            CK(hipEventRecord(e0));
            for (int it = 0; it < 10; it++) {
                if (v == 0) rowload<16, 1><<<blocks, 256>>>(da, doffs, dlens, n, dout);
                if (v == 1) rowload<16, 2><<<blocks, 256>>>(da, doffs, dlens, n, dout);
                if (v == 2) rowload<16, 4><<<blocks, 256>>>(da, doffs, dlens, n, dout);
                if (v == 3) rowload<8, 1><<<blocks, 256>>>(da, doffs, dlens, n, dout);
                if (v == 4) rowload<8, 2><<<blocks, 256>>>(da, doffs, dlens, n, dout);
                if (v == 5) rowload<32, 2><<<blocks, 256>>>(da, doffs, dlens, n, dout);
                if (v == 6) rowload<64, 2><<<blocks, 256>>>(da, doffs, dlens, n, dout);
                if (v == 7) varD<<<4096, 256>>>((const uint4*)da, tot / 16, dout);
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= 10;
            if (rep == 2) printf("%s: %.3f ms  %.0f GB/s\n", names[v], ms, tot / (ms * 1e-3) / 1e9);
        }
    return 0;
}
