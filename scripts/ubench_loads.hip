// Micro-benchmark (profiling only, not product code): read-throughput of the document
// arena under the access shapes a lane-per-request scan can use. Each variant touches
// every byte of every document once and folds it into a checksum per request.
//   A  per-lane 64-B windows (4 x dwordx4 of the lane's own document, next window prefetched)
//   B  per-lane 128-B windows (8 x dwordx4 = one full line, next line prefetched)
//   C  cooperative: 8 lanes load one 128-B line of one document (coalesced), via LDS
// build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_loads.hip -o /tmp/ubl
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);    \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__global__ __launch_bounds__(256) void varA(const uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                                            uint32_t n, uint32_t* out) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint8_t* d = arena + offs[r];
    const uint32_t len = lens[r];
    const uint32_t mis = (uint32_t)((uintptr_t)d & 15u);
    const uint4* a4 = (const uint4*)(d - mis);
    const uint32_t nblk = (len + mis + 15) / 16;
    uint32_t acc = 0;
    uint4 cur[4], nxt[4];
    for (int j = 0; j < 4; j++) cur[j] = j < (int)nblk ? a4[j] : make_uint4(0, 0, 0, 0);
    for (int j = 0; j < 4; j++) nxt[j] = 4 + j < (int)nblk ? a4[4 + j] : make_uint4(0, 0, 0, 0);
    for (uint32_t b0 = 0; b0 < nblk; b0 += 4) {
        for (int j = 0; j < 4; j++) acc ^= cur[j].x + cur[j].y * 3 + cur[j].z * 5 + cur[j].w * 7;
        for (int j = 0; j < 4; j++) {
            cur[j] = nxt[j];
            nxt[j] = b0 + 8 + j < nblk ? a4[b0 + 8 + j] : make_uint4(0, 0, 0, 0);
        }
    }
    out[r] = acc;
}

__global__ __launch_bounds__(256) void varB(const uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                                            uint32_t n, uint32_t* out) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint8_t* d = arena + offs[r];
    const uint32_t len = lens[r];
    const uint32_t mis = (uint32_t)((uintptr_t)d & 127u);
    const uint4* a4 = (const uint4*)(d - mis);
    const uint32_t nblk = (len + mis + 15) / 16;
    uint32_t acc = 0;
    uint4 cur[8], nxt[8];
    for (int j = 0; j < 8; j++) cur[j] = j < (int)nblk ? a4[j] : make_uint4(0, 0, 0, 0);
    for (int j = 0; j < 8; j++) nxt[j] = 8 + j < (int)nblk ? a4[8 + j] : make_uint4(0, 0, 0, 0);
    for (uint32_t b0 = 0; b0 < nblk; b0 += 8) {
        for (int j = 0; j < 8; j++) acc ^= cur[j].x + cur[j].y * 3 + cur[j].z * 5 + cur[j].w * 7;
        for (int j = 0; j < 8; j++) {
            cur[j] = nxt[j];
            nxt[j] = b0 + 16 + j < nblk ? a4[b0 + 16 + j] : make_uint4(0, 0, 0, 0);
        }
    }
    out[r] = acc;
}

// C: wave-cooperative line loads into an LDS ring (2 slots x 64 docs x 128 B per wave),
// 8 lanes per line; each lane then reads its own document's window from LDS.
__global__ __launch_bounds__(256) void varC(const uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                                            uint32_t n, uint32_t* out) {
    __shared__ uint4 ring[4][2][64 * 8];  // [wave][slot][doc*8 + chunk]
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t rr = r < n ? r : n - 1;
    const uint8_t* d = arena + offs[rr];
    const uint32_t len = r < n ? lens[rr] : 0;
    const uintptr_t first = (uintptr_t)d & ~(uintptr_t)127;
    const uint32_t nl = len ? (uint32_t)((((uintptr_t)d + len - 1) & ~(uintptr_t)127) - first) / 128 + 1 : 0;
    // max lines over the wave
    uint32_t wmax = nl;
    for (int o = 32; o; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, o));
    uint32_t acc = 0;
    auto issue = [&](uint32_t k, uint32_t slot) {
        for (uint32_t i = 0; i < 8; i++) {
            const uint32_t doc = 8 * i + (lane >> 3);
            const uintptr_t f = (uintptr_t)__shfl((long long)first, doc);
            const uint32_t l = (uint32_t)__shfl((int)nl, doc);
            const uint32_t kk = k < l ? k : (l ? l - 1 : 0);
            const uint32_t c = (lane & 7) ^ (doc & 7);
            const uint4* src = (const uint4*)(f + 128 * kk + 16 * c);
            ring[wv][slot][doc * 8 + (lane & 7)] = *src;
        }
    };
    issue(0, 0);
    for (uint32_t k = 0; k < wmax; k++) {
        if (k + 1 < wmax) issue(k + 1, (k + 1) & 1);
        __builtin_amdgcn_wave_barrier();
        if (k < nl)
            for (uint32_t j = 0; j < 8; j++) {
                const uint4 v = ring[wv][k & 1][lane * 8 + (j ^ (lane & 7))];
                acc ^= v.x + v.y * 3 + v.z * 5 + v.w * 7;
            }
        __builtin_amdgcn_wave_barrier();
    }
    if (r < n) out[r] = acc;
}

// D: perfectly coalesced grid-stride stream over the whole arena (the practical ceiling)
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

// E: per-lane 128-B windows, two lines in flight ahead
__global__ __launch_bounds__(256) void varE(const uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                                            uint32_t n, uint32_t* out) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint8_t* d = arena + offs[r];
    const uint32_t len = lens[r];
    const uint32_t mis = (uint32_t)((uintptr_t)d & 127u);
    const uint4* a4 = (const uint4*)(d - mis);
    const uint32_t nblk = (len + mis + 15) / 16;
    uint32_t acc = 0;
    uint4 c0[8], c1[8], c2[8];
    for (int j = 0; j < 8; j++) c0[j] = j < (int)nblk ? a4[j] : make_uint4(0, 0, 0, 0);
    for (int j = 0; j < 8; j++) c1[j] = 8 + j < (int)nblk ? a4[8 + j] : make_uint4(0, 0, 0, 0);
    for (uint32_t b0 = 0; b0 < nblk; b0 += 8) {
        for (int j = 0; j < 8; j++) c2[j] = b0 + 16 + j < nblk ? a4[b0 + 16 + j] : make_uint4(0, 0, 0, 0);
        for (int j = 0; j < 8; j++) acc ^= c0[j].x + c0[j].y * 3 + c0[j].z * 5 + c0[j].w * 7;
        for (int j = 0; j < 8; j++) { c0[j] = c1[j]; c1[j] = c2[j]; }
    }
    out[r] = acc;
}


// F: per-lane 128-B windows landed in LDS by LDS-DMA (global_load_lds_dwordx4; no VGPRs
// hold the data), two windows per lane (the next one in flight while the current one is
// read back with ds_read_b128). Chunk-major ring: chunk j of slot s of lane l at
// ((s * 8 + j) * 64 + l) * 16 inside the wave's region.
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void varF(const uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                                                 uint32_t n, uint32_t* out) {
    extern __shared__ uint4 sm[];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint4* wr = sm + wv * (2 * 8 * 64);
    typedef __attribute__((address_space(3))) uint8_t lds8;
    lds8* wl = (lds8*)(uint8_t*)wr;
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t rr = r < n ? r : n - 1;
    const uint8_t* d = arena + offs[rr];
    const uint32_t len = r < n ? lens[rr] : 0;
    const uint32_t mis = (uint32_t)((uintptr_t)d & 15u);
    const uint8_t* a = d - mis;
    const uint32_t nblk = (len + mis + 15) / 16;
    uint32_t wmax = (nblk + 7) / 8;
    for (int o = 32; o; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, o));
    uint32_t acc = 0;
    auto issue = [&](uint32_t w, uint32_t slot) {
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t b = w * 8 + j;
            const uint8_t* src = a + 16 * (b < nblk ? b : 0);
            __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(wl + (slot * 8 + j) * 1024), 16, 0, 0);
        }
    };
    issue(0, 0);
    for (uint32_t w = 0; w < wmax; w++) {
        if (w + 1 < wmax) {
            issue(w + 1, (w + 1) & 1);
            __builtin_amdgcn_s_waitcnt(0x0F78);  // vmcnt(8): this window landed
        } else {
            __builtin_amdgcn_s_waitcnt(0x0F70);
        }
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint4 v = wr[((w & 1) * 8 + j) * 64 + lane];
            acc ^= v.x + v.y * 3 + v.z * 5 + v.w * 7;
        }
    }
    if (r < n) out[r] = acc;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : (1u << 20);
    std::mt19937 g(2);
    std::vector<uint32_t> lens(n);
    std::vector<uint64_t> offs(n);
    uint64_t tot = 0;
    for (uint32_t i = 0; i < n; i++) {
        lens[i] = 768 + g() % 513;
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
    CK(hipMalloc(&dout, n * 4));
    CK(hipMemcpy(doffs, offs.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlens, lens.data(), n * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[7] = {"A_lane64B", "B_lane128B", "C_coop_lds", "D_coalesced", "E_lane128B_2ahead", "F_dma128B_wpb4", "F_dma128B_wpb2"};
    CK(hipFuncSetAttribute((const void*)varF<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    for (int rep = 0; rep < 3; rep++)
        for (int v = 0; v < 7; v++) {
            CK(hipEventRecord(e0));
            for (int it = 0; it < 10; it++) {
                if (v == 0) varA<<<(n + 255) / 256, 256>>>(da, doffs, dlens, n, dout);
                if (v == 1) varB<<<(n + 255) / 256, 256>>>(da, doffs, dlens, n, dout);
                if (v == 2) varC<<<(n + 255) / 256, 256>>>(da, doffs, dlens, n, dout);
                if (v == 3) varD<<<4096, 256>>>((const uint4*)da, tot / 16, dout);
                if (v == 4) varE<<<(n + 255) / 256, 256>>>(da, doffs, dlens, n, dout);
                if (v == 5) varF<4><<<(n + 255) / 256, 256, 65536>>>(da, doffs, dlens, n, dout);
                if (v == 6) varF<2><<<(n + 127) / 128, 128, 32768>>>(da, doffs, dlens, n, dout);
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
