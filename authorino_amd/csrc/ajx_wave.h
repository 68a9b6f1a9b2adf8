// ajx_wave.h — wave64 primitives of the streaming scan (ajx_stream.h): ballots, lane
// shifts and 64-lane scans by DPP (gfx9 row_shr / row_bcast / wave_shr / wave_shl).
//
// Every primitive is called with the whole wave active (EXEC = all 64 lanes) and from
// wave-uniform control flow only.
//
// The test-only host builds (tests/native, g++) run the same code on 64 host
// threads per wave: each primitive exchanges the lanes' values through a shared array
// between two barriers (WaveEmu). The product library has no host copy of this code.
#pragma once
#include <stdint.h>

#if !defined(__HIPCC__)
#include <condition_variable>
#include <mutex>
#include <thread>
#endif

#ifndef AJX_HD
#define AJX_HD __device__ __forceinline__
#endif

namespace ajx {
namespace wave {

AJX_HD uint64_t mask_lt(uint32_t l) { return (1ull << l) - 1ull; }             // lanes < l
AJX_HD uint64_t mask_le(uint32_t l) { return l >= 63 ? ~0ull : (2ull << l) - 1ull; }  // lanes <= l

#if defined(__HIPCC__)

AJX_HD uint32_t lane() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
AJX_HD uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
// v of lane l - 1 (lane 0: fill)
AJX_HD uint32_t shr1(uint32_t v, uint32_t fill) { return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x138, 0xF, 0xF, false); }
// v of lane l + 1 (lane 63: fill)
AJX_HD uint32_t shl1(uint32_t v, uint32_t fill) { return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x130, 0xF, 0xF, false); }
AJX_HD uint32_t readlane(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }
AJX_HD uint32_t uniform(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
AJX_HD uint32_t bpermute(uint32_t v, uint32_t src_lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}
// keeps the compiler from moving LDS accesses across this point (lanes of the wave
// exchanging values through LDS; the LDS itself serves one wave's accesses in order)
AJX_HD void sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// x from lane l - k within each row of 16 (fill where there is none)
template <int CTRL, int ROWS = 0xF>
AJX_HD uint32_t dpp(uint32_t fill, uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)x, CTRL, ROWS, 0xF, false);
}

// inclusive scans over the 64 lanes (lane l: op over lanes 0..l)
template <class Op>
AJX_HD uint32_t scan_incl(uint32_t x, uint32_t ident, Op op) {
    x = op(dpp<0x111>(ident, x), x);
    x = op(dpp<0x112>(ident, x), x);
    x = op(dpp<0x114>(ident, x), x);
    x = op(dpp<0x118>(ident, x), x);
    x = op(dpp<0x142, 0xA>(ident, x), x);
    x = op(dpp<0x143, 0xC>(ident, x), x);
    return x;
}

// the same for a struct of dwords
template <int CTRL, int ROWS, class T>
AJX_HD T dpp_t(const T& fill, const T& x) {
    T r;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); i++)
        reinterpret_cast<uint32_t*>(&r)[i] =
            dpp<CTRL, ROWS>(reinterpret_cast<const uint32_t*>(&fill)[i], reinterpret_cast<const uint32_t*>(&x)[i]);
    return r;
}
template <class T, class Op>
AJX_HD T scan_incl_t(T x, const T& ident, Op op) {
    x = op(dpp_t<0x111, 0xF>(ident, x), x);
    x = op(dpp_t<0x112, 0xF>(ident, x), x);
    x = op(dpp_t<0x114, 0xF>(ident, x), x);
    x = op(dpp_t<0x118, 0xF>(ident, x), x);
    x = op(dpp_t<0x142, 0xA>(ident, x), x);
    x = op(dpp_t<0x143, 0xC>(ident, x), x);
    return x;
}
template <class T>
AJX_HD T shr1_t(const T& x, const T& fill) {
    T r;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); i++)
        reinterpret_cast<uint32_t*>(&r)[i] =
            shr1(reinterpret_cast<const uint32_t*>(&x)[i], reinterpret_cast<const uint32_t*>(&fill)[i]);
    return r;
}
template <class T>
AJX_HD T readlane_t(const T& x, uint32_t l) {
    T r;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); i++)
        reinterpret_cast<uint32_t*>(&r)[i] = readlane(reinterpret_cast<const uint32_t*>(&x)[i], l);
    return r;
}
// LDS atomics (the wave's own LDS region)
AJX_HD void lds_min(uint32_t* p, uint32_t v) { atomicMin(p, v); }
AJX_HD void lds_or64(uint64_t* p, uint64_t v) { atomicOr((unsigned long long*)p, (unsigned long long)v); }
AJX_HD uint32_t lds_cas(uint32_t* p, uint32_t cmp, uint32_t v) { return atomicCAS(p, cmp, v); }

#else  // host emulation (tests only): 64 threads per wave

struct Barrier {  // (C++17: no std::barrier)
    std::mutex m;
    std::condition_variable cv;
    uint32_t count = 0, gen = 0;
    void arrive_and_wait() {
        std::unique_lock<std::mutex> lk(m);
        const uint32_t g = gen;
        if (++count == 64) {
            count = 0;
            gen++;
            cv.notify_all();
            return;
        }
        cv.wait(lk, [&] { return gen != g; });
    }
};
struct WaveEmu {
    Barrier bar;
    uint64_t x[64];
};
inline thread_local WaveEmu* t_emu = nullptr;
inline thread_local uint32_t t_lane = 0;

inline uint32_t lane() { return t_lane; }
// every lane publishes v; f(array) is evaluated by each lane after the first barrier
template <class F>
inline uint64_t exchange(uint64_t v, F f) {
    WaveEmu* e = t_emu;
    e->x[t_lane] = v;
    e->bar.arrive_and_wait();
    const uint64_t r = f(e->x);
    e->bar.arrive_and_wait();
    return r;
}
inline uint64_t ballot(bool p) {
    return exchange(p ? 1u : 0u, [](const uint64_t* a) {
        uint64_t m = 0;
        for (int i = 0; i < 64; i++) m |= (a[i] & 1ull) << i;
        return m;
    });
}
inline uint32_t shr1(uint32_t v, uint32_t fill) {
    const uint32_t l = t_lane;
    return (uint32_t)exchange(v, [&](const uint64_t* a) { return l ? a[l - 1] : (uint64_t)fill; });
}
inline uint32_t shl1(uint32_t v, uint32_t fill) {
    const uint32_t l = t_lane;
    return (uint32_t)exchange(v, [&](const uint64_t* a) { return l < 63 ? a[l + 1] : (uint64_t)fill; });
}
inline uint32_t readlane(uint32_t v, uint32_t src) {
    return (uint32_t)exchange(v, [&](const uint64_t* a) { return a[src & 63]; });
}
inline uint32_t uniform(uint32_t v) {
    return (uint32_t)exchange(v, [](const uint64_t* a) { return a[0]; });
}
inline uint32_t bpermute(uint32_t v, uint32_t src) {
    // (each lane names its own source: publish (v, src), read a[src])
    return (uint32_t)exchange(v, [&](const uint64_t* a) { return a[src & 63]; });
}
inline void sync() {
    t_emu->bar.arrive_and_wait();
}
template <class Op>
inline uint32_t scan_incl(uint32_t x, uint32_t ident, Op op) {
    const uint32_t l = t_lane;
    (void)ident;
    return (uint32_t)exchange(x, [&](const uint64_t* a) {
        uint32_t r = (uint32_t)a[0];
        for (uint32_t i = 1; i <= l; i++) r = op(r, (uint32_t)a[i]);
        return (uint64_t)r;
    });
}
// structs travel as pointers to the lanes' own copies (valid until the second barrier)
template <class T, class F>
inline T exchange_t(const T& v, F f) {
    WaveEmu* e = t_emu;
    e->x[t_lane] = (uint64_t)(uintptr_t)&v;
    e->bar.arrive_and_wait();
    const T r = f([&](uint32_t i) -> const T& { return *reinterpret_cast<const T*>((uintptr_t)e->x[i]); });
    e->bar.arrive_and_wait();
    return r;
}
template <class T, class Op>
inline T scan_incl_t(T x, const T& ident, Op op) {
    const uint32_t l = t_lane;
    (void)ident;
    return exchange_t(x, [&](auto at) {
        T r = at(0);
        for (uint32_t i = 1; i <= l; i++) r = op(r, at(i));
        return r;
    });
}
template <class T>
inline T shr1_t(const T& x, const T& fill) {
    const uint32_t l = t_lane;
    return exchange_t(x, [&](auto at) { return l ? at(l - 1) : fill; });
}
template <class T>
inline T readlane_t(const T& x, uint32_t src) {
    return exchange_t(x, [&](auto at) { return at(src & 63); });
}
inline void lds_min(uint32_t* p, uint32_t v) {
    uint32_t o = __atomic_load_n(p, __ATOMIC_RELAXED);
    while (v < o && !__atomic_compare_exchange_n(p, &o, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
    }
}
inline void lds_or64(uint64_t* p, uint64_t v) { __atomic_fetch_or(p, v, __ATOMIC_RELAXED); }
inline uint32_t lds_cas(uint32_t* p, uint32_t cmp, uint32_t v) {
    __atomic_compare_exchange_n(p, &cmp, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED);
    return cmp;
}

// runs body(lane) on 64 threads as one emulated wave
template <class Body>
inline void run_wave(Body body) {
    WaveEmu emu;
    std::thread th[64];
    for (uint32_t i = 0; i < 64; i++)
        th[i] = std::thread([&, i] {
            t_emu = &emu;
            t_lane = i;
            body(i);
        });
    for (auto& t : th) t.join();
}

#endif

AJX_HD uint32_t scan_add(uint32_t x) {
    return scan_incl(x, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}
AJX_HD uint32_t scan_max(uint32_t x) {
    return scan_incl(x, 0u, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
}

}  // namespace wave
}  // namespace ajx
