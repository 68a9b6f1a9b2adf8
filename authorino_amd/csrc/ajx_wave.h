// ajx_wave.h — the vector-style primitives the wave-cooperative kernel (ajx_row.h) is
// written in, so that one source runs as gfx950 device code and, for the CPU test
// suite, as a 64-lane emulation on the host.
//
// The kernel is written as the program of one wavefront: a `V` is a per-lane u32 (a
// VGPR), a `M` a per-lane condition (a lane mask), plain integers are wave-uniform
// (SGPRs). Control flow is uniform: per-lane choices are selects (`sel`), per-lane
// loops run while any lane still has work (`any`). Cross-lane steps are explicit
// (ballot, DPP row shifts inside 16-lane rows, bpermute).
//
// Device build: V = uint32_t, M = bool; every primitive is one or a few instructions.
// Host build (tests/native only; the product library has no host copy): V holds the 64
// lanes' values and every operation loops over them in lane order, which also fixes
// the order of LDS atomics within an instruction.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
// (both passes of a hipcc compile: the host pass only parses these __device__ bodies)
#define AJW_DEV 1
#include <hip/hip_runtime.h>
#define AJW __device__ __forceinline__
#define AJW_HD __host__ __device__ inline
#if defined(__HIP_DEVICE_COMPILE__)
#define AJW_GPU(x) x
#else
#define AJW_GPU(x) 0
#endif
#else
#define AJW_DEV 0
#define AJW inline
#define AJW_HD inline
#include <cstring>
#endif

namespace ajx {
namespace w {

#if AJW_DEV
using V = uint32_t;
using M = bool;
typedef __attribute__((address_space(3))) uint8_t lds_u8_t;
using Lds = lds_u8_t*;  // a byte address in the workgroup's LDS

AJW V lane() { return AJW_GPU(__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u))); }
AJW V sel(M m, V a, V b) { return m ? a : b; }
AJW uint64_t ballot(M m) { return __ballot(m); }
AJW bool any(M m) { return __ballot(m) != 0; }
AJW V popc(V x) { return (V)__builtin_popcount(x); }
AJW V ctz(V x) { return x ? (V)__builtin_ctz(x) : 32u; }
AJW V hibit(V x) { return x ? 31u - (V)__builtin_clz(x) : 0xFFFFFFFFu; }  // highest set bit
AJW V alignbyte(V hi, V lo, V sh) { return AJW_GPU(__builtin_amdgcn_alignbyte(hi, lo, sh)); }
// value of lane (lane - k) of the same 16-lane row, 0 for the first k lanes of a row
template <int K>
AJW V row_shr(V v) {
    return (V)AJW_GPU(__builtin_amdgcn_update_dpp(0, (int)v, 0x110 + K, 0xF, 0xF, true));
}
// value of lane (lane + k) of the same row, 0 for the last k lanes
template <int K>
AJW V row_shl(V v) {
    return (V)AJW_GPU(__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + K, 0xF, 0xF, true));
}
AJW V shfl(V v, V src) { return (V)AJW_GPU(__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v)); }
AJW uint32_t readlane(V v, uint32_t l) { return (uint32_t)AJW_GPU(__builtin_amdgcn_readlane((int)v, (int)l)); }
AJW uint32_t readfirst(V v) { return (uint32_t)AJW_GPU(__builtin_amdgcn_readfirstlane((int)v)); }

// LDS: every offset is a byte offset from `b`
AJW V ld8(Lds b, V o) { return b[o]; }
AJW V ld16(Lds b, V o) { return *reinterpret_cast<__attribute__((address_space(3))) const uint16_t*>(b + o); }
AJW V ld32(Lds b, V o) { return *reinterpret_cast<__attribute__((address_space(3))) const uint32_t*>(b + o); }
AJW void st8(Lds b, M m, V o, V v) {
    if (m) b[o] = (uint8_t)v;
}
AJW void st16(Lds b, M m, V o, V v) {
    if (m) *reinterpret_cast<__attribute__((address_space(3))) uint16_t*>(b + o) = (uint16_t)v;
}
AJW void st32(Lds b, M m, V o, V v) {
    if (m) *reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(b + o) = v;
}
typedef uint32_t ajw_u32x4 __attribute__((ext_vector_type(4)));
AJW void st128(Lds b, M m, V o, V x, V y, V z, V ww) {
    if (m) *reinterpret_cast<__attribute__((address_space(3))) ajw_u32x4*>(b + o) = ajw_u32x4{x, y, z, ww};
}
AJW void min32(Lds b, M m, V o, V v) {
    if (m) __hip_atomic_fetch_min(reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(b + o), v,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// a generic pointer to LDS byte `o` (for per-lane scalar code)
AJW const uint8_t* gptr(Lds b, uint32_t o) { return (const uint8_t*)(b + o); }
// the wave's own LDS stores are visible to its later loads (LDS ops of one wave complete
// in order; this only stops the compiler from reordering across it)
AJW void lds_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#endif
}

// global memory: per-lane address p (a generic pointer value)
struct G16 {
    V x, y, z, w;
};
AJW G16 ld128(Lds b, V o) {
    const ajw_u32x4 v = *reinterpret_cast<__attribute__((address_space(3))) const ajw_u32x4*>(b + o);
    return G16{v.x, v.y, v.z, v.w};
}
// LDS-DMA: 16 bytes from each active lane's global address p to dst + 16 * lane (dst is
// wave-uniform; global_load_lds_dwordx4, counted in vmcnt)
AJW void dma16(const uint8_t* p, Lds dst, M m) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (m) __builtin_amdgcn_global_load_lds((const void*)p, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
#else
    (void)p; (void)dst; (void)m;
#endif
}
// wait for every vector memory operation of the wave (the DMA above included)
AJW void wait_vm() {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
#endif
}
AJW G16 gld128(const uint8_t* p, M m) {
    if (m) {
        const uint4 v = *reinterpret_cast<const uint4*>(p);
        return G16{v.x, v.y, v.z, v.w};
    }
    return G16{0u, 0u, 0u, 0u};
}
AJW V gld32(const uint32_t* p, V i) { return p[i]; }
#else
// ---------------------------------------------------------------- host emulation
struct M;
struct V {
    uint32_t x[64];
    V() = default;
    V(uint32_t u) {
        for (int l = 0; l < 64; l++) x[l] = u;
    }
};
struct M {
    uint64_t b;
    M() = default;
    M(bool u) : b(u ? ~0ull : 0ull) {}
    bool at(int l) const { return (b >> l) & 1; }
};
#define AJW_BIN(op)                                                           \
    AJW V operator op(const V& a, const V& c) {                              \
        V r;                                                                  \
        for (int l = 0; l < 64; l++) r.x[l] = (uint32_t)(a.x[l] op c.x[l]);  \
        return r;                                                             \
    }                                                                         \
    AJW V operator op(const V& a, uint32_t c) { return a op V(c); }          \
    AJW V operator op(uint32_t a, const V& c) { return V(a) op c; }          \
    AJW V& operator op##=(V& a, const V& c) { return a = a op c; }
AJW_BIN(+)
AJW_BIN(-)
AJW_BIN(*)
AJW_BIN(&)
AJW_BIN(|)
AJW_BIN(^)
#undef AJW_BIN
AJW V operator<<(const V& a, const V& c) {
    V r;
    for (int l = 0; l < 64; l++) r.x[l] = a.x[l] << (c.x[l] & 31u);  // (v_lshlrev: amount & 31)
    return r;
}
AJW V operator>>(const V& a, const V& c) {
    V r;
    for (int l = 0; l < 64; l++) r.x[l] = a.x[l] >> (c.x[l] & 31u);
    return r;
}
AJW V operator<<(const V& a, uint32_t c) { return a << V(c); }
AJW V operator>>(const V& a, uint32_t c) { return a >> V(c); }
AJW V& operator<<=(V& a, uint32_t c) { return a = a << c; }
AJW V& operator>>=(V& a, uint32_t c) { return a = a >> c; }
AJW V operator~(const V& a) {
    V r;
    for (int l = 0; l < 64; l++) r.x[l] = ~a.x[l];
    return r;
}
#define AJW_CMP(op)                                                           \
    AJW M operator op(const V& a, const V& c) {                              \
        M r{false};                                                           \
        for (int l = 0; l < 64; l++)                                          \
            if (a.x[l] op c.x[l]) r.b |= 1ull << l;                           \
        return r;                                                             \
    }                                                                         \
    AJW M operator op(const V& a, uint32_t c) { return a op V(c); }          \
    AJW M operator op(uint32_t a, const V& c) { return V(a) op c; }
AJW_CMP(==)
AJW_CMP(!=)
AJW_CMP(<)
AJW_CMP(<=)
AJW_CMP(>)
AJW_CMP(>=)
#undef AJW_CMP
AJW M operator&(const M& a, const M& c) { M r; r.b = a.b & c.b; return r; }
AJW M operator|(const M& a, const M& c) { M r; r.b = a.b | c.b; return r; }
AJW M operator^(const M& a, const M& c) { M r; r.b = a.b ^ c.b; return r; }
AJW M operator!(const M& a) { M r; r.b = ~a.b; return r; }
AJW M operator==(const M& a, const M& c) { M r; r.b = ~(a.b ^ c.b); return r; }
AJW M operator!=(const M& a, const M& c) { M r; r.b = a.b ^ c.b; return r; }
AJW M& operator&=(M& a, const M& c) { return a = a & c; }
AJW M& operator|=(M& a, const M& c) { return a = a | c; }
AJW M operator&(const M& a, bool c) { return a & M(c); }
AJW M operator|(const M& a, bool c) { return a | M(c); }

using Lds = uint8_t*;

AJW V lane() {
    V r;
    for (int l = 0; l < 64; l++) r.x[l] = (uint32_t)l;
    return r;
}
AJW V sel(const M& m, const V& a, const V& b) {
    V r;
    for (int l = 0; l < 64; l++) r.x[l] = m.at(l) ? a.x[l] : b.x[l];
    return r;
}
AJW uint64_t ballot(const M& m) { return m.b; }
AJW bool any(const M& m) { return m.b != 0; }
#define AJW_UN(name, expr)                                 \
    AJW V name(const V& a) {                               \
        V r;                                               \
        for (int l = 0; l < 64; l++) {                     \
            const uint32_t x = a.x[l];                     \
            r.x[l] = (expr);                               \
        }                                                  \
        return r;                                          \
    }
AJW_UN(popc, (uint32_t)__builtin_popcount(x))
AJW_UN(ctz, x ? (uint32_t)__builtin_ctz(x) : 32u)
AJW_UN(hibit, x ? 31u - (uint32_t)__builtin_clz(x) : 0xFFFFFFFFu)
#undef AJW_UN
AJW V alignbyte(const V& hi, const V& lo, const V& sh) {
    V r;
    for (int l = 0; l < 64; l++) {
        const uint64_t v = ((uint64_t)hi.x[l] << 32) | lo.x[l];
        r.x[l] = (uint32_t)(v >> (8 * (sh.x[l] & 3)));
    }
    return r;
}
template <int K>
AJW V row_shr(const V& v) {
    V r;
    for (int l = 0; l < 64; l++) r.x[l] = (l & 15) >= K ? v.x[l - K] : 0u;
    return r;
}
template <int K>
AJW V row_shl(const V& v) {
    V r;
    for (int l = 0; l < 64; l++) r.x[l] = (l & 15) + K <= 15 ? v.x[l + K] : 0u;
    return r;
}
AJW V shfl(const V& v, const V& src) {
    V r;
    for (int l = 0; l < 64; l++) r.x[l] = v.x[src.x[l] & 63];
    return r;
}
AJW uint32_t readlane(const V& v, uint32_t l) { return v.x[l & 63]; }
AJW uint32_t readfirst(const V& v) { return v.x[0]; }  // (callers pass wave-uniform values)

AJW V ld8(Lds b, const V& o) {
    V r;
    for (int l = 0; l < 64; l++) r.x[l] = b[o.x[l]];
    return r;
}
AJW V ld16(Lds b, const V& o) {
    V r;
    for (int l = 0; l < 64; l++) {
        uint16_t t;
        std::memcpy(&t, b + o.x[l], 2);
        r.x[l] = t;
    }
    return r;
}
AJW V ld32(Lds b, const V& o) {
    V r;
    for (int l = 0; l < 64; l++) std::memcpy(&r.x[l], b + o.x[l], 4);
    return r;
}
AJW void st8(Lds b, const M& m, const V& o, const V& v) {
    for (int l = 0; l < 64; l++)
        if (m.at(l)) b[o.x[l]] = (uint8_t)v.x[l];
}
AJW void st16(Lds b, const M& m, const V& o, const V& v) {
    for (int l = 0; l < 64; l++)
        if (m.at(l)) {
            const uint16_t t = (uint16_t)v.x[l];
            std::memcpy(b + o.x[l], &t, 2);
        }
}
AJW void st32(Lds b, const M& m, const V& o, const V& v) {
    for (int l = 0; l < 64; l++)
        if (m.at(l)) std::memcpy(b + o.x[l], &v.x[l], 4);
}
AJW void st128(Lds b, const M& m, const V& o, const V& x, const V& y, const V& z, const V& ww) {
    for (int l = 0; l < 64; l++)
        if (m.at(l)) {
            const uint32_t t[4] = {x.x[l], y.x[l], z.x[l], ww.x[l]};
            std::memcpy(b + o.x[l], t, 16);
        }
}
AJW void min32(Lds b, const M& m, const V& o, const V& v) {
    for (int l = 0; l < 64; l++)
        if (m.at(l)) {
            uint32_t t;
            std::memcpy(&t, b + o.x[l], 4);
            if (v.x[l] < t) std::memcpy(b + o.x[l], &v.x[l], 4);
        }
}
AJW void lds_fence() {}
AJW const uint8_t* gptr(Lds b, uint32_t o) { return b + o; }

struct G16 {
    V x, y, z, w;
};
AJW G16 ld128(Lds b, const V& o) {
    G16 r;
    for (int l = 0; l < 64; l++) {
        uint32_t t[4];
        std::memcpy(t, b + o.x[l], 16);
        r.x.x[l] = t[0];
        r.y.x[l] = t[1];
        r.z.x[l] = t[2];
        r.w.x[l] = t[3];
    }
    return r;
}
// per-lane global addresses: the host build passes them as 64 pointers
struct P {
    const uint8_t* p[64];
};
AJW G16 gld128(const P& a, const M& m) {
    G16 r;
    for (int l = 0; l < 64; l++) {
        uint32_t t[4] = {0, 0, 0, 0};
        if (m.at(l)) std::memcpy(t, a.p[l], 16);
        r.x.x[l] = t[0];
        r.y.x[l] = t[1];
        r.z.x[l] = t[2];
        r.w.x[l] = t[3];
    }
    return r;
}
AJW V gld32(const uint32_t* p, const V& i) {
    V r;
    for (int l = 0; l < 64; l++) r.x[l] = p[i.x[l]];
    return r;
}
#endif

// debugging aid of the host build: AJW_TRACE(mask, "what") prints the rows where it holds
#if AJW_DEV
#define AJW_TRACE(m, what) ((void)0)
#else
#include <cstdio>
#include <cstdlib>
inline bool ajw_trace_on() {
    static int on = std::getenv("AJW_TRACE") ? 1 : 0;
    return on != 0;
}
#define AJW_TRACE(m, what)                                                                 \
    do {                                                                                   \
        if (ajw_trace_on()) {                                                              \
            const ::ajx::w::M _m = (m);                                                    \
            for (int _l = 0; _l < 64; _l++)                                                \
                if (_m.at(_l)) std::fprintf(stderr, "[row %d lane %d] %s (line %d)\n", _l >> 4, _l & 15, what, \
                                            __LINE__);                                     \
        }                                                                                  \
    } while (0)
#endif
#if AJW_DEV
#define AJW_TRACEV(m, what, v) ((void)0)
#else
#define AJW_TRACEV(m, what, v)                                                             \
    do {                                                                                   \
        if (ajw_trace_on()) {                                                              \
            const ::ajx::w::M _m = (m);                                                    \
            const ::ajx::w::V _v = (v);                                                    \
            for (int _l = 0; _l < 64; _l++)                                                \
                if (_m.at(_l)) std::fprintf(stderr, "[row %d lane %d] %s = %u (0x%x)\n", _l >> 4, _l & 15, what, \
                                            _v.x[_l], _v.x[_l]);                           \
        }                                                                                  \
    } while (0)
#endif

// Per-lane scalar code inside the vector program (calls into the per-document device
// functions of ajx_device.h / ajx_fast.h): AJW_LANES(m) { ... } runs the block for every
// lane of m, AJW_L(v) is the lane's value of v, AJW_SET(v, x) sets it. On the device
// that is the lane itself (divergent code under an exec mask); on the host a loop.
#if AJW_DEV
#define AJW_LANES(m) if (m)
#define AJW_L(v) (v)
#define AJW_SET(out, val) ((out) = (val))
#else
#define AJW_LANES(m) for (int ajw_l = 0; ajw_l < 64; ajw_l++) if ((m).at(ajw_l))
#define AJW_L(v) ((v).x[ajw_l])
#define AJW_SET(out, val) ((out).x[ajw_l] = (val))
#endif

// ---------------------------------------------------------------- shared helpers
// inclusive sums / maxima inside each 16-lane row
AJW V row_sum(V v) {
    v = v + row_shr<1>(v);
    v = v + row_shr<2>(v);
    v = v + row_shr<4>(v);
    v = v + row_shr<8>(v);
    return v;
}
AJW V vmax(V a, V b) { return sel(a > b, a, b); }
AJW V vmin(V a, V b) { return sel(a < b, a, b); }
AJW V row_max(V v) {
    v = vmax(v, row_shr<1>(v));
    v = vmax(v, row_shr<2>(v));
    v = vmax(v, row_shr<4>(v));
    v = vmax(v, row_shr<8>(v));
    return v;
}
// the value lane 15 of each lane's row holds (four readlanes: no LDS round trip)
AJW V row_bcast15(V v) {
    const uint32_t a = readlane(v, 15), b = readlane(v, 31), c = readlane(v, 47), d = readlane(v, 63);
    const V row = lane() >> 4;
    return sel(row == 0u, V(a), sel(row == 1u, V(b), sel(row == 2u, V(c), V(d))));
}
// the 16 bits of ballot `b` that belong to each lane's row
AJW V row_bits(uint64_t b, V row) {
    const V lo = V((uint32_t)b), hi = V((uint32_t)(b >> 32));
    return (sel(row < 2u, lo, hi) >> ((row & 1u) << 4)) & 0xFFFFu;
}
// byte-flag helpers (SWAR on 4 bytes): 0x80 in every byte equal to c
AJW V eq_bytes(V x, uint32_t c4) {
    const V t = x ^ c4;
    return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
}
// the 0x80 flags of 16 bytes (f_i: bytes 4i..4i+3) -> 16-bit mask, bit 4i + j = byte j
AJW V gather16(V f0, V f1, V f2, V f3) {
    const V y = (f0 >> 7) | (f1 >> 6) | (f2 >> 5) | (f3 >> 4);
    const V t0 = (y | (y >> 4)) & 0x00FF00FFu;
    V z = (t0 | (t0 >> 8)) & 0xFFFFu;
    V t = (z ^ (z >> 3)) & 0x0A0Au;
    z = z ^ t ^ (t << 3);
    t = (z ^ (z >> 6)) & 0x00CCu;
    z = z ^ t ^ (t << 6);
    return z;
}

}  // namespace w
}  // namespace ajx
