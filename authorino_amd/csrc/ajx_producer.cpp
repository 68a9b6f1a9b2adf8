// ajx_producer.cpp — the Authorization JSON producer's output stage, native (SURVEY.md §8
// f3): documents packed straight into the batch arena, in the bytes Go's encoding/json
// writes for GetAuthorizationJSON (pkg/service/auth_pipeline.go:542-616;
// well_known_attributes.go:29-200 for the struct shapes), instead of a json.Marshal per
// evaluator call (the reference marshals at least twice per authorization evaluator).
//
// The caller (a Go shim that knows its struct types, or authorino_amd/producer.py) walks
// each request's values once into a TAPE (include/authjx.h AUTHJX_TAPE_*): structs as
// ordered objects (declaration order, omitempty already applied), Go maps as maps (the
// packer sorts their keys by bytes, as encoding/json does), strings as their bytes,
// float64 and integers as 8-byte values, pre-marshalled JSON as raw bytes. The packer
// writes, for every request in parallel on the host threads:
//   strings   encodeState.string with escapeHTML: '"' '\\' as \" \\, \n \r \t, other
//             bytes < 0x20 and '<' '>' '&' as \u00XX, U+2028 / U+2029 as \u2028 \u2029,
//             invalid UTF-8 as \ufffd (one per invalid byte)
//   float64   floatEncoder: strconv.AppendFloat(f, 'f' or, for |f| < 1e-6 or >= 1e21,
//             'e', -1, 64) with e-0X shortened to e-X; NaN / Inf: UnsupportedValueError
//   int       strconv.AppendInt
// The shortest float digits are ajx_float.h's f64_shortest (Go's ryuFtoaShortest result).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/authjx.h"

#define AJX_HD inline
#include "ajx_float.h"

namespace {

struct Tape {
    const uint8_t* p;
    size_t n, i;
    bool ok;
    uint8_t u8() {
        if (i >= n) { ok = false; return 0; }
        return p[i++];
    }
    uint32_t u32() {
        if (i + 4 > n) { ok = false; i = n; return 0; }
        uint32_t v;
        std::memcpy(&v, p + i, 4);
        i += 4;
        return v;
    }
    uint64_t u64() {
        if (i + 8 > n) { ok = false; i = n; return 0; }
        uint64_t v;
        std::memcpy(&v, p + i, 8);
        i += 8;
        return v;
    }
    const uint8_t* bytes(uint32_t len) {
        if (i + len > n) { ok = false; i = n; return nullptr; }
        const uint8_t* b = p + i;
        i += len;
        return b;
    }
};

const char kHex[] = "0123456789abcdef";

// utf8.DecodeRune's validity: the length of a valid sequence at s (n bytes left), 0 if
// invalid
uint32_t utf8_len(const uint8_t* s, size_t n) {
    const uint8_t c = s[0];
    uint32_t need;
    uint8_t lo = 0x80, hi = 0xBF;
    if (c < 0x80) return 1;
    if (c >= 0xC2 && c <= 0xDF) need = 2;
    else if (c >= 0xE0 && c <= 0xEF) {
        need = 3;
        if (c == 0xE0) lo = 0xA0;
        if (c == 0xED) hi = 0x9F;
    } else if (c >= 0xF0 && c <= 0xF4) {
        need = 4;
        if (c == 0xF0) lo = 0x90;
        if (c == 0xF4) hi = 0x8F;
    } else {
        return 0;
    }
    if (n < need || s[1] < lo || s[1] > hi) return 0;
    for (uint32_t k = 2; k < need; k++)
        if (s[k] < 0x80 || s[k] > 0xBF) return 0;
    return need;
}

void put_string(std::string& o, const uint8_t* s, size_t n) {
    o.push_back('"');
    size_t i = 0;
    while (i < n) {
        const uint8_t c = s[i];
        if (c < 0x80) {
            if (c >= 0x20 && c != '"' && c != '\\' && c != '<' && c != '>' && c != '&') {
                o.push_back((char)c);
            } else if (c == '"' || c == '\\') {
                o.push_back('\\');
                o.push_back((char)c);
            } else if (c == '\n') {
                o += "\\n";
            } else if (c == '\r') {
                o += "\\r";
            } else if (c == '\t') {
                o += "\\t";
            } else {
                o += "\\u00";
                o.push_back(kHex[c >> 4]);
                o.push_back(kHex[c & 15]);
            }
            i++;
            continue;
        }
        const uint32_t L = utf8_len(s + i, n - i);
        if (L == 0) {
            o += "\\ufffd";
            i++;
            continue;
        }
        if (L == 3 && c == 0xE2 && s[i + 1] == 0x80 && (s[i + 2] == 0xA8 || s[i + 2] == 0xA9)) {
            o += s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
            i += 3;
            continue;
        }
        o.append(reinterpret_cast<const char*>(s + i), L);
        i += L;
    }
    o.push_back('"');
}

// floatEncoder (encoding/json encode.go) for a finite float64
void put_float(std::string& o, double f) {
    if (f == 0) {
        o += std::signbit(f) ? "-0" : "0";
        return;
    }
    const bool neg = f < 0;
    const double a = neg ? -f : f;
    uint8_t dig[20];
    int nd = 0, dp = 0;
    ajx::Big T, t, u;
    ajx::f64_shortest(a, dig, &nd, &dp, T, t, u);
    if (neg) o.push_back('-');
    if (a < 1e-6 || a >= 1e21) {  // 'e': d[.ddd]e±XX, then e-0X -> e-X
        o.push_back((char)dig[0]);
        if (nd > 1) {
            o.push_back('.');
            o.append(reinterpret_cast<const char*>(dig + 1), (size_t)(nd - 1));
        }
        int x = dp - 1;
        o.push_back('e');
        o.push_back(x < 0 ? '-' : '+');
        if (x < 0) x = -x;
        if (x < 10) {
            if (dp - 1 >= 0) o.push_back('0');  // (the e-0X cleanup leaves negative ones short)
            o.push_back((char)('0' + x));
        } else if (x < 100) {
            o.push_back((char)('0' + x / 10));
            o.push_back((char)('0' + x % 10));
        } else {
            o.push_back((char)('0' + x / 100));
            o.push_back((char)('0' + x / 10 % 10));
            o.push_back((char)('0' + x % 10));
        }
        return;
    }
    // 'f' -1
    if (dp <= 0) {
        o += "0.";
        o.append((size_t)(-dp), '0');
        o.append(reinterpret_cast<const char*>(dig), (size_t)nd);
    } else if (dp >= nd) {
        o.append(reinterpret_cast<const char*>(dig), (size_t)nd);
        o.append((size_t)(dp - nd), '0');
    } else {
        o.append(reinterpret_cast<const char*>(dig), (size_t)dp);
        o.push_back('.');
        o.append(reinterpret_cast<const char*>(dig + dp), (size_t)(nd - dp));
    }
}

bool put_value(Tape& tp, std::string& o, int depth);

// a value's extent on the tape without writing it (map members are written sorted)
bool skip_value(Tape& tp, int depth) {
    std::string sink;
    return put_value(tp, sink, depth);
}

bool put_value(Tape& tp, std::string& o, int depth) {
    if (depth > 512) return false;
    const uint8_t tag = tp.u8();
    switch (tag) {
        case AUTHJX_TAPE_NULL: o += "null"; return tp.ok;
        case AUTHJX_TAPE_TRUE: o += "true"; return tp.ok;
        case AUTHJX_TAPE_FALSE: o += "false"; return tp.ok;
        case AUTHJX_TAPE_F64: {
            const uint64_t b = tp.u64();
            double f;
            std::memcpy(&f, &b, 8);
            if (!tp.ok || std::isnan(f) || std::isinf(f)) return false;  // UnsupportedValueError
            put_float(o, f);
            return true;
        }
        case AUTHJX_TAPE_I64: {
            const int64_t v = (int64_t)tp.u64();
            o += std::to_string(v);
            return tp.ok;
        }
        case AUTHJX_TAPE_STRING: {
            const uint32_t len = tp.u32();
            const uint8_t* s = tp.bytes(len);
            if (!tp.ok) return false;
            put_string(o, s, len);
            return true;
        }
        case AUTHJX_TAPE_RAW: {
            const uint32_t len = tp.u32();
            const uint8_t* s = tp.bytes(len);
            if (!tp.ok) return false;
            o.append(reinterpret_cast<const char*>(s), len);
            return true;
        }
        case AUTHJX_TAPE_ARRAY: {
            const uint32_t cnt = tp.u32();
            o.push_back('[');
            for (uint32_t k = 0; k < cnt && tp.ok; k++) {
                if (k) o.push_back(',');
                if (!put_value(tp, o, depth + 1)) return false;
            }
            o.push_back(']');
            return tp.ok;
        }
        case AUTHJX_TAPE_OBJECT: {  // a struct: members in tape order
            const uint32_t cnt = tp.u32();
            o.push_back('{');
            for (uint32_t k = 0; k < cnt && tp.ok; k++) {
                if (k) o.push_back(',');
                const uint32_t kl = tp.u32();
                const uint8_t* ks = tp.bytes(kl);
                if (!tp.ok) return false;
                put_string(o, ks, kl);
                o.push_back(':');
                if (!put_value(tp, o, depth + 1)) return false;
            }
            o.push_back('}');
            return tp.ok;
        }
        case AUTHJX_TAPE_MAP: {  // a Go map: members sorted by key bytes (mapEncoder)
            const uint32_t cnt = tp.u32();
            struct M {
                const uint8_t* k;
                uint32_t kl;
                size_t v0, v1;
            };
            std::vector<M> ms;
            // (a member takes >= 5 tape bytes: a malformed count must not size the vector)
            ms.reserve(std::min<size_t>(cnt, (tp.n - std::min(tp.i, tp.n)) / 5));
            for (uint32_t k = 0; k < cnt && tp.ok; k++) {
                M m;
                m.kl = tp.u32();
                m.k = tp.bytes(m.kl);
                m.v0 = tp.i;
                if (!tp.ok || !skip_value(tp, depth + 1)) return false;
                m.v1 = tp.i;
                ms.push_back(m);
            }
            std::sort(ms.begin(), ms.end(), [](const M& a, const M& b) {
                const int c = std::memcmp(a.k, b.k, std::min(a.kl, b.kl));
                return c < 0 || (c == 0 && a.kl < b.kl);
            });
            o.push_back('{');
            for (size_t k = 0; k < ms.size(); k++) {
                if (k) o.push_back(',');
                put_string(o, ms[k].k, ms[k].kl);
                o.push_back(':');
                Tape sub{tp.p, ms[k].v1, ms[k].v0, true};
                if (!put_value(sub, o, depth + 1)) return false;
            }
            o.push_back('}');
            return tp.ok;
        }
        default: return false;
    }
}

}  // namespace

extern "C" {

int authjx_pack_json(const uint8_t* tapes, const uint64_t* tape_offs, const uint32_t* tape_lens, uint32_t n,
                     uint8_t* arena, uint64_t arena_cap, uint64_t* out_offs, uint32_t* out_lens,
                     uint64_t* out_total, uint32_t n_threads) {
    if ((n && (!tapes || !tape_offs || !tape_lens || !out_offs || !out_lens)) || !out_total) return AUTHJX_EINVAL;
    uint32_t nt = n_threads ? n_threads : std::max(1u, std::thread::hardware_concurrency());
    nt = std::max(1u, std::min<uint32_t>(nt, (n + 255u) / 256u));
    // each thread encodes a contiguous slice into its own buffer; the slices are then laid
    // out one after another in the arena (request order)
    std::vector<std::string> outs(nt);
    std::vector<int> rcs(nt, AUTHJX_OK);
    const uint32_t step = (n + nt - 1) / std::max(1u, nt);
    auto work = [&](uint32_t t) {
        const uint32_t lo = t * step, hi = std::min(n, lo + step);
        std::string& o = outs[t];
        for (uint32_t r = lo; r < hi; r++) {
            const size_t at = o.size();
            Tape tp{tapes + tape_offs[r], tape_lens[r], 0, true};
            if (!put_value(tp, o, 0) || tp.i != tp.n) {
                rcs[t] = AUTHJX_EINVAL;
                out_offs[r] = ~0ull;  // (marks the failing request)
                out_lens[r] = 0;
                o.resize(at);
                continue;
            }
            out_offs[r] = at;  // (relative to the slice; rebased below)
            out_lens[r] = (uint32_t)(o.size() - at);
        }
    };
    try {
        if (nt == 1) {
            work(0);
        } else {
            std::vector<std::thread> th;
            for (uint32_t t = 0; t < nt; t++) th.emplace_back(work, t);
            for (auto& x : th) x.join();
        }
    } catch (...) {
        return AUTHJX_ENOMEM;
    }
    uint64_t total = 0;
    for (const std::string& o : outs) total += o.size();
    *out_total = total;
    if (total > arena_cap || (total && !arena)) return AUTHJX_ELIMIT;  // (the size needed is in *out_total)
    uint64_t base = 0;
    for (uint32_t t = 0; t < nt; t++) {
        if (!outs[t].empty()) std::memcpy(arena + base, outs[t].data(), outs[t].size());
        const uint32_t lo = t * step, hi = std::min(n, lo + step);
        for (uint32_t r = lo; r < hi; r++)
            if (out_offs[r] != ~0ull) out_offs[r] += base;
        base += outs[t].size();
    }
    for (int rc : rcs)
        if (rc != AUTHJX_OK) return rc;
    return AUTHJX_OK;
}

}  // extern "C"
