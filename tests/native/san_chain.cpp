// san_chain.cpp — TEST-ONLY: ASan + UBSan driver for the host parts of the device chain
// (SURVEY.md §8 f3/f4): the Authorization-JSON packer (ajx_producer.cpp,
// authjx_pack_json) on random well-formed and malformed value tapes, arenas that are too
// small and several thread counts, and the AuthConfig index (ajx_index.cpp) under random
// Set / DeleteKey / Get / batched lookups. Any sanitizer report aborts the binary; it
// prints "ok <cases>" at the end. Usage: san_chain <iterations> <seed>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/authjx.h"

namespace {
std::mt19937_64 rng;
uint32_t rnd(uint32_t n) { return n ? (uint32_t)(rng() % n) : 0u; }

void put32(std::vector<uint8_t>& t, uint32_t v) {
    for (int k = 0; k < 4; k++) t.push_back((uint8_t)(v >> (8 * k)));
}
void put64(std::vector<uint8_t>& t, uint64_t v) {
    for (int k = 0; k < 8; k++) t.push_back((uint8_t)(v >> (8 * k)));
}
std::string rand_bytes(uint32_t max) {
    static const char pool[] = "ab<>&\"\\/\x01\x1f\x7f\xe2\x80\xa8\xc3\xa9\xff\xfe {}[]:,0";
    std::string s;
    const uint32_t n = rnd(max + 1);
    for (uint32_t i = 0; i < n; i++) s.push_back(pool[rnd(sizeof pool - 1)]);
    return s;
}

void value(std::vector<uint8_t>& t, int depth) {
    const uint32_t k = depth <= 0 ? rnd(7) : rnd(10);
    switch (k) {
        case 0: t.push_back(AUTHJX_TAPE_NULL); break;
        case 1: t.push_back(rnd(2) ? AUTHJX_TAPE_TRUE : AUTHJX_TAPE_FALSE); break;
        case 2: {
            t.push_back(AUTHJX_TAPE_F64);
            const double vals[] = {0.0, -0.0, 1.5, 1e21, 1e-7, 123456789.0, 5e-324, 1.7976931348623157e308,
                                   NAN, INFINITY};
            double d = vals[rnd(rnd(8) ? 8 : 10)];
            uint64_t b;
            std::memcpy(&b, &d, 8);
            put64(t, b);
            break;
        }
        case 3: t.push_back(AUTHJX_TAPE_I64); put64(t, rng()); break;
        case 4:
        case 5: {
            t.push_back(k == 4 ? AUTHJX_TAPE_STRING : AUTHJX_TAPE_RAW);
            const std::string s = k == 4 ? rand_bytes(40) : std::string(rnd(2) ? "{\"a\":1}" : "[1,2]");
            put32(t, (uint32_t)s.size());
            t.insert(t.end(), s.begin(), s.end());
            break;
        }
        case 6: t.push_back(AUTHJX_TAPE_STRING); put32(t, 0); break;
        case 7: {
            t.push_back(AUTHJX_TAPE_ARRAY);
            const uint32_t n = rnd(4);
            put32(t, n);
            for (uint32_t i = 0; i < n; i++) value(t, depth - 1);
            break;
        }
        default: {
            t.push_back(rnd(2) ? AUTHJX_TAPE_OBJECT : AUTHJX_TAPE_MAP);
            const uint32_t n = rnd(5);
            put32(t, n);
            for (uint32_t i = 0; i < n; i++) {
                const std::string key = rand_bytes(6);
                put32(t, (uint32_t)key.size());
                t.insert(t.end(), key.begin(), key.end());
                value(t, depth - 1);
            }
        }
    }
}

void corrupt(std::vector<uint8_t>& t) {
    if (t.empty()) return;
    switch (rnd(4)) {
        case 0: t.resize(rnd((uint32_t)t.size())); break;                 // truncated
        case 1: t[rnd((uint32_t)t.size())] = (uint8_t)rng(); break;       // a byte flipped
        case 2: t.push_back((uint8_t)rng()); break;                       // trailing bytes
        default: {                                                       // a huge length
            const size_t at = rnd((uint32_t)t.size());
            for (size_t k = at; k < t.size() && k < at + 4; k++) t[k] = 0xFF;
        }
    }
}

size_t producer_round() {
    const uint32_t n = 1 + rnd(64);
    std::vector<uint8_t> tapes;
    std::vector<uint64_t> offs(n);
    std::vector<uint32_t> lens(n);
    for (uint32_t r = 0; r < n; r++) {
        std::vector<uint8_t> t;
        value(t, 1 + (int)rnd(4));
        if (rnd(5) == 0) corrupt(t);
        offs[r] = tapes.size();
        lens[r] = (uint32_t)t.size();
        tapes.insert(tapes.end(), t.begin(), t.end());
    }
    const uint64_t cap = rnd(3) ? (uint64_t)1 << 20 : rnd(256);
    std::vector<uint8_t> arena(cap + 1);
    std::vector<uint64_t> oo(n);
    std::vector<uint32_t> ol(n);
    uint64_t total = 0;
    const int rc = authjx_pack_json(tapes.empty() ? nullptr : tapes.data(), offs.data(), lens.data(), n,
                                    arena.data(), cap, oo.data(), ol.data(), &total, 1 + rnd(4));
    if (rc == AUTHJX_OK || rc == AUTHJX_EINVAL) {
        for (uint32_t r = 0; r < n; r++)
            if (oo[r] != ~0ull && (oo[r] + ol[r] > cap)) {
                std::printf("producer: request %u outside the arena\n", r);
                std::abort();
            }
    }
    return n;
}

std::string rand_host() {
    static const char* labels[] = {"a", "b", "api", "x-y", "*", "127", "", "io", "svc"};
    std::string h;
    const uint32_t parts = 1 + rnd(4);
    for (uint32_t i = 0; i < parts; i++) {
        if (i) h += '.';
        h += labels[rnd(9)];
    }
    if (rnd(4) == 0) h += ":" + std::to_string(rnd(70000));
    return h;
}

size_t index_round(authjx_index* ix) {
    size_t ops = 0;
    for (int k = 0; k < 40; k++, ops++) {
        const std::string h = rand_host();
        int32_t id = -1;
        switch (rnd(4)) {
            case 0: (void)authjx_index_set(ix, h.data(), (uint32_t)h.size(), (int32_t)rnd(50), (int)rnd(2)); break;
            case 1: (void)authjx_index_delete_key(ix, h.data(), (uint32_t)h.size(), (int32_t)rnd(50)); break;
            default: (void)authjx_index_get(ix, h.data(), (uint32_t)h.size(), &id);
        }
    }
    const uint32_t n = rnd(200);
    std::string all;
    std::vector<uint64_t> offs(n);
    std::vector<uint32_t> lens(n);
    for (uint32_t r = 0; r < n; r++) {
        const std::string h = rand_host();
        offs[r] = all.size();
        lens[r] = (uint32_t)h.size();
        all += h;
    }
    std::vector<int32_t> out(n + 1);
    (void)authjx_index_lookup_batch(ix, (const uint8_t*)all.data(), offs.data(), lens.data(), n, out.data(),
                                    1 + rnd(4));
    for (uint32_t r = 0; r < n; r++) {
        int32_t one = -2;
        (void)authjx_index_get(ix, all.data() + offs[r], lens[r], &one);
        if (one != out[r]) {
            std::printf("index: batched lookup %d != get %d\n", out[r], one);
            std::abort();
        }
    }
    return ops + n;
}
}  // namespace

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
    rng.seed(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1);
    size_t cases = 0;
    authjx_index* ix = nullptr;
    if (authjx_index_new(&ix) != AUTHJX_OK) return 2;
    for (int i = 0; i < iters; i++) {
        cases += producer_round();
        cases += index_round(ix);
    }
    authjx_index_free(ix);
    std::printf("ok %zu\n", cases);
    return 0;
}
