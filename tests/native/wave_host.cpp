// wave_host.cpp — TEST-ONLY harness for the wave kernel's per-request logic
// (authorino_amd/csrc/ajx_wave.h) on the host CPU. Phase 1 (the lexer) is written for a
// 64-lane wavefront with explicit cross-lane operations; here each lane is a thread and
// every cross-lane operation a barrier round, which gives the hardware's results for
// code whose cross-lane operations are reached by all lanes (as the kernel's are).
// Phases 2 and 3 are per-request code and run on the calling thread. Not part of
// libauthjx.so; the product path has no CPU fallback.
#define AJX_HD inline
#include <barrier>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "../../authorino_amd/csrc/ajx_compiler.h"
#include "../../authorino_amd/csrc/ajx_wave.h"

using namespace ajx;

namespace {

struct WaveShared {
    std::barrier<> bar{64};
    uint64_t slot[64];
};

struct WaveEmu {
    WaveShared* sh;
    uint32_t l;
    uint32_t lane() const { return l; }
    void sync() { sh->bar.arrive_and_wait(); }
    uint64_t exchange(uint64_t v, uint32_t src) {
        sh->slot[l] = v;
        sync();
        const uint64_t r = sh->slot[src & 63];
        sync();
        return r;
    }
    uint64_t ballot(bool b) {
        sh->slot[l] = b ? 1 : 0;
        sync();
        uint64_t m = 0;
        for (int i = 0; i < 64; i++) m |= (sh->slot[i] & 1ull) << i;
        sync();
        return m;
    }
    bool any(bool b) { return ballot(b) != 0; }
    uint32_t shfl_up(uint32_t v) { return (uint32_t)exchange(v, l ? l - 1 : 0); }
    uint32_t shfl_down(uint32_t v) { return (uint32_t)exchange(v, l < 63 ? l + 1 : 63); }
    uint32_t readlane(uint32_t v, uint32_t src) { return (uint32_t)exchange(v, src); }
    uint32_t bpermute(uint32_t v, uint32_t src) { return (uint32_t)exchange(v, src); }
    uint32_t excl_sum(uint32_t v, uint32_t* total) {
        sh->slot[l] = v;
        sync();
        uint32_t pre = 0, tot = 0;
        for (uint32_t i = 0; i < 64; i++) {
            if (i < l) pre += (uint32_t)sh->slot[i];
            tot += (uint32_t)sh->slot[i];
        }
        sync();
        *total = tot;
        return pre;
    }
    uint64_t lanemask_lt() const { return l ? (~0ull >> (64 - l)) : 0ull; }
    uint32_t mbcnt(uint64_t m) const { return (uint32_t)__builtin_popcountll(m & lanemask_lt()); }
    void lds_fence() { sync(); }
};

// a wave of 64 persistent threads
struct WavePool {
    WaveShared sh;
    std::barrier<> start{65}, done{65};
    std::function<void(WaveEmu&)> job;
    std::vector<std::thread> th;
    bool stop = false;
    WavePool() {
        for (uint32_t l = 0; l < 64; l++)
            th.emplace_back([this, l] {
                WaveEmu w{&sh, l};
                for (;;) {
                    start.arrive_and_wait();
                    if (stop) return;
                    job(w);
                    done.arrive_and_wait();
                }
            });
    }
    void run(std::function<void(WaveEmu&)> f) {
        job = std::move(f);
        start.arrive_and_wait();
        done.arrive_and_wait();
    }
    ~WavePool() {
        stop = true;
        start.arrive_and_wait();
        for (auto& t : th) t.join();
    }
};

WavePool& pool() {
    static WavePool p;
    return p;
}

struct HtRuleset {
    CompiledRuleset c;
};

}  // namespace

extern "C" {

void* hw_compile(const authjx_tree* tree, int* rc) {
    HtRuleset* r = new HtRuleset();
    std::string e;
    *rc = compile_tree(tree, &r->c, &e);
    if (*rc != AUTHJX_OK) { delete r; return nullptr; }
    return r;
}
void hw_free(void* h) { delete (HtRuleset*)h; }
int hw_wave_ok(void* h) {
    const RulesetHdr* hd = (const RulesetHdr*)((HtRuleset*)h)->c.blob.data();
    return (hd->flags & kFlagWaveOk) ? 1 : 0;
}

// One request through the wave kernel's logic: the document is placed `mis` bytes into a
// 16-B aligned buffer surrounded by `fill` bytes (the kernel reads whole 16-B blocks).
// Returns the tri-state, -1 when the request goes to the exact scan (lexer or walker
// could not prove it compact valid JSON), -2 when the ruleset is not wave-eligible.
// res[p]: each pattern's value; row (1 + n_selectors u64): the capture row; ntok: tokens.
int hw_eval(void* h, const uint8_t* doc, uint32_t len, uint32_t mis, uint8_t fill, uint8_t* res, int32_t* err,
            uint64_t* row_out, uint32_t* ntok_out, uint32_t* tok_out, uint32_t tok_out_cap) {
    const uint8_t* blob = ((HtRuleset*)h)->c.blob.data();
    const RulesetHdr* hd = (const RulesetHdr*)blob;
    if (!(hd->flags & kFlagWaveOk)) return -2;
    mis &= 15;
    std::vector<uint8_t> buf(len + 4096 + 64, fill);
    uint8_t* base = (uint8_t*)(((uintptr_t)buf.data() + 15) & ~(uintptr_t)15);
    uint8_t* d = base + mis;
    std::memcpy(d, doc, len);
    alignas(16) static uint8_t ring[2 * kWaveChunk];
    const uint32_t cap = 8192;
    static std::vector<uint32_t> tok(cap);
    static std::vector<uint8_t> lab(cap);
    uint32_t status = 0, ntok = 0;
    pool().run([&](WaveEmu& w) {
        uint32_t nt;
        const uint32_t st = lex_doc(w, blob, d, len, ring, tok.data(), lab.data(), 0, cap, &nt);
        if (w.lane() == 0) { status = st; ntok = nt; }
    });
    *ntok_out = ntok;
    for (uint32_t i = 0; i < ntok && i < tok_out_cap; i++) tok_out[i] = tok[i];
    if (status != LEX_OK) return -1;
    std::vector<uint64_t> row(1 + hd->n_selectors, 0);
    if (!walk_doc(blob, blob_tables(blob), tok.data(), lab.data(), 0, ntok, d, row.data())) return -1;
    for (uint32_t s = 0; s <= hd->n_selectors; s++) row_out[s] = row[s];
    uint64_t t[2], u[2];
    patterns_from_row(blob, d, row.data(), t, u);
    const uint32_t* code = (const uint32_t*)(blob + hd->off_code);
    for (uint32_t p = 0; p < hd->n_patterns; p++) {
        const uint64_t bit = 1ull << (p & 63);
        const uint32_t k = p >> 6;
        res[p] = (hd->static_error[k] & bit) ? V_E : (u[k] & bit) ? V_U : (t[k] & bit) ? V_T : V_F;
    }
    return run_fold(code, hd->n_code, [&](uint32_t p) { return res[p]; }, err);
}
}
