// lane_host.cpp — TEST-ONLY harness for the lane kernel's per-request scanner
// (authorino_amd/csrc/ajx_lane.h) on the host CPU, with the kernel's window staging
// emulated for one lane. Not part of libauthjx.so; the product path has no CPU fallback.
#define AJX_HD inline
#include <cstring>
#include <string>
#include <vector>

#include "../../authorino_amd/csrc/ajx_compiler.h"
#include "../../authorino_amd/csrc/ajx_lane.h"

using namespace ajx;

namespace {

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
// the blob header's first 32 words (sizes and section offsets, for layout checks)
void hw_header(void* h, uint32_t* out) { std::memcpy(out, ((HtRuleset*)h)->c.blob.data(), 32 * sizeof(uint32_t)); }
int hw_lane_ok(void* h) {
    const RulesetHdr* hd = (const RulesetHdr*)((HtRuleset*)h)->c.blob.data();
    return (hd->flags & kFlagFastOk) ? 1 : 0;
}

// One request through the lane kernel's scanner (ajx_lane.h) as lane 0 of a wavefront:
// the windows are staged into a 3-slot buffer the way ajx_lane_eval stages them (blocks
// past the document's last 16-B block read as zero; window w + 1 staged before window w
// is scanned). Returns the tri-state, -1 when the request goes to the exact scan, -2
// when the ruleset has no single-pass tables; res[p]: each pattern's value; row: the
// capture row; nwin: windows scanned.
int hw_eval_lane(void* h, const uint8_t* doc, uint32_t len, uint32_t mis, uint8_t fill, uint8_t* res, int32_t* err,
                 uint64_t* row_out, uint32_t* nwin_out) {
    const uint8_t* blob = ((HtRuleset*)h)->c.blob.data();
    const RulesetHdr* hd = (const RulesetHdr*)blob;
    if (!(hd->flags & kFlagFastOk)) return -2;
    mis &= 15;
    std::vector<uint8_t> buf(len + 4096 + 64, fill);
    uint8_t* base = (uint8_t*)(((uintptr_t)buf.data() + 15) & ~(uintptr_t)15);
    uint8_t* d = base + mis;
    std::memcpy(d, doc, len);
    *nwin_out = 0;
    if (len == 0) return -1;
    std::vector<uint64_t> row(1 + hd->n_selectors, 0);
    alignas(16) static uint8_t stage[3 * kLaneSlot];
    const uint32_t nblk = (mis + len + 15) / 16, nwin = (mis + len + kLaneWin - 1) / kLaneWin;
    auto put = [&](uint32_t w) {
        uint8_t* s = stage + (w % 3) * kLaneSlot;
        for (uint32_t j = 0; j < 4; j++) {
            const uint32_t b = w * 4 + j;
            if (b < nblk) std::memcpy(s + 16 * j, base + 16 * b, 16);
            else std::memset(s + 16 * j, 0, 16);
        }
    };
    LaneScan sc;
    sc.init(blob, blob_tables(blob), d, len, row.data());
    sc.stage = stage;
    sc.lane_off = 0;
    put(0);
    if (nwin > 1) put(1);
    for (uint32_t w = 0; w < nwin && !sc.bad; w++) {
        uint32_t x[16];
        std::memcpy(x, stage + (w % 3) * kLaneSlot, 64);
        sc.window(x, w);
        *nwin_out = w + 1;
        if (w + 2 < nwin) put(w + 2);
    }
    if (sc.bad || !sc.finish()) return -1;
    for (uint32_t s = 0; s <= hd->n_selectors; s++) row_out[s] = row[s];
    uint64_t t[2], u[2];
    patterns_from_row(blob, d, row.data(), t, u);
    if ((u[0] & ~hd->unsupported[0]) | (u[1] & ~hd->unsupported[1])) return -1;  // a number for the exact scan
    const uint32_t* code = (const uint32_t*)(blob + hd->off_code);
    for (uint32_t p = 0; p < hd->n_patterns; p++) {
        const uint64_t bit = 1ull << (p & 63);
        const uint32_t k = p >> 6;
        res[p] = (hd->static_error[k] & bit) ? V_E : (u[k] & bit) ? V_U : (t[k] & bit) ? V_T : V_F;
    }
    return run_fold(code, hd->n_code, [&](uint32_t p) { return res[p]; }, err);
}
}
