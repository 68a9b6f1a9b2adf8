// batcher_host.cpp — TEST-ONLY: the micro-batcher's queue / flush / deadline / ordering
// logic (authorino_amd/csrc/ajx_batcher.h) driven on the CPU with a stand-in evaluator
// that sleeps like a device launch and writes a result derived from each request, so
// the tests can check that every caller gets its own answer.
#include <atomic>
#include <chrono>
#include <cstring>
#include <thread>

#include "../../authorino_amd/csrc/ajx_batcher.h"

using namespace ajx;

namespace {
struct Host {
    BatchCore* core = nullptr;
    uint32_t delay_us = 0;
    std::atomic<uint64_t> order_violations{0}, shape_violations{0};
};
}  // namespace

uint32_t g_wake = 0;  // the BatchCore wake mode of batchers created afterwards

extern "C" {

void hb_set_wake(uint32_t mode) { g_wake = mode; }

void* hb_create(uint32_t max_batch, uint32_t window_us, uint32_t queue_cap, uint32_t delay_us) {
    Host* h = new Host();
    h->delay_us = delay_us;
    h->core = new BatchCore(max_batch, (uint64_t)window_us * 1000ull, queue_cap, [h](std::vector<BatchReq*>& reqs, uint32_t) {
        for (size_t i = 1; i < reqs.size(); i++) {
            if (reqs[i - 1]->rs > reqs[i]->rs) h->order_violations++;
            if (reqs[i]->n_out != reqs[0]->n_out) h->shape_violations++;
        }
        if (h->delay_us) std::this_thread::sleep_for(std::chrono::microseconds(h->delay_us));
        for (BatchReq* r : reqs)
            for (uint32_t k = 0; k < r->n_out; k++)
                r->out_tri[k] = (uint8_t)(r->doc[0] ^ (uint8_t)(uintptr_t)r->rs ^ (uint8_t)k);
        return 0;
    }, 1, g_wake);
    return h;
}

// one request: ruleset id `rs` (nonzero), result shape n_out, one document byte
int hb_eval(void* hv, uint64_t rs, uint32_t n_out, uint8_t byte, uint64_t timeout_us, uint8_t* out) {
    Host* h = (Host*)hv;
    BatchReq r;
    r.rs = (const void*)(uintptr_t)rs;
    r.n_out = n_out;
    r.doc = &byte;
    r.len = 1;
    r.deadline_ns = timeout_us ? mono_ns() + timeout_us * 1000ull : 0;
    r.out_tri = out;
    return h->core->submit(r);
}

void hb_stats(void* hv, uint64_t* out) {
    Host* h = (Host*)hv;
    const BatchStats st = h->core->stats();
    out[0] = st.batches;
    out[1] = st.requests;
    out[2] = st.expired;
    out[3] = st.max_batch_seen;
    out[4] = h->order_violations.load();
    out[5] = h->shape_violations.load();
}

void hb_destroy(void* hv) {
    Host* h = (Host*)hv;
    delete h->core;
    delete h;
}
}
