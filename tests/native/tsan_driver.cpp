// tsan_driver.cpp — TEST-ONLY: ThreadSanitizer driver for the host concurrency of the
// serving path: the micro-batcher's queue / window / worker threads (ajx_batcher.h, two
// workers as authjx_batcher runs them) under many producer threads with deadlines, and
// the AuthConfig index's reader / writer lock (ajx_index.cpp) under concurrent lookups
// and Set / DeleteKey. Prints "ok <requests>"; TSan reports go to stderr (the test fails
// on any). Usage: tsan_driver <producers> <requests per producer>
// (gcc 11's TSan does not intercept pthread_cond_clockwait, which libstdc++ uses for
// condition_variable::wait_for: without it the mutex re-acquired inside the wait is
// invisible and every access after a timed wait is reported. The timedwait path is
// intercepted.)
#include <bits/c++config.h>
#undef _GLIBCXX_USE_PTHREAD_COND_CLOCKWAIT
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../authorino_amd/csrc/ajx_batcher.h"
#include "../../include/authjx.h"

using namespace ajx;

int main(int argc, char** argv) {
    const uint32_t producers = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 16;
    const uint32_t per = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 500;
    std::atomic<uint64_t> wrong{0}, done{0}, expired{0};
    {
        BatchCore core(64, 100 * 1000ull, 256,
                       [](std::vector<BatchReq*>& reqs, uint32_t wid) {
                           std::this_thread::sleep_for(std::chrono::microseconds(20 + 10 * wid));
                           for (BatchReq* r : reqs)
                               for (uint32_t k = 0; k < r->n_out; k++)
                                   r->out_tri[k] = (uint8_t)(r->doc[0] ^ (uint8_t)(uintptr_t)r->rs ^ (uint8_t)k);
                           return 0;
                       },
                       2);
        std::vector<std::thread> ts;
        for (uint32_t p = 0; p < producers; p++)
            ts.emplace_back([&, p] {
                for (uint32_t i = 0; i < per; i++) {
                    uint8_t byte = (uint8_t)(p * 31 + i);
                    uint8_t out[4] = {0, 0, 0, 0};
                    BatchReq r;
                    r.rs = (const void*)(uintptr_t)(1 + (i % 5));
                    r.n_out = 1 + (p % 4);
                    r.doc = &byte;
                    r.len = 1;
                    r.deadline_ns = (i % 7 == 0) ? mono_ns() + 50 * 1000ull : 0;
                    r.out_tri = out;
                    const int rc = core.submit(r);
                    if (rc == 0) {
                        for (uint32_t k = 0; k < r.n_out; k++)
                            if (out[k] != (uint8_t)(byte ^ (uint8_t)(uintptr_t)r.rs ^ (uint8_t)k)) wrong++;
                        done++;
                    } else {
                        expired++;
                    }
                }
            });
        for (auto& t : ts) t.join();
    }
    // the index: readers (single and batched lookups) against a writer
    authjx_index* ix = nullptr;
    if (authjx_index_new(&ix) != AUTHJX_OK) return 2;
    std::atomic<bool> stop{false};
    std::thread writer([&] {
        for (uint32_t i = 0; i < 4000; i++) {
            const std::string h = "h" + std::to_string(i % 97) + ".example.com";
            if (i % 3 == 2) (void)authjx_index_delete_key(ix, h.data(), (uint32_t)h.size(), (int32_t)(i % 11));
            else (void)authjx_index_set(ix, h.data(), (uint32_t)h.size(), (int32_t)(i % 11), 1);
        }
        stop = true;
    });
    std::vector<std::thread> readers;
    for (int t = 0; t < 4; t++)
        readers.emplace_back([&, t] {
            std::string all;
            std::vector<uint64_t> offs;
            std::vector<uint32_t> lens;
            for (int i = 0; i < 64; i++) {
                const std::string h = "h" + std::to_string((i * 7 + t) % 97) + ".example.com" + (i % 5 ? "" : ":8080");
                offs.push_back(all.size());
                lens.push_back((uint32_t)h.size());
                all += h;
            }
            std::vector<int32_t> out(64);
            while (!stop) {
                (void)authjx_index_lookup_batch(ix, (const uint8_t*)all.data(), offs.data(), lens.data(), 64,
                                                out.data(), 2);
                int32_t one;
                (void)authjx_index_get(ix, all.data(), lens[0], &one);
            }
        });
    writer.join();
    for (auto& t : readers) t.join();
    authjx_index_free(ix);
    std::printf("ok %llu expired %llu wrong %llu\n", (unsigned long long)done.load(),
                (unsigned long long)expired.load(), (unsigned long long)wrong.load());
    return wrong.load() ? 1 : 0;
}
