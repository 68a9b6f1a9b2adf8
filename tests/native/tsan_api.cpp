// tsan_api.cpp — TEST-ONLY: ThreadSanitizer driver for the C-ABI's workspace lifetime
// (authorino_amd/csrc/ajx_api.cpp) on the host stand-in of the HIP runtime
// (hipstub/, hip_stub.cpp): threads evaluating on short-lived streams of their own and
// releasing them (authjx_release_stream) while others read authjx_last_exact_count /
// authjx_last_kernel_ms, evaluate from host buffers on the context's stream, run a
// micro-batcher, and compile / evaluate / free rulesets of their own. Prints "ok ...";
// TSan reports go to stderr (the test fails on any). Usage: tsan_api <rounds>
#include <bits/c++config.h>
#undef _GLIBCXX_USE_PTHREAD_COND_CLOCKWAIT  // (see tsan_driver.cpp)
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/authjx.h"

namespace {

authjx_ruleset* compile(authjx_ctx* ctx, const char* sel, const char* val) {
    authjx_pattern p{sel, (uint32_t)std::strlen(sel), AUTHJX_OP_EQ, val, (uint32_t)std::strlen(val)};
    authjx_node nd{AUTHJX_NODE_PATTERN, -1, -1, 0};
    authjx_tree t{&p, 1, &nd, 1, 0};
    authjx_ruleset* rs = nullptr;
    return authjx_compile(ctx, &t, &rs, nullptr, nullptr, 0) == AUTHJX_OK ? rs : nullptr;
}

struct DevBatch {  // a batch in "device" memory (host memory under the stub)
    std::string arena;
    std::vector<uint64_t> offs;
    std::vector<uint32_t> lens;
    std::vector<uint8_t> tri;
    explicit DevBatch(uint32_t n) {
        for (uint32_t i = 0; i < n; i++) {
            const std::string d = "{\"a\":" + std::to_string(i) + "}";
            offs.push_back(arena.size());
            lens.push_back((uint32_t)d.size());
            arena += d;
        }
        arena.append(16, '\0');
        tri.resize(n);
    }
};

}  // namespace

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 200;
    authjx_ctx* ctx = nullptr;
    if (authjx_init(0, &ctx) != AUTHJX_OK) return 2;
    authjx_ruleset* shared = compile(ctx, "a", "1");
    if (!shared) return 2;
    std::atomic<bool> stop{false};
    std::atomic<uint64_t> evals{0}, reads{0}, errors{0};
    std::vector<std::thread> ts;
    // streams that come and go: evaluate on a fresh stream, then release it
    for (int t = 0; t < 3; t++)
        ts.emplace_back([&, t] {
            DevBatch b(64 + 32 * t);
            for (int i = 0; i < rounds; i++) {
                hipStream_t s;
                (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
                for (int k = 0; k < 3; k++) {
                    if (authjx_eval_batch_device(ctx, &shared, 1, nullptr, (const uint8_t*)b.arena.data(),
                                                 b.offs.data(), b.lens.data(), (uint32_t)b.lens.size(), b.tri.data(),
                                                 nullptr, nullptr, 0, s) != AUTHJX_OK)
                        errors++;
                    evals++;
                }
                if (authjx_release_stream(ctx, s) != AUTHJX_OK) errors++;
                (void)hipStreamDestroy(s);
            }
        });
    // one stream released while another thread is still calling on it
    ts.emplace_back([&] {
        DevBatch b(48);
        for (int i = 0; i < rounds; i++) {
            hipStream_t s;
            (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
            std::thread caller([&] {
                for (int k = 0; k < 4; k++)
                    (void)authjx_eval_batch_device(ctx, &shared, 1, nullptr, (const uint8_t*)b.arena.data(),
                                                   b.offs.data(), b.lens.data(), (uint32_t)b.lens.size(),
                                                   b.tri.data(), nullptr, nullptr, 0, s);
            });
            (void)authjx_release_stream(ctx, s);
            caller.join();
            (void)authjx_release_stream(ctx, s);  // (the caller may have made a new workspace)
            (void)hipStreamDestroy(s);
        }
    });
    // readers of the last call's workspace
    for (int t = 0; t < 2; t++)
        ts.emplace_back([&] {
            while (!stop) {
                (void)authjx_last_exact_count(ctx);
                (void)authjx_last_kernel_ms(ctx);
                reads++;
            }
        });
    // host-buffer entry points on the context's stream, with rulesets compiled and freed
    ts.emplace_back([&] {
        DevBatch b(40);
        for (int i = 0; i < rounds; i++) {
            authjx_ruleset* own = compile(ctx, "a", std::to_string(i % 40).c_str());
            if (!own) {
                errors++;
                continue;
            }
            const authjx_ruleset* sets[2] = {shared, own};
            std::vector<uint32_t> sor(b.lens.size());
            for (size_t r = 0; r < sor.size(); r++) sor[r] = (uint32_t)(r & 1);
            if (authjx_eval_batch(ctx, sets, 2, sor.data(), (const uint8_t*)b.arena.data(), b.arena.size(),
                                  b.offs.data(), b.lens.data(), (uint32_t)b.lens.size(), b.tri.data(), nullptr,
                                  nullptr, 0) != AUTHJX_OK)
                errors++;
            evals++;
            authjx_free(own);
        }
    });
    // a micro-batcher: its own streams' workspaces go with authjx_batcher_destroy
    ts.emplace_back([&] {
        for (int i = 0; i < rounds / 20 + 1; i++) {
            authjx_batcher* bt = nullptr;
            if (authjx_batcher_create(ctx, 16, 50, 0, &bt) != AUTHJX_OK) {
                errors++;
                continue;
            }
            std::vector<std::thread> prod;
            for (int p = 0; p < 3; p++)
                prod.emplace_back([&, p] {
                    for (int k = 0; k < 10; k++) {
                        const std::string d = "{\"a\":" + std::to_string(p * 10 + k) + "}";
                        uint8_t tri = 0;
                        if (authjx_batcher_eval(bt, shared, (const uint8_t*)d.data(), d.size(), 0, &tri, nullptr) !=
                            AUTHJX_OK)
                            errors++;
                    }
                });
            for (auto& p : prod) p.join();
            authjx_batcher_destroy(bt);
        }
    });
    for (size_t i = 0; i < ts.size(); i++)
        if (i < 4 || i >= 6) ts[i].join();
    stop = true;
    ts[4].join();
    ts[5].join();
    authjx_free(shared);
    authjx_shutdown(ctx);
    std::printf("ok evals %llu reads %llu errors %llu\n", (unsigned long long)evals.load(),
                (unsigned long long)reads.load(), (unsigned long long)errors.load());
    return errors.load() ? 1 : 0;
}
