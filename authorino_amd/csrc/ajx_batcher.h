// ajx_batcher.h — the micro-batcher's queue and flush policy (host C++, no HIP): the
// admission point a serving loop puts in front of the batched evaluator.
//
// In the reference every request's goroutine evaluates its AuthConfig's expressions
// itself (pkg/service/auth_pipeline.go:150-164, one goroutine per evaluator; up to 10k
// concurrent gRPC streams, main.go:69,451). Here callers submit one request each and
// block; `workers` worker threads (2 by default: one packs and launches the next batch
// while the other's batch runs on the device) each
//   - wait until max_batch requests are queued or the oldest has waited `window`,
//   - takes up to max_batch of them that share the oldest one's result shape (n_trees),
//   - completes the ones whose deadline has passed with AUTHJX_ETIMEDOUT unevaluated,
//   - orders the rest by ruleset (AuthConfig buckets: index.bucket_order — workgroups of
//     the multi-tenant kernel then mostly see one ruleset and stage it in LDS),
//   - hands the batch to the evaluator (one device launch) and wakes each caller.
// The queue is bounded: a producer waits for room (up to its deadline).
// BatchCore is evaluator-agnostic so the CPU tests drive it with a stand-in evaluator
// (tests/native/batcher_host.cpp); ajx_api.cpp plugs in the device evaluation.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace ajx {

using Clock = std::chrono::steady_clock;

inline uint64_t mono_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

constexpr int kBatchOk = 0;
constexpr int kBatchTimedOut = -5;  // AUTHJX_ETIMEDOUT
constexpr int kBatchClosed = -6;    // AUTHJX_ECLOSED

struct BatchReq {
    const void* rs = nullptr;  // the ruleset (opaque to the core)
    uint32_t n_out = 1;        // results per request (the ruleset's trees)
    const uint8_t* doc = nullptr;
    size_t len = 0;
    uint64_t deadline_ns = 0;  // steady-clock ns, 0 = none
    uint64_t enq_ns = 0;
    uint8_t* out_tri = nullptr;  // n_out entries
    int32_t* out_err = nullptr;  // n_out entries or null
    // completion
    int rc = kBatchOk;
    bool done = false;
    std::mutex m;
    std::condition_variable cv;
    void complete(int code) {
        std::lock_guard<std::mutex> lock(m);
        rc = code;
        done = true;
        cv.notify_one();
    }
};

struct BatchStats {
    uint64_t batches = 0, requests = 0, expired = 0, max_batch_seen = 0;
};

class BatchCore {
   public:
    // queue_cap 0: 4 * max_batch. evaluate(batch, worker): fills out_tri / out_err of every
    // request and returns an AUTHJX code (applied to the whole batch on failure); worker is
    // the calling worker's index (its own buffers and stream)
    using Evaluator = std::function<int(std::vector<BatchReq*>&, uint32_t)>;

    BatchCore(uint32_t max_batch, uint64_t window_ns, uint32_t queue_cap, Evaluator ev, uint32_t workers = 1)
        : max_batch_(max_batch ? max_batch : 1), window_ns_(window_ns),
          queue_cap_(queue_cap ? queue_cap : 4 * (max_batch ? max_batch : 1)),
          eval_(std::move(ev)) {
        for (uint32_t k = 0; k < (workers ? workers : 1); k++) workers_.emplace_back([this, k] { run(k); });
    }
    ~BatchCore() { close(); }

    // stop admitting; what is queued is evaluated, then the worker ends
    void close() {
        {
            std::lock_guard<std::mutex> lock(mu_);
            if (stopping_) return;
            stopping_ = true;
        }
        cv_work_.notify_all();
        cv_room_.notify_all();
        for (std::thread& t : workers_)
            if (t.joinable()) t.join();
    }

    // blocking submit; returns the request's code
    int submit(BatchReq& r) {
        r.enq_ns = mono_ns();
        {
            std::unique_lock<std::mutex> lock(mu_);
            while (q_.size() >= queue_cap_ && !stopping_) {
                if (r.deadline_ns) {
                    const uint64_t now = mono_ns();
                    if (now >= r.deadline_ns) {
                        stats_.expired++;
                        return kBatchTimedOut;
                    }
                    cv_room_.wait_for(lock, std::chrono::nanoseconds(r.deadline_ns - now));
                } else {
                    cv_room_.wait(lock);
                }
            }
            if (stopping_) return kBatchClosed;
            q_.push_back(&r);
        }
        cv_work_.notify_one();
        std::unique_lock<std::mutex> lock(r.m);
        r.cv.wait(lock, [&] { return r.done; });
        return r.rc;
    }

    BatchStats stats() {
        std::lock_guard<std::mutex> lock(mu_);
        return stats_;
    }

   private:
    void run(uint32_t wid) {
        std::vector<BatchReq*> batch;
        for (;;) {
            batch.clear();
            {
                std::unique_lock<std::mutex> lock(mu_);
                cv_work_.wait(lock, [&] { return stopping_ || !q_.empty(); });
                if (q_.empty()) return;  // stopping, nothing left
                // a full batch or the oldest request's window, whichever comes first (the
                // oldest is looked up after every wake: another worker may have taken the
                // requests this one was waiting for, and newer ones get their own window)
                while (!stopping_ && !q_.empty() && q_.size() < max_batch_) {
                    const uint64_t flush_at = q_.front()->enq_ns + window_ns_;
                    const uint64_t now = mono_ns();
                    if (now >= flush_at) break;
                    cv_work_.wait_for(lock, std::chrono::nanoseconds(flush_at - now));
                }
                if (q_.empty()) continue;  // (another worker took them)
                // up to max_batch requests of the oldest request's result shape
                const uint32_t shape = q_.front()->n_out;
                for (auto it = q_.begin(); it != q_.end() && batch.size() < max_batch_;) {
                    if ((*it)->n_out == shape) {
                        batch.push_back(*it);
                        it = q_.erase(it);
                    } else {
                        ++it;
                    }
                }
            }
            cv_room_.notify_all();
            // deadlines: a request past its deadline is not evaluated
            const uint64_t now = mono_ns();
            uint64_t expired = 0;
            std::vector<BatchReq*> live;
            live.reserve(batch.size());
            std::vector<BatchReq*> late;
            for (BatchReq* r : batch) {
                if (r->deadline_ns && now >= r->deadline_ns) late.push_back(r);
                else live.push_back(r);
            }
            expired = late.size();
            if (expired) {
                std::lock_guard<std::mutex> lock(mu_);
                stats_.expired += expired;
            }
            for (BatchReq* r : late) r->complete(kBatchTimedOut);
            // AuthConfig buckets (stable: arrival order inside a bucket)
            std::stable_sort(live.begin(), live.end(),
                             [](const BatchReq* a, const BatchReq* b) { return a->rs < b->rs; });
            int rc = live.empty() ? kBatchOk : eval_(live, wid);
            {  // counted before the callers wake, so a caller that returns sees its batch
                std::lock_guard<std::mutex> lock(mu_);
                if (!live.empty()) {
                    stats_.batches++;
                    stats_.requests += live.size();
                    stats_.max_batch_seen = std::max<uint64_t>(stats_.max_batch_seen, live.size());
                }
            }
            for (BatchReq* r : live) r->complete(rc);
        }
    }

    const uint32_t max_batch_;
    const uint64_t window_ns_;
    const uint32_t queue_cap_;
    Evaluator eval_;
    std::mutex mu_;
    std::condition_variable cv_work_, cv_room_;
    std::deque<BatchReq*> q_;
    bool stopping_ = false;
    BatchStats stats_;
    std::vector<std::thread> workers_;
};

}  // namespace ajx
