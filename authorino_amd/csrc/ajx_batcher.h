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

#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
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
    // completion. Wake mode 0: this request's condition variable; 1: `flag`, then one
    // broadcast on the core's completion word for the whole batch; 2: `flag` as this
    // request's own futex word; 3: as 2, woken as node `idx` of a binary tree over the batch
    // (`fan`): each woken caller wakes its two children before it returns, so the worker
    // makes two wake calls per batch and a batch of n is woken in log2(n) rounds
    int rc = kBatchOk;
    bool done = false;
    std::atomic<uint32_t> flag{0};
    uint64_t done_ns = 0;
    struct Fan* fan = nullptr;
    uint32_t idx = 0;
    std::mutex m;
    std::condition_variable cv;
    void complete(int code) {
        std::lock_guard<std::mutex> lock(m);
        rc = code;
        done = true;
        done_ns = mono_ns();
        cv.notify_one();
    }
};

// wake mode 3: the batch's requests in wake order, shared by the callers that wake each
// other; freed by the last one done with it
struct Fan {
    std::vector<BatchReq*> rs;
    std::atomic<uint32_t> left{0};
};

struct BatchStats {
    uint64_t batches = 0, requests = 0, expired = 0, max_batch_seen = 0;
    // profiling sums (ns): queue wait (enqueue to the batch's evaluation, per request), the
    // evaluations (per batch), waking the batch's callers (per batch), and the time from a
    // request's completion to its caller running again (per request)
    uint64_t wait_ns = 0, eval_ns = 0, wake_ns = 0, resume_ns = 0;
};

inline long futex_op(std::atomic<uint32_t>* w, int op, uint32_t v) {
    return syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), op | FUTEX_PRIVATE_FLAG, v, nullptr, nullptr, 0);
}

// publishes r's completion on its own futex word. (r's caller may return as soon as the
// store lands, so the wake can reach a word no longer in use: that is a spurious wake of a
// waiter there, or EFAULT, and every wait here loops on its own condition.)
inline void wake_one(BatchReq* r) {
    r->flag.store(1, std::memory_order_release);
    futex_op(&r->flag, FUTEX_WAKE, 1);
}

// wake mode 3: node i wakes nodes 2i+1 and 2i+2, then drops its share of the fan
inline void fan_out(Fan* f, uint32_t i) {
    const uint32_t n = (uint32_t)f->rs.size();
    for (uint32_t c = 2 * i + 1; c <= 2 * i + 2 && c < n; c++) wake_one(f->rs[c]);
    if (f->left.fetch_sub(1, std::memory_order_acq_rel) == 1) delete f;
}

class BatchCore {
   public:
    // queue_cap 0: 4 * max_batch. evaluate(batch, worker): fills out_tri / out_err of every
    // request and returns an AUTHJX code (applied to the whole batch on failure); worker is
    // the calling worker's index (its own buffers and stream)
    using Evaluator = std::function<int(std::vector<BatchReq*>&, uint32_t)>;

    BatchCore(uint32_t max_batch, uint64_t window_ns, uint32_t queue_cap, Evaluator ev, uint32_t workers = 1,
              uint32_t wake_mode = 0)
        : max_batch_(max_batch ? max_batch : 1), window_ns_(window_ns), wake_mode_(wake_mode),
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
        if (wake_mode_ == 1) {
            for (;;) {
                const uint32_t g = gen_.load(std::memory_order_acquire);
                if (r.flag.load(std::memory_order_acquire)) break;
                futex_op(&gen_, FUTEX_WAIT, g);
            }
        } else if (wake_mode_ >= 2) {
            while (!r.flag.load(std::memory_order_acquire)) futex_op(&r.flag, FUTEX_WAIT, 0);
            if (r.fan) fan_out(r.fan, r.idx);
        } else {
            std::unique_lock<std::mutex> lock(r.m);
            r.cv.wait(lock, [&] { return r.done; });
        }
        resume_ns_.fetch_add(mono_ns() - r.done_ns, std::memory_order_relaxed);
        return r.rc;
    }

    BatchStats stats() {
        std::lock_guard<std::mutex> lock(mu_);
        BatchStats st = stats_;
        st.resume_ns = resume_ns_.load(std::memory_order_relaxed);
        return st;
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
            finish(late, kBatchTimedOut, now);
            // AuthConfig buckets (stable: arrival order inside a bucket)
            std::stable_sort(live.begin(), live.end(),
                             [](const BatchReq* a, const BatchReq* b) { return a->rs < b->rs; });
            const uint64_t t_eval = mono_ns();
            int rc = live.empty() ? kBatchOk : eval_(live, wid);
            const uint64_t t_done = mono_ns();
            {  // counted before the callers wake, so a caller that returns sees its batch
                std::lock_guard<std::mutex> lock(mu_);
                if (!live.empty()) {
                    stats_.batches++;
                    stats_.requests += live.size();
                    stats_.max_batch_seen = std::max<uint64_t>(stats_.max_batch_seen, live.size());
                    for (BatchReq* r : live) stats_.wait_ns += t_eval - r->enq_ns;
                    stats_.eval_ns += t_done - t_eval;
                }
            }
            finish(live, rc, t_done);
            const uint64_t t_woke = mono_ns();
            std::lock_guard<std::mutex> lock(mu_);
            stats_.wake_ns += t_woke - t_done;
        }
    }

    // wakes the callers of `rs` with `code` (a caller may return, and its request go out
    // of scope, as soon as its own completion is published)
    void finish(std::vector<BatchReq*>& rs, int code, uint64_t t) {
        if (rs.empty()) return;
        if (wake_mode_ == 1) {
            for (BatchReq* r : rs) {
                r->rc = code;
                r->done_ns = t;
                r->flag.store(1, std::memory_order_release);
            }
            gen_.fetch_add(1, std::memory_order_acq_rel);
            futex_op(&gen_, FUTEX_WAKE, 0x7FFFFFFF);
        } else if (wake_mode_ == 2 || (wake_mode_ == 3 && rs.size() <= 2)) {
            for (BatchReq* r : rs) {
                r->rc = code;
                r->done_ns = t;
            }
            for (BatchReq* r : rs) wake_one(r);
        } else if (wake_mode_ == 3) {
            Fan* f = new Fan();
            f->rs = rs;
            f->left.store((uint32_t)rs.size(), std::memory_order_relaxed);
            for (uint32_t i = 0; i < (uint32_t)rs.size(); i++) {
                rs[i]->rc = code;
                rs[i]->done_ns = t;
                rs[i]->fan = f;
                rs[i]->idx = i;
            }
            wake_one(rs[0]);  // (node 0 wakes 1 and 2, and so on)
        } else {
            for (BatchReq* r : rs) r->complete(code);
        }
    }

    const uint32_t max_batch_;
    const uint64_t window_ns_;
    const uint32_t wake_mode_;
    const uint32_t queue_cap_;
    Evaluator eval_;
    std::mutex mu_;
    std::condition_variable cv_work_, cv_room_;
    std::deque<BatchReq*> q_;
    bool stopping_ = false;
    BatchStats stats_;
    std::vector<std::thread> workers_;
    std::atomic<uint32_t> gen_{0};  // wake mode 1: bumped and broadcast once per batch
    std::atomic<uint64_t> resume_ns_{0};
};

}  // namespace ajx
