// ajx_index.cpp — the host-side AuthConfig index, native.
//
// Restates pkg/index/index.go's authConfigTree (:37-243): hostnames are keys, each '.'
// one tree level read from the TLD down (revertKey :236-243), the entry of the longest
// common path wins when it matches the whole key, otherwise the search climbs to the root
// taking the first '*' child that holds an entry (treeNode.get :153-174); Set / DeleteKey
// as :67-98 / :176-203. The batched lookup adds the ':port' retry of
// pkg/service/auth.go:270-280 and resolves a micro-batch of hosts into `set_of_req` ids on
// all host threads: each distinct host is walked once per thread (a per-thread memo, the
// Zipf host traffic of config C4 repeats a few hosts), labels are read straight from the
// host bytes from the last one up (no reversed copy of the key), and the tree's child maps
// are looked up by string_view. Readers share a lock the writers (reconcile) take
// exclusively, as the reference's RWMutex does (:51, :57, :68) — writer-preferring like
// Go's sync.RWMutex (a waiting Lock blocks new RLocks), so a constant lookup stream
// cannot starve a reconcile.
#include <pthread.h>

#include <algorithm>
#include <deque>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/authjx.h"

namespace {

struct Node {
    std::string label;
    int32_t entry = -1;  // AuthConfig (set) id, -1 = none
    int32_t parent = -1;
    std::unordered_map<std::string_view, int32_t> children;  // views of the children's labels
};

// the key's labels from the last one up (the reverted key, without the root label)
struct RevLabels {
    std::string_view s;
    size_t end;  // one past the next label to return
    bool done;
    explicit RevLabels(std::string_view k) : s(k), end(k.size()), done(false) {}
    bool next(std::string_view* out) {
        if (done) return false;
        const size_t dot = end == 0 ? std::string_view::npos : s.rfind('.', end - 1);
        const size_t b = dot == std::string_view::npos ? 0 : dot + 1;
        *out = s.substr(b, end - b);
        if (dot == std::string_view::npos) done = true;
        else end = dot;
        return true;
    }
};

// a reader / writer lock with writer preference (glibc's rwlock kind
// PREFER_WRITER_NONRECURSIVE); the SharedMutex interface of std::shared_lock / unique_lock
class RwLock {
   public:
    RwLock() {
        pthread_rwlockattr_t a;
        pthread_rwlockattr_init(&a);
        pthread_rwlockattr_setkind_np(&a, PTHREAD_RWLOCK_PREFER_WRITER_NONRECURSIVE_NP);
        pthread_rwlock_init(&l_, &a);
        pthread_rwlockattr_destroy(&a);
    }
    ~RwLock() { pthread_rwlock_destroy(&l_); }
    RwLock(const RwLock&) = delete;
    RwLock& operator=(const RwLock&) = delete;
    void lock() { pthread_rwlock_wrlock(&l_); }
    void unlock() { pthread_rwlock_unlock(&l_); }
    void lock_shared() { pthread_rwlock_rdlock(&l_); }
    void unlock_shared() { pthread_rwlock_unlock(&l_); }

   private:
    pthread_rwlock_t l_;
};

}  // namespace

struct authjx_index {
    std::deque<Node> nodes;  // (a deque: children's keys view labels that must not move)
    mutable RwLock mu;
    authjx_index() { nodes.emplace_back(); }  // the root, label "" (rootKeyLabel, index.go:13)

    // longestCommonLabel (index.go:205-223): the deepest node on the key's path and
    // whether the whole key was consumed
    int32_t longest(std::string_view key, bool* whole, RevLabels* rest) const {
        RevLabels it(key);
        int32_t cur = 0;
        std::string_view lab;
        RevLabels save = it;
        while (true) {
            save = it;
            if (!it.next(&lab)) {
                *whole = true;
                *rest = it;
                return cur;
            }
            const auto f = nodes[(size_t)cur].children.find(lab);
            if (f == nodes[(size_t)cur].children.end()) {
                // the labels from `lab` on are the tail; like the reference, a tail that is
                // one empty label joins to "" and counts as the whole key
                // (strings.Join([""], ".") == "", index.go:216)
                *whole = lab.empty() && it.done;
                *rest = save;
                return cur;
            }
            cur = f->second;
        }
    }

    // treeNode.get (index.go:153-174)
    int32_t get(std::string_view key) const {
        bool whole;
        RevLabels rest(key);
        const int32_t node = longest(key, &whole, &rest);
        if (whole && nodes[(size_t)node].entry >= 0) return nodes[(size_t)node].entry;
        for (int32_t cur = node; cur >= 0; cur = nodes[(size_t)cur].parent) {
            const auto f = nodes[(size_t)cur].children.find(std::string_view("*", 1));
            if (f != nodes[(size_t)cur].children.end() && nodes[(size_t)f->second].entry >= 0)
                return nodes[(size_t)f->second].entry;
        }
        return -1;
    }

    // treeNode.set (index.go:176-203)
    int set(std::string_view key, int32_t entry, bool override) {
        bool whole;
        RevLabels rest(key);
        const int32_t target = longest(key, &whole, &rest);
        if (whole) {
            if (!override) return AUTHJX_EEXIST;
            nodes[(size_t)target].entry = entry;
            return AUTHJX_OK;
        }
        std::string_view lab;
        int32_t parent = target;
        while (rest.next(&lab)) {
            nodes.emplace_back();
            Node& nn = nodes.back();
            nn.label.assign(lab.data(), lab.size());
            nn.parent = parent;
            const int32_t id = (int32_t)nodes.size() - 1;
            // (a new subtree: the first label replaces any child of that name, as
            // `target.children[tld] = node` does; below it every node is new)
            nodes[(size_t)parent].children[std::string_view(nn.label)] = id;
            parent = id;
        }
        nodes[(size_t)parent].entry = entry;
        return AUTHJX_OK;
    }

    // deleteKey (index.go:132-136): the longest common node's entry, if it is this id's
    void del(std::string_view key, int32_t entry) {
        bool whole;
        RevLabels rest(key);
        const int32_t node = longest(key, &whole, &rest);
        if (nodes[(size_t)node].entry == entry) nodes[(size_t)node].entry = -1;
    }
};

// pkg/service/auth.go:270-280: Get(host), then Get(host before its first ':') when the
// host has a port and nothing was found
static int32_t lookup_host(const authjx_index* ix, std::string_view host) {
    int32_t id = ix->get(host);
    if (id < 0) {
        const size_t c = host.find(':');
        if (c != std::string_view::npos) id = ix->get(host.substr(0, c));
    }
    return id;
}

extern "C" {

int authjx_index_new(authjx_index** out) {
    if (!out) return AUTHJX_EINVAL;
    try {
        *out = new authjx_index();
    } catch (...) {
        return AUTHJX_ENOMEM;
    }
    return AUTHJX_OK;
}

void authjx_index_free(authjx_index* ix) { delete ix; }

int authjx_index_set(authjx_index* ix, const char* key, uint32_t key_len, int32_t set_id, int override_) {
    if (!ix || (!key && key_len) || set_id < 0) return AUTHJX_EINVAL;
    std::unique_lock<RwLock> g(ix->mu);
    try {
        return ix->set(std::string_view(key ? key : "", key_len), set_id, override_ != 0);
    } catch (...) {
        return AUTHJX_ENOMEM;
    }
}

int authjx_index_delete_key(authjx_index* ix, const char* key, uint32_t key_len, int32_t set_id) {
    if (!ix || (!key && key_len)) return AUTHJX_EINVAL;
    std::unique_lock<RwLock> g(ix->mu);
    ix->del(std::string_view(key ? key : "", key_len), set_id);
    return AUTHJX_OK;
}

int authjx_index_get(const authjx_index* ix, const char* host, uint32_t host_len, int32_t* out_set) {
    if (!ix || !out_set || (!host && host_len)) return AUTHJX_EINVAL;
    std::shared_lock<RwLock> g(ix->mu);
    *out_set = lookup_host(ix, std::string_view(host ? host : "", host_len));
    return AUTHJX_OK;
}

int authjx_index_lookup_batch(const authjx_index* ix, const uint8_t* hosts, const uint64_t* offs,
                              const uint32_t* lens, uint32_t n, int32_t* out_sets, uint32_t n_threads) {
    if (!ix || (n && (!hosts || !offs || !lens || !out_sets))) return AUTHJX_EINVAL;
    std::shared_lock<RwLock> g(ix->mu);
    uint32_t nt = n_threads ? n_threads : std::max(1u, std::thread::hardware_concurrency());
    nt = std::min<uint32_t>(nt, std::max<uint32_t>(1u, n / 4096u));
    auto work = [&](uint32_t lo, uint32_t hi) {
        std::unordered_map<std::string_view, int32_t> memo;
        memo.reserve(1024);
        for (uint32_t r = lo; r < hi; r++) {
            const std::string_view h(reinterpret_cast<const char*>(hosts + offs[r]), lens[r]);
            const auto f = memo.find(h);
            if (f != memo.end()) {
                out_sets[r] = f->second;
                continue;
            }
            const int32_t id = lookup_host(ix, h);
            if (memo.size() < (1u << 16)) memo.emplace(h, id);
            out_sets[r] = id;
        }
    };
    if (nt <= 1) {
        work(0, n);
        return AUTHJX_OK;
    }
    try {
        std::vector<std::thread> th;
        const uint32_t step = (n + nt - 1) / nt;
        for (uint32_t t = 0; t < nt; t++) {
            const uint32_t lo = t * step, hi = std::min(n, lo + step);
            if (lo < hi) th.emplace_back(work, lo, hi);
        }
        for (auto& t : th) t.join();
    } catch (...) {
        return AUTHJX_ENOMEM;
    }
    return AUTHJX_OK;
}

}  // extern "C"
