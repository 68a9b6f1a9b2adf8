// san_fuzz.cpp — TEST-ONLY: the host code (reconcile-time compiler, Go-RE2 -> DFA builder,
// selector parser) and the host builds of the per-document device logic (exact scan,
// single-pass scan, the row kernel on its 64-lane emulation, number canon) under
// AddressSanitizer / UBSan, driven by random selectors, regexes and (mutated) documents.
// Besides the sanitizers' own reports, it checks the single-pass and row paths against
// the exact path wherever
// they decide (an internal differential; the oracle comparisons live in the Python
// suites). Built by `make san` (tests/native/Makefile); run by tests/test_sanitizers.py.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/authjx.h"

extern "C" {
void* ht_compile(const authjx_tree* tree, int32_t* status, char* err, size_t cap, int* rc);
void ht_free(void* h);
int ht_eval(void* h, const uint8_t* doc, uint32_t len, uint8_t* res, int32_t* err);
int ht_eval_fast(void* h, const uint8_t* doc, uint32_t len, uint32_t mis, uint8_t* res, int32_t* err);
int ht_eval_lean(void* h, const uint8_t* doc, uint32_t len, uint32_t mis, uint8_t* res, int32_t* err);
}

static std::mt19937_64 rng;
static uint64_t rnd(uint64_t n) { return n ? rng() % n : 0; }

static const char* kKeys[] = {"a", "b", "c", "ab", "x.y", "0", "1", "k\xc3\xa9", "long-key-name-0123456789", "",
                              "q\"t", "s\\l", "n", "a b"};
static const char* kStrs[] = {"", "x", "hello", "a\\\"b", "back\\\\slash", "t\\tab", "\xc3\xa9", "\\u00e9",
                              "\\ud83d\\ude00", "<&>", "true", "GET", "/api/v1/orders/7", "\\ud800"};
static const char* kNums[] = {"0", "-0", "1", "-12", "1.5", "1e3", "1E-7", "0.30000000000000004", "1e400",
                              "4.9406564584124654e-324", "12345678901234567890", "1.7976931348623157e308",
                              "-2.5e-3", "9.999999999999999e20"};
static const char* kRegex[] = {"^a", "b$", "[0-9]+", "(?i)get", "^/api/v[12]/", "a|b|c", "\\bword\\b", ".*",
                               "x{2,3}", "[^a-z]", "\\d{3}-\\d{4}", "(a+)+$", "\\p{L}", "[[:alpha:]]", "(", "a{1001}",
                               "\\Qa.b\\E", "^$", "\xc3\xa9+", "(?s).", "[\\x00-\\x1f]"};

static std::string json_string(const char* s) { return std::string("\"") + s + "\""; }

static std::string rand_value(int depth) {
    const uint64_t r = rnd(100);
    if (depth <= 0 || r < 45) {
        switch (rnd(4)) {
            case 0: return json_string(kStrs[rnd(sizeof kStrs / sizeof *kStrs)]);
            case 1: return kNums[rnd(sizeof kNums / sizeof *kNums)];
            case 2: return (const char*[]){"true", "false", "null"}[rnd(3)];
            default: return "\"v" + std::to_string(rnd(20)) + "\"";
        }
    }
    std::string s;
    const int n = (int)rnd(5);
    if (r < 75) {
        s = "{";
        for (int i = 0; i < n; i++) {
            if (i) s += ",";
            s += json_string(kKeys[rnd(sizeof kKeys / sizeof *kKeys)]) + ":" + rand_value(depth - 1);
        }
        return s + "}";
    }
    s = "[";
    for (int i = 0; i < n; i++) {
        if (i) s += ",";
        s += rand_value(depth - 1);
    }
    return s + "]";
}

static std::string rand_doc() {
    std::string s = "{";
    const int n = 1 + (int)rnd(6);
    for (int i = 0; i < n; i++) {
        if (i) s += ",";
        s += json_string(kKeys[rnd(sizeof kKeys / sizeof *kKeys)]) + ":" + rand_value(3);
    }
    return s + "}";
}

static std::string mutate(std::string d) {
    const char pool[] = "{}[]\":,\\ 0ae-u.\x01\xff";
    switch (rnd(4)) {
        case 0:
            if (!d.empty()) d.resize(rnd(d.size()));
            break;
        case 1:
            for (int k = 0; k < 3 && !d.empty(); k++) d[rnd(d.size())] = pool[rnd(sizeof pool - 1)];
            break;
        case 2:
            if (d.size() > 4) d.erase(rnd(d.size() - 1), 1 + rnd(3));
            break;
        default: d = " \n" + d + " x";
    }
    return d;
}

static std::string rand_selector() {
    std::string s;
    const int n = 1 + (int)rnd(3);
    for (int i = 0; i < n; i++) {
        if (i) s += ".";
        const uint64_t r = rnd(10);
        if (r < 2) s += std::to_string(rnd(3));
        else if (r == 2) s += "x\\.y";
        else if (r == 3) s += (const char*[]){"#", "@this", "a*", "b?", "[a,b]", "a|b"}[rnd(6)];
        else s += kKeys[rnd(6)];
    }
    return s;
}

int main(int argc, char** argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 300;
    rng.seed(argc > 2 ? (uint64_t)atoll(argv[2]) : 7);
    long docs = 0, fast_decided = 0, lean_decided = 0, bad = 0;
    for (long it = 0; it < iters; it++) {
        const int np = 1 + (int)rnd(8);
        std::vector<std::string> sels(np), vals(np);
        std::vector<authjx_pattern> pats(np);
        std::vector<authjx_node> nodes;
        for (int i = 0; i < np; i++) {
            sels[i] = rand_selector();
            const int op = (int)rnd(7);  // 0 and 6: unknown operators
            vals[i] = op == 5 ? kRegex[rnd(sizeof kRegex / sizeof *kRegex)]
                              : (rnd(2) ? std::string(kStrs[rnd(sizeof kStrs / sizeof *kStrs)])
                                        : std::string(kNums[rnd(sizeof kNums / sizeof *kNums)]));
            pats[i] = authjx_pattern{sels[i].c_str(), (uint32_t)sels[i].size(), op, vals[i].c_str(),
                                     (uint32_t)vals[i].size()};
            nodes.push_back(authjx_node{AUTHJX_NODE_PATTERN, -1, -1, i});
        }
        int root = -1;
        for (int i = np - 1; i >= 0; i--) {
            nodes.push_back(authjx_node{rnd(3) ? AUTHJX_NODE_AND : AUTHJX_NODE_OR, i, root, -1});
            root = (int)nodes.size() - 1;
        }
        const authjx_tree tree{pats.data(), (uint32_t)np, nodes.data(), (uint32_t)nodes.size(), root};
        int rc = 0;
        std::vector<int32_t> st(np);
        char err[256];
        void* h = ht_compile(&tree, st.data(), err, sizeof err, &rc);
        if (!h) continue;
        for (int k = 0; k < 12; k++) {
            std::string d = rand_doc();
            if (rnd(3) == 0) d = mutate(d);
            std::vector<uint8_t> r0(np), r1(np), r2(np);
            int32_t e0 = 0, e1 = 0, e2 = 0;
            const int t0 = ht_eval(h, (const uint8_t*)d.data(), (uint32_t)d.size(), r0.data(), &e0);
            const int t1 = ht_eval_fast(h, (const uint8_t*)d.data(), (uint32_t)d.size(), (uint32_t)rnd(16), r1.data(), &e1);
            const int t2 = ht_eval_lean(h, (const uint8_t*)d.data(), (uint32_t)d.size(), (uint32_t)rnd(16), r2.data(), &e2);
            docs++;
            if (t1 >= 0) {
                fast_decided++;
                if (t1 != t0 || r1 != r0) {
                    if (bad < 10) printf("FAST MISMATCH doc=%s\n", d.c_str());
                    bad++;
                }
            }
            if (t2 >= 0 && std::find(r0.begin(), r0.end(), (uint8_t)3) == r0.end()) {
                lean_decided++;
                if (t2 != t0 || r2 != r0) {
                    if (bad < 10) printf("LEAN MISMATCH doc=%s\n", d.c_str());
                    bad++;
                }
            }
        }
        ht_free(h);
    }
    printf("docs %ld fast_decided %ld lean_decided %ld mismatches %ld\n", docs, fast_decided, lean_decided, bad);
    return bad ? 1 : 0;
}
