// float_diff.cpp — TEST-ONLY: gjson Result.String() of JSON numbers, the device code
// (authorino_amd/csrc/ajx_device.h num_canon + ajx_float.h, host build) against the
// oracle (oracle/gofloat_ref.c: Go ParseFloat via strtod, FormatFloat shortest by
// round-trip search), on generated number texts:
//   go        Go-shortest text of random float64 bit patterns (what encoding/json writes)
//   g17/g16   %.17g / %.16g of random doubles (16-17 significant digits)
//   long      random 18..60-digit decimals with random exponents
//   sub       subnormals and values near the float64 ends (2^-1074.., MaxFloat64..)
//   half      exact decimal midpoints between neighbouring doubles, and just above /
//             below them (ties to even, the hardest rounding cases)
//   edge      1e21 boundary, powers of ten, 0.1 + 0.2 sums, MaxFloat64 neighbours
// Usage: float_diff N SEED  -> prints "checked C mismatches M" and the first mismatches.
#define AJX_HD inline
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>

#include "../../authorino_amd/csrc/ajx_fast.h"

extern "C" {
#include "../../oracle/oracle.h"
}

using namespace ajx;

static std::string device_string(const std::string& raw) {
    // gjson: a raw -?[0-9]+ is its own String(); otherwise the number canon
    size_t k = 0;
    if (k < raw.size() && raw[k] == '-') k++;
    bool integer = k < raw.size();
    for (; k < raw.size(); k++)
        if (raw[k] < '0' || raw[k] > '9') integer = false;
    if (integer) return raw;
    StrSrc s;
    if (!s.init_num<true>((const uint8_t*)raw.data(), 0, (uint32_t)raw.size())) return "<undecided>";
    std::string out;
    for (int c; (c = s.next()) >= 0;) out.push_back((char)c);
    return out;
}

static std::string oracle_string(const std::string& raw) {
    size_t k = 0;
    if (k < raw.size() && raw[k] == '-') k++;
    bool integer = k < raw.size();
    for (; k < raw.size(); k++)
        if (raw[k] < '0' || raw[k] > '9') integer = false;
    if (integer) return raw;
    double f;
    or_go_parse_float(raw.data(), raw.size(), &f);
    or_buf b;
    memset(&b, 0, sizeof b);
    or_go_format_float(f, &b);
    std::string out(b.p, b.n);
    or_buf_free(&b);
    return out;
}

static std::string go_text(double f) {  // FormatFloat(f, 'g'-like) via the oracle: 'f' shortest
    or_buf b;
    memset(&b, 0, sizeof b);
    or_go_format_float(f, &b);
    std::string out(b.p, b.n);
    or_buf_free(&b);
    return out;
}

// --stdin: one number text per line in, "device<TAB>oracle<TAB>raw-fast" out (raw-fast:
// 1 when the single-pass kernels' raw rule, -?[0-9]+ or a simple decimal, takes the text
// as its own String()), for an independent check of both against numpy/Python
static int stdin_mode() {
    static char line[4096];
    while (fgets(line, sizeof line, stdin)) {
        size_t n = strlen(line);
        while (n && (line[n - 1] == '\n' || line[n - 1] == '\r')) line[--n] = 0;
        const std::string raw(line, n);
        uint32_t k = 0;
        if (k < n && raw[k] == '-') k++;
        bool integer = k < n;
        for (uint32_t j = k; j < n; j++)
            if (raw[j] < '0' || raw[j] > '9') integer = false;
        const bool fast = integer || simple_decimal((const uint8_t*)raw.data() + k, (uint32_t)(n - k));
        printf("%s\t%s\t%d\n", device_string(raw).c_str(), oracle_string(raw).c_str(), fast ? 1 : 0);
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && strcmp(argv[1], "--stdin") == 0) return stdin_mode();
    const long N = argc > 1 ? atol(argv[1]) : 100000;
    const unsigned seed = argc > 2 ? (unsigned)atol(argv[2]) : 1;
    std::mt19937_64 rng(seed);
    long checked = 0, bad = 0;
    auto check = [&](const std::string& raw, const char* kind) {
        const std::string a = device_string(raw), b = oracle_string(raw);
        checked++;
        if (a != b) {
            if (bad < 20) printf("MISMATCH %s raw=%s device=%s oracle=%s\n", kind, raw.c_str(), a.c_str(), b.c_str());
            bad++;
        }
    };
    char buf[1200];
    auto rand_double = [&]() {
        for (;;) {
            uint64_t bits = rng();
            double f;
            memcpy(&f, &bits, 8);
            if (std::isfinite(f)) return f;
        }
    };
    for (long i = 0; i < N; i++) {
        const double f = rand_double();
        // Go's shortest text (fixed layout) and an exponent form of the same digits
        check(go_text(f), "go");
        snprintf(buf, sizeof buf, "%.17g", f);
        check(buf, "g17");
        snprintf(buf, sizeof buf, "%.16g", f);
        check(buf, "g16");
        // a double of ordinary magnitude, as metadata floats look
        const double g = std::ldexp((double)(rng() >> 11), -(int)(rng() % 80)) * ((rng() & 1) ? 1 : -1);
        check(go_text(g), "go");
        snprintf(buf, sizeof buf, "%.17g", g);
        check(buf, "g17");
        if (i % 4 == 0) {  // long decimals
            const int nd = 18 + (int)(rng() % 43);
            std::string s = (rng() & 1) ? "-" : "";
            s.push_back((char)('1' + rng() % 9));
            const int dot = (int)(rng() % nd);
            for (int k = 1; k < nd; k++) {
                if (k == dot) s.push_back('.');
                s.push_back((char)('0' + rng() % 10));
            }
            if (s.find('.') == std::string::npos) s += ".5";
            const int e = (int)(rng() % 700) - 350;
            s += "e" + std::to_string(e);
            check(s, "long");
        }
        if (i % 8 == 0) {  // subnormals and the ends of the range
            const uint64_t bits = rng() % (1ull << 52);
            double sub;
            memcpy(&sub, &bits, 8);
            check(go_text(sub), "sub");
            snprintf(buf, sizeof buf, "%.17g", sub);
            check(buf, "sub");
            const uint64_t hb = 0x7FEFFFFFFFFFFFFFull - (rng() % 1000000);
            double hi;
            memcpy(&hi, &hb, 8);
            check(go_text(hi), "sub");
            snprintf(buf, sizeof buf, "%.17g", hi);
            check(buf, "sub");
        }
        if (i % 16 == 0) {  // exact midpoints between neighbours, and a hair off them
            const double a = std::fabs(rand_double());
            const double b = std::nextafter(a, INFINITY);
            if (std::isfinite(b)) {
                const long double mid = ((long double)a + (long double)b) / 2;
                snprintf(buf, sizeof buf, "%.780Le", mid);
                std::string m = buf;
                const size_t epos = m.find('e');
                std::string mant = m.substr(0, epos), ex = m.substr(epos);
                while (mant.size() > 2 && mant.back() == '0') mant.pop_back();
                check(mant + ex, "half");
                check(mant + "0000001" + ex, "half");
                // just below: decrement the last digit when it is not 0
                std::string lo = mant;
                if (lo.back() > '0' && lo.back() <= '9') {
                    lo.back()--;
                    check(lo + "9999999" + ex, "half");
                }
            }
        }
    }
    const char* edges[] = {"1e21", "9.999999999999999e20", "1e20", "123456789012345678901234.5", "0.1", "0.2",
                           "0.30000000000000004", "1.7976931348623157e308", "1.7976931348623158e308",
                           "1.7976931348623159e308", "2e308", "-1.7976931348623157e308", "4.9406564584124654e-324",
                           "2.4703282292062327e-324", "2.4703282292062328e-324", "2.2250738585072014e-308",
                           "2.2250738585072011e-308", "1e-400", "-1e-400", "1e400", "0.000001", "1e-7",
                           "37.77492950000001", "-122.41941550000001", "9007199254740993", "9007199254740993.0",
                           "1.00000000000000011102230246251565404236316680908203125",
                           "1.00000000000000011102230246251565404236316680908203124",
                           "1.00000000000000011102230246251565404236316680908203126", "5e-324", "1e-323",
                           "100000000000000000000000", "1e23", "8.41e21", "5.0e-324", "0.0000000000000000000000001",
                           "-0.0", "0e10", "1E5", "1.5E-5", "-2.5e+3"};
    for (const char* e : edges) check(e, "edge");
    for (int p = -325; p <= 310; p++) {
        snprintf(buf, sizeof buf, "1e%d", p);
        check(buf, "edge");
        snprintf(buf, sizeof buf, "9.999999999999999e%d", p);
        check(buf, "edge");
    }
    printf("checked %ld mismatches %ld\n", checked, bad);
    return bad ? 1 : 0;
}
