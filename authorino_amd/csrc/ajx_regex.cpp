// ajx_regex.cpp — Go regexp (RE2 syntax, Go 1.21) -> DFA over rune classes.
//
// Front end: the operator-stack parser of regexp/syntax with the Perl flag set
// (ClassNL | OneLine | PerlX | UnicodeGroups), keeping every rule that decides whether
// regexp.Compile fails (the reference turns that failure into Pattern.Matches' error,
// pkg/jsonexp/expressions.go:87-90, pinned by
// pkg/evaluators/authorization/json_test.go:182-193).
//
// Back end: Thompson NFA over rune sets with empty-width assertions, then a subset
// construction for the UNANCHORED boolean search MatchString performs:
//   DFA state = (threads waiting for the next rune, kind of the previous rune)
//   on rune class c: closure(threads + start) under EmptyOpContext(prev, c);
//                    MATCH reachable -> absorbing accept state; else step on c.
//   end of text:     accept if MATCH is reachable under EmptyOpContext(prev, EOT).
// The alphabet is the partition of all runes by (membership in every rune set of the
// program, word / newline / other), so assertions only need the class of each rune.
#include "ajx_regex.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>

namespace ajx {
namespace {

constexpr uint32_t kMaxRune = 0x10FFFF;

struct Range {
    uint32_t lo, hi;
};
using RuneSet = std::vector<Range>;

void normalize(RuneSet& s) {
    if (s.empty()) return;
    std::sort(s.begin(), s.end(), [](const Range& a, const Range& b) { return a.lo < b.lo || (a.lo == b.lo && a.hi < b.hi); });
    RuneSet o;
    for (const Range& r : s) {
        if (!o.empty() && r.lo <= o.back().hi + 1) o.back().hi = std::max(o.back().hi, r.hi);
        else o.push_back(r);
    }
    s.swap(o);
}

RuneSet negate(RuneSet s) {
    normalize(s);
    RuneSet o;
    uint32_t next = 0;
    for (const Range& r : s) {
        if (r.lo > next) o.push_back({next, r.lo - 1});
        next = r.hi + 1;
    }
    if (next <= kMaxRune) o.push_back({next, kMaxRune});
    return o;
}

// ---- AST --------------------------------------------------------------------------
enum Op {
    kLit,     // rune set
    kEmpty,
    kAssert,
    kStar, kPlus, kQuest, kRepeat,
    kConcat, kAlt, kCapture,
    kLeftParen, kVerticalBar  // pseudo
};
enum { kBOL = 1, kEOL = 2, kBOT = 4, kEOT = 8, kWB = 16, kNWB = 32 };
enum { fFold = 1, fDotNL = 2, fOneLine = 4, fNonGreedy = 8 };

struct Node {
    Op op;
    int flags = 0;
    RuneSet set;
    int bits = 0;
    std::vector<Node*> sub;
    int min = 0, max = 0;
    int cap = 0;
};

struct ParseError {
    std::string code, expr;
};
struct Unsupported {};

bool is_word_byte(uint32_t c) {
    return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_';
}

class Parser {
  public:
    explicit Parser(const std::string& s) : whole_(s) {}

    Node* parse() {
        flags_ = fOneLine;
        const std::string& s = whole_;
        size_t i = 0;
        size_t last_repeat = std::string::npos;  // start of the previous repeat operator
        while (i < s.size()) {
            size_t repeat = std::string::npos;
            char c = s[i];
            switch (c) {
                case '(':
                    if (i + 1 < s.size() && s[i + 1] == '?') {
                        i = perl_flags(i);
                        break;
                    }
                    {
                        Node* lp = make(kLeftParen);
                        lp->cap = ++ncap_;
                        push(lp);
                    }
                    i++;
                    break;
                case '|':
                    collapse_concat();
                    push(make(kVerticalBar));
                    i++;
                    break;
                case ')': {
                    collapse_concat();
                    collapse_alt();
                    size_t n = stack_.size();
                    if (n < 2 || stack_[n - 2]->op != kLeftParen) throw ParseError{"unexpected )", whole_};
                    Node* body = stack_[n - 1];
                    Node* lp = stack_[n - 2];
                    stack_.resize(n - 2);
                    flags_ = lp->flags;
                    if (lp->cap == 0) push(body);
                    else {
                        Node* capn = make(kCapture);
                        capn->sub.push_back(body);
                        push(capn);
                    }
                    i++;
                    break;
                }
                case '^': {
                    Node* a = make(kAssert);
                    a->bits = (flags_ & fOneLine) ? kBOT : kBOL;
                    push(a);
                    i++;
                    break;
                }
                case '$': {
                    Node* a = make(kAssert);
                    a->bits = (flags_ & fOneLine) ? kEOT : kEOL;
                    push(a);
                    i++;
                    break;
                }
                case '.': {
                    Node* d = make(kLit);
                    if (flags_ & fDotNL) d->set = {{0, kMaxRune}};
                    else d->set = {{0, 9}, {11, kMaxRune}};
                    push(d);
                    i++;
                    break;
                }
                case '[':
                    i = parse_class(i);
                    break;
                case '*': case '+': case '?': case '{': {
                    Op op;
                    int mn = 0, mx = 0;
                    size_t end = i + 1;
                    if (c == '{') {
                        if (!parse_repeat(i, &mn, &mx, &end)) {
                            literal('{');
                            i++;
                            break;
                        }
                        op = kRepeat;
                        if (mn < 0 || mn > 1000 || mx > 1000 || (mx >= 0 && mn > mx))
                            throw ParseError{"invalid repeat count", s.substr(i, end - i)};
                    } else {
                        op = c == '*' ? kStar : c == '+' ? kPlus : kQuest;
                    }
                    size_t after = end;
                    if (after < s.size() && s[after] == '?') after++;
                    if (last_repeat != std::string::npos)
                        throw ParseError{"invalid nested repetition operator", s.substr(last_repeat, after - last_repeat)};
                    if (stack_.empty() || stack_.back()->op >= kLeftParen)
                        throw ParseError{"missing argument to repetition operator", s.substr(i, after - i)};
                    Node* r = make(op);
                    r->min = mn;
                    r->max = mx;
                    r->sub.push_back(stack_.back());
                    stack_.back() = r;
                    if (op == kRepeat && (mn >= 2 || mx >= 2) && !repeat_ok(r, 1000))
                        throw ParseError{"invalid repeat count", s.substr(i, after - i)};
                    repeat = i;
                    i = after;
                    break;
                }
                case '\\':
                    i = parse_backslash(i);
                    break;
                default: {
                    uint32_t r;
                    size_t k = next_rune(i, &r);
                    literal(r);
                    i += k;
                    break;
                }
            }
            last_repeat = repeat;
        }
        collapse_concat();
        collapse_alt();
        if (stack_.size() != 1) throw ParseError{"missing closing )", whole_};
        return stack_[0];
    }

  private:
    const std::string& whole_;
    std::vector<std::unique_ptr<Node>> pool_;
    std::vector<Node*> stack_;
    int flags_ = 0;
    int ncap_ = 0;

    Node* make(Op op) {
        pool_.emplace_back(new Node());
        Node* n = pool_.back().get();
        n->op = op;
        n->flags = flags_;
        return n;
    }
    void push(Node* n) { stack_.push_back(n); }

    size_t next_rune(size_t i, uint32_t* r) const {
        const unsigned char* u = reinterpret_cast<const unsigned char*>(whole_.data());
        size_t n = whole_.size() - i;
        if (n == 0) { *r = 0xFFFD; return 0; }
        uint32_t b0 = u[i];
        if (b0 < 0x80) { *r = b0; return 1; }
        int sz = 0;
        uint32_t lo = 0x80, hi = 0xBF, v = 0;
        if (b0 >= 0xC2 && b0 <= 0xDF) { sz = 2; v = b0 & 0x1F; }
        else if (b0 >= 0xE0 && b0 <= 0xEF) { sz = 3; v = b0 & 0x0F; if (b0 == 0xE0) lo = 0xA0; if (b0 == 0xED) hi = 0x9F; }
        else if (b0 >= 0xF0 && b0 <= 0xF4) { sz = 4; v = b0 & 0x07; if (b0 == 0xF0) lo = 0x90; if (b0 == 0xF4) hi = 0x8F; }
        bool ok = sz > 0 && n >= (size_t)sz && u[i + 1] >= lo && u[i + 1] <= hi;
        if (ok) {
            v = (v << 6) | (u[i + 1] & 0x3F);
            for (int k = 2; k < sz; k++) {
                if (u[i + k] < 0x80 || u[i + k] > 0xBF) { ok = false; break; }
                v = (v << 6) | (u[i + k] & 0x3F);
            }
        }
        if (!ok) throw ParseError{"invalid UTF-8", whole_.substr(i)};
        *r = v;
        return (size_t)sz;
    }

    // (?i) folding: ASCII orbits (plus U+017F and U+212A which fold with s and k)
    void add_range(RuneSet& set, uint32_t lo, uint32_t hi, int flags) const {
        set.push_back({lo, hi});
        if (!(flags & fFold)) return;
        if (lo <= 0x41 && hi >= 0x1E943) return;  // appendFoldedRange: already full
        for (uint32_t r = lo; r <= hi && r < 0x80; r++) {
            if (r >= 'a' && r <= 'z') set.push_back({r - 32, r - 32});
            if (r >= 'A' && r <= 'Z') set.push_back({r + 32, r + 32});
            if (r == 'k' || r == 'K') set.push_back({0x212A, 0x212A});
            if (r == 's' || r == 'S') set.push_back({0x17F, 0x17F});
        }
        uint32_t a = std::max<uint32_t>(lo, 0x80);
        if (a <= hi && a <= 0x1E943) throw Unsupported{};  // non-ASCII case orbits
    }

    void literal(uint32_t r) {
        Node* n = make(kLit);
        add_range(n->set, r, r, flags_);
        push(n);
    }

    void collapse_concat() {
        size_t i = stack_.size();
        while (i > 0 && stack_[i - 1]->op < kLeftParen) i--;
        size_t cnt = stack_.size() - i;
        Node* r;
        if (cnt == 0) r = make(kEmpty);
        else if (cnt == 1) r = stack_[i];
        else {
            r = make(kConcat);
            r->sub.assign(stack_.begin() + (long)i, stack_.end());
        }
        stack_.resize(i);
        push(r);
    }

    void collapse_alt() {
        size_t i = stack_.size();
        while (i > 0 && stack_[i - 1]->op != kLeftParen) i--;
        std::vector<Node*> alts;
        for (size_t k = i; k < stack_.size(); k++)
            if (stack_[k]->op != kVerticalBar) alts.push_back(stack_[k]);
        Node* r;
        if (alts.size() == 1) r = alts[0];
        else {
            r = make(kAlt);
            r->sub = alts;
        }
        stack_.resize(i);
        push(r);
    }

    static bool repeat_ok(const Node* re, int n) {
        if (re->op == kRepeat) {
            int m = re->max;
            if (m == 0) return true;
            if (m < 0) m = re->min;
            if (m > n) return false;
            if (m > 0) n /= m;
        }
        for (const Node* s : re->sub)
            if (!repeat_ok(s, n)) return false;
        return true;
    }

    // {n} {n,} {n,m}; Go parseInt: no leading zeros, >= 1e8 -> -1
    bool parse_int(size_t* i, int* v) const {
        const std::string& s = whole_;
        size_t k = *i;
        if (k >= s.size() || s[k] < '0' || s[k] > '9') return false;
        if (s.size() - k >= 2 && s[k] == '0' && s[k + 1] >= '0' && s[k + 1] <= '9') return false;
        size_t st = k;
        while (k < s.size() && s[k] >= '0' && s[k] <= '9') k++;
        int x = 0;
        for (size_t j = st; j < k; j++) {
            if (x >= 100000000) { x = -1; break; }
            x = x * 10 + (s[j] - '0');
        }
        *v = x;
        *i = k;
        return true;
    }
    bool parse_repeat(size_t i, int* mn, int* mx, size_t* end) const {
        const std::string& s = whole_;
        size_t k = i + 1;
        if (!parse_int(&k, mn)) return false;
        if (k >= s.size()) return false;
        if (s[k] != ',') *mx = *mn;
        else {
            k++;
            if (k >= s.size()) return false;
            if (s[k] == '}') *mx = -1;
            else {
                if (!parse_int(&k, mx)) return false;
                if (*mx < 0) *mn = -1;
            }
        }
        if (k >= s.size() || s[k] != '}') return false;
        *end = k + 1;
        return true;
    }

    static int unhex(uint32_t c) {
        if (c >= '0' && c <= '9') return (int)(c - '0');
        if (c >= 'a' && c <= 'f') return (int)(c - 'a' + 10);
        if (c >= 'A' && c <= 'F') return (int)(c - 'A' + 10);
        return -1;
    }

    // parseEscape at s[i] == '\\'; returns index after the escape
    size_t parse_escape(size_t i, uint32_t* out) const {
        const std::string& s = whole_;
        if (i + 1 >= s.size()) throw ParseError{"trailing backslash at end of expression", ""};
        uint32_t c;
        size_t p = i + 1;
        p += next_rune(p, &c);
        switch (c) {
            default:
                if (c < 0x80 && !((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'))) {
                    *out = c;
                    return p;
                }
                break;
            case '1': case '2': case '3': case '4': case '5': case '6': case '7':
                if (p >= s.size() || s[p] < '0' || s[p] > '7') break;  // backreference
                // fallthrough
            case '0': {
                uint32_t r = c - '0';
                for (int k = 1; k < 3; k++) {
                    if (p >= s.size() || s[p] < '0' || s[p] > '7') break;
                    r = r * 8 + (uint32_t)(s[p] - '0');
                    p++;
                }
                *out = r;
                return p;
            }
            case 'x': {
                if (p >= s.size()) break;
                uint32_t d;
                p += next_rune(p, &d);
                if (d == '{') {
                    int nhex = 0;
                    uint32_t r = 0;
                    for (;;) {
                        if (p >= s.size()) goto bad;
                        p += next_rune(p, &d);
                        if (d == '}') break;
                        int v = unhex(d);
                        if (v < 0) goto bad;
                        r = r * 16 + (uint32_t)v;
                        if (r > kMaxRune) goto bad;
                        nhex++;
                    }
                    if (nhex == 0) goto bad;
                    *out = r;
                    return p;
                }
                int x = unhex(d);
                uint32_t e = 0xFFFD;
                if (p < s.size()) p += next_rune(p, &e);
                int y = unhex(e);
                if (x < 0 || y < 0) break;
                *out = (uint32_t)(x * 16 + y);
                return p;
            }
            case 'a': *out = 7; return p;
            case 'f': *out = 12; return p;
            case 'n': *out = 10; return p;
            case 'r': *out = 13; return p;
            case 't': *out = 9; return p;
            case 'v': *out = 11; return p;
        }
    bad:
        throw ParseError{"invalid escape sequence", s.substr(i, p - i)};
    }

    // Perl classes \d \s \w and negations (ASCII)
    bool perl_class(size_t i, RuneSet* set, size_t* end) const {
        const std::string& s = whole_;
        if (i + 1 >= s.size() || s[i] != '\\') return false;
        char k = s[i + 1];
        bool neg = k == 'D' || k == 'S' || k == 'W';
        char l = neg ? (char)(k + 32) : k;
        RuneSet g;
        if (l == 'd') g = {{'0', '9'}};
        else if (l == 's') g = {{'\t', '\n'}, {'\f', '\r'}, {' ', ' '}};
        else if (l == 'w') g = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};
        else return false;
        append_group(set, g, neg);
        *end = i + 2;
        return true;
    }

    void append_group(RuneSet* set, const RuneSet& g, bool neg) const {
        RuneSet t;
        for (const Range& r : g) add_range(t, r.lo, r.hi, flags_);
        if (neg) t = negate(t);
        set->insert(set->end(), t.begin(), t.end());
    }

    // [:name:] inside a class; returns 0 when not one
    size_t named_class(size_t i, RuneSet* set) const {
        const std::string& s = whole_;
        if (s.size() - i <= 2 || s[i] != '[' || s[i + 1] != ':') return 0;
        size_t e = s.find(":]", i + 2);
        if (e == std::string::npos) return 0;
        std::string name = s.substr(i, e + 2 - i);
        bool neg = false;
        std::string key = name;
        if (key.size() > 3 && key[2] == '^') {
            neg = true;
            key.erase(2, 1);
        }
        static const std::map<std::string, RuneSet> groups = {
            {"[:alnum:]", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}},
            {"[:alpha:]", {{'A', 'Z'}, {'a', 'z'}}},
            {"[:ascii:]", {{0, 0x7F}}},
            {"[:blank:]", {{'\t', '\t'}, {' ', ' '}}},
            {"[:cntrl:]", {{0, 0x1F}, {0x7F, 0x7F}}},
            {"[:digit:]", {{'0', '9'}}},
            {"[:graph:]", {{'!', '~'}}},
            {"[:lower:]", {{'a', 'z'}}},
            {"[:print:]", {{' ', '~'}}},
            {"[:punct:]", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}},
            {"[:space:]", {{'\t', '\r'}, {' ', ' '}}},
            {"[:upper:]", {{'A', 'Z'}}},
            {"[:word:]", {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}},
            {"[:xdigit:]", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}},
        };
        auto it = groups.find(key);
        if (it == groups.end()) throw ParseError{"invalid character class range", name};
        append_group(set, it->second, neg);
        return e + 2 - i;
    }

    size_t class_char(size_t i, uint32_t* r) const {
        if (i >= whole_.size()) throw ParseError{"missing closing ]", whole_};
        if (whole_[i] == '\\') return parse_escape(i, r);
        return i + next_rune(i, r);
    }

    size_t parse_class(size_t start) {
        const std::string& s = whole_;
        size_t i = start + 1;
        Node* nd = make(kLit);
        bool neg = false;
        if (i < s.size() && s[i] == '^') {
            neg = true;  // ClassNL: '\n' is not excluded
            i++;
        }
        bool first = true;
        while (i >= s.size() || s[i] != ']' || first) {
            first = false;
            if (i < s.size() && s.size() - i > 2 && s[i] == '[' && s[i + 1] == ':') {
                size_t k = named_class(i, &nd->set);
                if (k) { i += k; continue; }
            }
            if (i + 1 < s.size() && s[i] == '\\' && (s[i + 1] == 'p' || s[i + 1] == 'P')) throw Unsupported{};
            size_t e;
            if (perl_class(i, &nd->set, &e)) { i = e; continue; }
            size_t rng = i;
            uint32_t lo, hi;
            i = class_char(i, &lo);
            hi = lo;
            if (s.size() >= i + 2 && s[i] == '-' && s[i + 1] != ']') {
                i = class_char(i + 1, &hi);
                if (hi < lo) throw ParseError{"invalid character class range", s.substr(rng, i - rng)};
            }
            add_range(nd->set, lo, hi, flags_);
        }
        i++;
        normalize(nd->set);
        if (neg) nd->set = negate(nd->set);
        push(nd);
        return i;
    }

    size_t perl_flags(size_t i) {
        const std::string& s = whole_;
        if (s.size() - i > 4 && s[i + 2] == 'P' && s[i + 3] == '<') {
            size_t e = s.find('>', i);
            if (e == std::string::npos) throw ParseError{"invalid named capture", s.substr(i)};
            std::string name = s.substr(i + 4, e - i - 4);
            bool ok = !name.empty();
            for (char ch : name) ok = ok && is_word_byte((unsigned char)ch);
            if (!ok) throw ParseError{"invalid named capture", s.substr(i, e + 1 - i)};
            Node* lp = make(kLeftParen);
            lp->cap = ++ncap_;
            push(lp);
            return e + 1;
        }
        size_t p = i + 2;
        int fl = flags_;
        int sign = 1;
        bool saw = false;
        while (p < s.size()) {
            uint32_t c;
            p += next_rune(p, &c);
            switch (c) {
                default: goto bad;
                case 'i': fl |= fFold; saw = true; break;
                case 'm': fl &= ~fOneLine; saw = true; break;
                case 's': fl |= fDotNL; saw = true; break;
                case 'U': fl |= fNonGreedy; saw = true; break;
                case '-':
                    if (sign < 0) goto bad;
                    sign = -1;
                    fl = ~fl;
                    saw = false;
                    break;
                case ':': case ')':
                    if (sign < 0) {
                        if (!saw) goto bad;
                        fl = ~fl;
                    }
                    if (c == ':') push(make(kLeftParen));
                    flags_ = fl;
                    return p;
            }
        }
    bad:
        throw ParseError{"invalid or unsupported Perl syntax", s.substr(i, p - i)};
    }

    size_t parse_backslash(size_t i) {
        const std::string& s = whole_;
        if (i + 1 < s.size()) {
            char k = s[i + 1];
            int a = k == 'A' ? kBOT : k == 'b' ? kWB : k == 'B' ? kNWB : k == 'z' ? kEOT : 0;
            if (a) {
                Node* n = make(kAssert);
                n->bits = a;
                push(n);
                return i + 2;
            }
            if (k == 'C') throw ParseError{"invalid escape sequence", "\\C"};
            if (k == 'Q') {
                size_t e = s.find("\\E", i + 2);
                size_t stop = e == std::string::npos ? s.size() : e;
                size_t p = i + 2;
                while (p < stop) {
                    uint32_t r;
                    p += next_rune(p, &r);
                    literal(r);
                }
                return e == std::string::npos ? s.size() : e + 2;
            }
            if (k == 'p' || k == 'P') throw Unsupported{};
        }
        Node* cn = make(kLit);
        size_t e;
        if (perl_class(i, &cn->set, &e)) {
            push(cn);
            return e;
        }
        uint32_t r;
        size_t p = parse_escape(i, &r);
        literal(r);
        return p;
    }
};

// ---- NFA ----------------------------------------------------------------------------
enum IOp { iRune, iEmpty, iSplit, iNop, iMatch };
struct Inst {
    IOp op;
    int x = -1, y = -1;
    int bits = 0;
    int set = -1;  // index into the distinct rune-set table
};

struct Prog {
    std::vector<Inst> inst;
    std::vector<RuneSet> sets;
    std::map<std::vector<uint64_t>, int> set_ids;
    int start = 0;
    bool too_big = false;

    int emit(IOp op) {
        if (inst.size() > 300000) too_big = true;
        inst.push_back(Inst{op});
        return (int)inst.size() - 1;
    }
    int set_id(RuneSet s) {
        normalize(s);
        std::vector<uint64_t> key;
        for (const Range& r : s) key.push_back(((uint64_t)r.lo << 32) | r.hi);
        auto it = set_ids.find(key);
        if (it != set_ids.end()) return it->second;
        sets.push_back(s);
        set_ids[key] = (int)sets.size() - 1;
        return (int)sets.size() - 1;
    }
};

struct Frag {
    int start;
    std::vector<int> out;  // pc*2 + (0: x, 1: y)
};

void patch(Prog& p, Frag& f, int to) {
    for (int o : f.out) {
        if (o & 1) p.inst[o >> 1].y = to;
        else p.inst[o >> 1].x = to;
    }
    f.out.clear();
}

Frag compile_node(Prog& p, const Node* n);

Frag nop(Prog& p) {
    int pc = p.emit(iNop);
    return Frag{pc, {pc * 2}};
}

Frag star_of(Prog& p, Frag s) {
    int sp = p.emit(iSplit);
    p.inst[sp].x = s.start;
    patch(p, s, sp);
    return Frag{sp, {sp * 2 + 1}};
}

Frag concat2(Prog& p, Frag a, Frag b) {
    patch(p, a, b.start);
    a.out = std::move(b.out);
    return a;
}

Frag compile_node(Prog& p, const Node* n) {
    if (p.too_big) return nop(p);
    switch (n->op) {
        case kLit: {
            int pc = p.emit(iRune);
            p.inst[pc].set = p.set_id(n->set);
            return Frag{pc, {pc * 2}};
        }
        case kEmpty: return nop(p);
        case kAssert: {
            int pc = p.emit(iEmpty);
            p.inst[pc].bits = n->bits;
            return Frag{pc, {pc * 2}};
        }
        case kCapture: return compile_node(p, n->sub[0]);
        case kConcat: {
            Frag f = compile_node(p, n->sub[0]);
            for (size_t k = 1; k < n->sub.size(); k++) f = concat2(p, f, compile_node(p, n->sub[k]));
            return f;
        }
        case kAlt: {
            Frag acc = compile_node(p, n->sub.back());
            for (int k = (int)n->sub.size() - 2; k >= 0; k--) {
                Frag g = compile_node(p, n->sub[(size_t)k]);
                int sp = p.emit(iSplit);
                p.inst[sp].x = g.start;
                p.inst[sp].y = acc.start;
                g.out.insert(g.out.end(), acc.out.begin(), acc.out.end());
                acc = Frag{sp, g.out};
            }
            return acc;
        }
        case kStar: return star_of(p, compile_node(p, n->sub[0]));
        case kPlus: {
            Frag s = compile_node(p, n->sub[0]);
            int sp = p.emit(iSplit);
            p.inst[sp].x = s.start;
            patch(p, s, sp);
            return Frag{s.start, {sp * 2 + 1}};
        }
        case kQuest: {
            Frag s = compile_node(p, n->sub[0]);
            int sp = p.emit(iSplit);
            p.inst[sp].x = s.start;
            s.out.push_back(sp * 2 + 1);
            return Frag{sp, s.out};
        }
        case kRepeat: {
            if (n->max == 0) return nop(p);
            bool have = false;
            Frag acc{0, {}};
            for (int k = 0; k < n->min; k++) {
                Frag g = compile_node(p, n->sub[0]);
                acc = have ? concat2(p, acc, g) : g;
                have = true;
            }
            if (n->max < 0) {
                Frag g = star_of(p, compile_node(p, n->sub[0]));
                return have ? concat2(p, acc, g) : g;
            }
            bool have_tail = false;
            Frag tail{0, {}};
            for (int k = 0; k < n->max - n->min; k++) {
                Frag g = compile_node(p, n->sub[0]);
                if (have_tail) g = concat2(p, g, tail);
                int sp = p.emit(iSplit);
                p.inst[sp].x = g.start;
                g.out.push_back(sp * 2 + 1);
                tail = Frag{sp, g.out};
                have_tail = true;
            }
            if (!have_tail) return acc;  // x{n}: no optional copies
            if (!have) return tail;
            return concat2(p, acc, tail);
        }
        default: return nop(p);
    }
}

// ---- DFA ------------------------------------------------------------------------------
// previous-rune kinds and next-rune kinds for syntax.EmptyOpContext
enum { kPrevBOT = 0, kPrevWord = 1, kPrevNL = 2, kPrevOther = 3 };
enum { kNextWord = 0, kNextNL = 1, kNextOther = 2, kNextEOT = 3 };

int empty_ctx(int prev, int next) {
    int op = kNWB;
    int boundary = 0;
    if (prev == kPrevWord) boundary = 1;
    else if (prev == kPrevNL) op |= kBOL;
    else if (prev == kPrevBOT) op |= kBOT | kBOL;
    if (next == kNextWord) boundary ^= 1;
    else if (next == kNextNL) op |= kEOL;
    else if (next == kNextEOT) op |= kEOT | kEOL;
    if (boundary) op ^= (kWB | kNWB);
    return op;
}

struct Closure {
    std::vector<int> runes;  // rune instructions reached
    bool match = false;
};

void closure(const Prog& p, const std::vector<int>& seeds, int ctx, Closure* c, std::vector<uint8_t>& mark) {
    std::fill(mark.begin(), mark.end(), 0);
    std::vector<int> st(seeds.rbegin(), seeds.rend());
    c->runes.clear();
    c->match = false;
    while (!st.empty()) {
        int q = st.back();
        st.pop_back();
        if (q < 0 || mark[(size_t)q]) continue;
        mark[(size_t)q] = 1;
        const Inst& in = p.inst[(size_t)q];
        switch (in.op) {
            case iMatch: c->match = true; break;
            case iRune: c->runes.push_back(q); break;
            case iNop: st.push_back(in.x); break;
            case iSplit: st.push_back(in.y); st.push_back(in.x); break;
            case iEmpty:
                if ((in.bits & ~ctx) == 0) st.push_back(in.x);
                break;
        }
    }
    std::sort(c->runes.begin(), c->runes.end());
}

bool set_has(const RuneSet& s, uint32_t r) {
    auto it = std::upper_bound(s.begin(), s.end(), r, [](uint32_t v, const Range& x) { return v < x.lo; });
    if (it == s.begin()) return false;
    --it;
    return r >= it->lo && r <= it->hi;
}

RegexStatus build_dfa(const Prog& p, RegexDfa* out) {
    // 1. alphabet partition
    std::vector<uint32_t> cuts = {0, 0x80, '\n', '\n' + 1, '0', '9' + 1, 'A', 'Z' + 1, '_', '_' + 1, 'a', 'z' + 1, kMaxRune + 1};
    for (const RuneSet& s : p.sets)
        for (const Range& r : s) {
            cuts.push_back(r.lo);
            cuts.push_back(r.hi + 1);
        }
    std::sort(cuts.begin(), cuts.end());
    cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
    struct Interval {
        uint32_t lo, hi;
        int cls;
    };
    std::vector<Interval> iv;
    std::map<std::vector<uint64_t>, int> sig_ids;
    std::vector<int> class_next_kind;
    std::vector<uint32_t> class_rep;  // a representative rune per class
    for (size_t k = 0; k + 1 < cuts.size(); k++) {
        uint32_t lo = cuts[k], hi = cuts[k + 1] - 1;
        if (lo > kMaxRune) break;
        std::vector<uint64_t> sig((p.sets.size() + 63) / 64 + 1, 0);
        for (size_t si = 0; si < p.sets.size(); si++)
            if (set_has(p.sets[si], lo)) sig[si / 64] |= 1ull << (si % 64);
        int kind = is_word_byte(lo) && lo < 0x80 ? kNextWord : lo == '\n' ? kNextNL : kNextOther;
        sig.back() = (uint64_t)kind;
        auto it = sig_ids.find(sig);
        int cls;
        if (it == sig_ids.end()) {
            cls = (int)class_rep.size();
            sig_ids[sig] = cls;
            class_rep.push_back(lo);
            class_next_kind.push_back(kind);
        } else {
            cls = it->second;
        }
        iv.push_back({lo, hi, cls});
    }
    const int K = (int)class_rep.size();
    if (K > (int)kMaxDfaClasses) return RX_UNSUPPORTED;
    out->n_classes = (uint32_t)K;
    for (const Interval& v : iv) {
        for (uint32_t r = v.lo; r <= v.hi && r < 0x80; r++) out->ascii_class[r] = (uint8_t)v.cls;
        if (v.hi >= 0x80) {
            uint32_t lo = std::max<uint32_t>(v.lo, 0x80);
            if (!out->ranges.empty() && out->ranges.back().cls == (uint32_t)v.cls && out->ranges.back().hi + 1 == lo)
                out->ranges.back().hi = v.hi;
            else
                out->ranges.push_back(RuneRange{lo, v.hi, (uint32_t)v.cls, 0});
        }
    }
    // per class, which rune instructions accept it
    // 2. subset construction
    std::map<std::pair<std::vector<int>, int>, uint32_t> ids;
    std::vector<std::pair<std::vector<int>, int>> states;
    std::vector<uint8_t> mark(p.inst.size(), 0);
    auto intern = [&](std::vector<int> s, int prev) -> uint32_t {
        auto key = std::make_pair(std::move(s), prev);
        auto it = ids.find(key);
        if (it != ids.end()) return it->second;
        uint32_t id = (uint32_t)states.size();
        ids[key] = id;
        states.push_back(key);
        return id;
    };
    const uint32_t kMatch = 0;  // state 0 = absorbing match
    states.push_back({{-1}, -1});
    out->start = intern({}, kPrevBOT);
    std::vector<uint16_t>& tr = out->trans;
    std::vector<uint8_t>& eot = out->eot;
    Closure cl;
    for (uint32_t s = 0; s < states.size(); s++) {
        if (states.size() > kMaxDfaStates) return RX_UNSUPPORTED;
        tr.resize((size_t)(s + 1) * (size_t)K, 0);
        eot.resize(s + 1, 0);
        if (s == kMatch) {
            for (int c = 0; c < K; c++) tr[(size_t)s * K + c] = (uint16_t)kMatch;
            eot[s] = 1;
            continue;
        }
        const std::vector<int> threads = states[s].first;
        const int prev = states[s].second;
        std::vector<int> seeds = threads;
        seeds.push_back(p.start);
        // end of text
        closure(p, seeds, empty_ctx(prev, kNextEOT), &cl, mark);
        eot[s] = cl.match ? 1 : 0;
        for (int c = 0; c < K; c++) {
            const int nk = class_next_kind[(size_t)c];
            closure(p, seeds, empty_ctx(prev, nk), &cl, mark);
            uint32_t target;
            if (cl.match) {
                target = kMatch;
            } else {
                std::vector<int> nxt;
                const uint32_t rep = class_rep[(size_t)c];
                for (int pc : cl.runes) {
                    const Inst& in = p.inst[(size_t)pc];
                    if (set_has(p.sets[(size_t)in.set], rep)) nxt.push_back(in.x);
                }
                std::sort(nxt.begin(), nxt.end());
                nxt.erase(std::unique(nxt.begin(), nxt.end()), nxt.end());
                int pk = nk == kNextWord ? kPrevWord : nk == kNextNL ? kPrevNL : kPrevOther;
                target = intern(nxt, pk);
            }
            if (target > 0xFFFF) return RX_UNSUPPORTED;
            tr[(size_t)s * K + c] = (uint16_t)target;
        }
    }
    out->n_states = (uint32_t)states.size();
    out->match_state = kMatch;
    tr.resize((size_t)out->n_states * K);
    eot.resize(out->n_states);
    return RX_OK;
}

}  // namespace

RegexStatus compile_go_regex(const std::string& pat, RegexDfa* out, std::string* err) {
    try {
        Parser ps(pat);
        Node* root = ps.parse();
        Prog prog;
        Frag f = compile_node(prog, root);
        int m = prog.emit(iMatch);
        patch(prog, f, m);
        prog.start = f.start;
        if (prog.too_big) {
            if (err) *err = "regexp too large for the device compiler";
            return RX_UNSUPPORTED;
        }
        RegexStatus st = build_dfa(prog, out);
        if (st != RX_OK && err) *err = "regexp DFA exceeds the device limits";
        return st;
    } catch (const ParseError& e) {
        if (err) *err = "error parsing regexp: " + e.code + ": `" + e.expr + "`";
        return RX_ERROR;
    } catch (const Unsupported&) {
        if (err) *err = "regexp syntax not compiled for the device (\\p{..} or non-ASCII case folding)";
        return RX_UNSUPPORTED;
    }
}

}  // namespace ajx
