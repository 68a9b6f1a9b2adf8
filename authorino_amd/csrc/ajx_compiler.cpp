// ajx_compiler.cpp — jsonexp tree -> ruleset blob (see ajx_blob.h for the layout).
#include "ajx_compiler.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>

#include "ajx_regex.h"

namespace ajx {

namespace {

uint32_t fnv1a(const std::string& s) {
    uint32_t h = 2166136261u;
    for (unsigned char c : s) {
        h ^= c;
        h *= 16777619u;
    }
    return h;
}

// gjson parseUint on the raw array-context part; -1 when it can never equal an index
int32_t array_index_of(const std::string& raw) {
    if (raw.empty()) return -1;
    uint64_t v = 0;
    for (char c : raw) {
        if (c < '0' || c > '9') return -1;
        v = v * 10 + (uint64_t)(c - '0');  // wraps like Go's uint64
    }
    int64_t iv = (int64_t)v;  // int(n)
    if (iv < 0 || iv > 0x7fffffff) return -1;
    return (int32_t)iv;
}

}  // namespace

bool split_selector(const std::string& p, std::vector<PathComponent>* out) {
    out->clear();
    const size_t n = p.size();
    // gjson.Get special forms: modifiers '@', static '!', multipaths '[' '{', JSON lines '..'
    if (n > 1 && (p[0] == '@' || p[0] == '!' || p[0] == '[' || p[0] == '{')) return false;
    if (n >= 2 && p[0] == '.' && p[1] == '.') return false;
    for (size_t i = 0; i < n; i++) {
        char c = p[i];
        if (c == '\\') {
            i++;
            if (i < n && (p[i] == '|' || p[i] == '#')) return false;  // special in array context
            continue;
        }
        if (c == '|' || c == '*' || c == '?') return false;
        // '#' starts gjson's array forms: "#.key" (a JSON array of each element's key), "#("
        // / "#[" queries — not compiled; a last part "#" is the element count (kArrCount)
        if (c == '#' && i + 1 < n && (p[i + 1] == '(' || p[i + 1] == '[')) return false;
        if (c == '.' && i + 1 < n && (p[i + 1] == '@' || p[i + 1] == '[' || p[i + 1] == '{')) return false;
    }
    // parseObjectPath repeatedly on the remainder
    size_t pos = 0;
    bool list_seen = false;
    for (;;) {
        PathComponent comp;
        std::string part;
        size_t i = pos;
        bool more = false, escaped = false;
        size_t next = n;
        for (; i < n; i++) {
            char c = p[i];
            if (c == '.') {
                more = true;
                next = i + 1;
                break;
            }
            if (c == '\\') {
                escaped = true;
                i++;
                if (i < n) part.push_back(p[i]);  // a trailing lone backslash is dropped
                continue;
            }
            part.push_back(c);
        }
        // array context (parseArrayPath): raw text up to the first '.', no escape handling
        size_t dot = p.find('.', pos);
        std::string raw = p.substr(pos, (dot == std::string::npos ? n : dot) - pos);
        comp.key = part;
        comp.array_index = raw == "#" ? (more ? kArrList : kArrCount)
                           : escaped && raw.find('\\') != std::string::npos ? -1 : array_index_of(raw);
        // "#." lists: the key path after the list part holds no '#' (gjson would run a
        // nested '#' form per element); other parts with a '#' never match an element
        // (parseArrayPath's arrch without a count or a list)
        if (list_seen && raw.find('#') != std::string::npos) return false;
        if (comp.array_index == kArrList) list_seen = true;
        out->push_back(comp);
        if (!more) break;
        pos = next;
    }
    return out->size() <= kMaxComponents;
}

namespace {

// ---- gjson modifier chains (pkg/json/json.go:161-264) ---------------------------------
struct ModSpec {
    uint8_t kind = 0, variant = 0;
    std::string a, b;
    uint32_t pos = 0;
};

// gjson's squash of a JSON argument at s[i] ('{' '[' '"'): its end (exclusive), or npos
size_t squash_arg(const std::string& s, size_t i) {
    if (s[i] == '"') {
        for (size_t k = i + 1; k < s.size(); k++) {
            if (s[k] == '\\') { k++; continue; }
            if (s[k] == '"') return k + 1;
        }
        return std::string::npos;
    }
    int depth = 0;
    for (size_t k = i; k < s.size(); k++) {
        const char c = s[k];
        if (c == '"') {
            for (k++; k < s.size(); k++) {
                if (s[k] == '\\') { k++; continue; }
                if (s[k] == '"') break;
            }
            if (k >= s.size()) return std::string::npos;
            continue;
        }
        if (c == '{' || c == '[' || c == '(') depth++;
        if (c == '}' || c == ']' || c == ')') {
            if (--depth == 0) return k + 1;
        }
    }
    return std::string::npos;
}

void put_utf8(uint32_t r, std::string* o) {
    if (r > 0x10FFFF || (r >= 0xD800 && r < 0xE000)) r = 0xFFFD;
    if (r < 0x80) o->push_back((char)r);
    else if (r < 0x800) { o->push_back((char)(0xC0 | (r >> 6))); o->push_back((char)(0x80 | (r & 0x3F))); }
    else if (r < 0x10000) {
        o->push_back((char)(0xE0 | (r >> 12))); o->push_back((char)(0x80 | ((r >> 6) & 0x3F)));
        o->push_back((char)(0x80 | (r & 0x3F)));
    } else {
        o->push_back((char)(0xF0 | (r >> 18))); o->push_back((char)(0x80 | ((r >> 12) & 0x3F)));
        o->push_back((char)(0x80 | ((r >> 6) & 0x3F))); o->push_back((char)(0x80 | (r & 0x3F)));
    }
}

// a JSON string token at s[i] ('"') -> its unescaped text; false if not well formed
bool json_string_at(const std::string& s, size_t* i, std::string* out) {
    out->clear();
    size_t k = *i + 1;
    auto hex4 = [&](size_t at, uint32_t* v) {
        if (at + 4 > s.size()) return false;
        uint32_t x = 0;
        for (size_t j = 0; j < 4; j++) {
            const char c = s[at + j];
            x <<= 4;
            if (c >= '0' && c <= '9') x |= (uint32_t)(c - '0');
            else if ((c | 0x20) >= 'a' && (c | 0x20) <= 'f') x |= (uint32_t)((c | 0x20) - 'a' + 10);
            else return false;
        }
        *v = x;
        return true;
    };
    for (; k < s.size(); k++) {
        const char c = s[k];
        if (c == '"') { *i = k + 1; return true; }
        if ((unsigned char)c < 0x20) return false;
        if (c != '\\') { out->push_back(c); continue; }
        if (++k >= s.size()) return false;
        switch (s[k]) {
            case '"': out->push_back('"'); break;
            case '\\': out->push_back('\\'); break;
            case '/': out->push_back('/'); break;
            case 'b': out->push_back('\b'); break;
            case 'f': out->push_back('\f'); break;
            case 'n': out->push_back('\n'); break;
            case 'r': out->push_back('\r'); break;
            case 't': out->push_back('\t'); break;
            case 'u': {
                uint32_t r;
                if (!hex4(k + 1, &r)) return false;
                k += 4;
                if (r >= 0xD800 && r < 0xDC00 && k + 6 < s.size() + 0 && s[k + 1] == '\\' && s[k + 2] == 'u') {
                    uint32_t r2;
                    if (hex4(k + 3, &r2) && r2 >= 0xDC00 && r2 < 0xE000) {
                        r = (((r - 0xD800) << 10) | (r2 - 0xDC00)) + 0x10000;
                        k += 6;
                    }
                }
                put_utf8(r, out);
                break;
            }
            default: return false;
        }
    }
    return false;
}

// the members of a JSON object argument ({"sep":"@","pos":1}): key -> ('s', text) for
// strings, ('n', raw) for numbers, ('o', raw) otherwise; false if not a plain object
bool object_members(const std::string& a, std::vector<std::pair<std::string, std::pair<char, std::string>>>* m) {
    size_t i = 0;
    auto ws = [&] { while (i < a.size() && (unsigned char)a[i] <= ' ') i++; };
    ws();
    if (i >= a.size() || a[i] != '{') return false;
    i++;
    ws();
    if (i < a.size() && a[i] == '}') return true;
    for (;;) {
        ws();
        std::string key, val;
        if (i >= a.size() || a[i] != '"' || !json_string_at(a, &i, &key)) return false;
        ws();
        if (i >= a.size() || a[i] != ':') return false;
        i++;
        ws();
        if (i >= a.size()) return false;
        char kind;
        if (a[i] == '"') {
            if (!json_string_at(a, &i, &val)) return false;
            kind = 's';
        } else {
            const size_t b = i;
            if (a[i] == '{' || a[i] == '[') {
                const size_t e = squash_arg(a, i);
                if (e == std::string::npos) return false;
                i = e;
                kind = 'o';
            } else {
                while (i < a.size() && a[i] != ',' && a[i] != '}' && (unsigned char)a[i] > ' ') i++;
                kind = (a[b] == '-' || (a[b] >= '0' && a[b] <= '9')) ? 'n' : 'o';
            }
            val = a.substr(b, i - b);
        }
        m->push_back({key, {kind, val}});
        ws();
        if (i < a.size() && a[i] == ',') { i++; continue; }
        if (i < a.size() && a[i] == '}') return true;
        return false;
    }
}

// Split `path` into a plain base path and a chain of the reference's modifiers, as
// gjson.Get runs it: parseObjectPath pipes at '|' or at '.' before '@'
// (isDotPiperChar); execModifier reads a name up to ':' '|' '.', a JSON argument by
// squash or a plain one up to the next '|'; the result goes on through '|' or '.'.
// 0: no modifier; 1: base + mods; -1: a form the device does not evaluate (other
// modifiers, a path after a modifier, arguments outside the supported ones).
int split_modifiers(const std::string& path, std::string* base, std::vector<ModSpec>* mods) {
    mods->clear();
    size_t cut = std::string::npos;
    for (size_t i = 0; i + 1 < path.size(); i++) {
        if (path[i] == '\\') { i++; continue; }
        // a modifier, or a pipe: `a|b` is Get(Get(json, a).Raw, b) (a path after the cut)
        if (((path[i] == '.' || path[i] == '|') && path[i + 1] == '@') || path[i] == '|') { cut = i; break; }
    }
    if (cut == std::string::npos || cut == 0) return 0;
    *base = path.substr(0, cut);
    size_t i = cut + 1;  // at '@'
    while (i < path.size()) {
        if (path[i] != '@') {
            // a path after a modifier (`...|@fromstr|request.object.kind`): gjson Gets it
            // from the modifier's output (Get: execModifier, then Get(rjson, path[1:])),
            // up to the next '|@' / '.@'
            size_t e = i;
            for (; e < path.size(); e++) {
                if (path[e] == '\\') { e++; continue; }
                if (path[e] == '|' || (path[e] == '.' && e + 1 < path.size() && path[e + 1] == '@')) break;
            }
            if (e > path.size()) e = path.size();
            ModSpec m;
            m.kind = M_PATH;
            m.a = path.substr(i, e - i);
            mods->push_back(m);
            if (e >= path.size()) break;
            i = e + 1;
            continue;
        }
        size_t k = i + 1;
        while (k < path.size() && path[k] != ':' && path[k] != '|' && path[k] != '.') k++;
        const std::string name = path.substr(i + 1, k - i - 1);
        std::string arg;
        bool has_args = false;
        size_t next = k;
        if (k < path.size() && path[k] == ':') {
            const size_t a = k + 1;
            has_args = a < path.size();
            if (has_args && (path[a] == '{' || path[a] == '[' || path[a] == '"')) {
                const size_t e = squash_arg(path, a);
                if (e == std::string::npos) return -1;
                arg = path.substr(a, e - a);
                next = e;
            } else {
                size_t e = path.find('|', a);
                if (e == std::string::npos) e = path.size();
                arg = path.substr(a, e - a);
                next = e;
            }
        }
        ModSpec m;
        if (name == "extract") {
            m.kind = M_EXTRACT;
            m.a = " ";
            m.pos = 0;
            std::vector<std::pair<std::string, std::pair<char, std::string>>> mem;
            if (has_args && !arg.empty() && arg[0] == '{') {
                if (!object_members(arg, &mem)) return -1;
                for (auto& kv : mem) {
                    if (kv.first == "sep") {
                        if (kv.second.first != 's') return -1;
                        m.a = kv.second.second;
                    } else if (kv.first == "pos") {
                        if (kv.second.first != 'n') return -1;
                        char* endp = nullptr;
                        const double v = std::strtod(kv.second.second.c_str(), &endp);
                        if (!endp || *endp || !(v >= 0) || v > 9007199254740991.0) return -1;
                        m.pos = (uint32_t)std::min<double>(std::trunc(v), 0xFFFFFFF0u);
                    }
                }
            } else if (has_args && !arg.empty() && arg[0] != '[' && arg[0] != '"') {
                // a scalar argument: gjson ForEach visits it with an empty key (defaults)
            } else if (has_args && !arg.empty()) {
                return -1;
            }
            if (m.a.empty()) return -1;  // strings.Split on "" splits into runes
        } else if (name == "replace") {
            m.kind = M_REPLACE;
            if (has_args && !arg.empty()) {
                std::vector<std::pair<std::string, std::pair<char, std::string>>> mem;
                if (arg[0] != '{' || !object_members(arg, &mem)) return -1;
                bool have_old = false;
                for (auto& kv : mem) {
                    if (kv.first == "old") {
                        if (kv.second.first != 's') return -1;
                        m.a = kv.second.second;
                        have_old = true;
                    } else if (kv.first == "new") {
                        if (kv.second.first != 's') return -1;
                        m.b = kv.second.second;
                    }
                }
                if (!have_old || m.a.empty()) return -1;  // ReplaceAll with "" inserts between runes
                m.variant = 1;
            }
        } else if (name == "case") {
            m.kind = M_CASE;
            m.variant = arg == "upper" ? 1 : arg == "lower" ? 2 : 0;
        } else if (name == "base64") {
            m.kind = M_BASE64;
            m.variant = arg == "encode" ? 1 : arg == "decode" ? 2 : 0;
        } else if (name == "strip") {
            m.kind = M_STRIP;
        } else if (name == "fromstr") {  // gjson v1.14.0 modFromStr
            m.kind = M_FROMSTR;
        } else {
            return -1;  // gjson's other built-ins (@this, @reverse, @tostr, ...) are not compiled
        }
        mods->push_back(m);
        if (next >= path.size()) break;
        if (path[next] != '|' && path[next] != '.') return -1;
        i = next + 1;
        if (i >= path.size()) return -1;
    }
    return mods->empty() ? -1 : 1;
}

struct NormNode {
    int kind;  // 0 = AND, 1 = OR, 2 = leaf pattern, 3 = const T, 4 = const F
    int pattern = -1;
    std::vector<NormNode> kids;
};

struct Builder {
    std::vector<uint8_t> blob;
    size_t align16() {
        while (blob.size() % 16) blob.push_back(0);
        return blob.size();
    }
    size_t append(const void* p, size_t n) {
        size_t off = blob.size();
        blob.resize(off + n);
        if (n) std::memcpy(blob.data() + off, p, n);
        return off;
    }
};

}  // namespace

namespace {
// the shape of one tree's fold code that tree_fold reads off the bitmaps: [open X,
// (pattern | open Y, pattern+, close)*, close], Y != X, pattern indices consecutive in code
// order (base, base + 1, ...), at most 64 of them
bool tree_fold_shape(const uint32_t* code, uint32_t n, TreeFold* f) {
    if (n < 3 || (code[n - 1] >> 24) != C_CLOSE) return false;
    const uint32_t outer = code[0] >> 24;
    if (outer != C_OPEN_AND && outer != C_OPEN_OR) return false;
    const uint32_t inner = outer == C_OPEN_AND ? C_OPEN_OR : C_OPEN_AND;
    uint32_t base = ~0u, next = 0, k = 1;
    uint64_t g_any = 0, g_in = 0, g_start = 0;
    auto take = [&](uint32_t w) {  // the next pattern in order
        const uint32_t p = w & 0xFFFFFFu;
        if (base == ~0u) {
            base = p;
            next = p;
        }
        if (p != next || p - base >= 64) return false;
        next++;
        return true;
    };
    while (k < n - 1) {
        const uint32_t op = code[k] >> 24;
        if (op == C_PAT) {
            if (!take(code[k])) return false;
            k++;
        } else if (op == inner) {
            k++;
            bool first = true;
            uint32_t lo_rel = 0;
            while (k < n - 1 && (code[k] >> 24) == C_PAT) {
                if (!take(code[k])) return false;
                if (first) lo_rel = (code[k] & 0xFFFFFFu) - base;
                first = false;
                k++;
            }
            if (first || k >= n - 1 || (code[k] >> 24) != C_CLOSE) return false;
            k++;
            const uint32_t hi_rel = next - base;
            const uint64_t m = (hi_rel >= 64 ? ~0ull : (1ull << hi_rel) - 1ull) & ~((1ull << lo_rel) - 1ull);
            g_in |= m;
            if (inner == C_OPEN_OR) g_any |= m;
            g_start |= 1ull << lo_rel;
        } else {
            return false;
        }
    }
    if (base == ~0u || next > kFastMaxPatterns) return false;  // (the kernels' bitmaps are 128 bits)
    f->base = base;
    f->n = next - base;
    f->shape = 1;
    f->any = outer == C_OPEN_OR ? 1u : 0u;
    f->g_any = g_any;
    f->g_in = g_in;
    f->g_start = g_start;
    return true;
}

int compile_core(const authjx_tree* tree, const std::vector<int32_t>& roots, bool forest, CompiledRuleset* out,
                 std::string* err, const std::vector<uint8_t>* kept = nullptr);
}

int compile_tree(const authjx_tree* tree, CompiledRuleset* out, std::string* err) {
    if (!tree) return AUTHJX_EINVAL;
    return compile_core(tree, {tree->root}, false, out, err);
}

// Several trees over the same documents as one ruleset: patterns and nodes concatenated
// in tree order (selectors shared by the trees share one trie path), one fold program per
// tree (RulesetHdr::pad1[0] = tree count, pad1[1] = offset of {code_begin, code_len}[]).
int compile_forest(const authjx_tree* trees, uint32_t n_trees, CompiledRuleset* out, std::string* err) {
    if (!trees || n_trees == 0) return AUTHJX_EINVAL;
    std::vector<authjx_pattern> pats;
    std::vector<authjx_node> nodes;
    std::vector<int32_t> roots;
    std::vector<uint8_t> kept;  // patterns of root-less trees: selectors a caller reads back
    for (uint32_t k = 0; k < n_trees; k++) {
        const authjx_tree& t = trees[k];
        if ((t.n_patterns && !t.patterns) || (t.n_nodes && !t.nodes) || t.root >= (int32_t)t.n_nodes)
            return AUTHJX_EINVAL;
        const int32_t po = (int32_t)pats.size(), no = (int32_t)nodes.size();
        pats.insert(pats.end(), t.patterns, t.patterns + t.n_patterns);
        kept.insert(kept.end(), t.n_patterns, t.root < 0 ? 1 : 0);
        for (uint32_t i = 0; i < t.n_nodes; i++) {
            authjx_node nd = t.nodes[i];
            if (nd.left >= (int32_t)t.n_nodes || nd.right >= (int32_t)t.n_nodes) return AUTHJX_EINVAL;
            if (nd.kind == AUTHJX_NODE_PATTERN && (nd.pattern < 0 || (uint32_t)nd.pattern >= t.n_patterns))
                return AUTHJX_EINVAL;
            if (nd.left >= 0) nd.left += no;
            if (nd.right >= 0) nd.right += no;
            if (nd.kind == AUTHJX_NODE_PATTERN) nd.pattern += po;
            nodes.push_back(nd);
        }
        roots.push_back(t.root < 0 ? -1 : t.root + no);
    }
    authjx_tree all{pats.data(), (uint32_t)pats.size(), nodes.data(), (uint32_t)nodes.size(), -1};
    return compile_core(&all, roots, true, out, err, &kept);
}

namespace {
int compile_core(const authjx_tree* tree, const std::vector<int32_t>& roots, bool forest, CompiledRuleset* out,
                 std::string* err, const std::vector<uint8_t>* kept) {
    const uint32_t np = tree->n_patterns, nn = tree->n_nodes;
    if ((np && !tree->patterns) || (nn && !tree->nodes)) return AUTHJX_EINVAL;
    for (int32_t rt : roots)
        if (rt >= (int32_t)nn) return AUTHJX_EINVAL;

    // ---- normalise the And/Or tree into n-ary fold nodes ----
    std::vector<int> visiting(nn, 0);
    bool bad = false;
    std::function<void(int, int, std::vector<NormNode>*)> gather;
    std::function<NormNode(int)> norm = [&](int idx) -> NormNode {
        const authjx_node& nd = tree->nodes[idx];
        if (nd.kind == AUTHJX_NODE_PATTERN) {
            if (nd.pattern < 0 || (uint32_t)nd.pattern >= np) { bad = true; return NormNode{3}; }
            NormNode l{2};
            l.pattern = nd.pattern;
            return l;
        }
        if (nd.kind != AUTHJX_NODE_AND && nd.kind != AUTHJX_NODE_OR) { bad = true; return NormNode{3}; }
        int k = nd.kind == AUTHJX_NODE_AND ? 0 : 1;
        NormNode r{k};
        gather(idx, k, &r.kids);
        if (r.kids.empty()) return NormNode{k == 0 ? 3 : 4};  // And{} = T, Or{} = F
        if (r.kids.size() == 1) return r.kids[0];
        return r;
    };
    // flatten same-kind descendants (fold is associative), skipping nil sides
    gather = [&](int idx, int k, std::vector<NormNode>* kids) {
        if (bad) return;
        if (visiting[(size_t)idx]) { bad = true; return; }
        visiting[(size_t)idx] = 1;
        const authjx_node& nd = tree->nodes[idx];
        for (int child : {nd.left, nd.right}) {
            if (child < 0) continue;
            if ((uint32_t)child >= nn) { bad = true; break; }
            const authjx_node& cn = tree->nodes[child];
            int ck = cn.kind == AUTHJX_NODE_AND ? 0 : cn.kind == AUTHJX_NODE_OR ? 1 : -1;
            if (ck == k) {
                gather(child, k, kids);
            } else {
                if (visiting[(size_t)child]) { bad = true; break; }
                kids->push_back(norm(child));
            }
        }
        visiting[(size_t)idx] = 0;
    };
    std::vector<NormNode> normed;
    for (int32_t rt : roots) normed.push_back(rt < 0 ? NormNode{3} : norm(rt));
    if (bad) {
        if (err) *err = "malformed expression tree";
        return AUTHJX_EINVAL;
    }

    std::vector<uint32_t> code;
    uint32_t max_depth = 0;
    std::function<void(const NormNode&, uint32_t)> emit = [&](const NormNode& n, uint32_t depth) {
        switch (n.kind) {
            case 2: code.push_back((C_PAT << 24) | (uint32_t)n.pattern); return;
            case 3: code.push_back(C_CONST_T << 24); return;
            case 4: code.push_back(C_CONST_F << 24); return;
            default:
                max_depth = std::max(max_depth, depth + 1);
                code.push_back((n.kind == 0 ? C_OPEN_AND : C_OPEN_OR) << 24);
                for (const NormNode& c : n.kids) emit(c, depth + 1);
                code.push_back(C_CLOSE << 24);
        }
    };
    std::vector<uint32_t> root_code;  // {begin, len} per tree
    for (const NormNode& rn : normed) {
        const uint32_t b0 = (uint32_t)code.size();
        emit(rn, 0);
        root_code.push_back(b0);
        root_code.push_back((uint32_t)code.size() - b0);
    }
    if (max_depth > kMaxDepth) {
        if (err) *err = "expression nests And/Or deeper than the device fold stack";
        return AUTHJX_ELIMIT;
    }
    if (np > 0xFFFFFF) return AUTHJX_ELIMIT;

    // ---- selectors, patterns, literals, DFAs ----
    std::string lits;
    std::map<std::string, uint32_t> sel_ids;
    std::vector<Selector> sels;
    std::vector<Component> comps;
    std::vector<Modifier> mods;  // modifier chains of the selectors
    std::vector<Pattern> pats(np);
    std::vector<RegexDfa> dfas;
    std::vector<int> dfa_of(np, -1);
    out->pattern_status.assign(np, AUTHJX_PAT_OK);
    out->pattern_error.assign(np, "");
    uint32_t flags = 0;
    for (uint32_t i = 0; i < np; i++) {
        const authjx_pattern& ap = tree->patterns[i];
        std::string sel(ap.selector ? ap.selector : "", ap.selector_len);
        std::string val(ap.value ? ap.value : "", ap.value_len);
        Pattern& p = pats[i];
        std::memset(&p, 0, sizeof p);
        p.op = (uint8_t)(ap.op >= 0 && ap.op <= 5 ? ap.op : 0);
        while (lits.size() % 4) lits.push_back('\0');  // dword-aligned literals (line engine compares)
        p.lit_off = (uint32_t)lits.size();
        p.lit_len = (uint32_t)val.size();
        p.litf = (uint16_t)((val == "true" ? kLitTrue : 0) | (val == "false" ? kLitFalse : 0) | (val.empty() ? kLitEmpty : 0));
        lits += val;
        // Pattern.Matches: the operator decides first whether an error is returned
        if (ap.op < AUTHJX_OP_EQ || ap.op > AUTHJX_OP_MATCHES) {
            p.state = P_STATIC_E;
            out->pattern_status[i] = AUTHJX_PAT_STATIC_ERROR;
            out->pattern_error[i] = "unsupported operator for json authorization";
            continue;
        }
        if (ap.op == AUTHJX_OP_MATCHES) {
            RegexDfa dfa;
            std::string rerr;
            RegexStatus st = compile_go_regex(val, &dfa, &rerr);
            if (st == RX_ERROR) {
                p.state = P_STATIC_E;
                out->pattern_status[i] = AUTHJX_PAT_STATIC_ERROR;
                out->pattern_error[i] = rerr;
                continue;
            }
            if (st == RX_UNSUPPORTED) {
                p.state = P_UNSUPPORTED;
                out->pattern_status[i] = AUTHJX_PAT_UNSUPPORTED;
                out->pattern_error[i] = rerr;
                flags |= 2;
                continue;
            }
            dfa_of[i] = (int)dfas.size();
            dfas.push_back(std::move(dfa));
            flags |= 1;
        }
        auto it = sel_ids.find(sel);
        if (it == sel_ids.end()) {
            std::vector<PathComponent> pc;
            std::string base = sel;
            std::vector<ModSpec> mspec;
            const int mr = split_modifiers(sel, &base, &mspec);
            bool ok_path = mr >= 0 && split_selector(base, &pc);
            bool counted = false;  // a '#' count or list: the exact scan (no modifier chain after it)
            for (const PathComponent& c : pc) counted = counted || c.array_index == kArrCount || c.array_index == kArrList;
            // the paths after modifiers: plain keys / indices (no '#', no modifier inside)
            std::vector<std::vector<PathComponent>> tails(mspec.size());
            size_t n_tail = 0;
            for (size_t k = 0; k < mspec.size() && ok_path; k++) {
                if (mspec[k].kind != M_PATH) continue;
                ok_path = split_selector(mspec[k].a, &tails[k]) && !tails[k].empty();
                for (const PathComponent& c : tails[k]) ok_path = ok_path && c.array_index != kArrCount && c.array_index != kArrList;
                n_tail += tails[k].size();
            }
            if (!ok_path || (counted && !mspec.empty()) || comps.size() + pc.size() + n_tail > 0xFFFFu ||
                mods.size() + mspec.size() > 0xFFFFu) {
                p.state = P_UNSUPPORTED;
                out->pattern_status[i] = AUTHJX_PAT_UNSUPPORTED;
                out->pattern_error[i] = "selector syntax not compiled for the device";
                flags |= 2;
                continue;
            }
            Selector s;
            s.comp_begin = (uint16_t)comps.size();
            s.comp_count = (uint16_t)pc.size();
            s.mod_begin = (uint16_t)mods.size();
            s.mod_count = (uint16_t)mspec.size();
            auto push_comps = [&](const std::vector<PathComponent>& v) {
                for (const PathComponent& c : v) {
                    Component k;
                    k.lit_off = (uint32_t)lits.size();
                    k.lit_len = (uint32_t)c.key.size();
                    k.array_index = c.array_index;
                    k.hash = fnv1a(c.key);
                    lits += c.key;
                    comps.push_back(k);
                }
            };
            push_comps(pc);  // (the selector's own components first: comp_begin)
            for (size_t k = 0; k < mspec.size(); k++) {
                const ModSpec& m = mspec[k];
                Modifier r;
                std::memset(&r, 0, sizeof r);
                r.kind = m.kind;
                r.variant = m.variant;
                if (m.kind == M_PATH) {  // a_off / a_len: its components
                    r.a_off = (uint32_t)comps.size();
                    r.a_len = (uint32_t)tails[k].size();
                    push_comps(tails[k]);
                    mods.push_back(r);
                    continue;
                }
                r.a_off = (uint32_t)lits.size();
                r.a_len = (uint32_t)m.a.size();
                lits += m.a;
                r.b_off = (uint32_t)lits.size();
                r.b_len = (uint32_t)m.b.size();
                lits += m.b;
                r.pos = m.pos;
                mods.push_back(r);
            }
            it = sel_ids.emplace(sel, (uint32_t)sels.size()).first;
            sels.push_back(s);
        }
        p.selector = it->second;
    }

    // ---- selector trie + per-selector pattern lists (single-pass fast path) ----
    struct TNode {
        std::vector<std::pair<std::string, int32_t>> keys;  // (key, array_index)
        std::vector<uint32_t> kids;
        int16_t selector = -1;
    };
    std::vector<TNode> trie(1);
    std::vector<std::vector<uint16_t>> sel_pats(sels.size());
    uint64_t null_true[2] = {0, 0}, static_err[2] = {0, 0}, unsup[2] = {0, 0};
    // (modifier chains run in the exact scan only: such a ruleset has no single-pass tables)
    // (a count selector is answered by the exact scan only)
    bool fast_ok = np <= kFastMaxPatterns && sels.size() <= kFastMaxSelectors && mods.empty();
    for (const Component& c : comps) {
        fast_ok = fast_ok && c.array_index != kArrCount && c.array_index != kArrList;
        if (c.array_index == kArrList) flags |= kFlagBufs;
    }
    for (size_t s = 0; s < sels.size() && fast_ok; s++) {
        uint32_t cur = 0;
        for (uint32_t k = 0; k < sels[s].comp_count; k++) {
            const Component& c = comps[sels[s].comp_begin + k];
            std::string key = lits.substr(c.lit_off, c.lit_len);
            uint32_t next = 0;
            bool found = false;
            for (size_t j = 0; j < trie[cur].kids.size(); j++)
                if (trie[cur].keys[j].first == key) { next = trie[cur].kids[j]; found = true; break; }
            if (!found) {
                for (size_t j = 0; j < trie[cur].keys.size(); j++)
                    if (c.array_index >= 0 && trie[cur].keys[j].second == c.array_index) fast_ok = false;
                next = (uint32_t)trie.size();
                trie.push_back(TNode{});
                trie[cur].keys.push_back({key, c.array_index});
                trie[cur].kids.push_back(next);
            }
            cur = next;
        }
        trie[cur].selector = (int16_t)s;
    }
    if (trie.size() > kFastMaxNodes) fast_ok = false;
    for (uint32_t i = 0; i < np; i++) {
        const Pattern& p = pats[i];
        const uint64_t bit = 1ull << (i & 63);
        if (p.state == P_STATIC_E) { if (i < 128) static_err[i >> 6] |= bit; continue; }
        if (p.state == P_UNSUPPORTED) { if (i < 128) unsup[i >> 6] |= bit; continue; }
        if (p.selector < sels.size()) sel_pats[p.selector].push_back((uint16_t)i);
        bool nt = false;  // Pattern.Matches on a Null result (String() == "", Array() == [])
        switch (p.op) {
            case OP_EQ: nt = p.lit_len == 0; break;
            case OP_NEQ: nt = p.lit_len != 0; break;
            case OP_INCL: nt = false; break;
            case OP_EXCL: nt = true; break;
            case OP_MATCHES: {
                const RegexDfa& d = dfas[(size_t)dfa_of[i]];
                nt = d.start == d.match_state || d.eot[d.start] != 0;
                break;
            }
        }
        if (nt && i < 128) null_true[i >> 6] |= bit;
    }
    if (fast_ok) flags |= kFlagFastOk;
    uint32_t lean_feat = 0;
    for (const TNode& t : trie) {
        for (const auto& k : t.keys) lean_feat |= k.second >= 0 ? kLeanArr : 0u;
        if (t.selector >= 0 && !t.kids.empty()) lean_feat |= kLeanCaps;
    }

    // ---- assemble ----
    Builder b;
    bool sd_on = false;  // the streaming scan's tables, appended after the hot prefix
    StreamHdr sd_sh;
    std::vector<StreamKeySlot> sd_k;
    std::vector<StreamPathSlot> sd_p;
    std::vector<StreamTail> sd_t;
    RulesetHdr hdr;
    std::memset(&hdr, 0, sizeof hdr);
    b.append(&hdr, sizeof hdr);
    {
        std::vector<TrieNode> tn(trie.size());
        std::vector<TrieChild> tc;
        for (size_t i = 0; i < trie.size(); i++) {
            tn[i].child_begin = (uint16_t)tc.size();
            tn[i].n_children = (uint8_t)trie[i].kids.size();
            tn[i].flags = 0;
            tn[i].selector = trie[i].selector;
            tn[i].pad = 0;
            for (size_t j = 0; j < trie[i].kids.size(); j++) {
                TrieChild ch;
                std::memset(&ch, 0, sizeof ch);
                const std::string& key = trie[i].keys[j].first;
                ch.sig = key_signature((const uint8_t*)key.data(), (uint32_t)key.size());
                ch.key_len = (uint32_t)key.size();
                // (8-byte aligned: the lane kernel compares long keys a word at a time)
                while (lits.size() % 8) lits.push_back('\0');
                ch.key_off = (uint32_t)lits.size();
                lits += key;
                ch.array_index = trie[i].keys[j].second;
                if (ch.array_index >= 0) tn[i].flags |= 1;
                ch.node = trie[i].kids[j];
                tc.push_back(ch);
            }
        }
        // key table (linear probing): every (parent, key) edge, and every (parent, array
        // index) edge as an entry of length kIndexKeyLen. Sizes from load 1/2 up to
        // kMaxKeySlotsLog2, and per size a search over hash multipliers for a table where
        // every entry sits in its home slot (key_probes 1: a lookup is one slot read); else
        // the smallest largest distance found (key_probes bounds every lookup's probes)
        struct Ent {
            uint64_t sig;
            uint32_t len, parent, node, key_off;
        };
        std::vector<Ent> ents;
        for (size_t i = 0; i < trie.size(); i++)
            for (uint32_t j = 0; j < tn[i].n_children; j++) {
                const TrieChild& ch = tc[tn[i].child_begin + j];
                if (ch.key_len < kIndexKeyLen) ents.push_back({ch.sig, ch.key_len, (uint32_t)i, ch.node, ch.key_off});
                if (ch.array_index >= 0)
                    ents.push_back({(uint64_t)(uint32_t)ch.array_index, kIndexKeyLen, (uint32_t)i, ch.node, 0});
            }
        uint32_t log2 = 4;
        while ((1u << log2) < 2 * ents.size() && log2 < kMaxKeySlotsLog2) log2++;
        std::vector<KeySlot> slots, best_slots;
        uint32_t probes = 0xFFFFFFFFu, best_log2 = log2, mult = 0x9E3779B1u;
        auto build = [&](uint32_t lg, uint32_t m, std::vector<KeySlot>& out) -> uint32_t {
            out.assign(1u << lg, KeySlot{0, kEmptySlot, 0, 0});
            uint32_t worst = 1;
            for (const Ent& e : ents) {
                uint32_t at = key_slot_hash(e.sig, e.len, e.parent, lg, m), dist = 1;
                while (out[at].meta != kEmptySlot) at = (at + 1) & ((1u << lg) - 1), dist++;
                out[at].sig = e.sig;
                out[at].meta = e.len | (e.parent << 16) | (e.node << 24);
                out[at].key_off8 = (uint16_t)(e.key_off / 8u);  // (a pool past 512 KiB: no fast path, below)
                worst = std::max(worst, dist);
            }
            return worst;
        };
        for (uint32_t lg = log2; lg <= kMaxKeySlotsLog2 && probes > 1; lg++) {
            uint32_t m = 0x9E3779B1u;
            for (int t = 0; t < 512 && probes > 1; t++) {
                const uint32_t worst = build(lg, m, slots);
                if (worst < probes) {
                    probes = worst;
                    best_log2 = lg;
                    mult = m;
                    best_slots = slots;
                }
                m = m * 0x2C1B3C6Du + 0x297A2D38u;  // next candidate (odd)
                m |= 1u;
            }
        }
        log2 = best_log2;
        slots = best_slots;
        hdr.key_mult = mult;
        hdr.key_slots_log2 = log2;
        hdr.key_probes = probes;
        hdr.n_trie_nodes = (uint32_t)tn.size();
        hdr.off_trie_nodes = (uint32_t)b.align16();
        b.append(tn.data(), tn.size() * sizeof(TrieNode));
        hdr.off_trie_children = (uint32_t)b.align16();
        b.append(tc.data(), tc.size() * sizeof(TrieChild));
        hdr.off_key_slots = (uint32_t)b.align16();
        b.append(slots.data(), slots.size() * sizeof(KeySlot));
        // eager patterns (ajx_lean.h): per selector its first two eq / neq / incl / excl
        // patterns with a literal of <= 16 bytes (pattern index < 64)
        if (fast_ok) {
            std::vector<EagerSel> eg(sels.size(), EagerSel{});
            bool any = false;
            for (size_t sidx = 0; sidx < sels.size(); sidx++) {
                uint32_t k = 0;
                bool all = true;
                for (uint16_t pi : sel_pats[sidx]) {
                    const Pattern& pt = pats[pi];
                    if (k >= 2 || pi >= 64 || pt.state != P_OK || pt.lit_len > 16 ||
                        (pt.op != OP_EQ && pt.op != OP_NEQ && pt.op != OP_INCL && pt.op != OP_EXCL)) {
                        all = false;
                        continue;
                    }
                    if (pt.lit_len) std::memcpy(eg[sidx].lit[k], lits.data() + pt.lit_off, pt.lit_len);
                    eg[sidx].m[k] = (uint32_t)pi | ((uint32_t)pt.op << 8) | (pt.lit_len << 16) |
                                    ((uint32_t)(pt.litf & 7u) << 24) | kEagerValid;
                    k++;
                    any = true;
                }
                if (all && k) eg[sidx].pad[0] = kEagerAll;
                // a selector of a root-less forest tree: its record is written even when its
                // patterns were decided in the scan (authjx_select_from_eval_device reads it)
                bool keep = false;
                for (uint16_t pi : sel_pats[sidx]) keep = keep || (kept && pi < kept->size() && (*kept)[pi]);
                if (keep) eg[sidx].pad[0] |= kEagerKeep;

            }
            if (any) {
                hdr.off_eager = (uint32_t)b.align16();
                b.append(eg.data(), eg.size() * sizeof(EagerSel));
            }
        }
        // streaming scan tables (ajx_stream.h): key ids, and the selectors by their
        // component ids
        // (a selector with an array index, too many components or a long key is left to
        // stage B's exact Get: the walk below does not enter those edges)
        bool stream_ok = fast_ok && trie[0].selector < 0;
        uint64_t sexact = 0;
        for (size_t si = 0; si < sels.size(); si++) {
            bool ex = sels[si].comp_count > kStreamMaxComps;
            for (uint32_t k = 0; k < sels[si].comp_count; k++) {
                const Component& c = comps[sels[si].comp_begin + k];
                ex = ex || c.array_index >= 0 || c.lit_len > kStreamMaxKeyLen;
            }
            if (ex) sexact |= 1ull << si;
        }
        if (stream_ok) {
            std::map<std::string, uint32_t> key_id;
            std::vector<std::pair<uint64_t, uint32_t>> paths;  // (path bytes, selector)
            uint32_t max_len = 0;
            struct Walk {
                uint32_t node;
                uint64_t path;
                uint32_t depth;
            };
            // an edge the stream follows: a key (not an array index), of at most
            // kStreamMaxKeyLen bytes, within kStreamMaxComps components
            auto stream_edge = [&](size_t j, const Walk& w) {
                return trie[w.node].keys[j].second < 0 && trie[w.node].keys[j].first.size() <= kStreamMaxKeyLen &&
                       w.depth < kStreamMaxComps;
            };
            // an exact selector's longest prefix the stream follows: its record is the
            // prefix node's selector's, or an extra one after the selectors' (the stream
            // captures that value, stage B runs the rest of the path inside it)
            std::map<uint32_t, uint32_t> extra;  // trie node -> record
            std::vector<StreamTail> tails;
            uint32_t nrec = (uint32_t)sels.size();
            for (size_t si = 0; si < sels.size(); si++) {
                if (!((sexact >> si) & 1ull)) continue;
                uint32_t node = 0, k = 0;
                for (; k < sels[si].comp_count && k < kStreamMaxComps; k++) {
                    const Component& c = comps[sels[si].comp_begin + k];
                    if (c.array_index >= 0 || c.lit_len > kStreamMaxKeyLen) break;
                    const std::string key = lits.substr(c.lit_off, c.lit_len);
                    uint32_t next = 0;
                    for (size_t j = 0; j < trie[node].kids.size() && !next; j++)
                        if (trie[node].keys[j].second < 0 && trie[node].keys[j].first == key) next = trie[node].kids[j];
                    if (!next) break;
                    node = next;
                }
                uint32_t slot = 0xFFFFu;
                if (k > 0) {
                    if (trie[node].selector >= 0) {
                        slot = (uint32_t)trie[node].selector;
                    } else {
                        auto it = extra.find(node);
                        if (it == extra.end()) it = extra.emplace(node, nrec++).first;
                        slot = it->second;
                    }
                }
                tails.push_back(StreamTail{(uint16_t)si, (uint16_t)slot, (uint16_t)(sels[si].comp_begin + k),
                                           (uint16_t)(sels[si].comp_count - k)});
            }
            if (nrec > kFastMaxSelectors) stream_ok = false;  // (found bits)
            std::vector<Walk> stack{{0u, 0ull, 0u}};
            while (!stack.empty() && stream_ok) {
                const Walk w = stack.back();
                stack.pop_back();
                // (a node's meta: its record — its selector, an exact selector's prefix — 0xFFFF
                // none; kStreamHasKids when keys the stream follows go on below it)
                bool kids = false;
                for (size_t j = 0; j < trie[w.node].kids.size(); j++) kids = kids || stream_edge(j, w);
                const auto xt = extra.find(w.node);
                const uint32_t rec = trie[w.node].selector >= 0 ? (uint32_t)trie[w.node].selector
                                     : xt != extra.end()       ? xt->second
                                                               : 0xFFFFu;
                if (w.node && (rec != 0xFFFFu || kids)) paths.push_back({w.path, rec | (kids ? kStreamHasKids : 0u)});
                for (size_t j = 0; j < trie[w.node].kids.size(); j++) {
                    const std::string& key = trie[w.node].keys[j].first;
                    if (!stream_edge(j, w)) continue;  // (the selectors below: exact Get)
                    auto it = key_id.find(key);
                    if (it == key_id.end()) it = key_id.emplace(key, (uint32_t)key_id.size() + 1).first;
                    max_len = std::max(max_len, (uint32_t)key.size());
                    if (it->second > kStreamMaxKeys) {
                        stream_ok = false;
                        break;
                    }
                    stack.push_back({trie[w.node].kids[j], w.path | ((uint64_t)it->second << (8 * w.depth)), w.depth + 1});
                }
            }
            if (stream_ok) {
                // key slots: (sig, len) -> id; key bytes in the literal pool for the head compare
                struct KEnt {
                    uint64_t sig;
                    uint32_t len, id, off;
                };
                std::vector<KEnt> kents;
                for (const auto& kv : key_id) {
                    while (lits.size() % 8) lits.push_back('\0');
                    const uint32_t off = (uint32_t)lits.size();
                    lits += kv.first;
                    kents.push_back({key_signature((const uint8_t*)kv.first.data(), (uint32_t)kv.first.size()),
                                     (uint32_t)kv.first.size(), kv.second, off});
                }
                // open addressing: the multiplier (and size) with the fewest probes
                auto best_table = [](size_t n_ents, auto place, uint32_t& lg_out, uint32_t& mult_out,
                                     uint32_t& probes_out) {
                    uint32_t lg = 3;
                    while ((1u << lg) < 2 * n_ents) lg++;
                    uint32_t probes = 0xFFFFFFFFu;
                    for (uint32_t l2 = lg; l2 <= lg + 2 && probes > 1; l2++) {
                        uint32_t m = 0x9E3779B1u;
                        for (int t = 0; t < 512 && probes > 1; t++) {
                            const uint32_t worst = place(l2, m, false);
                            if (worst < probes) probes = worst, lg_out = l2, mult_out = m;
                            m = (m * 0x2C1B3C6Du + 0x297A2D38u) | 1u;
                        }
                    }
                    probes_out = probes;
                };
                std::vector<StreamKeySlot> kslots;
                auto place_keys = [&](uint32_t lg, uint32_t m, bool keep) -> uint32_t {
                    std::vector<StreamKeySlot> out(1u << lg, StreamKeySlot{0, kEmptySlot, 0});
                    uint32_t worst = 1;
                    for (const KEnt& e : kents) {
                        uint32_t at = key_slot_hash(e.sig, e.len, 0, lg, m), dist = 1;
                        while (out[at].meta != kEmptySlot) at = (at + 1) & ((1u << lg) - 1), dist++;
                        out[at] = StreamKeySlot{e.sig, e.len | (e.id << 16), e.off};
                        worst = std::max(worst, dist);
                    }
                    if (keep) kslots = out;
                    return worst;
                };
                std::vector<StreamPathSlot> pslots;
                auto place_paths = [&](uint32_t lg, uint32_t m, bool keep) -> uint32_t {
                    std::vector<StreamPathSlot> out(1u << lg, StreamPathSlot{0, 0, 0});
                    uint32_t worst = 1;
                    for (const auto& pe : paths) {
                        uint32_t at = stream_path_hash(pe.first, lg, m), dist = 1;
                        while (out[at].meta != 0) at = (at + 1) & ((1u << lg) - 1), dist++;
                        out[at] = StreamPathSlot{pe.first, pe.second | (1u << 31), 0};
                        worst = std::max(worst, dist);
                    }
                    if (keep) pslots = out;
                    return worst;
                };
                StreamHdr sh;
                std::memset(&sh, 0, sizeof sh);
                best_table(kents.size(), place_keys, sh.key_log2, sh.key_mult, sh.key_probes);
                place_keys(sh.key_log2, sh.key_mult, true);
                best_table(paths.size(), place_paths, sh.path_log2, sh.path_mult, sh.path_probes);
                place_paths(sh.path_log2, sh.path_mult, true);
                sh.n_keys = (uint32_t)kents.size();
                sh.max_key_len = max_len;
                // light: every pattern is one of its selector's eager patterns (the stream
                // decides them all while it captures)
                bool light = np <= 64 && hdr.off_eager != 0;
                for (uint32_t i = 0; i < np && light; i++) {
                    const Pattern& pt = pats[i];
                    light = pt.state == P_OK && pt.lit_len <= 16 &&
                            (pt.op == OP_EQ || pt.op == OP_NEQ || pt.op == OP_INCL || pt.op == OP_EXCL);
                }
                for (size_t sidx = 0; sidx < sel_pats.size() && light; sidx++) light = sel_pats[sidx].size() <= 2;
                sh.light = light && !sexact ? 1u : 0u;
                sh.exact_lo = (uint32_t)sexact;
                sh.exact_hi = (uint32_t)(sexact >> 32);
                sh.n_rec = nrec;
                sh.n_tails = (uint32_t)tails.size();
                // (appended after hot_bytes: only the streaming kernel reads them, and it
                // stages the whole blob; the multi-tenant kernel's staged prefix stays small)
                sd_on = true;
                sd_sh = sh;
                sd_k = kslots;
                sd_p = pslots;
                sd_t = tails;
            }
        }
        std::vector<SelectorPatterns> sp(sels.size());
        std::vector<uint16_t> plist;
        for (size_t s = 0; s < sels.size(); s++) {
            sp[s].begin = (uint32_t)plist.size();
            sp[s].count = (uint32_t)sel_pats[s].size();
            sp[s].mask[0] = sp[s].mask[1] = 0;
            for (uint16_t pi : sel_pats[s]) {
                plist.push_back(pi);
                if (pi < 128) sp[s].mask[pi >> 6] |= 1ull << (pi & 63);
            }
        }
        hdr.off_sel_patterns = (uint32_t)b.align16();
        b.append(sp.data(), sp.size() * sizeof(SelectorPatterns));
        hdr.off_pattern_lists = (uint32_t)b.align16();
        b.append(plist.data(), plist.size() * sizeof(uint16_t));
        for (int k = 0; k < 2; k++) {
            hdr.null_true[k] = null_true[k];
            hdr.static_error[k] = static_err[k];
            hdr.unsupported[k] = unsup[k];
        }
    }
    hdr.n_modifiers = (uint32_t)mods.size();
    hdr.off_code = (uint32_t)b.align16();
    b.append(code.data(), code.size() * sizeof(uint32_t));
    if (forest) {
        hdr.pad1[0] = (uint32_t)roots.size();
        hdr.pad1[1] = (uint32_t)b.align16();
        b.append(root_code.data(), root_code.size() * sizeof(uint32_t));
        std::vector<TreeFold> tf(roots.size());
        bool any_tf = false;
        for (size_t k = 0; k < roots.size(); k++) {
            tf[k] = TreeFold{};
            any_tf |= tree_fold_shape(code.data() + root_code[2 * k], root_code[2 * k + 1], &tf[k]);
        }
        if (any_tf) {
            hdr.pad1[2] = (uint32_t)b.align16();
            b.append(tf.data(), tf.size() * sizeof(TreeFold));
        }
    }
    hdr.off_literals = (uint32_t)b.align16();
    lits.append(16, '\0');  // dword reads past a literal's end stay inside the pool
    b.append(lits.data(), lits.size());
    for (uint32_t i = 0; i < np; i++) {
        if (dfa_of[i] < 0) continue;
        const RegexDfa& d = dfas[(size_t)dfa_of[i]];
        DfaHdr dh;
        std::memset(&dh, 0, sizeof dh);
        dh.n_states = d.n_states;
        dh.n_classes = d.n_classes;
        dh.start = d.start;
        dh.match_state = d.match_state;
        dh.n_ranges = (uint32_t)d.ranges.size();
        std::memcpy(dh.ascii_class, d.ascii_class, 128);
        size_t hoff = b.align16();
        b.append(&dh, sizeof dh);
        size_t toff = b.align16();
        b.append(d.trans.data(), d.trans.size() * sizeof(uint16_t));
        size_t eoff = b.align16();
        b.append(d.eot.data(), d.eot.size());
        size_t roff = b.align16();
        b.append(d.ranges.data(), d.ranges.size() * sizeof(RuneRange));
        DfaHdr* hp = reinterpret_cast<DfaHdr*>(b.blob.data() + hoff);
        hp->trans_off = (uint32_t)toff;
        hp->eot_off = (uint32_t)eoff;
        hp->ranges_off = (uint32_t)roff;
        pats[i].dfa_off = (uint32_t)hoff;
    }
    hdr.off_patterns = (uint32_t)b.align16();
    b.append(pats.data(), pats.size() * sizeof(Pattern));
    // the exact scan's tables last: the multi-tenant kernel stages only [0, hot_bytes)
    hdr.hot_bytes = (uint32_t)b.align16();
    if (sd_on) {
        hdr.off_stream = (uint32_t)b.align16();
        b.append(&sd_sh, sizeof sd_sh);
        StreamHdr* shp = reinterpret_cast<StreamHdr*>(b.blob.data() + hdr.off_stream);
        shp->off_keys = (uint32_t)b.align16();
        b.append(sd_k.data(), sd_k.size() * sizeof(StreamKeySlot));
        shp = reinterpret_cast<StreamHdr*>(b.blob.data() + hdr.off_stream);
        shp->off_paths = (uint32_t)b.align16();
        b.append(sd_p.data(), sd_p.size() * sizeof(StreamPathSlot));
        shp = reinterpret_cast<StreamHdr*>(b.blob.data() + hdr.off_stream);
        shp->off_tails = (uint32_t)b.align16();
        b.append(sd_t.data(), sd_t.size() * sizeof(StreamTail));
    }
    hdr.off_modifiers = (uint32_t)b.align16();
    b.append(mods.data(), mods.size() * sizeof(Modifier));
    hdr.off_selectors = (uint32_t)b.align16();
    b.append(sels.data(), sels.size() * sizeof(Selector));
    hdr.off_components = (uint32_t)b.align16();
    b.append(comps.data(), comps.size() * sizeof(Component));
    b.align16();
    if (b.blob.size() > 0xFFFFFFFFull) return AUTHJX_ELIMIT;
    hdr.magic = kMagic;
    hdr.total_bytes = (uint32_t)b.blob.size();
    hdr.n_patterns = np;
    hdr.n_selectors = (uint32_t)sels.size();
    hdr.n_code = (uint32_t)code.size();
    hdr.max_depth = max_depth;
    hdr.lit_bytes = (uint32_t)lits.size();
    hdr.n_components = (uint32_t)comps.size();
    // (KeySlot::key_off8 reaches 512 KiB of literal pool)
    if (lits.size() >= 8u * 65536u) flags &= ~kFlagFastOk;
    if (!forest && roots.size() == 1 && np >= 1 && np <= 64 && code.size() == np + 2u &&
        ((code[0] >> 24) == C_OPEN_AND || (code[0] >> 24) == C_OPEN_OR) && (code[np + 1] >> 24) == C_CLOSE) {
        bool flat = true;
        for (uint32_t k = 0; k < np; k++) flat = flat && code[1 + k] == ((uint32_t)C_PAT << 24 | k);
        if (flat) flags |= kFlagFlatFold;
    }
    if (!forest && roots.size() == 1 && np >= 1 && np <= 64 && !(flags & kFlagFlatFold) && code.size() >= 3 &&
        ((code[0] >> 24) == C_OPEN_AND || (code[0] >> 24) == C_OPEN_OR) && (code.back() >> 24) == C_CLOSE) {
        // [open X, (pattern | open Y, pattern+, close)*, close], Y != X, patterns in order
        const uint32_t outer = code[0] >> 24, inner = outer == C_OPEN_AND ? C_OPEN_OR : C_OPEN_AND;
        uint64_t g_any = 0, g_in = 0, g_start = 0;
        uint32_t next = 0, k = 1;
        bool ok = true;
        const uint32_t last = (uint32_t)code.size() - 1;
        while (ok && k < last) {
            const uint32_t op = code[k] >> 24;
            if (op == C_PAT && (code[k] & 0xFFFFFFu) == next) {
                next++;
                k++;
            } else if (op == inner) {
                const uint32_t lo = next;
                k++;
                while (k < last && (code[k] >> 24) == C_PAT && (code[k] & 0xFFFFFFu) == next) {
                    next++;
                    k++;
                }
                ok = next > lo && k < last && (code[k] >> 24) == C_CLOSE;
                k++;
                if (ok) {
                    const uint64_t m = (next >= 64 ? ~0ull : (1ull << next) - 1ull) & ~((1ull << lo) - 1ull);
                    g_in |= m;
                    if (inner == C_OPEN_OR) g_any |= m;
                    g_start |= 1ull << lo;
                }
            } else {
                ok = false;
            }
        }
        if (ok && k == last && next == np && g_start) {
            flags |= kFlagGroupFold;
            hdr.fold_grp[0] = g_any;
            hdr.fold_grp[1] = g_in;
            hdr.fold_grp[2] = g_start;
        }
    }
    hdr.flags = flags;
    hdr.lean_feat = lean_feat;
    std::memcpy(b.blob.data(), &hdr, sizeof hdr);
    out->blob = std::move(b.blob);
    out->n_patterns = np;
    out->n_selectors = (uint32_t)sels.size();
    out->max_depth = max_depth;
    out->n_trees = (uint32_t)roots.size();
    return AUTHJX_OK;
}
}  // namespace

}  // namespace ajx
