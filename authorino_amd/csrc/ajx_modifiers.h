// ajx_modifiers.h — the reference's gjson modifiers on the device (exact scan only):
// pkg/json/json.go:161-264, registered globally at :258-264. A selector such as
// `auth.identity.email.@extract:{"sep":"@","pos":1}|@case:upper` is its base path (gj_get)
// followed by a chain of Modifier records (ajx_blob.h); gjson runs each modifier on the
// previous result's raw JSON text and parses the last output (gjson.Parse) into the
// Result the pattern compares. The texts are materialised in three work-item buffers.
//
//   extract  Parse(json).String() split on sep; part pos wrapped in quotes, "n" past the end
//   replace  Parse(json).String() with every old -> new, wrapped (no argument: unchanged)
//   case     strings.ToUpper / ToLower of the raw text (upper / lower; else unchanged),
//            Unicode simple mappings from ajx_unicode.h
//   base64   encode: StdEncoding of Parse(json).String(), wrapped; decode: StdEncoding when
//            the length is a multiple of 4 and it decodes, else RawStdEncoding's partial
//            result; quotes escaped, wrapped (else unchanged)
//   strip    the runes unicode.IsPrint keeps, of the raw text (ajx_unicode.h)
// Code points ajx_unicode.h cannot vouch for (unassigned in its Unicode version, special
// casing), texts over kModBuf bytes and Parse of a
// text starting with an uncommon number character ('+' 'i' 'I' 'N', "n" not "null") are
// left undecided (the request's pattern is AUTHJX_UNDECIDED).
#pragma once
#include "ajx_device.h"
#include "ajx_unicode.h"

namespace ajx {

constexpr uint32_t kModBuf = 2048;

struct ModBufs {
    uint8_t a[kModBuf], b[kModBuf], t[kModBuf];
};

struct OutBuf {
    uint8_t* p;
    uint32_t n, cap;
    bool ok;
    AJX_HD void put(uint32_t c) {
        if (n < cap) p[n++] = (uint8_t)c;
        else ok = false;
    }
    AJX_HD void put(const uint8_t* s, uint32_t len) {
        for (uint32_t i = 0; i < len; i++) put(s[i]);
    }
};

// gjson tostr on j[i..n) (j[i] == '"'): the end of the contents (*str_end) and whether
// they need unescape; returns false when no closing quote ends them (the contents then
// run to the end of the text)
AJX_HD bool mod_tostr(const uint8_t* j, uint32_t n, uint32_t i, uint32_t* str_end, bool* esc) {
    for (uint32_t k = i + 1; k < n; k++) {
        if (j[k] > '\\') continue;
        if (j[k] == '"') {
            *str_end = k;
            *esc = false;
            return true;
        }
        if (j[k] == '\\') {
            for (; k < n; k++) {
                if (j[k] > '\\') continue;
                if (j[k] == '"') {
                    if (j[k - 1] == '\\') {
                        uint32_t nb = 0;
                        for (uint32_t q = k - 2; q > i && q < k; q--) {
                            if (j[q] != '\\') break;
                            nb++;
                        }
                        if (nb % 2 == 0) continue;
                    }
                    *str_end = k;
                    *esc = true;
                    return true;
                }
            }
            *str_end = n;
            *esc = true;
            return false;
        }
    }
    *str_end = n;
    *esc = false;
    return false;
}

// gjson tonum extent of a number at j[i]
AJX_HD uint32_t mod_tonum(const uint8_t* j, uint32_t n, uint32_t i) {
    for (uint32_t k = i + 1; k < n; k++) {
        if (j[k] <= '-') {
            if (j[k] <= ' ' || j[k] == ',') return k;
        } else if (j[k] == ']' || j[k] == '}') {
            return k;
        }
    }
    return n;
}
AJX_HD uint32_t mod_tolit(const uint8_t* j, uint32_t n, uint32_t i) {
    for (uint32_t k = i + 1; k < n; k++)
        if (j[k] < 'a' || j[k] > 'z') return k;
    return n;
}

// gjson.Parse(j[0..n)) as a value over a text; `spare` receives an unterminated string's
// contents re-quoted. Returns false when undecided.
AJX_HD bool mod_parse(const uint8_t* j, uint32_t n, uint8_t* spare, const uint8_t** rdoc, ValueRef* v) {
    *rdoc = j;
    v->start = v->end = 0;
    v->type = T_NULL;
    v->esc = 0;
    uint32_t i = 0;
    while (i < n && j[i] <= ' ') i++;
    if (i >= n) return true;  // nothing: not found (Null)
    const uint8_t c = j[i];
    if (c == '{' || c == '[') {
        v->start = i;
        v->end = n;
        v->type = T_JSON;
        return true;
    }
    if (c == '"') {
        uint32_t se;
        bool esc;
        if (mod_tostr(j, n, i, &se, &esc)) {
            v->start = i;
            v->end = se + 1;
            v->type = T_STRING;
            v->esc = esc ? 1 : 0;
            return true;
        }
        // unterminated: the contents j[i+1..n), unescaped when a backslash came first
        OutBuf o{spare, 0, kModBuf, true};
        o.put('"');
        if (esc) {
            StrSrc s;
            s.init_unesc(j, i + 1, n);
            for (int ch; (ch = s.next()) >= 0;) o.put((uint32_t)ch);
        } else {
            o.put(j + i + 1, n - i - 1);
        }
        o.put('"');
        if (!o.ok) return false;
        *rdoc = spare;
        v->start = 0;
        v->end = o.n;
        v->type = T_STRING;
        return true;
    }
    if (c == '-' || (c >= '0' && c <= '9')) {
        v->start = i;
        v->end = mod_tonum(j, n, i);
        v->type = T_NUMBER;
        return true;
    }
    if (c == 't' || c == 'f' || (c == 'n' && (i + 1 >= n || j[i + 1] == 'u'))) {
        v->start = i;
        v->end = mod_tolit(j, n, i);
        v->type = c == 't' ? T_TRUE : c == 'f' ? T_FALSE : T_NULL;
        return true;
    }
    return false;  // '+' 'i' 'I' 'N', "n..." as NaN, other bytes: undecided
}

// gjson.Parse(j).String() into o; false when undecided
AJX_HD bool mod_result_string(const uint8_t* j, uint32_t n, uint8_t* spare, OutBuf& o) {
    const uint8_t* d;
    ValueRef v;
    if (!mod_parse(j, n, spare, &d, &v)) return false;
    StrSrc s;
    if (!string_of<true>(d, v, &s)) return false;
    for (int ch; (ch = s.next()) >= 0;) o.put((uint32_t)ch);
    return o.ok;
}

AJX_HD uint32_t b64_val(uint8_t c) {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    return 0xFF;
}

// encoding/base64 Decode (StdEncoding when pad, else RawStdEncoding; not strict): the
// bytes written before the first error go to o; returns true when the whole input
// decoded (Go: err == nil)
AJX_HD bool b64_decode(const uint8_t* s, uint32_t n, bool pad, OutBuf& o) {
    uint32_t si = 0;
    for (;;) {
        uint32_t q[4];
        uint32_t jn = 0, dlen = 4;
        bool err = false, end = false;
        for (uint32_t j = 0; j < 4; j++) {
            if (si == n) {
                if (j == 0) return true;  // clean end
                if (j == 1 || pad) return false;
                dlen = j;
                end = true;
                break;
            }
            const uint8_t in = s[si++];
            const uint32_t v = b64_val(in);
            if (v != 0xFF) {
                q[j] = v;
                jn = j + 1;
                continue;
            }
            if (in == '\n' || in == '\r') {
                j--;
                continue;
            }
            if (!pad || in != '=') return false;
            // padding
            if (j < 2) return false;
            if (j == 2) {
                while (si < n && (s[si] == '\n' || s[si] == '\r')) si++;
                if (si == n || s[si] != '=') return false;
                si++;
            }
            while (si < n && (s[si] == '\n' || s[si] == '\r')) si++;
            if (si < n) err = true;
            dlen = j;
            end = true;
            break;
        }
        (void)jn;
        for (uint32_t j = dlen; j < 4; j++) q[j] = 0;
        const uint32_t val = (q[0] << 18) | (q[1] << 12) | (q[2] << 6) | q[3];
        if (dlen >= 2) o.put((val >> 16) & 0xFF);
        if (dlen >= 3) o.put((val >> 8) & 0xFF);
        if (dlen >= 4) o.put(val & 0xFF);
        if (err) return false;
        if (end) return true;
    }
}

AJX_HD void b64_encode(const uint8_t* s, uint32_t n, OutBuf& o) {
    const char* al = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    uint32_t i = 0;
    for (; i + 3 <= n; i += 3) {
        const uint32_t v = ((uint32_t)s[i] << 16) | ((uint32_t)s[i + 1] << 8) | s[i + 2];
        o.put((uint8_t)al[(v >> 18) & 63]);
        o.put((uint8_t)al[(v >> 12) & 63]);
        o.put((uint8_t)al[(v >> 6) & 63]);
        o.put((uint8_t)al[v & 63]);
    }
    if (n - i == 1) {
        const uint32_t v = (uint32_t)s[i] << 16;
        o.put((uint8_t)al[(v >> 18) & 63]);
        o.put((uint8_t)al[(v >> 12) & 63]);
        o.put('=');
        o.put('=');
    } else if (n - i == 2) {
        const uint32_t v = ((uint32_t)s[i] << 16) | ((uint32_t)s[i + 1] << 8);
        o.put((uint8_t)al[(v >> 18) & 63]);
        o.put((uint8_t)al[(v >> 12) & 63]);
        o.put((uint8_t)al[(v >> 6) & 63]);
        o.put('=');
    }
}

// '"' + escapeQuotes(s) + '"' (json.go escapeQuotes: '"' -> '\"', nothing else)
AJX_HD void wrap_escaped(const uint8_t* s, uint32_t n, OutBuf& o) {
    o.put('"');
    for (uint32_t i = 0; i < n; i++) {
        if (s[i] == '"') o.put('\\');
        o.put(s[i]);
    }
    o.put('"');
}

// gjson's "#." list (parseArray with alogok, at the array's ']'): for every element of
// the array v (kValList), Get(element, the selector's parts after the list part); the raw
// texts of those that exist, comma-joined in '[' ']', parsed as the Result (*rdoc, *rv).
// False when the text exceeds the buffer (undecided).
AJX_HD bool build_list(const uint8_t* blob, const Selector& sel, const uint8_t* doc, const ValueRef& v, ModBufs& mb,
                       const uint8_t** rdoc, ValueRef* rv) {
    const RulesetHdr* h = (const RulesetHdr*)blob;
    const Component* comps = (const Component*)(blob + h->off_components) + sel.comp_begin;
    const uint8_t* lits = blob + h->off_literals;
    uint32_t k = 0;
    while (k < sel.comp_count && comps[k].array_index != kArrList) k++;
    OutBuf o{mb.a, 0, kModBuf, true};
    o.put('[');
    ArrIter it;
    ValueRef arr = v;
    arr.esc = 0;
    it.init(doc, arr);
    ValueRef e;
    uint32_t cnt = 0;
    while (it.next(&e)) {
        const ValueRef sub = gj_get(doc + e.start, e.end - e.start, comps + k + 1, sel.comp_count - k - 1, lits);
        if (sub.end <= sub.start) continue;  // (not found; a synthetic value needs no list here)
        if (cnt++) o.put(',');
        o.put(doc + e.start + sub.start, sub.end - sub.start);
    }
    o.put(']');
    if (!o.ok) return false;
    *rdoc = mb.a;
    rv->start = 0;
    rv->end = o.n;
    rv->type = T_JSON;
    rv->esc = 0;
    return true;
}

// Go's utf8.DecodeRune of s[i..n): the rune and its width; an invalid or truncated
// sequence (overlong, surrogate, > U+10FFFF) is U+FFFD of width 1, as `range` over a
// string yields it
AJX_HD uint32_t go_decode_rune(const uint8_t* s, uint32_t n, uint32_t i, uint32_t* w) {
    const uint32_t b0 = s[i];
    *w = 1;
    if (b0 < 0x80) return b0;
    auto cont = [&](uint32_t k, uint32_t lo, uint32_t hi) { return i + k < n && s[i + k] >= lo && s[i + k] <= hi; };
    if (b0 >= 0xC2 && b0 <= 0xDF) {
        if (!cont(1, 0x80, 0xBF)) return 0xFFFD;
        *w = 2;
        return ((b0 & 0x1F) << 6) | (s[i + 1] & 0x3F);
    }
    if (b0 >= 0xE0 && b0 <= 0xEF) {
        const uint32_t lo = b0 == 0xE0 ? 0xA0 : 0x80, hi = b0 == 0xED ? 0x9F : 0xBF;
        if (!cont(1, lo, hi) || !cont(2, 0x80, 0xBF)) return 0xFFFD;
        *w = 3;
        return ((b0 & 0x0F) << 12) | ((s[i + 1] & 0x3Fu) << 6) | (s[i + 2] & 0x3F);
    }
    if (b0 >= 0xF0 && b0 <= 0xF4) {
        const uint32_t lo = b0 == 0xF0 ? 0x90 : 0x80, hi = b0 == 0xF4 ? 0x8F : 0xBF;
        if (!cont(1, lo, hi) || !cont(2, 0x80, 0xBF) || !cont(3, 0x80, 0xBF)) return 0xFFFD;
        *w = 4;
        return ((b0 & 0x07) << 18) | ((s[i + 1] & 0x3Fu) << 12) | ((s[i + 2] & 0x3Fu) << 6) | (s[i + 3] & 0x3F);
    }
    return 0xFFFD;
}

// utf8.EncodeRune (the runes here are valid)
AJX_HD void put_rune(OutBuf& o, uint32_t r) {
    if (r < 0x80) {
        o.put(r);
    } else if (r < 0x800) {
        o.put(0xC0 | (r >> 6));
        o.put(0x80 | (r & 0x3F));
    } else if (r < 0x10000) {
        o.put(0xE0 | (r >> 12));
        o.put(0x80 | ((r >> 6) & 0x3F));
        o.put(0x80 | (r & 0x3F));
    } else {
        o.put(0xF0 | (r >> 18));
        o.put(0x80 | ((r >> 12) & 0x3F));
        o.put(0x80 | ((r >> 6) & 0x3F));
        o.put(0x80 | (r & 0x3F));
    }
}

// ajx_unicode.h tables: is r inside one of n sorted (lo, hi) ranges; r's mapping in n
// sorted (code point, mapping) pairs (r itself when absent)
AJX_HD bool uni_in_ranges(const uint32_t* t, uint32_t n, uint32_t r) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (t[2 * mid + 1] < r) lo = mid + 1;
        else hi = mid;
    }
    return lo < n && t[2 * lo] <= r;
}
AJX_HD uint32_t uni_map(const uint32_t* t, uint32_t n, uint32_t r) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (t[2 * mid] < r) lo = mid + 1;
        else hi = mid;
    }
    return lo < n && t[2 * lo] == r ? t[2 * lo + 1] : r;
}

// gjson Valid (v1.14.0 validpayload / validany / validobject / validarray / validstring /
// validnumber / validtrue...): one JSON value with surrounding ' ' '\t' '\n' '\r' and
// nothing else; strings are not checked for UTF-8. Iterative, containers on a bit stack.
// Returns false when undecided (nesting deeper than the stack), *ok the verdict.
AJX_HD bool json_valid(const uint8_t* d, uint32_t n, bool* ok) {
    constexpr uint32_t kDepth = 256;
    uint64_t stk[kDepth / 64];  // bit: 1 object, 0 array
    uint32_t depth = 0, i = 0;
    *ok = false;
    auto ws = [&]() {
        while (i < n && (d[i] == ' ' || d[i] == '\t' || d[i] == '\n' || d[i] == '\r')) i++;
    };
    auto is_digit = [&](uint32_t k) { return k < n && d[k] >= '0' && d[k] <= '9'; };
    auto hex = [](uint8_t c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); };
    auto string = [&]() -> bool {  // at the opening quote
        for (i++; i < n; i++) {
            const uint8_t c = d[i];
            if (c < ' ') return false;
            if (c == '"') {
                i++;
                return true;
            }
            if (c == '\\') {
                if (++i == n) return false;
                const uint8_t e = d[i];
                if (e == 'u') {
                    for (int j = 0; j < 4; j++)
                        if (++i >= n || !hex(d[i])) return false;
                } else if (e != '"' && e != '\\' && e != '/' && e != 'b' && e != 'f' && e != 'n' && e != 'r' &&
                           e != 't') {
                    return false;
                }
            }
        }
        return false;
    };
    auto word = [&](const char* w, uint32_t len) {
        for (uint32_t k = 0; k < len; k++)
            if (i + k >= n || d[i + k] != (uint8_t)w[k]) return false;
        i += len;
        return true;
    };
    ws();
    for (;;) {
        // a value at i
        if (i >= n) return true;
        const uint8_t c = d[i];
        if (c == '{' || c == '[') {  // (an empty one goes on after it, like a scalar)
            i++;
            ws();
            if (i < n && d[i] == (c == '{' ? '}' : ']')) {
                i++;
            } else {
                if (depth == kDepth) return false;
                if (c == '{') stk[depth >> 6] |= 1ull << (depth & 63);
                else stk[depth >> 6] &= ~(1ull << (depth & 63));
                depth++;
                if (c == '{') {  // a key, ':' and the member's value
                    if (i >= n || d[i] != '"' || !string()) return true;
                    ws();
                    if (i >= n || d[i] != ':') return true;
                    i++;
                    ws();
                }
                continue;
            }
        } else if (c == '"') {
            if (!string()) return true;
        } else if (c == '-' || (c >= '0' && c <= '9')) {
            if (c == '-') {
                i++;
                if (!is_digit(i)) return true;
            }
            if (d[i] == '0') i++;
            else
                while (is_digit(i)) i++;
            if (i < n && d[i] == '.') {
                i++;
                if (!is_digit(i)) return true;
                while (is_digit(i)) i++;
            }
            if (i < n && (d[i] == 'e' || d[i] == 'E')) {
                i++;
                if (i < n && (d[i] == '+' || d[i] == '-')) i++;
                if (!is_digit(i)) return true;
                while (is_digit(i)) i++;
            }
        } else if (c == 't') {
            if (!word("true", 4)) return true;
        } else if (c == 'f') {
            if (!word("false", 5)) return true;
        } else if (c == 'n') {
            if (!word("null", 4)) return true;
        } else {
            return true;
        }
        // after a value: the container's ',' / closer, or the end of the text
        for (;;) {
            ws();
            if (depth == 0) {
                *ok = i == n;
                return true;
            }
            const bool obj = (stk[(depth - 1) >> 6] >> ((depth - 1) & 63)) & 1u;
            if (i >= n) return true;
            if (d[i] == ',') {
                i++;
                ws();
                if (obj) {
                    if (i >= n || d[i] != '"' || !string()) return true;
                    ws();
                    if (i >= n || d[i] != ':') return true;
                    i++;
                    ws();
                }
                break;  // the next value
            }
            if (d[i] != (obj ? '}' : ']')) return true;
            i++;
            depth--;
        }
    }
}

// Run the selector's modifier chain on the value v of document doc: the final gjson
// Result as (*rdoc, *rv). Returns false when undecided. A value that does not exist stays
// Null (gjson pipes into the modifiers only from a found value).
AJX_HD bool apply_modifiers(const uint8_t* blob, const Selector& sel, const uint8_t* doc, const ValueRef& v,
                            ModBufs& mb, const uint8_t** rdoc, ValueRef* rv) {
    if (v.end <= v.start) {
        *rdoc = doc;
        *rv = v;
        return true;
    }
    const RulesetHdr* h = (const RulesetHdr*)blob;
    const Modifier* mods = (const Modifier*)(blob + h->off_modifiers) + sel.mod_begin;
    const uint8_t* lits = blob + h->off_literals;
    const uint8_t* in = doc + v.start;
    uint32_t in_n = v.end - v.start;
    uint8_t* bufs[2] = {mb.a, mb.b};
    for (uint32_t k = 0; k < sel.mod_count; k++) {
        const Modifier m = mods[k];
        uint8_t* outp = bufs[k & 1];
        OutBuf o{outp, 0, kModBuf, true};
        OutBuf t{mb.t, 0, kModBuf, true};
        switch (m.kind) {
            case M_EXTRACT: {
                if (!mod_result_string(in, in_n, outp, t)) return false;
                const uint8_t* sep = lits + m.a_off;
                const uint32_t sl = m.a_len;
                uint32_t part = 0, ps = 0, i = 0;
                bool done = false;
                while (!done) {
                    // the next separator at or after i (or the end)
                    uint32_t e = i;
                    while (e + sl <= t.n && !bytes_equal(mb.t + e, sep, sl)) e++;
                    const bool last = e + sl > t.n;
                    if (last) e = t.n;
                    if (part == m.pos) {
                        o.put('"');
                        o.put(mb.t + ps, e - ps);
                        o.put('"');
                        done = true;
                        break;
                    }
                    if (last) break;
                    part++;
                    i = e + sl;
                    ps = i;
                }
                if (!done) o.put('n');
                break;
            }
            case M_REPLACE: {
                if (m.variant == 0) {
                    o.put(in, in_n);
                    break;
                }
                if (!mod_result_string(in, in_n, outp, t)) return false;
                const uint8_t* old = lits + m.a_off;
                o.put('"');
                uint32_t i = 0;
                while (i < t.n) {
                    if (i + m.a_len <= t.n && bytes_equal(mb.t + i, old, m.a_len)) {
                        o.put(lits + m.b_off, m.b_len);
                        i += m.a_len;
                    } else {
                        o.put(mb.t[i++]);
                    }
                }
                o.put('"');
                break;
            }
            case M_CASE: {  // strings.ToUpper / ToLower: Map(unicode.ToUpper / ToLower)
                for (uint32_t i = 0; i < in_n;) {
                    uint8_t c = in[i];
                    if (c < 0x80 || !m.variant) {
                        if (m.variant == 1 && c >= 'a' && c <= 'z') c = (uint8_t)(c - 32);
                        if (m.variant == 2 && c >= 'A' && c <= 'Z') c = (uint8_t)(c + 32);
                        o.put(c);
                        i++;
                        continue;
                    }
                    uint32_t w;
                    const uint32_t r = go_decode_rune(in, in_n, i, &w);  // (invalid: U+FFFD)
                    i += w;
                    if (uni_in_ranges(kUniUndecided, kUniUndecided_n, r)) return false;
                    put_rune(o, m.variant == 1 ? uni_map(kUniUpper, kUniUpper_n, r) : uni_map(kUniLower, kUniLower_n, r));
                }
                break;
            }
            case M_BASE64: {
                if (m.variant == 0) {
                    o.put(in, in_n);
                    break;
                }
                if (!mod_result_string(in, in_n, outp, t)) return false;
                if (m.variant == 1) {
                    o.put('"');
                    b64_encode(mb.t, t.n, o);
                    o.put('"');
                    break;
                }
                // decode into the spare half of the output buffer, then wrap
                OutBuf dec{outp + kModBuf / 2, 0, kModBuf / 2, true};
                bool ok = false;
                if (t.n % 4 == 0) ok = b64_decode(mb.t, t.n, true, dec);
                if (!ok) {
                    dec.n = 0;
                    (void)b64_decode(mb.t, t.n, false, dec);
                }
                if (!dec.ok) return false;
                OutBuf w{outp, 0, kModBuf / 2, true};
                wrap_escaped(dec.p, dec.n, w);
                if (!w.ok) return false;
                o.n = w.n;
                break;
            }
            case M_STRIP: {  // strings.Map dropping the runes unicode.IsPrint rejects
                for (uint32_t i = 0; i < in_n;) {
                    const uint8_t c = in[i];
                    if (c < 0x80) {
                        if (c >= 0x20 && c != 0x7F) o.put(c);
                        i++;
                        continue;
                    }
                    uint32_t w;
                    const uint32_t r = go_decode_rune(in, in_n, i, &w);
                    i += w;
                    if (uni_in_ranges(kUniUndecided, kUniUndecided_n, r)) return false;
                    if (uni_in_ranges(kUniPrint, kUniPrint_n, r)) put_rune(o, r);
                }
                break;
            }
            case M_FROMSTR: {  // gjson modFromStr: "" unless Valid(json), else Parse(json).String()
                bool ok;
                if (!json_valid(in, in_n, &ok)) return false;
                if (!ok) break;
                if (!mod_result_string(in, in_n, outp, t)) return false;
                o.put(mb.t, t.n);
                break;
            }
            case M_PATH: {  // Get(previous output, path): its raw text; not found: Null
                const Component* tc = (const Component*)(blob + h->off_components) + m.a_off;
                const ValueRef v = gj_get(in, in_n, tc, m.a_len, lits);
                if (v.esc == kValCount || v.esc == kValList) return false;  // (not compiled in tails)
                if (v.end <= v.start) {
                    *rdoc = in;
                    *rv = ValueRef{0, 0, T_NULL, 0};
                    return true;
                }
                o.put(in + v.start, v.end - v.start);
                break;
            }
            default: return false;
        }
        if (!o.ok) return false;
        in = outp;
        in_n = o.n;
    }
    return mod_parse(in, in_n, mb.t, rdoc, rv);
}

// authjx_value.esc flag of a value that is built text (a modifier chain's output, a "#."
// list), not a span of the document: [start, start + len) of the request's text slot
constexpr uint8_t kValText = 4;

// The value of selector `sl` as JSONValue.ResolveFor / ReplaceJSONPlaceholders see it
// (pkg/json/json.go:41-53, :96-151: gjson.Get with the path's modifiers): a span of the
// document, or, after a modifier chain or for a "#." list, the final Result's raw text
// appended to the request's text slot text[*used, cap) (esc | kValText). out = {start,
// len, type | esc << 8}. False when undecided (the slot or a buffer is full, Unicode case
// mapping, ...).
AJX_HD bool select_value(const uint8_t* blob, const Selector& sl, const uint8_t* doc, uint32_t len, ModBufs& mb,
                         uint8_t* text, uint32_t cap, uint32_t* used, uint32_t* out) {
    const RulesetHdr* h = (const RulesetHdr*)blob;
    const Component* comps = (const Component*)(blob + h->off_components);
    const uint8_t* lits = blob + h->off_literals;
    const ValueRef v = gj_get(doc, len, comps + sl.comp_begin, sl.comp_count, lits);
    const uint8_t* rd = doc;
    ValueRef rv = v;
    if (v.esc == kValList) {  // (a "#." list has no modifier chain after it)
        if (!build_list(blob, sl, doc, v, mb, &rd, &rv)) return false;
    } else if (sl.mod_count) {
        if (!apply_modifiers(blob, sl, doc, v, mb, &rd, &rv)) return false;
    }
    if (rd == doc) {  // the document's own span (or a count, or Null)
        out[0] = rv.start;
        out[1] = rv.end - rv.start;
        out[2] = (uint32_t)rv.type | ((uint32_t)rv.esc << 8);
        return true;
    }
    const uint32_t n = rv.end - rv.start;
    if (!text || n > cap - *used) return false;
    for (uint32_t i = 0; i < n; i++) text[*used + i] = rd[rv.start + i];
    out[0] = *used;
    out[1] = n;
    out[2] = (uint32_t)rv.type | ((uint32_t)(rv.esc | kValText) << 8);
    *used += n;
    return true;
}

}  // namespace ajx
