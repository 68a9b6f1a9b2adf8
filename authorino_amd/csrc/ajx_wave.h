// ajx_wave.h — the wave kernel: one wavefront per request for the structural scan, one
// work-item per request for the token walk and the patterns.
//
// Phase 1, LEX (wave-wide, one document at a time): the document is read in 1 KiB chunks,
// 16 bytes per lane, with coalesced dwordx4 loads. Each lane classifies its 16 bytes
// (SWAR) into 16-bit masks: quote, backslash, brackets, ':' ',', whitespace. Escapes are
// resolved with the odd-backslash-run rule and a lane-to-lane carry; string interiors
// with an in-lane prefix-XOR plus a wavefront ballot of per-lane quote parities. Every
// byte outside strings is checked against the byte before it (compact JSON grammar:
// what may follow '{' '[' ':' ',' a closing quote, a scalar, a closing bracket). The
// lexer then emits one 32-bit token per ELEMENT START (the root, every array element,
// every object member — the member token carries the key's label and the offset of its
// value) and per closing bracket, in document order, into the wave's LDS token buffer.
// Key labels are looked up by (length, last <= 8 bytes) in the ruleset's label table,
// one token per lane.
//
// Phase 2, WALK (one work-item per request, a batch of the requests the wave lexed):
// the tokens drive a JSON pushdown automaton (objects take member tokens, arrays element
// tokens, brackets must match, exactly one root) that also follows every selector through
// the trie (edge table keyed by (node, label)), so the first value in document order
// on each selector's path is captured — the value gjson v1.14.0 Get returns for valid
// JSON (its scan is a depth-first walk in document order that descends into matching
// keys only). Anything the lexer or the walker can not prove to be compact, valid JSON
// (whitespace between tokens, a bad literal, a key with escapes, ...) sends the request
// to the exact per-selector scan (ajx_device.h gj_get), which is exact on any bytes.
//
// Phase 3, PATTERNS (one work-item per request): Pattern.Matches on the captured values,
// the T bitmap and the And/Or fold (ajx_fast.h patterns_from_row, ajx_kernels fold).
//
// The cross-lane operations go through a wave-ops object W so that the same source runs
// on gfx950 (W = WaveHw) and in the CPU test harness (tests/native: 64 threads, one per
// lane, barriers in place of the hardware's lockstep).
#pragma once
#include "ajx_fast.h"

namespace ajx {

// ---- token entries ------------------------------------------------------------------
// pos (16) | voff (8) | vc (4) | kind (2) | 0 (2)
//   ELEMENT  pos = the value's first byte (root, array element); voff = 0
//   MEMBER   pos = the key's opening quote; the value starts at pos + voff
//   CLOSE    pos = the closing bracket; vc = 0 '}' / 1 ']'
enum : uint32_t { TK_ELEM = 0, TK_MEMBER = 1, TK_CLOSE = 2 };
enum : uint32_t { VC_STR = 0, VC_OBJ = 1, VC_ARR = 2, VC_NUM = 3, VC_TRUE = 4, VC_FALSE = 5, VC_NULL = 6 };
AJX_HD uint32_t tok_make(uint32_t pos, uint32_t voff, uint32_t vc, uint32_t kind) {
    return (pos & 0xFFFFu) | ((voff & 0xFFu) << 16) | ((vc & 0xFu) << 24) | (kind << 28);
}
AJX_HD uint32_t tok_pos(uint32_t e) { return e & 0xFFFFu; }
AJX_HD uint32_t tok_voff(uint32_t e) { return (e >> 16) & 0xFFu; }
AJX_HD uint32_t tok_vc(uint32_t e) { return (e >> 24) & 0xFu; }
AJX_HD uint32_t tok_kind(uint32_t e) { return (e >> 28) & 3u; }

constexpr uint32_t kWaveMaxDoc = 0xFFFFu;  // documents the lexer takes (16-bit positions)
constexpr uint32_t kWaveChunk = 1024;      // bytes per wave step (64 lanes x 16 B)

// value class of a value's first byte (the grammar checks guarantee it starts a value)
AJX_HD uint32_t value_class(uint32_t b) {
    return b == '"' ? VC_STR : b == '{' ? VC_OBJ : b == '[' ? VC_ARR : b == 't' ? VC_TRUE
         : b == 'f' ? VC_FALSE : b == 'n' ? VC_NULL : VC_NUM;
}

// byte j (0..15) of four dwords (selected, not indexed: a runtime index would put the
// array in scratch memory)
AJX_HD uint32_t byte_of4(const uint32_t (&x)[4], uint32_t j) {
    const uint32_t q = j >> 2;
    const uint32_t v = q == 0 ? x[0] : q == 1 ? x[1] : q == 2 ? x[2] : x[3];
    return (v >> (8 * (j & 3))) & 0xFFu;
}

AJX_HD void load16(const uint8_t* p, uint32_t (&v)[4]) {  // p 16-B aligned
#if defined(__HIP_DEVICE_COMPILE__)
    const uint4 q = *reinterpret_cast<const uint4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
#else
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
    v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
#endif
}
AJX_HD void store16(uint8_t* p, const uint32_t (&v)[4]) {  // p 16-B aligned
#if defined(__HIP_DEVICE_COMPILE__)
    *reinterpret_cast<uint4*>(p) = uint4{v[0], v[1], v[2], v[3]};
#else
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
    q[0] = v[0]; q[1] = v[1]; q[2] = v[2]; q[3] = v[3];
#endif
}

// escaped bytes of a lane's 16 (simdjson's odd-backslash-run rule); cin: byte 0 is
// escaped by the previous lane; *cout: byte 16 (the next lane's byte 0) is escaped
AJX_HD uint32_t escaped16(uint32_t bs, uint32_t cin, uint32_t* cout) {
    const uint32_t b = bs & ~cin;
    const uint32_t follows = ((b << 1) | cin) & 0xFFFFu;
    const uint32_t even = 0x5555u;
    const uint32_t odd_starts = b & ~even & ~follows;
    const uint32_t seq = odd_starts + b;
    *cout = (seq >> 16) & 1u;
    return (even ^ (seq << 1)) & follows & 0xFFFFu;
}

AJX_HD uint32_t prefix_xor16(uint32_t x) {
    x ^= x << 1;
    x ^= x << 2;
    x ^= x << 4;
    x ^= x << 8;
    return x & 0xFFFFu;
}

// the lane-local 16 classification masks of 16 bytes
struct Classes16 {
    uint32_t q, bs, o, c, k, m, ws;
};
AJX_HD Classes16 classify16(const uint32_t (&x)[4]) {
    Classes16 r{0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t v = x[j], lx = v | 0x20202020u;
        const uint32_t sh = 4u * (uint32_t)j;
        r.q |= gather4(eq_bytes(v, 0x22222222u)) << sh;
        r.bs |= gather4(eq_bytes(v, 0x5C5C5C5Cu)) << sh;
        r.o |= gather4(eq_bytes(lx, 0x7B7B7B7Bu)) << sh;
        r.c |= gather4(eq_bytes(lx, 0x7D7D7D7Du)) << sh;
        r.k |= gather4(eq_bytes(v, 0x3A3A3A3Au)) << sh;
        r.m |= gather4(eq_bytes(v, 0x2C2C2C2Cu)) << sh;
        r.ws |= gather4(le20_bytes(v)) << sh;
    }
    return r;
}

// ring of the last two chunks of the document, in LDS (key bytes for the label lookup;
// a key may start in the previous chunk)
AJX_HD uint32_t ring_byte(const uint8_t* ring, uint32_t a) { return ring[a & (2 * kWaveChunk - 1)]; }

// gjson's unescape (the S_UNESC stream of ajx_device.h StrSrc) over ring bytes [i, n):
// the next output byte, -1 at the end (or where gjson's unescape stops).
struct RingUnesc {
    const uint8_t* ring;
    uint32_t i, n;
    uint8_t buf[4];
    uint8_t bn, bi;
    bool done;
    AJX_HD uint32_t at(uint32_t k) const { return ring_byte(ring, k); }
    AJX_HD uint32_t hex4(uint32_t k) const {
        uint32_t v = 0;
        for (uint32_t j = 0; j < 4; j++) {
            const uint32_t c = at(k + j);
            uint32_t x;
            if (c >= '0' && c <= '9') x = c - '0';
            else if (c >= 'a' && c <= 'f') x = c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') x = c - 'A' + 10;
            else return 0;
            v = v * 16 + x;
        }
        return v;
    }
    AJX_HD int next() {
        if (bi < bn) return buf[bi++];
        if (done || i >= n) return -1;
        const uint32_t c = at(i);
        if (c < ' ') { done = true; return -1; }
        if (c != '\\') { i++; return (int)c; }
        i++;
        if (i >= n) { done = true; return -1; }
        const uint32_t e = at(i);
        uint32_t out;
        switch (e) {
            case '\\': out = '\\'; break;
            case '/': out = '/'; break;
            case 'b': out = '\b'; break;
            case 'f': out = '\f'; break;
            case 'n': out = '\n'; break;
            case 'r': out = '\r'; break;
            case 't': out = '\t'; break;
            case '"': out = '"'; break;
            case 'u': {
                if (i + 5 > n) { done = true; return -1; }
                uint32_t r = hex4(i + 1);
                i += 5;
                if (r >= 0xD800 && r < 0xE000) {
                    if (n - i >= 6 && at(i) == '\\' && at(i + 1) == 'u') {
                        const uint32_t r2 = hex4(i + 2);
                        if (r < 0xDC00 && r2 >= 0xDC00 && r2 < 0xE000) r = (((r - 0xD800) << 10) | (r2 - 0xDC00)) + 0x10000;
                        else r = 0xFFFD;
                        i += 6;
                    }
                }
                bn = (uint8_t)utf8_put(r, buf);
                bi = 1;
                return buf[0];
            }
            default: done = true; return -1;
        }
        i++;
        return (int)out;
    }
};

// Label of the key whose bytes are at aligned-base offsets [a0, a0 + len) in the ring
// (0: not a trie key). Keys holding a backslash are compared unescaped, as gjson does.
AJX_HD uint32_t key_label(const uint8_t* blob, const uint8_t* ring, uint32_t a0, uint32_t len) {
    const RulesetHdr* h = (const RulesetHdr*)blob;
    bool bsl = false;
    for (uint32_t j = 0; j < len; j++) bsl |= ring_byte(ring, a0 + j) == '\\';
    const LabelSlot* ls = (const LabelSlot*)(blob + h->off_label_slots);
    const uint8_t* lits = blob + h->off_literals;
    const uint32_t log2 = h->label_slots_log2, mask = (1u << log2) - 1u;
    if (!bsl) {
        const uint32_t m = len < 8 ? len : 8u;
        uint64_t sig = 0;
        for (uint32_t j = 0; j < m; j++) sig |= (uint64_t)ring_byte(ring, a0 + len - m + j) << (8 * j);
        uint32_t at = key_slot_hash(sig, len, 0, log2);
        for (uint32_t probe = 0; probe <= mask; probe++, at = (at + 1) & mask) {
            const LabelSlot s = ls[at];
            if (s.meta == kEmptySlot) return 0;
            if (s.sig != sig || (s.meta & 0xFFFFu) != len) continue;
            bool eq = true;
            for (uint32_t j = 0; j + 8 < len; j++)
                if (ring_byte(ring, a0 + j) != lits[s.key_off + j]) { eq = false; break; }
            if (eq) return s.meta >> 16;
        }
        return 0;
    }
    // escaped key: the unescaped length and last 8 bytes, then a compare of the rest
    RingUnesc u{ring, a0, a0 + len, {0, 0, 0, 0}, 0, 0, false};
    uint32_t ulen = 0;
    uint64_t last = 0;
    for (int c; (c = u.next()) >= 0;) {
        last = (last >> 8) | ((uint64_t)(uint32_t)c << 56);
        ulen++;
    }
    const uint32_t m = ulen < 8 ? ulen : 8u;
    const uint64_t sig = m ? last >> (8 * (8 - m)) : 0ull;
    uint32_t at = key_slot_hash(sig, ulen, 0, log2);
    for (uint32_t probe = 0; probe <= mask; probe++, at = (at + 1) & mask) {
        const LabelSlot s = ls[at];
        if (s.meta == kEmptySlot) return 0;
        if (s.sig != sig || (s.meta & 0xFFFFu) != ulen) continue;
        RingUnesc v{ring, a0, a0 + len, {0, 0, 0, 0}, 0, 0, false};
        bool eq = true;
        for (uint32_t j = 0; j + 8 < ulen; j++)
            if ((uint32_t)v.next() != lits[s.key_off + j]) { eq = false; break; }
        if (eq) return s.meta >> 16;
    }
    return 0;
}

// ---- phase 1: lex one document (every lane of the wave calls it) ---------------------
enum : uint32_t { LEX_OK = 0, LEX_BAD = 1, LEX_OVERFLOW = 2 };

// ablate (profiling only): 0 full; 1 loads + classification + strings + grammar checks,
// no tokens; 2 loads only
template <class W>
AJX_HD uint32_t lex_doc(W& w, const uint8_t* blob, const uint8_t* d, uint32_t n, uint8_t* ring, uint32_t* tok,
                        uint8_t* lab, uint32_t tok_base, uint32_t tok_cap, uint32_t* ntok, uint32_t ablate = 0) {
    const uint32_t lane = w.lane();
    *ntok = 0;
    if (n == 0 || n > kWaveMaxDoc) return LEX_BAD;
    const uint32_t mis = (uint32_t)((uintptr_t)d & 15u);
    const uint8_t* abase = d - mis;  // 16-B aligned; byte a of the chunk stream is doc position a - mis
    const uint32_t end = mis + n;    // aligned-base offset one past the last document byte
    const uint32_t nch = (end + kWaveChunk - 1) / kWaveChunk;
    // chunk state carried from chunk to chunk (wave-uniform)
    uint32_t in_str = 0, esc = 0, pin = 0;  // pin: classes of the previous chunk's last byte
    uint32_t oq_pos = 0, oq_es = 0;         // the string open at the chunk start: its opener
    uint32_t cnt = 0;                       // tokens so far
    uint32_t bad = 0;
    uint32_t cur[4], nxt[4];
    auto load = [&](uint32_t c, uint32_t (&v)[4]) {
        const uint32_t a = c * kWaveChunk + 16u * lane;
        if (c < nch && a < end) {
            load16(abase + a, v);
        } else {
            v[0] = v[1] = v[2] = v[3] = 0u;
        }
    };
    load(0, cur);
    if (ablate == 2) {  // loads only
        uint32_t acc = 0;
        for (uint32_t c = 0; c < nch; c++) {
            load(c + 1, nxt);
            acc ^= cur[0] ^ cur[1] ^ cur[2] ^ cur[3];
#pragma unroll
            for (int j = 0; j < 4; j++) cur[j] = nxt[j];
        }
        *ntok = w.any(acc == 0x12345678u) ? 1u : 0u;
        return LEX_BAD;
    }
    for (uint32_t c = 0; c < nch; c++) {
        load(c + 1, nxt);
        const uint32_t a0 = c * kWaveChunk + 16u * lane;  // aligned offset of the lane's byte 0
        // the lane's bytes into the ring (key bytes for the label pass)
        store16(ring + (a0 & (2 * kWaveChunk - 1)), cur);
        uint32_t valid = 0xFFFFu;
        if (a0 < mis) valid &= 0xFFFFu << (mis - a0 < 16 ? mis - a0 : 16);
        if (a0 + 16 > end) valid &= a0 >= end ? 0u : (1u << (end - a0)) - 1u;
        Classes16 k = classify16(cur);
        k.q &= valid; k.bs &= valid; k.o &= valid; k.c &= valid; k.k &= valid; k.m &= valid; k.ws &= valid;
        // next lane's first 16 bytes (lane 63: the next chunk's first lane)
        uint32_t nx[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t v = w.shfl_down(cur[j]);
            const uint32_t v0 = w.readlane(nxt[j], 0);
            nx[j] = lane == 63 ? v0 : v;
        }
        // ---- escapes ----
        uint32_t E = 0;
        const bool any_bs = w.any(k.bs != 0);
        if (any_bs || esc) {
            if (w.any(k.bs == 0xFFFFu)) bad = 1;  // a 16-byte backslash run: carry chain not resolved here
            uint32_t cout0;
            escaped16(k.bs, 0u, &cout0);
            uint32_t cin = w.shfl_up(cout0);
            if (lane == 0) cin = esc;
            uint32_t cout;
            E = escaped16(k.bs, cin, &cout);
            esc = w.readlane(cout, 63);
        }
        // ---- strings ----
        const uint32_t QU = k.q & ~E;
        const uint64_t par = w.ballot((__builtin_popcount(QU) & 1u) != 0);
        const uint32_t start_in = in_str ^ (w.mbcnt(par) & 1u);
        const uint32_t instr = prefix_xor16(QU) ^ (start_in ? 0xFFFFu : 0u);
        in_str ^= (uint32_t)__builtin_popcountll(par) & 1u;
        const uint32_t Qo = QU & instr, Qc = QU & ~instr;
        const uint32_t OUT = ~instr & ~QU & valid;
        const uint32_t Ko = k.k & OUT, Mo = k.m & OUT, Oo = k.o & OUT, Co = k.c & OUT;
        const uint32_t V = OUT & ~(Ko | Mo | Oo | Co | k.ws | k.bs);
        uint32_t lbad = (k.bs | k.ws) & OUT;
        // ---- predecessor classes (the byte before each byte) ----
        const uint32_t pk = ((Qc >> 15) & 1u) | ((Ko >> 14) & 2u) | ((Mo >> 13) & 4u) | ((Oo >> 12) & 8u) |
                            ((Co >> 11) & 16u) | ((V >> 10) & 32u);
        uint32_t pprev = w.shfl_up(pk);
        if (lane == 0) pprev = pin;
        pin = w.readlane(pk, 63);
        const uint32_t PQc = ((Qc << 1) | (pprev & 1u)) & 0xFFFFu;
        const uint32_t PKo = ((Ko << 1) | ((pprev >> 1) & 1u)) & 0xFFFFu;
        const uint32_t PMo = ((Mo << 1) | ((pprev >> 2) & 1u)) & 0xFFFFu;
        const uint32_t POo = ((Oo << 1) | ((pprev >> 3) & 1u)) & 0xFFFFu;
        const uint32_t PCo = ((Co << 1) | ((pprev >> 4) & 1u)) & 0xFFFFu;
        const uint32_t PV = ((V << 1) | ((pprev >> 5) & 1u)) & 0xFFFFu;
        // ---- compact-JSON successor rules ----
        lbad |= PQc & ~(Ko | Mo | Co) & valid;
        lbad |= (PKo | PMo) & ~(Qo | Oo | V) & valid;
        lbad |= POo & ~(Qo | Oo | V | Co) & valid;
        lbad |= PCo & ~(Mo | Co) & valid;
        lbad |= PV & ~(V | Mo | Co) & valid;
        // scalars: a number (digit or '-') or exactly true / false / null
        const uint32_t Vst = V & ~PV;
        {
            uint32_t t = Vst;
            while (t) {
                const uint32_t j = ctz32(t);
                t &= t - 1;
                const uint32_t b = byte_of4(cur, j);
                if (b == '-' || (b >= '0' && b <= '9')) continue;
                // the 5 bytes at j and the byte after the literal (own 16 + next lane's 16)
                uint64_t w8 = 0;
                for (uint32_t i = 0; i < 6; i++) {
                    const uint32_t p = j + i;
                    w8 |= (uint64_t)(p < 16 ? byte_of4(cur, p) : byte_of4(nx, p - 16)) << (8 * i);
                }
                bool ok;
                if (b == 't') ok = (w8 & 0xFFFFFFFFull) == 0x65757274ull;      // "true"
                else if (b == 'f') ok = (w8 & 0xFFFFFFFFFFull) == 0x65736C6166ull;  // "false"
                else if (b == 'n') ok = (w8 & 0xFFFFFFFFull) == 0x6C6C756Eull;  // "null"
                else ok = false;
                if (ok) {  // the run ends right after the literal: the next byte is ',' '}' ']'
                    const uint32_t L = b == 'f' ? 5u : 4u;
                    const uint32_t nb = (uint32_t)(w8 >> (8 * L)) & 0xFFu;
                    ok = nb == ',' || nb == '}' || nb == ']';
                }
                if (!ok) lbad |= 1u << j;
            }
        }
        // ---- element starts and the root ----
        uint32_t ES = (POo | PMo) & valid;
        const bool root_lane = c == 0 && lane == (mis >> 4);
        if (root_lane) {
            const uint32_t b0 = 1u << (mis & 15u);
            if (!(Oo & b0)) lbad |= b0;  // the document must start with its root container
            ES |= b0;
        }
        // ---- strings whose opening quote starts an element: marked at their closing quote ----
        const uint32_t ESQ = Qo & ES;
        // the string open at this lane's start: its opener (last opening quote before the lane)
        const uint64_t hasq = w.ballot(QU != 0);
        const uint32_t lane_lastq = Qo ? 31u - (uint32_t)__builtin_clz(Qo) : 0u;
        const uint32_t lane_lastq_pos = a0 + lane_lastq - mis;
        const uint64_t lastq_es = w.ballot(Qo != 0 && ((ESQ >> lane_lastq) & 1u));
        const uint64_t below = w.lanemask_lt() & hasq;
        const uint32_t src = below ? 63u - (uint32_t)__builtin_clzll(below) : 0u;
        const uint32_t from_lane_pos = w.bpermute(lane_lastq_pos, src);
        const uint32_t open_pos = below ? from_lane_pos : oq_pos;
        const uint32_t open_es = below ? (uint32_t)((lastq_es >> src) & 1u) : oq_es;
        const uint32_t cin_es = (start_in && open_es) ? 1u : 0u;
        const uint32_t QcES = ((instr + ESQ + cin_es) & ~instr) & Qc;
        // keys: a closing quote followed by ':' (lane 15's successor is the next lane's byte 0)
        const uint32_t nk0 = byte_of4(nx, 0) == ':' ? 1u : 0u;
        const uint32_t KC = Qc & ((Ko >> 1) | (nk0 << 15));
        lbad |= KC & ~QcES;  // a key whose string is not at an element start ("a":"k":v)
        if (hasq) {
            const uint32_t top = 63u - (uint32_t)__builtin_clzll(hasq);
            oq_pos = w.readlane(lane_lastq_pos, top);
            oq_es = (uint32_t)((lastq_es >> top) & 1u);
        }
        // the last byte of the document must close the root
        if (a0 < end && a0 + 16 >= end) {
            const uint32_t jl = end - 1 - a0;
            if (!((Co >> jl) & 1u)) lbad |= 1u << jl;
        }
        if (w.any(lbad != 0)) bad = 1;
        if (ablate == 1) {
            cnt += w.any(ES != 0 || KC != 0 || QcES != 0) ? 1u : 0u;
#pragma unroll
            for (int j = 0; j < 4; j++) cur[j] = nxt[j];
            continue;
        }
        // ---- tokens ----
        const uint32_t TOK = (Qc & QcES) | (ES & ~Qo) | Co;
        uint32_t total;
        const uint32_t pre = w.excl_sum((uint32_t)__builtin_popcount(TOK), &total);
        if (bad) break;
        if (tok_base + cnt + total > tok_cap) return LEX_OVERFLOW;
        uint32_t at = tok_base + cnt + pre;
        uint32_t t = TOK;
        while (t) {
            const uint32_t j = ctz32(t);
            t &= t - 1;
            const uint32_t pos = a0 + j - mis;
            uint32_t e;
            if ((Co >> j) & 1u) {
                e = tok_make(pos, 0, byte_of4(cur, j) == ']' ? 1u : 0u, TK_CLOSE);
            } else if ((Qc >> j) & 1u) {
                const uint32_t ob = Qo & ((1u << j) - 1u);
                const uint32_t qo = ob ? a0 + (31u - (uint32_t)__builtin_clz(ob)) - mis : open_pos;
                if ((KC >> j) & 1u) {
                    const uint32_t voff = pos + 2 - qo;
                    if (voff > 0xFFu) lbad |= 1u << j;  // a key over 252 bytes
                    const uint32_t j2 = j + 2;
                    const uint32_t vb = j2 < 16 ? byte_of4(cur, j2) : byte_of4(nx, j2 - 16);
                    e = tok_make(qo, voff, value_class(vb), TK_MEMBER);
                } else {
                    e = tok_make(qo, 0, VC_STR, TK_ELEM);
                }
            } else {
                e = tok_make(pos, 0, value_class(byte_of4(cur, j)), TK_ELEM);
            }
            tok[at++] = e;
        }
        if (w.any(lbad != 0)) {
            bad = 1;
            break;
        }
        w.lds_fence();
        // ---- labels: one member token per lane ----
        for (uint32_t t0 = 0; t0 < total; t0 += 64) {
            const uint32_t ti = tok_base + cnt + t0 + lane;
            uint32_t lb = 0;
            bool kbad = false;
            if (t0 + lane < total) {
                const uint32_t e = tok[ti];
                if (tok_kind(e) == TK_MEMBER) {
                    const uint32_t qo = tok_pos(e), len = tok_voff(e) - 3u;
                    const uint32_t ka = qo + mis + 1;  // aligned offset of the key's first byte
                    if (ka + kWaveChunk < c * kWaveChunk) kbad = true;  // starts before the ring's older chunk
                    else lb = key_label(blob, ring, ka, len);
                }
                lab[ti] = (uint8_t)lb;
            }
            if (w.any(kbad)) bad = 1;
        }
        cnt += total;
        if (bad) break;
        w.lds_fence();
#pragma unroll
        for (int j = 0; j < 4; j++) cur[j] = nxt[j];
    }
    if (in_str || esc) bad = 1;
    *ntok = cnt;
    return bad ? LEX_BAD : LEX_OK;
}

// ---- phase 2: walk one request's tokens (one work-item) ------------------------------
struct Walker {
    const uint8_t* blob;
    const TrieNode* tn;
    const TrieChild* tc;
    const uint32_t* edges;
    uint32_t elog2;
    uint64_t* row;   // capture row: [0] found, [1 + s] record
    const uint8_t* d;  // the document (string values are scanned for backslashes)
    uint64_t is_arr, nodes_lo, nodes_hi, found;
    uint32_t depth;
    uint32_t cap0, cap0_start, cap1, cap1_start, ncap;  // open container captures: sel | depth << 8
    uint32_t arr0, arr1, narr;                          // live arrays with index children: depth | h << 8

    AJX_HD uint32_t node_at(uint32_t dd) const {
        if (dd == 0) return 0;
        if (dd > kFastDepth) return kNoNode;
        const uint32_t k = dd - 1;
        const uint64_t wv = k < 8 ? nodes_lo : nodes_hi;
        return (uint32_t)((wv >> ((k & 7) * 8)) & 0xFFu);
    }
    AJX_HD void set_node(uint32_t dd, uint32_t v) {
        if (dd == 0 || dd > kFastDepth) return;
        const uint32_t k = dd - 1;
        const uint64_t m = 0xFFull << ((k & 7) * 8);
        const uint64_t x = ((uint64_t)(v & 0xFF)) << ((k & 7) * 8);
        const uint64_t lo = nodes_lo, hi = nodes_hi;
        nodes_lo = k < 8 ? (lo & ~m) | x : lo;
        nodes_hi = k < 8 ? hi : (hi & ~m) | x;
    }
    AJX_HD bool top_is_arr() const { return (is_arr >> depth) & 1; }
    AJX_HD uint32_t edge(uint32_t node, uint32_t label) const {
        if (node == kNoNode || label == 0) return kNoNode;
        const uint32_t mask = (1u << elog2) - 1u;
        uint32_t at = edge_hash(node, label, elog2);
        for (uint32_t probe = 0; probe <= mask; probe++, at = (at + 1) & mask) {
            const uint32_t e = edges[at];
            if (e == kEmptyEdge) return kNoNode;
            if ((e & 0xFFFFu) == (node | (label << 8))) return (e >> 16) & 0xFFu;
        }
        return kNoNode;
    }
    // node of the element about to start in the innermost (array) container
    AJX_HD uint32_t elem_node() const {
        if (!narr) return kNoNode;
        const uint32_t parent = node_at(depth);
        if (parent == kNoNode || !(tn[parent].flags & 1)) return kNoNode;
        uint32_t h;
        if (narr >= 2 && (arr1 & 0xFF) == depth) h = arr1 >> 8;
        else if ((arr0 & 0xFF) == depth) h = arr0 >> 8;
        else return kNoNode;
        const uint32_t cb = tn[parent].child_begin, nc = tn[parent].n_children;
        for (uint32_t c = 0; c < nc; c++)
            if (tc[cb + c].array_index == (int32_t)h) return tc[cb + c].node;
        return kNoNode;
    }
    AJX_HD void element_done() {
        if (!narr || !depth || !top_is_arr()) return;
        const bool h1 = narr >= 2 && (arr1 & 0xFF) == depth;
        const bool h0 = !h1 && (arr0 & 0xFF) == depth;
        arr1 += h1 ? 0x100u : 0u;
        arr0 += h0 ? 0x100u : 0u;
    }
    AJX_HD int32_t leaf_sel(uint32_t node) const {
        if (node == kNoNode) return -1;
        const int32_t s = tn[node].selector;
        if (s < 0 || ((found >> s) & 1)) return -1;
        return s;
    }
    AJX_HD void record(int32_t s, uint32_t start, uint32_t end, uint32_t type, uint32_t esc) {
        found |= 1ull << s;
        row[1 + s] = (uint64_t)start | ((uint64_t)(((end - start) & 0xFFFFFFu) | (type << 24) | (esc << 27)) << 32);
    }
    AJX_HD bool open(bool arr, uint32_t start, uint32_t node) {
        if (depth + 1 >= 63) return false;
        depth++;
        const uint64_t bit = 1ull << depth;
        is_arr = arr ? is_arr | bit : is_arr & ~bit;
        if (node == kNoNode) {
            set_node(depth, kNoNode);
            return true;
        }
        const int32_t s = leaf_sel(node);
        const uint32_t live = tn[node].n_children ? node : kNoNode;
        if (live != kNoNode && depth > kFastDepth) return false;
        set_node(depth, live);
        if (s >= 0) {
            found |= 1ull << s;
            if (ncap >= 2) return false;
            const uint32_t v = (uint32_t)s | (depth << 8);
            if (ncap == 0) { cap0 = v; cap0_start = start; }
            else { cap1 = v; cap1_start = start; }
            ncap++;
        }
        if (arr && live != kNoNode && (tn[live].flags & 1)) {
            if (narr >= 2) return false;
            if (narr == 0) arr0 = depth;
            else arr1 = depth;
            narr++;
        }
        return true;
    }
    AJX_HD void close(uint32_t pos) {
        if (ncap) {
            const uint32_t cs = ncap == 2 ? cap1 : cap0;
            if ((cs >> 8) == depth) {
                const uint32_t start = ncap == 2 ? cap1_start : cap0_start;
                row[1 + (cs & 0xFF)] =
                    (uint64_t)start | ((uint64_t)(((pos + 1 - start) & 0xFFFFFFu) | ((uint32_t)T_JSON << 24)) << 32);
                ncap--;
            }
        }
        if (narr) {
            const uint32_t at = narr == 2 ? arr1 : arr0;
            if ((at & 0xFF) == depth) narr--;
        }
        depth--;
        element_done();  // the container was an element of its parent array
    }
};

// any '\\' in doc[a, b)
AJX_HD uint32_t has_backslash(const uint8_t* d, uint32_t a, uint32_t b) {
    for (uint32_t k = a; k < b; k += 4) {
        const uint32_t wv = load_u32_upto(d + k, b - k);
        const uint32_t m = b - k >= 4 ? 0xFFFFFFFFu : (1u << (8 * (b - k))) - 1u;
        if (eq_bytes(wv, 0x5C5C5C5Cu) & m & 0x80808080u) return 1u;
    }
    return 0u;
}

// Walk tokens [t0, t1) of a document: fills the capture row; false = not provably valid
// compact JSON (the request goes to the exact scan).
AJX_HD bool walk_doc(const uint8_t* blob, const Tables& tab, const uint32_t* tok, const uint8_t* lab, uint32_t t0,
                     uint32_t t1, const uint8_t* d, uint64_t* row) {
    const RulesetHdr* h = (const RulesetHdr*)blob;
    Walker wk;
    wk.blob = blob;
    wk.tn = tab.tn;
    wk.tc = tab.tc;
    wk.edges = (const uint32_t*)(blob + h->off_edge_slots);
    wk.elog2 = h->edge_slots_log2;
    wk.row = row;
    wk.d = d;
    wk.is_arr = 0;
    wk.nodes_lo = wk.nodes_hi = ~0ull;
    wk.found = 0;
    wk.depth = 0;
    wk.cap0 = wk.cap0_start = wk.cap1 = wk.cap1_start = wk.ncap = 0;
    wk.arr0 = wk.arr1 = wk.narr = 0;
    bool done = false;
    for (uint32_t t = t0; t < t1; t++) {
        if (done) return false;  // a token after the root closed
        const uint32_t e = tok[t];
        const uint32_t kind = tok_kind(e), pos = tok_pos(e), vc = tok_vc(e);
        if (kind == TK_CLOSE) {
            if (wk.depth == 0 || wk.top_is_arr() != (vc == 1u)) return false;
            wk.close(pos);
            done = wk.depth == 0;
            continue;
        }
        uint32_t node;
        if (wk.depth == 0) {
            if (kind != TK_ELEM || pos != 0) return false;
            node = 0;
        } else if (wk.top_is_arr()) {
            if (kind != TK_ELEM) return false;
            node = wk.elem_node();
        } else {
            if (kind != TK_MEMBER) return false;
            node = wk.edge(wk.node_at(wk.depth), lab[t]);
        }
        const uint32_t vs = pos + tok_voff(e);
        if (vc == VC_OBJ || vc == VC_ARR) {
            if (!wk.open(vc == VC_ARR, vs, node)) return false;
            continue;
        }
        if (wk.depth == 0) return false;  // a scalar root
        const int32_t s = wk.leaf_sel(node);
        if (s >= 0) {
            // the value ends at the next token's separator (',' before the next element, or
            // the closing bracket)
            if (t + 1 >= t1) return false;
            const uint32_t e2 = tok[t + 1];
            const uint32_t ve = tok_kind(e2) == TK_CLOSE ? tok_pos(e2) : tok_pos(e2) - 1u;
            uint32_t type, esc = 0;
            switch (vc) {
                case VC_STR: type = T_STRING; esc = has_backslash(d, vs + 1, ve - 1); break;
                case VC_TRUE: type = T_TRUE; break;
                case VC_FALSE: type = T_FALSE; break;
                case VC_NULL: type = T_NULL; break;
                default: type = T_NUMBER; break;
            }
            wk.record(s, vs, ve, type, esc);
        }
        wk.element_done();
    }
    if (!done) return false;
    row[0] = wk.found;
    return true;
}

}  // namespace ajx
