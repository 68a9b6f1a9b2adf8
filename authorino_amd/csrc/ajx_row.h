// ajx_row.h — the row kernel: wave-cooperative stage A (structural index, key lookup,
// selector resolution, value capture) with 16 lanes per document.
//
// A wavefront is four rows of 16 lanes; each row takes one document, so a wave works on
// four documents at once and every instruction does the same work for all of them (no
// per-document control flow: loops run as long as the busiest row needs).
//
// P1, structural index. A row reads its document 256 bytes per step, 16 aligned bytes per
// lane (coalesced: a row reads two whole 128-B lines per step), stages the bytes in LDS
// and classifies them with SWAR compares into 16-bit masks (quote, backslash,
// structural). Escapes follow the odd-backslash-run rule with the carry passed lane to
// lane (DPP); string interiors are a prefix-XOR of the unescaped quotes inside the lane
// plus the parity of the lanes before it (ballot). Every structural byte outside strings
// ({ } [ ] : ,) becomes an event (position << 3 | code) in the row's LDS event list.
// Two local rules are checked on the masks: an opening quote follows a structural byte
// and a closing quote is followed by one. With them, the bytes between two consecutive
// events are empty, exactly one string, or one scalar.
//
// P2, events, 16 per lane-round. Depth is a row prefix sum. Each event is checked against
// the JSON grammar from (its code, the gap after it, the next event's code, the kind of
// its container), so a document that passes is valid JSON up to the root's close — for
// such documents gjson v1.14.0 Get returns the first complete path match in document
// order (its parseObject / parseArray walk descends into every matching key), which is
// what is captured here. Anything else (whitespace outside strings, escaped keys on a
// selector path, nesting deeper than kRowMaxLevel, too many events, containers inside an
// array a selector indexes) goes to the exact scan (ajx_eval_scan) instead.
// The container of an event is the nearest earlier open event one level up: per level
// present in the round, a ballot of the opens at that level (in-round containers) or the
// row's level stack in LDS (containers opened in earlier rounds). Levels are resolved in
// increasing order, so a container's trie node (its key's node, looked up through the
// blob's key dictionary and transition table) is known before the keys inside it.
// A key whose node ends a selector proposes its value span with an LDS atomic min keyed
// by position: the first match in document order wins.
//
// Output: the capture row of each document (header: found bits; one record per selector:
// start | (len | type << 24 | esc << 27) << 32), the format stage B (ajx_fast.h
// patterns_from_row) and the select kernels read.
#pragma once
#include "ajx_blob.h"
#include "ajx_fast.h"
#include "ajx_wave.h"

namespace ajx {
namespace w {

constexpr uint32_t kRowLanes = 16;
constexpr uint32_t kRowsPerWave = 4;
constexpr uint32_t kRowMaxLevel = 30;  // containers nested deeper go to the exact scan
constexpr uint32_t kRowMaxSel = 64;
constexpr uint32_t kRowMaxIdxArrays = 4;  // indexed live arrays tracked per document
constexpr uint32_t kKidNone = 0xFF, kKidEsc = 0xFE;
constexpr uint32_t kNodeNone = 0xFF;

// event codes (byte -> ((b >> 4) & 6) | ((b >> 2) & 1)): ':' 2, ',' 3, '[' 4, ']' 5,
// '{' 6, '}' 7; 0 marks the end of the list
enum : uint32_t { EV_END = 0, EV_COLON = 2, EV_COMMA = 3, EV_OARR = 4, EV_CARR = 5, EV_OOBJ = 6, EV_COBJ = 7 };

// container info word: bit 0 object, bits 1..8 node, bits 9..15 captured selector + 1
// (0 none), bits 16..31 position of the open byte
AJW V info_make(M obj, V node, V capsel1, V pos) {
    return sel(obj, V(1u), V(0u)) | (node << 1) | (capsel1 << 9) | (pos << 16);
}
AJW V info_node(V i) { return (i >> 1) & 0xFFu; }
AJW V info_cap1(V i) { return (i >> 9) & 0x7Fu; }
AJW V info_pos(V i) { return i >> 16; }
AJW M info_obj(V i) { return (i & 1u) != 0u; }
constexpr uint32_t kInfoNone = kNodeNone << 1;  // an array on no selector path

// Per-wave LDS layout (byte offsets inside the wave's region; every row region is
// 16-byte aligned). docbuf rows keep 16 bytes of slack before and after the document.
struct RowLayout {
    uint32_t maxb;  // document bytes a row can hold (multiple of 256, at most 8192)
    uint32_t maxe;  // events a row can hold
    uint32_t doc, doc_stride;
    uint32_t doc2;  // a second set of document rows (the DMA of the next group), or = doc
    uint32_t ev, ev_stride;
    uint32_t bsb, bsb_stride;
    uint32_t stk, cap, misc;  // per-row strides: 32 x 4, 64 x 4, 16 x 4
    uint32_t bytes;           // the wave's whole region
};
AJW_HD RowLayout row_layout(uint32_t maxb, uint32_t maxe, bool dbuf = false) {
    RowLayout L;
    L.maxb = maxb;
    L.maxe = maxe;
    uint32_t o = 0;
    L.doc = o;
    L.doc_stride = maxb + 32;
    o += kRowsPerWave * L.doc_stride;
    L.doc2 = L.doc;
    if (dbuf) {
        L.doc2 = o;
        o += kRowsPerWave * L.doc_stride;
    }
    L.ev = o;
    L.ev_stride = ((maxe + 17) * 2 + 15) & ~15u;
    o += kRowsPerWave * L.ev_stride;
    L.bsb = o;
    L.bsb_stride = ((maxb / 256) * 2 + 15) & ~15u;
    o += kRowsPerWave * L.bsb_stride;
    L.stk = o;
    o += kRowsPerWave * 32 * 4;
    L.cap = o;
    o += kRowsPerWave * kRowMaxSel * 4;
    L.misc = o;
    o += kRowsPerWave * 16 * 4;
    L.bytes = o;
    return L;
}
// misc words per row
enum : uint32_t { MS_BADPOS = 0, MS_NIDX = 1, MS_IDX0 = 2 /* ..2+kRowMaxIdxArrays */ };

// The row tables of a ruleset (RowHdr in the blob), resolved to LDS/generic offsets.
struct RowTabs {
    Lds blob;            // the ruleset blob (LDS copy)
    uint32_t nodes;      // u32 per trie node: leaf selector + 1 (bits 0..7), bit 8 index children
    uint32_t n_nodes;
    uint32_t trans;      // u8 [n_nodes][n_kids]
    uint32_t n_kids;
    uint32_t kdict;      // KeyDictSlot[1 << kd_log2]
    uint32_t kd_log2, kd_probes;
    uint32_t idx;        // u32 per (parent, index) edge: parent | child << 8 | index << 16
    uint32_t n_idx;
    uint32_t lits;       // literal pool
    uint32_t n_sel;
};

// x >> s for a 64-bit value (hi:lo), 0 <= s < 64
AJW void shr64(V& hi, V& lo, V s) {
    const M big = s >= 32u;
    const V s1 = s & 31u;
    const V inv = (32u - s1) & 31u;
    const V lo_small = sel(s1 == 0u, lo, (lo >> s1) | (hi << inv));
    lo = sel(big, hi >> s1, lo_small);
    hi = sel(big, V(0u), hi >> s1);
}
// the 4 bytes at LDS byte offset a (any alignment)
AJW V ld32u(Lds b, V a) {
    const V q = a & ~3u;
    return alignbyte(ld32(b, q + 4u), ld32(b, q), a & 3u);
}

AJW uint32_t kdict_hash(uint32_t lo, uint32_t hi, uint32_t len, uint32_t log2) {
    uint32_t x = lo ^ ((hi << 13) | (hi >> 19)) ^ (len << 24);
    x *= 0x9E3779B1u;
    return log2 ? x >> (32 - log2) : 0u;
}
AJW V kdict_hash_v(V lo, V hi, V len, uint32_t log2) {
    V x = lo ^ ((hi << 13u) | (hi >> 19u)) ^ (len << 24u);
    x = x * 0x9E3779B1u;
    return log2 ? x >> (32u - log2) : V(0u);
}

// Grammar table: for (code, gap kind, container is object) the set of codes the next
// event may have (bit c). gap kind: 0 empty, 1 one string, 2 one scalar.
AJW V next_allowed(V code, V gk, M obj) {
    // bits: ':' 2, ',' 3, '[' 4, ']' 5, '{' 6, '}' 7
    constexpr uint32_t VAL_OPEN = (1u << 4) | (1u << 6), COMMA = 1u << 3, COLON = 1u << 2;
    constexpr uint32_t CARR = 1u << 5, COBJ = 1u << 7;
    V a = V(0u);
    // ':'  (in an object) value container | atom then ',' or '}'
    a = sel((code == EV_COLON) & obj & (gk == 0u), V(VAL_OPEN), a);
    a = sel((code == EV_COLON) & obj & (gk != 0u), V(COMMA | COBJ), a);
    // ','  object: a key then ':' ; array: a value container | atom then ',' or ']'
    a = sel((code == EV_COMMA) & obj & (gk == 1u), V(COLON), a);
    a = sel((code == EV_COMMA) & !obj & (gk == 0u), V(VAL_OPEN), a);
    a = sel((code == EV_COMMA) & !obj & (gk != 0u), V(COMMA | CARR), a);
    // '['  empty | first element
    a = sel((code == EV_OARR) & (gk == 0u), V(VAL_OPEN | CARR), a);
    a = sel((code == EV_OARR) & (gk != 0u), V(COMMA | CARR), a);
    // '{'  empty | first key
    a = sel((code == EV_OOBJ) & (gk == 0u), V(COBJ), a);
    a = sel((code == EV_OOBJ) & (gk == 1u), V(COLON), a);
    // '}' / ']' closing a container of their own kind: then ',' or a close
    a = sel((code == EV_CARR) & !obj & (gk == 0u), V(COMMA | CARR | COBJ), a);
    a = sel((code == EV_COBJ) & obj & (gk == 0u), V(COMMA | CARR | COBJ), a);
    return a;
}

// Outputs of one wave-iteration (four documents).
struct RowResult {
    M ok;        // the row's document was captured (false: exact scan)
};

// Stage A of the row kernel for the wave's four documents. `len`/`mis` per lane are the
// row's document length and start misalignment (address & 15); `load(b, m)` returns block
// b (16 aligned bytes, b counted from the document's first aligned block) of each lane's
// document. wl = the wave's LDS region. On return the capture data of each row is in
// the row's cap words (start << 16 | end per selector, ~0 none) and `ok` says which rows
// hold a valid capture.
// PRE: the rows' documents are in the document rows at `docoff` already (the kernel's
// LDS-DMA of the group); otherwise `load` reads them and P1 stores them there.
template <bool PRE = false, class Load>
AJW M row_scan(const RowTabs& T, Lds wl, const RowLayout& L, M live, V len, V mis, Load load, uint32_t stop = 0,
               uint32_t docoff = 0xFFFFFFFFu) {
    if (docoff == 0xFFFFFFFFu) docoff = L.doc;
    const V ln = lane(), row = ln >> 4, rl = ln & 15u;
    const V dbase = docoff + row * L.doc_stride + 16u;  // docbuf offset of aligned byte 0
    const V ebase = L.ev + row * L.ev_stride;
    const V bbase = L.bsb + row * L.bsb_stride;
    const V sbase = L.stk + row * (32u * 4u);
    const V cbase = L.cap + row * (kRowMaxSel * 4u);
    const V mbase = L.misc + row * (16u * 4u);
    const V nblk = sel(len != 0u, (len + mis + 15u) >> 4, V(0u));
    M ok = live & (len != 0u) & (nblk * 16u <= L.maxb);

    // ---- row state in LDS: captures none, stack none, misc cleared
#pragma unroll
    for (uint32_t k = 0; k < kRowMaxSel / 16; k++) st32(wl, M(true), cbase + (rl + 16u * k) * 4u, V(0xFFFFFFFFu));
    st32(wl, M(true), sbase + rl * 4u, V(kInfoNone));
    st32(wl, M(true), sbase + (rl + 16u) * 4u, V(kInfoNone));
    st32(wl, M(true), mbase + rl * 4u, sel(rl == MS_BADPOS, V(0xFFFFFFFFu), V(0u)));
    lds_fence();

    // ---- P1: structural index
    const V nsp = (nblk + 15u) >> 4;
    uint32_t nsp_max = 0;
    {
        V t = sel(ok, nsp, V(0u));
        t = row_max(t);
        t = row_bcast15(t);
        nsp_max = readlane(t, 15);
        nsp_max = nsp_max > readlane(t, 31) ? nsp_max : readlane(t, 31);
        nsp_max = nsp_max > readlane(t, 47) ? nsp_max : readlane(t, 47);
        nsp_max = nsp_max > readlane(t, 63) ? nsp_max : readlane(t, 63);
    }
    V c_esc = V(0u), c_str = V(0u), c_s15 = V(0u), c_qc15 = V(0u), c_cnt = V(0u);
    G16 nx;
    if (!PRE) nx = load(rl, ok & (rl < nblk));
    for (uint32_t sp = 0; sp < nsp_max; sp++) {
        const V b = sp * 16u + rl;
        const M vb = ok & (b < nblk);
        G16 x;
        if (PRE) {
            x = ld128(wl, dbase + sel(vb, b, V(0u)) * 16u);
        } else {
            x = nx;
            const V bn = b + 16u;
            nx = load(bn, ok & (bn < nblk));
            st128(wl, vb, dbase + b * 16u, x.x, x.y, x.z, x.w);
        }
        // valid bytes of the block: doc positions b*16 - mis + k in [0, len)
        const V lo = sel(b == 0u, mis, V(0u));
        const V hi_raw = len + mis - b * 16u;  // (vb: > 0)
        const V hi = sel(hi_raw > 16u, V(16u), hi_raw);
        const V vm = sel(vb, ((1u << hi) - 1u) & ~((1u << lo) - 1u), V(0u)) & 0xFFFFu;
        // classification
        V qf[4], bf[4], sf[4];
        const V xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const V xx = xs[k];
            const V lx = xx | 0x20202020u;
            qf[k] = eq_bytes(xx, 0x22222222u);
            bf[k] = eq_bytes(xx, 0x5C5C5C5Cu);
            sf[k] = eq_bytes(lx, 0x7B7B7B7Bu) | eq_bytes(lx, 0x7D7D7D7Du) | eq_bytes(xx, 0x3A3A3A3Au) |
                    eq_bytes(xx, 0x2C2C2C2Cu);
        }
        const V Q = gather16(qf[0], qf[1], qf[2], qf[3]) & vm;
        const V BS = gather16(bf[0], bf[1], bf[2], bf[3]) & vm;
        const V S = gather16(sf[0], sf[1], sf[2], sf[3]) & vm;
        const V p0 = b * 16u - mis;  // doc position of the block's byte 0 (wraps for b = 0)
        V bad = V(0u);
        // escapes: the byte after an odd backslash run (carry from the previous lane)
        V escaped = V(0u);
        const uint64_t bsb_ballot = ballot(BS != 0u);
        if (bsb_ballot != 0 || any(c_esc != 0u)) {
            const M allbs = (vm == 0xFFFFu) & (BS == 0xFFFFu);
            bad = bad | sel(allbs, V(1u), V(0u));  // (a run across a whole lane: exact scan)
            auto esc_of = [&](V bsv, V cin, V& cout) -> V {
                const V bsx = bsv & ~cin;
                const V follows = ((bsx << 1) | cin) & 0xFFFFu;
                const V odd_starts = bsx & ~0x5555u & ~follows;
                const V seq = odd_starts + bsx;  // (17 bits: bit 16 = the run leaves the lane)
                cout = (seq >> 16) & 1u;
                return ((0x5555u ^ ((seq << 1) & 0xFFFFu)) & follows) & 0xFFFFu;
            };
            V co0;
            (void)esc_of(BS, V(0u), co0);
            const V cin = sel(rl == 0u, c_esc, row_shr<1>(co0));
            V co;
            escaped = esc_of(BS, cin, co);
            c_esc = row_bcast15(co) & sel(ok, V(1u), V(0u));
        }
        st16(wl, vb & (rl == 0u), bbase + sp * 2u, row_bits(bsb_ballot, row));
        // strings
        const V U = Q & ~escaped;
        V px = U;
        px = px ^ (px << 1);
        px = px ^ (px << 2);
        px = px ^ (px << 4);
        px = px ^ (px << 8);
        px = px & 0xFFFFu;
        const V pb = row_bits(ballot((popc(U) & 1u) != 0u), row);
        const V flip = (popc(pb & ((1u << rl) - 1u)) & 1u) ^ c_str;
        const V instr = px ^ sel(flip != 0u, V(0xFFFFu), V(0u));  // inside a string after byte k
        c_str = c_str ^ (popc(pb) & 1u);
        const V QO = U & instr, QC = U & ~instr;
        const V outside = ~instr & ~U & vm & 0xFFFFu;
        const V So = S & outside;
        bad = bad | (BS & outside);
        const V prevS = ((So << 1) | sel(rl == 0u, c_s15, row_shr<1>(So >> 15))) & 0xFFFFu;
        bad = bad | (QO & ~prevS);
        const V prevQC = ((QC << 1) | sel(rl == 0u, c_qc15, row_shr<1>(QC >> 15))) & 0xFFFFu;
        bad = bad | (prevQC & ~So & vm);
        c_s15 = row_bcast15(So >> 15);
        c_qc15 = row_bcast15(QC >> 15);
        min32(wl, vb & (bad != 0u), mbase + MS_BADPOS * 4u, p0 + ctz(bad));
        // events
        V E = So;
        const V cnt = popc(E);
        const V incl = row_sum(cnt);
        V idx = c_cnt + incl - cnt;
        c_cnt = c_cnt + row_bcast15(incl);
        while (any(E != 0u)) {
            const M m = E != 0u;
            const V k = ctz(E);
            E = E & (E - 1u);
            const V kw = k >> 2;
            const V wd = sel(kw == 0u, x.x, sel(kw == 1u, x.y, sel(kw == 2u, x.z, x.w)));
            const V byte = (wd >> ((k & 3u) << 3)) & 0xFFu;
            const V code = ((byte >> 4) & 6u) | ((byte >> 2) & 1u);
            st16(wl, m & (idx < L.maxe), ebase + idx * 2u, ((p0 + k) << 3) | code);
            idx = idx + sel(m, V(1u), V(0u));
        }
    }
    AJW_TRACE(ok & ((c_cnt > L.maxe) | (c_cnt == 0u)), "event count");
    ok = ok & (c_cnt <= L.maxe) & (c_cnt != 0u);
    const V cnt = sel(ok, c_cnt, V(0u));
    st16(wl, ok & (rl == 0u), ebase + cnt * 2u, V(0u));  // END
    lds_fence();
    {  // the root: an open at byte 0
        const V e0 = ld16(wl, ebase);
        AJW_TRACE(ok & !(((e0 & 7u) >= 4u) & ((e0 & 1u) == 0u) & ((e0 >> 3) == 0u)), "root not at byte 0");
        ok = ok & ((e0 & 7u) >= 4u) & ((e0 & 1u) == 0u) & ((e0 >> 3) == 0u);
    }

    AJW_TRACE(live & !ok, "not ok after P1");
    if (stop == 1) return ok;  // (profiling: P1 alone)
    // ---- P2: events
    const V nr = (cnt + 15u) >> 4;
    uint32_t nr_max = 0;
    {
        V t = row_max(sel(ok, nr, V(0u)));
        t = row_bcast15(t);
        for (uint32_t r = 0; r < 4; r++) nr_max = nr_max > readlane(t, 16 * r) ? nr_max : readlane(t, 16 * r);
    }
    V dc = V(0u), pcode = V(0u), ppos = V(0u), pnode = V(kNodeNone);
    M done = M(false);
    V rootpos = V(0u);
    M rej = M(false);
    const V dmis = dbase + mis;  // docbuf offset of document position 0
    for (uint32_t rr = 0; rr < nr_max; rr++) {
        const V i = rr * 16u + rl;
        M act = ok & !done & (i < cnt);
        const V e = ld16(wl, ebase + i * 2u), en = ld16(wl, ebase + i * 2u + 2u);
        const V code = e & 7u, pos = e >> 3, ncode = en & 7u, npos = en >> 3;
        const M isopen = (code >= 4u) & ((code & 1u) == 0u);
        const M isclose = (code >= 5u) & ((code & 1u) == 1u);
        const M iscolon = code == (V)EV_COLON;
        V delta = sel(act & isopen, V(1u), sel(act & isclose, V(0xFFFFFFFFu), V(0u)));
        const V incl = row_sum(delta);
        const V pre = dc + incl - delta, post = pre + delta;
        // the root's close ends the document: later events are not looked at
        const V rc = row_bits(ballot(act & isclose & (post == 0u)), row);
        const V first_rc = ctz(rc);
        act = act & (rl <= first_rc);
        const M is_root_close = act & (rl == first_rc);
        rej = rej | (act & (post > kRowMaxLevel));
        AJW_TRACE(act & (post > kRowMaxLevel), "too deep");
        const V prv_pos = sel(rl == 0u, ppos, row_shr<1>(pos));
        const V prv_code = sel(rl == 0u, pcode, row_shr<1>(code));
        // the gap after the event: empty, one string or one scalar
        const M need_gap = act & !is_root_close;
        rej = rej | (need_gap & (ncode == (V)EV_END));  // the root never closes
        AJW_TRACE(need_gap & (ncode == (V)EV_END), "root never closes");
        const V gs = pos + 1u;
        const V gl = npos - gs;
        const V b1 = ld8(wl, dmis + sel(need_gap, gs, V(0u)));
        const V gk = sel(gl == 0u, V(0u), sel(b1 == 0x22u, V(1u), V(2u)));
        M sc_ok = M(true);
        if (any(need_gap & (gk == 2u))) {
            const M g2 = need_gap & (gk == 2u);
            const V w0 = ld32u(wl, dmis + sel(g2, gs, V(0u)));
            const V b4 = ld8(wl, dmis + sel(g2, gs + 4u, V(0u)));
            const V last = ld8(wl, dmis + sel(g2, npos - 1u, V(0u)));
            const M lit = ((b1 == 0x74u) & (gl == 4u) & (w0 == 0x65757274u)) |
                          ((b1 == 0x66u) & (gl == 5u) & (w0 == 0x736C6166u) & (b4 == 0x65u)) |
                          ((b1 == 0x6Eu) & (gl == 4u) & (w0 == 0x6C6C756Eu));
            const M num = ((b1 == 0x2Du) | ((b1 - 0x30u) < 10u)) & (last > 0x20u);
            sc_ok = !g2 | lit | num;
        }
        // key lookup for colons: the key is the string between the previous event and the ':'
        V kid = V(kKidNone);
        const M colon = act & iscolon;
        if (any(colon)) {
            const V ks = prv_pos + 2u, ke = pos - 1u;
            const M kv = colon & (prv_pos + 3u <= pos);
            const V klen = sel(kv, ke - ks, V(0u));
            // the key's last 8 bytes (bytes before ks are masked off below)
            const V a = dmis + sel(kv, ke, V(8u)) - 8u;
            const V q = a & ~3u, sh = a & 3u;
            const V w0 = ld32(wl, q), w1 = ld32(wl, q + 4u), w2 = ld32(wl, q + 8u);
            V slo = alignbyte(w1, w0, sh), shi = alignbyte(w2, w1, sh);
            const V cut = sel(klen < 8u, (8u - klen) * 8u, V(0u));
            shr64(shi, slo, cut & 63u);
            slo = sel(klen == 0u, V(0u), slo);
            shi = sel(klen == 0u, V(0u), shi);
            const V slot0 = kdict_hash_v(slo, shi, klen, T.kd_log2);
            const uint32_t dmask = (1u << T.kd_log2) - 1u;
            M found = M(false);
            for (uint32_t t = 0; t < T.kd_probes; t++) {
                const V so = T.kdict + ((slot0 + t) & dmask) * 16u;
                const V e_lo = ld32(T.blob, so), e_hi = ld32(T.blob, so + 4u), meta = ld32(T.blob, so + 8u);
                const V koff = ld32(T.blob, so + 12u);
                M hit = kv & !found & (meta != 0xFFFFFFFFu) & (e_lo == slo) & (e_hi == shi) &
                        ((meta & 0xFFFFu) == klen);
                // keys longer than 8 bytes: the rest compared with the literal (keys that
                // share their last 8 bytes and length sit in later slots)
                M need = hit & (klen > 8u);
                V j = V(0u);
                while (any(need)) {
                    const V r = klen - 8u - j;  // bytes left (> 0)
                    const V dw = ld32u(wl, dmis + sel(need, ks + j, V(0u)));
                    const V lw = ld32(T.blob, T.lits + sel(need, koff + j, V(0u)));
                    const V msk = sel(r >= 4u, V(0xFFFFFFFFu), (1u << (r << 3)) - 1u);
                    const M diff = need & (((dw ^ lw) & msk) != 0u);
                    hit = hit & !diff;
                    j = j + 4u;
                    need = need & !diff & (j < klen - 8u);
                }
                kid = sel(hit, (meta >> 16) & 0xFFu, kid);
                found = found | hit;
            }
            // a key with a backslash: its unescaped text is not compared here
            {
                const V b0 = (ks + mis) >> 4, b1k = (ke + mis + 15u) >> 4;  // blocks [b0, b1k)
                M chk = kv;
                M has = M(false);
                V bk = b0;
                while (any(chk)) {
                    const V word = ld16(wl, bbase + ((bk >> 4) << 1));
                    has = has | (chk & (((word >> (bk & 15u)) & 1u) != 0u));
                    bk = bk + 1u;
                    chk = chk & !has & (bk < b1k);
                }
                M esc = M(false);
                if (any(has)) {
                    V jj = V(0u);
                    M scan = has;
                    while (any(scan)) {
                        const V dw = ld32u(wl, dmis + sel(scan, ks + jj, V(0u)));
                        const V r = klen - jj;
                        const V msk = sel(r >= 4u, V(0xFFFFFFFFu), (1u << (r << 3)) - 1u);
                        esc = esc | (scan & ((eq_bytes(dw, 0x5C5C5C5Cu) & msk) != 0u));
                        jj = jj + 4u;
                        scan = scan & !esc & (jj < klen);
                    }
                }
                kid = sel(esc, V(kKidEsc), kid);
            }
        }
        // containers, level by level (a container's node before the keys inside it)
        V Lmin_v = row_max(sel(act, 64u - pre, V(0u)));
        V Lmax_v = row_max(sel(act, vmax(pre, post), V(0u)));
        Lmin_v = row_bcast15(Lmin_v);
        Lmax_v = row_bcast15(Lmax_v);
        uint32_t Lmin = 64, Lmax = 0;
        for (uint32_t r = 0; r < 4; r++) {
            const uint32_t a = 64u - readlane(Lmin_v, 16 * r), bmax = readlane(Lmax_v, 16 * r);
            if (readlane(Lmin_v, 16 * r) != 0u && a < Lmin) Lmin = a;
            if (bmax > Lmax) Lmax = bmax;
        }
        if (Lmax > kRowMaxLevel) Lmax = kRowMaxLevel;
        V ctx = V(kInfoNone), myinfo = V(kInfoNone), node = V(kNodeNone);
        for (uint32_t Lv = Lmin; Lv <= Lmax; Lv++) {
            const M needctx = act & (pre == Lv);
            const M opensL = act & isopen & (post == Lv);
            const V OL = row_bits(ballot(opensL), row);
            const V cand = OL & ((1u << rl) - 1u);
            const V sv = ld32(wl, sbase + Lv * 4u);
            // the node of each open at this level: its key's (the ':' just before it), the
            // root's, or none (an element of an array: only atoms of indexed arrays are
            // resolved, in the post pass)
            const V onode_key = sel(rl == 0u, pnode, row_shr<1>(node));
            const M owner_colon = prv_code == (V)EV_COLON;
            V onode = sel(Lv == 1u ? M(true) : M(false), V(0u), sel(owner_colon, onode_key, V(kNodeNone)));
            onode = sel(onode < T.n_nodes, onode, V(kNodeNone));
            const V ninfo = ld32(T.blob, T.nodes + sel(onode < T.n_nodes, onode, V(0u)) * 4u);
            const V capsel1 = sel(onode < T.n_nodes, ninfo & 0xFFu, V(0u));
            const M idxarr = opensL & (onode < T.n_nodes) & (((ninfo >> 8) & 1u) != 0u) & (code == (V)EV_OARR);
            // an element container inside an indexed array: exact scan
            {
                const V pn = info_node(ctx);
                const V pinfo = ld32(T.blob, T.nodes + sel(pn < T.n_nodes, pn, V(0u)) * 4u);
                rej = rej | (opensL & !owner_colon & (Lv > 1u) & (pn < T.n_nodes) & (((pinfo >> 8) & 1u) != 0u));
                AJW_TRACE(opensL & !owner_colon & (Lv > 1u) & (pn < T.n_nodes) & (((pinfo >> 8) & 1u) != 0u),
                          "container element of an indexed array");
            }
            myinfo = sel(opensL, info_make(code == (V)EV_OOBJ, onode, capsel1, pos), myinfo);
            // indexed arrays: remembered for the post pass
            if (any(idxarr)) {
                const V nidx = ld32(wl, mbase + MS_NIDX * 4u);
                const V ib = row_bits(ballot(idxarr), row);
                const V before = popc(ib & ((1u << rl) - 1u));
                const V tot = popc(ib);
                const V slot = nidx + before;
                st32(wl, idxarr & (slot < kRowMaxIdxArrays), mbase + (MS_IDX0 + slot) * 4u, i | (onode << 16));
                rej = rej | (idxarr & (slot >= kRowMaxIdxArrays));
                AJW_TRACE(idxarr & (slot >= kRowMaxIdxArrays), "indexed arrays");
                st32(wl, (rl == 0u) & (tot != 0u), mbase + MS_NIDX * 4u, nidx + tot);
            }
            // the row's last open at this level is the level's container for later rounds
            const M last = opensL & ((OL >> (rl + 1u)) == 0u);
            st32(wl, last, sbase + Lv * 4u, myinfo);
            const V cl = hibit(cand) & 15u;
            const V inr = shfl(myinfo, (row << 4) | cl);
            ctx = sel(needctx, sel(cand != 0u, inr, sv), ctx);
            // keys at this level
            const V cnode = info_node(ctx);
            const M colonL = needctx & iscolon;
            const M live_ctx = cnode < T.n_nodes;
            rej = rej | (colonL & live_ctx & (kid == kKidEsc));
            AJW_TRACE(colonL & live_ctx & (kid == kKidEsc), "escaped key on a selector path");
            const M look = colonL & live_ctx & (kid < T.n_kids);
            const V tn = ld8(T.blob, T.trans + sel(look, cnode * T.n_kids + kid, V(0u)));
            node = sel(colonL, sel(look & (tn < T.n_nodes), tn, V(kNodeNone)), node);
            // a key ending a selector proposes its value: (start << 16 | end), end 0 for a
            // container (set at its close)
            const V kinfo = ld32(T.blob, T.nodes + sel(node < T.n_nodes, node, V(0u)) * 4u);
            const M leaf = colonL & (node < T.n_nodes) & ((kinfo & 0xFFu) != 0u);
            const M cont_val = (ncode == (V)EV_OARR) | (ncode == (V)EV_OOBJ);
            min32(wl, leaf, cbase + ((kinfo & 0xFFu) - 1u) * 4u, (gs << 16) | sel(cont_val, V(0u), npos));
            // a captured container closing: its end
            const M closeL = needctx & isclose & (info_cap1(ctx) != 0u);
            if (any(closeL)) {
                const V co = cbase + ((info_cap1(ctx) - 1u) & 63u) * 4u;
                const V cur = ld32(wl, co);
                st32(wl, closeL & ((cur >> 16) == info_pos(ctx)), co, (info_pos(ctx) << 16) | (pos + 1u));
            }
        }
        // grammar
        const M obj = info_obj(ctx);
        const V allowed = next_allowed(code, gk, obj);
        const M tr_ok = ((allowed >> ncode) & 1u) != 0u;
        const M close_ok = obj == (code == (V)EV_COBJ);
        const M valid = sel(is_root_close, sel(close_ok, V(1u), V(0u)), sel(tr_ok & sc_ok, V(1u), V(0u))) != 0u;
        rej = rej | (act & !valid);
        AJW_TRACE(act & !valid, "grammar");
        AJW_TRACEV(act & !valid, "  round", V(rr));
        AJW_TRACEV(act & !valid, "  code", code);
        AJW_TRACEV(act & !valid, "  pos", pos);
        AJW_TRACEV(act & !valid, "  ncode", ncode);
        AJW_TRACEV(act & !valid, "  gk", gk);
        AJW_TRACEV(act & !valid, "  ctx", ctx);
        AJW_TRACEV(act & !valid, "  pre", pre);
        // carries
        rootpos = sel(is_root_close, pos, rootpos);
        rootpos = row_bcast15(row_max(rootpos));
        done = done | (rc != 0u);
        dc = row_bcast15(post);
        pcode = row_bcast15(code);
        ppos = row_bcast15(pos);
        pnode = row_bcast15(node);
        lds_fence();
    }
    {
        const V rj = row_max(sel(rej, V(1u), V(0u)));
        AJW_TRACE(ok & !done, "root not closed");
        ok = ok & done & (row_bcast15(rj) == 0u);
    }
    // problems P1 saw before the root's close
    AJW_TRACE(ok & (ld32(wl, mbase + MS_BADPOS * 4u) <= rootpos), "P1 local rule");
    ok = ok & (ld32(wl, mbase + MS_BADPOS * 4u) > rootpos);

    AJW_TRACE(live & !ok, "not ok after P2");
    if (stop == 2) return ok;  // (profiling: P1 + P2)
    // ---- post pass: atoms of indexed arrays. Element k of an array whose events right
    // after its open are k commas is the gap after the k-th one (the open for k = 0).
    if (T.n_idx != 0) {
        const V nidx = sel(ok, ld32(wl, mbase + MS_NIDX * 4u), V(0u));
        for (uint32_t a = 0; a < kRowMaxIdxArrays; a++) {
            if (!any(nidx > a)) break;
            const M has = nidx > a;
            const V ent = ld32(wl, mbase + (MS_IDX0 + a) * 4u);
            const V oi = ent & 0xFFFFu, anode = ent >> 16;
            for (uint32_t j0 = 0; j0 < T.n_idx; j0 += 16) {
                const V j = j0 + rl;
                const V edge = ld32(T.blob, T.idx + sel(j < T.n_idx, j, V(0u)) * 4u);
                M m = has & (j < T.n_idx) & ((edge & 0xFFu) == anode);
                const V child = (edge >> 8) & 0xFFu, k = edge >> 16;
                // walk the k separators
                V t = V(1u);
                M walk = m & (k != 0u);
                while (any(walk)) {
                    const V ec = ld16(wl, ebase + sel(walk, oi + t, V(0u)) * 2u) & 7u;
                    const M sep = ec == (V)EV_COMMA;
                    rej = rej | (walk & ((ec == (V)EV_OARR) | (ec == (V)EV_OOBJ)));  // a container first
                    m = m & (!walk | sep);  // (the array ended before element k: no element)
                    t = t + sel(walk & sep, V(1u), V(0u));
                    walk = walk & sep & (t <= k);
                }
                const V se = ld16(wl, ebase + sel(m, oi + k, V(0u)) * 2u);
                const V ne = ld16(wl, ebase + sel(m, oi + k + 1u, V(0u)) * 2u);
                const V nc = ne & 7u;
                const V st = (se >> 3) + 1u, en2 = ne >> 3;
                rej = rej | (m & ((nc == (V)EV_OARR) | (nc == (V)EV_OOBJ)));  // element k is a container
                const M atom = m & ((nc == (V)EV_COMMA) | (nc == (V)EV_CARR)) & (en2 > st);
                const V cinfo = ld32(T.blob, T.nodes + sel(child < T.n_nodes, child, V(0u)) * 4u);
                const M leaf = atom & (child < T.n_nodes) & ((cinfo & 0xFFu) != 0u);
                min32(wl, leaf, cbase + ((cinfo & 0xFFu) - 1u) * 4u, (st << 16) | en2);
            }
        }
        const V rj = row_max(sel(rej, V(1u), V(0u)));
        ok = ok & (row_bcast15(rj) == 0u);
    }
    return ok;
}

// The row tables of the ruleset at `gblob` (uniform header reads) for a copy of it at `lblob`.
AJW RowTabs row_tabs(const uint8_t* gblob, Lds lblob) {
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(gblob);
    const RowHdr* rh = reinterpret_cast<const RowHdr*>(gblob + h->off_row);
    RowTabs T;
    T.blob = lblob;
    T.nodes = rh->off_nodes;
    T.n_nodes = rh->n_nodes;
    T.trans = rh->off_trans;
    T.n_kids = rh->n_kids;
    T.kdict = rh->off_kdict;
    T.kd_log2 = rh->kd_log2;
    T.kd_probes = rh->kd_probes;
    T.idx = rh->off_idx;
    T.n_idx = rh->n_idx;
    T.lits = h->off_literals;
    T.n_sel = h->n_selectors;
    return T;
}

// The capture records of the rows after row_scan: each found selector's value type and
// escape flag from its bytes. emit(s, m, found, start, len, type, esc) is called for the
// selectors s = s0 + lane-in-row of every chunk of 16; rows whose captured number holds
// whitespace (gjson would stop there) are dropped from `ok`. hdr_lo/hdr_hi: the found
// bits of the row.
template <class Emit>
AJW M row_finish(const RowTabs& T, Lds wl, const RowLayout& L, M ok, V mis, V& hdr_lo, V& hdr_hi, Emit emit,
                 uint32_t docoff = 0xFFFFFFFFu) {
    if (docoff == 0xFFFFFFFFu) docoff = L.doc;
    const V ln = lane(), row = ln >> 4, rl = ln & 15u;
    const V dbase = docoff + row * L.doc_stride + 16u;
    const V dmis = dbase + mis;
    const V bbase = L.bsb + row * L.bsb_stride;
    const V cbase = L.cap + row * (kRowMaxSel * 4u);
    M rej = M(false);
    hdr_lo = V(0u);
    hdr_hi = V(0u);
    for (uint32_t s0 = 0; s0 < T.n_sel; s0 += 16) {
        const V s = s0 + rl;
        const M m = ok & (s < T.n_sel);
        const V c = ld32(wl, cbase + sel(m, s, V(0u)) * 4u);
        const M found = m & (c != 0xFFFFFFFFu);
        const V start = c >> 16, end = c & 0xFFFFu;
        rej = rej | (found & (end <= start));
        AJW_TRACE(found & (end <= start), "empty capture");
        const V b0 = ld8(wl, dmis + sel(found, start, V(0u)));
        V type = V(T_NUMBER);
        type = sel(b0 == 0x22u, V(T_STRING), type);
        type = sel((b0 == 0x7Bu) | (b0 == 0x5Bu), V(T_JSON), type);
        type = sel(b0 == 0x74u, V(T_TRUE), type);
        type = sel(b0 == 0x66u, V(T_FALSE), type);
        type = sel(b0 == 0x6Eu, V(T_NULL), type);
        // strings: a backslash inside (the blocks P1 saw one in, then the bytes)
        M esc = M(false);
        {
            const M str = found & (type == (V)T_STRING);
            const V blo = (start + mis) >> 4, bhi = (end + mis + 15u) >> 4;
            M chk = str;
            M hasb = M(false);
            V bk = blo;
            while (any(chk)) {
                const V word = ld16(wl, bbase + ((bk >> 4) << 1));
                hasb = hasb | (chk & (((word >> (bk & 15u)) & 1u) != 0u));
                bk = bk + 1u;
                chk = chk & !hasb & (bk < bhi);
            }
            V j = start + 1u;
            M scan = hasb & (j + 1u < end);
            while (any(scan)) {
                const V r = end - 1u - j;
                const V dw = ld32u(wl, dmis + sel(scan, j, V(0u)));
                const V msk = sel(r >= 4u, V(0xFFFFFFFFu), (1u << (r << 3)) - 1u);
                esc = esc | (scan & ((eq_bytes(dw, 0x5C5C5C5Cu) & msk) != 0u));
                j = j + 4u;
                scan = scan & !esc & (j + 1u < end);
            }
        }
        // numbers: no byte <= 0x20 inside (gjson's parseNumber stops at whitespace)
        {
            V j = start;
            M scan = found & (type == (V)T_NUMBER);
            while (any(scan)) {
                const V r = end - j;
                const V dw = ld32u(wl, dmis + sel(scan, j, V(0u)));
                const V msk = sel(r >= 4u, V(0xFFFFFFFFu), (1u << (r << 3)) - 1u);
                const V t = (dw & 0x7F7F7F7Fu) + 0x5F5F5F5Fu;  // 0x80 in bytes <= 0x20 (with ~(t | dw))
                rej = rej | (scan & (((~(t | dw)) & 0x80808080u & msk) != 0u));
                AJW_TRACE(scan & (((~(t | dw)) & 0x80808080u & msk) != 0u), "number with whitespace");
                j = j + 4u;
                scan = scan & (j < end);
            }
        }
        // the finished record for stage B: start | end << 13 | type << 26 | esc << 29 | 1 << 30
        st32(wl, m, cbase + s * 4u,
             sel(found, start | (end << 13) | (type << 26) | sel(esc, V(1u << 29), V(0u)) | (1u << 30), V(0u)));
        const V fb = row_bits(ballot(found), row);
        hdr_lo = hdr_lo | sel(V(s0) < 32u, fb << (s0 & 31u), V(0u));
        hdr_hi = hdr_hi | sel(V(s0) >= 32u, fb << (s0 & 31u), V(0u));
        emit(s, m, found, start, end - start, type, sel(esc, V(1u), V(0u)));
    }
    const V rj = row_max(sel(rej, V(1u), V(0u)));
    return ok & (row_bcast15(rj) == 0u);
}

// Stage B in the row kernel: Pattern.Matches (pkg/jsonexp/expressions.go:59-96) of every
// pattern on its selector's value, 16 patterns per row at a time (lane k of a row takes
// patterns k, k + 16, ...), the values read from the row's LDS copy of the document;
// then the T bitmap and the And/Or fold of every tree (expressions.go:111-154), one tree
// per lane. `blob` is a generic pointer to the blob copy the tables are read from. A row
// whose value only the exact scan decides (a number beyond the device's plain forms)
// comes back false. out(r, k, tri, err) writes tree k's result; bm(r, word, bits) the
// bitmap words.
template <class OutFn, class BmFn>
AJW M row_patterns(const uint8_t* blob, Lds wl, const RowLayout& L, M ok, V mis, V r, OutFn out, BmFn bm,
                   uint32_t bm_words, uint32_t docoff = 0xFFFFFFFFu) {
    if (docoff == 0xFFFFFFFFu) docoff = L.doc;
    const V ln = lane(), row = ln >> 4, rl = ln & 15u;
    const V dmis = docoff + row * L.doc_stride + 16u + mis;
    const V cbase = L.cap + row * (kRowMaxSel * 4u);
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
    const Pattern* pats = reinterpret_cast<const Pattern*>(blob + h->off_patterns);
    const uint8_t* lits = blob + h->off_literals;
    const uint32_t np = h->n_patterns < 128u ? h->n_patterns : 128u;
    V tw[4] = {V(0u), V(0u), V(0u), V(0u)}, uw[4] = {V(0u), V(0u), V(0u), V(0u)};
    for (uint32_t p0 = 0; p0 < np; p0 += 16) {
        const V p = p0 + rl;
        const M m = ok & (p < np);
        V res = V((uint32_t)V_F);
        AJW_LANES(m) {
            const uint32_t pi = AJW_L(p);
            const Pattern pt = pats[pi];
            uint8_t rv;
            if (pt.state != P_OK) {
                rv = pt.state == P_STATIC_E ? V_E : V_U;
            } else {
                const uint8_t* doc = gptr(wl, AJW_L(dmis));
                const uint32_t rec = *reinterpret_cast<const uint32_t*>(gptr(wl, AJW_L(cbase) + pt.selector * 4u));
                if (!((rec >> 30) & 1u)) {
                    const uint64_t nt = h->null_true[pi >> 6];
                    rv = ((nt >> (pi & 63)) & 1u) ? V_T : V_F;
                } else {
                    ValueRef v;
                    v.start = rec & 0x1FFFu;
                    v.end = (rec >> 13) & 0x1FFFu;
                    v.type = (uint8_t)((rec >> 26) & 7u);
                    v.esc = (uint8_t)((rec >> 29) & 1u);
                    const RawVal raw = raw_value(doc, v);
                    if (raw.ok && (pt.op == OP_EQ || pt.op == OP_NEQ)) {
                        rv = raw_equals(doc, raw, pt, lits) == (pt.op == OP_EQ) ? V_T : V_F;
                    } else if (raw.ok && pt.op == OP_MATCHES) {
                        const bool mm = raw.lit ? dfa_match_lit(blob, pt.dfa_off, raw.lit)
                                                : dfa_match_span(blob, pt.dfa_off, doc + raw.a, raw.n);
                        rv = mm ? V_T : V_F;
                    } else if ((pt.op == OP_INCL || pt.op == OP_EXCL) && v.type == T_NULL) {
                        rv = pt.op == OP_EXCL ? V_T : V_F;  // Array() of Null is empty
                    } else if ((pt.op == OP_INCL || pt.op == OP_EXCL) && raw.ok &&
                               !(v.type == T_JSON && doc[v.start] == '[')) {
                        // Array() of a value that is not an array: the value alone
                        rv = raw_equals(doc, raw, pt, lits) == (pt.op == OP_INCL) ? V_T : V_F;
                    } else if (v.type == T_STRING && v.esc) {
                        // a string with escapes: its unescaped text
                        UnescSrc us;
                        us.init(doc, v.start + 1, v.end - 1);
                        if (pt.op == OP_MATCHES)
                            rv = dfa_match_unesc(blob, pt.dfa_off, &us) ? V_T : V_F;
                        else
                            rv = unesc_equals(&us, lits + pt.lit_off, pt.lit_len) ==
                                         (pt.op == OP_EQ || pt.op == OP_INCL) ? V_T : V_F;
                    } else if (pt.op == OP_INCL || pt.op == OP_EXCL) {
                        uint32_t hits = 0;
                        const uint16_t one = 0;
                        // (a compact array of plain atoms, the common case; else the exact scan)
                        if (incl_hits(doc, v, &pt, &one, 0, 1, lits, &hits))
                            rv = ((hits & 1u) != 0) == (pt.op == OP_INCL) ? V_T : V_F;
                        else
                            rv = V_U;
                    } else {
                        rv = V_U;  // (numbers beyond the plain forms: the exact scan formats them)
                    }
                }
            }
            AJW_SET(res, (uint32_t)rv);
        }
        const V tb = row_bits(ballot(m & (res == (uint32_t)V_T)), row);
        const V ub = row_bits(ballot(m & (res == (uint32_t)V_U)), row);
        const uint32_t wi = p0 >> 5, sh = p0 & 31u;
        for (uint32_t k = 0; k < 4; k++) {
            tw[k] = tw[k] | sel(V(wi) == k, tb << sh, V(0u));
            uw[k] = uw[k] | sel(V(wi) == k, ub << sh, V(0u));
        }
    }
    // a pattern the device can not decide (beyond those unsupported by design): exact scan
    const V un0 = (uw[0] & ~(uint32_t)h->unsupported[0]) | (uw[1] & ~(uint32_t)(h->unsupported[0] >> 32));
    const V un1 = (uw[2] & ~(uint32_t)h->unsupported[1]) | (uw[3] & ~(uint32_t)(h->unsupported[1] >> 32));
    ok = ok & ((un0 | un1) == 0u);
    // bitmap words and the fold of each tree
    const uint32_t nt = h->pad1[0] ? h->pad1[0] : 1u;
    const uint32_t* code = reinterpret_cast<const uint32_t*>(blob + h->off_code);
    const uint32_t* rc = h->pad1[0] ? reinterpret_cast<const uint32_t*>(blob + h->pad1[1]) : nullptr;
    for (uint32_t k0 = 0; k0 < nt || k0 < bm_words; k0 += 16) {
        const V k = k0 + rl;
        AJW_LANES(ok & (k < nt)) {
            const uint64_t t[2] = {(uint64_t)AJW_L(tw[0]) | ((uint64_t)AJW_L(tw[1]) << 32),
                                   (uint64_t)AJW_L(tw[2]) | ((uint64_t)AJW_L(tw[3]) << 32)};
            const uint64_t u[2] = {(uint64_t)AJW_L(uw[0]) | ((uint64_t)AJW_L(uw[1]) << 32),
                                   (uint64_t)AJW_L(uw[2]) | ((uint64_t)AJW_L(uw[3]) << 32)};
            const uint64_t se[2] = {h->static_error[0], h->static_error[1]};
            const uint32_t kk = AJW_L(k);
            int32_t ep;
            const uint8_t tri = rc ? run_fold_bits(code + rc[2 * kk], rc[2 * kk + 1], t, u, se, &ep)
                                   : run_fold_bits(code, h->n_code, t, u, se, &ep);
            out(AJW_L(r), kk, nt, tri, ep);
        }
        AJW_LANES(ok & (k < bm_words)) {
            const uint32_t kk = AJW_L(k);
            const uint64_t word = kk == 0 ? ((uint64_t)AJW_L(tw[0]) | ((uint64_t)AJW_L(tw[1]) << 32))
                                  : kk == 1 ? ((uint64_t)AJW_L(tw[2]) | ((uint64_t)AJW_L(tw[3]) << 32))
                                            : 0ull;
            bm(AJW_L(r), kk, word);
        }
    }
    return ok;
}

}  // namespace w
}  // namespace ajx
