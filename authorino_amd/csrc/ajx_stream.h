// ajx_stream.h — stage A as a wave-cooperative stream over the document arena.
//
// One wave takes a span of kSpan consecutive requests (arena order) and walks their bytes
// as one stream of 32-byte blocks, 64 blocks (2 KiB) per step: lane l holds block l of the
// step, the loads of a step are contiguous (coalesced), and a document's first block is
// aligned down to 32 bytes (the block a document shares with its neighbour is loaded by a
// lane of each). Every lane classifies its 32 bytes into masks (ajx_lean.h's byte LUT and
// bit transpose); the context a byte needs from the bytes before it comes from the other
// lanes instead of a per-document loop:
//   * escapes: the previous lane's trailing odd backslash run (wave_shr);
//   * strings: the parity of the unescaped quotes before the lane (one ballot);
//   * grammar: the class of the previous byte (wave_shr) — the compact-JSON adjacency
//     rules of ajx_lean.h checked on whole masks;
//   * depth: a 64-lane prefix sum of opens minus closes, reset at each document's first
//     block (segmented by a forward fill of the head lanes' prefix);
//   * the last opening quote before the lane (a max-scan), for keys that start there;
//   * containers: a 64-lane scan of "container stack" transforms (the levels a lane opens,
//     array or object, and the id of the key each is the value of) gives the stack every
//     lane starts from.
// State that crosses a step boundary is carried in wave-uniform registers from lane 63 to
// the next step's lane 0.
//
// Object keys are identified without their parent (StreamKeySlot: the key's id among the
// ruleset's selector keys), so every lane looks its keys up independently; a key at depth
// L is then on a selector path when the ids of the keys its containers were opened under
// (the stack's bytes) followed by its own id are a selector's components (StreamPathSlot).
// Its value is captured into the document's capture row in LDS (first match in document
// order; a second match of the same selector sends the document to the exact scan), and
// the selector's eager patterns (EagerSel: eq / neq / incl / excl with a short literal) are
// decided on the spot from the ring (the step's bytes in LDS).
//
// Validity: compact JSON as in ajx_lean.h, plus what the lane-per-document walker knew from
// its stack, here from the scanned stack: every close has its container's kind, and the
// items between two brackets of one container agree with its kind — a key (a string
// before ':') only in an object, an item that does not follow ':' only in an array (so an
// object alternates key : value), a key never right after ':'. A document is proved when
// its first byte opens the root container, the root closes inside it, and no check fails
// before that close; everything else goes to the exact scan.
//
// After the span, each lane runs stage B (ajx_fast.h patterns_from_row) for one document
// of the span on its LDS capture row.
#pragma once
#include "ajx_lean_cls.h"
#include "ajx_wave.h"

namespace ajx {
namespace stream {

using lean::below;
using lean::ctz;
using lean::hib;
using lean::popc;

constexpr uint32_t kSpan = 32;                 // requests per wave (their lanes own them)
constexpr uint32_t kStepBytes = 64u * 32u;     // one step: 64 blocks of 32 B
constexpr uint32_t kWinBlocks = 66;            // the ring: the step's blocks and the 2 before
constexpr uint32_t kWinBytes = kWinBlocks * 32u;
constexpr uint32_t kMaxLevel = 16;             // container nesting tracked (deeper: exact scan)
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kMaxLen = (1u << 23) - 2u;  // longer documents: exact scan
// capture record (the row format of ajx_fast.h) with its end still open: stage B finds it
constexpr uint32_t kOpenEnd = 1u << 28;
constexpr uint32_t kTypeUnknown = 7u;

// a span's request: block 0 at arena + base (32-B aligned), its first byte at mis
// (profiling, kernel mode 53: phase clocks; 0 on the host)
AJX_HD uint64_t clk_now() {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_readcyclecounter();
#else
    return 0;
#endif
}
AJX_HD void clk_at(uint64_t* clk, uint32_t k) {
    if (clk) clk[k] = clk_now();
}

struct DocEnt {
    uint32_t base_lo, base_hi;
    uint32_t len_mis;  // len | mis << 24
    uint32_t start;    // the span's block index of block 0
};

// The container stack as a transform: levels 1..16 (bit L-1) set by it (k & 0xFFFF) with
// their kind (bit L-1 of k >> 16: 1 = array), and for levels 2..9 the id of the key each
// container is the value of (byte L-2 of iv1:iv0; kStreamElem for array elements; im:
// 0xFF per byte set). Composition: a then b.
struct Stk {
    uint32_t k, im0, im1, iv0, iv1;
};
AJX_HD Stk stk_then(const Stk& a, const Stk& b) {
    Stk r;
    const uint32_t mb = b.k & 0xFFFFu;
    r.k = ((a.k | b.k) & 0xFFFFu) | ((((a.k >> 16) & ~mb) | (b.k >> 16)) << 16);
    r.im0 = a.im0 | b.im0;
    r.im1 = a.im1 | b.im1;
    r.iv0 = (a.iv0 & ~b.im0) | b.iv0;
    r.iv1 = (a.iv1 & ~b.im1) | b.iv1;
    return r;
}

// the wave's LDS (rows follow it: kSpan x (1 + n_selectors) words, then 4 words per document
// of eager decisions: patterns decided, those of them true, array elements equal to a
// selector's eager literals (2 bits per selector < 32), selectors whose arrays hold other
// elements)
struct WaveLds {
    // the ring: the step's 64 blocks at 64 + 32 l, the previous step's last two at 0 and
    // 32 (byte address a of the span's stream at ring index a - (2048 t - 64)); 16 bytes of
    // slack on either side for the reads of short keys and values near its ends
    alignas(16) uint8_t ring_raw[16 + kWinBytes + 48];
    DocEnt doc[kSpan];
    uint32_t bad[kSpan];       // first position failing a check (min)
    uint32_t root_end[kSpan];  // position of the root's close (min)
    uint64_t heads[2];         // a step's lanes holding a document's first block (by parity)
    uint64_t clk[9];           // (profiling, kernel mode 53: phase clocks; LDS, not scratch)
};
#if defined(__HIPCC__)
__host__ __device__
#endif
constexpr uint32_t lds_bytes(uint32_t n_selectors) {
    return (uint32_t)sizeof(WaveLds) + kSpan * (1u + n_selectors) * 8u + 4u * kSpan * 8u;
}

struct alignas(16) V4 {
    uint32_t x, y, z, w;
};

// The stream's byte classes: ajx_lean.h's, with class 7 (control bytes there) replaced by
// 0x58..0x5F, which among the brackets holds [ and ] only (their kind, for the container
// stack). Control bytes outside strings are then scalar bytes: a scalar run may not start
// with one (the value-start check) and a captured or parsed scalar may not hold one (the
// captures and stage B check its bytes).
constexpr uint32_t K_SQ = 7;
constexpr uint32_t kSqH0[8] = {lean::kSetH0[0], lean::kSetH0[1], lean::kSetH0[2], lean::kSetH0[3], lean::kSetH0[4],
                               lean::kSetH0[5], lean::kSetH0[6], 0xFFu};
constexpr uint32_t kSqH1[8] = {lean::kSetH1[0], lean::kSetH1[1], lean::kSetH1[2], lean::kSetH1[3], lean::kSetH1[4],
                               lean::kSetH1[5], lean::kSetH1[6], 1u << 3};
constexpr uint32_t kSqH2[8] = {lean::kSetH2[0], lean::kSetH2[1], lean::kSetH2[2], lean::kSetH2[3], lean::kSetH2[4],
                               lean::kSetH2[5], lean::kSetH2[6], 1u << 1};
constexpr uint32_t kS0lo = lean::lut_word(kSqH0, 0), kS0hi = lean::lut_word(kSqH0, 4);
constexpr uint32_t kS1lo = lean::lut_word(kSqH1, 0), kS1hi = lean::lut_word(kSqH1, 4);
constexpr uint32_t kS2lo = lean::lut_word(kSqH2, 0);
constexpr bool sq_lut_ok() {
    for (uint32_t b = 0; b < 256; b++) {
        const uint32_t c = lean::lut_byte(kSqH0, b & 7) & lean::lut_byte(kSqH1, (b >> 3) & 7) & lean::lut_byte(kSqH2, b >> 6);
        const uint32_t want = (lean::class_ref(b) & 0x7Fu) | ((b >= 0x58 && b <= 0x5F) ? 0x80u : 0u);
        if (c != want) return false;
    }
    return true;
}
static_assert(sq_lut_ok(), "stream byte-class LUT");
AJX_HD uint32_t classify4(uint32_t x) {
    const uint32_t a = lean::perm(kS0hi, kS0lo, x & 0x07070707u);
    const uint32_t b = lean::perm(kS1hi, kS1lo, (x >> 3) & 0x07070707u);
    const uint32_t c = lean::perm(0u, kS2lo, (x >> 6) & 0x03030303u);
    return a & b & c;
}

// ring reads (index any int within the slack; unaligned)
AJX_HD uint32_t ring32(const uint8_t* ring, int32_t a) {
    const int32_t q = a & ~3;
    const uint32_t sh = (uint32_t)a & 3u;
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(ring + q);
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(ring + q + 4);
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbyte(w1, w0, sh);
#else
    return sh ? (w0 >> (8 * sh)) | (w1 << (32 - 8 * sh)) : w0;
#endif
}
AJX_HD uint64_t ring64(const uint8_t* ring, int32_t a) {
    return (uint64_t)ring32(ring, a) | ((uint64_t)ring32(ring, a + 4) << 32);
}
AJX_HD bool in_ring(int32_t a, uint32_t n) { return a >= 0 && a + (int32_t)n <= (int32_t)kWinBytes; }

// carried from lane 63 of one step to lane 0 of the next (wave-uniform)
struct Carry {
    uint32_t esc;       // an odd backslash run ends the step
    uint32_t str;       // the step ends inside a string
    uint32_t prevf;     // classes of the step's last byte (grammar flags)
    uint32_t loq;       // last opening quote: (position + 1) << 1 | preceded by ':' (0 none)
    uint32_t kid31;     // id of a key whose ':' is the step's last byte
    uint32_t bs63;      // backslashes of the step's last block
    uint32_t bs_any;    // the step had a backslash
    int32_t depth;      // depth after the step
    Stk stk;            // container stack after the step
};
AJX_HD void carry_init(Carry& c) {
    c.esc = c.str = c.prevf = c.loq = c.kid31 = c.bs63 = c.bs_any = 0;
    c.depth = 0;
    c.stk = Stk{0u, 0u, 0u, 0u, 0u};
}

// The ruleset's tables the stream reads (LDS copies when the blob is staged)
struct Tabs {
    const StreamKeySlot* ks;
    const StreamPathSlot* ps;
    const EagerSel* eg;  // (null: none)
    const uint8_t* lits;
    uint32_t k_log2, k_mult, k_probes, p_log2, p_mult, p_probes, max_key_len, ns;
    uint32_t nr;     // capture records (the selectors', then exact selectors' prefixes')
    uint32_t exact;  // some selector takes the exact Get in stage B (StreamHdr exact_lo / hi)
};
AJX_HD Tabs tabs_of(const uint8_t* blob) {
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
    const StreamHdr* s = reinterpret_cast<const StreamHdr*>(blob + h->off_stream);
    Tabs t;
    // (blob plus uniform offsets, not pointers made uniform through integers: a staged blob's
    // tables are then read with ds_reads, not flat loads that also wait for the stream's
    // document loads in flight)
    t.ks = reinterpret_cast<const StreamKeySlot*>(blob + lean::uni(s->off_keys));
    t.ps = reinterpret_cast<const StreamPathSlot*>(blob + lean::uni(s->off_paths));
    t.eg = lean::uni(h->off_eager) ? reinterpret_cast<const EagerSel*>(blob + lean::uni(h->off_eager)) : nullptr;
    t.lits = blob + lean::uni(h->off_literals);
    t.k_log2 = lean::uni(s->key_log2);
    t.k_mult = lean::uni(s->key_mult);
    t.k_probes = lean::uni(s->key_probes);
    t.p_log2 = lean::uni(s->path_log2);
    t.p_mult = lean::uni(s->path_mult);
    t.p_probes = lean::uni(s->path_probes);
    t.max_key_len = lean::uni(s->max_key_len);
    t.ns = lean::uni(h->n_selectors);
    t.nr = lean::uni(s->n_rec);
    t.exact = lean::uni(s->exact_lo | s->exact_hi);
    return t;
}

// the id of the key whose len bytes end before ring index ra_end (0: none); the key lies in
// the ring
AJX_HD uint32_t key_id(const Tabs& T, const uint8_t* ring, int32_t ra_end, uint32_t len) {
    if (len > T.max_key_len) return 0;
    uint64_t sig = ring64(ring, ra_end - 8);
    sig = len >= 8 ? sig : (len ? sig >> (8u * (8u - len)) : 0ull);
    const uint32_t mask = (1u << T.k_log2) - 1u;
    uint32_t at = key_slot_hash(sig, len, 0, T.k_log2, T.k_mult);
    uint32_t id = 0;
    for (uint32_t p = 0; p < T.k_probes; p++) {
        const StreamKeySlot s = T.ks[(at + p) & mask];
        if (s.meta != kEmptySlot && s.sig == sig && (s.meta & 0xFFFFu) == len) {
            bool hit = true;
            if (len > 8) {  // the head: bytes [0, len - 8) against the literal pool
                const int32_t ra0 = ra_end - (int32_t)len;
                const uint8_t* kl = T.lits + s.key_off;
                for (uint32_t k = 0; k < len - 8u; k += 4u) {
                    const uint32_t n = len - 8u - k;
                    const uint32_t m = n >= 4 ? ~0u : (1u << (8u * n)) - 1u;
                    if ((ring32(ring, ra0 + (int32_t)k) ^ *reinterpret_cast<const uint32_t*>(kl + k)) & m) {
                        hit = false;
                        break;
                    }
                }
            }
            if (hit) id = s.meta >> 16;
        }
    }
    return id;
}

// the path table's meta of the node at path bytes `path` (selector in the low 16 bits,
// 0xFFFF none; kStreamHasKids; 0: no such node)
AJX_HD uint32_t path_meta(const Tabs& T, uint64_t path) {
    const uint32_t mask = (1u << T.p_log2) - 1u;
    const uint32_t at = stream_path_hash(path, T.p_log2, T.p_mult);
    uint32_t meta = 0;
    for (uint32_t p = 0; p < T.p_probes; p++) {
        const StreamPathSlot s = T.ps[(at + p) & mask];
        if (s.meta && s.path == path) meta = s.meta;
    }
    return meta;
}

// bit j of the result: eager entry j of `e` equals the string content at ring index ra
// (cl bytes)
AJX_HD uint32_t eager_hits(const EagerSel& e, const uint8_t* ring, int32_t ra, uint32_t cl) {
    uint64_t c0 = 0, c1 = 0;
    if (cl <= 16) {
        c0 = ring64(ring, ra);
        c1 = ring64(ring, ra + 8);
    }
    const uint64_t m0 = cl >= 8 ? ~0ull : ((1ull << (8 * cl)) - 1ull);
    const uint64_t m1 = cl >= 16 ? ~0ull : (cl > 8 ? ((1ull << (8 * (cl - 8))) - 1ull) : 0ull);
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const uint64_t l0 = (uint64_t)e.lit[k][0] | ((uint64_t)e.lit[k][1] << 32);
        const uint64_t l1 = (uint64_t)e.lit[k][2] | ((uint64_t)e.lit[k][3] << 32);
        const bool eq = (e.m[k] & kEagerValid) && cl == ((e.m[k] >> 16) & 0xFFu) && ((c0 ^ l0) & m0) == 0 &&
                        ((c1 ^ l1) & m1) == 0;
        r |= eq ? 1u << k : 0u;
    }
    return r;
}

// Per-span setup: the document table and per-document results (lane l < kSpan: request r).
AJX_HD void span_setup(WaveLds& L, uint64_t* rows, uint32_t ns, uint32_t l, bool my_doc, uint64_t off,
                       uint32_t len, uint32_t& my_start, uint32_t& total) {
    const uint32_t mis = (uint32_t)(off & 31u);
    const bool ok = my_doc && len > 0 && len <= kMaxLen;
    const uint32_t nb = !my_doc ? 0u : ok ? (mis + len + 31u) >> 5 : 1u;
    const uint32_t incl = wave::scan_add(nb);
    my_start = incl - nb;
    total = wave::readlane(incl, 63);
    if (l < kSpan) {
        const uint64_t base = off - mis;
        L.doc[l] = DocEnt{(uint32_t)base, (uint32_t)(base >> 32), (ok ? len : 0u) | (mis << 24), my_start};
        L.bad[l] = my_doc && !ok ? 0u : kNone;  // empty and oversized documents: exact scan
        L.root_end[l] = kNone;
        // the document's capture row (records: start kNone = not found) and eager decisions
        uint64_t* row = rows + (size_t)l * (1u + ns);
        for (uint32_t s = 0; s <= ns; s++) row[s] = s ? (uint64_t)kNone : 0ull;
        uint64_t* dec = rows + (size_t)kSpan * (1u + ns) + 4u * l;
        dec[0] = dec[1] = dec[2] = dec[3] = 0;
    }
    if (l < 2) L.heads[l] = 0;
    wave::sync();
}

// A lane's block of a step, loaded ahead of its processing.
struct Blk {
    uint32_t x[8];
    uint32_t doc;    // span index of the document
    int32_t pos0;    // document position of byte 0
    uint32_t valid;  // bytes of the document
    uint32_t vbase;  // stream byte address of the document's position 0
    uint32_t mis;
    bool head, live;
};
// the heads of step t (H) and this lane's block of it; last_doc: the document of the block
// before the step (kNone before the first)
AJX_HD void fetch(WaveLds& L, const uint8_t* __restrict__ arena, uint32_t t, uint32_t total, uint32_t l,
                  uint32_t my_start, bool my_doc, uint32_t last_doc, Blk& B, uint64_t& H) {
    uint64_t* hp = &L.heads[t & 1u];
    const uint32_t h = my_start - t * 64u;
    if (my_doc && h < 64u) wave::lds_or64(hp, 1ull << h);
    wave::sync();
    H = *hp;
    wave::sync();
    if (l == 0) *hp = 0;
    const uint32_t v = t * 64u + l;
    B.live = v < total;
    B.doc = (last_doc + (uint32_t)__builtin_popcountll(H & wave::mask_le(l))) & (kSpan - 1u);
    B.head = ((H >> l) & 1ull) != 0;
    const DocEnt e = L.doc[B.doc];
    const uint32_t len = e.len_mis & 0xFFFFFFu;
    B.mis = e.len_mis >> 24;
    const uint32_t b = v - e.start;
    B.pos0 = (int32_t)(b * 32u) - (int32_t)B.mis;
    B.vbase = e.start * 32u + B.mis;
    B.valid = 0;
    if (B.live) {
        const uint32_t lo = b == 0 ? B.mis : 0u;
        const int32_t hi = (int32_t)len - B.pos0;
        B.valid = (hi >= 32 ? ~0u : hi <= 0 ? 0u : below((uint32_t)hi)) & ~below(lo);
        const uint64_t base = ((uint64_t)e.base_hi << 32 | e.base_lo) + (uint64_t)b * 32u;
        const V4* p = reinterpret_cast<const V4*>(arena + base);
        const V4 q0 = p[0], q1 = p[1];
        B.x[0] = q0.x, B.x[1] = q0.y, B.x[2] = q0.z, B.x[3] = q0.w;
        B.x[4] = q1.x, B.x[5] = q1.y, B.x[6] = q1.z, B.x[7] = q1.w;
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) B.x[j] = 0;
    }
}

// One step of the stream for this lane (all 64 lanes call it), on its prefetched block.
// MODE 1 (profiling): the structural pass only (no keys, no captures); 2: no stage B.
template <int MODE>
AJX_HD void step(WaveLds& L, uint64_t* rows, const Tabs& T, uint32_t t, uint32_t l, const Blk& B, uint64_t H,
                 Carry& c, uint64_t* clk = nullptr) {
    uint8_t* ring = L.ring_raw + 16;
    const uint32_t doc = B.doc;
    const bool head = B.head, live = B.live;
    const int32_t pos0 = B.pos0;
    const uint32_t valid = B.valid, mis = B.mis;
    const int32_t roff = (int32_t)(B.vbase - (t * 2048u - 64u));  // ring index of document position p: roff + p
    wave::sync();  // (the previous step's ring reads are done)
    {  // the ring: the previous step's last two blocks move to its front, this step's follow
        if (t && l >= 62) {
            const V4* src = reinterpret_cast<const V4*>(ring + 64 + 32 * l);
            const V4 a = src[0], b2 = src[1];
            V4* dst = reinterpret_cast<V4*>(ring + 32 * (l - 62));
            dst[0] = a;
            dst[1] = b2;
        }
        V4* rp = reinterpret_cast<V4*>(ring + 64 + 32 * l);
        rp[0] = V4{B.x[0], B.x[1], B.x[2], B.x[3]};
        rp[1] = V4{B.x[4], B.x[5], B.x[6], B.x[7]};
    }
    clk_at(clk, 0);  // (the block's loads arrived)

    // ---- classification (ajx_lean.h)
    uint32_t d[8];
#pragma unroll
    for (int j = 0; j < 8; j++) d[j] = classify4(B.x[j]);
    lean::transpose(d);
    const uint32_t Q = d[lean::creg(lean::K_Q)] & valid, BS = d[lean::creg(lean::K_BS)] & valid;
    uint32_t bad = 0;

    // ---- escapes: the byte after an odd backslash run; the run may come from the lane
    // before (a lane of 32 backslashes, whose carry depends on its own, is left to the
    // exact scan)
    uint32_t escaped = 0, esc_out = 0;
    const bool bs_step = wave::ballot(BS != 0) != 0;
    // keys may hold a backslash (then the exact scan decides) when this step or the one
    // before has one; pBS: the block before's backslashes
    const bool bs_keys = bs_step || c.bs_any;
    uint32_t pBS = 0;
    if (bs_keys) {
        pBS = wave::shr1(BS, c.bs63);
        if (head) pBS = 0;
    }
    c.bs63 = wave::readlane(BS, 63);
    c.bs_any = bs_step ? 1u : 0u;
    if (bs_step || c.esc) {
        auto run = [&](uint32_t ein, uint32_t& out) -> uint32_t {
            const uint32_t bsx = BS & ~ein;
            const uint32_t follows = (bsx << 1) | ein;
            const uint32_t even = 0x55555555u;
            const uint32_t odd_starts = bsx & ~even & ~follows;
            const uint64_t seq = (uint64_t)odd_starts + bsx;
            out = (uint32_t)(seq >> 32);
            return (even ^ ((uint32_t)seq << 1)) & follows;
        };
        uint32_t o0;
        (void)run(0u, o0);
        uint32_t ein = wave::shr1(o0, c.esc);
        if (head) ein = 0;
        escaped = run(ein, esc_out);
        if (BS == ~0u) bad |= 1u;
    }
    c.esc = wave::readlane(esc_out, 63);

    // ---- strings: prefix XOR of the unescaped quotes, the parity of the lanes before
    // (from the document's first block, or the carry) coming from one ballot
    const uint32_t U = Q & ~escaped;
    uint32_t X = U;
    X ^= X << 1;
    X ^= X << 2;
    X ^= X << 4;
    X ^= X << 8;
    X ^= X << 16;
    const uint64_t P = wave::ballot((popc(U) & 1u) != 0);
    const uint64_t lt = wave::mask_lt(l), hle = H & wave::mask_le(l);
    uint32_t s_in;
    if (hle) {
        const uint32_t hb = 63u - (uint32_t)__builtin_clzll(hle);
        s_in = (uint32_t)__builtin_popcountll(P & lt & ~wave::mask_lt(hb)) & 1u;
    } else {
        s_in = ((uint32_t)__builtin_popcountll(P & lt) & 1u) ^ c.str;
    }
    X ^= s_in ? ~0u : 0u;  // inside a string at byte k (the opening quote included)
    c.str = (wave::readlane(X, 63) >> 31) & 1u;
    const uint32_t OQ = U & X, CQ = U & ~X;
    const uint32_t outside = ~X & ~U & valid;
    const uint32_t OP = d[lean::creg(lean::K_OPEN)] & outside, CL = d[lean::creg(lean::K_CLOSE)] & outside;
    const uint32_t CO = d[lean::creg(lean::K_COLON)] & outside, CM = d[lean::creg(lean::K_COMMA)] & outside;
    const uint32_t badb = (d[lean::creg(lean::K_BAD1)] | BS) & outside;
    const uint32_t ST = OP | CL | CO | CM;
    const uint32_t SC = outside & ~ST & ~badb;

    // ---- grammar (ajx_lean.h classify): the previous byte's class from the lane before.
    // flags: OP, CO|CM, CO, CQ, SC, CL of byte 31; bit 6: byte 31 closes a string that
    // started after ':' (a second exchange, below)
    uint32_t myf = (OP >> 31) | (((CO | CM) >> 31) << 1) | ((CO >> 31) << 2) | ((CQ >> 31) << 3) |
                   ((SC >> 31) << 4) | ((CL >> 31) << 5);
    uint32_t f = wave::shr1(myf, c.prevf & 63u);
    if (head) f = 0;
    const uint32_t nOP = (OP << 1) | (f & 1u), nCOCM = ((CO | CM) << 1) | ((f >> 1) & 1u);
    const uint32_t nCO = (CO << 1) | ((f >> 2) & 1u);
    const uint32_t nCQ = (CQ << 1) | ((f >> 3) & 1u);
    const uint32_t nSC = (SC << 1) | ((f >> 4) & 1u), nCL = (CL << 1) | ((f >> 5) & 1u);
    const uint32_t nSEP = nOP | nCOCM;
    const uint32_t SCS = SC & ~nSC;  // scalar run starts
    bad |= badb | (OQ & ~nSEP) | (nCQ & ~(CO | CM | CL)) | (SCS & ~nSEP) | (nSC & ~(SC | CM | CL)) |
           (nSEP & (CO | CM)) | (nCOCM & CL) | (nCL & ~(CM | CL));
    // the root container opens at the document's first byte
    if (head && !((OP >> mis) & 1u)) bad |= 1u << mis;
    // a scalar starts with one of gjson's value-start bytes (t f n - + 0-9 i I N)
    for (uint32_t m = SCS; m; m &= m - 1u)
        if (!lean::scalar_start(ring[64 + 32 * l + ctz(m)])) bad |= m & (0u - m);

    // ---- the last opening quote before the lane (position + 1, and whether ':' precedes
    // it), for keys that start in an earlier lane and for the string open at byte 0
    const uint32_t oqv = OQ ? (((uint32_t)(pos0 + (int32_t)hib(OQ)) + 1u) << 1) | ((nCO >> hib(OQ)) & 1u) : 0u;
    // (oqv >= 2; lane 0 without one: the carry, lane field 0)
    const uint32_t loq_incl = wave::scan_max(oqv ? (l << 26) | oqv : (l == 0 ? c.loq : 0u));
    const uint32_t loq = wave::shr1(loq_incl, c.loq);  // (lanes before; lane 0: the carry)
    {
        const uint32_t last = wave::readlane(loq_incl, 63);
        if (last) c.loq = last & ((1u << 26) - 1u);
    }
    // (positions are the document's own: the last opening quote before a key or an open
    // string of a valid document is that document's)
    const uint32_t loqv = loq & ((1u << 26) - 1u);  // (position + 1) << 1 | after ':'
    // ---- strings that start after ':' (values): their closing quotes (Mv), by carrying each
    // such opening quote through its run of X; the string open at byte 0 from the scan
    const uint32_t cin = (s_in && (loqv & 1u)) ? 1u : 0u;
    const uint32_t Mv = (uint32_t)((X + (OQ & nCO)) + cin) & ~X & CQ;
    myf |= (Mv >> 31) << 6;
    const uint32_t fM = wave::shr1(myf >> 6, (c.prevf >> 6) & 1u) & (head ? 0u : 1u);
    c.prevf = wave::readlane(myf, 63);
    const uint32_t nMv = (Mv << 1) | fM;            // the byte after such a closing quote
    const uint32_t KEYC = CO & nCQ;                  // colons ending a key
    bad |= KEYC & nMv;                               // a key right after ':' ("a":"b":)
    // items that do not follow ':' (at a string's end / a scalar's start)
    const uint32_t NONKEY = (nCQ & ~CO & ~nMv) | (SCS & ~nCO);

    // ---- depth before byte 0: prefix sum of opens minus closes, segmented at heads
    const int32_t net = (int32_t)popc(OP) - (int32_t)popc(CL);
    const int32_t Ei = (int32_t)wave::scan_add((uint32_t)net);
    const int32_t Ex = Ei - net;
    const uint32_t hk = head ? ((l + 1u) << 20) | (uint32_t)(Ex + (1 << 19)) : 0u;
    const uint32_t ff = wave::scan_max(hk);
    const int32_t depth_in = ff ? Ex - ((int32_t)(ff & 0xFFFFFu) - (1 << 19)) : Ex + c.depth;
    c.depth = (int32_t)wave::readlane((uint32_t)(depth_in + net), 63);

    const uint32_t ARR = d[lean::creg(K_SQ)] & (OP | CL);  // [ and ]
    clk_at(clk, 1);  // (classification, strings, grammar, depth)

    // ---- keys (ids) and brackets in document order: the lane's container transform, kind
    // and alternation checks, root close
    Stk tr{0u, 0u, 0u, 0u, 0u};
    if (head) tr = Stk{0xFFFFu, ~0u, ~0u, 0u, 0u};  // a document starts from an empty stack
    uint32_t req_m = 0, req_v = 0, req_pos = kNone;   // kinds the incoming stack must have
    uint64_t kids = 0;      // key ids by key ordinal in the lane
    uint32_t kbs_ord = 0;   // keys holding a backslash, by key ordinal
    uint32_t keym = 0;      // keys with an id or a backslash (the only ones the captures look at)
    uint64_t oids = 0;      // container ids by open ordinal
    uint32_t pend_lvl = 0;  // a level opened at byte 0 right after ':' in the lane before
    uint32_t kid31 = 0;     // id of the key whose ':' is byte 31
    {
        int32_t dd = depth_in;
        uint32_t lm = 0, lv = 0;  // levels opened in this lane, their kinds
        uint32_t seg_lo = 0, nk = 0, no = 0, last_kid = 0;
        // the items of the segment (seg_lo, i] belong to the container at level dd
        auto need = [&](uint32_t bit, uint32_t want, uint32_t at) {
            if (lm & bit) {
                if ((lv & bit) != want) bad |= 1u << at;
            } else if (req_m & bit) {
                if ((req_v & bit) != want) bad |= 1u << at;
            } else {
                req_m |= bit;
                req_v |= want;
                req_pos = req_pos == kNone ? at : req_pos;
            }
        };
        auto segment = [&](uint32_t i) {
            const uint32_t items = (KEYC | NONKEY) & below(i + 1u) & ~below(seg_lo);
            if (!items || dd < 1) return;
            const bool need_obj = (KEYC & items) != 0, need_arr = (NONKEY & items) != 0;
            const uint32_t first = ctz(items);
            if (dd > (int32_t)kMaxLevel || (need_obj && need_arr)) {
                bad |= 1u << first;
                return;
            }
            const uint32_t bit = 1u << (dd - 1);
            need(bit, need_arr ? bit : 0u, first);
        };
        for (uint32_t m = OP | CL | KEYC; m; m &= m - 1u) {
            const uint32_t i = ctz(m);
            if ((KEYC >> i) & 1u) {
                uint32_t id = 0;
                if constexpr (MODE != 1) {
                    // the key: (its opening quote, the closing quote at i - 1)
                    const uint32_t oqb = i >= 2 ? OQ & below(i - 1u) : 0u;
                    const uint32_t oqpos = oqb ? (uint32_t)(pos0 + (int32_t)hib(oqb)) : (loqv >> 1) - 1u;
                    const uint32_t cqpos = (uint32_t)(pos0 + (int32_t)i) - 1u;
                    if ((oqb || loqv) && cqpos > oqpos) {
                        const uint32_t klen = cqpos - oqpos - 1u;
                        const int32_t ra_end = roff + (int32_t)cqpos;
                        if (in_ring(ra_end - (int32_t)klen, klen)) id = key_id(T, ring, ra_end, klen);
                        // a key holding a backslash: gjson compares it unescaped (exact scan)
                        if (bs_keys) {
                            const int32_t lo = (int32_t)oqpos + 1 - pos0, hi = (int32_t)cqpos - pos0;
                            auto bits = [](int32_t a, int32_t b) -> uint32_t {
                                a = a < 0 ? 0 : a;
                                b = b > 32 ? 32 : b;
                                return a >= b ? 0u : below((uint32_t)b) & ~below((uint32_t)a);
                            };
                            bool kbs = (BS & bits(lo, hi)) || (pBS & bits(lo + 32, hi + 32));
                            if (lo < -32) {  // (more than a block back: the ring, else the exact scan)
                                if (!in_ring(roff + (int32_t)oqpos + 1, klen)) kbs = true;
                                for (uint32_t q = 0; q < klen && !kbs; q++)
                                    kbs = ring[roff + (int32_t)oqpos + 1 + (int32_t)q] == '\\';
                            }
                            if (kbs) {
                                kbs_ord |= 1u << (nk & 31u);
                                keym |= 1u << i;
                            }
                        }
                    }
                }
                if (id) keym |= 1u << i;
                if (nk < 8) kids |= (uint64_t)id << (8u * nk);
                if (nk == 8) bad |= 1u << i;  // (a 9th key in the block: exact scan, see below)
                nk++;
                last_kid = id;
                if (i == 31) kid31 = id;
                continue;
            }
            const uint32_t arr = (ARR >> i) & 1u;
            segment(i);
            seg_lo = i + 1u;
            if ((OP >> i) & 1u) {
                // a container that does not follow ':' is an array element
                const bool after_colon = ((nCO >> i) & 1u) != 0;
                if (dd >= 1 && !after_colon) {
                    if (dd > (int32_t)kMaxLevel)
                        bad |= 1u << i;
                    else
                        need(1u << (dd - 1), 1u << (dd - 1), i);
                }
                dd++;
                if (dd < 1 || dd > (int32_t)kMaxLevel) {
                    bad |= 1u << i;
                    continue;
                }
                const uint32_t bit = 1u << (dd - 1);
                lm |= bit;
                lv = arr ? lv | bit : lv & ~bit;
                tr.k = (tr.k | bit) & ~(bit << 16);
                tr.k |= arr ? bit << 16 : 0u;
                uint32_t id = kStreamElem;
                if (after_colon) id = i ? last_kid : 0u;
                if (after_colon && !i)
                    pend_lvl = (uint32_t)dd;  // (the key is the lane before's: patched below)
                else if (pend_lvl == (uint32_t)dd)
                    pend_lvl = 0;
                if (no < 8) oids |= (uint64_t)id << (8u * no);
                if (no == 8) bad |= 1u << i;  // (a 9th open in the block: exact scan, see below)
                no++;
                if (dd >= 2 && dd <= 9) {
                    const uint32_t sh = 8u * ((uint32_t)(dd - 2) & 3u);
                    if (dd <= 5) {
                        tr.im0 |= 0xFFu << sh;
                        tr.iv0 = (tr.iv0 & ~(0xFFu << sh)) | (id << sh);
                    } else {
                        tr.im1 |= 0xFFu << sh;
                        tr.iv1 = (tr.iv1 & ~(0xFFu << sh)) | (id << sh);
                    }
                }
            } else {
                if (dd < 1 || dd > (int32_t)kMaxLevel) {
                    bad |= 1u << i;
                    dd--;
                    continue;
                }
                need(1u << (dd - 1), arr << (dd - 1), i);
                dd--;
                if (dd == 0) wave::lds_min(&L.root_end[doc], (uint32_t)(pos0 + (int32_t)i));
            }
        }
        segment(31u);
        // (the capture loop keeps the ids of 8 keys and 8 opens per block: a 9th of either
        // sends the document to the exact scan, marked at its own position above. Not at the
        // block's byte 0: in a document's first block that byte can lie before the document,
        // where the mark would be lost and a selector under the 9th open missed; found by
        // tests/test_gpu_stream.py::test_stream_dense_blocks)
    }
    // the id of a key whose ':' ended the lane before (or the step before)
    {
        const uint32_t prev31 = wave::shr1(kid31, c.kid31);
        c.kid31 = wave::readlane(kid31, 63);
        if (pend_lvl >= 2 && pend_lvl <= 9) {
            const uint32_t sh = 8u * ((pend_lvl - 2u) & 3u);
            if (pend_lvl <= 5)
                tr.iv0 |= prev31 << sh;
            else
                tr.iv1 |= prev31 << sh;
        }
        if (OP & 1u & nCO) oids |= (uint64_t)prev31;  // (the lane's first open is that container)
    }

    // ---- container stack before byte 0: scan of the transforms (the carry composed into
    // lane 0)
    if (l == 0 && !head) tr = stk_then(c.stk, tr);
    const Stk ident{0u, 0u, 0u, 0u, 0u};
    const Stk incl = wave::scan_incl_t(tr, ident, stk_then);
    const Stk stk_in = wave::shr1_t(incl, c.stk);
    c.stk = wave::readlane_t(incl, 63);
    if (req_m && (((stk_in.k >> 16) & req_m) != req_v)) bad |= 1u << req_pos;
    if (bad && live) wave::lds_min(&L.bad[doc], (uint32_t)(pos0 + (int32_t)ctz(bad)));
    bad = 0;
    clk_at(clk, 2);  // (keys, brackets, the container stack)

    if constexpr (MODE != 1) {
        // ---- keys on selector paths: capture their values; elements of captured arrays
        // with incl / excl patterns: compare them. The next lane's first bytes (a value that
        // starts or ends there)
        const uint32_t fcq = CQ ? ctz(CQ) : 32u, fst = (ST & valid) ? ctz(ST & valid) : 32u;
        const uint32_t nx_info = (OQ & 1u) | ((OP & 1u) << 1) | ((SCS & 1u) << 2) | (fcq << 3) | (fst << 9) |
                                 (((BS & below(fcq)) ? 1u : 0u) << 15) | ((head ? 1u : 0u) << 16) |
                                 ((CO & 1u) << 17) | ((ARR & 1u) << 18);
        const uint32_t nx = wave::shl1(nx_info, 1u << 16);  // (lane 63: as if the next were another document)
        // element strings (closing quotes of strings neither keys nor values after ':') and
        // element scalars, looked at only in arrays on selector paths
        const uint32_t ELQ = T.eg ? CQ & ~Mv & ~((CO >> 1) | (((nx >> 17) & 1u) << 31)) : 0u;
        const uint32_t ELS = T.eg ? SCS & ~nCO : 0u;
        wave::sync();  // (the ring holds every lane's block)
        // the tokens the captures act on: keys with an id (or a backslash), element strings
        // and scalars, container elements; brackets only up to the last of them
        const uint32_t OPE = T.eg ? OP & ~nCO : 0u;
        const uint32_t want = keym | ELQ | ELS | OPE;
        if (want) {
            uint64_t* row = rows + (size_t)doc * (1u + T.nr);
            uint64_t* dec = rows + (size_t)kSpan * (1u + T.nr) + 4u * doc;
            int32_t dd = depth_in;
            uint64_t iv = (uint64_t)stk_in.iv0 | ((uint64_t)stk_in.iv1 << 32);
            // the selector whose path is the container at level dd (kNone: none)
            auto container_sel = [&]() -> uint32_t {
                if (dd < 2 || dd > (int32_t)kStreamMaxComps + 1) return kNone;
                const uint32_t nb = (uint32_t)dd - 1u;
                const uint64_t keep = ~0ull >> (64u - 8u * nb);
                const uint64_t pth = iv & keep;
                if (((pth - 0x0101010101010101ull) & ~pth & 0x8080808080808080ull) & keep) return kNone;
                const uint32_t pm = path_meta(T, pth);
                // (a selector's: its eager tables; an exact selector's prefix record has none)
                return (pm && (pm & 0xFFFFu) < T.ns) ? (pm & 0xFFFFu) : kNone;
            };
            for (uint32_t m = (OP | CL | want) & below(hib(want) + 1u); m; m &= m - 1u) {
                const uint32_t i = ctz(m);
                if ((OP >> i) & 1u) {
                    if ((OPE >> i) & 1u) {  // a container element: its array is not all strings
                        const uint32_t sa = container_sel();
                        if (sa < 32u) wave::lds_or64(&dec[3], 1ull << sa);
                    }
                    dd++;
                    const uint32_t no = popc(OP & below(i));  // (the open's ordinal in the lane)
                    if (dd >= 2 && dd <= 9) {
                        const uint32_t sh = 8u * (uint32_t)(dd - 2);
                        const uint64_t id = no < 8 ? (oids >> (8u * no)) & 0xFFu : 0ull;
                        iv = (iv & ~(0xFFull << sh)) | (id << sh);
                    }
                    continue;
                }
                if ((CL >> i) & 1u) {
                    dd--;
                    continue;
                }
                if ((ELQ | ELS) & (1u << i)) {
                    const uint32_t sa = container_sel();
                    if (sa >= 32u) continue;
                    const EagerSel eg = T.eg[sa];
                    bool simple = ((ELQ >> i) & 1u) != 0;
                    uint32_t hit = 0;
                    if (simple) {  // the element's text: (its opening quote, i)
                        const uint32_t oqb = i ? OQ & below(i) : 0u;
                        const uint32_t oqpos = oqb ? (uint32_t)(pos0 + (int32_t)hib(oqb)) : (loqv >> 1) - 1u;
                        const uint32_t cqpos = (uint32_t)(pos0 + (int32_t)i);
                        const uint32_t cl = cqpos - oqpos - 1u;
                        simple = (oqb || loqv) && cqpos > oqpos &&
                                 (cl > 16u || in_ring(roff + (int32_t)oqpos + 1, cl));
                        if (simple && bs_keys) {  // (an escape: the exact compare of stage B)
                            const int32_t lo = (int32_t)oqpos + 1 - pos0, hi = (int32_t)cqpos - pos0;
                            auto bits = [](int32_t a, int32_t b) -> uint32_t {
                                a = a < 0 ? 0 : a;
                                b = b > 32 ? 32 : b;
                                return a >= b ? 0u : below((uint32_t)b) & ~below((uint32_t)a);
                            };
                            simple = !((BS & bits(lo, hi)) || (pBS & bits(lo + 32, hi + 32)) || lo < -32);
                        }
                        if (simple) hit = eager_hits(eg, ring, roff + (int32_t)oqpos + 1, cl);
                    }
                    if (!simple)
                        wave::lds_or64(&dec[3], 1ull << sa);
                    else if (hit)
                        wave::lds_or64(&dec[2], (uint64_t)hit << (2u * sa));
                    continue;
                }
                const uint32_t nk = popc(KEYC & below(i));  // (the key's ordinal in the lane)
                const uint32_t own = nk < 8 ? (uint32_t)(kids >> (8u * nk)) & 0xFFu : 0u;
                const bool kbs = ((kbs_ord >> (nk & 31u)) & 1u) != 0;
                if ((!own && !kbs) || dd < 1 || dd > (int32_t)kStreamMaxComps) continue;
                // the path bytes: the container ids of levels 2..dd, then the key's own id
                const uint32_t nb = (uint32_t)dd - 1u;
                const uint64_t keep = nb ? ~0ull >> (64u - 8u * nb) : 0ull;
                const uint64_t anc = iv & keep;
                if (((anc - 0x0101010101010101ull) & ~anc & 0x8080808080808080ull) & keep)
                    continue;  // (an ancestor that is no selector key)
                if (kbs) {  // a key to unescape in a container on a selector path: exact scan
                    if (!nb || (path_meta(T, anc) & kStreamHasKids)) bad |= 1u << i;
                    continue;
                }
                const uint32_t pm = path_meta(T, anc | ((uint64_t)own << (8u * nb)));
                const uint32_t s = pm & 0xFFFFu;
                if (!pm || s == 0xFFFFu) continue;
                // the value: at i + 1 (this lane) or the next lane's byte 0
                const uint32_t vpos = (uint32_t)(pos0 + (int32_t)i) + 1u;
                uint32_t type = kTypeUnknown, end = 0, esc = 0, open = 1, arr = 0;
                if (i < 31) {
                    const uint32_t j = i + 1u;
                    if ((OQ >> j) & 1u) {
                        type = T_STRING;
                        const uint32_t q = CQ & ~below(j + 1u);
                        if (q) {
                            end = (uint32_t)(pos0 + (int32_t)ctz(q)) + 1u;
                            esc = (BS & below(ctz(q)) & ~below(j)) ? 1u : 0u;
                            open = 0;
                        } else if (!((nx >> 16) & 1u) && ((nx >> 3) & 63u) < 32u) {
                            end = (uint32_t)(pos0 + 32 + (int32_t)((nx >> 3) & 63u)) + 1u;
                            esc = ((BS & ~below(j)) || ((nx >> 15) & 1u)) ? 1u : 0u;
                            open = 0;
                        }
                    } else if ((OP >> j) & 1u) {
                        type = T_JSON;
                        arr = (ARR >> j) & 1u;
                    } else if ((SCS >> j) & 1u) {
                        type = T_NUMBER;
                        const uint32_t q = ST & valid & ~below(j);
                        if (q) {
                            end = (uint32_t)(pos0 + (int32_t)ctz(q));
                            open = 0;
                        } else if (!((nx >> 16) & 1u) && ((nx >> 9) & 63u) < 32u) {
                            end = (uint32_t)(pos0 + 32 + (int32_t)((nx >> 9) & 63u));
                            open = 0;
                        }
                    }
                } else if (!((nx >> 16) & 1u)) {
                    type = (nx & 1u) ? T_STRING : ((nx >> 1) & 1u) ? T_JSON : ((nx >> 2) & 1u) ? T_NUMBER : kTypeUnknown;
                    arr = type == T_JSON ? (nx >> 18) & 1u : 0u;
                }
                // the text eager patterns compare: a string's contents, a literal's or an
                // integer's raw text (its String()); none for null, floats, containers
                int32_t ta = 0;
                uint32_t tn = 0xFFFFFFFFu;
                const int32_t ra = roff + (int32_t)vpos;
                if (type == T_STRING && !open && !esc) {
                    ta = ra + 1;
                    tn = end - vpos - 2u;
                } else if (type == T_NUMBER && !open) {  // literals must be exact (gjson takes any letters)
                    const uint32_t b0 = ring[ra];
                    const uint32_t n = end - vpos;
                    const uint64_t w = ring64(ring, ra);
                    for (uint32_t k = 0; k < n; k += 4u) {  // (gjson's scalar ends at a byte <= ' ')
                        const uint32_t q = ring32(ring, ra + (int32_t)k);
                        const uint32_t m = n - k >= 4 ? ~0u : (1u << (8u * (n - k))) - 1u;
                        if (le20_bytes(q) & m) {
                            bad |= 1u << i;
                            break;
                        }
                    }
                    if (b0 == 't' || b0 == 'f' || b0 == 'n') {
                        if (b0 == 't' && n == 4 && (uint32_t)w == 0x65757274u) type = T_TRUE;
                        else if (b0 == 'f' && n == 5 && (w & 0xFFFFFFFFFFull) == 0x65736C6166ull) type = T_FALSE;
                        else if (b0 == 'n' && n == 4 && (uint32_t)w == 0x6C6C756Eu) type = T_NULL;
                        else bad |= 1u << i;  // (left to the exact scan)
                        if (type == T_TRUE || type == T_FALSE) ta = ra, tn = n;
                    } else if (n <= 16) {  // -?[0-9]+ is its own String()
                        const uint64_t w1 = ring64(ring, ra + 8);
                        const uint32_t k0 = b0 == '-' ? 1u : 0u;
                        const uint64_t m0 = n >= 8 ? ~0ull : (1ull << (8 * n)) - 1ull;
                        const uint64_t m1 = n >= 16 ? ~0ull : n > 8 ? (1ull << (8 * (n - 8))) - 1ull : 0ull;
                        const uint64_t d0 = w ^ 0x3030303030303030ull, d1 = w1 ^ 0x3030303030303030ull;
                        const uint64_t nd0 = ((d0 + 0x7676767676767676ull) | d0) & 0x8080808080808080ull &
                                             m0 & ~(k0 ? 0xFFull : 0ull);
                        const uint64_t nd1 = ((d1 + 0x7676767676767676ull) | d1) & 0x8080808080808080ull & m1;
                        if (!nd0 && !nd1 && n > k0) ta = ra, tn = n;
                    }
                }
                // first match in document order: a second one sends the document to the exact scan
                const uint32_t prev = wave::lds_cas(reinterpret_cast<uint32_t*>(&row[1u + s]), kNone, vpos);
                if (prev != kNone) {
                    bad |= 1u << i;
                    continue;
                }
                const uint32_t meta = open ? (kOpenEnd | (kTypeUnknown << 24) | (arr << 29))
                                           : (((end - vpos) & 0xFFFFFFu) | (type << 24) | (esc << 27));
                reinterpret_cast<uint32_t*>(&row[1u + s])[1] = meta;
                // eager patterns on the value's text
                if (T.eg && tn != 0xFFFFFFFFu && s < T.ns) {
                    const EagerSel eg = T.eg[s];
                    const uint32_t hit = eager_hits(eg, ring, ta, tn);
                    uint64_t dD = 0, dT = 0;
#pragma unroll
                    for (int k = 0; k < 2; k++) {
                        const uint32_t em = eg.m[k], op = (em >> 8) & 0xFFu;
                        if (!(em & kEagerValid)) continue;
                        const uint64_t bit = 1ull << (em & 63u);
                        dD |= bit;
                        if (((hit >> k) & 1u) == (op == OP_EQ || op == OP_INCL ? 1u : 0u)) dT |= bit;
                    }
                    if (dD) {
                        wave::lds_or64(&dec[0], dD);
                        if (dT) wave::lds_or64(&dec[1], dT);
                    }
                }
            }
        }
        if (bad && live) wave::lds_min(&L.bad[doc], (uint32_t)(pos0 + (int32_t)ctz(bad)));
    }
    clk_at(clk, 3);  // (captures, eager patterns)
}

// Stage B's prelude for a value whose end the stream left open (long values, containers,
// a value in the next step): its type and end from the document, which the stream proved
// valid compact JSON. false: a literal gjson would read differently (exact scan).
AJX_HD bool resolve_open(const uint8_t* d, uint32_t n, uint32_t a, uint64_t* rec) {
    if (a >= n) return false;
    // the bytes come through one aligned 16-byte block at a time (a byte loop of global
    // loads would pay a load latency per byte)
    const V4* dq = reinterpret_cast<const V4*>((uintptr_t)d & ~(uintptr_t)15);
    const uint32_t dm = (uint32_t)((uintptr_t)d & 15u);
    uint32_t qi = 0xFFFFFFFFu;
    V4 q{0u, 0u, 0u, 0u};
    auto byte = [&](uint32_t i) -> uint32_t {
        const uint32_t g = i + dm;
        if ((g >> 4) != qi) {
            qi = g >> 4;
            q = dq[qi];
        }
        const uint32_t w = (g >> 2) & 3u;
        const uint32_t v = w == 0 ? q.x : w == 1 ? q.y : w == 2 ? q.z : q.w;
        return (v >> (8u * (g & 3u))) & 0xFFu;
    };
    const uint32_t b0 = byte(a);
    uint32_t type, end = a + 1u, esc = 0;
    if (b0 == '"') {
        type = T_STRING;
        while (end < n && byte(end) != '"') {
            if (byte(end) == '\\') {
                esc = 1;
                end++;
            }
            end++;
        }
        end++;
    } else if (b0 == '{' || b0 == '[') {
        type = T_JSON;
        uint32_t depth = 1;
        while (end < n && depth) {
            const uint32_t ch = byte(end);
            if (ch == '"') {
                end++;
                while (end < n && byte(end) != '"') end += byte(end) == '\\' ? 2u : 1u;
            } else if (ch == '{' || ch == '[') {
                depth++;
            } else if (ch == '}' || ch == ']') {
                depth--;
            }
            end++;
        }
    } else {
        type = T_NUMBER;
        while (end < n && byte(end) != ',' && byte(end) != '}' && byte(end) != ']') {
            if (byte(end) <= ' ') return false;  // (gjson's scalar would end there)
            end++;
        }
        const uint32_t k = end - a;
        if (b0 == 't' || b0 == 'f' || b0 == 'n') {  // literals must be exact (as the stream's)
            const bool t = b0 == 't' && k == 4 && byte(a + 1) == 'r' && byte(a + 2) == 'u' && byte(a + 3) == 'e';
            const bool f = b0 == 'f' && k == 5 && byte(a + 1) == 'a' && byte(a + 2) == 'l' && byte(a + 3) == 's' && byte(a + 4) == 'e';
            const bool z = b0 == 'n' && k == 4 && byte(a + 1) == 'u' && byte(a + 2) == 'l' && byte(a + 3) == 'l';
            if (!(t || f || z)) return false;
            type = t ? T_TRUE : f ? T_FALSE : T_NULL;
        }
    }
    if (end > n) return false;
    *rec = (uint64_t)a | ((uint64_t)(((end - a) & 0xFFFFFFu) | (type << 24) | (esc << 27)) << 32);
    return true;
}

// The arrays the stream compared element by element decide their selectors' incl / excl
// patterns: dD / dT (decided, true) from the eager words dw and the row's records.
AJX_HD void array_decisions(const EagerSel* eg, uint32_t ns, RowRef row, const uint64_t dw[4], uint64_t& dD,
                            uint64_t& dT, uint32_t s0 = 0, uint32_t sstep = 1) {
    if (!eg) return;
    for (uint32_t s = s0; s < ns && s < 32u; s += sstep) {
        const uint64_t rec = row[1u + s];
        const uint32_t meta = (uint32_t)(rec >> 32);
        if ((uint32_t)rec == kNone || !(meta & kOpenEnd) || !((meta >> 29) & 1u) || ((dw[3] >> s) & 1ull)) continue;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const uint32_t em = eg[s].m[k], op = (em >> 8) & 0xFFu;
            if (!(em & kEagerValid) || (op != OP_INCL && op != OP_EXCL)) continue;
            const uint64_t bit = 1ull << (em & 63u);
            dD |= bit;
            if (((dw[2] >> (2u * s + (uint32_t)k)) & 1ull) == (op == OP_INCL ? 1ull : 0ull)) dT |= bit;
        }
    }
}

// Folds request r when the stream decided every one of its patterns (eager patterns, arrays
// compared element by element, selectors not found): the T bitmap and every tree's
// result. false: some pattern needs stage B (ajx_stream_finish).
AJX_HD bool finish_light(uint32_t r, const uint8_t* blob, const Tabs& T, const uint64_t* row, const uint64_t dw[4],
                         uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err, uint64_t* __restrict__ out_bm,
                         uint32_t stride) {
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
    const uint32_t np = h->n_patterns;
    if (np > 64 || (h->static_error[0] | h->unsupported[0]) || T.exact) return false;
    uint64_t dD = dw[0], dT = dw[1];
    array_decisions(T.eg, T.ns, RowRef(row), dw, dD, dT);
    const SelectorPatterns* sps = reinterpret_cast<const SelectorPatterns*>(blob + h->off_sel_patterns);
    uint64_t t0 = dT & dD, all = dD;
    for (uint32_t s = 0; s < T.ns; s++)
        if ((uint32_t)row[1u + s] == kNone) {  // Null: the compiler's null_true bits
            t0 |= sps[s].mask[0] & h->null_true[0];
            all |= sps[s].mask[0];
        }
    const uint64_t want = np >= 64 ? ~0ull : (1ull << np) - 1ull;
    if ((all & want) != want) return false;
    const uint64_t t[2] = {t0 & want, 0ull}, u[2] = {0ull, 0ull}, se[2] = {0ull, 0ull};
    if (out_bm) {
        uint64_t* orow = out_bm + (size_t)r * stride;
        orow[0] = t[0];
        for (uint32_t w = 1; w < stride; w++) orow[w] = 0ull;
    }
    const uint32_t* code = reinterpret_cast<const uint32_t*>(blob + h->off_code);
    const uint32_t nt = h->pad1[0];
    if (nt == 0) {
        int32_t ep;
        out_tri[r] = (h->flags & kFlagFlatFold)    ? flat_fold(h, code, t, u, se, &ep)
                     : (h->flags & kFlagGroupFold) ? group_fold(h, code, t, u, se, &ep)
                                                   : run_fold_bits(code, h->n_code, t, u, se, &ep);
        if (out_err) out_err[r] = ep;
        return true;
    }
    const uint32_t* rc = reinterpret_cast<const uint32_t*>(blob + h->pad1[1]);
    const TreeFold* tf = h->pad1[2] ? reinterpret_cast<const TreeFold*>(blob + h->pad1[2]) : nullptr;
    for (uint32_t k = 0; k < nt; k++) {
        int32_t ep;
        out_tri[(size_t)r * nt + k] = tf && tf[k].shape ? tree_fold(tf[k], t, u, se, &ep)
                                                        : run_fold_bits(code + rc[2 * k], rc[2 * k + 1], t, u, se, &ep);
        if (out_err) out_err[(size_t)r * nt + k] = ep;
    }
    return true;
}

// Stage B for a request the stream did not decide (ajx_stream_finish, one work-item per
// request; its row in HBM: found word, records, the 4 eager words): the open values from
// the document, the arrays' decisions, ajx_fast.h's patterns_from_row, the T bitmap and the
// fold. false: the exact scan decides the request (the row is marked kRowSlow).
// dwp: the eager words (null: they follow the row's records, as in the stage-B rows).
// WAVE: all 64 lanes of a wave share the one request (the row in LDS): lane l resolves the
// records, tails and selectors l, l + 64, ...; the pattern bits meet by a wave-wide OR and
// lane 0 writes the outputs (the result is the same on every lane).
template <bool WAVE = false>
AJX_HD bool finish_full(uint32_t r, const uint8_t* blob, const uint8_t* d, uint32_t n, RowRef row,
                        uint8_t* __restrict__ out_tri, int32_t* __restrict__ out_err, uint64_t* __restrict__ out_bm,
                        uint32_t stride, const uint64_t* dwp = nullptr, uint64_t* clk = nullptr) {
    const uint32_t lane = WAVE ? wave::lane() : 0u, step = WAVE ? 64u : 1u;
    // (WAVE: a failure in any lane fails the request)
    auto fail_any = [&](bool f) -> bool {
        if constexpr (WAVE) return wave::ballot(f) != 0;
        return f;
    };
    const RulesetHdr* h = reinterpret_cast<const RulesetHdr*>(blob);
    const uint32_t ns = h->n_selectors;
    const StreamHdr* sh = reinterpret_cast<const StreamHdr*>(blob + h->off_stream);
    const uint32_t nr = sh->n_rec;
    const EagerSel* eg = h->off_eager ? reinterpret_cast<const EagerSel*>(blob + h->off_eager) : nullptr;
    const uint64_t dw[4] = {dwp ? dwp[0] : row[1u + nr], dwp ? dwp[1] : row[2u + nr], dwp ? dwp[2] : row[3u + nr],
                            dwp ? dwp[3] : row[4u + nr]};
    uint64_t dD = dw[0], dT = dw[1];
    array_decisions(eg, ns, row, dw, dD, dT, lane, step);
    // (WAVE: OR over the lanes)
    auto orall = [](uint64_t x) -> uint64_t {
        const auto OR = [](uint32_t a, uint32_t b) { return a | b; };
        const uint32_t lo = wave::readlane(wave::scan_incl((uint32_t)x, 0u, OR), 63);
        const uint32_t hi = wave::readlane(wave::scan_incl((uint32_t)(x >> 32), 0u, OR), 63);
        return (uint64_t)lo | ((uint64_t)hi << 32);
    };
    if constexpr (WAVE) {
        dD = orall(dD);
        dT = orall(dT);
    }
    clk_at(clk, 5);
    const SelectorPatterns* sps = reinterpret_cast<const SelectorPatterns*>(blob + h->off_sel_patterns);
    bool bad = false;
    for (uint32_t s = lane; s < nr; s += step) {
        uint64_t rec = row[1u + s];
        if ((uint32_t)rec == kNone || !((rec >> 32) & kOpenEnd)) continue;
        // (every pattern of the selector decided already: its value is not read; a forest's
        // rows are kept for authjx_select_from_eval_device, whose values must all be closed)
        if (s < ns && !h->pad1[0] && !(sps[s].mask[0] & ~dD) && !sps[s].mask[1]) continue;
        if (!resolve_open(d, n, (uint32_t)rec, &rec)) {
            bad = true;
            break;
        }
        row[1u + s] = rec;
    }
    if (fail_any(bad)) {
        if (lane == 0) row[0] = kRowSlow;
        return false;
    }
    if constexpr (WAVE) wave::sync();
    clk_at(clk, 6);
    // the selectors the stream does not follow to the end: the exact Get of the rest of the
    // path inside their prefix's value (or on the whole proved document)
    if (sh->n_tails) {
        const Selector* sels = reinterpret_cast<const Selector*>(blob + h->off_selectors);
        const Component* comps = reinterpret_cast<const Component*>(blob + h->off_components);
        const StreamTail* tl = reinterpret_cast<const StreamTail*>(blob + sh->off_tails);
        const uint8_t* lits = blob + h->off_literals;
        for (uint32_t k = lane; k < sh->n_tails; k += step) {
            const StreamTail e = tl[k];
            ValueRef v;
            v.type = T_NULL;
            v.start = v.end = 0;
            if (e.slot == 0xFFFFu) {  // (no prefix the stream follows: the whole document)
                v = gj_get(d, n, comps + sels[e.sel].comp_begin, sels[e.sel].comp_count, lits);
            } else {
                // the prefix's match is the document's only one (the stream sends a second
                // match of a record to the exact scan), so gjson's first complete match of
                // the whole path, if any, lies inside it
                uint64_t pre = row[1u + e.slot];
                if ((uint32_t)pre == kNone) continue;  // (no prefix: not found)
                // (a prefix whose own patterns were all decided may still be open)
                if (((pre >> 32) & kOpenEnd) && !resolve_open(d, n, (uint32_t)pre, &pre)) {
                    bad = true;
                    break;
                }
                const uint32_t a = (uint32_t)pre, len = (uint32_t)(pre >> 32) & 0xFFFFFFu;
                v = gj_get(d + a, len, comps + e.comp_begin, e.comp_count, lits);
                v.start += a;
                v.end += a;
            }
            if (v.type == T_NULL && v.start == v.end) continue;  // (not found: Null)
            row[1u + e.sel] = (uint64_t)v.start |
                              ((uint64_t)(((v.end - v.start) & 0xFFFFFFu) | ((uint32_t)v.type << 24) |
                                          ((uint32_t)(v.esc & 1u) << 27)) << 32);
            if constexpr (WAVE)
                wave::lds_or64(&row[0], 1ull << e.sel);
            else
                row[0] = row[0] | (1ull << e.sel);
        }
        if (fail_any(bad)) {
            if (lane == 0) row[0] = kRowSlow;
            return false;
        }
        if constexpr (WAVE) wave::sync();
    }
    clk_at(clk, 7);
    uint64_t t[2], u[2];
    const uint64_t dec[2] = {dD, dT};
    patterns_from_row(blob, d, row, t, u, dec, lane, step);
    if constexpr (WAVE) {  // (OR over the lanes)
        t[0] = orall(t[0]);
        t[1] = orall(t[1]);
        u[0] = orall(u[0]);
        u[1] = orall(u[1]);
    }
    clk_at(clk, 8);
    if ((u[0] & ~h->unsupported[0]) | (u[1] & ~h->unsupported[1])) {
        if (lane == 0) row[0] = kRowSlow;
        return false;
    }
    if (lane == 0 && out_bm) {
        uint64_t* orow = out_bm + (size_t)r * stride;
        orow[0] = t[0];
        if (stride > 1) orow[1] = t[1];
        for (uint32_t w = 2; w < stride; w++) orow[w] = 0ull;
    }
    const uint64_t se[2] = {h->static_error[0], h->static_error[1]};
    const uint32_t* code = reinterpret_cast<const uint32_t*>(blob + h->off_code);
    const uint32_t nt = h->pad1[0];
    // WAVE: every lane runs the (uniform) fold, its code words handed out from registers
    // (64 per coalesced read) instead of one dependent memory read each
    auto fold = [&](const uint32_t* c, uint32_t nc, int32_t* ep) -> uint8_t {
        // (one tree whose fold reads off the bitmaps: kFlagFlatFold / kFlagGroupFold)
        if (c == code && nt == 0 && (h->flags & kFlagGroupFold)) return group_fold(h, code, t, u, se, ep);
        if (!WAVE && c == code && nt == 0 && (h->flags & kFlagFlatFold)) return flat_fold(h, code, t, u, se, ep);
        if constexpr (WAVE) {
            // a flat All / Any (open, patterns, close; up to 64 words): the lanes hold one
            // word each and the result is the first leaf, in code order, that is not the
            // group's identity (the interpreter's sticky value), else the identity
            if (nc >= 3 && nc <= 64) {
                const uint32_t cw = lane < nc ? c[lane] : 0u;
                const uint32_t op0 = wave::readlane(cw, 0) >> 24, opl = wave::readlane(cw, nc - 1u) >> 24;
                const bool leaf = lane >= 1 && lane + 1u < nc;
                const uint64_t leaves = wave::ballot(leaf), pats = wave::ballot(leaf && (cw >> 24) == C_PAT);
                if ((op0 == C_OPEN_AND || op0 == C_OPEN_OR) && opl == C_CLOSE && pats == leaves) {
                    const uint32_t arg = cw & 0xFFFFFFu, q = arg >> 6;
                    const uint64_t bit = 1ull << (arg & 63u);
                    const uint32_t v = ((q ? se[1] : se[0]) & bit)  ? (uint32_t)V_E
                                       : ((q ? u[1] : u[0]) & bit) ? (uint32_t)V_U
                                       : ((q ? t[1] : t[0]) & bit) ? (uint32_t)V_T
                                                                    : (uint32_t)V_F;
                    const uint32_t ident = op0 == C_OPEN_OR ? (uint32_t)V_F : (uint32_t)V_T;
                    const uint64_t stick = wave::ballot(leaf && v != ident);
                    if (!stick) {
                        *ep = -1;
                        return (uint8_t)ident;
                    }
                    const uint32_t k = (uint32_t)__builtin_ctzll(stick);
                    const uint32_t vk = wave::readlane(v, k), ak = wave::readlane(arg, k);
                    *ep = (vk == V_E || vk == V_U) ? (int32_t)ak : -1;
                    return (uint8_t)vk;
                }
            }
            uint32_t creg = 0, cbase = 0xFFFFFFFFu;
            return run_fold_bits_f(
                [&](uint32_t k) -> uint32_t {
                    const uint32_t b = k & ~63u;
                    if (b != cbase) {
                        cbase = b;
                        creg = b + lane < nc ? c[b + lane] : 0u;
                    }
                    return wave::readlane(creg, k & 63u);
                },
                nc, t, u, se, ep);
        }
        return run_fold_bits(c, nc, t, u, se, ep);
    };
    if (nt == 0) {
        int32_t ep;
        const uint8_t v = fold(code, h->n_code, &ep);
        if (lane == 0) {
            out_tri[r] = v;
            if (out_err) out_err[r] = ep;
        }
        return true;
    }
    const uint32_t* rc = reinterpret_cast<const uint32_t*>(blob + h->pad1[1]);
    const TreeFold* tf = h->pad1[2] ? reinterpret_cast<const TreeFold*>(blob + h->pad1[2]) : nullptr;
    for (uint32_t k = 0; k < nt; k++) {
        int32_t ep;
        const uint8_t v = tf && tf[k].shape ? tree_fold(tf[k], t, u, se, &ep) : fold(code + rc[2 * k], rc[2 * k + 1], &ep);
        if (lane == 0) {
            out_tri[(size_t)r * nt + k] = v;
            if (out_err) out_err[(size_t)r * nt + k] = ep;
        }
    }
    return true;
}

enum : uint32_t { R_DONE = 0, R_SLOW = 1, R_STAGE_B = 2 };

// The whole span for this lane: setup, the steps, then request r = span * per + l
// (l < per <= kSpan requests per span): R_DONE (decided and folded; its row holds captures
// with possibly open ends), R_SLOW (the exact scan decides it) or R_STAGE_B (its row and
// eager words, *row_out / *dw_out, go to finish_full).
template <int MODE = 0>
AJX_HD uint32_t scan_span(WaveLds& L, uint64_t* rows, const uint8_t* blob, const uint8_t* __restrict__ arena,
                          const uint64_t* __restrict__ offs, const uint32_t* __restrict__ lens, uint32_t n,
                          uint32_t span, uint32_t per, uint32_t l, uint8_t* __restrict__ out_tri,
                          int32_t* __restrict__ out_err, uint64_t* __restrict__ out_bm, uint32_t stride,
                          const uint64_t** row_out, const uint64_t** dw_out, const uint8_t** lds_doc = nullptr,
                          uint64_t* clk = nullptr) {
    const Tabs T = tabs_of(blob);
    const uint32_t r = span * per + l;
    const bool my = l < per && r < n;
    const uint64_t off = my ? offs[r] : 0ull;
    const uint32_t len = my ? lens[r] : 0u;
    uint32_t my_start, total;
    span_setup(L, rows, T.nr, l, my, off, len, my_start, total);
    Carry c;
    carry_init(c);
    const uint32_t nsteps = (total + 63u) / 64u;
    // the next step's blocks are loaded while this one is processed
    Blk cur;
    uint64_t Hc;
    fetch(L, arena, 0, total, l, my_start, my, kNone, cur, Hc);
    uint32_t last_doc = kNone + (uint32_t)__builtin_popcountll(Hc);
    for (uint32_t t = 0; t < nsteps; t++) {
        Blk nxt{};
        uint64_t Hn = 0;
        if (t + 1u < nsteps) fetch(L, arena, t + 1u, total, l, my_start, my, last_doc, nxt, Hn);
        step<MODE>(L, rows, T, t, l, cur, Hc, c, t == 0 ? clk : nullptr);
        cur = nxt;
        Hc = Hn;
        last_doc += (uint32_t)__builtin_popcountll(Hn);
    }
    wave::sync();
    if (!my) return R_DONE;
    if constexpr (MODE == 1) {
        out_tri[r] = (uint8_t)(L.bad[l] > L.root_end[l]);
        return R_DONE;
    }
    const bool proved = L.root_end[l] != kNone && L.bad[l] > L.root_end[l];
    if (!proved) return R_SLOW;
    // (a span of one step: its documents are still in the ring, at ring index 64 + their
    // stream byte address)
    if (lds_doc && nsteps == 1) {
        const DocEnt e = L.doc[l];
        *lds_doc = L.ring_raw + 16 + 64 + e.start * 32u + (e.len_mis >> 24);
    }
    uint64_t* row = rows + (size_t)l * (1u + T.nr);
    const uint64_t* dp = rows + (size_t)kSpan * (1u + T.nr) + 4u * l;
    *row_out = row;
    *dw_out = dp;
    uint64_t found = 0;
    for (uint32_t s = 0; s < T.ns; s++)
        if ((uint32_t)row[1u + s] != kNone) found |= 1ull << s;
    row[0] = found;
    if constexpr (MODE == 2) {  // (profiling: no stage B)
        out_tri[r] = (uint8_t)(row[1] ^ dp[0] ^ dp[1] ^ dp[2]);
        return R_DONE;
    }
    const uint64_t dw[4] = {dp[0], dp[1], dp[2], dp[3]};
    return finish_light(r, blob, T, row, dw, out_tri, out_err, out_bm, stride) ? R_DONE : R_STAGE_B;
}

}  // namespace stream
}  // namespace ajx
