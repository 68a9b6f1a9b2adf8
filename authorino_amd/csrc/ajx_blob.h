// ajx_blob.h — layout of a compiled ruleset as it sits in HBM (one contiguous blob per
// ruleset, written by the reconcile-time compiler, read by the kernels).
//
// A ruleset is one jsonexp.Expression (pkg/jsonexp/expressions.go:102-104) compiled at
// the point the reference builds it (controllers/auth_config_controller.go:805-852):
//   selectors   deduplicated gjson paths, split into components the way gjson v1.14.0
//               parseObjectPath / parseArrayPath split them (escapes removed for object
//               keys, numeric index for arrays)
//   patterns    (selector, op, literal, dfa) per jsonexp.Pattern
//   code        fold bytecode of the And/Or tree: right-nested All/Any chains are
//               flattened to n-ary AND/OR nodes whose value is the first child value
//               that is not the node's identity (T for AND, F for OR) — exactly the
//               short-circuit results of And.Matches :111-125 / Or.Matches :136-154
//   literals    byte pool (component keys, pattern values)
//   dfas        Go-regexp DFAs over rune classes (one per `matches` pattern)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define AJX_BLOB_HD __host__ __device__
#else
#define AJX_BLOB_HD
#endif

namespace ajx {

constexpr uint32_t kMagic = 0x414A5842u;  // "AJXB"
constexpr uint32_t kMaxComponents = 16;    // selector depth compiled for the device
constexpr uint32_t kMaxDepth = 16;         // AND/OR nesting depth of the fold code
constexpr uint32_t kMaxDfaStates = 4096;
constexpr uint32_t kMaxDfaClasses = 255;

// gjson.Type
enum : uint8_t { T_NULL = 0, T_FALSE = 1, T_NUMBER = 2, T_STRING = 3, T_TRUE = 4, T_JSON = 5 };
// tri-state values (= AUTHJX_F/T/E/UNDECIDED)
enum : uint8_t { V_F = 0, V_T = 1, V_E = 2, V_U = 3 };
// pattern state
enum : uint8_t { P_OK = 0, P_STATIC_E = 1, P_UNSUPPORTED = 2 };
// ops (= AUTHJX_OP_*)
enum : uint8_t { OP_UNKNOWN = 0, OP_EQ = 1, OP_NEQ = 2, OP_INCL = 3, OP_EXCL = 4, OP_MATCHES = 5 };
// fold code (op in bits 24..31, argument in bits 0..23)
enum : uint32_t { C_OPEN_AND = 1, C_OPEN_OR = 2, C_PAT = 3, C_CLOSE = 4, C_CONST_T = 5, C_CONST_F = 6 };

// Component::array_index of a last path part that is exactly "#": on an array, gjson's
// parseArray answers the element count (Number, Raw = strconv.Itoa, at the ']'); on an
// object the part is the key "#"
constexpr int32_t kArrCount = -2;
// ... of a part "#" followed by more parts (gjson's alog, "friends.#.first"): on an array,
// the JSON array of Get(element, rest) over the elements where it exists (raw values,
// comma-joined, at the ']'); on an object the part is the key "#" and the path goes on
constexpr int32_t kArrList = -3;

struct Component {
    uint32_t lit_off;     // object-key bytes (escapes removed) in the literal pool
    uint32_t lit_len;
    int32_t array_index;  // element index when the value is an array, -1 = never, kArrCount
    uint32_t hash;        // FNV-1a of the key bytes
};

struct Selector {
    // 8 B (u16 fields: the compiler caps components and modifiers at 65535), so that the
    // LDS-staged blob stays small (it shares a CU's 160 KiB with the window rings)
    uint16_t comp_begin;
    uint16_t comp_count;
    uint16_t mod_begin;  // gjson modifiers applied to the path's value (Modifier records)
    uint16_t mod_count;
};

// The reference's custom gjson modifiers (pkg/json/json.go:161-264, registered at
// :258-264), applied in order to the raw JSON of the selected value (a path such as
// `auth.identity.email.@extract:{"sep":"@","pos":1}|@case:upper`). Evaluated by the
// exact scan only (ajx_modifiers.h).
// M_FROMSTR is gjson's own @fromstr (v1.14.0 modFromStr: Parse(json).String() of a Valid
// text); M_PATH is the path gjson Gets from a modifier's output (`@fromstr|a.b`,
// a_off / a_len: its Components).
enum : uint8_t { M_EXTRACT = 1, M_REPLACE = 2, M_CASE = 3, M_BASE64 = 4, M_STRIP = 5, M_FROMSTR = 6, M_PATH = 7 };
struct Modifier {
    uint8_t kind;
    uint8_t variant;  // CASE 1 upper / 2 lower; BASE64 1 encode / 2 decode; 0: returns its input
    uint16_t pad;
    uint32_t a_off, a_len;  // EXTRACT: sep; REPLACE: old (literal pool)
    uint32_t b_off, b_len;  // REPLACE: new
    uint32_t pos;           // EXTRACT: part index
};

struct Pattern {
    uint32_t selector;
    uint8_t op;
    uint8_t state;
    uint16_t litf;     // kLit*: the literal equals "true" / "false" / "" (String() of a literal value)
    uint32_t lit_off;
    uint32_t lit_len;
    uint32_t dfa_off;  // byte offset of a DfaHdr in the blob (0 = none)
};

constexpr uint16_t kLitTrue = 1, kLitFalse = 2, kLitEmpty = 4;

struct DfaHdr {
    uint32_t n_states;
    uint32_t n_classes;
    uint32_t start;
    uint32_t match_state;  // absorbing accept
    uint32_t trans_off;    // uint16_t[n_states * n_classes], blob offset
    uint32_t eot_off;      // uint8_t[n_states]: accept at end of text
    uint32_t ranges_off;   // RuneRange[n_ranges] for runes >= 0x80, sorted by lo
    uint32_t n_ranges;
    uint8_t ascii_class[128];
};

struct RuneRange {
    uint32_t lo, hi, cls, pad;
};

// ---- single-pass fast path: selector trie ---------------------------------------
// All selectors of a ruleset merged into one trie over path components; node 0 is
// the document root. A key (object context) or an element index (array context)
// moves from a node to one of its children.
constexpr uint32_t kFastMaxPatterns = 128;
constexpr uint32_t kFastMaxNodes = 255;
constexpr uint32_t kFastMaxSelectors = 63;  // found bits 0..62 (bit 63 of the row header is kRowSlow)
constexpr uint8_t kNoNode = 0xFF;

struct TrieNode {
    uint16_t child_begin;  // index into TrieChild[]
    uint8_t n_children;
    uint8_t flags;         // bit0: has array-index children
    int16_t selector;      // selector whose path ends here, -1 none
    uint16_t pad;
};

// A key is matched by (length, signature) where the signature is its last min(8, len)
// bytes little-endian (key byte len-m+j in bits 8j..8j+7) — the bytes just before the
// closing quote, which the scanner still holds in registers; longer keys then compare
// their first len-8 bytes against the literal pool.
struct TrieChild {
    uint64_t sig;
    uint32_t key_len;
    uint32_t key_off;      // key bytes in the literal pool
    int32_t array_index;   // -1 never matches an element
    uint32_t node;
};
static_assert(sizeof(Selector) == 8, "Selector layout");
static_assert(sizeof(TrieChild) == 24, "TrieChild layout");
static_assert(sizeof(TrieNode) == 8, "TrieNode layout");

AJX_BLOB_HD inline uint64_t key_signature(const uint8_t* key, uint32_t len) {
    const uint32_t m = len < 8 ? len : 8;
    uint64_t s = 0;
    for (uint32_t j = 0; j < m; j++) s |= (uint64_t)key[len - m + j] << (8 * j);
    return s;
}

// Key lookup for the single-pass path: every (parent node, key) edge of the trie in
// one open-addressing table (linear probing), so a closing key quote costs one 16-byte
// LDS read instead of a walk over the parent's children.
struct KeySlot {
    uint64_t sig;       // key_signature(key)
    uint32_t meta;      // key_len | parent << 16 | node << 24; kEmptySlot = free
    uint16_t key_off8;  // key bytes in the literal pool, / 8 (keys are 8-byte aligned)
    uint16_t pad;
};
static_assert(sizeof(KeySlot) == 16, "KeySlot layout");
constexpr uint32_t kEmptySlot = 0xFFFFFFFFu;
constexpr uint32_t kMaxKeySlotsLog2 = 9;
constexpr uint32_t kKeyProbes = 4;  // the table is grown until every key is this close to home

// (mult: an odd multiplier the compiler picks per ruleset, so that keys sit in their home
// slots; key_mult in the header)
AJX_BLOB_HD inline uint32_t key_slot_hash(uint64_t sig, uint32_t klen, uint32_t parent, uint32_t log2,
                                          uint32_t mult) {
    uint32_t x = (uint32_t)sig ^ (((uint32_t)(sig >> 32) << 13) | ((uint32_t)(sig >> 32) >> 19)) ^ (klen << 24) ^
                 (parent << 16);
    x *= mult;
    return x >> (32 - log2);
}
// the key-length field of a key-table entry that is an array index (sig = the index): the
// lean scan looks up array elements in the same table (keys that long go to the exact scan)
constexpr uint32_t kIndexKeyLen = 0xFFFFu;

struct SelectorPatterns {
    uint32_t begin;        // index into the uint16 pattern list
    uint32_t count;
    uint64_t mask[2];      // the same patterns as a bitmask
};

struct RulesetHdr {
    uint32_t magic;
    uint32_t total_bytes;
    uint32_t n_patterns;
    uint32_t n_selectors;
    uint32_t n_code;
    uint32_t max_depth;
    uint32_t off_selectors;
    uint32_t off_components;
    uint32_t off_patterns;
    uint32_t off_code;
    uint32_t off_literals;
    uint32_t lit_bytes;
    uint32_t n_components;
    uint32_t flags;  // bit0: has regex; bit1: has unsupported pattern; bit2: fast path ok
    uint32_t n_trie_nodes;
    uint32_t off_trie_nodes;
    uint32_t off_trie_children;
    uint32_t off_sel_patterns;  // SelectorPatterns[n_selectors]
    uint32_t off_pattern_lists; // uint16_t[]
    uint32_t key_slots_log2;    // KeySlot table of 1 << key_slots_log2 entries
    uint32_t off_key_slots;
    uint32_t pad1[3];
    uint32_t off_modifiers;     // Modifier[n_modifiers]
    uint32_t n_modifiers;
    uint32_t hot_bytes;         // [0, hot_bytes): every table the single-pass kernels read
                                // (selectors, components, modifiers follow: exact scan only)
    uint32_t key_probes;        // every key sits within key_probes slots of its home slot
    uint32_t key_mult;          // key_slot_hash multiplier
    uint32_t off_eager;         // EagerSel[n_selectors] (0: none)
    uint32_t off_stream;        // StreamHdr (0: the streaming scan can not take this ruleset)
    uint32_t lean_feat;         // walker features the ruleset needs: kLeanArr | kLeanCaps
    uint64_t null_true[2];      // pattern p is T when its selector finds nothing (Null)
    uint64_t static_error[2];   // pattern p is a static E
    uint64_t unsupported[2];    // pattern p can not be decided on the device
    // kFlagGroupFold: {patterns in Any groups, patterns in groups, each group's first pattern}
    uint64_t fold_grp[3];
};
constexpr uint32_t kFlagFastOk = 4;
// RulesetHdr::lean_feat: some trie node has array-index children (the lean walk enters
// arrays); some selector's node has children (a captured container is walked into)
constexpr uint32_t kLeanArr = 1, kLeanCaps = 2;

constexpr uint32_t kFlagBufs = 8;  // a selector builds a text (a '#' list): the exact scan's buffers
// the fold code is one flat All / Any of patterns 0..n_patterns - 1 in order (n_patterns
// <= 64, one tree): its result is the first pattern, in index order, that is not the
// group's identity (fold_outputs reads it off the bitmaps, no code interpreted)
constexpr uint32_t kFlagFlatFold = 16;
// the fold code is one All / Any whose children are patterns and groups of the other kind
// over patterns only, patterns 0..n_patterns - 1 in code order (n_patterns <= 64, one
// tree; c3's All(Any x4, All x4) flattens to one): group_fold reads it off the bitmaps,
// one step per group, with the group layout in RulesetHdr::fold_grp
constexpr uint32_t kFlagGroupFold = 32;
// A forest's trees of the same shapes (RulesetHdr::pad1[2]: offset of TreeFold[n_trees], 0
// when the forest has none): tree k's patterns base .. base + n - 1 in code order
// (n <= 64), its fold read off those bits of the bitmaps; shape 0: the code is interpreted
struct TreeFold {
    uint32_t base, n, shape, any;  // shape 1: one flat All / Any or a two-level one
    uint64_t g_any, g_in, g_start;  // as RulesetHdr::fold_grp, bit j = pattern base + j
};

// Patterns the lean scan decides while it captures (ajx_lean.h): per selector, its first
// two patterns (index < 64) that compare an unescaped string value's text with a literal
// of at most 16 bytes (eq, neq, incl / excl on the value alone); a literal value (true /
// false / null) decides them by the literal's litf. (The streaming kernel also compares
// arrays of strings with them, element by element.) m: pattern | op << 8 | literal length << 16 | litf << 24 | 1 << 31.
// pad[0] bit 0 (kEagerAll): those are every pattern of the selector (a decided value needs
// no capture record for stage B); bit 1 (kEagerKeep): a selector of a forest's root-less
// tree, whose record a caller reads back (authjx_select_from_eval_device): written whenever
// the kernel keeps rows.
struct EagerSel {
    uint32_t lit[2][4];
    uint32_t m[2];
    uint32_t pad[2];
};
static_assert(sizeof(EagerSel) == 48, "EagerSel layout");
constexpr uint32_t kEagerValid = 1u << 31;  // EagerSel::m[k] holds an eager pattern
constexpr uint32_t kEagerAll = 1u;           // EagerSel::pad[0]
constexpr uint32_t kEagerKeep = 2u;          // EagerSel::pad[0]

// ---- streaming scan (ajx_stream.h) ------------------------------------------------
// The stream resolves object keys without their parent: every distinct object key of the
// trie has an id 1..kStreamMaxKeys (0: not a key of any selector). A key of the document
// at depth L is then named by the ids of the keys its containers were opened under
// (levels 2..L) followed by its own: the path bytes, byte j = component j + 1. A selector
// is found where those bytes equal its components' ids (the path table). Rulesets the
// stream takes: the single-pass path's (kFlagFastOk), selectors of at most
// kStreamMaxComps object keys (no array indices), keys of at most kStreamMaxKeyLen bytes.
constexpr uint32_t kStreamMaxKeys = 250;
constexpr uint32_t kStreamMaxComps = 8;
constexpr uint32_t kStreamMaxKeyLen = 64;
constexpr uint32_t kStreamElem = 0xFE;  // the id of an array element's container

struct StreamKeySlot {
    uint64_t sig;      // key_signature(key)
    uint32_t meta;     // key_len | id << 16; kEmptySlot = free
    uint32_t key_off;  // key bytes in the literal pool
};
struct StreamPathSlot {
    uint64_t path;     // component ids, byte j = component j + 1
    uint32_t meta;     // selector (0xFFFF: none) | kStreamHasKids | 1 << 31; 0 = free
    uint32_t pad;
};
constexpr uint32_t kStreamHasKids = 1u << 30;  // a path node with keys below it
static_assert(sizeof(StreamKeySlot) == 16 && sizeof(StreamPathSlot) == 16, "stream slot layout");

struct StreamHdr {
    uint32_t off_keys, key_log2, key_mult, key_probes;      // StreamKeySlot[1 << key_log2]
    uint32_t off_paths, path_log2, path_mult, path_probes;  // StreamPathSlot[1 << path_log2]
    uint32_t n_keys, max_key_len;
    uint32_t light;  // every pattern is an eager one (EagerSel): stage B is the fold alone
    uint32_t n_rec;  // capture records per request: the selectors', then the extra prefixes'
    // selectors the stream does not follow to the end (an array index, more than
    // kStreamMaxComps components, a key longer than kStreamMaxKeyLen): stage B takes their
    // values with the exact Get inside their longest followed prefix's captured value
    // (StreamTail), or on the whole proved document
    uint32_t exact_lo, exact_hi;
    uint32_t off_tails, n_tails;  // StreamTail[n_tails]
};
struct StreamTail {
    uint16_t sel;         // the selector
    uint16_t slot;        // the record of its prefix's value (0xFFFF: no prefix, whole document)
    uint16_t comp_begin;  // the rest of its path: components [comp_begin, comp_begin + comp_count)
    uint16_t comp_count;
};

AJX_BLOB_HD inline uint32_t stream_path_hash(uint64_t p, uint32_t log2, uint32_t mult) {
    uint32_t x = (uint32_t)p ^ (((uint32_t)(p >> 32) << 11) | ((uint32_t)(p >> 32) >> 21));
    x *= mult;
    return x >> (32 - log2);
}

}  // namespace ajx
