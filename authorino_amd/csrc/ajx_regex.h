// ajx_regex.h — reconcile-time compiler from a Go regexp (the `matches` operator,
// pkg/jsonexp/expressions.go:87-91) to a DFA the kernels run over rune classes.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "ajx_blob.h"

namespace ajx {

struct RegexDfa {
    uint32_t n_states = 0, n_classes = 0, start = 0, match_state = 0;
    std::vector<uint16_t> trans;  // [n_states * n_classes]
    std::vector<uint8_t> eot;     // [n_states]
    uint8_t ascii_class[128] = {};
    std::vector<RuneRange> ranges;  // runes >= 0x80, contiguous, sorted
};

enum RegexStatus { RX_OK = 0, RX_ERROR = 1, RX_UNSUPPORTED = 2 };

// Parses `pat` with Go 1.21 regexp.Compile rules (Perl flags). On a syntax error returns
// RX_ERROR with Go's message in *err ("error parsing regexp: ..."). Syntax the device
// compiler does not handle (\p{..} Unicode groups, case folding of non-ASCII runes,
// DFAs over kMaxDfaStates states) returns RX_UNSUPPORTED.
RegexStatus compile_go_regex(const std::string& pat, RegexDfa* out, std::string* err);

}  // namespace ajx
