// ajx_compiler.h — reconcile-time compiler: one flattened jsonexp tree -> ruleset blob.
// Hook point in the reference: controllers/auth_config_controller.go:805-852
// (buildJSONExpression / buildJSONExpressionPatterns / buildJSONExpressionPattern).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/authjx.h"
#include "ajx_blob.h"

namespace ajx {

struct CompiledRuleset {
    std::vector<uint8_t> blob;                // RulesetHdr + tables, copied to HBM as-is
    std::vector<int32_t> pattern_status;      // AUTHJX_PAT_*
    std::vector<std::string> pattern_error;   // static error text ("" when none)
    uint32_t n_patterns = 0;
    uint32_t n_selectors = 0;
    uint32_t max_depth = 0;
    uint32_t n_trees = 1;                     // fold programs (results per request)
};

// Split a gjson path into device components. Returns false when the path uses gjson
// syntax the device does not compile (modifiers, wildcards, '#', pipes, multipaths).
struct PathComponent {
    std::string key;      // object key, escapes removed (gjson parseObjectPath)
    int32_t array_index;  // gjson parseArrayPath + parseUint, -1 = matches no element
};
bool split_selector(const std::string& path, std::vector<PathComponent>* out);

// Returns AUTHJX_OK or an AUTHJX_E* code (malformed tree, nesting over kMaxDepth).
int compile_tree(const authjx_tree* tree, CompiledRuleset* out, std::string* err);
// Several trees as one ruleset (one scan of a document evaluates all of them).
int compile_forest(const authjx_tree* trees, uint32_t n_trees, CompiledRuleset* out, std::string* err);

}  // namespace ajx
