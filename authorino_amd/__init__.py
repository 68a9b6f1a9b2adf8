"""authorino_amd — MI355X-native batched evaluator for Authorino's pattern-matching
authorization hot path (pkg/jsonexp + JSON pattern-matching authz + `when` conditions).

The product is libauthjx.so (authorino_amd/csrc, C-ABI declared in include/authjx.h):
a reconcile-time compiler from jsonexp trees to device-resident tables and HIP kernels
for gfx950 that evaluate micro-batches of Authorization-JSON documents. This Python
package mirrors the reference's Go interfaces on top of that C-ABI:

  authorino_amd.jsonexp        pkg/jsonexp/expressions.go   (Pattern, And, Or, All, Any)
  authorino_amd.authorization  pkg/evaluators/authorization/json.go (JSONPatternMatching) and
                               controllers/auth_config_controller.go:805-852 (CRD -> tree)
  authorino_amd.pipeline       pkg/service/auth_pipeline.go (evaluateConditions, authz phase)
  authorino_amd.runtime        C-ABI binding (ctypes), device context, batch evaluation
  authorino_amd.workloads      BASELINE configs c1-c3 (synthetic Authorization JSON, Go encoding)
"""
from . import jsonexp  # noqa: F401

from . import authorization, pipeline  # noqa: F401,E402

__all__ = ["jsonexp", "authorization", "pipeline"]
