"""Host-side mirror of the JSON pattern-matching authorization evaluator and the
reconcile-time tree construction.

  JSONPatternMatching.call        pkg/evaluators/authorization/json.go:15-27
  UNAUTHORIZED ("Unauthorized")   pkg/evaluators/authorization/constants.go:4
  build_json_expression           controllers/auth_config_controller.go:805-852
                                  (buildJSONExpression / buildJSONExpressionPatterns /
                                  buildJSONExpressionPattern)

`call` evaluates one Authorization JSON; `call_batch` evaluates a micro-batch in one
device launch (the pkg/service micro-batcher's unit of work). Both run the HIP kernels
through libauthjx (authorino_amd.runtime); there is no CPU evaluation path.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Mapping, Optional, Sequence, Tuple

from . import jsonexp

UNAUTHORIZED = "Unauthorized"


class UnauthorizedError(Exception):
    """fmt.Errorf(unauthorizedErrorMsg) (json.go:24)."""

    def __init__(self):
        super().__init__(UNAUTHORIZED)


class JSONPatternMatching:
    """authorization.JSONPatternMatching{Rules jsonexp.Expression} (json.go:11-13)."""

    def __init__(self, rules: Optional[jsonexp.Expression] = None):
        self.rules = rules

    @staticmethod
    def _result(ok: bool, err: Optional[Exception]):
        if err is not None:  # json.go:20-22
            return False, err
        if not ok:  # json.go:23-25
            return False, UnauthorizedError()
        return True, None  # json.go:26

    def call(self, authorization_json) -> Tuple[object, Optional[Exception]]:
        """Call(pipeline, ctx) (interface{}, error) on pipeline.GetAuthorizationJSON()."""
        if self.rules is None:  # json.go:16-18
            return True, None
        return self._result(*self.rules.matches(authorization_json))

    Call = call

    def call_batch(self, docs: Sequence) -> List[Tuple[object, Optional[Exception]]]:
        if self.rules is None:
            return [(True, None)] * len(docs)
        return [self._result(ok, err) for ok, err in self.rules.matches_batch(docs)]


# ---- reconcile time: CRD JSONPattern lists -> jsonexp trees -------------------------
# A JSONPattern (api/v1beta1/auth_config_types.go:150-182) is given as a mapping with the
# CRD's JSON field names: "patternRef", "selector", "operator", "value", "all", "any".


def build_json_expression_pattern(expression: Mapping) -> jsonexp.Pattern:
    """buildJSONExpressionPattern (auth_config_controller.go:846-852)."""
    return jsonexp.Pattern(
        expression.get("selector", ""),
        jsonexp.operator_from_string(expression.get("operator", "")),
        expression.get("value", ""),
    )


def build_json_expression_patterns(named: Mapping[str, Sequence[Mapping]], pattern: Mapping) -> List[jsonexp.Expression]:
    """buildJSONExpressionPatterns (:830-844): the named patterns a ref points at, else
    the inline expression when it has an operator."""
    ref = pattern.get("patternRef", "")
    if ref in named:
        to_add = list(named[ref])
    elif pattern.get("operator", ""):
        to_add = [pattern]
    else:
        to_add = []
    return [build_json_expression_pattern(e) for e in to_add]


def build_json_expression(named: Mapping[str, Sequence[Mapping]], patterns: Sequence[Mapping],
                          op: Callable[..., jsonexp.Expression] = jsonexp.All) -> jsonexp.Expression:
    """buildJSONExpression (:805-828): per JSONPattern in order, its patterns/refs, then
    its `all` sub-list as an All, then its `any` sub-list as an Any; wrapped by `op`."""
    expression: List[jsonexp.Expression] = []
    for pattern in patterns:
        expression.extend(build_json_expression_patterns(named, pattern))
        if pattern.get("all"):
            expression.append(build_json_expression(named, pattern["all"], jsonexp.All))
        if pattern.get("any"):
            expression.append(build_json_expression(named, pattern["any"], jsonexp.Any))
    return op(*expression)


def named_patterns(spec_patterns: Optional[Mapping[str, Sequence[Mapping]]]) -> Dict[str, List[Mapping]]:
    """AuthConfig.Spec.Patterns (the named pattern sets a patternRef resolves against)."""
    return {k: list(v) for k, v in (spec_patterns or {}).items()}
