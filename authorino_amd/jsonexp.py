"""Host-side mirror of pkg/jsonexp (reference: pkg/jsonexp/expressions.go).

Same names, argument meaning and error behaviour as the Go package:

  Operator / operator_from_string      expressions.go:10-51
  Pattern(selector, operator, value)   expressions.go:53-57  (Matches: :59-96)
  And(left, right) / Or(left, right)   expressions.go:106-154 (nil sides allowed)
  All(*exprs) / Any(*exprs)            expressions.go:160-178 (right-nested chains)
  Expression.matches(json) -> (bool, error)   expressions.go:102-104

Evaluation never happens in Python: an expression is compiled (once) by libauthjx's
reconcile-time compiler into device tables, and `matches` / `matches_batch` run the HIP
kernels through the C-ABI (authorino_amd.runtime). There is no CPU fallback: without a
GPU and the built extension the calls raise.
"""
from __future__ import annotations

import enum
from typing import List, Optional, Sequence, Tuple


class Operator(enum.IntEnum):
    """jsonexp.Operator (expressions.go:10-19)."""

    UnknownOperator = 0
    EqualOperator = 1
    NotEqualOperator = 2
    IncludesOperator = 3
    ExcludesOperator = 4
    RegexOperator = 5

    def __str__(self) -> str:  # Operator.String, expressions.go:21-35
        return {1: "eq", 2: "neq", 3: "incl", 4: "excl", 5: "matches"}.get(int(self), "unknown")


UnknownOperator = Operator.UnknownOperator
EqualOperator = Operator.EqualOperator
NotEqualOperator = Operator.NotEqualOperator
IncludesOperator = Operator.IncludesOperator
ExcludesOperator = Operator.ExcludesOperator
RegexOperator = Operator.RegexOperator


def operator_from_string(s: str) -> Operator:
    """OperatorFromString (expressions.go:37-51)."""
    return {
        "eq": EqualOperator,
        "neq": NotEqualOperator,
        "incl": IncludesOperator,
        "excl": ExcludesOperator,
        "matches": RegexOperator,
    }.get(s, UnknownOperator)


OperatorFromString = operator_from_string

# Flat node encoding shared with the C-ABI (include/authjx.h, authjx_node).
NODE_PATTERN, NODE_AND, NODE_OR = 0, 1, 2


class Expression:
    """jsonexp.Expression (expressions.go:102-104)."""

    _compiled = None

    def matches(self, json: str | bytes) -> Tuple[bool, Optional[Exception]]:
        """Matches(json string) (bool, error) — evaluated on the GPU (batch of one)."""
        from . import runtime

        return runtime.expression_for(self).matches(json)

    Matches = matches

    def matches_batch(self, docs: Sequence[str | bytes]):
        """Evaluate many documents in one device batch; returns a list of (bool, error)."""
        from . import runtime

        return runtime.expression_for(self).matches_batch(docs)

    # -- flattening for the C-ABI --------------------------------------------
    def flatten(self) -> Tuple[List["Pattern"], List[Tuple[int, int, int, int]], int]:
        """Return (patterns, nodes, root) with nodes as (kind, left, right, pattern)."""
        patterns: List[Pattern] = []
        nodes: List[Tuple[int, int, int, int]] = []

        def walk(e: Optional[Expression]) -> int:
            if e is None:
                return -1
            if isinstance(e, Pattern):
                patterns.append(e)
                nodes.append((NODE_PATTERN, -1, -1, len(patterns) - 1))
                return len(nodes) - 1
            if isinstance(e, (And, Or)):
                idx = len(nodes)
                nodes.append((0, -1, -1, -1))  # placeholder, children first-come order
                left = walk(e.left)
                right = walk(e.right)
                nodes[idx] = (NODE_AND if isinstance(e, And) else NODE_OR, left, right, -1)
                return idx
            raise TypeError(f"not a jsonexp expression: {e!r}")

        root = walk(self)
        return patterns, nodes, root


class Pattern(Expression):
    """jsonexp.Pattern{Selector, Operator, Value} (expressions.go:53-57)."""

    def __init__(self, selector: str = "", operator: Operator | int | str = UnknownOperator, value: str = ""):
        self.selector = selector
        if isinstance(operator, str):
            operator = operator_from_string(operator)
        self.operator = Operator(int(operator)) if int(operator) in range(6) else int(operator)
        self.value = value

    def __repr__(self) -> str:  # Pattern.String, expressions.go:98-100
        return f"{self.selector} {Operator(self.operator) if isinstance(self.operator, Operator) else 'unknown'} {self.value}"


class And(Expression):
    """jsonexp.And{Left, Right} (expressions.go:106-125); nil sides are skipped."""

    def __init__(self, left: Optional[Expression] = None, right: Optional[Expression] = None):
        self.left = left
        self.right = right

    def __repr__(self) -> str:
        return f"({self.left} && {self.right})"


class Or(Expression):
    """jsonexp.Or{Left, Right} (expressions.go:131-154); nil sides are skipped."""

    def __init__(self, left: Optional[Expression] = None, right: Optional[Expression] = None):
        self.left = left
        self.right = right

    def __repr__(self) -> str:
        return f"({self.left} || {self.right})"


def All(*expressions: Expression) -> Expression:
    """All(expressions...) = And{e0, All(e1...)}; All() = And{} (expressions.go:160-168)."""
    out: Expression = And()
    for e in reversed(expressions):
        out = And(e, out)
    return out


def Any(*expressions: Expression) -> Expression:
    """Any(expressions...) = Or{e0, Any(e1...)}; Any() = Or{} (expressions.go:170-178)."""
    out: Expression = Or()
    for e in reversed(expressions):
        out = Or(e, out)
    return out
