"""Helpers to turn tests/golden/reference_kats.json trees into jsonexp expressions."""
import json
import os

from authorino_amd.jsonexp import All, And, Any, Or, Pattern, operator_from_string

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def build(tree):
    if tree is None:
        return None
    kind = tree[0]
    if kind == "pattern":
        return Pattern(tree[1], operator_from_string(tree[2]), tree[3])
    if kind == "and":
        return And(build(tree[1]), build(tree[2]))
    if kind == "or":
        return Or(build(tree[1]), build(tree[2]))
    if kind == "all":
        return All(*[build(t) for t in tree[1]])
    if kind == "any":
        return Any(*[build(t) for t in tree[1]])
    raise ValueError(kind)


def load_kats():
    with open(os.path.join(GOLDEN, "reference_kats.json")) as f:
        return json.load(f)["cases"]


def flat(expr):
    pats, nodes, root = expr.flatten()
    return [(p.selector, int(p.operator), p.value) for p in pats], nodes, root
