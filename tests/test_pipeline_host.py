"""Host logic of the authorization mirrors (authorino_amd.authorization / .pipeline) on
CPU: the device context is replaced by a stand-in that evaluates with the oracle, so
these tests check the `when` gating, priorities, deny selection, error texts and the
CRD -> tree construction — not the kernels (tests/test_gpu_parity.py::test_pipeline_*
runs the same cases on the GPU).

Cases follow pkg/service/auth_pipeline_test.go:389-495 (conditions at AuthConfig and
evaluator level), pkg/evaluators/authorization/json_test.go (Unauthorized / regex error)
and controllers/auth_config_controller.go:805-852 (tree order)."""
import json
import re

import numpy as np
import pytest

import pyoracle as O
from authorino_amd import authorization as AZ
from authorino_amd import jsonexp as J
from authorino_amd import pipeline as P


class _OracleRuleset:
    def __init__(self, expr):
        pats, nodes, root = expr.flatten()
        self.rs = O.Ruleset([(p.selector, int(p.operator), p.value) for p in pats], nodes, root)
        self.n_patterns = len(pats)

    def pattern_error(self, i):
        return self.rs.error(i)


class _OracleForest:
    def __init__(self, exprs):
        self.trees = [_OracleRuleset(e) for e in exprs]
        self.offsets = list(np.cumsum([0] + [t.n_patterns for t in self.trees])[:-1])
        self.n_trees = len(self.trees)

    def pattern_error(self, i):
        k = max(j for j, o in enumerate(self.offsets) if o <= i and self.trees[j].n_patterns > i - o)
        return self.trees[k].pattern_error(i - self.offsets[k])


class _OracleSelectors:
    def __init__(self, pats):
        self.paths = [p[0] for p in pats]
        self.n_patterns = len(pats)
        self.status = [0] * len(pats)


class OracleCtx:
    """Stand-in for runtime.Context with the calls the pipeline makes."""

    def __init__(self):
        self.launches = 0

    def compile_expression(self, expr):
        return _OracleRuleset(expr)

    def compile_forest(self, exprs):
        return _OracleForest(exprs)

    def compile(self, pats, nodes, root):  # selector-only rulesets (response selectors)
        return _OracleSelectors(pats)

    def select_host_arena(self, sets, arena, offs, lens, set_of_req=None):
        n = len(lens)
        out = np.zeros((n, max(s.n_patterns for s in sets), 3), dtype=np.uint32)
        for r in range(n):
            doc = arena[int(offs[r]):int(offs[r]) + int(lens[r])].tobytes()
            for p, path in enumerate(sets[0 if set_of_req is None else int(set_of_req[r])].paths):
                try:
                    t, st, ln = O.gjson_span(doc, path)
                except ValueError:  # modifiers: not a span of the document (device: 0xFF)
                    t, st, ln = 255, 0, 0
                out[r, p] = (st, ln, t)
        return out

    def select_text_host_arena(self, sets, arena, offs, lens, set_of_req=None, text_stride=4096):
        """authjx_select_text_batch's contract: document spans, or (modifier chains, "#."
        lists) the oracle's raw Result text in the request's slot, esc | VALUE_TEXT."""
        n = len(lens)
        out = np.zeros((n, max(s.n_patterns for s in sets), 3), dtype=np.uint32)
        text = np.zeros((n, text_stride), dtype=np.uint8)
        for r in range(n):
            doc = arena[int(offs[r]):int(offs[r]) + int(lens[r])].tobytes()
            used = 0
            for p, path in enumerate(sets[0 if set_of_req is None else int(set_of_req[r])].paths):
                if "@" not in path and not re.search(r"(^|(?<!\\)\.)#\.", path):
                    t, st, ln = O.gjson_span(doc, path)
                    out[r, p] = (st, ln, t)
                    continue
                got = O.gjson_get_mods(doc, path)
                if got is None or used + len(got[1]) > text_stride:
                    out[r, p] = (0, 0, 255)
                    continue
                t, raw = got
                if not raw:  # (Null: no text)
                    out[r, p] = (0, 0, t)
                    continue
                text[r, used:used + len(raw)] = np.frombuffer(raw, dtype=np.uint8)
                esc = (1 if t == 3 and b"\\" in raw else 0) | 4
                out[r, p] = (used, len(raw), t | esc << 8)
                used += len(raw)
        return out, text

    def eval_host_arena(self, sets, arena, offs, lens, set_of_req=None, with_bitmap=True):
        self.launches += 1
        if isinstance(sets[0], _OracleForest):  # one result per tree, errors in forest numbering
            f = sets[0]
            res = [O.eval_batch([t.rs], arena, offs, lens) for t in f.trees]
            tri = np.stack([r[0] for r in res], axis=1)
            err = np.stack([np.where(r[1] >= 0, r[1] + o, r[1]) for r, o in zip(res, f.offsets)], axis=1)
            return tri, err, None
        tri, err, bm = O.eval_batch([s.rs for s in sets], arena, offs, lens, set_of_req=set_of_req)
        return tri, err, (bm if with_bitmap else None)


def _doc(path="/operation", sub="alice", groups=("users",), authz=None):
    d = {"context": {"request": {"http": {"method": "GET", "path": path}}},
         "auth": {"authorization": authz or {}, "identity": {"groups": list(groups), "sub": sub},
                  "metadata": {}, "response": {}}}
    return json.dumps(d, separators=(",", ":")).encode()


def test_authconfig_conditions_gate():
    """auth_pipeline_test.go:389-437: AuthConfig-level `when` not met -> OK, nothing runs."""
    cfg = P.AuthConfig(
        conditions=J.All(J.Pattern("context.request.http.path", J.NotEqualOperator, "/operation")),
        authorization=[P.AuthorizationConfig("deny-all", rules=J.All(J.Pattern("auth.identity.sub", J.EqualOperator, "nobody")))],
    )
    ctx = OracleCtx()
    res = P.AuthPipelineBatch(cfg, ctx=ctx).evaluate([_doc("/operation"), _doc("/other")])
    assert res[0].skipped and res[0].code == P.CODE_OK  # conditions unmet: skipped, allowed
    assert not res[1].skipped and res[1].code == P.CODE_PERMISSION_DENIED
    assert res[1].message == "Unauthorized" and res[1].denied_by == "deny-all"


def test_evaluator_conditions_gate():
    """auth_pipeline_test.go:439-495: evaluator-level `when` not met -> evaluator ignored."""
    rules = J.All(J.Pattern("auth.identity.sub", J.EqualOperator, "nobody"))
    cond = J.All(J.Pattern("context.request.http.path", J.EqualOperator, "/operation"))
    cfg = P.AuthConfig(authorization=[P.AuthorizationConfig("gated", rules=rules, conditions=cond)])
    res = P.AuthPipelineBatch(cfg, ctx=OracleCtx()).evaluate([_doc("/operation"), _doc("/elsewhere")])
    assert res[0].code == P.CODE_PERMISSION_DENIED
    assert res[1].code == P.CODE_OK and res[1].authorization == {}


def test_priorities_and_first_denial():
    ok = J.All(J.Pattern("auth.identity.groups", J.IncludesOperator, "users"))
    bad_re = J.All(J.Pattern("context.request.http.path", J.RegexOperator, "(["))
    deny = J.All(J.Pattern("auth.identity.sub", J.EqualOperator, "bob"))
    cfg = P.AuthConfig(authorization=[
        P.AuthorizationConfig("p1-regex", rules=bad_re, priority=1),
        P.AuthorizationConfig("p0-ok", rules=ok, priority=0),
        P.AuthorizationConfig("p0-deny", rules=deny, priority=0),
        P.AuthorizationConfig("p0-nil", rules=None, priority=0),
    ])
    ctx = OracleCtx()
    res = P.AuthPipelineBatch(cfg, ctx=ctx).evaluate([_doc(sub="bob"), _doc(sub="alice")])
    # request 0 passes priority 0 and fails priority 1 on the regex's static error
    assert res[0].code == P.CODE_PERMISSION_DENIED and res[0].denied_by == "p1-regex"
    assert res[0].message.startswith("error parsing regexp: missing closing ]")
    assert res[0].authorization == {"p0-ok": True, "p0-deny": True, "p0-nil": True}
    # request 1 is denied at priority 0; priority 1 never runs for it
    assert res[1].code == P.CODE_PERMISSION_DENIED and res[1].denied_by == "p0-deny"
    assert ctx.launches == 1  # one forest launch: no later priority reads auth.authorization.*


def test_later_priority_reads_earlier_authorization():
    """auth_pipeline.go:312 / :556-560: a granted config is auth.authorization.<name> for
    later priorities; the producer rebuilds the document."""
    cfg = P.AuthConfig(authorization=[
        P.AuthorizationConfig("first", rules=J.All(J.Pattern("auth.identity.sub", J.EqualOperator, "alice"))),
        P.AuthorizationConfig("second", priority=1,
                              rules=J.All(J.Pattern("auth.authorization.first", J.EqualOperator, "true"))),
    ])
    batch = P.AuthPipelineBatch(cfg, ctx=OracleCtx())
    docs = [_doc(sub="alice"), _doc(sub="bob")]
    with pytest.raises(ValueError):
        batch.evaluate(docs)
    subs = ["alice", "bob"]
    res = batch.evaluate(docs, producer=lambda i, objs: _doc(sub=subs[i], authz=objs))
    assert res[0].code == P.CODE_OK and res[0].authorization == {"first": True, "second": True}
    assert res[1].code == P.CODE_PERMISSION_DENIED and res[1].denied_by == "first"


def test_json_pattern_matching_call_results():
    """authorization/json.go:15-27 result mapping (rules nil / T / F / E)."""
    m = AZ.JSONPatternMatching(None)
    assert m.call(b"{}") == (True, None)
    assert AZ.JSONPatternMatching._result(True, None) == (True, None)
    ok, err = AZ.JSONPatternMatching._result(False, None)
    assert ok is False and str(err) == "Unauthorized"
    e = RuntimeError("error parsing regexp: x")
    assert AZ.JSONPatternMatching._result(False, e) == (False, e)


def _shape(e):
    if e is None:
        return None
    if isinstance(e, J.Pattern):
        return (e.selector, int(e.operator), e.value)
    return (type(e).__name__, _shape(e.left), _shape(e.right))


def test_build_json_expression_order():
    """auth_config_controller.go:805-852: per JSONPattern, refs/inline first, then `all`,
    then `any`; unknown operator strings map to UnknownOperator; empty list = All()."""
    named = {"admins": [{"selector": "auth.identity.groups", "operator": "incl", "value": "admins"},
                        {"selector": "auth.identity.sub", "operator": "neq", "value": ""}]}
    spec = [
        {"patternRef": "admins"},
        {"selector": "context.request.http.method", "operator": "eq", "value": "GET",
         "all": [{"selector": "a", "operator": "eq", "value": "1"}],
         "any": [{"selector": "b", "operator": "matches", "value": "^x"}, {"patternRef": "admins"}]},
        {"selector": "x", "operator": "bogus", "value": "v"},
        {"patternRef": "missing"},
    ]
    expr = AZ.build_json_expression(named, spec)
    want = J.All(
        J.Pattern("auth.identity.groups", J.IncludesOperator, "admins"),
        J.Pattern("auth.identity.sub", J.NotEqualOperator, ""),
        J.Pattern("context.request.http.method", J.EqualOperator, "GET"),
        J.All(J.Pattern("a", J.EqualOperator, "1")),
        J.Any(J.Pattern("b", J.RegexOperator, "^x"), J.Pattern("auth.identity.groups", J.IncludesOperator, "admins"),
              J.Pattern("auth.identity.sub", J.NotEqualOperator, "")),
        J.Pattern("x", J.UnknownOperator, "v"),
    )
    assert _shape(expr) == _shape(want)
    assert _shape(AZ.build_json_expression(named, [])) == _shape(J.All())
    # the built tree evaluates like the hand-built one (oracle)
    doc = _doc()
    r1 = O.Ruleset.from_expression(expr).matches(doc)
    r2 = O.Ruleset.from_expression(want).matches(doc)
    assert r1 == r2


def test_batch_matches_single_requests():
    """Randomised: the batched phase gives, per request, what evaluating its configs one
    document at a time gives (the sequential restatement of auth_pipeline.go:287-322)."""
    rng = np.random.default_rng(3)
    paths = ["/operation", "/api/v1/orders/7", "/admin", "/x"]
    subs = ["alice", "bob", "carol"]
    groups = ["users", "admins", "devs"]
    cfgs = []
    for k in range(6):
        rules = J.Any(J.Pattern("auth.identity.sub", J.EqualOperator, str(rng.choice(subs))),
                      J.Pattern("auth.identity.groups", J.IncludesOperator, str(rng.choice(groups))))
        cond = None if rng.random() < 0.4 else J.All(
            J.Pattern("context.request.http.path", J.RegexOperator, "^/" + str(rng.choice(["api", "op", "a"]))))
        cfgs.append(P.AuthorizationConfig(f"c{k}", rules=rules, conditions=cond, priority=int(rng.integers(0, 3))))
    cfg = P.AuthConfig(conditions=J.All(J.Pattern("context.request.http.path", J.NotEqualOperator, "/x")),
                       authorization=cfgs)
    docs = [_doc(str(rng.choice(paths)), str(rng.choice(subs)), list(rng.choice(groups, size=2, replace=False)))
            for _ in range(300)]
    res = P.AuthPipelineBatch(cfg, ctx=OracleCtx()).evaluate(docs)

    def one(doc):
        top = O.Ruleset.from_expression(cfg.conditions).matches(doc)[0]
        if top != 1:
            return "skip", None
        for prio in sorted({c.priority for c in cfgs}):
            for c in [c for c in cfgs if c.priority == prio]:
                if c.conditions is not None and O.Ruleset.from_expression(c.conditions).matches(doc)[0] != 1:
                    continue
                if O.Ruleset.from_expression(c.rules).matches(doc)[0] != 1:
                    return "deny", c.name
        return "allow", None

    for d, r in zip(docs, res):
        kind, by = one(d)
        if kind == "skip":
            assert r.skipped and r.code == P.CODE_OK
        elif kind == "deny":
            assert r.code == P.CODE_PERMISSION_DENIED and r.denied_by == by
        else:
            assert r.code == P.CODE_OK and not r.skipped
