"""denyWith (customizeDenyWith, pkg/service/auth_pipeline.go:581-608) and the evaluator
cache (pkg/evaluators/cache.go, authorization.go:56-76) of the batched pipeline on CPU,
with the oracle stand-in for the device (tests/test_gpu_parity.py::test_denywith_and_cache_on_device
runs the same configuration through the kernels)."""
import json

import numpy as np

from authorino_amd import cache as CA
from authorino_amd import jsonexp as J
from authorino_amd import pipeline as P
from authorino_amd.response import JSONValue
from test_pipeline_host import OracleCtx


def _req(host="my-api", path="/operation", sub="alice", tenant="acme", roles=("user",)):
    d = {"context": {"request": {"http": {"host": host, "method": "GET", "path": path}}},
         "auth": {"authorization": {}, "identity": {"sub": sub, "tenant": tenant, "roles": list(roles), "level": 3},
                  "metadata": {}, "response": {}}}
    return json.dumps(d, separators=(",", ":")).encode()


def _deny_all():
    return P.AuthorizationConfig("deny", rules=J.All(J.Pattern("auth.identity.sub", J.EqualOperator, "nobody")))


def test_custom_deny_options_kat():
    """auth_pipeline_test.go:326-362 (TestEvaluateWithCustomDenyOptions): code 302, a
    static and a templated header, a static body; the headers marshal to the test's bytes.
    Here through Unauthorized, which customizeDenyWith treats the same way (:478-481)."""
    dw = P.DenyWithValues(
        code=302,
        headers=[("X-Static-Header", JSONValue(static="some-value")),
                 ("Location", JSONValue(pattern="https://my-app.io/login?redirect_to=https://"
                                                "{context.request.http.host}{context.request.http.path}"))],
        body=JSONValue(static="testing"))
    cfg = P.AuthConfig(authorization=[_deny_all()], unauthorized=dw)
    (r,) = P.AuthPipelineBatch(cfg, ctx=OracleCtx()).evaluate([_req()])
    assert r.code == P.CODE_PERMISSION_DENIED and r.status == 302
    assert r.message == "Unauthorized" and r.body == "testing"
    assert json.dumps(r.deny_headers, separators=(",", ":")) == \
        '[{"X-Static-Header":"some-value"},{"Location":"https://my-app.io/login?redirect_to=https://my-api/operation"}]'


def test_deny_with_selectors_and_stringify():
    """message / body from selectors: StringifyJSON of ResolveFor (json.go:41-53, :153-159):
    strings unquoted, numbers in Go form, arrays/objects as JSON, a missing path -> ""."""
    dw = P.DenyWithValues(
        message=JSONValue(pattern="auth.identity.sub"),
        body=JSONValue(pattern="auth.identity.roles"),
        headers=[("X-Level", JSONValue(pattern="auth.identity.level")),
                 ("X-Missing", JSONValue(pattern="auth.identity.nope")),
                 ("X-Who", JSONValue(pattern="{auth.identity.sub}@{auth.identity.tenant}"))])
    cfg = P.AuthConfig(authorization=[_deny_all()], unauthorized=dw)
    docs = [_req(sub="bob", roles=("a", "b")), _req(sub="carol", tenant="zeta", roles=())]
    res = P.AuthPipelineBatch(cfg, ctx=OracleCtx()).evaluate(docs)
    assert res[0].message == "bob" and res[0].body == '["a","b"]' and res[0].status == 0
    assert res[0].deny_headers == [{"X-Level": "3"}, {"X-Missing": ""}, {"X-Who": "bob@acme"}]
    assert res[1].message == "carol" and res[1].body == "[]"
    assert res[1].deny_headers[2] == {"X-Who": "carol@zeta"}


def test_modifier_value_selectors_resolve_to_built_text():
    """denyWith / cache-key selectors with the reference's modifiers and "#." lists
    (json.go:96-151, :161-264): their values are the modifier chain's Result (built text
    in the request's select text slot, AUTHJX_VALUE_TEXT), never the unmodified value; a
    value the oracle stand-in cannot build (@case on non-ASCII text: it restates ASCII only)
    leaves that request undecided (the device decides it: tests/test_gpu_select_text.py)."""
    dw = P.DenyWithValues(message=JSONValue(pattern="auth.identity.tenant.@case:upper"),
                          body=JSONValue(pattern='{auth.identity.sub|@extract:{"sep":"i","pos":0}}-{auth.identity.roles.#.x}'),
                          headers=[("X-Roles", JSONValue(pattern="auth.identity.roles|@case:upper"))])
    cfg = P.AuthConfig(authorization=[_deny_all()], unauthorized=dw)
    # (non-ASCII under @case: the oracle stand-in leaves it undecided)
    raw_tenant = _req(sub="bob", tenant="zeta").replace(b'"zeta"', '"straße"'.encode())
    res = P.AuthPipelineBatch(cfg, ctx=OracleCtx()).evaluate([_req(), raw_tenant])
    r = res[0]
    assert not r.undecided and r.code == P.CODE_PERMISSION_DENIED
    assert r.message == "ACME" and r.body == "al-[]"
    assert r.deny_headers == [{"X-Roles": '["USER"]'}]
    assert res[1].undecided and res[1].code == P.CODE_UNKNOWN  # (the oracle: ASCII only)
    # a cache key through a modifier: requests with the same key after @case:lower share
    # the cached decision (authorization.go:59-74)
    cached = P.AuthorizationConfig(
        "c", rules=J.All(J.Pattern("auth.identity.sub", J.EqualOperator, "alice")),
        cache=CA.EvaluatorCache(JSONValue(pattern="{auth.identity.tenant|@case:lower}/{auth.identity.sub}"), 60))
    b = P.AuthPipelineBatch(P.AuthConfig(authorization=[cached]), ctx=OracleCtx())
    first = b.evaluate([_req(tenant="ACME")])
    assert first[0].code == P.CODE_OK and not first[0].undecided
    assert cached.cache.get("acme/alice") is True


def test_deny_with_only_on_denied_requests():
    ok = P.AuthorizationConfig("ok", rules=J.All(J.Pattern("auth.identity.sub", J.EqualOperator, "alice")))
    cfg = P.AuthConfig(authorization=[ok], unauthorized=P.DenyWithValues(code=403, message=JSONValue(static="nope")))
    res = P.AuthPipelineBatch(cfg, ctx=OracleCtx()).evaluate([_req(sub="alice"), _req(sub="bob")])
    assert (res[0].code, res[0].status, res[0].message) == (P.CODE_OK, 0, "")
    assert (res[1].code, res[1].status, res[1].message) == (P.CODE_PERMISSION_DENIED, 403, "nope")


class _Clock:
    def __init__(self, t=1000.0):
        self.t = t

    def __call__(self):
        return self.t


def test_evaluator_cache_ttl():
    """metadata_test.go:61-86: a static key, 2 s TTL; within the TTL the cached object is
    returned, after it expires the evaluator runs again."""
    clk = _Clock()
    c = CA.EvaluatorCache(JSONValue(static="x"), 2, clock=clk)
    assert not CA.is_hit(c.get("x"))
    assert c.set("x", {"foo": "bar"})
    assert c.get("x") == {"foo": "bar"}
    clk.t += 1.5
    assert c.get("x") == {"foo": "bar"}
    clk.t += 5
    assert not CA.is_hit(c.get("x"))
    # ttl 0: freecache keeps the entry without expiry, GetWithTTL reports 0 -> never a hit
    z = CA.EvaluatorCache(JSONValue(static="x"), 0, clock=clk)
    z.set("x", True)
    assert not CA.is_hit(z.get("x"))
    # nil key: neither Get nor Set; non-string keys by (type, %v)
    assert not c.set(None, True) and not CA.is_hit(c.get(None))
    c.set(3.0, True)
    assert CA.is_hit(c.get(3.0)) and not CA.is_hit(c.get("3"))
    c.set(["a", 1.0], True)
    assert CA.is_hit(c.get(["a", 1.0]))


def test_cached_authorization_grants_without_rules():
    """authorization.go:56-76 in a batch: the first request of a tenant that passes stores
    `true` under the resolved key; later requests of that tenant (same batch, later in
    order, or a later batch) are granted from the cache even where the rules would deny;
    a denial is never stored; after the TTL the rules run again."""
    clk = _Clock()
    rules = J.All(J.Pattern("auth.identity.sub", J.EqualOperator, "alice"))
    cached = P.AuthorizationConfig("tenant-gate", rules=rules,
                                   cache=CA.EvaluatorCache(JSONValue(pattern="auth.identity.tenant"), 60, clock=clk))
    cfg = P.AuthConfig(authorization=[cached])
    batch = P.AuthPipelineBatch(cfg, ctx=OracleCtx())
    docs = [_req(sub="bob", tenant="acme"), _req(sub="alice", tenant="acme"), _req(sub="bob", tenant="acme"),
            _req(sub="bob", tenant="zeta")]
    res = batch.evaluate(docs)
    assert [r.code for r in res] == [P.CODE_PERMISSION_DENIED, P.CODE_OK, P.CODE_OK, P.CODE_PERMISSION_DENIED]
    assert res[2].authorization == {"tenant-gate": True}
    assert len(cached.cache) == 1  # only acme (a success) is stored
    res = batch.evaluate([_req(sub="bob", tenant="acme")])
    assert res[0].code == P.CODE_OK
    clk.t += 61
    res = batch.evaluate([_req(sub="bob", tenant="acme")])
    assert res[0].code == P.CODE_PERMISSION_DENIED


def test_cache_respects_conditions_and_missing_keys():
    """The evaluator-level `when` runs before Call (auth_pipeline.go:120-125), so a cached
    key never grants a request the conditions exclude; a key path that is missing resolves
    to nil and disables caching for that request."""
    clk = _Clock()
    rules = J.All(J.Pattern("auth.identity.sub", J.EqualOperator, "alice"))
    cond = J.All(J.Pattern("context.request.http.path", J.EqualOperator, "/operation"))
    c = P.AuthorizationConfig("g", rules=rules, conditions=cond,
                              cache=CA.EvaluatorCache(JSONValue(pattern="auth.identity.nope"), 60, clock=clk))
    d = P.AuthorizationConfig("t", rules=rules,
                              cache=CA.EvaluatorCache(JSONValue(pattern="auth.identity.tenant"), 60, clock=clk),
                              priority=1)
    cfg = P.AuthConfig(authorization=[c, d])
    res = P.AuthPipelineBatch(cfg, ctx=OracleCtx()).evaluate(
        [_req(sub="alice"), _req(sub="bob"), _req(sub="bob", path="/x", tenant="acme")])
    assert len(c.cache) == 0  # nil key
    assert res[0].code == P.CODE_OK
    assert res[1].code == P.CODE_PERMISSION_DENIED and res[1].denied_by == "g"
    # request 2 skips g (conditions) and is granted t from acme's entry stored by request 0
    assert res[2].code == P.CODE_OK and res[2].authorization == {"t": True}


def test_batched_cache_equals_serial_requests():
    """Randomised: a batch gives what serving the same requests one at a time gives."""
    rng = np.random.default_rng(5)
    tenants, subs = ["a", "b", "c", "d"], ["alice", "bob", "carol"]

    def cfg_and_cache():
        clk = _Clock()
        rules = J.Any(J.Pattern("auth.identity.sub", J.EqualOperator, "alice"),
                      J.Pattern("auth.identity.roles", J.IncludesOperator, "admin"))
        cc = P.AuthorizationConfig("x", rules=rules,
                                   cache=CA.EvaluatorCache(JSONValue(pattern="{auth.identity.tenant}/{context.request.http.path}"),
                                                           30, clock=clk))
        return P.AuthConfig(authorization=[cc], unauthorized=P.DenyWithValues(message=JSONValue(pattern="auth.identity.tenant")))

    docs = [_req(path=str(rng.choice(["/p", "/q"])), sub=str(rng.choice(subs)), tenant=str(rng.choice(tenants)),
                 roles=list(rng.choice(["admin", "user"], size=1))) for _ in range(200)]
    batched = P.AuthPipelineBatch(cfg_and_cache(), ctx=OracleCtx()).evaluate(docs)
    one = P.AuthPipelineBatch(cfg_and_cache(), ctx=OracleCtx())
    serial = [one.evaluate([d])[0] for d in docs]
    for b, s in zip(batched, serial):
        assert (b.code, b.message, b.authorization) == (s.code, s.message, s.authorization)
    assert any(b.code == P.CODE_OK for b in batched) and any(b.code != P.CODE_OK for b in batched)


def test_later_reads_of_granted_objects_need_a_producer():
    """A cache key at a later priority, or denyWith over more than one priority, that reads
    auth.authorization.* resolves on the JSON with the earlier priorities' grants
    (authorization.go:56-66, auth_pipeline.go:581-608): the batch rebuilds the documents
    through the producer, and refuses to run without one (no key collides on a missing
    grant)."""
    import pytest

    allow = J.All(J.Pattern("auth.identity.sub", J.EqualOperator, "alice"))
    first = P.AuthorizationConfig("first", rules=allow, priority=0)
    keyed = P.AuthorizationConfig("second", rules=allow, priority=1,
                                  cache=CA.EvaluatorCache(JSONValue(pattern="auth.authorization.first"), ttl=60))
    cfg = P.AuthConfig(authorization=[first, keyed])
    with pytest.raises(ValueError):
        P.AuthPipelineBatch(cfg, ctx=OracleCtx()).evaluate([_req()])
    # the same key at the first priority reads nothing granted yet: no producer needed
    keyed0 = P.AuthorizationConfig("second", rules=allow, priority=0,
                                   cache=CA.EvaluatorCache(JSONValue(pattern="auth.authorization.first"), ttl=60))
    (r,) = P.AuthPipelineBatch(P.AuthConfig(authorization=[first, keyed0]), ctx=OracleCtx()).evaluate([_req()])
    assert r.code != P.CODE_PERMISSION_DENIED
    dw = P.DenyWithValues(message=JSONValue(pattern="auth.authorization.first"))
    cfg = P.AuthConfig(authorization=[first, P.AuthorizationConfig("deny", rules=_deny_all().rules, priority=1)],
                       unauthorized=dw)
    with pytest.raises(ValueError):
        P.AuthPipelineBatch(cfg, ctx=OracleCtx()).evaluate([_req()])

    def producer(i, granted):
        d = json.loads(_req())
        d["auth"]["authorization"] = granted
        return json.dumps(d, separators=(",", ":")).encode()

    (r,) = P.AuthPipelineBatch(cfg, ctx=OracleCtx()).evaluate([_req()], producer=producer)
    assert r.code == P.CODE_PERMISSION_DENIED and r.message == "true"
