"""Response-header selectors (authorino_amd.response) on CPU.

Vectors follow the reference's own tests: pkg/json/json_test.go (TestJSONValueResolveFor,
TestIsTemplate, TestReplaceJSONPlaceholders, TestStringifyJSON),
pkg/evaluators/response_test.go (TestWrapResponseObjectAsHeader) and
pkg/evaluators/response/{plain,dynamic_json}_test.go. Selector lookups use the oracle
through a stand-in context (the device path is tests/test_gpu_parity.py::test_select_*).
Cases with gjson modifiers (@extract, @case) only check the template split: modifiers are
not compiled for the device. Go number formatting beyond the reference's vectors is
restated from strconv (parity unpinned)."""
import json

import numpy as np
import pytest

import pyoracle as O
from authorino_amd import jsonexp as J
from authorino_amd import pipeline as P
from authorino_amd import response as R
from test_pipeline_host import OracleCtx

# json_test.go:13-30 (the reference's document, trailing comma and all)
DOC = b"""{
		"auth": {
			"identity": {
				"username": "john",
				"email": "john@test",
				"email_verified": true,
				"address": {
					"line_1": "123 Test St",
					"postal_code": 987654
				},
				"roles": [
					"user",
					"admin"
				],
				"exp": 1629884250,
				"github.com": "https://github.com/john",
			}
		}
	}"""


def _sel(paths_values, doc=DOC):
    cfgs = [R.ResponseConfig("r", plain=v) for v in paths_values]
    s = R.ResponseSelectors(cfgs, OracleCtx())
    arena = np.frombuffer(doc, dtype=np.uint8)
    spans = s.resolve([doc], arena, np.zeros(1, np.uint64), np.array([len(doc)], np.uint32))
    return [s.call(c, doc, spans[0]) for c in cfgs]


def test_is_template():
    """json_test.go:75-133"""
    cases = [("Just a static string", False), ("Hello, {auth.identity.username}!", True),
             ("http://talker-api.authorino.svc.cluster.local:3000/metadata?encoding=text/plain&original_path="
              "{context.request.http.path}", True),
             (r"auth.identity.metadata.annotations.authorino\.kuadrant\.io/username", False),
             (r"auth.identity.metadata.annotations.authorino\.kuadrant\.io/username|@case:lower", False),
             ("auth.identity.metadata.creationTimestamp", False),
             ('auth.identity.metadata.name.@replace:{"old":"john","new":"John"}', False),
             ("{auth.identity.metadata.creationTimestamp}", True),
             (r'Hello, {auth.identity.metadata.annotations.authorino\.kuadrant\.io/name|@extract:{"pos":1}}!', True),
             (r'Hello, \{auth.identity.metadata.annotations.authorino\.kuadrant\.io/name|@extract:\{"pos":1}}!', True),
             ('Email domain: {auth.identity.email.@extract:{"sep":"@","pos":1}}', True),
             ('Email username: {auth.identity.email.@extract:{"sep":"@","pos":0}} | Email domain: '
              '{auth.identity.email.@extract:{"sep":"@","pos":1}}', True),
             (r'The JSON path is \{auth.identity.metadata.annotations.name.@replace:\{"old":"john","new":"John"\}\}!',
              True),
             (r"Hello, {auth.identity.metadata.annotations.authorino\.kuadrant\.io/name}!", True),
             ("http://echo-api.3scale.net/login?redirect_to=https://{context.request.http.host}"
              "{context.request.http.path}", True),
             ("Not a valid {template!", True)]
    for pat, want in cases:
        assert R.JSONValue(pattern=pat).is_template() == want, pat


def test_resolve_for():
    """json_test.go:36-73 (modifier cases: split only)"""
    assert _sel([R.JSONValue(static="foo")]) == ["foo"]
    got = _sel([R.JSONValue(pattern="auth.identity.username"), R.JSONValue(pattern="auth.identity.email_verified"),
                R.JSONValue(pattern="auth.identity.address"), R.JSONValue(pattern="auth.identity.roles"),
                R.JSONValue(pattern="Hello, {auth.identity.username}!")])
    assert got[0] == "john" and got[1] is True
    assert got[2] == {"line_1": "123 Test St", "postal_code": 987654.0}
    assert got[3] == ["user", "admin"]
    assert got[4] == "Hello, john!"
    v = R.JSONValue(pattern='Email domain: {auth.identity.email.@extract:{"sep":"@","pos":1}}')
    assert v.paths() == ['auth.identity.email.@extract:{"sep":"@","pos":1}']
    v = R.JSONValue(pattern='auth.identity.email.@extract:{"sep":"@","pos":1}')
    assert not v.is_template() and v.paths() == [v.pattern]


def test_replace_json_placeholders():
    """json_test.go:136-205, through the compile-time split + per-placeholder String()"""
    cases = [("Nothing to replace", "Nothing to replace"), ("Username: {auth.identity.username}", "Username: john"),
             ("Username: {auth.identity.username}, Email: {auth.identity.email}", "Username: john, Email: john@test"),
             ("{auth.identity.email_verified} (bool)", "true (bool)"),
             (r"Github.com: {auth.identity.github\.com}", "Github.com: https://github.com/john"),
             (r"This is NOT a \{variable placeholder\}, {auth.identity.username}!",
              "This is NOT a {variable placeholder}, john!"),
             ("{auth.identity.username}", "john"), (r"\\{auth.identity.username} \\o/", r"\john \o/"),
             (r"\\\{auth.identity.username\}", r"\{auth.identity.username}"),
             ("username: {auth.identity.username", "username: "),
             (r"username: {auth.ide{ntit/y.u\sername}", "username: ")]
    for tpl, want in cases:
        out = []
        for kind, s in R.template_segments(tpl):
            out.append(s if kind == "lit" else O.gjson_get(DOC, s)[2].decode())
        assert "".join(out) == want, tpl
        if R.JSONValue(pattern=tpl).is_template() and "{" in tpl:
            assert _sel([R.JSONValue(pattern=tpl)]) == [want], tpl
    # placeholders with the reference's modifiers (json_test.go:165-169, :180-187): built
    # text from the select path's text slots
    mod_cases = [("Username: {auth.identity.username.@case:upper}", "Username: JOHN"),
                 ('Domain: {auth.identity.email.@extract:{"sep":"@","pos":1}}', "Domain: test"),
                 (r'Github username: {auth.identity.github\.com|@extract:{"sep":"/","pos":3}|@case:upper}',
                  "Github username: JOHN"),
                 (r'\{"msg":"I can build a JSON with dynamic values","username":"{auth.identity.github\.com|'
                  r'@extract:{"sep":"/","pos":3}|@case:upper}"\}',
                  '{"msg":"I can build a JSON with dynamic values","username":"JOHN"}')]
    for tpl, want in mod_cases:
        out = []
        for kind, s in R.template_segments(tpl):
            out.append(s if kind == "lit" else O.gjson_string_mods(DOC, s).decode())
        assert "".join(out) == want, tpl
        assert _sel([R.JSONValue(pattern=tpl)]) == [want], tpl
    segs = R.template_segments(r'\{"msg":"x","username":"{auth.identity.github\.com|@extract:{"sep":"/","pos":3}'
                               r'|@case:upper}"\}')
    assert segs == [("lit", '{"msg":"x","username":"'),
                    ("path", r'auth.identity.github\.com|@extract:{"sep":"/","pos":3}|@case:upper'), ("lit", '"}')]


def test_stringify_json():
    """json_test.go:265-320"""
    assert R.stringify_json("this is a json string") == "this is a json string"
    assert R.stringify_json(123.0) == "123"
    assert R.stringify_json(True) == "true" and R.stringify_json(False) == "false"
    assert R.stringify_json(None) == ""
    assert R.stringify_json({"a_prop": "a_value"}) == '{"a_prop":"a_value"}'
    assert R.stringify_json(["a", "b", "c"]) == '["a","b","c"]'
    src = {"prop_str": "str", "prop_num": 123.0, "prop_bool": False, "prop_null": None,
           "prop_obj": {"a_prop": "a_value"}, "prop_arr": ["a", "b", "c"]}
    assert R.stringify_json(src) == ('{"prop_arr":["a","b","c"],"prop_bool":false,"prop_null":null,"prop_num":123,'
                                     '"prop_obj":{"a_prop":"a_value"},"prop_str":"str"}')


def test_wrap_and_call():
    """response_test.go:13-32, dynamic_json_test.go:15-45, plain_test.go:30-46"""
    c = R.ResponseConfig("resp", json_properties=[], wrapper_key="my-key")
    assert c.wrap_object_as_header_value({"my-prop": "my-value"}) == '{"my-prop":"my-value"}'
    c = R.ResponseConfig("resp", plain=R.JSONValue(), wrapper_key="my-key")
    assert c.wrap_object_as_header_value("my-value") == "my-value"
    doc = b'{"auth":{"identity":{"username":"john"}}}'
    dj = R.ResponseConfig("r", json_properties=[("prop1", R.JSONValue(static="value1")),
                                                ("prop2", R.JSONValue(pattern="auth.identity.username"))])
    s = R.ResponseSelectors([dj], OracleCtx())
    spans = s.resolve([doc], np.frombuffer(doc, np.uint8), np.zeros(1, np.uint64), np.array([len(doc)], np.uint32))
    assert R.go_json_marshal(s.call(dj, doc, spans[0])) == '{"prop1":"value1","prop2":"john"}'
    assert R.go_sprint_v(_sel([R.JSONValue(pattern="auth.identity.username")], doc)[0]) == "john"


def test_go_number_formatting():
    """fmt %v / encoding/json / Result.String() of float64 (strconv; SURVEY.md §8 a14
    example 1.685557675e+09)"""
    v = {1685557675.0: "1.685557675e+09", 123456.0: "123456", 1e6: "1e+06", 0.0001: "0.0001",
         1e-05: "1e-05", 0.5: "0.5", -2.25: "-2.25", 0.0: "0", 1e21: "1e+21", 5e-324: "5e-324",
         1234567.0: "1.234567e+06"}
    for x, want in v.items():
        assert R.go_format_float(x, "g") == want, x
    j = {1e21: "1e+21", 1e20: "100000000000000000000", 1e-7: "1e-7", 1e-6: "0.000001", 123.0: "123",
         0.1: "0.1", -1.5e-10: "-1.5e-10", 1.7976931348623157e308: "1.7976931348623157e+308"}
    for x, want in j.items():
        assert R.go_json_marshal(x) == want, x
    assert R.stringify_json(float("inf")) == ""
    assert R.go_sprint_v({"b": [1.0, "x", None], "a": True}) == "map[a:true b:[1 x <nil>]]"
    assert R.go_json_marshal("<a&b>\u2028\x01\"\\") == '"\\u003ca\\u0026b\\u003e\\u2028\\u0001\\"\\\\"'


def _rand_doc(rng):
    nums = ["0", "-0", "12", "-7", "1.5", "1.50", "1e3", "-2.5E-3", "123456789.125", "1e21", "0.000001",
            "3.14159", "1E+2", "99999999999999999999", "1.0e-7"]
    strs = ["plain", "tab\\tx", "q\\\"q", "uni\\u00e9\\u0041", "pair\\ud83d\\ude00", "lone\\ud800x", "sl\\/sh",
            "bad\\ud800\\u0041", "<&>", "caf\u00e9"]
    d = {}
    for k in range(int(rng.integers(4, 10))):
        r = rng.random()
        if r < 0.35:
            d["n%d" % k] = ("N", str(rng.choice(nums)))
        elif r < 0.7:
            d["s%d" % k] = ("S", str(rng.choice(strs)))
        elif r < 0.8:
            d["b%d" % k] = ("R", str(rng.choice(["true", "false", "null"])))
        elif r < 0.9:
            d["a%d" % k] = ("R", '[1,"x",{"y":2.50},[true,null],-0.5e1]')
        else:
            d["o%d" % k] = ("R", '{"z":"q\\u0041","y":[1,2],"z":3.0e0}')
    body = ",".join('"%s":%s' % (k, '"%s"' % v if t == "S" else v) for k, (t, v) in d.items())
    return ('{"x":{%s},"pad":1}' % body).encode(), ["x." + k for k in d] + ["x.missing", "pad"]


def test_values_and_strings_against_oracle():
    """Result.String() / Value() from spans vs the oracle's gjson restatement, random
    numbers, escapes, surrogates, nested containers, duplicate keys."""
    rng = np.random.default_rng(11)
    for _ in range(300):
        doc, paths = _rand_doc(rng)
        for p in paths:
            t, raw, st = O.gjson_get(doc, p)
            t2, s0, ln = O.gjson_span(doc, p)
            assert t2 == t and doc[s0:s0 + ln] == raw
            assert R.result_string(doc, s0, ln, t).encode("utf-8") == st, (doc, p)
            v = R.result_value(doc, s0, ln, t)
            if t == R.NUMBER:
                assert v == float(raw)
            if t == R.JSON:
                # gjson Value() then json.Marshal: compare with Python's parse of the same raw
                ref = json.loads(raw.decode(), parse_int=float, object_pairs_hook=dict)
                assert R.go_json_marshal(v) == R.go_json_marshal(_fix_surrogates(ref)), (raw,)


def _fix_surrogates(v):
    if isinstance(v, str):
        return R.gjson_unescape(json.dumps(v)[1:-1].encode()).decode("utf-8", "replace")
    if isinstance(v, dict):
        return {_fix_surrogates(k): _fix_surrogates(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_fix_surrogates(x) for x in v]
    return v


def test_pipeline_response_phase_host():
    """Phase 4 after a successful authorization phase: `when`-gated Plain and DynamicJSON
    responses wrapped as headers (auth_pipeline.go:490-494, response.go:150-174)."""
    from test_pipeline_host import _doc

    resp = [R.ResponseConfig("p", plain=R.JSONValue(pattern="auth.identity.sub"), wrapper_key="x-sub"),
            R.ResponseConfig("j", json_properties=[("g", R.JSONValue(pattern="auth.identity.groups")),
                                                   ("s", R.JSONValue(static="k")),
                                                   ("t", R.JSONValue(pattern="{context.request.http.method} {auth.identity.sub}"))],
                             wrapper_key="x-json"),
            R.ResponseConfig("w", plain=R.JSONValue(pattern="auth.identity.groups"), wrapper_key="x-when",
                             conditions=J.All(J.Pattern("auth.identity.sub", J.EqualOperator, "bob")), priority=1),
            R.ResponseConfig("m", plain=R.JSONValue(pattern="auth.identity.sub"),
                             wrapper=R.ENVOY_DYNAMIC_METADATA_WRAPPER, wrapper_key="meta")]
    cfg = P.AuthConfig(authorization=[P.AuthorizationConfig(
        "a", rules=J.All(J.Pattern("auth.identity.groups", J.IncludesOperator, "users")))], response=resp)
    docs = [_doc(sub="alice", groups=("users", "devs")), _doc(sub="bob", groups=("users",)),
            _doc(sub="carol", groups=("admins",))]
    out = P.AuthPipelineBatch(cfg, ctx=OracleCtx()).evaluate(docs)
    assert out[0].headers == {"x-sub": "alice", "x-json": '{"g":["users","devs"],"s":"k","t":"GET alice"}'}
    assert out[0].metadata == {"meta": "alice"}
    assert out[1].headers["x-when"] == "[users]"
    assert out[2].code == P.CODE_PERMISSION_DENIED and out[2].headers == {}


def test_c5_full_phase_host():
    """C5 on CPU through the oracle stand-in: the phase decides both ways and every
    allowed request gets its 4 headers."""
    from authorino_amd import workloads as W

    w = W.make("c5", n=300, seed=51)
    docs = [w.doc(i) for i in range(w.n)]
    out = P.AuthPipelineBatch(w.auth_config, ctx=OracleCtx()).evaluate(docs)
    ok = [r for r in out if r.code == P.CODE_OK and not r.skipped]
    assert 0 < len(ok) < w.n and any(r.skipped for r in out)
    for r in ok:
        assert set(r.headers) == {"x-auth-user", "x-auth-exp", "x-auth-claims", "x-auth-ctx"}
        assert "e+09" in r.headers["x-auth-exp"]
        assert r.headers["x-auth-claims"].startswith('{"acr":0.5,"groups":["reader"')
