"""gjson's own @fromstr and a path after a modifier (`body.@fromstr|request.object.kind`,
the `when` of docs/user-guides/validating-webhook.md:156; the JWT chain of
pkg/json/json_test.go:247-257) on the device's exact path (ajx_modifiers.h, host build)
against the oracle (gjson_mods_ref.c). @fromstr is gjson v1.14.0 modFromStr:
Parse(json).String() of a text that passes Valid, else "". Valid is pinned three ways:
the device's iterative restatement, the oracle's recursive one, and Python's json
module (strict, no NaN/Infinity) on ASCII texts."""
import json
import random
import re

import pytest

import _hosttest as H
import pyoracle as O


def _jwt_doc():
    # an access token shaped as TestParseJWTFromAuthzHeader's (json_test.go:249): the
    # header and claims its comment (:248) decodes to, base64url without padding
    import base64

    hdr = base64.urlsafe_b64encode(b'{"alg":"RS256","kid":"Ruk8dcoOv7kJqmchIJPtks7sHirl27ErFhfOVpBClHE"}').rstrip(b"=")
    claims = (b'{"aud":["https://kubernetes.default.svc.cluster.local"],"exp":1685557675,"iat":1685554075,'
              b'"iss":"https://kubernetes.default.svc.cluster.local","kubernetes.io":{"namespace":"default",'
              b'"serviceaccount":{"name":"default","uid":"1edfd768-d05a-445f-a03a-0a834b45688e"}},'
              b'"nbf":1685554075,"sub":"system:serviceaccount:default:default"}')
    pay = base64.urlsafe_b64encode(claims).rstrip(b"=")
    return b'{"access_token":"Bearer ' + hdr + b"." + pay + b'.c2lnbmF0dXJl"}'


def _python_valid(t: str) -> bool:
    def no_const(x):
        raise ValueError(x)

    try:
        json.loads(t, parse_constant=no_const)
        return True
    except (ValueError, RecursionError):
        return False


def _mutate(rng, s: str) -> str:
    k = rng.randrange(6)
    i = rng.randrange(len(s) + 1)
    if k == 0:
        return s[:i] + s[i + 1:]
    if k == 1:
        return s[:i] + rng.choice(list('{}[]",:0-.eE+ \t\n\\u/tnfx')) + s[i:]
    if k == 2:
        return s[:i]
    if k == 3:
        return s + rng.choice([" ", "x", "}", "\n", ",1"])
    if k == 4:
        return s.replace(":", rng.choice([" :", ": ", "::", ""]), 1)
    return s.replace('"', "'", 1)


def _rand_json(rng, depth=3):
    r = rng.random()
    if depth == 0 or r < 0.4:
        return rng.choice([0, -1, 12.5, -0.0, 1e21, 3e-7, "", "a\"b\\c", "é", "\x01", True, False, None,
                           "x" * rng.randrange(0, 30), 10 ** rng.randrange(0, 25)])
    if r < 0.7:
        return {rng.choice(["a", "b", "k", "request", "kind", ""]): _rand_json(rng, depth - 1)
                for _ in range(rng.randrange(0, 4))}
    return [_rand_json(rng, depth - 1) for _ in range(rng.randrange(0, 4))]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_valid_three_ways(seed):
    rng = random.Random(4100 + seed)
    n_valid = n_invalid = 0
    for _ in range(3000):
        v = _rand_json(rng)
        t = json.dumps(v, separators=rng.choice([(",", ":"), (", ", ": ")]), indent=rng.choice([None, 1]))
        for _ in range(rng.randrange(0, 3)):
            t = _mutate(rng, t)
        want = _python_valid(t)
        assert O.valid(t) == want, t
        assert H.json_valid(t) == int(want), t
        n_valid += want
        n_invalid += not want
    assert n_valid > 1000 and n_invalid > 1000
    for t in ["", " ", "0", "-", "-0", "01", "1.", ".5", "1e", "1e+", "1E-2", "tru", "true ", " null", "nul",
              '"\\u12"', '"\\u12G4"', '"\\x"', '"\t"', "[1,]", "[,1]", "{,}", '{"a" 1}', '{"a":}', "[]]", "{}x",
              "[" * 300 + "]" * 300, "[" * 200 + "]" * 200]:
        want = _python_valid(t)
        assert O.valid(t) == want, t
        got = H.json_valid(t)
        assert got == int(want) or (got == -1 and t.startswith("[" * 257)), t


def _fromstr_doc(rng):
    inner = _rand_json(rng, 3)
    if not isinstance(inner, dict):
        inner = {"request": inner}
    if rng.random() < 0.5:
        inner["request"] = {"object": {"metadata": {"namespace": rng.choice(["authorino", "default", "é"])}},
                            "kind": {"kind": "AdmissionReview"}}
    text = json.dumps(inner, separators=(",", ":"), ensure_ascii=rng.random() < 0.5)
    r = rng.random()
    if r < 0.2:
        text = _mutate(rng, text)
    elif r < 0.3:
        text = rng.choice(["12", "true", "null", '"str"', "[1,2]", "", "  {}  "])
    body = json.dumps(text, ensure_ascii=rng.random() < 0.5)
    return ('{"context":{"request":{"http":{"body":%s,"n":5,"o":{"k":"v"}}}}}' % body).encode()


PATHS = ["context.request.http.body.@fromstr",
         "context.request.http.body.@fromstr|request.object.metadata.namespace",
         "context.request.http.body|@fromstr.request.kind",
         "context.request.http.body.@fromstr|request.kind.kind",
         "context.request.http.body.@fromstr|request.object.metadata.namespace|@case:upper",
         "context.request.http.body.@fromstr|a|@fromstr",
         "context.request.http.body.@fromstr|request.object|@case:lower",
         "context.request.http.n.@fromstr",
         "context.request.http.o.@fromstr",
         "context.request.http.o.@fromstr|k",
         "context.request.http.missing.@fromstr|k",
         "context.request.http.body.@base64:encode|@base64:decode|@fromstr|request.kind"]


@pytest.mark.parametrize("seed", [0, 1])
def test_fromstr_and_tails_match_oracle(seed):
    """Pattern results (eq against the oracle's String() must be T; a different value F)
    and selected values (type + raw) on AdmissionReview-shaped bodies, truncated /
    malformed / scalar bodies, non-string inputs, missing keys."""
    rng = random.Random(4200 + seed)
    hrs = {}
    checked = 0
    for _ in range(400):
        d = _fromstr_doc(rng)
        for p in PATHS:
            want = O.gjson_get_mods(d, p)
            want_s = O.gjson_string_mods(d, p)
            if want is None:
                continue
            if p not in hrs:
                hrs[p] = H.HostRuleset([(p, 1, "")], [(0, -1, -1, 0)], 0)
                assert hrs[p].status == [0], p
            rc, out, _ = hrs[p].select_value(0, d, text := bytearray(8192), 0)
            assert rc == 0, ("undecided", d, p)  # (no reason to leave one undecided here)
            st, ln, tt = out
            src = bytes(text) if (tt >> 8) & 4 else d
            assert (tt & 0xFF, src[st:st + ln]) == want, (d, p)
            hr = H.HostRuleset([(p, 1, want_s), (p, 1, want_s + b"?")],
                               [(0, -1, -1, 0), (0, -1, -1, 1), (1, 0, 1, -1)], 2)
            _, _, res = hr.eval(d)
            assert res == [1, 0], (d, p, want_s)
            checked += 1
    assert checked > 2500, checked


def test_reference_jwt_chain():
    """json_test.go:247-257: ...|@base64:decode|@fromstr is JSON, |@fromstr.exp the Number."""
    d = _jwt_doc()
    base = 'access_token.@extract:{"pos":1}|@extract:{"sep":".","pos":1}|@base64:decode|@fromstr'
    for path, t, raw in [(base, 5, None), (base + ".exp", 2, b"1685557675"),
                         (base + r"|kubernetes\.io.namespace", 3, b'"default"')]:
        assert O.gjson_get_mods(d, path)[0] == t
        hr = H.HostRuleset([(path, 1, "")], [(0, -1, -1, 0)], 0)
        rc, out, _ = hr.select_value(0, d, text := bytearray(4096), 0)
        assert rc == 0 and out[2] & 0xFF == t
        got = bytes(text[out[0]:out[0] + out[1]])
        assert got == O.gjson_get_mods(d, path)[1]
        if raw is not None:
            assert got == raw
    hr = H.HostRuleset([(base + ".exp", 1, "1685557675")], [(0, -1, -1, 0)], 0)
    assert hr.eval(d)[2] == [1]


def test_webhook_when_condition():
    """validating-webhook.md:156: `context.request.http.body.@fromstr|request.object.metadata.namespace`
    neq authorino."""
    sel = "context.request.http.body.@fromstr|request.object.metadata.namespace"
    hr = H.HostRuleset([(sel, 2, "authorino")], [(0, -1, -1, 0)], 0)
    for ns, want in [("authorino", 0), ("default", 1)]:
        review = {"kind": "AdmissionReview", "request": {"object": {"metadata": {"namespace": ns}}}}
        d = ('{"context":{"request":{"http":{"body":%s}}}}' % json.dumps(json.dumps(review))).encode()
        assert hr.eval(d)[0] == want
        assert re.search(ns, O.gjson_string_mods(d, sel).decode())
