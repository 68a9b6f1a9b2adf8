"""The Authorization JSON producer's packing stage (authorino_amd/producer.py ->
libauthjx.so authjx_pack_json) against the reference's byte-format test
(pkg/service/auth_pipeline_test.go:583-596, TestNewAuthorizationJSON) and against the
encoding/json restatement the response selectors use (authorino_amd.response
go_json_marshal), on random values: Go map key order, HTML-safe escapes, U+2028/U+2029,
invalid UTF-8, float64 'f'/'e' layouts."""
import math

import numpy as np
import pytest

from authorino_amd import producer as P
from authorino_amd import response as R

EXPECTED = ('{"context":{"request":{"http":{"method":"GET","headers":{"authorization":"Bearer n3ex87bye9238ry8"},'
            '"path":"/operation","host":"my-api"}}},"request":{"host":"my-api","method":"GET","path":"/operation",'
            '"url_path":"/operation","headers":{"authorization":"Bearer n3ex87bye9238ry8"}},"source":{},'
            '"destination":{},"auth":{"identity":"leeloo","authorization":{"credential":"multipass"}}}')


def _docs(values, **kw):
    arena, offs, lens = P.pack(values, **kw)
    return [bytes(arena[int(o):int(o) + int(n)]).decode("utf-8") for o, n in zip(offs, lens)]


def test_reference_authorization_json_bytes():
    headers = P.go_map({"authorization": "Bearer n3ex87bye9238ry8"})
    doc = P.authorization_json(
        context={"request": {"http": {"method": "GET", "headers": headers, "path": "/operation", "host": "my-api"}}},
        request={"host": "my-api", "method": "GET", "path": "/operation", "url_path": "/operation",
                 "headers": headers},
        identity="leeloo", metadata={}, authorization={"credential": "multipass"}, response={})
    assert _docs([doc]) == [EXPECTED]


@pytest.mark.parametrize("f,want", [
    (0.5, "0.5"), (100.0, "100"), (1e20, "100000000000000000000"), (1e21, "1e+21"), (1e-7, "1e-7"),
    (1.5e-6, "0.0000015"), (1e-6, "0.000001"), (0.1 + 0.2, "0.30000000000000004"), (5e-324, "5e-324"),
    (-0.0, "-0"), (1.7976931348623157e308, "1.7976931348623157e+308"), (123456789.0, "123456789"),
    (-2.5e-10, "-2.5e-10"), (37.77492950000001, "37.77492950000001"), (1.2345e21, "1.2345e+21"),
])
def test_float64_layouts(f, want):
    assert _docs([[f]]) == ["[" + want + "]"]
    assert R.go_json_marshal(f) == want


def test_strings_ints_and_raw():
    vals = [["<a&b>  \x01\"\\\n\t", b"\xff\xfeok\xe2\x82", 2 ** 62, -7, True, None, P.RawJSON(b'{"x":1}')]]
    assert _docs(vals) == ['["\\u003ca\\u0026b\\u003e\\u2028\\u2029\\u0001\\"\\\\\\n\\t","\\ufffd\\ufffdok\\ufffd\\ufffd",'
                           '4611686018427387904,-7,true,null,{"x":1}]']


def test_nan_and_inf_fail_like_marshal():
    for bad in (math.nan, math.inf, -math.inf):
        with pytest.raises(P.PackError):
            P.pack([{"a": [1.0, bad]}])


def _rand_value(rng, depth):
    r = rng.random()
    if depth == 0 or r < 0.5:
        k = int(rng.integers(0, 6))
        if k == 0:
            return "".join(chr(int(c)) for c in rng.choice([0x41, 0x3C, 0x26, 0x22, 0x5C, 0x0A, 0x01, 0xE9, 0x2028,
                                                             0x1F600, 0x7F, 0x3E], size=int(rng.integers(0, 8))))
        if k == 1:
            return float(rng.choice([0.0, 1.0, -3.25, 1e21, 9.99e20, 1e-6, 9e-7, 1e300, 2.5e-308, 0.1]))
        if k == 2:
            return float(np.frombuffer(rng.bytes(8), dtype=np.float64)[0]) if rng.random() < 0.5 else float(rng.normal() * 10.0 ** int(rng.integers(-12, 25)))
        if k == 3:
            return bool(rng.integers(0, 2))
        if k == 4:
            return None
        return "k%d" % rng.integers(0, 100)
    if r < 0.75:
        return P.GoMap({"".join(rng.choice(list("abz<&é_"), size=int(rng.integers(0, 4)))): _rand_value(rng, depth - 1)
                        for _ in range(int(rng.integers(0, 5)))})
    return [_rand_value(rng, depth - 1) for _ in range(int(rng.integers(0, 5)))]


def _finite(v):
    if isinstance(v, float):
        return math.isfinite(v)
    if isinstance(v, dict):
        return all(_finite(x) for x in v.values())
    if isinstance(v, list):
        return all(_finite(x) for x in v)
    return True


def test_random_values_match_encoding_json_restatement():
    rng = np.random.default_rng(61)
    vals = [v for v in (_rand_value(rng, 4) for _ in range(3000)) if _finite(v)]
    for nt in (1, 4):
        got = _docs(vals, n_threads=nt)
        assert got == [R.go_json_marshal(v) for v in vals]
