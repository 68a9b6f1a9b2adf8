"""The synthetic Authorization JSON producer (authorino_amd.workloads) against the
reference's byte-format test: go_json / go_map with Go struct field order and Go map key
order reproduce NewAuthorizationJSON's output byte for byte
(pkg/service/auth_pipeline_test.go:583-596, TestNewAuthorizationJSON)."""
from authorino_amd import workloads as W

# auth_pipeline_test.go:593
EXPECTED = ('{"context":{"request":{"http":{"method":"GET","headers":{"authorization":"Bearer n3ex87bye9238ry8"},'
            '"path":"/operation","host":"my-api"}}},"request":{"host":"my-api","method":"GET","path":"/operation",'
            '"url_path":"/operation","headers":{"authorization":"Bearer n3ex87bye9238ry8"}},"source":{},'
            '"destination":{},"auth":{"identity":"leeloo","authorization":{"credential":"multipass"}}}')


def test_go_json_matches_reference_authorization_json():
    headers = W.go_map({"authorization": "Bearer n3ex87bye9238ry8"})
    doc = {
        # envoy CheckRequest attributes (struct order, omitempty)
        "context": {"request": {"http": {"method": "GET", "headers": headers, "path": "/operation", "host": "my-api"}}},
        # well-known attributes (well_known_attributes.go struct order, omitempty)
        "request": {"host": "my-api", "method": "GET", "path": "/operation", "url_path": "/operation",
                    "headers": headers},
        "source": {},
        "destination": {},
        # auth: identity, then authorization (struct order); map values sorted by key
        "auth": {"identity": "leeloo", "authorization": W.go_map({"credential": "multipass"})},
    }
    assert W.go_json(doc) == EXPECTED


def test_go_json_escapes_like_encoding_json():
    # HTML-safe escapes and U+2028 / U+2029, as encoding/json writes them
    assert W.go_json({"a": "<&>\u2028\u2029"}) == '{"a":"\\u003c\\u0026\\u003e\\u2028\\u2029"}'
    assert W.go_json(W.go_map({"b": 1, "a": [True, None, 0.5]})) == '{"a":[true,null,0.5],"b":1}'
