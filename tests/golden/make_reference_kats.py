"""Writes tests/golden/reference_kats.json: the known-answer vectors the reference's own
tests hold for this hot path, transcribed as data (inputs and expected outputs only).

Sources (paths relative to the reference tree):
  pkg/jsonexp/expressions_test.go:9-15      fixture document `testJsonData`
  pkg/jsonexp/expressions_test.go:17-551    And/Or/All/Any truth tables, empty nodes
  pkg/evaluators/authorization/json_test.go:19-41   document built by encoding/json from
      an Envoy AttributeContext (headers x-secret-header, x-origin) + auth data
  pkg/evaluators/authorization/json_test.go:52-272  eq/neq/incl/excl/matches/invalid
      regex/multi-rule/empty cases with expected (authorized, error)
  pkg/evaluators/authorization/json_test.go:275-303 benchmark doc + rules
  pkg/service/auth_pipeline_test.go:389-495 `when` conditions on path "/operation"
  pkg/service/auth_pipeline_test.go:583-596 Authorization JSON of NewAuthorizationJSON
  pkg/json/json_test.go:174-181             bool stringification, escaped-dot key
  pkg/json/json_test.go:165-187,207-263     the custom gjson modifiers (@extract @replace
      @case @base64 @strip, chains through '|'): each gjson.Get(..).String() expectation
      becomes an eq pattern that must be T (and a wrong value that must be F)
  tests/v1beta2/authconfig.yaml:9-17,131-150  e2e patterns (matches ^/admin(/.*)?$, eq 'true')

The Go encoding/json output for the AttributeContext document is reproduced by hand:
protobuf-generated structs with `omitempty` tags drop every nil/zero field, maps are
written with sorted keys.

Each case: {"doc": str, "tree": nested expression, "expect": "T"|"F"|"E", "source": str,
            "error_contains": optional str}
Tree encoding: ["pattern", selector, op, value] | ["and", l, r] | ["or", l, r] |
               ["all", [...]] | ["any", [...]] | null (nil)
Run:  python tests/golden/make_reference_kats.py
"""
import json
import os

EXPR_DOC = '''{
\t"str": "my-value",
\t"int": 123,
\t"bool": true,
\t"obj": {"my-obj-str": "my-obj-value"},
\t"arr": ["my-arr-value-1", "my-arr-value-2"]
}'''

AUTHZ_DOC = ('{"context":{"request":{"http":{"headers":{"x-origin":"some-origin",'
             '"x-secret-header":"no-one-knows"}}}},"auth":{"identity":"some-user-data",'
             '"metadata":{"letters":["a","b","c"]}}}')

BENCH_DOC = '{"context":{"request":{"http":{"method":"GET","path":"/allow"}}},"auth":{"identity":{"anonymous":true}}}'

PIPELINE_DOC = ('{"context":{"request":{"http":{"method":"GET","headers":{"authorization":"Bearer n3ex87bye9238ry8"},'
                '"path":"/operation","host":"my-api"}}},"request":{"host":"my-api","method":"GET","path":"/operation",'
                '"url_path":"/operation","headers":{"authorization":"Bearer n3ex87bye9238ry8"}},"source":{},'
                '"destination":{},"auth":{"identity":"leeloo","authorization":{"credential":"multipass"}}}')

JSON_TEST_DOC = ('{"auth":{"identity":{"username":"john","email":"john@test","email_verified":true,'
                 '"github.com":"https://github.com/john"}}}')


def P(sel, op, val):
    return ["pattern", sel, op, val]


T_STR = P("str", "eq", "my-value")
T_INT = P("int", "eq", "123")
F_STR = P("str", "eq", "wrong-value")
F_INT = P("int", "eq", "wrong-value")

cases = []


def add(doc, tree, expect, source, **kw):
    c = {"doc": doc, "tree": tree, "expect": expect, "source": source}
    c.update(kw)
    cases.append(c)


src = "pkg/jsonexp/expressions_test.go"
# TestAnd :17-88
add(EXPR_DOC, ["and", T_STR, T_INT], "T", src + ":19-34")
add(EXPR_DOC, ["and", F_STR, T_INT], "F", src + ":36-51")
add(EXPR_DOC, ["and", T_STR, F_INT], "F", src + ":53-68")
add(EXPR_DOC, ["and", F_STR, F_INT], "F", src + ":70-85")
# TestOneBranchAnd :89-134
add(EXPR_DOC, ["and", T_STR, None], "T", src + ":91-99")
add(EXPR_DOC, ["and", None, T_STR], "T", src + ":101-110")
add(EXPR_DOC, ["and", F_STR, None], "F", src + ":112-121")
add(EXPR_DOC, ["and", None, F_STR], "F", src + ":123-132")
# TestEmptyAnd :136-142
add(EXPR_DOC, ["and", None, None], "T", src + ":136-142")
# TestOr :144-215
add(EXPR_DOC, ["or", T_STR, T_INT], "T", src + ":146-161")
add(EXPR_DOC, ["or", F_STR, T_INT], "T", src + ":163-178")
add(EXPR_DOC, ["or", T_STR, F_INT], "T", src + ":180-195")
add(EXPR_DOC, ["or", F_STR, F_INT], "F", src + ":197-212")
# TestOneBranchOr :216-261
add(EXPR_DOC, ["or", T_STR, None], "T", src + ":218-226")
add(EXPR_DOC, ["or", None, T_STR], "T", src + ":228-237")
add(EXPR_DOC, ["or", F_STR, None], "F", src + ":239-248")
add(EXPR_DOC, ["or", None, F_STR], "F", src + ":250-259")
# TestEmptyOr :263-269
add(EXPR_DOC, ["or", None, None], "F", src + ":263-269")
# TestAll / TestTrivialAll / TestEmptyAll :271-333
add(EXPR_DOC, ["all", [T_STR, T_INT]], "T", src + ":271-285")
add(EXPR_DOC, ["all", [T_STR, F_INT]], "F", src + ":287-300")
add(EXPR_DOC, ["all", [T_STR]], "T", src + ":303-311")
add(EXPR_DOC, ["all", [F_STR]], "F", src + ":313-321")
add(EXPR_DOC, ["all", []], "T", src + ":329-333")
# TestAny / TestTrivialAny / TestEmptyAny :335-397
add(EXPR_DOC, ["any", [T_STR, T_INT]], "T", src + ":335-349")
add(EXPR_DOC, ["any", [T_STR, F_INT]], "T", src + ":351-364")
add(EXPR_DOC, ["any", [T_STR]], "T", src + ":367-375")
add(EXPR_DOC, ["all", [F_STR]], "F", src + ":377-385")
add(EXPR_DOC, ["any", []], "F", src + ":393-397")
# TestAndOr :399-460 (and the nested variants up to :551 follow the same tables)
add(EXPR_DOC, ["all", [["any", [T_STR, F_INT]], ["any", [F_STR, T_INT]]]], "T", src + ":399-428")
add(EXPR_DOC, ["all", [["any", [F_STR, F_INT]], ["any", [F_STR, T_INT]]]], "F", src + ":430-459")
add(EXPR_DOC, ["any", [["all", [T_STR, F_INT]], ["all", [F_STR, T_INT]]]], "F", src + ":461-492 (TestOrAnd)")
add(EXPR_DOC, ["any", [["all", [F_STR, F_INT]], ["all", [F_STR, T_INT]]]], "F", src + ":493-520 (TestOrAnd)")
add(EXPR_DOC, ["any", [["all", [T_STR, T_INT]], ["all", [F_STR, T_INT]]]], "T", src + ":521-550 (TestOrAnd)")
# object / array values stringify to their raw JSON; integer -> "123"
add(EXPR_DOC, P("obj.my-obj-str", "eq", "my-obj-value"), "T", src + ":9-15 fixture (nested key)")
add(EXPR_DOC, P("arr", "incl", "my-arr-value-2"), "T", src + ":9-15 fixture (array)")
add(EXPR_DOC, P("bool", "eq", "true"), "T", src + ":9-15 fixture (bool)")

src = "pkg/evaluators/authorization/json_test.go"
H = "context.request.http.headers.x-secret-header"
L = "auth.metadata.letters"
add(AUTHZ_DOC, ["all", [P(H, "eq", "no-one-knows")]], "T", src + ":52-62")
add(AUTHZ_DOC, ["all", [P(H, "eq", "other-expected")]], "F", src + ":64-75", error_contains="Unauthorized")
add(AUTHZ_DOC, ["all", [P(H, "neq", "other-expected")]], "T", src + ":77-88")
add(AUTHZ_DOC, ["all", [P(H, "neq", "no-one-knows")]], "F", src + ":90-101", error_contains="Unauthorized")
add(AUTHZ_DOC, ["all", [P(L, "incl", "a")]], "T", src + ":103-114")
add(AUTHZ_DOC, ["all", [P(L, "incl", "d")]], "F", src + ":116-127", error_contains="Unauthorized")
add(AUTHZ_DOC, ["all", [P(L, "excl", "d")]], "T", src + ":129-140")
add(AUTHZ_DOC, ["all", [P(L, "excl", "b")]], "F", src + ":142-153", error_contains="Unauthorized")
add(AUTHZ_DOC, ["all", [P(H, "matches", "(.+)-knows")]], "T", src + ":155-166")
add(AUTHZ_DOC, ["all", [P(H, "matches", "(\\d)+")]], "F", src + ":168-179", error_contains="Unauthorized")
add(AUTHZ_DOC, ["all", [P(H, "matches", "$$^[not-a-regex")]], "E", src + ":181-192",
    error_contains="error parsing regexp")
add(AUTHZ_DOC, ["all", [P(H, "eq", "no-one-knows"), P(H, "neq", "other-expected"), P(L, "incl", "a"),
                        P(L, "incl", "c"), P(L, "excl", "d")]], "T", src + ":194-230")
add(AUTHZ_DOC, ["all", [P(H, "eq", "no-one-knows"), P(H, "neq", "no-one-knows"), P(L, "incl", "xxxxx"),
                        P(L, "incl", "c"), P(L, "excl", "d")]], "F", src + ":232-263",
    error_contains="Unauthorized")
add(AUTHZ_DOC, ["all", []], "T", src + ":265-272")
add(BENCH_DOC, ["all", [P("context.request.http.method", "eq", "GET"),
                        P("context.request.http.path", "eq", "/allow")]], "T", src + ":275-303 (benchmark)")
# unknown operator: expressions.go:93-95 (OperatorFromString of an unknown name -> UnknownOperator)
add(AUTHZ_DOC, ["all", [P(H, "contains", "no")]], "E", "pkg/jsonexp/expressions.go:93-95",
    error_contains="unsupported operator for json authorization")

src = "pkg/service/auth_pipeline_test.go"
add(PIPELINE_DOC, ["all", [P("context.request.http.path", "neq", "/operation")]], "F", src + ":389-412 (unmatching when)")
add(PIPELINE_DOC, ["all", [P("context.request.http.path", "eq", "/operation")]], "T", src + ":414-439 (matching when)")
add(PIPELINE_DOC, ["all", [P("auth.identity", "eq", "leeloo"), P("auth.authorization.credential", "eq", "multipass")]],
    "T", src + ":583-596 (NewAuthorizationJSON document)")

src = "pkg/json/json_test.go"
add(JSON_TEST_DOC, P("auth.identity.email_verified", "eq", "true"), "T", src + ":174-175 (bool -> \"true\")")
add(JSON_TEST_DOC, P("auth.identity.github\\.com", "eq", "https://github.com/john"), "T",
    src + ":177-178 (escaped dot in key)")
add(JSON_TEST_DOC, P("auth.identity.username", "eq", "john"), "T", src + ":162-163")

SA_DOC = '{"auth":{"identity":{"serviceaccount":{"name":"my:ns:sa","long-name":"SA in the NS namespace"}}}}'
NAME_DOC = '{"auth":{"identity":{"fullname":"John Doe"}}}'
B64_UNPADDED = '{"auth":{"identity":{"username":{"encoded":"am9obg","decoded":"john"}}}}'
B64_PADDED = '{"auth":{"identity":{"username":{"encoded":"am9obg==","decoded":"john"}}}}'
B64_QUOTES = ('{"auth":{"identity":{"username":{"encoded":"bXkgbmFtZSBpcyAiam9obiI=",'
              '"decoded":"my name is \\"john\\""}}}}')
STRIP_DOC = "{\"auth\":{\"identity\":{\"username\": \"\n\nbob\u0012\"}}}"
MODIFIER_CASES = [
    (JSON_TEST_DOC, "auth.identity.username.@case:upper", "JOHN", ":165-166"),
    (JSON_TEST_DOC, 'auth.identity.email.@extract:{"sep":"@","pos":1}', "test", ":168-169"),
    (JSON_TEST_DOC, 'auth.identity.github\\.com|@extract:{"sep":"/","pos":3}|@case:upper', "JOHN", ":180-181"),
    (SA_DOC, "auth.identity.serviceaccount.long-name.@extract", "SA", ":210"),
    (SA_DOC, 'auth.identity.serviceaccount.long-name.@extract:{"pos":0}', "SA", ":211"),
    (SA_DOC, 'auth.identity.serviceaccount.long-name.@extract:{"pos":8}', "", ":212"),
    (SA_DOC, 'auth.identity.serviceaccount.name.@extract:{"sep":":","pos":1}', "ns", ":213"),
    (NAME_DOC, 'auth.identity.fullname.@replace:{"old":"John","new":"Jane"}', "Jane Doe", ":219"),
    (NAME_DOC, 'auth.identity.fullname.@replace:{"old":"Peter","new":"Jane"}', "John Doe", ":220"),
    (NAME_DOC, "auth.identity.fullname.@case:upper", "JOHN DOE", ":226"),
    (NAME_DOC, "auth.identity.fullname.@case:lower", "john doe", ":227"),
    (B64_UNPADDED, "auth.identity.username.encoded.@base64:decode", "john", ":233"),
    (B64_UNPADDED, "auth.identity.username.decoded.@base64:encode", "am9obg==", ":234"),
    (B64_PADDED, "auth.identity.username.encoded.@base64:decode", "john", ":238"),
    (B64_PADDED, "auth.identity.username.decoded.@base64:encode", "am9obg==", ":239"),
    (B64_QUOTES, "auth.identity.username.encoded.@base64:decode", 'my name is "john"', ":243"),
    (B64_QUOTES, "auth.identity.username.decoded.@base64:encode", "bXkgbmFtZSBpcyAiam9obiI=", ":244"),
    (STRIP_DOC, "auth.identity.username.@strip", "bob", ":262"),
]
for doc, sel, val, lines in MODIFIER_CASES:
    add(doc, P(sel, "eq", val), "T", src + lines + " (modifier)")
    add(doc, P(sel, "eq", val + "?"), "F", src + lines + " (modifier, another value)")

src = "tests/v1beta2/authconfig.yaml"
add(PIPELINE_DOC, P("context.request.http.path", "matches", "^/admin(/.*)?$"), "F", src + ":131-137")
add(PIPELINE_DOC.replace('"/operation","host"', '"/admin/x","host"'),
    P("context.request.http.path", "matches", "^/admin(/.*)?$"), "T", src + ":131-137")


def main():
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(out, "w") as f:
        json.dump({"generator": "tests/golden/make_reference_kats.py", "cases": cases}, f, indent=1)
    print(f"wrote {len(cases)} cases to {out}")


if __name__ == "__main__":
    main()
