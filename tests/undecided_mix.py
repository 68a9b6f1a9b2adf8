"""A realistic selector mix for the UNDECIDED surface: every selector the reference's
user guides and examples put in `when` / `patterns` (docs/user-guides/*.md,
docs/features.md; collected by grep over `selector:`), over Authorization-JSON documents
shaped like the reference's (pkg/service/auth_pipeline_test.go:593,
well_known_attributes.go), with eq / neq / incl / excl / matches values drawn from the
documents. Also the gjson forms the device leaves UNSUPPORTED by design."""
import base64
import json
import random

# selectors of the reference's docs (the `|` in the jwt_authn one is a gjson pipe)
DOC_SELECTORS = [
    "context.request.http.path", "context.request.http.method", "auth.identity.realm_access.roles",
    'context.request.http.path.@extract:{"sep":"/","pos":2}',
    r"context.metadata_context.filter_metadata.envoy\.filters\.http\.jwt_authn|verified_jwt",
    "auth.identity.username", 'context.request.http.headers.x-forwarded-for.@extract:{"sep":","}',
    'context.request.http.headers.x-forwarded-for.@extract:{"sep": ","}',
    "context.request.http.headers.authorization", "auth.identity.sub", "auth.identity.roles",
    "auth.identity.email_verified", "auth.identity.anonymous", "context.request.time.seconds",
    'context.request.http.method.@replace:{"old":"GET","new":"read"}.@replace:{"old":"POST","new":"write"}',
    "context.request.http.method.@case:lower",
    'context.request.http.headers.authorization.@extract:{"pos":1}|@base64:decode|@extract:{"sep":":"}',
    "context.request.http.body.@fromstr|request.userInfo",
    "context.request.http.body.@fromstr|request.object.metadata.namespace",
    "auth.metadata.userinfo.email", "auth.metadata.geoinfo.country_iso_code", "auth.identity.user.username",
    "auth.identity.privileges.talker-api", "auth.identity.metadata.labels.tier",
    r"auth.identity.metadata.annotations.authorino\.kuadrant\.io/username",
    r"auth.identity.metadata.annotations.auth-data\/username", "auth.identity.authorization.permissions",
    "auth.identity", "auth.authorization.features.apiKey", "auth.identity.roles.#", "auth.identity.roles.1",
]

# gjson forms the device does not compile (AUTHJX_PAT_UNSUPPORTED by design; the Go
# jsonexp tree evaluates them): wildcards, queries, multipaths, JSON
# lines, gjson's other built-in modifiers, '#' inside a path after a pipe
BY_DESIGN_UNSUPPORTED = [
    "auth.identity.rol*", "auth.identity.r?les", "auth.identity.roles.#(==\"admin\")",
    "auth.identity.groups.#(name==\"a\")#", "[auth.identity.sub,auth.identity.username]",
    "{auth.identity.sub}", "..0", "auth.identity.roles|@reverse", "auth.identity|@keys", "auth.identity|@this",
    "auth.identity|roles.#",
]


def make_doc(rng: random.Random, non_ascii: bool = False) -> bytes:
    user = rng.choice(["john", "jane", "alice", "bob"]) + str(rng.randrange(100))
    if non_ascii and rng.random() < 0.5:
        user += rng.choice(["é", "ß"])  # (ß: SpecialCasing; Go's simple mapping keeps it)
    review = {"kind": "AdmissionReview", "request": {
        "userInfo": {"username": "system:serviceaccount:" + user}, "object": {"metadata": {
            "namespace": rng.choice(["authorino", "default", "kube-system"])}}}}
    d = {
        "context": {
            "request": {
                "http": {
                    "id": str(rng.randrange(10 ** 9)), "method": rng.choice(["GET", "POST", "DELETE", "PUT"]),
                    "path": "/" + "/".join(rng.choice(["pets", "posts", "admin", "api", str(rng.randrange(99))])
                                           for _ in range(rng.randrange(1, 4))),
                    "headers": {"authorization": "Basic " + base64.b64encode(
                        (user + ":" + rng.choice(["pw", "s3cret"])).encode()).decode(),
                        "x-forwarded-for": ",".join("10.0.%d.%d" % (rng.randrange(9), rng.randrange(9))
                                                    for _ in range(rng.randrange(1, 4)))},
                    "body": json.dumps(review, separators=(",", ":")),
                    "host": "talker-api.127.0.0.1.nip.io"},
                "time": {"seconds": rng.randrange(1_600_000_000, 1_800_000_000), "nanos": rng.randrange(10 ** 9)}},
            "metadata_context": {"filter_metadata": {"envoy.filters.http.jwt_authn": {
                "verified_jwt": {"sub": user, "iss": "https://idp"}}}}},
        "auth": {
            "identity": {"sub": user, "username": user, "email_verified": rng.random() < 0.5,
                         "anonymous": rng.random() < 0.2,
                         "roles": rng.sample(["admin", "user", "reader", "writer"], rng.randrange(0, 4)),
                         "realm_access": {"roles": rng.sample(["admin", "member"], rng.randrange(0, 3))},
                         "user": {"username": user}, "privileges": {"talker-api": ["read", "write"][: rng.randrange(3)]},
                         "metadata": {"labels": {"tier": rng.choice(["gold", "silver"])}, "annotations": {
                             "authorino.kuadrant.io/username": user, "auth-data/username": user}},
                         "authorization": {"permissions": ["read"]}},
            "metadata": {"userinfo": {"email": user + "@example.com"}, "geoinfo": {"country_iso_code": "DE"}},
            "authorization": {"features": {"apiKey": rng.random() < 0.5}}, "response": {}},
    }
    return json.dumps(d, separators=(",", ":"), ensure_ascii=False).encode()


def make_rulesets(rng: random.Random, docs, k: int = 12):
    """k AuthConfig-like rulesets of 4-10 patterns over DOC_SELECTORS (values from the
    documents' own Strings, through the oracle) as right-nested All / Any chains."""
    import pyoracle as O

    out = []
    for _ in range(k):
        pats = []
        for _ in range(rng.randrange(4, 11)):
            sel = rng.choice(DOC_SELECTORS)
            s = O.gjson_string_mods(rng.choice(docs), sel)
            val = (s or b"").decode("utf-8", "replace")
            op = rng.choice([1, 2, 3, 4, 5])
            if op == 5:
                val = "^" + "".join(c for c in val[:4] if c.isalnum())
            pats.append((sel, op, val))
        nodes = [(0, -1, -1, i) for i in range(len(pats))]
        root = -1
        kind = rng.choice([1, 2])
        for i in reversed(range(len(pats))):
            nodes.append((kind, i, root, -1))
            root = len(nodes) - 1
        out.append((pats, nodes, root))
    return out
