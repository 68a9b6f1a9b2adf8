"""Synthetic Authorization-JSON workloads for the BASELINE.json configs.

Documents follow the shape pkg/service/auth_pipeline.go:542-616 produces with Go's
encoding/json (compact, map keys sorted, `<>&` escaped as \\u003c \\u003e \\u0026):
  {"context":{"request":{"http":{...headers...}}},"request":{...},"source":{...},
   "destination":{...},"auth":{"identity":{...JWT claims...},"metadata":{...}}}
No dataset is fetched: everything is generated from numpy default_rng(seed).

  c1  1 doc, All(eq auth.identity.sub, incl auth.identity.groups, matches path)
  c2  N docs of 768..1280 B, one All of 16 eq/neq/incl patterns over 12 selectors
  c3  N docs, 64 patterns (24 eq, 12 neq, 10 incl, 10 excl, 8 matches),
      All(Any x4 of 8, All x4 of 8)
  c4  N docs x 10k multi-tenant AuthConfigs (8-32 patterns each, regex in 10 %), each
      request's AuthConfig selected on the host through the pkg/index restatement from a
      Zipf(1.1) request host; requests bucketed by AuthConfig (set_of_req sorted), longest
      first inside a bucket
  c5  N JWT-claims-heavy docs of 4096 +- 64 B, one AuthConfig with the full authz phase:
      4 top-level `when`, 4 authz configs (2 `when` + 16 rules each, 2 `matches`), 4
      response header selectors (2 plain, 2 json)
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from .jsonexp import (All, Any, EqualOperator, ExcludesOperator, IncludesOperator, NotEqualOperator, Pattern,
                      RegexOperator)

_GO_ESC = {"<": "\\u003c", ">": "\\u003e", "&": "\\u0026", " ": "\\u2028", " ": "\\u2029"}


def go_json(obj) -> str:
    """encoding/json.Marshal: compact, HTML-safe escapes (the form GetAuthorizationJSON
    hands to Matches). Dict insertion order stands for Go struct field order; callers
    pass Go maps through go_map() so their keys come out sorted like Go's."""
    s = json.dumps(obj, separators=(",", ":"), ensure_ascii=False)
    for k, v in _GO_ESC.items():
        s = s.replace(k, v)
    return s


@dataclass
class Workload:
    name: str
    arena: np.ndarray  # uint8
    offs: np.ndarray   # uint64
    lens: np.ndarray   # uint32
    expr: object       # jsonexp.Expression (the first AuthConfig's, for multi-tenant batches)
    description: str
    exprs: Optional[list] = None          # multi-tenant: one expression per AuthConfig (set id)
    set_of_req: Optional[np.ndarray] = None  # multi-tenant: u32[n] set id per request
    hosts: Optional[List[str]] = None     # multi-tenant: request host per request (index input)
    auth_config: object = None            # c5: the pipeline.AuthConfig of the full phase

    @property
    def sets(self) -> list:
        return self.exprs if self.exprs is not None else [self.expr]

    @property
    def n(self) -> int:
        return int(self.lens.shape[0])

    @property
    def n_patterns(self) -> int:
        return len(self.expr.flatten()[0])

    def patterns_per_request(self) -> np.ndarray:
        """R of each request's selected rule set (request x rule evaluations per request)."""
        counts = np.array([len(e.flatten()[0]) for e in self.sets], dtype=np.int64)
        if self.set_of_req is None:
            return np.full(self.n, counts[0], dtype=np.int64)
        return counts[self.set_of_req]

    def doc(self, i: int) -> bytes:
        o = int(self.offs[i])
        return self.arena[o:o + int(self.lens[i])].tobytes()


METHODS = ["GET"] * 19 + ["POST"]
HEADER_NAMES = ["accept", "accept-encoding", "accept-language", "cache-control", "content-type", "cookie",
                "origin", "referer", "user-agent", "x-b3-spanid", "x-b3-traceid", "x-envoy-attempt-count",
                "x-forwarded-for", "x-forwarded-proto", "x-request-id", "x-amzn-trace-id", "x-client-version",
                "x-correlation-id", "x-device-id", "x-session", "sec-fetch-mode", "sec-fetch-site", "pragma",
                "dnt"]
GROUPS = ["users", "admins", "devs", "ops", "billing", "support", "qa", "sales"]
ROLES = ["reader", "writer", "auditor", "owner", "viewer", "editor"]


def go_map(d: dict) -> dict:
    """A Go map: encoding/json writes its keys sorted."""
    return {k: d[k] for k in sorted(d)}


def _hex(rng, k):
    return "".join(rng.choice(list("0123456789abcdef"), size=k))


def _make_doc(rng: np.random.Generator, target_len: int, uid: int) -> bytes:
    p = rng.random(16)
    method = "GET" if p[0] < 0.95 else rng.choice(["POST", "PUT", "DELETE"])
    sub = "user-%04d" % (uid % 10000) if p[1] < 0.95 else "user-0000"
    headers = {}
    for name in rng.choice(HEADER_NAMES, size=int(rng.integers(1, 5)), replace=False):
        headers[str(name)] = _hex(rng, int(rng.integers(4, 13)))
    headers["x-tenant"] = "acme" if p[2] < 0.95 else "globex"
    if p[3] >= 0.95:
        headers["x-blocked"] = "1"
    headers["authorization"] = "Bearer " + _hex(rng, 16)
    headers["user-agent"] = "Mozilla/5.0 curl/8.%d <bot>" % int(rng.integers(0, 9))
    headers[":path"] = "/api/v%d/orders/%d" % (int(rng.integers(1, 4)), int(rng.integers(1, 100000)))
    host = "api.example.com" if p[4] < 0.95 else "api.example.org"
    path = headers[":path"] if p[5] < 0.95 else "/admin/metrics"
    groups = [g for g in GROUPS if rng.random() < 0.3]
    if p[6] < 0.95:
        groups.append("users")
    if p[7] < 0.05:
        groups.append("banned")
    roles = [r for r in ROLES if rng.random() < 0.3]
    if p[8] < 0.95:
        roles.append("reader")
    http = {"id": str(int(rng.integers(10**15, 10**16))), "method": str(method), "headers": go_map(headers),
            "path": path, "host": host, "scheme": "https" if p[9] < 0.95 else "http", "protocol": "HTTP/1.1"}
    identity = go_map({
        "aud": "talker-api" if p[10] < 0.95 else "other-api",
        "azp": "talker-api", "email": "%s@%s" % (sub, "example.com" if p[11] < 0.95 else "evil.io"),
        "email_verified": bool(p[12] < 0.95), "exp": int(1700000000 + rng.integers(0, 10**6)),
        "groups": sorted(set(groups)), "iat": int(1699990000 + rng.integers(0, 10**6)),
        "iss": "https://sso.example.com/realms/acme" if p[13] < 0.95 else "https://sso.evil.io/realms/x",
        "name": "User %d" % uid, "preferred_username": sub,
        "realm_access": {"roles": sorted(set(roles))}, "scope": "openid email profile",
        "sub": sub, "typ": "Bearer", "acr": 0.5,
    })
    doc = {
        "context": {"source": {"address": {"socketAddress": {"address": "10.%d.%d.%d" % tuple(rng.integers(0, 255, 3)),
                                                              "portValue": int(rng.integers(1024, 65535))}}},
                    "request": {"time": {"seconds": int(1700000000 + uid)}, "http": http}},
        "request": {"host": host, "method": str(method), "path": path, "url_path": path.split("?")[0],
                    },
        "source": {"address": "10.0.0.%d" % int(rng.integers(1, 250)) if p[14] < 0.95 else "10.66.6.6"},
        "destination": {"address": "10.1.0.1", "port": 8080},
        "auth": {"identity": identity, "metadata": go_map({"tenant": {"plan": "gold" if p[15] < 0.95 else "free"}})},
    }
    s = go_json(doc)
    # over the target: drop optional parts (random headers first, then Envoy metadata
    # no selector reads) until it fits or nothing optional is left
    optional = [k for k in headers if k not in ("x-tenant", "x-blocked", "authorization", "user-agent", ":path")]
    while len(s) > target_len and optional:
        del headers[optional.pop()]
        http["headers"] = go_map(headers)
        s = go_json(doc)
    for drop in (lambda: doc["context"].pop("source"), lambda: doc["context"]["request"].pop("time"),
                 lambda: http.pop("id")):
        if len(s) <= target_len:
            break
        drop()
        s = go_json(doc)
    # pad (a header value) to the target length
    short = target_len - len(s)
    if short > 20:
        headers["x-padding"] = "p" * (short - len(',"x-padding":""'))
        http["headers"] = go_map(headers)
        s = go_json(doc)
    return s.encode("utf-8")


C5_GROUPS = ["grp-%02d" % i for i in range(64)]
C5_ROLES = ["role-%02d" % i for i in range(40)]


def _make_doc_c5(rng: np.random.Generator, target_len: int, uid: int) -> bytes:
    """A JWT-claims-heavy Authorization JSON (~4 KiB): the c2 document plus 32 groups, 20
    realm roles and nested resource_access client roles in the identity."""
    base = json.loads(_make_doc(rng, 900, uid))
    ident = base["auth"]["identity"]
    groups = sorted(set(rng.choice(C5_GROUPS, size=31, replace=False).tolist()) | {"users"})
    if rng.random() < 0.05:
        groups = [g for g in groups if g != "users"]
    ident["groups"] = groups
    ident["realm_access"] = {"roles": sorted(set(rng.choice(C5_ROLES, size=19, replace=False).tolist()) | {"reader"})}
    ident["resource_access"] = go_map({
        "talker-api": {"roles": sorted(rng.choice(["read", "write", "admin", "audit"], size=2, replace=False).tolist())},
        "account": {"roles": ["manage-account", "view-profile"]},
        "billing-%d" % int(rng.integers(0, 9)): {"roles": ["viewer"]},
    })
    ident["session_state"] = _hex(rng, 32)
    ident["sid"] = _hex(rng, 32)
    ident["jti"] = _hex(rng, 24)
    ident["auth_time"] = int(1699990000 + rng.integers(0, 10**6))
    ident["given_name"] = "User"
    ident["family_name"] = str(uid)
    base["auth"]["identity"] = go_map(ident)
    s = go_json(base)
    # the rest is the bearer token itself (a signed JWT of these claims is this long)
    short = target_len - len(s)
    if short > 0:
        hdrs = base["context"]["request"]["http"]["headers"]
        b64 = np.array(list("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_"))
        tok = hdrs["authorization"][len("Bearer "):]
        extra = "".join(rng.choice(b64, size=short).tolist())
        hdrs["authorization"] = "Bearer eyJ" + extra[:max(0, short - 3)] + tok
        s = go_json(base)
    return s.encode("utf-8")


def _volatile_spans(doc: bytes):
    """Byte spans of a document whose contents no pattern depends on (bearer-token hex,
    x-padding, the start of a c5 JWT): (start, length, alphabet) with at most 32 bytes
    each, rewritten per copy so that tiled documents are all distinct."""
    import re

    out = []
    for m in re.finditer(rb"Bearer (?:eyJ)?([0-9a-zA-Z_-]{8,})", doc):
        out.append((m.start(1), min(32, m.end(1) - m.start(1)), 0))
    for m in re.finditer(rb'"x-padding":"(p{8,})"', doc):
        out.append((m.start(1), min(32, m.end(1) - m.start(1)), 1))
    return out


_ALPHABETS = [np.frombuffer(b"0123456789abcdef", dtype=np.uint8), np.frombuffer(b"pqrstuvwxyz", dtype=np.uint8)]


def make_docs(n: int, seed: int, lo: int = 768, hi: int = 1280, unique: int = 4096,
              maker=None, uniquify: bool = False) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """n documents (lengths ~U[lo, hi]) packed into (arena, offs, lens). `unique` distinct
    documents are generated and tiled by a random permutation; with `uniquify` every copy
    also gets its own random bearer-token / padding bytes (same length and structure, no
    pattern reads them), so no two documents of the batch are byte-identical."""
    rng = np.random.default_rng(seed)
    m = min(n, unique)
    maker = maker or _make_doc
    base = [maker(rng, int(rng.integers(lo, hi + 1)), i) for i in range(m)]
    idx = rng.integers(0, m, size=n) if n > m else np.arange(n)
    parts = [base[i] for i in idx]
    lens = np.fromiter((len(b) for b in parts), dtype=np.uint32, count=n)
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    if uniquify and n > m:
        spans = [_volatile_spans(b) for b in base]
        for alpha_id, alpha in enumerate(_ALPHABETS):
            # (template, start, length) of this alphabet's spans, then every copy's bytes
            tmpl = [(t, st, ln) for t, sp in enumerate(spans) for st, ln, a in sp if a == alpha_id]
            if not tmpl:
                continue
            per = {}
            for t, st, ln in tmpl:
                per.setdefault(t, []).append((st, ln))
            rel = [np.concatenate([np.arange(st, st + ln) for st, ln in per.get(t, [])]).astype(np.int64)
                   if t in per else np.zeros(0, dtype=np.int64) for t in range(m)]
            cnt = np.array([len(r) for r in rel], dtype=np.int64)[idx]
            step = 1 << 16  # copies per chunk (bounded index arrays)
            for c0 in range(0, n, step):
                ii = np.arange(c0, min(n, c0 + step))
                pos = np.concatenate([rel[idx[i]] for i in ii]) + np.repeat(offs[ii].astype(np.int64), cnt[ii])
                arena[pos] = alpha[rng.integers(0, len(alpha), size=len(pos))]
    return arena, offs, lens


def c1_expression():
    return All(
        Pattern("auth.identity.sub", EqualOperator, "user-0042"),
        Pattern("auth.identity.groups", IncludesOperator, "admins"),
        Pattern("context.request.http.path", RegexOperator, r"^/api/v[0-9]+/orders/[0-9]+$"),
    )


def c2_expression():
    """16 patterns (8 eq, 4 neq, 4 incl) over 12 distinct selectors, each true w.p. ~0.95."""
    return All(
        Pattern("context.request.http.method", EqualOperator, "GET"),
        Pattern("context.request.http.host", EqualOperator, "api.example.com"),
        Pattern("context.request.http.scheme", EqualOperator, "https"),
        Pattern("context.request.http.headers.x-tenant", EqualOperator, "acme"),
        Pattern("auth.identity.iss", EqualOperator, "https://sso.example.com/realms/acme"),
        Pattern("auth.identity.aud", EqualOperator, "talker-api"),
        Pattern("auth.identity.email_verified", EqualOperator, "true"),
        Pattern("auth.metadata.tenant.plan", EqualOperator, "gold"),
        Pattern("context.request.http.headers.x-blocked", NotEqualOperator, "1"),
        Pattern("auth.identity.sub", NotEqualOperator, "user-0000"),
        Pattern("context.request.http.method", NotEqualOperator, "DELETE"),
        Pattern("source.address", NotEqualOperator, "10.66.6.6"),
        Pattern("auth.identity.groups", IncludesOperator, "users"),
        Pattern("auth.identity.realm_access.roles", IncludesOperator, "reader"),
        Pattern("auth.identity.groups", IncludesOperator, "users"),
        Pattern("auth.identity.realm_access.roles", IncludesOperator, "reader"),
    )


def c3_expression():
    """64 patterns: 24 eq, 12 neq, 10 incl, 10 excl, 8 matches; All(Any x4 of 8, All x4 of 8)."""
    eq = [
        ("context.request.http.method", "GET"), ("context.request.http.host", "api.example.com"),
        ("context.request.http.scheme", "https"), ("context.request.http.headers.x-tenant", "acme"),
        ("auth.identity.iss", "https://sso.example.com/realms/acme"), ("auth.identity.aud", "talker-api"),
        ("auth.identity.email_verified", "true"), ("auth.metadata.tenant.plan", "gold"),
        ("request.method", "GET"), ("request.host", "api.example.com"), ("auth.identity.typ", "Bearer"),
        ("auth.identity.azp", "talker-api"), ("context.request.http.protocol", "HTTP/1.1"),
        ("destination.port", "8080"), ("auth.identity.acr", "0.5"), ("destination.address", "10.1.0.1"),
        ("auth.identity.scope", "openid email profile"), ("request.url_path", "/admin/metrics"),
        ("context.request.http.headers.x-blocked", "1"), ("auth.identity.sub", "user-0042"),
        ("auth.identity.realm_access.roles.0", "auditor"), ("auth.identity.groups.0", "admins"),
        ("context.request.http.headers.content-type", "application/json"), ("auth.identity.name", "User 42"),
    ]
    neq = [
        ("context.request.http.headers.x-blocked", "1"), ("auth.identity.sub", "user-0000"),
        ("context.request.http.method", "DELETE"), ("source.address", "10.66.6.6"),
        ("auth.identity.aud", "other-api"), ("auth.metadata.tenant.plan", "free"),
        ("context.request.http.scheme", "http"), ("request.host", "api.example.org"),
        ("auth.identity.iss", "https://sso.evil.io/realms/x"), ("context.request.http.headers.x-tenant", "globex"),
        ("auth.identity.email_verified", "false"), ("request.method", "PUT"),
    ]
    incl = [("auth.identity.groups", "users"), ("auth.identity.realm_access.roles", "reader"),
            ("auth.identity.groups", "admins"), ("auth.identity.realm_access.roles", "owner"),
            ("auth.identity.groups", "devs"), ("auth.identity.realm_access.roles", "writer"),
            ("auth.identity.groups", "ops"), ("auth.identity.realm_access.roles", "viewer"),
            ("auth.identity.groups", "qa"), ("auth.identity.aud", "talker-api")]
    excl = [("auth.identity.groups", "banned"), ("auth.identity.realm_access.roles", "root"),
            ("auth.identity.groups", "sales"), ("auth.identity.realm_access.roles", "editor"),
            ("auth.identity.groups", "billing"), ("auth.identity.groups", "support"),
            ("auth.identity.realm_access.roles", "auditor"), ("auth.identity.groups", "guests"),
            ("auth.identity.realm_access.roles", "nobody"), ("auth.identity.sub", "user-0000")]
    rx = [
        ("context.request.http.path", r"^/api/v[0-9]+/orders/[0-9]+$"),
        ("context.request.http.method", r"^(GET|HEAD|OPTIONS)$"),
        ("auth.identity.email", r"@example\.com$"),
        ("context.request.http.headers.user-agent", r"(?i)mozilla/5\.0 .*curl/\d+"),
        ("auth.identity.iss", r"^https://sso\.[a-z]+\.com/realms/[a-z]+$"),
        ("context.request.http.headers.x-request-id", r"^[0-9a-f]{4,16}$"),
        ("request.url_path", r"^/admin(/.*)?$"),
        ("auth.identity.preferred_username", r"^user-\d{4}$"),
    ]
    likely_eq, rare_eq = eq[:17], eq[17:]
    likely_incl, med_incl = [incl[0], incl[1], incl[9]], incl[2:9]
    likely_excl, med_excl = [excl[0], excl[1], excl[7], excl[8], excl[9]], excl[2:7]
    likely_rx, med_rx = [rx[0], rx[1], rx[2], rx[3], rx[4], rx[7]], [rx[5], rx[6]]
    likely = ([Pattern(s, EqualOperator, v) for s, v in likely_eq] + [Pattern(s, NotEqualOperator, v) for s, v in neq]
              + [Pattern(s, IncludesOperator, v) for s, v in likely_incl]
              + [Pattern(s, ExcludesOperator, v) for s, v in likely_excl]
              + [Pattern(s, RegexOperator, v) for s, v in likely_rx])
    other = ([Pattern(s, EqualOperator, v) for s, v in rare_eq] + [Pattern(s, IncludesOperator, v) for s, v in med_incl]
             + [Pattern(s, ExcludesOperator, v) for s, v in med_excl] + [Pattern(s, RegexOperator, v) for s, v in med_rx])
    rng = np.random.default_rng(33)
    likely = [likely[i] for i in rng.permutation(len(likely))]
    all_pats, spare = likely[:32], likely[32:]
    any_pats = spare + other
    any_pats = [any_pats[i] for i in rng.permutation(len(any_pats))]
    all_groups = [all_pats[8 * k:8 * k + 8] for k in range(4)]
    any_groups = [any_pats[8 * k:8 * k + 8] for k in range(4)]
    return All(*[Any(*g) for g in any_groups], *[All(*g) for g in all_groups])


def _c4_pattern_pool():
    """(selector, operator, value) candidates for the multi-tenant rule sets: the c3 pools
    plus per-tenant literals."""
    e = c3_expression()
    pats, _, _ = e.flatten()
    plain = [(p.selector, p.operator, p.value) for p in pats if p.operator != RegexOperator]
    rx = [(p.selector, p.operator, p.value) for p in pats if p.operator == RegexOperator]
    return plain, rx


def c4_expression(rng: np.random.Generator, tenant: int, plain, rx):
    """One tenant's AuthConfig rules: 8-32 patterns (1-2 `matches` in 10 % of the configs)
    in a random two- or three-level All/Any tree."""
    k = int(rng.integers(8, 33))
    n_rx = int(rng.integers(1, 3)) if rng.random() < 0.10 else 0
    chosen = [plain[i] for i in rng.choice(len(plain), size=k - n_rx, replace=True)]
    chosen += [rx[i] for i in rng.choice(len(rx), size=n_rx, replace=False)]
    # per-tenant literals so that no two configs are the same
    extra = [("auth.identity.sub", NotEqualOperator, "user-%04d" % (tenant % 9973)),
             ("context.request.http.headers.x-tenant", NotEqualOperator, "t%d" % tenant)]
    chosen[:2] = extra
    pats = [Pattern(sel, op, val) for sel, op, val in chosen]
    pats = [pats[i] for i in rng.permutation(len(pats))]
    groups, i = [], 0
    while i < len(pats):
        g = int(rng.integers(2, 9))
        grp = pats[i:i + g]
        i += g
        node = Any(*grp) if rng.random() < 0.3 else All(*grp)
        if rng.random() < 0.2 and len(groups) > 0:  # a third level
            node = All(groups.pop(), node) if rng.random() < 0.5 else Any(groups.pop(), node)
        groups.append(node)
    return All(*groups)


def c4_index_entries(n_configs: int = 10000, n_wild: int = 100):
    """(host key, set id) of C4's AuthConfigs: t<i>.example.com, then the wildcards
    *.r<j>.example.com"""
    n_exact = n_configs - n_wild
    return [("t%d.example.com" % i if i < n_exact else "*.r%d.example.com" % (i - n_exact), i)
            for i in range(n_configs)]


def c4_index_and_rules(n_configs: int = 10000, n_wild: int = 100, seed: int = 4):
    """The AuthConfigs: hosts t<i>.example.com (i < n_configs - n_wild) and wildcards
    *.r<j>.example.com, in a pkg/index restatement whose entries are set ids."""
    from .index import Index

    rng = np.random.default_rng(seed)
    plain, rx = _c4_pattern_pool()
    idx = Index()
    exprs = []
    for host, i in c4_index_entries(n_configs, n_wild):
        err = idx.set("ns/cfg-%d" % i, host, i, False)
        assert err is None, err
        exprs.append(c4_expression(rng, i, plain, rx))
    return idx, exprs


def c4_hosts(n: int, n_configs: int, n_wild: int, rng: np.random.Generator) -> List[str]:
    """Request hosts: 85 % exact tenant hosts and 10 % wildcard hits, both Zipf(1.1) over
    tenants; 3 % carry a :port (the auth.go:270-289 retry); 2 % match no AuthConfig."""
    n_exact = n_configs - n_wild
    def zipf(m, size):
        w = 1.0 / np.arange(1, m + 1) ** 1.1
        return rng.choice(m, size=size, p=w / w.sum())
    kind = rng.random(n)
    ex = zipf(n_exact, n)
    wi = zipf(n_wild, n)
    sub = rng.integers(0, 1000, size=n)
    hosts = []
    for i in range(n):
        if kind[i] < 0.85:
            h = "t%d.example.com" % ex[i]
        elif kind[i] < 0.95:
            h = "h%d.r%d.example.com" % (sub[i], wi[i])
        elif kind[i] < 0.98:
            h = "t%d.example.com:8443" % ex[i]
        else:
            h = "u%d.nowhere.io" % sub[i]
        hosts.append(h)
    return hosts


def make_c4(n: int, seed: int = 4, n_configs: int = 10000, n_wild: int = 100, unique: int = 4096,
            uniquify: bool = False) -> Workload:
    """C4: multi-tenant batch. Each request's AuthConfig comes from the
    host index (requests without one are dropped, as the reference answers NOT_FOUND
    before any evaluation); the batch is bucketed by AuthConfig. Document bodies are the
    c2 generator's (Authorization JSON of ~1 KiB)."""
    from .index import bucket_order, select_sets

    idx, exprs = c4_index_and_rules(n_configs, n_wild, seed=4)
    rng = np.random.default_rng(seed)
    m = int(n * 1.03) + 16
    hosts = c4_hosts(m, n_configs, n_wild, rng)
    sets = select_sets(idx, hosts)
    keep = np.nonzero(sets >= 0)[0][:n]
    sets = sets[keep]
    arena, offs, lens = make_docs(len(keep), seed, unique=unique, uniquify=uniquify)
    order = bucket_order(sets, lens)  # bucket by AuthConfig, longest first inside a bucket
    return Workload("c4", arena, offs[order], lens[order], exprs[0],
                    f"{len(keep)} docs x {n_configs} AuthConfigs (8-32 patterns, regex in 10 %), "
                    "host-index selection, bucketed by AuthConfig and length class",
                    exprs=exprs, set_of_req=sets[order].astype(np.uint32),
                    hosts=[hosts[keep[i]] for i in order])


def c5_auth_config():
    """C5's AuthConfig: top-level `when` of 4 patterns; 4 authorization
    configs, each with a 2-pattern `when` and 16 rules (2 `matches`); 4 response header
    selectors (2 plain, 2 DynamicJSON, one with a template)."""
    from .pipeline import AuthConfig, AuthorizationConfig
    from .response import JSONValue, ResponseConfig

    P = Pattern
    top = All(P("context.request.http.method", NotEqualOperator, "DELETE"),
              P("context.request.http.host", EqualOperator, "api.example.com"),
              P("context.request.http.path", RegexOperator, r"^/(api|admin)/"),
              P("context.request.http.headers.x-tenant", EqualOperator, "acme"))
    authz = []
    for k in range(4):
        g = ["grp-%02d" % ((7 * k + j) % 64) for j in range(4)]
        r = ["role-%02d" % ((5 * k + j) % 40) for j in range(4)]
        cond = All(P("context.request.http.scheme", EqualOperator, "https"),
                   P("auth.identity.aud", EqualOperator, "talker-api") if k % 2 == 0
                   else P("auth.identity.azp", NotEqualOperator, "other"))
        rules = All(
            P("auth.identity.iss", EqualOperator, "https://sso.example.com/realms/acme"),
            P("auth.identity.email_verified", EqualOperator, "true"),
            P("auth.identity.groups", IncludesOperator, "users"),
            P("auth.identity.realm_access.roles", IncludesOperator, "reader"),
            Any(*[P("auth.identity.groups", IncludesOperator, x) for x in g]),
            Any(*[P("auth.identity.realm_access.roles", IncludesOperator, x) for x in r]),
            P("auth.identity.groups", ExcludesOperator, "banned"),
            P("auth.identity.sub", NotEqualOperator, "user-0000"),
            P("auth.identity.email", RegexOperator, r"@example\.com$"),
            P("auth.identity.preferred_username", RegexOperator, r"^user-\d{4}$"))
        authz.append(AuthorizationConfig("authz-%d" % k, rules=rules, conditions=cond, priority=0))
    resp = [
        ResponseConfig("user", plain=JSONValue(pattern="auth.identity.sub"), wrapper_key="x-auth-user"),
        ResponseConfig("exp", plain=JSONValue(pattern="auth.identity.exp"), wrapper_key="x-auth-exp"),
        ResponseConfig("claims", json_properties=[("groups", JSONValue(pattern="auth.identity.realm_access.roles")),
                                                  ("tenant", JSONValue(pattern="auth.metadata.tenant")),
                                                  ("acr", JSONValue(pattern="auth.identity.acr"))],
                       wrapper_key="x-auth-claims"),
        ResponseConfig("ctx", json_properties=[
            ("user", JSONValue(pattern="{auth.identity.preferred_username}@{context.request.http.host}")),
            ("client_roles", JSONValue(pattern="auth.identity.resource_access.talker-api.roles")),
            ("static", JSONValue(static="v1"))], wrapper_key="x-auth-ctx"),
    ]
    return AuthConfig(conditions=top, authorization=authz, response=resp)


DEFAULT_SEEDS = {"c1": 1, "c2": 2, "c3": 3, "c4": 4, "c5": 5}


def make(name: str, n: Optional[int] = None, seed: Optional[int] = None, unique: Optional[int] = None,
         uniquify: bool = False) -> Workload:
    """A BASELINE config's workload. unique / uniquify: see make_docs (the bench uses
    16384 templates for c2/c3/c4 and distinct bytes in every copy)."""
    name = name.lower()
    seed = seed if seed is not None else DEFAULT_SEEDS.get(name, 0)
    kw = {"uniquify": uniquify}
    if unique is not None:
        kw["unique"] = unique
    if name == "c1":
        arena, offs, lens = make_docs(1, seed, 680, 720)
        return Workload("c1", arena, offs, lens, c1_expression(), "1 doc x All(eq, incl, matches)")
    if name == "c2":
        n = n if n is not None else 1 << 20
        arena, offs, lens = make_docs(n, seed, **kw)
        return Workload("c2", arena, offs, lens, c2_expression(),
                        f"{n} docs (768-1280 B) x All of 16 eq/neq/incl over 12 selectors")
    if name == "c3":
        n = n if n is not None else 1 << 20
        arena, offs, lens = make_docs(n, seed, **kw)
        return Workload("c3", arena, offs, lens, c3_expression(),
                        f"{n} docs x 64 patterns (24 eq/12 neq/10 incl/10 excl/8 matches), All(Any x4, All x4)")
    if name == "c4":
        return make_c4(n if n is not None else 1 << 21, seed, **kw)
    if name == "c5":
        n = n if n is not None else 1 << 21
        arena, offs, lens = make_docs(n, seed, 4032, 4160, maker=_make_doc_c5, **kw)
        cfg = c5_auth_config()
        return Workload("c5", arena, offs, lens, cfg.authorization[0].rules,
                        f"{n} docs of 4096+-64 B x full authz phase (4 when, 4 authz x (2 when + 16 rules), "
                        "4 response selectors)", auth_config=cfg)
    raise ValueError(f"unknown workload {name!r}")
