"""Host-side mirror of the parts of pkg/service/auth_pipeline.go that sit on the hot path:
the `when` gates and the authorization phase, batched over many requests.

  evaluate_conditions              auth_pipeline.go:378-388  (nil -> pass; err -> err;
                                   false -> "unmatching conditions for config")
  AuthConfig-level conditions      auth_pipeline.go:454-457  (not met -> OK, skipped)
  evaluator-level conditions       auth_pipeline.go:120-125  (not met -> evaluator ignored)
  authorization phase              auth_pipeline.go:287-322  + groupAuthConfigsByPriority
                                   :184-201: priorities ascending, every config of a
                                   priority evaluated, the first failure is PERMISSION_DENIED
                                   (:478-481); a success stores the object under
                                   auth.authorization.<name> for later priorities (:312).
  evaluator cache                  authorization.go:56-76 (authorino_amd.cache): the key is
                                   resolved on the device for every request whose `when`
                                   passed; a hit grants without the rules, a success is
                                   stored. Requests of a batch see the cache in batch order
                                   (what serving them one after another would give).
  denyWith (Unauthorized)          auth_pipeline.go:478-481 + customizeDenyWith :581-608:
                                   code -> status, message / body / headers resolved on the
                                   device against the document the denial was decided on
                                   and stringified (json.StringifyJSON).
  response phase                   auth_pipeline.go:324-349 + :490-494 (only after a
                                   successful authorization phase): per priority, each
                                   response config's `when`, then Plain / DynamicJSON
                                   objects wrapped as headers (evaluators.WrapResponses,
                                   pkg/evaluators/response.go:150-174). Selector lookups
                                   run on the device (authorino_amd.response).

AuthPipelineBatch compiles every expression once (the reconcile-time compile point,
controllers/auth_config_controller.go) and evaluates each priority level of a batch in ONE
device launch: the (request, expression) pairs are a set_of_req batch whose offsets all
point into the same document arena. Identity / metadata / response phases are out of
scope; the documents given are GetAuthorizationJSON's output after those
phases.

Where the reference is nondeterministic the mirror fixes one order: configs of one
priority run concurrently in Go and the denial reported is whichever goroutine answers
first; here it is the first failing config in declaration order (the decision itself,
deny or not, is the same either way).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import jsonexp
from .authorization import JSONPatternMatching, UnauthorizedError
from .cache import EvaluatorCache, is_hit
from .response import JSONValue, ResponseConfig, ResponseSelectors, ValueSelectors, stringify_json, wrap_responses

UNMATCHING_CONDITIONS = "unmatching conditions for config"
CODE_OK = 0  # rpc.OK
CODE_UNKNOWN = 2  # rpc.UNKNOWN: the device left the request undecided (AuthResult.undecided)
CODE_PERMISSION_DENIED = 7  # rpc.PERMISSION_DENIED
UNDECIDED_MESSAGE = "authjx: undecided on the device"


class ConditionsError(Exception):
    """fmt.Errorf("unmatching conditions for config") (auth_pipeline.go:385)."""

    def __init__(self):
        super().__init__(UNMATCHING_CONDITIONS)


def evaluate_conditions(conditions: Optional[jsonexp.Expression], authorization_json) -> Optional[Exception]:
    """AuthPipeline.evaluateConditions (auth_pipeline.go:378-388), one document."""
    if conditions is None:
        return None
    match, err = conditions.matches(authorization_json)
    if err is not None:
        return err
    if not match:
        return ConditionsError()
    return None


@dataclass
class AuthorizationConfig:
    """evaluators.AuthorizationConfig with a JSON pattern-matching evaluator
    (pkg/evaluators/authorization.go; Priority and Conditions from the CRD)."""

    name: str
    rules: Optional[jsonexp.Expression] = None  # JSONPatternMatching.Rules
    conditions: Optional[jsonexp.Expression] = None  # `when`
    priority: int = 0
    cache: Optional[EvaluatorCache] = None  # AuthorizationConfig.Cache (authorization.go:56-76)


@dataclass
class DenyWithValues:
    """evaluators.DenyWithValues (pkg/evaluators/config.go:70-80)."""

    code: int = 0
    message: Optional[JSONValue] = None
    headers: List[Tuple[str, JSONValue]] = field(default_factory=list)  # []json.JSONProperty
    body: Optional[JSONValue] = None

    def values(self) -> List[JSONValue]:
        return [v for v in [self.message, self.body] + [h for _, h in self.headers] if v is not None]


@dataclass
class AuthConfig:
    """The slice of auth.AuthConfig the authorization phase reads."""

    conditions: Optional[jsonexp.Expression] = None  # AuthConfig-level `when`
    authorization: List[AuthorizationConfig] = field(default_factory=list)
    response: List[ResponseConfig] = field(default_factory=list)
    unauthorized: Optional[DenyWithValues] = None  # AuthConfig.Unauthorized (denyWith)


@dataclass
class AuthResult:
    """auth.AuthResult (code / message) plus the authorization objects granted."""

    code: int = CODE_OK
    message: str = ""
    skipped: bool = False  # AuthConfig-level conditions not met (auth_pipeline.go:454-457)
    denied_by: Optional[str] = None
    # the device could not decide this request (AUTHJX_UNDECIDED: a pattern compiled as
    # unsupported, or a hex / '_' number literal in a malformed document); the caller
    # routes it to its own evaluator. The other requests of the batch are unaffected.
    undecided: bool = False
    authorization: Dict[str, object] = field(default_factory=dict)
    status: int = 0  # denyWith code (envoy HTTP status); 0 = the gRPC code's default
    body: str = ""   # denyWith body
    deny_headers: List[Dict[str, str]] = field(default_factory=list)  # denyWith headers
    headers: Dict[str, str] = field(default_factory=dict)      # success: WrapResponses headers
    metadata: Dict[str, object] = field(default_factory=dict)  # success: dynamic metadata


def _paths_select_authorization(paths) -> bool:
    return any(p == "auth.authorization" or p.startswith("auth.authorization.") for p in paths)


def _selects_authorization(expr: Optional[jsonexp.Expression]) -> bool:
    if expr is None:
        return False
    pats, _, _ = expr.flatten()
    return any(p.selector == "auth.authorization" or p.selector.startswith("auth.authorization.") for p in pats)


class AuthPipelineBatch:
    """The `when` gates + authorization phase of AuthPipeline.Evaluate for a batch."""

    def __init__(self, auth_config: AuthConfig, device: int = 0, ctx=None):
        from . import runtime

        self.config = auth_config
        self.ctx = ctx if ctx is not None else runtime.context(device)
        self._rs: Dict[int, object] = {}
        exprs = [auth_config.conditions] + [e for c in auth_config.authorization for e in (c.conditions, c.rules)]
        exprs += [c.conditions for c in auth_config.response]
        for e in exprs:
            if e is not None and id(e) not in self._rs:
                self._rs[id(e)] = self.ctx.compile_expression(e)
        prios = sorted({c.priority for c in auth_config.authorization})
        self.levels = [[c for c in auth_config.authorization if c.priority == p] for p in prios]
        # a later priority reads what an earlier one granted (auth.authorization.*): its
        # conditions and rules, its cache keys (ResolveKeyFor on GetAuthorizationJSON,
        # authorization.go:56-66), and denyWith, which resolves on the JSON of the priority
        # that denied (auth_pipeline.go:581-608): the documents must be rebuilt per level
        dw = auth_config.unauthorized
        self._needs_regen = (
            any(_selects_authorization(e) for lvl in self.levels[1:] for c in lvl for e in (c.conditions, c.rules))
            or any(c.cache is not None and _paths_select_authorization(c.cache.key.paths())
                   for lvl in self.levels[1:] for c in lvl)
            or (dw is not None and len(self.levels) > 1
                and any(v is not None and _paths_select_authorization(v.paths()) for v in dw.values())))
        # one forest ruleset for every expression of the phase when no later priority reads
        # what an earlier one granted: one document scan per request for all of them
        self._forest = None
        self._col: Dict[int, int] = {}
        if not self._needs_regen and hasattr(self.ctx, "compile_forest"):
            uniq = []
            for e in exprs:
                if e is not None and id(e) not in self._col:
                    self._col[id(e)] = len(uniq)
                    uniq.append(e)
            if uniq:
                self._forest = self.ctx.compile_forest(uniq)
        self._all = None
        rprios = sorted({c.priority for c in auth_config.response})
        self.response_levels = [[c for c in auth_config.response if c.priority == p] for p in rprios]
        self.selectors = ResponseSelectors(auth_config.response, self.ctx) if auth_config.response else None
        for c in auth_config.response:
            for v in c.values():
                if any(p.startswith("auth.authorization") or p.startswith("auth.response") for p in v.paths()):
                    raise ValueError("response selectors over auth.authorization/auth.response are not batched")
        # cache keys: one selector ruleset per priority level (the keys of its cached configs)
        self.key_selectors = []
        for level in self.levels:
            keys = [c.cache.key for c in level if c.cache is not None]
            self.key_selectors.append(ValueSelectors(keys, self.ctx, "cache keys") if keys else None)
        dw = auth_config.unauthorized
        self.deny_selectors = ValueSelectors(dw.values(), self.ctx, "denyWith selectors") if dw is not None else None

    # one launch: expression k of `exprs` on every request in `reqs`
    def _eval(self, exprs: Sequence[jsonexp.Expression], reqs: np.ndarray, arena, offs, lens):
        from . import runtime

        if self._forest is not None:
            if self._all is None or self._all[0] is not arena:
                tri, err, _ = self.ctx.eval_host_arena([self._forest], arena, offs, lens, with_bitmap=False)
                tri = tri.reshape(len(lens), -1)
                self._all = (arena, tri, err.reshape(len(lens), -1))
            _, tri, err = self._all
            cols = [self._col[id(e)] for e in exprs]
            return tri[reqs][:, cols].T, err[reqs][:, cols].T, [self._forest] * len(exprs)

        sets = [self._rs[id(e)] for e in exprs]
        k = len(exprs)
        sor = np.repeat(np.arange(k, dtype=np.uint32), len(reqs))
        o = np.tile(offs[reqs], k)
        ln = np.tile(lens[reqs], k)
        tri, err, _ = self.ctx.eval_host_arena(sets, arena, o, ln, set_of_req=sor, with_bitmap=False)
        return tri.reshape(k, len(reqs)), err.reshape(k, len(reqs)), sets

    def evaluate(self, docs: Sequence, producer: Optional[Callable[[int, Dict[str, object]], bytes]] = None
                 ) -> List[AuthResult]:
        """Evaluate the batch. `producer(i, authorization_objs)` rebuilds request i's
        Authorization JSON (GetAuthorizationJSON, auth_pipeline.go:542-579) once earlier
        priorities granted objects; it is required only when a later priority selects
        auth.authorization.*."""
        from . import runtime

        if self._needs_regen and producer is None:
            raise ValueError("a later priority selects auth.authorization.*: pass a producer")
        n = len(docs)
        results = [AuthResult() for _ in range(n)]
        docs = [runtime._b(d) for d in docs]

        def pack(ds):
            lens = np.fromiter((len(d) for d in ds), dtype=np.uint32, count=len(ds))
            offs = np.zeros(len(ds), dtype=np.uint64)
            if len(ds):
                offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
            return np.frombuffer(b"".join(ds) + b"\0", dtype=np.uint8), offs, lens

        arena, offs, lens = pack(docs)
        self._all = None
        live = np.arange(n)

        def set_aside(tri):  # requests the device left undecided leave the batch
            nonlocal live
            und = (tri == runtime.UNDECIDED).any(axis=0)
            for i in live[und]:
                results[i].undecided = True
                results[i].code = CODE_UNKNOWN
                results[i].message = UNDECIDED_MESSAGE
            live = live[~und]
            return ~und

        # AuthConfig-level `when` (auth_pipeline.go:454-457): not met -> OK, skipped
        top = self.config.conditions
        if top is not None and n:
            tri, _, _ = self._eval([top], live, arena, offs, lens)
            tri = tri[:, set_aside(tri)]
            met = tri[0] == runtime.T
            for i in live[~met]:
                results[i].skipped = True
            live = live[met]
        for li, level in enumerate(self.levels):
            if not len(live):
                break
            if li and producer is not None:
                for i in live.tolist():
                    docs[i] = runtime._b(producer(i, results[i].authorization))
                arena, offs, lens = pack(docs)
            exprs = [e for c in level for e in (c.conditions, c.rules) if e is not None]
            tri = err = sets = None
            if exprs:
                tri, err, sets = self._eval(exprs, live, arena, offs, lens)
                keep = set_aside(tri)
                tri, err = tri[:, keep], err[:, keep]
            col = {id(e): j for j, e in enumerate(exprs)}
            keys = self.key_selectors[li]
            und_key = np.zeros(len(live), dtype=bool)
            if keys is not None:
                kspans = self._spans(keys, docs, live)
                und_key = self._set_aside_spans(kspans, live, results)
            denied = np.zeros(len(live), dtype=bool)
            for c in level:
                # evaluator-level `when` (auth_pipeline.go:120-125): not met -> ignored
                ok_cond = np.ones(len(live), dtype=bool) if c.conditions is None else tri[col[id(c.conditions)]] == runtime.T
                if c.rules is None:
                    r_t = np.ones(len(live), dtype=bool)
                    r_tri = None
                else:
                    r_tri = tri[col[id(c.rules)]]
                    r_t = r_tri == runtime.T
                for j in np.nonzero(ok_cond & ~und_key)[0]:
                    i = live[j]
                    if c.cache is not None:
                        key = keys.value(c.cache.key, docs[i], kspans[j])  # ResolveKeyFor
                        hit = c.cache.get(key)
                        if is_hit(hit):  # authorization.go:61-65: the evaluator is not called
                            results[i].authorization[c.name] = hit
                            continue
                        if r_t[j]:
                            c.cache.set(key, True)  # authorization.go:70-74
                    if r_t[j]:
                        results[i].authorization[c.name] = True  # json.go:26 -> setAuthorizationObj
                    elif not denied[j]:
                        denied[j] = True
                        res = results[i]
                        res.code = CODE_PERMISSION_DENIED
                        res.denied_by = c.name
                        if r_tri[j] == runtime.E:
                            res.message = sets[col[id(c.rules)]].pattern_error(int(err[col[id(c.rules)]][j]))
                        else:
                            res.message = str(UnauthorizedError())
            live = live[~(denied | und_key)]
        if self.deny_selectors is not None:
            self._deny_with(results, docs)
        if self.selectors is not None and len(live):
            self._responses(results, docs, live, arena, offs, lens)
        return results

    def _spans(self, sel: ValueSelectors, docs, idx):
        """The selector values of docs[idx] (one device select launch)."""
        sub = [docs[i] for i in np.asarray(idx).tolist()]
        lens = np.fromiter((len(d) for d in sub), dtype=np.uint32, count=len(sub))
        offs = np.zeros(len(sub), dtype=np.uint64)
        if len(sub):
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        arena = np.frombuffer(b"".join(sub) + b"\0", dtype=np.uint8)
        return sel.resolve(sub, arena, offs, lens)

    @staticmethod
    def _set_aside_spans(spans, idx, results) -> np.ndarray:
        """Requests whose selector values the device left unresolved (type 255: a value
        over its text slot, non-ASCII @case / @strip) become undecided; returns that mask
        over idx."""
        und = spans.unresolved()
        for i in np.asarray(idx)[und].tolist():
            results[i].undecided = True
            results[i].code = CODE_UNKNOWN
            results[i].message = UNDECIDED_MESSAGE
            results[i].authorization = {}
        return und

    def _deny_with(self, results, docs):
        """customizeDenyWith(result, AuthConfig.Unauthorized) (auth_pipeline.go:581-608) for
        the requests the authorization phase denied."""
        dw = self.config.unauthorized
        idx = np.array([i for i, r in enumerate(results) if r.code == CODE_PERMISSION_DENIED], dtype=np.int64)
        if not len(idx):
            return
        if dw.code:
            for i in idx.tolist():
                results[i].status = dw.code
        sel = self.deny_selectors
        spans = self._spans(sel, docs, idx)
        und = self._set_aside_spans(spans, idx, results)
        for j, i in enumerate(idx.tolist()):
            if und[j]:
                continue
            r, doc = results[i], docs[i]
            if dw.message is not None:
                r.message = stringify_json(sel.value(dw.message, doc, spans[j]))
            if dw.body is not None:
                r.body = stringify_json(sel.value(dw.body, doc, spans[j]))
            if dw.headers:
                r.deny_headers = [{name: stringify_json(sel.value(v, doc, spans[j]))} for name, v in dw.headers]

    def _responses(self, results, docs, live, arena_all, offs_all, lens_all):
        """Phase 4 for the requests that passed authorization (auth_pipeline.go:490-494)."""
        from . import runtime

        sub = [docs[i] for i in live.tolist()]
        lens = np.fromiter((len(d) for d in sub), dtype=np.uint32, count=len(sub))
        offs = np.zeros(len(sub), dtype=np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        arena = np.frombuffer(b"".join(sub) + b"\0", dtype=np.uint8)
        spans = self.selectors.resolve(sub, arena, offs, lens)
        if spans.unresolved().any():
            raise runtime.AuthjxError("device could not resolve a response selector")
        granted = [dict() for _ in sub]
        idx = np.arange(len(sub))
        for level in self.response_levels:
            conds = [c.conditions for c in level if c.conditions is not None]
            met = {}
            if conds:
                tri, _, _ = self._eval(conds, live, arena_all, offs_all, lens_all)
                # (an undecided response condition withholds that response only)
                met = {id(e): tri[j] == runtime.T for j, e in enumerate(conds)}
            for c in level:
                ok = met[id(c.conditions)] if c.conditions is not None else None
                for j in range(len(sub)):
                    if ok is None or ok[j]:
                        granted[j][c.name] = (c, self.selectors.call(c, sub[j], spans[j]))
        for j, i in enumerate(live.tolist()):
            results[i].headers, results[i].metadata = wrap_responses(granted[j])


def evaluate_json_authorization(rules: Optional[jsonexp.Expression], docs: Sequence):
    """JSONPatternMatching.Call over a batch (authorization/json.go:15-27)."""
    return JSONPatternMatching(rules).call_batch(docs)
