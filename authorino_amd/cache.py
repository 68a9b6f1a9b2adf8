"""evaluators.EvaluatorCache (pkg/evaluators/cache.go) for the authorization phase.

  NewEvaluatorCache(keyTemplate, ttl)   cache.go:23-32   TTL in whole seconds
  Get(key)                              cache.go:40-51   hit only while the stored entry's
                                                         remaining TTL is > 0
  Set(key, value)                       cache.go:53-59   the value as json.Marshal bytes
  ResolveKeyFor(authJSON)               cache.go:61-63   keyTemplate.ResolveFor — resolved
                                                         on the device here (ValueSelectors)
  AuthorizationConfig.Call              authorization.go:56-76: a hit returns the cached
                                        object without calling the evaluator; only a
                                        successful (err == nil) result is stored; a nil key
                                        disables both.

Store semantics restated from the pinned dependencies (go.mod: eko/gocache v1.2.0 over
coocood/freecache v1.1.1; neither is vendored under /root/reference):
  - gocache maps the key object to a string: a string key is itself, any other value a
    checksum of its Go type and fmt.Sprint form. The key identity here is therefore
    (Go type, %v text), with strings as themselves.
  - freecache stores `expireAt = now + ttl` in unix seconds (0 when ttl <= 0, no expiry)
    and reports the remaining TTL as expireAt - now; Get misses once now >= expireAt. An
    entry without expiry reports TTL 0, so with ttl <= 0 the reference never hits: kept.
  - freecache evicts by memory (EvaluatorCacheSize MiB); `max_entries` bounds the store
    here (least recently set first), 0 = unbounded.
"""
from __future__ import annotations

import json
import time
from collections import OrderedDict
from typing import Callable, Optional, Tuple

from .response import JSONValue, _UnsupportedValue, go_json_marshal, go_sprint_v

_MISS = object()


def _go_type(v) -> str:
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, float):
        return "float64"
    if isinstance(v, str):
        return "string"
    if isinstance(v, dict):
        return "map[string]interface {}"
    if isinstance(v, list):
        return "[]interface {}"
    return type(v).__name__


def cache_key_identity(key) -> Optional[Tuple[str, str]]:
    """The store key a resolved key value maps to; None for a nil key (no caching)."""
    if key is None:
        return None
    if isinstance(key, str):
        return ("string", key)
    return (_go_type(key), go_sprint_v(key))


class EvaluatorCache:
    def __init__(self, key: JSONValue, ttl: int, clock: Callable[[], float] = time.time, max_entries: int = 0):
        self.key = key
        self.ttl = int(ttl)
        self._clock = clock
        self._max = int(max_entries)
        self._store: "OrderedDict[Tuple[str, str], Tuple[str, int]]" = OrderedDict()

    def _now(self) -> int:
        return int(self._clock())

    def get(self, key):
        """cache.go:40-51: the cached object, or _MISS."""
        ident = cache_key_identity(key)
        if ident is None:
            return _MISS
        e = self._store.get(ident)
        if e is None:
            return _MISS
        raw, expire_at = e
        if expire_at == 0:  # no expiry: TTL reads 0, `ttl > 0` fails
            return _MISS
        if self._now() >= expire_at:
            del self._store[ident]
            return _MISS
        v = json.loads(raw, parse_int=float)  # gojson.Unmarshal into interface{}: float64
        return _MISS if v is None else v  # `cachedObj != nil` (authorization.go:63)

    def set(self, key, value) -> bool:
        """cache.go:53-59; False when the value does not marshal or the key is nil."""
        ident = cache_key_identity(key)
        if ident is None:
            return False
        try:
            raw = go_json_marshal(value)
        except _UnsupportedValue:
            return False
        expire_at = self._now() + self.ttl if self.ttl > 0 else 0
        self._store.pop(ident, None)
        self._store[ident] = (raw, expire_at)
        if self._max and len(self._store) > self._max:
            self._store.popitem(last=False)
        return True

    def clear(self) -> None:
        """Shutdown (cache.go:65-67)."""
        self._store.clear()

    def __len__(self) -> int:
        return len(self._store)


def is_hit(v) -> bool:
    return v is not _MISS
