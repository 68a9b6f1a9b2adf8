"""Response-header selectors on the device (SURVEY.md §8 a14, config C5 tail).

Host-side mirror of:
  JSONValue{Static, Pattern}, ResolveFor, IsTemplate     pkg/json/json.go:24-61
  ReplaceJSONPlaceholders                                pkg/json/json.go:96-151
  StringifyJSON                                          pkg/json/json.go:153-159
  response.Plain / response.DynamicJSON .Call            pkg/evaluators/response/plain.go,
                                                         dynamic_json.go:20-31
  ResponseConfig.WrapObjectAsHeaderValue, WrapResponses  pkg/evaluators/response.go:150-174

Split of the work: every gjson path a response reads (a pattern, or a `{placeholder}` of a
template) is compiled once into a selector ruleset; `authjx_select_batch` resolves all of
them for a batch on the GPU (the document scan) and returns spans. The host turns spans
into Go values (gjson `Result.Value()` / `Result.String()`) and formats the header
(`fmt.Sprintf("%v")` or `json.Marshal`), which is per-output string building, not a scan.
There is no CPU path for the lookup: without the HIP library the calls raise.

Go formatting restated here (Go 1.21):
  * fmt %v of float64 = strconv.FormatFloat(f, 'g', -1, 64): shortest digits, %e form
    when the decimal exponent is < -4 or >= 6 (1685557675 -> "1.685557675e+09")
  * fmt %v of map[string]interface{} = "map[k:v k:v]" (keys sorted), []interface{} =
    "[a b]", nil = "<nil>"
  * encoding/json: HTML-safe string escapes, float64 'f' unless |f| < 1e-6 or >= 1e21
    (then 'e' with "e-07" -> "e-7"), map keys sorted, NaN/Inf -> error (StringifyJSON
    returns "" and the error is dropped by WrapObjectAsHeaderValue).
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

# gjson.Type (= AUTHJX_JSON_*)
NULL, FALSE, NUMBER, STRING, TRUE, JSON = 0, 1, 2, 3, 4, 5
UNSUPPORTED = 255

_ALL_CURLY = re.compile(r"{")                      # json.go:18
_MODIFIER_CURLY = re.compile(r"[^@]+@\w+:{", re.ASCII)  # json.go:19 (Go's \w is ASCII)

RESPONSE_PLAIN = "plain"      # pkg/evaluators/response.go (responsePlain)
RESPONSE_JSON = "json"        # responseJSON
HTTP_HEADER_WRAPPER = "httpHeader"              # response.go wrapper kinds
ENVOY_DYNAMIC_METADATA_WRAPPER = "envoyDynamicMetadata"


# ------------------------------------------------------------------------------------
# JSONValue and templates (json.go:24-151)
# ------------------------------------------------------------------------------------
@dataclass
class JSONValue:
    """json.JSONValue: a static value, or a gjson pattern / template resolved per request."""

    static: object = None
    pattern: str = ""

    def is_template(self) -> bool:
        """json.go:58-61: not every '{' opens a modifier argument."""
        return len(_MODIFIER_CURLY.findall(self.pattern)) != len(_ALL_CURLY.findall(self.pattern))

    def paths(self) -> List[str]:
        """The gjson paths ResolveFor reads (one for a pattern, the placeholders of a template)."""
        if not self.pattern:
            return []
        if self.is_template():
            return [p for kind, p in template_segments(self.pattern) if kind == "path"]
        return [self.pattern]


def template_segments(source: str) -> List[Tuple[str, str]]:
    """ReplaceJSONPlaceholders (json.go:96-151) split at compile time: the literal text and
    the placeholder paths depend only on the template. Returns [("lit", s) | ("path", p)];
    an empty placeholder `{}` contributes nothing (json.go:119-122)."""
    out: List[Tuple[str, str]] = []
    replaced, buffer = bytearray(), bytearray()
    escaping = inside = False
    nested = 0
    for b in source.encode("utf-8"):
        if b == 123:  # '{'
            if escaping:
                replaced.append(b)
            elif inside:
                buffer.append(b)
                nested += 1
            else:
                inside = True
            escaping = False
        elif b == 125:  # '}'
            if inside:
                if nested > 0:
                    buffer.append(b)
                    nested -= 1
                else:
                    if buffer:
                        if replaced:
                            out.append(("lit", replaced.decode("utf-8", "replace")))
                            replaced = bytearray()
                        out.append(("path", buffer.decode("utf-8", "replace")))
                        buffer = bytearray()
                    inside = False
            else:
                replaced.append(b)
            escaping = False
        elif b == 92:  # '\\'
            if inside:
                buffer.append(b)
            else:
                if escaping:
                    replaced.append(b)
                escaping = not escaping
        else:
            if inside:
                buffer.append(b)
            else:
                replaced.append(b)
            escaping = False
    if replaced:
        out.append(("lit", replaced.decode("utf-8", "replace")))
    return out


# ------------------------------------------------------------------------------------
# gjson Result.String() / Result.Value() from a span
# ------------------------------------------------------------------------------------
def _runeit(s: bytes) -> int:
    try:
        return int(s[:4].decode("ascii"), 16) if len(s) >= 4 else 0
    except ValueError:
        return 0  # strconv.ParseUint error -> 0


def _encode_rune(r: int) -> bytes:
    """utf8.EncodeRune: surrogates and out-of-range runes become U+FFFD."""
    if r < 0 or r > 0x10FFFF or 0xD800 <= r <= 0xDFFF:
        r = 0xFFFD
    return chr(r).encode("utf-8")


def gjson_unescape(s: bytes) -> bytes:
    """gjson `unescape` (v1.14.0) over a string's contents (between the quotes)."""
    out = bytearray()
    i, n = 0, len(s)
    while i < n:
        c = s[i]
        if c >= 0x20 and c != 0x5C:  # plain byte (gjson copies >= ' ' as-is; < ' ' stops)
            out.append(c)
            i += 1
            continue
        if c < 0x20:
            return bytes(out)
        i += 1
        if i >= n:
            return bytes(out)
        e = s[i]
        simple = {0x5C: b"\\", 0x2F: b"/", 0x62: b"\b", 0x66: b"\f", 0x6E: b"\n", 0x72: b"\r",
                  0x74: b"\t", 0x22: b'"'}
        if e in simple:
            out += simple[e]
            i += 1
        elif e == 0x75:  # 'u'
            if i + 5 > n:
                return bytes(out)
            r = _runeit(s[i + 1:])
            i += 5
            if 0xD800 <= r < 0xE000:
                if n - i >= 6 and s[i] == 0x5C and s[i + 1] == 0x75:
                    r2 = _runeit(s[i + 2:])
                    i += 6
                    if 0xD800 <= r < 0xDC00 and 0xDC00 <= r2 < 0xE000:
                        r = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00)
                    else:
                        r = 0xFFFD  # utf16.DecodeRune of an invalid pair
            out += _encode_rune(r)
        else:
            return bytes(out)
    return bytes(out)


def _go_bytes_str(b: bytes) -> str:
    # Go strings are bytes; documents from encoding/json are valid UTF-8
    return b.decode("utf-8", "replace")


# authjx_value.esc of an element count (a `#` path part; ajx_device.h kValCount): the
# count is in `start`, not a document span
VAL_COUNT = 2
# authjx_value.esc flag of built text (a modifier chain's or a "#." list's Result;
# ajx_modifiers.h kValText): [start, start + len) of the request's text slot
VAL_TEXT = 4


class SelectedRow:
    """One request's selected values: spans[k] = {start, len, type | esc << 8} and the text
    slot that VAL_TEXT values point into."""

    __slots__ = ("spans", "text")

    def __init__(self, spans, text=None):
        self.spans, self.text = spans, text

    def __getitem__(self, k):
        return self.spans[k]

    def source(self, t: int, doc: bytes) -> bytes:
        if (int(t) >> 8) & VAL_TEXT:
            return self.text.tobytes()
        return doc


class Selected:
    """ValueSelectors.resolve's output for n requests: spans u32[n][k][3] and text slots
    u8[n][text_stride] (authjx_select_text_batch)."""

    def __init__(self, spans: np.ndarray, text: Optional[np.ndarray] = None):
        self.spans, self.text = spans, text

    def __len__(self):
        return len(self.spans)

    def __getitem__(self, j) -> SelectedRow:
        return SelectedRow(self.spans[j], None if self.text is None else self.text[j])

    def unresolved(self) -> np.ndarray:
        """Requests with a value the device left unresolved (type 255)."""
        if not self.spans.size:
            return np.zeros(len(self.spans), dtype=bool)
        return ((self.spans[:, :, 2] & 0xFF) == 255).any(axis=1)


def result_string(doc: bytes, start: int, length: int, typ: int) -> str:
    """gjson Result.String()."""
    raw = doc[start:start + length]
    if typ == STRING:
        return _go_bytes_str(gjson_unescape(raw[1:-1]) if b"\\" in raw else raw[1:-1])
    if typ == NUMBER:
        if re.fullmatch(rb"-?[0-9]+", raw):
            return raw.decode()
        return go_format_float(go_parse_float(raw), "f")
    if typ == TRUE:
        return "true"
    if typ == FALSE:
        return "false"
    if typ == JSON:
        return _go_bytes_str(raw)
    return ""


class _JSONReader:
    """gjson Result.Value() of an object / array span: map[string]interface{} (the last
    duplicate key wins), []interface{}, float64, string, bool, nil."""

    _ws = b" \t\n\r"

    def __init__(self, raw: bytes):
        self.s, self.i = raw, 0

    def _skip(self):
        while self.i < len(self.s) and self.s[self.i] in self._ws:
            self.i += 1

    def value(self):
        self._skip()
        c = self.s[self.i:self.i + 1]
        if c == b"{":
            self.i += 1
            obj: Dict[str, object] = {}
            while True:
                self._skip()
                if self.s[self.i:self.i + 1] == b"}":
                    self.i += 1
                    return obj
                k = self._string()
                self._skip()
                self.i += 1  # ':'
                obj[k] = self.value()
                self._skip()
                if self.s[self.i:self.i + 1] == b",":
                    self.i += 1
        if c == b"[":
            self.i += 1
            arr = []
            while True:
                self._skip()
                if self.s[self.i:self.i + 1] == b"]":
                    self.i += 1
                    return arr
                arr.append(self.value())
                self._skip()
                if self.s[self.i:self.i + 1] == b",":
                    self.i += 1
        if c == b'"':
            return self._string()
        m = re.compile(rb"[^,\]} \t\n\r]+").match(self.s, self.i)
        tok = m.group(0) if m else b""
        self.i += len(tok)
        if tok == b"true":
            return True
        if tok == b"false":
            return False
        if tok == b"null":
            return None
        return float(tok)

    def _string(self) -> str:
        j = self.i + 1
        while True:
            if self.s[j] == 0x5C:
                j += 2
                continue
            if self.s[j] == 0x22:
                break
            j += 1
        body = self.s[self.i + 1:j]
        self.i = j + 1
        return _go_bytes_str(gjson_unescape(body) if b"\\" in body else body)


def result_value(doc: bytes, start: int, length: int, typ: int):
    """gjson Result.Value(): the Go interface{} ResolveFor returns for a pattern."""
    raw = doc[start:start + length]
    if typ == STRING:
        return result_string(doc, start, length, typ)
    if typ == NUMBER:
        return float(raw)
    if typ == TRUE:
        return True
    if typ == FALSE:
        return False
    if typ == JSON:
        return _JSONReader(raw).value()
    return None


# ------------------------------------------------------------------------------------
# Go number and value formatting
# ------------------------------------------------------------------------------------
def _shortest_digits(x: float) -> Tuple[str, int]:
    """Shortest round-trip decimal digits of |x| > 0 and the decimal-point position dp
    (|x| = 0.d1d2... x 10^dp): the digits strconv's shortest mode produces."""
    r = repr(abs(x))
    mant, _, exp = r.partition("e")
    e = int(exp) if exp else 0
    ip, _, fp = mant.partition(".")
    digits = (ip + fp).lstrip("0")
    lead = len(ip + fp) - len((ip + fp).lstrip("0"))
    dp = len(ip) - lead + e
    return digits.rstrip("0") or "0", dp


_GO_DEC = re.compile(rb"[+-]?([0-9]+\.?[0-9]*|\.[0-9]+)([eE][+-]?[0-9]+)?")
_GO_HEX = re.compile(rb"[+-]?0[xX]([0-9a-fA-F]+\.?[0-9a-fA-F]*|\.[0-9a-fA-F]+)[pP][+-]?[0-9]+")


def go_parse_float(raw: bytes) -> float:
    """strconv.ParseFloat(raw, 64) as gjson keeps it (the value even on error: a syntax
    error gives 0, a range error +-Inf). Python's float() rounds decimal text to
    nearest-even exactly as Go does; '_' separators (valid in Go only after a base
    prefix) are not expected in JSON number tokens and read as a syntax error."""
    if _GO_DEC.fullmatch(raw):
        return float(raw)
    if _GO_HEX.fullmatch(raw):
        return float.fromhex(raw.decode())
    m = re.fullmatch(rb"([+-]?)(inf|infinity)", raw, re.I)
    if m:
        return -math.inf if m.group(1) == b"-" else math.inf
    if re.fullmatch(rb"nan", raw, re.I):
        return math.nan
    return 0.0


def go_format_float(x: float, fmt: str) -> str:
    """strconv.FormatFloat(x, fmt, -1, 64) for fmt in 'f', 'e', 'g'."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "+Inf" if x > 0 else "-Inf"
    neg = math.copysign(1.0, x) < 0
    sign = "-" if neg else ""
    if x == 0:
        return sign + ("0e+00" if fmt == "e" else "0")
    d, dp = _shortest_digits(x)
    if fmt == "g":
        # strconv ftoa %g: "if precision was the shortest possible, use precision 6 for
        # this decision": %e when exp < -4 || exp >= 6
        exp = dp - 1
        fmt = "e" if (exp < -4 or exp >= 6) else "f"
    if fmt == "e":
        m = d[0] + ("." + d[1:] if len(d) > 1 else "")
        exp = dp - 1
        return "%s%se%s%02d" % (sign, m, "-" if exp < 0 else "+", abs(exp))
    # 'f'
    if dp <= 0:
        return sign + "0." + "0" * (-dp) + d
    if dp >= len(d):
        return sign + d + "0" * (dp - len(d))
    return sign + d[:dp] + "." + d[dp:]


def go_sprint_v(v) -> str:
    """fmt.Sprintf("%v", v) for the values gjson Value() produces."""
    if v is None:
        return "<nil>"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float):
        return go_format_float(v, "g")
    if isinstance(v, str):
        return v
    if isinstance(v, dict):
        return "map[" + " ".join("%s:%s" % (k, go_sprint_v(v[k])) for k in sorted(v, key=lambda s: s.encode())) + "]"
    if isinstance(v, list):
        return "[" + " ".join(go_sprint_v(e) for e in v) + "]"
    return str(v)


class _UnsupportedValue(Exception):
    pass


def _json_string(s: str) -> str:
    """encoding/json string encoding, escapeHTML = true (Go 1.21)."""
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch in ('"', "\\"):
            out.append("\\" + ch)
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif o < 0x20 or ch in "<>&":
            out.append("\\u00%02x" % o)
        elif o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        elif 0xD800 <= o <= 0xDFFF:
            out.append("\\ufffd")
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def go_json_marshal(v) -> str:
    """json.Marshal of gjson Value() results (and maps of them)."""
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float):
        if math.isnan(v) or math.isinf(v):
            raise _UnsupportedValue(v)
        a = abs(v)
        if a != 0 and (a < 1e-6 or a >= 1e21):
            s = go_format_float(v, "e")
            s = re.sub(r"e-0(\d)$", r"e-\1", s)
            return s
        return go_format_float(v, "f")
    if isinstance(v, str):
        return _json_string(v)
    if isinstance(v, dict):
        return "{" + ",".join(_json_string(k) + ":" + go_json_marshal(v[k])
                              for k in sorted(v, key=lambda s: s.encode())) + "}"
    if isinstance(v, list):
        return "[" + ",".join(go_json_marshal(e) for e in v) + "]"
    raise _UnsupportedValue(v)


def stringify_json(v) -> str:
    """json.StringifyJSON (json.go:153-159) with its error dropped, as
    WrapObjectAsHeaderValue does: "" when Marshal fails. gjson.ParseBytes(...).String() of
    Marshal's output is the output itself, except for a top-level string, which String()
    unescapes."""
    try:
        j = go_json_marshal(v)
    except _UnsupportedValue:
        return ""
    if j.startswith('"'):
        b = j.encode("utf-8")
        return _go_bytes_str(gjson_unescape(b[1:-1]))
    if j in ("true", "false"):
        return j
    if j == "null":
        return ""
    if re.fullmatch(r"-?[0-9.eE+\-]+", j):  # a number: Result.String()
        return result_string(j.encode(), 0, len(j), NUMBER)
    return j


# ------------------------------------------------------------------------------------
# Response configs and the batched response phase
# ------------------------------------------------------------------------------------
@dataclass
class ResponseConfig:
    """evaluators.ResponseConfig with a Plain or DynamicJSON evaluator (response.go)."""

    name: str
    plain: Optional[JSONValue] = None                      # response.Plain
    json_properties: Optional[List[Tuple[str, JSONValue]]] = None  # response.DynamicJSON
    wrapper: str = HTTP_HEADER_WRAPPER
    wrapper_key: str = ""
    conditions: object = None  # `when` (jsonexp.Expression)
    priority: int = 0

    def get_type(self) -> str:
        if self.json_properties is not None:
            return RESPONSE_JSON
        if self.plain is not None:
            return RESPONSE_PLAIN
        return ""

    def values(self) -> List[JSONValue]:
        if self.json_properties is not None:
            return [v for _, v in self.json_properties]
        return [self.plain] if self.plain is not None else []

    def wrap_object_as_header_value(self, obj) -> str:
        """response.go:150-158"""
        if self.get_type() == RESPONSE_JSON:
            return stringify_json(obj)
        return go_sprint_v(obj)


class ValueSelectors:
    """Every gjson path of a list of JSONValues compiled into one selector ruleset (the
    reconcile-time compile point), resolved per batch on the device (one span per path and
    request); value() is JSONValue.ResolveFor on those spans (pkg/json/json.go:41-53)."""

    def __init__(self, values: Sequence[JSONValue], ctx, what: str = "selectors"):
        from . import jsonexp

        self.ctx = ctx
        self.paths: List[str] = []
        self._slot: Dict[str, int] = {}
        for v in values:
            if v is None:
                continue
            for p in v.paths():
                if p not in self._slot:
                    self._slot[p] = len(self.paths)
                    self.paths.append(p)
        self.ruleset = None
        if self.paths:
            pats = [(p, int(jsonexp.EqualOperator), "") for p in self.paths]
            self.ruleset = ctx.compile(pats, [], -1)
            bad = [p for p, st in zip(self.paths, self.ruleset.status) if st != 0]
            if bad:
                from .runtime import AuthjxError

                raise AuthjxError(f"{what} not compiled for the device: {bad}")

    # bytes of built text per request (modifier chains, "#." lists); a request whose
    # values do not fit is left undecided
    TEXT_STRIDE = 8192

    def resolve(self, docs: Sequence[bytes], arena, offs, lens) -> Selected:
        """The values of every path for each request from the device: spans {start, len,
        type | esc << 8} of the document or of the request's text slot (VAL_TEXT)."""
        if self.ruleset is None:
            return Selected(np.zeros((len(docs), 0, 3), dtype=np.uint32))
        spans, text = self.ctx.select_text_host_arena([self.ruleset], arena, offs, lens,
                                                      text_stride=self.TEXT_STRIDE)
        return Selected(spans, text)

    def value(self, v: JSONValue, doc: bytes, spans_r) -> object:
        return self._value(v, doc, spans_r)

    @staticmethod
    def _src(spans_r, t, doc: bytes) -> bytes:
        return spans_r.source(t, doc) if isinstance(spans_r, SelectedRow) else doc

    def _value(self, v: JSONValue, doc: bytes, spans_r) -> object:
        if not v.pattern:
            return v.static
        if v.is_template():
            parts = []
            for kind, s in template_segments(v.pattern):
                if kind == "lit":
                    parts.append(s)
                else:
                    st, ln, t = spans_r[self._slot[s]]
                    if int(t) >> 8 == VAL_COUNT:
                        parts.append(str(int(st)))
                    else:
                        parts.append(result_string(self._src(spans_r, t, doc), int(st), int(ln), int(t) & 0xFF))
            return "".join(parts)
        st, ln, t = spans_r[self._slot[v.pattern]]
        if int(t) >> 8 == VAL_COUNT:  # an array's element count (a `#` part): Number
            return float(int(st))
        return result_value(self._src(spans_r, t, doc), int(st), int(ln), int(t) & 0xFF)


class ResponseSelectors(ValueSelectors):
    """Every gjson path of a list of response configs compiled into one selector ruleset
    (the reconcile-time compile point), resolved per batch on the device."""

    def __init__(self, configs: Sequence[ResponseConfig], ctx):
        self.configs = list(configs)
        super().__init__([v for c in self.configs for v in c.values()], ctx, "response selectors")

    def call(self, c: ResponseConfig, doc: bytes, spans_r) -> object:
        """Plain.Call / DynamicJSON.Call (plain.go, dynamic_json.go:20-31)."""
        if c.json_properties is not None:
            return {name: self._value(v, doc, spans_r) for name, v in c.json_properties}
        if c.plain is not None:
            return self._value(c.plain, doc, spans_r)
        return None


def wrap_responses(responses: Dict[str, Tuple[ResponseConfig, object]]):
    """evaluators.WrapResponses (response.go:161-174): headers and dynamic metadata."""
    headers: Dict[str, str] = {}
    metadata: Dict[str, object] = {}
    for c, obj in responses.values():
        if c.wrapper == HTTP_HEADER_WRAPPER:
            headers[c.wrapper_key] = c.wrap_object_as_header_value(obj)
        elif c.wrapper == ENVOY_DYNAMIC_METADATA_WRAPPER:
            metadata[c.wrapper_key] = obj
    return headers, metadata
