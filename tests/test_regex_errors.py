"""Go 1.21 regexp.Compile errors (the E of a `matches` pattern, expressions.go:87-91, and
its text, asserted by pkg/evaluators/authorization/json_test.go:193): a known-answer
table restated from the published Go source — regexp/syntax/parse.go, whose ErrorCode
strings are (regexp/syntax/parse.go, Go 1.21):
  ErrInvalidCharRange    "invalid character class range"
  ErrInvalidEscape       "invalid escape sequence"
  ErrInvalidNamedCapture "invalid named capture"
  ErrInvalidPerlOp       "invalid or unsupported Perl syntax"
  ErrInvalidRepeatOp     "invalid nested repetition operator"
  ErrInvalidRepeatSize   "invalid repeat count"
  ErrMissingBracket      "missing closing ]"
  ErrMissingParen        "missing closing )"
  ErrMissingRepeatArgument "missing argument to repetition operator"
  ErrTrailingBackslash   "trailing backslash at end of expression"
  ErrUnexpectedParen     "unexpected )"
and regexp.Compile's text is "error parsing regexp: " + code + ": `" + expr + "`"
(Error.Error(), regexp/syntax/parse.go). The repeat limit is 1000 (parse.go repeat:
`if min > 1000 || max > 1000`); `(?<name>` is Go 1.22 syntax, unsupported in 1.21.
The device compiler (csrc/ajx_regex.cpp, host build) must give these texts, and the
oracle must decide the pattern E."""
import pytest

import _hosttest as H
import pyoracle as O

GO_121_COMPILE_ERRORS = [
    ("a**", "invalid nested repetition operator: `**`"),
    ("a++", "invalid nested repetition operator: `++`"),
    ("x{2}{3}", "invalid nested repetition operator: `{2}{3}`"),
    ("*a", "missing argument to repetition operator: `*`"),
    ("a|*", "missing argument to repetition operator: `*`"),
    ("a{1001}", "invalid repeat count: `{1001}`"),
    ("a{1,1001}", "invalid repeat count: `{1,1001}`"),
    ("x{1001,}", "invalid repeat count: `{1001,}`"),
    ("(?<n>x)", "invalid or unsupported Perl syntax: `(?<`"),
    ("(?i", "invalid or unsupported Perl syntax: `(?i`"),
    ("[z-a]", "invalid character class range: `z-a`"),
    ("[[:foo:]]", "invalid character class range: `[:foo:]`"),
    ("\\8", "invalid escape sequence: `\\8`"),
    ("(?P<>x)", "invalid named capture: `(?P<>`"),
    ("(?P<n>x", "missing closing ): `(?P<n>x`"),
    ("(a", "missing closing ): `(a`"),
    ("a)", "unexpected ): `a)`"),
    ("[a", "missing closing ]: `[a`"),
    ("[not-a-regex", "invalid character class range: `t-a`"),  # (the range fails before the end)
    ("\\", "trailing backslash at end of expression: ``"),
]


@pytest.mark.parametrize("pat,msg", GO_121_COMPILE_ERRORS)
def test_go_compile_error_text(pat, msg):
    r = H.HostRegex(pat)
    assert r.status == 1, (pat, r.status, r.error)
    assert r.error == "error parsing regexp: " + msg


@pytest.mark.parametrize("pat,msg", GO_121_COMPILE_ERRORS)
def test_oracle_decides_compile_errors_e(pat, msg):
    pats = [("a", 5, pat)]
    rs = O.Ruleset(pats, [(0, -1, -1, 0)], 0)
    assert rs.pattern(0, b'{"a":"x"}') == O.E


@pytest.mark.parametrize("pat", ["\\Q", "(?P<n>a)(?P<n>b)", "a{1000}", "x{0,1000}", "(?i)abc", "[[:alpha:]]"])
def test_go_accepts(pat):
    assert H.HostRegex(pat).status == 0, pat
