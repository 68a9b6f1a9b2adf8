"""The number path pinned to an implementation neither restatement shares: gjson's
Result.String() of a non-integer JSON number is Go's FormatFloat(ParseFloat(raw), 'f',
-1, 64). Python's float() is a correctly rounded ParseFloat for JSON number texts, and
numpy's format_float_positional(x, unique=True, trim='-') is the shortest round-trip
digits in the 'f' layout (Dragon4), i.e. FormatFloat(x, 'f', -1, 64) for finite x.
Both the device code (ajx_device.h / ajx_float.h, host build) and the oracle
(oracle/gofloat_ref.c) are checked against them on 10^6 random doubles (their Go
shortest texts, %.17g and %.16g forms), long decimals, exact midpoints between
neighbouring doubles, subnormals, the 1e21 boundary and the float64 ends. The raw rule
the single-pass kernels use (-?[0-9]+, or a decimal of at most 15 digits that is its
own shortest text) is checked too: whenever it takes a text as its own String(), numpy
agrees."""
import os
import subprocess

import numpy as np
import pytest

import pyoracle as O

_NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


def go_f(x: float) -> str:
    """FormatFloat(x, 'f', -1, 64) by numpy (finite x; Go spells the specials +Inf/-Inf/NaN)."""
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "+Inf" if x > 0 else "-Inf"
    return np.format_float_positional(x, unique=True, trim="-")


def gjson_string(raw: str) -> str:
    body = raw[1:] if raw.startswith("-") else raw
    if body and body.isdigit():
        return raw  # Result.String(): a raw -?[0-9]+ is returned as is
    return go_f(float(raw))


def _texts(rng, n):
    bits = rng.integers(0, 2**63, size=n, dtype=np.int64).view(np.uint64) | (
        rng.integers(0, 2, size=n, dtype=np.uint64) << np.uint64(63))
    xs = bits.view(np.float64)
    xs = xs[np.isfinite(xs)]
    # ordinary magnitudes too (what metadata floats look like)
    ys = np.ldexp(rng.integers(1, 2**53, size=n).astype(np.float64), -rng.integers(0, 80, size=n)) * \
        np.where(rng.random(n) < 0.5, -1.0, 1.0)
    out = []
    for x in np.concatenate([xs, ys]).tolist():
        out.append(repr(x).replace("inf", "1e400"))  # Go-shortest digits (exponent form)
        out.append("%.17g" % x)
    for x in xs[: n // 2].tolist():
        out.append("%.16g" % x)
    # long decimals, exact midpoints and their neighbours, the ends
    for _ in range(n // 20):
        nd = int(rng.integers(18, 60))
        s = str(int(rng.integers(1, 10))) + "".join(map(str, rng.integers(0, 10, size=nd - 1)))
        dot = int(rng.integers(1, nd))
        out.append(("-" if rng.random() < 0.5 else "") + s[:dot] + "." + s[dot:] + "e%d" % int(rng.integers(-30, 30)))
    from decimal import Decimal, getcontext

    getcontext().prec = 800
    for x in xs[: n // 50].tolist():
        if x == 0:
            continue
        a = Decimal(x)
        b = Decimal(float(np.nextafter(x, np.inf)))
        mid = (a + b) / 2
        for t in (mid, mid + Decimal(10) ** (mid.adjusted() - 700), mid - Decimal(10) ** (mid.adjusted() - 700)):
            out.append(format(t, "f") if abs(t.adjusted()) < 40 else format(t, "e"))
    out += ["5e-324", "4.9406564584124654e-324", "2.4703282292062328e-324", "2.2250738585072014e-308",
            "1.7976931348623157e308", "-1.7976931348623157e308", "1.7976931348623159e308", "1e21", "1e+21",
            "9.999999999999999e20", "1e20", "0.1", "0.30000000000000004", "-0.0", "0.000001", "1e-7", "100.5",
            "123456789012.345", "1234567890123.456", "0.5", "-0.5", "12.25", "0.05"]
    return out


@pytest.fixture(scope="module")
def harness():
    O.build()
    subprocess.run(["make", "-s", "-C", _NATIVE, "float_diff"], check=True)
    return os.path.join(_NATIVE, "float_diff")


def test_number_strings_match_numpy(harness):
    rng = np.random.default_rng(2024)
    texts = _texts(rng, 500_000)  # 10^6 random doubles (bit patterns and ordinary magnitudes)
    assert len(texts) >= 2_000_000
    r = subprocess.run([harness, "--stdin"], input="\n".join(texts) + "\n", capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0
    lines = r.stdout.split("\n")
    bad = []
    fast = 0
    for raw, line in zip(texts, lines):
        dev, orc, rawfast = line.split("\t")
        want = gjson_string(raw)
        if dev != want or orc != want:
            bad.append((raw, dev, orc, want))
        if rawfast == "1":
            fast += 1
            if raw != want:
                bad.append((raw, "raw-rule", raw, want))
    assert not bad, bad[:10]
    assert fast > 1000


def test_simple_decimals_are_their_own_string(harness):
    """Random decimals of <= 15 digits in canonical form: the raw rule takes each, and
    numpy's FormatFloat agrees with the text."""
    rng = np.random.default_rng(7)
    texts = []
    for _ in range(200_000):
        nd = int(rng.integers(2, 16))
        ip = int(rng.integers(0, nd))
        digs = "".join(map(str, rng.integers(0, 10, size=nd)))
        a, b = digs[:ip].lstrip("0") or "0", digs[ip:].rstrip("0")
        if not b:
            b = "5"
        if len(a) + len(b) > 15:
            continue
        texts.append(("-" if rng.random() < 0.3 else "") + a + "." + b)
    r = subprocess.run([harness, "--stdin"], input="\n".join(texts) + "\n", capture_output=True, text=True,
                       timeout=300)
    lines = r.stdout.split("\n")
    for raw, line in zip(texts, lines):
        dev, orc, rawfast = line.split("\t")
        assert rawfast == "1", raw
        assert go_f(float(raw)) == raw == dev == orc, raw
