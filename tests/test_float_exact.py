"""gjson Result.String() of JSON numbers (Go FormatFloat(ParseFloat(raw), 'f', -1, 64)):
the device number code (authorino_amd/csrc/ajx_device.h num_canon + ajx_float.h, host
build in tests/native/float_diff.cpp) against the oracle (oracle/gofloat_ref.c), on
Go-shortest texts of random float64 values, %.16g / %.17g texts, long decimals, subnormals,
exact midpoints between neighbouring doubles and the range ends. A 10^6-value run of the
same harness is recorded in DESIGN.md; this test runs a bounded sample per seed."""
import os
import subprocess

import pytest

import pyoracle as O

_NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


@pytest.fixture(scope="module")
def harness():
    O.build()
    subprocess.run(["make", "-s", "-C", _NATIVE, "float_diff"], check=True)
    return os.path.join(_NATIVE, "float_diff")


@pytest.mark.parametrize("seed", [1, 2])
def test_number_strings_match_oracle(harness, seed):
    r = subprocess.run([harness, "6000", str(seed)], capture_output=True, text=True, timeout=300)
    last = r.stdout.strip().splitlines()[-1]
    assert r.returncode == 0 and last.startswith("checked") and last.endswith("mismatches 0"), r.stdout[-3000:]


def test_hard_numbers_decided_by_exact_path():
    """Documents whose selected values are 16-17-digit floats: the exact host path decides
    them (no UNDECIDED) and equals the oracle; the single-pass path hands them over."""
    import _hosttest as H

    pats = [("v", 1, "0.30000000000000004"), ("w", 1, "1e+21"), ("x", 3, "x"), ("y", 1, "1000000000000000000000")]
    nodes = [(0, -1, -1, i) for i in range(len(pats))] + [(1, 0, 1, -1), (1, 4, 2, -1), (1, 5, 3, -1)]
    root = len(nodes) - 1
    hr = H.HostRuleset(pats, nodes, root)
    ors = O.Ruleset(pats, nodes, root)
    docs = [b'{"v":0.30000000000000004,"w":1e21,"x":["a"],"y":1e21}',
            b'{"v":3.0000000000000004e-1,"w":1.0e21,"y":9.999999999999999e20}',
            b'{"v":0.1,"w":2.2250738585072011e-308,"y":1.7976931348623159e308}']
    for d in docs:
        t, err, res = hr.eval(d)
        assert 3 not in res, (d, res)
        assert res == [ors.pattern(p, d) for p in range(len(pats))], d
        assert t == ors.matches(d)[0]
        tf, _, _ = H.eval_fast(hr, d)
        assert tf == -1 or tf == t
