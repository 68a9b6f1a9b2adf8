"""The value checkers of the device parity tests catch a one-byte truncation: the host build
of the select code (tests/native/host_eval.cpp, ht_inject_truncate) drops the last byte of
every built text value, as a kernel bug would, and the same checks the GPU tests run
(tests/test_gpu_select_text.py, and the host tests test_unicode_case / test_fromstr /
test_modifiers) must then fail; without the injection they pass on the same inputs."""
import collections
import random

import numpy as np
import pytest

import _hosttest as H
import pyoracle as O


@pytest.fixture
def truncate():
    H.lib().ht_inject_truncate(1)
    yield
    H.lib().ht_inject_truncate(0)


def _host_select(paths, docs, stride):
    """vals / text arrays in the device entry point's layout (authjx_select_text_batch):
    values of one request in slot order, built text appended to its text slot."""
    hrs = [H.HostRuleset([(p, 1, "")], [(0, -1, -1, 0)], 0) for p in paths]
    vals = np.zeros((len(docs), len(paths), 3), dtype=np.uint32)
    text = np.zeros((len(docs), stride), dtype=np.uint8)
    for k, d in enumerate(docs):
        slot = bytearray(stride)
        used = 0
        for j, hr in enumerate(hrs):
            rc, out, used = hr.select_value(0, d, slot, used)
            vals[k, j] = out if rc == 0 else (0, 0, 255)
        text[k] = np.frombuffer(bytes(slot), dtype=np.uint8)
    return vals, text


def _unicode_case(n):
    from test_gpu_select_text import UNICODE_PATHS, check_unicode_values
    from test_unicode_case import _raw_string

    rng = random.Random(6200)
    raws = [_raw_string(rng) for _ in range(n)]
    vals, text = _host_select(UNICODE_PATHS, [b'{"s":' + r + b',"n":1}' for r in raws], 2048)
    return check_unicode_values(vals, text, raws)


def _fromstr(n):
    from test_fromstr import PATHS, _fromstr_doc
    from test_gpu_select_text import _check_request

    rng = random.Random(99)
    docs = [_fromstr_doc(rng) for _ in range(n)]
    vals, text = _host_select(PATHS, docs, 8192)
    counts = collections.Counter()
    for k, d in enumerate(docs):
        _check_request(vals, text, k, d, [O.gjson_get_mods(d, p) for p in PATHS], 8192, counts)
    return counts


def test_device_checkers_pass_on_the_exact_code():
    assert _unicode_case(300)["decided"] > 500
    assert _fromstr(100)["checked"] > 800


def test_device_checkers_catch_a_truncated_value(truncate):
    with pytest.raises(AssertionError):
        _unicode_case(300)
    with pytest.raises(AssertionError):
        _fromstr(100)


def test_host_tests_catch_a_truncated_value(truncate):
    from test_fromstr import test_fromstr_and_tails_match_oracle
    from test_modifiers import test_select_value_text_matches_oracle
    from test_unicode_case import test_case_and_strip_on_unicode_match_go

    for t in (test_case_and_strip_on_unicode_match_go, test_fromstr_and_tails_match_oracle,
              test_select_value_text_matches_oracle):
        with pytest.raises(AssertionError):
            t(0)
