"""The reference's gjson modifiers (pkg/json/json.go:161-264) on the device's exact path
(authorino_amd/csrc/ajx_modifiers.h, host build) against the oracle (gjson_mods_ref.c):
random documents (strings with escapes and quotes, base64 texts padded / unpadded /
corrupted / with line breaks, numbers, literals, containers, non-ASCII) under random
modifier chains (@extract @replace @case @base64 @strip through '|' or '.'). Each case is
an eq pattern on the oracle's String() (must be T) and one on another value (must be F);
the reference's own expectations are in tests/golden/reference_kats.json."""
import base64
import json
import random

import pytest

import _hosttest as H
import pyoracle as O


def _values(rng):
    raw = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 12)))
    b64 = base64.b64encode(raw).decode()
    v = [
        "John Doe", "a:b:c::d", "x@y.z", "https://github.com/john", "my:ns:sa", "  spaced  out ",
        'with "quotes" and \\ backslash', "tab\there", "line\nbreak", "\x01ctl\x7f", "é ü", "",
        b64, b64.rstrip("="), b64[:-1] + "!" if b64 else "!", b64[:4] + "\n" + b64[4:], "am9obg", "bXkgbmFtZSBpcyAiam9obiI=",
        "Zm9vYmFy", "Zm9v\\YmFy", "====", "a===",
    ]
    return v


def _doc(rng):
    vals = _values(rng)
    pick = rng.choice
    obj = {"s": pick(vals), "t": pick(vals), "n": pick([0, -12, 1.5, 1e21, 0.30000000000000004]),
           "b": pick([True, False, None]), "o": {"k": pick(vals)}, "a": [pick(vals), 1]}
    return json.dumps(obj, ensure_ascii=rng.random() < 0.5).encode()


def _chain(rng):
    mods = []
    for _ in range(rng.randrange(1, 4)):
        k = rng.randrange(6)
        if k == 0:
            arg = rng.choice(['', ':{"sep":":","pos":1}', ':{"sep":"@","pos":0}', ':{"pos":2}', ':{"sep":"/","pos":3}',
                              ':{"sep":"ab","pos":1}', ':{"sep":" ","pos":5}', ':5'])
            mods.append("@extract" + arg)
        elif k == 1:
            mods.append("@replace" + rng.choice(['', ':{"old":"o","new":"0"}', ':{"old":"John","new":"Jane"}',
                                                 ':{"old":"\\"","new":"\'"}', ':{"new":"x","old":":"}']))
        elif k == 2:
            mods.append("@case:" + rng.choice(["upper", "lower", "title"]))
        elif k == 3:
            mods.append("@base64:" + rng.choice(["encode", "decode", "other"]))
        else:
            mods.append("@strip")
    sep = [rng.choice(["|", "."]) for _ in mods]
    base = rng.choice(["s", "t", "n", "b", "o", "a", "o.k", "a.0", "missing"])
    path = base
    for s, m in zip(sep, mods):
        path += s + m
    return path


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_modifier_chains_match_oracle(seed):
    rng = random.Random(900 + seed)
    checked = 0
    for _ in range(250):
        sel = _chain(rng)
        for _ in range(4):
            d = _doc(rng)
            try:
                want = O.gjson_string_mods(d, sel)
            except ValueError:
                break  # a form neither side compiles
            if want is None:
                continue
            w = want.decode("utf-8", "surrogateescape")
            pats = [(sel, 1, want), (sel, 1, want + b"?")]
            nodes = [(0, -1, -1, 0), (0, -1, -1, 1), (1, 0, 1, -1)]
            hr = H.HostRuleset(pats, nodes, 2)
            assert hr.status == [0, 0], (sel, hr.status)
            t, _, res = hr.eval(d)
            assert res == [1, 0], (sel, d, w, res)  # (decided: no reason for UNDECIDED here)
            checked += 1
    assert checked > 300, checked


def _check_select(hr, p, d, want, text):
    rc, out, used = hr.select_value(p, d, text, 0)
    if rc != 0:
        return False
    st, ln, tt = out
    src = bytes(text) if (tt >> 8) & 4 else d  # (AUTHJX_VALUE_TEXT: the request's text slot)
    t, raw = want
    assert (tt & 0xFF, src[st:st + ln]) == (t, raw), (d, out)
    return True


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_select_value_text_matches_oracle(seed):
    """The select kernel's value of a modifier-chain selector (select_value, host build):
    the final Result's type and raw text, copied into the request's text slot, equal the
    oracle's gjson.Get with the same modifiers (json.go:96-151 ReplaceJSONPlaceholders)."""
    rng = random.Random(1900 + seed)
    checked = 0
    for _ in range(200):
        sel = _chain(rng)
        hr = None
        for _ in range(3):
            d = _doc(rng)
            try:
                want = O.gjson_get_mods(d, sel)
            except ValueError:
                break
            if hr is None:
                hr = H.HostRuleset([(sel, 1, "")], [(0, -1, -1, 0)], 0)
                assert hr.status == [0], sel
            if want is None:
                continue
            assert _check_select(hr, 0, d, want, bytearray(4096)), ("undecided", sel, d)
            checked += 1
    assert checked > 300, checked


def test_select_value_lists_and_slot_overflow():
    """"#." lists as built text; several built values share one slot (offsets advance);
    a value larger than what is left of the slot is undecided."""
    d = b'{"a":[{"k":"x"},{"k":2},{"j":1},{"k":[1,{"z":"q"}]}],"s":"abc","e":[]}'
    pats = [("a.#.k", 1, ""), ("s|@case:upper", 1, ""), ("e.#.k", 1, ""), ("s", 1, "")]
    hr = H.HostRuleset(pats, [(0, -1, -1, i) for i in range(4)] + [(1, 0, 1, -1), (1, 4, 2, -1), (1, 5, 3, -1)], 6)
    text = bytearray(64)
    used = 0
    got = []
    for p, (sel, _, _) in enumerate(pats):
        rc, out, used = hr.select_value(p, d, text, used)
        assert rc == 0
        got.append(out)
        st, ln, tt = out
        src = bytes(text) if (tt >> 8) & 4 else d
        t, raw, _ = O.gjson_get(d, sel) if "@" not in sel else (*O.gjson_get_mods(d, sel), None)
        assert (tt & 0xFF, src[st:st + ln]) == (t, raw), sel
    assert got[1][0] == got[0][1] and got[3][2] >> 8 == 0  # (the second built value follows the first)
    small = bytearray(8)
    rc, _, _ = hr.select_value(0, d, small, 0)
    assert rc == -1
