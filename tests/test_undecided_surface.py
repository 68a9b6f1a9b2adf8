"""The UNDECIDED surface on a realistic selector mix (tests/undecided_mix.py: every
selector of the reference's user guides, on Authorization-JSON documents shaped like the
reference's), host build of the device logic (ajx_device.h / ajx_modifiers.h) against
the oracle: every doc selector compiles, no request is UNDECIDED on ASCII documents, and
the forms left UNSUPPORTED are exactly the by-design list
(tests/test_gpu_undecided.py runs the same through the kernels)."""
import random

import _hosttest as H
import pyoracle as O
import undecided_mix as M


def test_doc_selectors_compile_and_by_design_forms_do_not():
    for s in M.DOC_SELECTORS:
        assert H.HostRuleset([(s, 1, "x")], [(0, -1, -1, 0)], 0).status == [0], s
    for s in M.BY_DESIGN_UNSUPPORTED:
        assert H.HostRuleset([(s, 1, "x")], [(0, -1, -1, 0)], 0).status == [2], s


def test_no_undecided_on_the_reference_selector_mix():
    rng = random.Random(8)
    docs = [M.make_doc(rng) for _ in range(150)]
    n = 0
    for pats, nodes, root in M.make_rulesets(rng, docs, k=10):
        hr = H.HostRuleset(pats, nodes, root)
        rs = O.Ruleset(pats, nodes, root)
        assert hr.status == [0] * len(pats)
        for d in docs:
            t, _, res = hr.eval(d)
            assert 3 not in res and t != 3, (pats, d)
            assert res == [rs.pattern(p, d) for p in range(len(pats))]
            assert t == rs.matches(d)[0]
            n += 1
    assert n == 1500
