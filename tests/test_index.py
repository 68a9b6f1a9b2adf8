"""Host AuthConfig index (authorino_amd/index.py) against the reference's own test,
pkg/index/index_test.go:38-140 (TestAuthConfigTree), plus the `:port` retry of
pkg/service/auth.go:270-280 and wildcard climbing from deeper keys."""
import numpy as np

from authorino_amd import index as ix


def test_auth_config_tree():
    """index_test.go:38-140, step by step (configs are plain markers here)"""
    c = ix.Index()
    ac1, ac2, ac3, ac4 = "cfg-1", "cfg-2", "cfg-3", "cfg-4"
    assert c.set("auth-1", "*.io", ac1, False) is None  # the more generic host first
    assert c.set("auth-2", "talker-api.nip.io", ac2, False) is None  # ...then the more specific one
    assert c.set("auth-2", "*.pets.com", ac2, False) is None
    assert c.set("auth-3", "api.acme.com", ac3, False) is None  # the more specific host first
    assert c.set("auth-4", "*.acme.com", ac4, False) is None  # ...then the more generic one

    assert sorted(c.find_keys("auth-1")) == ["*.io"]
    assert sorted(c.find_keys("auth-2")) == ["*.pets.com", "talker-api.nip.io"]
    assert c.find_keys("auth-x") is None

    assert c.find_id("*.pets.com") == ("auth-2", True)
    assert c.find_id("talker-api.nip.io") == ("auth-2", True)
    assert c.find_id("*.acme.com") == ("auth-4", True)
    assert c.find_id("undefined.com") == ("", False)

    err = c.set("auth-5", "talker-api.nip.io", "cfg-5", False)  # same host, no override
    assert isinstance(err, ix.AlreadyExistsError)
    # (treeNode.set formats the reverted key it was handed, index.go:71,184)
    assert str(err) == "authconfig already exists in the index: .io.nip.talker-api"

    assert c.get("dogs.pets.com") == ac2
    assert c.get("api.acme.com") == ac3
    assert c.get("www.acme.com") == ac4
    assert c.get("talker-api.nip.io") == ac2
    assert c.get("foo.nip.io") == ac1
    assert c.get("foo.org") is None

    c.delete("auth-2")  # all entries of the id go
    assert c.get("dogs.pets.com") is None
    assert c.get("talker-api.nip.io") == ac1  # `*.io <- auth-1` is still in the tree
    assert c.get("api.acme.com") == ac3

    c.delete("auth-3")
    assert c.get("api.acme.com") == ac4  # `*.acme.com <- auth-4` is still in the tree


def test_override_list_and_empty():
    c = ix.Index()
    assert c.empty()
    assert c.set("a", "x.example.com", 1) is None
    assert c.set("b", "x.example.com", 2, True) is None  # override replaces the entry
    assert c.get("x.example.com") == 2
    assert sorted(c.list()) == [2]
    assert not c.empty()
    c.delete_key("a", "x.example.com")  # not a's entry any more: stays
    assert c.get("x.example.com") == 2
    c.delete_key("b", "x.example.com")
    assert c.get("x.example.com") is None


def test_wildcard_climbs_from_the_longest_common_path():
    c = ix.Index()
    c.set("root-wild", "*.com", 1)
    c.set("deep", "a.b.example.com", 2)
    c.set("mid-wild", "*.example.com", 3)
    assert c.get("a.b.example.com") == 2
    assert c.get("z.b.example.com") == 3   # b.example.com has no entry: climb to *.example.com
    assert c.get("b.example.com") == 3     # an interior node without entry: climb
    assert c.get("q.other.com") == 1
    assert c.get("example.org") is None
    assert ix.revert_key("talker-api.nip.io") == ".io.nip.talker-api"


def test_port_retry_and_batch_selection():
    """auth.go:270-280: a host with a port is retried without it"""
    c = ix.Index()
    c.set("t1", "t1.example.com", 0)
    c.set("t2", "t2.example.com:8080", 1)  # a key with a port matches only with it
    c.set("w", "*.r0.example.com", 2)
    assert ix.lookup(c, "t1.example.com:443") == 0
    assert ix.lookup(c, "t2.example.com:8080") == 1
    assert ix.lookup(c, "t2.example.com") is None
    assert ix.lookup(c, "api.r0.example.com:443") == 2
    sel = ix.select_sets(c, ["t1.example.com", "x.r0.example.com", "nope.example.net", "t1.example.com:1"])
    assert sel.dtype == np.int64 and sel.tolist() == [0, 2, -1, 0]


def test_c4_workload_selection_and_bucketing():
    """The C4 batch: every request's set id is what the index lookup (with the :port
    retry) gives for its host, unknown hosts are dropped, and the batch is bucketed."""
    from authorino_amd import workloads as W

    idx, exprs = W.c4_index_and_rules(600, 20, seed=4)
    rng = np.random.default_rng(5)
    hosts = W.c4_hosts(3000, 600, 20, rng)
    sel = ix.select_sets(idx, hosts)
    for h, s in zip(hosts, sel):
        if h.startswith("u"):
            assert s == -1
        elif h.startswith("h"):
            assert exprs[s] is exprs[580 + int(h.split(".")[1][1:])]
        else:
            assert s == int(h.split(".")[0][1:])
    w = W.make_c4(2000, seed=9, n_configs=600, n_wild=20)
    assert w.n == 2000 and np.all(np.diff(w.set_of_req.astype(np.int64)) >= 0)
    assert all(8 <= len(e.flatten()[0]) <= 32 for e in w.exprs)
    assert sum(any(p.operator == 5 for p in e.flatten()[0]) for e in w.exprs) > 20


def test_bucket_order_groups_by_config_then_longest_first():
    rng = np.random.default_rng(5)
    sets = rng.integers(0, 50, 5000)
    lens = rng.integers(700, 1400, 5000)
    o = ix.bucket_order(sets, lens)
    assert np.array_equal(np.sort(o), np.arange(5000))
    s, c = sets[o], lens[o] >> 3
    assert (np.diff(s) >= 0).all()
    same = np.diff(s) == 0
    assert (np.diff(c)[same] <= 0).all()


# ---- the native index (authorino_amd/csrc/ajx_index.cpp, authjx_index_*) ----------------

def test_native_index_reference_tree():
    """index_test.go:38-140 on the native tree (entries are ruleset ids)"""
    n = ix.NativeIndex()
    assert n.set("*.io", 1) is None
    assert n.set("talker-api.nip.io", 2) is None
    assert n.set("*.pets.com", 2) is None
    assert n.set("api.acme.com", 3) is None
    assert n.set("*.acme.com", 4) is None
    assert isinstance(n.set("talker-api.nip.io", 5), ix.AlreadyExistsError)
    assert n.get("dogs.pets.com") == 2
    assert n.get("api.acme.com") == 3
    assert n.get("www.acme.com") == 4
    assert n.get("talker-api.nip.io") == 2
    assert n.get("foo.nip.io") == 1
    assert n.get("foo.org") == -1
    n.delete_key("talker-api.nip.io", 2)
    n.delete_key("*.pets.com", 2)
    assert n.get("talker-api.nip.io") == 1  # the wildcard above it now
    assert n.get("dogs.pets.com") == -1
    n.delete_key("*.acme.com", 3)  # not its id: stays
    assert n.get("www.acme.com") == 4
    assert n.set("talker-api.nip.io", 7, override=True) is None
    assert n.get("talker-api.nip.io") == 7
    assert n.get("talker-api.nip.io:8080") == 7  # the ':port' retry (auth.go:270-280)
    assert n.get("api.acme.com:443") == 3


def _rand_host(rng, labels):
    k = int(rng.integers(1, 5))
    return ".".join(labels[int(rng.integers(0, len(labels)))] for _ in range(k))


def test_native_index_matches_restatement():
    """random keys (wildcards, empty labels, overrides, deletes) and hosts (ports):
    the native lookups equal index.lookup on the Python restatement"""
    rng = np.random.default_rng(41)
    labels = ["a", "b", "io", "com", "*", "", "api", "x-1"]
    for _ in range(30):
        py, nat = ix.Index(), ix.NativeIndex()
        keys = []
        for j in range(int(rng.integers(1, 40))):
            key = _rand_host(rng, labels)
            ov = bool(rng.random() < 0.3)
            e1 = py.set("id%d" % j, key, j, ov)
            e2 = nat.set(key, j, ov)
            assert (e1 is None) == (e2 is None), key
            keys.append((key, j))
        for key, j in keys[: int(rng.integers(0, len(keys) + 1))]:
            if rng.random() < 0.3:
                py.delete_key("id%d" % j, key)
                nat.delete_key(key, j)
        hosts = [_rand_host(rng, labels) + (":%d" % rng.integers(1, 9999) if rng.random() < 0.3 else "")
                 for _ in range(300)]
        want = [ix.lookup(py, h) for h in hosts]
        want = np.array([-1 if w is None else w for w in want], dtype=np.int32)
        assert [nat.get(h) for h in hosts] == list(want)
        a, o, ln = ix.pack_hosts(hosts)
        for nt in (1, 3):
            assert np.array_equal(nat.lookup_batch(a, o, ln, n_threads=nt), want)


def test_native_index_batch_c4_hosts():
    """the C4 host population (10k tenants + wildcards, Zipf traffic): the batched native
    lookup equals the restatement's select_sets"""
    from authorino_amd import workloads as W

    index, nat = ix.Index(), ix.NativeIndex()
    for key, sid in W.c4_index_entries(n_configs=2000, n_wild=50):
        assert index.set("ns/cfg-%d" % sid, key, sid, False) is None
        assert nat.set(key, sid) is None
    hosts = W.c4_hosts(20000, 2000, 50, np.random.default_rng(5))
    a, o, ln = ix.pack_hosts(hosts)
    got = nat.lookup_batch(a, o, ln, n_threads=4)
    assert np.array_equal(got, ix.select_sets(index, hosts).astype(np.int32))
