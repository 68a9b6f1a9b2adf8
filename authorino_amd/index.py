"""Host-side AuthConfig index: per-request AuthConfig selection for multi-tenant batches
(SURVEY.md §8 a15, config C4).

Restates pkg/index/index.go (the `Index` interface :16-27 and its radix tree :37-243)
and the `:port` retry of pkg/service/auth.go:270-289. Selection stays on the host, as in
the reference: the micro-batcher resolves each request's host to an AuthConfig id, and
the device batch carries that id as `set_of_req` (include/authjx.h).

Keys are hostnames. Each '.' starts a new tree level, read from the TLD down
(`revertKey`, index.go:236-243). A `*` label matches any host below the longest common
path between the searched key and the tree; the search climbs from that node to the
root, taking the first `*` child that holds an entry (`treeNode.get`, index.go:153-174).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np

KEY_LABELS_SEPARATOR = "."  # index.go:11
ROOT_KEY_LABEL = ""          # index.go:12


class AlreadyExistsError(Exception):
    """the error `Set` returns for a taken key without override (index.go:180-182)"""


class IndexEntry:
    """index.go:32-35"""
    __slots__ = ("id", "auth_config")

    def __init__(self, id: str, auth_config):
        self.id = id
        self.auth_config = auth_config


class _TreeNode:
    """index.go:138-151"""
    __slots__ = ("label", "entry", "parent", "children")

    def __init__(self, label: str, parent: Optional["_TreeNode"]):
        self.label = label
        self.entry: Optional[IndexEntry] = None
        self.parent = parent
        self.children: Dict[str, _TreeNode] = {}

    def longest_common_label(self, key: str) -> Tuple["_TreeNode", str]:
        """index.go:205-223, iteratively: the deepest node on the key's path, and the
        labels of the key below it ("" when the key ends at that node)."""
        labels = key.split(KEY_LABELS_SEPARATOR)
        if self.label != labels[0]:
            raise RuntimeError("cannot traverse index tree")  # index.go:208-213 (a panic there)
        node, i = self, 0
        while i + 1 < len(labels):
            child = node.children.get(labels[i + 1])
            if child is None:
                break
            node, i = child, i + 1
        return node, KEY_LABELS_SEPARATOR.join(labels[i + 1:])

    def get(self, key: str) -> Optional[IndexEntry]:
        """index.go:153-174"""
        node, tail = self.longest_common_label(key)
        if tail == "" and node.entry is not None:  # the longest common node matches the key
            return node.entry
        curr = node  # look upwards until the root for a wildcard
        while True:
            child = curr.children.get("*")
            if child is not None and child.entry is not None:
                return child.entry
            if curr.parent is None:
                break
            curr = curr.parent
        return None

    def set(self, key: str, entry: IndexEntry, override: bool) -> Optional[Exception]:
        """index.go:176-203"""
        target, tail = self.longest_common_label(key)
        if tail == "":
            if not override:
                return AlreadyExistsError("authconfig already exists in the index: %s" % key)
            target.entry = entry
            return None
        labels = tail.split(KEY_LABELS_SEPARATOR)
        node = _TreeNode(labels[0], target)
        curr = node
        for label in labels[1:]:
            curr.children[label] = _TreeNode(label, curr)
            curr = curr.children[label]
        curr.entry = entry
        target.children[labels[0]] = node
        return None

    def list(self) -> List[IndexEntry]:
        """index.go:225-234"""
        out, stack = [], [self]
        while stack:
            n = stack.pop()
            if n.entry is not None:
                out.append(n.entry)
            stack.extend(reversed(list(n.children.values())))
        return out


def revert_key(key: str) -> str:
    """index.go:236-243: "talker-api.nip.io" -> ".io.nip.talker-api" (root label first)"""
    labels = key.split(KEY_LABELS_SEPARATOR) + [ROOT_KEY_LABEL]
    return KEY_LABELS_SEPARATOR.join(reversed(labels))


class Index:
    """`index.NewIndex()` (index.go:28-30): the AuthConfig tree (authConfigTree, :37-136).
    Errors are returned, as the Go methods do, rather than raised."""

    def __init__(self):
        self._root = _TreeNode(ROOT_KEY_LABEL, None)
        self._keys: Dict[str, List[str]] = {}

    def get(self, key: str):
        """index.go:56-65: the AuthConfig for a host, or None"""
        e = self._root.get(revert_key(key))
        return e.auth_config if e is not None else None

    def set(self, id: str, key: str, config, override: bool = False) -> Optional[Exception]:
        """index.go:67-80"""
        err = self._root.set(revert_key(key), IndexEntry(id, config), override)
        if err is None:
            self._keys.setdefault(id, []).append(key)
        return err

    def delete(self, id: str) -> None:
        """index.go:82-91"""
        for key in self._keys.get(id, []):
            self._delete_key(id, key)

    def delete_key(self, id: str, key: str) -> None:
        """index.go:93-98"""
        self._delete_key(id, key)

    def list(self) -> list:
        """index.go:100-109"""
        return [e.auth_config for e in self._root.list()]

    def empty(self) -> bool:
        """index.go:111-113"""
        return len(self._keys) == 0

    def find_id(self, key: str) -> Tuple[str, bool]:
        """index.go:115-123"""
        e = self._root.get(revert_key(key))
        return (e.id, True) if e is not None else ("", False)

    def find_keys(self, id: str) -> Optional[List[str]]:
        """index.go:125-130"""
        return self._keys.get(id)

    def _delete_key(self, id: str, key: str) -> None:
        """index.go:132-136 (the keys map keeps the id, as in the reference)"""
        node, _ = self._root.longest_common_label(revert_key(key))
        if node is not None and node.entry is not None and node.entry.id == id:
            node.entry = None


def lookup(index: Index, host: str):
    """pkg/service/auth.go:270-280: Index.Get(host); when not found and the host has a
    port, retry with the part before the first ':'"""
    cfg = index.get(host)
    if cfg is None and ":" in host:
        cfg = index.get(host.split(":")[0])
    return cfg


def select_sets(index: Index, hosts: Iterable[str], not_found: int = -1) -> np.ndarray:
    """The micro-batcher's selection step for a batch: `lookup` per request, each distinct
    host resolved once. The index's configs are set ids (ints) here; requests whose host
    resolves to nothing get `not_found` (the reference answers NOT_FOUND, auth.go:282-287,
    without evaluating anything)."""
    memo: Dict[str, int] = {}
    hosts = list(hosts)
    out = np.empty(len(hosts), dtype=np.int64)
    for i, h in enumerate(hosts):
        v = memo.get(h)
        if v is None:
            cfg = lookup(index, h)
            v = memo[h] = not_found if cfg is None else int(cfg)
        out[i] = v
    return out


class NativeIndex:
    """The same tree in libauthjx.so (authorino_amd/csrc/ajx_index.cpp, include/authjx.h
    authjx_index_*): entries are ruleset ids; `lookup_batch` resolves a micro-batch of
    hosts (with the ':port' retry) on all host threads — the batched host lookup of
    SURVEY.md §8 f4 (pkg/index/index.go:153-174, pkg/service/auth.go:270-289)."""

    def __init__(self):
        from . import runtime

        self._L = runtime.load_library()
        h = C.c_void_p()
        rc = self._L.authjx_index_new(C.byref(h))
        if rc != 0:
            raise MemoryError("authjx_index_new: %d" % rc)
        self._h = h

    def close(self):
        if self._h:
            self._L.authjx_index_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set(self, key: str, set_id: int, override: bool = False) -> Optional[Exception]:
        """index.go:67-80 (the entry is the ruleset id)"""
        b = key.encode("utf-8")
        rc = self._L.authjx_index_set(self._h, b, len(b), int(set_id), 1 if override else 0)
        if rc == -7:
            return AlreadyExistsError("authconfig already exists in the index: %s" % key)
        if rc != 0:
            raise ValueError("authjx_index_set: %d" % rc)
        return None

    def delete_key(self, key: str, set_id: int) -> None:
        """index.go:93-98"""
        b = key.encode("utf-8")
        self._L.authjx_index_delete_key(self._h, b, len(b), int(set_id))

    def get(self, host: str) -> int:
        """`lookup` (Index.Get + the ':port' retry): the ruleset id, -1 when none"""
        b = host.encode("utf-8")
        out = C.c_int32(-1)
        self._L.authjx_index_get(self._h, b, len(b), C.byref(out))
        return out.value

    def lookup_batch(self, arena: np.ndarray, offs: np.ndarray, lens: np.ndarray, n_threads: int = 0) -> np.ndarray:
        """host r = arena[offs[r] : offs[r] + lens[r]] -> ruleset id (-1: none)"""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        out = np.empty(len(lens), dtype=np.int32)
        rc = self._L.authjx_index_lookup_batch(self._h, arena.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                               len(lens), out.ctypes.data, int(n_threads))
        if rc != 0:
            raise ValueError("authjx_index_lookup_batch: %d" % rc)
        return out


def pack_hosts(hosts: Iterable[str]):
    """hosts -> (arena u8, offs u64, lens u32), the layout lookup_batch takes"""
    bs = [h.encode("utf-8") for h in hosts]
    lens = np.fromiter((len(b) for b in bs), dtype=np.uint32, count=len(bs))
    offs = np.zeros(len(bs), dtype=np.uint64)
    if len(bs) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = np.frombuffer(b"".join(bs), dtype=np.uint8) if bs else np.zeros(0, np.uint8)
    return arena, offs, lens


def bucket_order(sets: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """The micro-batcher's bucketing of a multi-tenant batch: the permutation that groups
    requests by AuthConfig (set id ascending) and, inside a bucket, by 8-byte document
    length class, longest first. The first key lets a workgroup of the single-pass kernel
    stage one ruleset in LDS; the second gives a wave's lanes similar token loads, as the
    device length sort does for uniform batches (c4: 10.0 -> 7.7 ms per 2 M requests)."""
    sets = np.asarray(sets, dtype=np.int64)
    cls = np.asarray(lens, dtype=np.int64) >> 3
    return np.lexsort((-cls, sets))
