"""Tie-aware kNN parity checks (SURVEY.md §8(a) parity contract).

Bar: squared distances are bit-identical (so sqrt distances are too); indices
are bit-exact at every rank whose distance is not tied with another candidate;
inside an exact-distance tie group the indices are compared as sets, and at the
k boundary any member of the tied group is accepted (the reference keeps
whichever its traversal met first).  Every returned index is also re-checked
against its own distance with the reference formula
((dx^2 + dy^2) + dz^2 in float32, periodic per-axis min of the three images,
kdtree/src/cpp/include/kdtree/kdtree.hpp:23-31,72-84).
"""
from __future__ import annotations

import numpy as np

PAD = np.uint32(0xFFFFFFFF)


def d2_ref(q, p, boxsize=None):
    """float32 squared distance exactly as the reference computes it (no FMA)."""
    q = np.asarray(q, np.float32)
    p = np.asarray(p, np.float32)
    d = p - q
    if boxsize is not None:
        L = np.float32(boxsize)
        dm = d - L
        dp = d + L
        s = np.minimum(np.minimum(d * d, dm * dm), dp * dp)
    else:
        s = d * d
    return (s[..., 0] + s[..., 1]) + s[..., 2]


def assert_knn_equal(d_got, i_got, d_ref, i_ref, points, queries, boxsize=None, sqrt=True,
                     max_report=5):
    d_got = np.asarray(d_got, np.float32)
    d_ref = np.asarray(d_ref, np.float32)
    i_got = np.asarray(i_got, np.uint32)
    i_ref = np.asarray(i_ref, np.uint32)
    assert d_got.shape == d_ref.shape and i_got.shape == i_ref.shape
    bad = np.nonzero((d_got.view(np.uint32) != d_ref.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, (f"{bad.size} rows with different distances, first rows {bad[:max_report]}:"
                           f"\n got {d_got[bad[:2]]}\n ref {d_ref[bad[:2]]}")
    pts = np.asarray(points, np.float32)
    q = np.asarray(queries, np.float32)
    rows = np.nonzero((i_got != i_ref).any(axis=1))[0]
    k = d_got.shape[1]
    for r in rows:
        dg, ig, ir = d_got[r], i_got[r], i_ref[r]
        valid = ig != PAD
        assert np.array_equal(valid, ir != PAD), f"row {r}: padding differs"
        ids = ig[valid].astype(np.int64)
        assert len(np.unique(ids)) == len(ids), f"row {r}: duplicate indices {ig}"
        dd = d2_ref(q[r], pts[ids], boxsize)
        if sqrt:
            dd = np.sqrt(dd)
        assert np.array_equal(dd.view(np.uint32), dg[valid].view(np.uint32)), (
            f"row {r}: returned indices do not have the returned distances")
        # tie groups strictly inside the row must match as sets
        boundary = dg[k - 1]
        for v in np.unique(dg[valid]):
            sel = dg == v
            if v == boundary:
                continue
            assert set(ig[sel].tolist()) == set(ir[sel].tolist()), (
                f"row {r}: index sets differ at distance {v}: {ig[sel]} vs {ir[sel]}")
    return rows.size  # number of rows where only tie order / boundary choice differed


def check_tree_structure(nodes, x, y, z, idx, n, leaf, n8=None):
    """Structural invariants of a reference-shaped tree (test_builders.cpp:86-139,
    kdtree_impl.hpp:98-146): preorder, left child = id + 1, leaves cover
    [0, n8) in order with sizes % 8 == 0 and <= max(leaf, 16), points of the left
    subtree <= split <= points of the right subtree, idx a permutation."""
    leaf = max(int(leaf), 16)
    n8 = n8 if n8 is not None else (n + 7) // 8 * 8
    assert len(idx) == n8
    assert np.array_equal(np.sort(idx), np.arange(n8, dtype=np.uint32))
    coords = np.stack([x, y, z])
    dims = nodes["dim"]
    # iterative DFS with ranges
    stack = [(0, 0, n8)]
    expect_next_leaf = 0
    order = []
    while stack:
        nid, lo, hi = stack.pop()
        order.append(nid)
        nd = nodes[nid]
        cnt = hi - lo
        if nd["dim"] < 0:
            assert cnt <= leaf and cnt % 8 == 0
            assert nd["left"] == lo and nd["right"] == hi
            assert lo == expect_next_leaf
            expect_next_leaf = hi
            continue
        assert cnt > leaf
        m = (cnt // 2) // 8 * 8
        assert nd["left"] == nid + 1
        d = int(nd["dim"])
        s = nd["split"]
        c = coords[d]
        assert c[lo:lo + m].max() <= s <= c[lo + m:hi].min(), f"node {nid}: split violated"
        assert c[lo + m] == s or np.any(c[lo + m:hi] == s)
        stack.append((int(nd["right"]), lo + m, hi))
        stack.append((int(nd["left"]), lo, lo + m))
    assert expect_next_leaf == n8
    assert order == list(range(len(nodes))), "nodes are not in preorder"
    # the dimension cycles with depth
    return True


def leaf_sets(nodes, idx):
    out = []
    for nd in nodes:
        if nd["dim"] < 0:
            out.append(frozenset(idx[nd["left"]:nd["right"]].tolist()))
    return out
