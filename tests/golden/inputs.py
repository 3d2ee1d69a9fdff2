"""Deterministic inputs for the golden fixtures (shared by gen_golden.py and tests).

Seeds follow SURVEY.md §4/§8(d): the reference pytest uses PCG64(42)
(kdtree/tests/test_kdtree.py:7,22); synthetic runs use 20261015 (points) and
20261016 (queries).
"""
from __future__ import annotations

import hashlib

import numpy as np


def sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(str(a.dtype).encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def uniform(n, seed, L=1.0):
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.uniform(0, L, size=(n, 3)).astype(np.float32)


def g1_inputs():
    """test_kdtree_basic: float64 points (cast to f32 by the binding), no box."""
    rng = np.random.Generator(np.random.PCG64(42))
    points = rng.uniform(0, 1, size=(10000, 3))
    query = rng.uniform(0, 1, size=(200, 3))
    return points, query, None


def g2_inputs():
    """test_kdtree_periodic: float32 points, boxsize 2.0."""
    rng = np.random.Generator(np.random.PCG64(42))
    boxsize = 2.0
    points = rng.uniform(0, boxsize, size=(10000, 3)).astype(np.float32)
    query = rng.uniform(0, boxsize, size=(200, 3)).astype(np.float32)
    return points, query, boxsize


def g3_inputs():
    return uniform(100_000, 20261015), uniform(1000, 20261016)


def g4_inputs():
    pts = uniform(1_000_000, 20261015)
    q = np.concatenate([uniform(1000, 20261016), pts[:1000]], axis=0)
    return pts, q


def g5_inputs():
    out = {}
    for n in (8, 13, 17, 129, 1000, 100_000):
        pts = uniform(n, 1000 + n)
        for leaf in (1, 16, 64, 128):
            out[f"n{n}_leaf{leaf}"] = (pts, leaf, None)
    pts = uniform(100_000, 7, L=2.0)
    out["n100000_leaf32_periodic"] = (pts, 32, 2.0)
    return out


def tie_free(n, seed, L=1.0):
    """n points whose coordinates are distinct on every axis (each axis a random
    sample without replacement of the 2^24 f32 values k / 2^24 * L), so no
    split value is tied and the node table is a pure function of the points,
    whatever partition the build runs (G7)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.empty((n, 3), np.float32)
    for a in range(3):
        out[:, a] = (rng.choice(1 << 24, size=n, replace=False).astype(np.float64)
                     * (L / float(1 << 24))).astype(np.float32)
    return out


def g7_inputs():
    """Node tables at scale: name -> (points, leafsize,
    boxsize, tie_free).  Tie-free sets must match the reference bit for bit;
    the plain uniform 1e7 set (the bench generator's seed; ~8.3e6 distinct x
    values, so split values are tied) is compared for shape and agreement."""
    return {
        "tiefree_1e6_leaf64_periodic": (lambda: tie_free(1_000_000, 70), 64, 1.0, True),
        "tiefree_1e6_leaf32": (lambda: tie_free(1_000_000, 71), 32, None, True),
        "tiefree_1e7_leaf64_periodic": (lambda: tie_free(10_000_000, 72), 64, 1.0, True),
        "uniform_1e7_leaf64_periodic": (lambda: uniform(10_000_000, 20261015), 64, 1.0, False),
    }


def node_shape(nodes):
    """(dim, left, right) of every node: the tree's shape, which depends only on
    (n8, leafsize) (dims cycle x, y, z: kdtree_impl.hpp:149-169)."""
    v = np.ascontiguousarray(nodes).view(np.uint32).reshape(-1, 4)
    return np.ascontiguousarray(v[:, [0, 2, 3]])


def edge_cases():
    """name -> (points, queries, k, leafsize, boxsize)"""
    out = {}
    pts = uniform(13, 5)
    q = uniform(7, 6)
    out["k_gt_n"] = (pts, q, 20, 16, None)  # k > n: padding rows (FLT_MAX, 0xFFFFFFFF)
    # points exactly at 0 and at L, periodic; queries outside [0, L] (not validated)
    L = 1.0
    pts = uniform(200, 8)
    pts[:8] = np.array([[0, 0, 0], [L, L, L], [0, L, 0], [L, 0, L], [0.5, 0, L], [0, 0.5, 0.5],
                        [L, 0.25, 0], [0.75, L, 0]], np.float32)
    q = np.concatenate([uniform(20, 9), np.array([[1.2, -0.1, 0.5], [-0.3, 1.4, 1.0],
                                                  [0.0, 0.0, 0.0], [1.0, 1.0, 1.0]],
                                                 np.float32)])
    out["box_faces"] = (pts, q, 6, 16, L)
    # duplicate points (forced exact ties)
    base = uniform(50, 10)
    pts = np.concatenate([base, base, base[:10]], axis=0)
    out["duplicates"] = (pts, uniform(30, 11), 5, 16, None)
    # fortran-ordered float64 input (the binding forcecasts)
    f = np.asfortranarray(np.random.Generator(np.random.PCG64(12)).uniform(0, 1, (3000, 3)))
    out["fortran_f64"] = (f, uniform(40, 13), 3, 64, None)
    # k = 1
    out["k1"] = (uniform(5000, 14), uniform(100, 15), 1, 128, 1.0)
    # a single point
    out["single"] = (np.array([[0.25, 0.5, 0.75]], np.float32), uniform(5, 16), 2, 128, 1.0)
    return out
