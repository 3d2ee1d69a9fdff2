"""Estimate for the kNN collect kernel's sub-leaf groups: the
(query, point) pairs a packet walk evaluates when its need test runs per leaf
versus per 8-point group (each leaf's points ordered by median splits on the
widest axis into groups of 8, each group with its own tight box), for
leafsize 32 and 64 trees.  The ball of a query is its exact k-th distance
times `--slack` (the collect kernel's bound starts at the seed and tightens
towards it).  Test infrastructure: reads the C oracle's tree.

    python tests/tools/knn_group_estimate.py --n 1e6 --queries 2000 --k 32
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nbodyhpc_amd import synth  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=float, default=1e6)
ap.add_argument("--queries", type=int, default=2000)
ap.add_argument("--k", type=int, default=32)
ap.add_argument("--slack", type=float, default=1.15)
ap.add_argument("--group", type=int, default=8)
a = ap.parse_args()
n, L = int(a.n), 1.0
GSIZE = a.group
pts = synth.uniform(n)
orc = Oracle()


def groups_of(q, size=GSIZE):
    if len(q) <= size:
        return [q]
    ax = np.argmax(q.max(0) - q.min(0))
    q = q[np.argsort(q[:, ax], kind="stable")]
    h = (len(q) // 2) // size * size
    return groups_of(q[:h], size) + groups_of(q[h:], size)


def boxes(t):
    nodes, x, y, z, _ = t.export()
    leaves = nodes[nodes["dim"] == -1]
    P = np.stack([x, y, z], 1).astype(np.float64)
    lb, gb = [], []
    for s, e in zip(leaves["left"].astype(np.int64), leaves["right"].astype(np.int64)):
        q = P[s:e]
        q = q[(np.abs(q) < 1e30).all(1)]
        if not len(q):
            continue
        lb.append((q.min(0), q.max(0), len(q)))
        gb += [(g.min(0), g.max(0), len(g)) for g in groups_of(q)]
    f = lambda bs: (np.array([b[0] for b in bs]), np.array([b[1] for b in bs]),  # noqa: E731
                    np.array([b[2] for b in bs]))
    return f(lb), f(gb)


def evals(lo, hi, c, qs, rad):
    tot, nbox = 0.0, 0.0
    for qv, r in zip(qs, rad):
        d = np.abs(np.stack([lo - qv, hi - qv]))
        lb = np.where((qv >= lo) & (qv <= hi), 0.0, np.minimum(d, L - d).min(0))
        need = (lb ** 2).sum(1) <= r * r
        tot += c[need].sum()
        nbox += need.sum()
    return tot / len(qs), nbox / len(qs)


sel = np.random.default_rng(1).choice(n, a.queries, replace=False)
qs = pts[sel].astype(np.float64)
for leaf in (32, 64):
    t = orc.tree(pts, leaf, L)
    d, _ = t.query(pts[sel], a.k, workers=8)
    rad = d[:, -1].astype(np.float64) * a.slack
    (llo, lhi, lc), (glo, ghi, gc) = boxes(t)
    pl, nl = evals(llo, lhi, lc, qs, rad)
    pg, ng = evals(glo, ghi, gc, qs, rad)
    print(f"leafsize {leaf}: per query  leaf test: {pl:6.1f} points in {nl:5.1f} leaves   "
          f"group test: {pg:6.1f} points in {ng:5.1f} groups")
