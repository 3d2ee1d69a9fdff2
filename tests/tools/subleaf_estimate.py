"""Estimate for the radius count's next lever: how many
(query, point) pairs fall in partially covered boxes at leaf granularity
versus 8-point groups (each leaf's points ordered by a two-level median split
on the widest axis, each group with its own tight box).  Test
infrastructure: it reads the C oracle's tree (test-only) on the C3 geometry at
a smaller N (r scaled by (1e8 / N)^(1/3)).

    python tests/tools/subleaf_estimate.py --n 1e6 --queries 300
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
ap.add_argument("--queries", type=int, default=300)
a = ap.parse_args()
n, L = int(a.n), 1.0
r = 0.01 * (1e8 / n) ** (1 / 3)
pts = synth.uniform(n)
nodes, x, y, z, _ = Oracle().tree(pts, 32, L).export()
leaves = nodes[nodes["dim"] == -1]
P = np.stack([x, y, z], 1).astype(np.float64)


def real(q):
    return q[(np.abs(q) < 1e30).all(1)]


lbox, groups = [], []
for s, e in zip(leaves["left"].astype(np.int64), leaves["right"].astype(np.int64)):
    q = real(P[s:e])
    lbox.append((q.min(0), q.max(0), len(q)))
    ax = np.argmax(q.max(0) - q.min(0))
    q = q[np.argsort(q[:, ax], kind="stable")]
    h = len(q) // 2
    for half in (q[:h], q[h:]):
        ax2 = np.argmax(half.max(0) - half.min(0))
        half = half[np.argsort(half[:, ax2], kind="stable")]
        hh = len(half) // 2
        groups += [half[:hh], half[hh:]]


def boxes(bs):
    return (np.array([b[0] for b in bs]), np.array([b[1] for b in bs]),
            np.array([b[2] for b in bs]))


def cost(lo, hi, c, qs):
    part = full = 0.0
    for qv in qs:
        d = np.abs(np.stack([lo - qv, hi - qv]))
        lb = np.where((qv >= lo) & (qv <= hi), 0.0, np.minimum(d, L - d).min(0))
        ub = np.minimum(d.max(0), L / 2)
        need = (lb ** 2).sum(1) <= r * r
        whole = need & ((ub ** 2).sum(1) <= r * r)
        part += c[need & ~whole].sum()
        full += c[whole].sum()
    return part / len(qs), full / len(qs)


qs = pts[np.random.default_rng(1).choice(n, a.queries, replace=False)].astype(np.float64)
gb = boxes([(g.min(0), g.max(0), len(g)) for g in groups if len(g)])
for name, (lo, hi, c) in (("leaf (32)", boxes(lbox)), ("group (8)", gb)):
    p, f = cost(lo, hi, c, qs)
    print(f"{name:10s} points evaluated/query {p:8.1f}   counted whole/query {f:7.1f}")
