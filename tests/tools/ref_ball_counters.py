"""Per-query traversal counters of a one-query-at-a-time radius DFS (the C
oracle's orc_ball_count_stats: same pruning as the reference's kNN DFS,
kdtree_impl.hpp:226-268, with the fixed bound r^2), which SURVEY.md §8(d) prices
the radius query with: B_r = 16 N + 12 P + 12 + 4.

Config C3 (1e8 uniform periodic, r = 0.01 L, leafsize 32) is reproduced at a
smaller N with r scaled by (1e8 / N)^(-1/3) (same mean count, same leaf-to-ball
geometry):  python tests/tools/ref_ball_counters.py --n 1e7 --queries 100000
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nbodyhpc_amd import synth  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=float, default=1e7)
ap.add_argument("--queries", type=int, default=100_000)
ap.add_argument("--r", type=float, default=0.01, help="radius at 1e8 points")
a = ap.parse_args()
n = int(a.n)
r = a.r * (1e8 / n) ** (1.0 / 3.0)
pts = synth.uniform(n)
orc = Oracle()
t = orc.tree(pts, 32, 1.0)
c, nodes, points = orc.ball_count_stats(t, pts[:a.queries], r)
m = a.queries
N, P = nodes / m, points / m
print(f"n={n:.0e} r={r:.5f} mean_count={c.mean():.2f} nodes/query={N:.2f} "
      f"points/query={P:.2f} B_r={16 * N + 12 * P + 16:.1f}")
