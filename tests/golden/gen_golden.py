"""Generate the committed golden fixtures under tests/golden/.

Runs ONLY in the build container, where /root/reference exists: the expected
outputs come from the reference's own C++ (oracle/_ref/libnbkd_ref.so, built
from /root/reference by oracle/Makefile) and, for the reference pytest cases,
also from scipy.spatial.KDTree — the reference's own test oracle
(kdtree/tests/test_kdtree.py:6-35).  Inputs are regenerated from numpy seeds
at test time; each fixture stores a SHA-256 of its inputs so a drift in the
generator is caught.

    PYTHONPATH=. python tests/golden/gen_golden.py [--only g7]
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np
import scipy.spatial

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.oracle import Reference  # noqa: E402
from tests.golden.inputs import (edge_cases, g1_inputs, g2_inputs, g3_inputs, g4_inputs,  # noqa: E402
                                 g5_inputs, g7_inputs, node_shape, sha)

OUT = os.path.dirname(os.path.abspath(__file__))


def g7(R):
    """G7: node tables at 1e6-1e7 (gen_golden.py --only g7).  Tie-free sets: the
    SHA-256 of the reference's whole node table.  The uniform 1e7 set (ties at
    split values): the SHA of its shape (dim, left, right) and its split values,
    so a test can measure how many nodes agree."""
    from oracle.oracle import Oracle
    O = Oracle()
    out = {}
    for key, (gen, leaf, box, tie_free) in g7_inputs().items():
        pts = gen()
        t = R.tree(pts, leaf, box)
        nodes, x, y, z, idx = t.export()
        out["sha_" + key] = np.array(sha(pts))
        out["n8_" + key] = np.array(t.n)
        out["nnodes_" + key] = np.array(t.size)
        out["table_sha_" + key] = np.array(sha(nodes.view(np.uint32).reshape(-1, 4)))
        out["shape_sha_" + key] = np.array(sha(node_shape(nodes)))
        on = O.tree(pts, leaf, box).export()[0]
        agree = float(np.mean(on["split"].view(np.uint32) == nodes["split"].view(np.uint32)))
        out["oracle_split_agreement_" + key] = np.array(agree)
        if not tie_free:
            out["splits_" + key] = np.ascontiguousarray(nodes["split"])
        print(key, t.n, t.size, "oracle agreement", agree, flush=True)
    np.savez_compressed(os.path.join(OUT, "g7_scale_nodes.npz"), **out)


def main():
    R = Reference()
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "g7":
        g7(R)
        return

    # G1 / G2: the reference pytest cases (kdtree/tests/test_kdtree.py:6-35), wrapper leafsize 128
    for name, (pts, q, box) in (("g1_basic", g1_inputs()), ("g2_periodic", g2_inputs())):
        t = R.tree(pts, 128, box)
        d, i = t.query(q, 4)
        d2, _ = t.query(q, 4, sqrt=False)
        ref = scipy.spatial.KDTree(pts, boxsize=box)
        sd, si = ref.query(q, k=4)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), dist=d, idx=i, d2=d2,
                            scipy_dist=sd, scipy_idx=si.astype(np.int64),
                            sha=np.array(sha(pts, q)))

    # G3: config 1 — 1e5 uniform, k=8, non-periodic, 1000 queries, leaf 128
    pts, q = g3_inputs()
    t = R.tree(pts, 128, None)
    d, i, st = t.query(q, 8, stats=True)
    d2, _ = t.query(q, 8, sqrt=False)
    np.savez_compressed(os.path.join(OUT, "g3_config1.npz"), dist=d, idx=i, d2=d2,
                        sha=np.array(sha(pts, q)),
                        stats=np.array([st["nodes_visited"], st["nodes_pruned"],
                                        st["points_visited"]], np.uint64))

    # G4: 1e6 periodic L=1, 1000 random + 1000 self queries, k=32, leaf 32 and 128
    pts, q = g4_inputs()
    out = {"sha": np.array(sha(pts, q))}
    for leaf in (32, 128):
        t = R.tree(pts, leaf, 1.0)
        d2, i, st = t.query(q, 32, sqrt=False, stats=True)
        out[f"d2_leaf{leaf}"] = d2
        out[f"idx_leaf{leaf}"] = i
        out[f"stats_leaf{leaf}"] = np.array([st["nodes_visited"], st["nodes_pruned"],
                                             st["points_visited"]], np.uint64)
    np.savez_compressed(os.path.join(OUT, "g4_periodic_1e6.npz"), **out)

    # G5: node tables, n x leafsize (+ periodic variant)
    out = {}
    for key, (pts, leaf, box) in g5_inputs().items():
        t = R.tree(pts, leaf, box)
        nodes, x, y, z, idx = t.export()
        out["nodes_" + key] = nodes.view(np.uint32).reshape(-1, 4)
        out["n8_" + key] = np.array(t.n)
        out["sha_" + key] = np.array(sha(pts))
    np.savez_compressed(os.path.join(OUT, "g5_nodes.npz"), **out)

    # G6: edge cases
    out = {}
    for key, (pts, q, k, leaf, box) in edge_cases().items():
        t = R.tree(pts, leaf, box)
        d, i = t.query(q, k)
        out["dist_" + key] = d
        out["idx_" + key] = i
        out["n_" + key] = np.array(t.n)
        out["size_" + key] = np.array(t.size)
    # error case: point outside the periodic box
    try:
        R.tree(np.array([[0.5, 0.5, 1.5]], np.float32), 16, 1.0)
        out["box_error"] = np.array(0)
    except RuntimeError:
        out["box_error"] = np.array(1)
    np.savez_compressed(os.path.join(OUT, "g6_edges.npz"), **out)
    g7(R)
    print("fixtures written to", OUT)


if __name__ == "__main__":
    main()
