import sys, numpy as np
sys.path.insert(0, '.')
from nbodyhpc_amd import capi
from oracle.oracle import Oracle
from tests.golden.inputs import g1_inputs, g2_inputs, uniform
from tests.parity import check_tree_structure
O = Oracle()
def chk(tag, pts, leaf, box, reps=6):
    pts = np.asarray(pts, np.float32)
    o = O.tree(pts, leaf, box); on, *_ = o.export()
    for r in range(reps):
        t = capi.Tree(pts, leafsize=leaf, boxsize=box)
        nodes, x, y, z, idx = t.export()
        n8 = t.n
        perm_ok = np.array_equal(np.sort(idx), np.arange(n8, dtype=np.uint32))
        pp = np.concatenate([pts, np.full((n8 - len(pts), 3), np.finfo(np.float32).max, np.float32)])
        coords_ok = perm_ok and np.array_equal(pp[idx, 0], x) and np.array_equal(pp[idx,1], y) and np.array_equal(pp[idx,2], z)
        nodes_eq = np.array_equal(nodes.view(np.uint32), on.view(np.uint32))
        try:
            st = check_tree_structure(nodes, x, y, z, idx, len(pts), leaf)
        except AssertionError as e:
            st = f"FAIL {e}"
        print(tag, r, "perm", perm_ok, "coords", coords_ok, "nodes==oracle", nodes_eq, "struct", st, "uniq x", len(np.unique(x)), flush=True)
p, q, b = g2_inputs(); chk("g2", p, 128, b)
p, q, b = g1_inputs(); chk("g1", p, 128, b)
chk("n1000", uniform(1000, 2000), 1, None)
chk("n5000p", uniform(5000, 3), 16, 1.0)
chk("n100k", uniform(100000, 4), 32, 1.0)
