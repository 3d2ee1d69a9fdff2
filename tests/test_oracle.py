"""CPU tests: the oracle (plain-C restatement of the reference) pinned against
the reference's golden vectors, the reference's own tests restated, and the
metric known-answer tests.  No GPU needed."""
import os

import numpy as np
import pytest
import scipy.spatial

from tests.golden.inputs import edge_cases, g1_inputs, g2_inputs, g3_inputs, g4_inputs, g5_inputs, sha, uniform
from tests.parity import assert_knn_equal, check_tree_structure, d2_ref


@pytest.mark.parametrize("name,inputs", [("g1_basic", g1_inputs), ("g2_periodic", g2_inputs)])
def test_oracle_reference_pytest(oracle, golden, name, inputs):
    """kdtree/tests/test_kdtree.py:6-35 against the oracle, plus the reference outputs."""
    pts, q, box = inputs()
    g = golden(name)
    assert str(g["sha"]) == sha(pts, q)
    t = oracle.tree(pts, 128, box)
    d, i = t.query(q, 4)
    assert np.allclose(g["scipy_dist"], d)
    assert np.all(g["scipy_idx"] == i)
    # bit-identical to the reference's own output
    assert np.array_equal(d.view(np.uint32), g["dist"].view(np.uint32))
    assert np.array_equal(i, g["idx"])


def test_oracle_config1(oracle, golden):
    pts, q = g3_inputs()
    g = golden("g3_config1")
    assert str(g["sha"]) == sha(pts, q)
    t = oracle.tree(pts, 128)
    d, i, st = t.query(q, 8, stats=True)
    assert np.array_equal(d.view(np.uint32), g["dist"].view(np.uint32))
    assert_knn_equal(d, i, g["dist"], g["idx"], pts, q)
    # the traversal does the same work as the reference's (KDTreeQueryStatistics)
    assert [st["nodes_visited"], st["nodes_pruned"], st["points_visited"]] == g["stats"].tolist()


@pytest.mark.parametrize("leaf", [32, 128])
def test_oracle_periodic_1e6(oracle, golden, leaf):
    pts, q = g4_inputs()
    g = golden("g4_periodic_1e6")
    assert str(g["sha"]) == sha(pts, q)
    t = oracle.tree(pts, leaf, 1.0)
    d2, i, st = t.query(q, 32, sqrt=False, stats=True)
    assert np.array_equal(d2.view(np.uint32), g[f"d2_leaf{leaf}"].view(np.uint32))
    assert_knn_equal(d2, i, g[f"d2_leaf{leaf}"], g[f"idx_leaf{leaf}"], pts, q, 1.0, sqrt=False)
    assert [st["nodes_visited"], st["nodes_pruned"], st["points_visited"]] == \
        g[f"stats_leaf{leaf}"].tolist()


def test_oracle_node_tables(oracle, golden):
    g = golden("g5_nodes")
    for key, (pts, leaf, box) in g5_inputs().items():
        assert str(g["sha_" + key]) == sha(pts)
        t = oracle.tree(pts, leaf, box)
        nodes, x, y, z, idx = t.export()
        assert t.n == int(g["n8_" + key])
        assert np.array_equal(nodes.view(np.uint32).reshape(-1, 4), g["nodes_" + key]), key
        check_tree_structure(nodes, x, y, z, idx, len(pts), leaf)


def test_oracle_edge_cases(oracle, golden):
    g = golden("g6_edges")
    for key, (pts, q, k, leaf, box) in edge_cases().items():
        t = oracle.tree(np.asarray(pts, np.float32), leaf, box)
        assert t.n == int(g["n_" + key]) and t.size == int(g["size_" + key]), key
        d, i = t.query(q, k)
        assert_knn_equal(d, i, g["dist_" + key], g["idx_" + key], np.asarray(pts, np.float32),
                         np.asarray(q, np.float32), box)
    assert int(g["box_error"]) == 1
    with pytest.raises(RuntimeError, match="within the box"):
        oracle.tree(np.array([[0.5, 0.5, 1.5]], np.float32), 16, 1.0)


def test_k_greater_than_n_padding(oracle, golden):
    """k > n: the unused slots are (sqrt(FLT_MAX), 0xFFFFFFFF) [SURVEY §8 a11]."""
    g = golden("g6_edges")
    d = g["dist_k_gt_n"]
    i = g["idx_k_gt_n"]
    assert np.all(i[:, 13:] == 0xFFFFFFFF)
    assert np.all(d[:, 13:] == np.sqrt(np.float32(np.finfo(np.float32).max)))


@pytest.mark.parametrize("n", [10, 100, 1000])
@pytest.mark.parametrize("box", [None, 2.0])
def test_oracle_tree_equals_naive(oracle, n, box):
    """test.cpp:43-111"""
    pts = uniform(n, 42, L=box or 1.0)
    q = uniform(100, 43, L=box or 1.0)
    t = oracle.tree(pts, 32, box)
    d, i = t.query(q, 4)
    db, ib = oracle.knn_brute(pts, q, 4, box)
    assert np.array_equal(d, db) and np.array_equal(i, ib)


def test_periodic_box_distance_27_images(oracle):
    """test.cpp:116-145: periodic box distance == min over 27 images (1e-6)."""
    pts = uniform(100, 42)
    box = np.array([0.2, 0.5, 0.4, 0.6, 0.0, 0.1], np.float32)
    for p in pts:
        dist = oracle.box_d2(p, box, 1.0)
        best = np.inf
        for s in np.array(np.meshgrid([-1, 0, 1], [-1, 0, 1], [-1, 0, 1])).T.reshape(-1, 3):
            best = min(best, oracle.box_d2(p + s.astype(np.float32), box, None))
        assert abs(dist - best) < 1e-6


def test_point_metric_kat(oracle):
    """d2 KATs: the oracle, numpy f32 and the hand formula agree bit for bit."""
    rng = np.random.Generator(np.random.PCG64(7))
    for _ in range(200):
        q = rng.uniform(-0.2, 1.2, 3).astype(np.float32)
        p = rng.uniform(0, 1, 3).astype(np.float32)
        for box in (None, 1.0):
            a = np.float32(oracle.point_d2(q, p, box))
            b = d2_ref(q, p[None], box)[0]
            assert a.view(np.uint32) == b.view(np.uint32)


def test_oracle_vs_scipy_random(oracle):
    for box in (None, 1.0):
        pts = uniform(20_000, 3)
        q = uniform(300, 4)
        t = oracle.tree(pts, 16, box)
        d, i = t.query(q, 10)
        sd, si = scipy.spatial.cKDTree(pts, boxsize=box).query(q, 10)
        assert np.allclose(sd, d, rtol=1e-5, atol=1e-7)
        assert (si == i).mean() > 0.999


def test_ball_count_oracle_vs_scipy(oracle):
    pts = uniform(10_000, 3)
    q = uniform(200, 4)
    for box in (None, 1.0):
        t = oracle.tree(pts, 32, box)
        c = oracle.ball_count(t, q, 0.07)
        cb = oracle.ball_count_brute(pts, q, 0.07, box)
        assert np.array_equal(c, cb)
        sc = scipy.spatial.cKDTree(pts, boxsize=box).query_ball_point(q, 0.07,
                                                                      return_length=True)
        # float32 vs float64 metric: only points within an ulp of r may differ
        assert np.abs(sc - cb.astype(np.int64)).max() <= 1


def test_tree_shape_function():
    """node count is a pure function of (n8, leaf): kdtree_impl.hpp:98-109"""
    from functools import lru_cache

    @lru_cache(None)
    def nodes(c, leaf):
        if c <= leaf:
            return 1
        m = (c // 2) // 8 * 8
        return 1 + nodes(m, leaf) + nodes(c - m, leaf)

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "g5_nodes.npz"))
    for key, (pts, leaf, box) in g5_inputs().items():
        assert nodes(int(g["n8_" + key]), max(leaf, 16)) == g["nodes_" + key].shape[0]


def test_ball_count_stats_counters(oracle):
    """orc_ball_count_stats: same counts as orc_ball_count; the counters that
    price the radius query (bench.py REF_BALL_*) are the DFS's visits: at
    least the leaves whose points were scanned, and every point counted was scanned."""
    pts = uniform(20_000, 5)
    q = uniform(300, 6)
    t = oracle.tree(pts, 32, 1.0)
    c0 = oracle.ball_count(t, q, 0.05)
    c, nodes, points = oracle.ball_count_stats(t, q, 0.05)
    assert np.array_equal(c, c0)
    assert points >= int(c.sum()) and points % 8 == 0
    assert nodes >= points // 32


def test_g7_tie_free_node_tables_pin_the_oracle(golden):
    """G7: on sets with no tied coordinate the C oracle's node table equals the
    reference's bit for bit at 1e6 and 1e7 points (tests/golden/gen_golden.py
    --only g7); the GPU tables are checked against the same fixture."""
    from oracle.oracle import Oracle
    from tests.golden.inputs import g7_inputs, node_shape, sha
    g = golden("g7_scale_nodes")
    O = Oracle()
    for key, (gen, leaf, box, tie_free) in g7_inputs().items():
        if not tie_free:
            continue
        pts = gen()
        assert str(g["sha_" + key]) == sha(pts)
        nodes = O.tree(pts, leaf, box).export()[0]
        assert sha(nodes.view(np.uint32).reshape(-1, 4)) == str(g["table_sha_" + key]), key
        assert sha(node_shape(nodes)) == str(g["shape_sha_" + key]), key
