"""GPU parity: the HIP path (through the C ABI and through the pybind surface)
against the reference's golden vectors and the oracle.  Run on an MI355X:
    python -m pytest tests -m gpu -x -q
"""
import os

import numpy as np
import pytest

from tests.golden.inputs import (edge_cases, g1_inputs, g2_inputs, g3_inputs, g4_inputs, g5_inputs,
                                 g7_inputs, node_shape, sha, uniform)
from tests.parity import assert_knn_equal, check_tree_structure, d2_ref, leaf_sets

pytestmark = pytest.mark.gpu


def _kdtree():
    from nbodyhpc import kdtree
    return kdtree


# ---------------------------------------------------------------- reference pytest (G1, G2)
@pytest.mark.parametrize("name,inputs", [("g1_basic", g1_inputs), ("g2_periodic", g2_inputs)])
def test_reference_pytest_cases(gpu, golden, name, inputs):
    """kdtree/tests/test_kdtree.py:6-35: allclose vs scipy, exact indices."""
    pts, q, box = inputs()
    g = golden(name)
    assert str(g["sha"]) == sha(pts, q)
    tree = _kdtree().KDTree(pts, boxsize=box)
    d, i = tree.query(q, k=4)
    assert np.allclose(g["scipy_dist"], d)
    assert np.all(g["scipy_idx"] == i)
    assert_knn_equal(d, i, g["dist"], g["idx"], np.asarray(pts, np.float32), q, box)
    assert np.array_equal(d.view(np.uint32), g["dist"].view(np.uint32))


def test_config1_golden(gpu, golden):
    pts, q = g3_inputs()
    g = golden("g3_config1")
    assert str(g["sha"]) == sha(pts, q)
    t = gpu.Tree(pts, leafsize=128)
    d, i = t.query(q, 8)
    assert_knn_equal(d, i, g["dist"], g["idx"], pts, q)


@pytest.mark.parametrize("leaf", [32, 128])
def test_periodic_1e6_golden(gpu, golden, leaf):
    pts, q = g4_inputs()
    g = golden("g4_periodic_1e6")
    assert str(g["sha"]) == sha(pts, q)
    t = gpu.Tree(pts, leafsize=leaf, boxsize=1.0)
    d, i = t.query(q, 32)
    d2 = g[f"d2_leaf{leaf}"]
    assert_knn_equal(d, i, np.sqrt(d2), g[f"idx_leaf{leaf}"], pts, q, 1.0)
    # self queries: the point itself is the nearest neighbour (distance 0)
    assert np.all(d[1000:, 0] == 0.0)


def test_node_tables_match_reference(gpu, golden):
    """G5: the GPU node table equals the reference's bit for bit."""
    g = golden("g5_nodes")
    for key, (pts, leaf, box) in g5_inputs().items():
        assert str(g["sha_" + key]) == sha(pts)
        t = gpu.Tree(pts, leafsize=leaf, boxsize=box)
        nodes, x, y, z, idx = t.export()
        ref = g["nodes_" + key]
        assert t.n == int(g["n8_" + key])
        assert t.size == ref.shape[0], key
        assert np.array_equal(nodes.view(np.uint32).reshape(-1, 4), ref), key
        check_tree_structure(nodes, x, y, z, idx, len(pts), leaf)


@pytest.mark.parametrize("key", list(g7_inputs()))
def test_node_tables_at_scale_match_reference(gpu, golden, key):
    """G7: node tables at 1e6-1e7 points against the
    reference's (kdtree_impl.hpp:98-146, split kdtree_selection.cpp:475-494).
    Tie-free sets (every coordinate distinct on its axis): the whole table bit
    for bit.  The plain uniform 1e7 set has tied coordinates at split values,
    where which tied points go left is the partition's choice (the reference's
    AVX2 Floyd-Rivest, our radix select) and the descendants' splits follow
    from it: there the shape (n8, node count, dims, every node's range) must be
    equal and the fraction of equal split values is measured (the C oracle's,
    over the same set, is in the fixture) and must stay >= 0.99."""
    g = golden("g7_scale_nodes")
    gen, leaf, box, tie_free = g7_inputs()[key]
    pts = gen()
    assert str(g["sha_" + key]) == sha(pts)
    t = gpu.Tree(pts, leafsize=leaf, boxsize=box)
    nodes = t.export()[0]
    assert t.n == int(g["n8_" + key]) and t.size == int(g["nnodes_" + key]), key
    assert sha(node_shape(nodes)) == str(g["shape_sha_" + key]), key
    if tie_free:
        assert sha(nodes.view(np.uint32).reshape(-1, 4)) == str(g["table_sha_" + key]), key
        return
    ref = g["splits_" + key]
    agree = float(np.mean(nodes["split"].view(np.uint32) == ref.view(np.uint32)))
    internal = nodes["dim"] >= 0
    agree_int = float(np.mean(nodes["split"][internal].view(np.uint32)
                              == ref[internal].view(np.uint32)))
    report = {"key": key, "nodes": int(t.size), "internal": int(internal.sum()),
              "split_agreement_all_nodes": agree, "split_agreement_internal": agree_int,
              "oracle_split_agreement_all_nodes": float(g["oracle_split_agreement_" + key])}
    print(report)
    out = os.environ.get("NBKD_TEST_REPORT_DIR")
    if out:
        import json
        with open(os.path.join(out, f"g7_{key}.json"), "w") as f:
            json.dump(report, f)
    assert agree >= 0.99, report


def test_leaf_membership_matches_oracle(gpu, oracle):
    for n, leaf, box in [(1000, 16, None), (50_000, 32, 1.0), (200_000, 128, None)]:
        pts = uniform(n, 77 + n)
        t = gpu.Tree(pts, leafsize=leaf, boxsize=box)
        o = oracle.tree(pts, leaf, box)
        gn, gx, gy, gz, gi = t.export()
        on, ox, oy, oz, oi = o.export()
        assert np.array_equal(gn.view(np.uint32), on.view(np.uint32))
        assert leaf_sets(gn, gi) == leaf_sets(on, oi)
        # coordinates travel with their index
        pp = np.concatenate([pts, np.full(((n + 7) // 8 * 8 - n, 3), np.finfo(np.float32).max,
                                          np.float32)])
        assert np.array_equal(pp[gi, 0], gx) and np.array_equal(pp[gi, 1], gy)
        assert np.array_equal(pp[gi, 2], gz)


def test_edge_cases_golden(gpu, golden):
    g = golden("g6_edges")
    kd = _kdtree()
    for key, (pts, q, k, leaf, box) in edge_cases().items():
        t = kd.KDTree(pts, leafsize=leaf, boxsize=box)
        assert t.n == int(g["n_" + key]), key
        assert t.size == int(g["size_" + key]), key
        d, i = t.query(q, k=k)
        assert_knn_equal(d, i, g["dist_" + key], g["idx_" + key], np.asarray(pts, np.float32),
                         np.asarray(q, np.float32), box)
    with pytest.raises(RuntimeError, match=r"all points must be within the box"):
        kd.KDTree(np.array([[0.5, 0.5, 1.5]], np.float32), boxsize=1.0)


# ---------------------------------------------------------------- sweeps vs oracle
@pytest.mark.parametrize("n,leaf,k,box", [
    (10, 16, 4, None), (100, 16, 4, 2.0), (1000, 32, 4, None), (4096, 16, 1, 1.0),
    (10_000, 64, 7, None), (33_333, 16, 16, 1.0), (100_000, 128, 20, None),
    (100_000, 32, 33, 1.0), (250_000, 24, 64, None), (250_000, 200, 5, 3.0),
    (50_000, 32, 100, 1.0), (20_000, 16, 200, None), (30_000, 64, 300, 1.0),
    (12_000, 32, 700, None), (3_000, 16, 1500, 1.0),
])
def test_knn_vs_oracle(gpu, oracle, n, leaf, k, box):
    pts = uniform(n, n + leaf, L=box or 1.0)
    rng = np.random.Generator(np.random.PCG64(n))
    q = np.concatenate([rng.uniform(0, box or 1.0, (1500, 3)).astype(np.float32), pts[:500]])
    t = gpu.Tree(pts, leafsize=leaf, boxsize=box)
    o = oracle.tree(pts, leaf, box)
    d, i = t.query(q, k)
    dr, ir = o.query(q, k)
    assert_knn_equal(d, i, dr, ir, pts, q, box)


def test_knn_brute_force_small(gpu, oracle):
    """test.cpp:43-111: tree == naive for n in {10, 100, 1000}, incl. periodic L=2."""
    for n in (10, 100, 1000):
        for box in (None, 2.0):
            pts = uniform(n, 42, L=box or 1.0)
            q = uniform(100, 43, L=box or 1.0)
            t = gpu.Tree(pts, leafsize=32, boxsize=box)
            d, i = t.query(q, 4)
            db, ib = oracle.knn_brute(pts, q, 4, box)
            assert_knn_equal(d, i, db, ib, pts, q, box)


def test_periodic_queries_outside_box(gpu, oracle):
    """Queries are not validated (pybind.cpp:90-98); outside [0, L]^3 the reference's
    periodic pruning is not a lower bound and the result depends on its exact
    traversal, which the lane-per-query path replays."""
    pts = uniform(30_000, 21)
    rng = np.random.Generator(np.random.PCG64(22))
    q = rng.uniform(-0.6, 1.6, (2000, 3)).astype(np.float32)
    t = gpu.Tree(pts, leafsize=32, boxsize=1.0)
    o = oracle.tree(pts, 32, 1.0)
    for k in (1, 8, 32):
        d, i = t.query(q, k)
        dr, ir = o.query(q, k)
        assert_knn_equal(d, i, dr, ir, pts, q, 1.0)


def test_duplicates_and_ties(gpu, oracle):
    base = uniform(300, 3)
    pts = np.concatenate([base] * 5)
    q = np.concatenate([base[:50], uniform(50, 4)])
    t = gpu.Tree(pts, leafsize=16)
    d, i = t.query(q, 12)
    db, ib = oracle.knn_brute(pts, q, 12)
    assert_knn_equal(d, i, db, ib, pts, q)


def test_grid_points_heavy_ties(gpu, oracle):
    """A lattice makes exact d2 ties everywhere (and coordinate ties at every split)."""
    g = np.arange(24, dtype=np.float32) / 24
    pts = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    q = pts[::37] + np.float32(0.01)
    t = gpu.Tree(pts, leafsize=16, boxsize=1.0)
    check_tree_structure(*t.export(), len(pts), 16)
    d, i = t.query(q, 10)
    db, ib = oracle.knn_brute(pts, q, 10, 1.0)
    assert_knn_equal(d, i, db, ib, pts, q, 1.0)


# ---------------------------------------------------------------- radius queries (NEW)
@pytest.mark.parametrize("box", [None, 1.0])
def test_ball_count_and_csr(gpu, oracle, box):
    pts = uniform(20_000, 5)
    q = uniform(700, 6)
    r = 0.05
    t = gpu.Tree(pts, leafsize=32, boxsize=box)
    c = t.ball_count(q, r)
    cb = oracle.ball_count_brute(pts, q, r, box)
    assert np.array_equal(c, cb)
    off, idx = t.ball_csr(q, r)
    assert np.array_equal(np.diff(off.astype(np.int64)), cb.astype(np.int64))
    for j in range(0, 700, 37):
        row = np.sort(idx[off[j]:off[j + 1]])
        d2 = d2_ref(q[j], pts, box)
        expect = np.nonzero(d2 <= np.float32(r) * np.float32(r))[0]
        assert np.array_equal(row, expect.astype(np.uint32))


def test_python_surface(gpu):
    kd = _kdtree()
    pts = uniform(5000, 9)
    t = kd.KDTree(pts, boxsize=1.0)
    assert t.n == 5000 and t.periodic and t.boxsize == 1.0
    with pytest.raises(RuntimeError, match="k must be positive integer"):
        t.query(pts[:3], k=0)
    with pytest.raises(RuntimeError, match=r"shape \(N, 3\)"):
        t.query(pts[:, :2])
    with pytest.warns(UserWarning, match="Unrecognized keyword arguments"):
        kd.KDTree(pts, foo=1)
    d, i = t.query(pts[:12].reshape(3, 4, 3), k=2)
    assert d.shape == (3, 4, 2) and i.shape == (3, 4, 2)
    rows = t.query_ball(pts[:5], 0.05)
    counts = t.query_ball(pts[:5], 0.05, return_length=True)
    assert [len(r) for r in rows] == counts.tolist()
    off, idx = t.query_ball(pts[:5], 0.05, return_csr=True)
    assert np.diff(off.astype(np.int64)).tolist() == counts.tolist()
    assert all(np.array_equal(rows[i], idx[off[i]:off[i + 1]]) for i in range(5))
    dens = t.density(pts[:100], k=8)
    assert np.all(np.isfinite(dens)) and np.all(dens > 0)
    rk = t.kth_distance(pts[:12].reshape(3, 4, 3), 8)
    assert rk.shape == (3, 4)
    assert np.array_equal(rk.reshape(-1), t.query(pts[:12], k=8)[0][:, 7])
    with pytest.raises(RuntimeError, match="k must be positive integer"):
        t.kth_distance(pts[:3], 0)


def test_device_pointer_path(gpu):
    """C ABI with device-resident inputs/outputs on a caller stream (the bench path)."""
    from nbodyhpc_amd import hip
    pts = uniform(100_000, 12)
    dev = hip.DeviceArray.from_numpy(pts)
    t = gpu.Tree(n=pts.shape[0], dev_ptr=dev.ptr, leafsize=32, boxsize=1.0)
    k = 16
    od = hip.DeviceArray((pts.shape[0], k), np.float32)
    oi = hip.DeviceArray((pts.shape[0], k), np.uint32)
    stream = hip.Stream()
    t.query_device(dev.ptr, pts.shape[0], k, od.ptr, oi.ptr, stream.handle)
    stream.synchronize()
    d_host, i_host = t.query(pts, k)
    # the device call is a self query (tree order, test_gpu_self_order.py), the
    # host one is bucketed and sorted: the same distances, ids up to ties
    assert np.array_equal(od.numpy().view(np.uint32), d_host.view(np.uint32))
    assert_knn_equal(od.numpy(), oi.numpy(), d_host, i_host, pts, pts, 1.0)
    cnt = hip.DeviceArray((pts.shape[0],), np.uint32)
    t.ball_count_device(dev.ptr, pts.shape[0], 0.02, cnt.ptr, stream.handle)
    stream.synchronize()
    assert np.array_equal(cnt.numpy(), t.ball_count(pts, 0.02))


# ---------------------------------------------------------------- seed ball retries
@pytest.fixture
def tuning(gpu):
    """nbkd_set_tuning knobs, restored after the test."""
    saved = {n: gpu.get_tuning(n) for n in ("knn_seed_margin", "candidate_bytes")}
    yield gpu.set_tuning
    for n, v in saved.items():
        gpu.set_tuning(n, v)


@pytest.mark.parametrize("box", [None, 1.0])
def test_knn_seed_retry(gpu, oracle, tuning, box):
    """A tiny seed ball (knn_seed_margin 0.05) makes most queries fail the
    collect pass: they go through the adaptive-seed retry, its second round
    (one query per wave, 64x column) and, failing those, the exact kernel.
    A candidate budget of a few packets cuts the first pass into many batches."""
    tuning("knn_seed_margin", 0.05)
    pts = uniform(60_000, 31, L=box or 1.0)
    rng = np.random.Generator(np.random.PCG64(32))
    q = np.concatenate([pts[:3000], rng.uniform(0, box or 1.0, (2000, 3)).astype(np.float32)])
    t = gpu.Tree(pts, leafsize=32, boxsize=box)
    o = oracle.tree(pts, 32, box)
    for k in (1, 16, 32, 50, 100, 150):
        d, i = t.query(q, k)
        dr, ir = o.query(q, k)
        assert_knn_equal(d, i, dr, ir, pts, q, box)
    tuning("knn_seed_margin", 3.5)
    tuning("candidate_bytes", 64 * 112 * 8 * 3)  # three 64-query packets per batch
    d, i = t.query(q, 32)
    dr, ir = o.query(q, 32)
    assert_knn_equal(d, i, dr, ir, pts, q, box)


def test_retry_rounds_take_failures_past_ten_percent(gpu, oracle, tuning):
    """with more than 10 % of the first pass failing (a small seed
    margin), round 1 takes them all in its batches, so the exact lane-per-query
    kernel sees few queries (round 4 sent everything past ~10 % + ~1 % there)."""
    tuning("knn_seed_margin", 0.5)
    pts = uniform(400_000, 33)
    q = pts[:200_000]
    t = gpu.Tree(pts, leafsize=64, boxsize=1.0)
    gpu.stats_enable(True)
    try:
        d, i = t.query(q, 32)
        st = gpu.stats_read_all()
    finally:
        gpu.stats_enable(False)
    assert st["retry_queries"] > 0.1 * len(q), st  # the case the advice names
    assert st["fallback_queries"] < 0.001 * len(q), st
    sel = np.arange(0, len(q), 97)
    dr, ir = oracle.tree(pts, 64, 1.0).query(q[sel], 32, workers=16)
    assert_knn_equal(d[sel], i[sel], dr, ir, pts, q[sel], 1.0)


def test_squared_output(gpu, oracle):
    """NBKD_SQUARED: the d2 the rows are sorted by (kdtree.cpp:149-151), whose
    sqrtf is the plain output, bit for bit (collect/select, exact and k > 64)."""
    pts = uniform(40_000, 61)
    rng = np.random.Generator(np.random.PCG64(62))
    q = np.concatenate([pts[:1000], rng.uniform(-0.2, 1.2, (500, 3)).astype(np.float32)])
    t = gpu.Tree(pts, leafsize=32, boxsize=None)
    tp = gpu.Tree(np.clip(pts, 0, 1), leafsize=32, boxsize=1.0)
    for tree in (t, tp):
        for k in (8, 32, 100):
            d, i = tree.query(q, k)
            d2, i2 = tree.query(q, k, squared=True)
            assert np.array_equal(np.sqrt(d2), d)
            assert np.array_equal(i2, i)


@pytest.mark.parametrize("box", [None, 1.0])
def test_knn_lognormal_vs_oracle(gpu, oracle, box):
    """Clustered inputs (SURVEY §8(d) config C5 recipe, small grid): dense knots
    and near-empty voids stress the density-based seed (retry and exact paths)."""
    from nbodyhpc_amd import synth
    pts = synth.lognormal(300_000, grid=64)
    rng = np.random.Generator(np.random.PCG64(33))
    q = np.concatenate([pts[:3000], rng.uniform(0, 1.0, (2000, 3)).astype(np.float32)])
    t = gpu.Tree(pts, leafsize=32, boxsize=box)
    o = oracle.tree(pts, 32, box)
    for k in (8, 32):
        d, i = t.query(q, k)
        dr, ir = o.query(q, k)
        assert_knn_equal(d, i, dr, ir, pts, q, box)


@pytest.mark.parametrize("box", [None, 1.0])
def test_ball_whole_leaf_shortcut_and_padding(gpu, oracle, box):
    """A radius several leaves wide: most leaves lie wholly inside the balls and
    are counted without evaluating their points; n % 8 != 0 puts padding
    points in the last leaf, which must never be counted.  Periodic queries
    outside [0, L]^3 take the per-query kernel."""
    pts = uniform(100_003, 8)
    rng = np.random.Generator(np.random.PCG64(9))
    q = np.concatenate([pts[:600], rng.uniform(0, 1.0, (300, 3)).astype(np.float32),
                        np.array([[1.0, 1.0, 1.0], [0.0, 0.0, 0.0], [1.0, 0.5, 0.0]], np.float32)])
    if box:
        q = np.concatenate([q, rng.uniform(-0.3, 1.3, (100, 3)).astype(np.float32)])
    r = 0.09
    t = gpu.Tree(pts, leafsize=16, boxsize=box)
    c = t.ball_count(q, r)
    cb = oracle.ball_count_brute(pts, q, r, box)
    assert np.array_equal(c, cb)
    off, idx = t.ball_csr(q, r)
    assert np.array_equal(np.diff(off.astype(np.int64)), cb.astype(np.int64))
    for j in range(0, len(q), 53):
        row = np.sort(idx[off[j]:off[j + 1]])
        d2 = d2_ref(q[j], pts, box)
        assert np.array_equal(row, np.nonzero(d2 <= np.float32(r) * np.float32(r))[0].astype(np.uint32))


@pytest.mark.parametrize("box", [None, 1.0])
def test_knn_degenerate_planar_points(gpu, oracle, box):
    """All points on one plane (zero-volume subtrees): the density seed is
    undefined (+inf), so no seed bound and no histogram tightening may apply."""
    rng = np.random.Generator(np.random.PCG64(41))
    pts = rng.uniform(0, 1.0, (40_000, 3)).astype(np.float32)
    pts[:, 2] = np.float32(0.5)
    pts[:5000, 1] = np.float32(0.25)  # a line inside the plane too
    q = np.concatenate([pts[:1500], rng.uniform(0, 1.0, (1500, 3)).astype(np.float32)])
    t = gpu.Tree(pts, leafsize=32, boxsize=box)
    o = oracle.tree(pts, 32, box)
    for k in (8, 32):
        d, i = t.query(q, k)
        dr, ir = o.query(q, k)
        assert_knn_equal(d, i, dr, ir, pts, q, box)


@pytest.mark.parametrize("box", [None, 1.0])
def test_kth_distance_equals_row_column(gpu, tuning, box):
    """nbkd_query_kth == column k-1 of nbkd_query_knn, bit for bit: the
    collect/select k-th-only output, the exact-kernel fallback (out-of-box
    periodic queries, forced seed failures) and the k > 64 row path."""
    pts = uniform(60_000, 51, L=box or 1.0)
    rng = np.random.Generator(np.random.PCG64(52))
    q = np.concatenate([pts[:2000], rng.uniform(0, box or 1.0, (2000, 3)).astype(np.float32)])
    if box:
        q = np.concatenate([q, rng.uniform(-0.4, 1.4, (300, 3)).astype(np.float32)])
    t = gpu.Tree(pts, leafsize=32, boxsize=box)
    for k in (1, 8, 32, 64, 100):
        d, _ = t.query(q, k)
        assert np.array_equal(t.query_kth(q, k), d[:, k - 1]), k
    tuning("knn_seed_margin", 0.05)  # most queries retried / exact
    for k in (16, 32):
        d, _ = t.query(q, k)
        assert np.array_equal(t.query_kth(q, k), d[:, k - 1]), k


@pytest.mark.parametrize("box", [None, 1.0])
def test_save_load_and_pickle(gpu, tmp_path, box):
    """Persistence: points() returns the input in input
    order; save/load and pickle rebuild a tree with the same node table and
    the same query results."""
    import pickle

    kd = _kdtree()
    pts = uniform(10_003, 41, L=box or 1.0)  # not a multiple of 8: padding
    t = kd.KDTree(pts, leafsize=32, boxsize=box)
    assert np.array_equal(t.points(), pts)
    q = uniform(500, 42, L=box or 1.0)
    d0, i0 = t.query(q, k=8)
    path = tmp_path / "tree.npz"
    t.save(path)
    for t2 in (kd.KDTree.load(path), pickle.loads(pickle.dumps(t))):
        assert t2.n == t.n and t2.size == t.size and t2.periodic == t.periodic
        assert t2.boxsize == t.boxsize
        assert np.array_equal(t2.export()[0], t.export()[0])
        d, i = t2.query(q, k=8)
        assert np.array_equal(d, d0)
        assert_knn_equal(d, i, d0, i0, pts, q, box)


# ---------------------------------------------------------------- sub-leaf groups
def _lattice(m):
    g = np.arange(m, dtype=np.float32) / m
    return np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)


@pytest.mark.parametrize("case", ["lattice64", "dups128", "lognormal64", "uniform64_self",
                                  "uniform128", "pad64"])
def test_group_leaves_vs_oracle(gpu, oracle, case):
    """The collect kernel's 8-point groups (build.hip group_kernel reorders
    each leaf; knn_collect.hip tests group boxes) at the bench's leafsize 64 and
    the reference wrapper's 128: exact ties inside a group (lattice, duplicated
    points), clustered groups, padding rows in the last leaf, and self-queries
    of every point of a 2e5 set (the bench's workload, smaller)."""
    from nbodyhpc_amd import synth
    rng = np.random.Generator(np.random.PCG64(77))
    if case == "lattice64":
        pts, leaf, box, k = _lattice(32), 64, 1.0, 16
        q = pts[::11] + np.float32(0.003)
    elif case == "dups128":
        base = uniform(3000, 5)
        pts, leaf, box, k = np.concatenate([base] * 4), 128, None, 9
        q = np.concatenate([base[:400], uniform(400, 6)])
    elif case == "lognormal64":
        pts, leaf, box, k = synth.lognormal(200_000, grid=64), 64, 1.0, 32
        q = np.concatenate([pts[::50], rng.uniform(0, 1, (1000, 3)).astype(np.float32)])
    elif case == "uniform64_self":
        pts, leaf, box, k = uniform(200_000, 12), 64, 1.0, 32
        q = pts
    elif case == "uniform128":
        pts, leaf, box, k = uniform(150_000, 13), 128, 1.0, 64
        q = rng.uniform(0, 1, (4000, 3)).astype(np.float32)
    else:  # n % 8 != 0: FLT_MAX padding rows share the last leaf's groups
        pts, leaf, box, k = uniform(70_005, 14), 64, None, 24
        q = np.concatenate([pts[-300:], uniform(300, 15)])
    t = gpu.Tree(pts, leafsize=leaf, boxsize=box)
    o = oracle.tree(pts, leaf, box)
    gn, _, _, _, gi = t.export()
    on, _, _, _, oi = o.export()
    assert leaf_sets(gn, gi) == leaf_sets(on, oi)
    d, i = t.query(q, k)
    dr, ir = o.query(q, k, workers=8)
    assert_knn_equal(d, i, dr, ir, pts, q, box)


def test_build_caches_alternating_sizes_and_threads(gpu, oracle):
    """build.hip keeps per-device scratch and shape tables keyed by (n8, leaf),
    and api.cpp a block cache for freed trees' arrays: alternating sizes,
    repeated same-size rebuilds (freed trees' blocks reused), builds from
    several threads at once and a failed (out-of-box) build in between must
    all give the oracle's node table."""
    import threading

    cases = [(70_000, 32, 1.0), (9_000, 16, None), (70_000, 32, 1.0), (131_072, 64, 1.0)]
    refs = {}
    for n, leaf, box in cases:
        pts = uniform(n, 5 + n, L=box or 1.0)
        refs[(n, leaf, box)] = (pts, oracle.tree(pts, leaf, box).export()[0].view(np.uint32))
    for rnd in range(2):
        for key in cases:
            pts, ref = refs[key]
            t = gpu.Tree(pts, leafsize=key[1], boxsize=key[2])
            assert np.array_equal(t.export()[0].view(np.uint32), ref), (rnd, key)
            t.close()
        with pytest.raises(Exception, match=r"all points must be within the box"):
            bad = np.array(refs[cases[0]][0], copy=True)
            bad[7, 2] = 1.5
            gpu.Tree(bad, leafsize=32, boxsize=1.0)
    errors = []

    def worker(key):
        try:
            pts, ref = refs[key]
            for _ in range(3):
                t = gpu.Tree(pts, leafsize=key[1], boxsize=key[2])
                if not np.array_equal(t.export()[0].view(np.uint32), ref):
                    errors.append(key)
                t.close()
        except Exception as e:  # reported below
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(key,)) for key in cases]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors


def test_device_queries_on_two_streams(gpu, oracle):
    """Two device-output queries of one tree on two streams: the tree's scratch
    is reused, so the second call waits on the device for the first's kernels
    (Workspace::enter); both results are exact."""
    from nbodyhpc_amd import hip
    pts = uniform(200_000, 81)
    qa, qb = uniform(150_000, 82), uniform(90_000, 83)
    t = gpu.Tree(pts, leafsize=64, boxsize=1.0)
    k = 32
    outs = []
    keep = []
    for q, s in ((qa, hip.Stream()), (qb, hip.Stream())):
        dq = hip.DeviceArray.from_numpy(q)
        od = hip.DeviceArray((len(q), k), np.float32)
        oi = hip.DeviceArray((len(q), k), np.uint32)
        t.query_device(dq.ptr, len(q), k, od.ptr, oi.ptr, s.handle)
        outs.append((q, od, oi))
        keep.append((dq, s))
    hip.synchronize()
    o = oracle.tree(pts, 64, 1.0)
    for q, od, oi in outs:
        dr, ir = o.query(q, k, workers=8)
        assert_knn_equal(od.numpy(), oi.numpy(), dr, ir, pts, q, 1.0)


def test_device_output_queries_are_asynchronous(gpu, oracle):
    """NBKD_OUTPUT_DEVICE kNN calls only enqueue (nbkd.h): the seed-failure
    re-walk runs on device-counted grids, so no call waits for the device.
    Two calls on one stream both return while the stream is still busy, and
    both results are exact (a tiny seed margin makes most queries take the
    re-walk rounds too)."""
    from nbodyhpc_amd import hip
    pts = uniform(2_000_000, 91)
    q2 = uniform(2_000_000, 92)
    t = gpu.Tree(pts, leafsize=64, boxsize=1.0)
    k = 32
    s = hip.Stream()
    dp, dq = hip.DeviceArray.from_numpy(pts), hip.DeviceArray.from_numpy(q2)
    outs = [(hip.DeviceArray((len(pts), k), np.float32), hip.DeviceArray((len(pts), k), np.uint32))
            for _ in range(2)]
    saved = gpu.get_tuning("knn_seed_margin")
    try:
        for margin in (3.5, 0.05):
            gpu.set_tuning("knn_seed_margin", margin)
            t.query_device(dp.ptr, len(pts), k, outs[0][0].ptr, outs[0][1].ptr, s.handle)  # warm
            s.synchronize()
            busy = []
            for (od, oi), src in zip(outs, (dp, dq)):
                t.query_device(src.ptr, len(pts), k, od.ptr, oi.ptr, s.handle)
                busy.append(s.busy())
            s.synchronize()
            assert all(busy), busy
            o = oracle.tree(pts, 64, 1.0)
            rng = np.random.Generator(np.random.PCG64(93))
            sel = np.sort(rng.choice(len(pts), 20_000, replace=False))
            for (od, oi), host_q in zip(outs, (pts, q2)):
                d, i = od.numpy()[sel], oi.numpy()[sel]
                dr, ir = o.query(host_q[sel], k, workers=8)
                assert_knn_equal(d, i, dr, ir, pts, host_q[sel], 1.0)
    finally:
        gpu.set_tuning("knn_seed_margin", saved)


@pytest.mark.parametrize("box,r", [(1.0, 0.35), (2.5, 0.6), (1.0, 0.499)])
def test_ball_count_wide_radius_periodic_images(gpu, oracle, box, r):
    """Radii comparable to L/2: many (query, leaf) pairs reach their points
    through the periodic image, where the count kernel must keep the periodic
    per-axis minimum; elsewhere it uses the plain d2 (same bits when every
    point of the leaf lies within L/2 on each axis).  Counts equal brute force."""
    rng = np.random.Generator(np.random.PCG64(31))
    pts = (rng.uniform(0, 1, (30_000, 3)) * box).astype(np.float32)
    pts = np.minimum(pts, np.float32(box))
    q = np.concatenate([pts[:300], (rng.uniform(0, 1, (300, 3)) * box).astype(np.float32),
                        np.array([[0, 0, 0], [box, box, box], [box / 2, 0, box]], np.float32)])
    t = gpu.Tree(pts, leafsize=64, boxsize=box)
    c = t.ball_count(q, r)
    assert np.array_equal(c, oracle.ball_count_brute(pts, q, r, box))


@pytest.mark.parametrize("k,box", [(65, 1.0), (100, None), (127, 1.0), (128, 1.0)])
def test_wave_select_pairs_vs_oracle(gpu, oracle, k, box):
    """64 < k <= 128 (round 6): the first pass's wave select takes two queries
    per wave; an odd query count leaves the last one unpaired, and columns it
    cannot take (failures, more than 128 below the bound) go to the one-query
    kernel.  Rows and the k-th distance against the oracle, plain and with a
    seed margin that fails most first passes."""
    pts = uniform(80_000, 900 + k, L=box or 1.0)
    rng = np.random.Generator(np.random.PCG64(k))
    q = np.concatenate([pts[:2001], rng.uniform(0, box or 1.0, (1000, 3)).astype(np.float32)])
    t = gpu.Tree(pts, leafsize=64, boxsize=box)
    o = oracle.tree(pts, 64, box)
    dr, ir = o.query(q, k)
    d, i = t.query(q, k)
    assert_knn_equal(d, i, dr, ir, pts, q, box)
    kth = t.query_kth(q, k)
    assert np.array_equal(kth.view(np.uint32), dr[:, k - 1].view(np.uint32))
    saved = gpu.get_tuning("knn_seed_margin")
    try:
        gpu.set_tuning("knn_seed_margin", 0.3)
        d, i = t.query(q, k)
        assert_knn_equal(d, i, dr, ir, pts, q, box)
    finally:
        gpu.set_tuning("knn_seed_margin", saved)
    t.close()
