"""Self queries (query.hip self_order): kNN, k-th and radius queries whose
queries are the first m rows of the device array the tree was built from run
in tree order, with seeds from each query's tree position, instead of
bucketing and sorting the queries.  Each case compares that path with the
bucketed-and-sorted one (nbkd_set_tuning("self_order", 0)) on the same
inputs -- distances bit for bit, ids up to exact-distance ties -- and samples
the oracle.  The reference answers every query the same way
(kdtree/src/cpp/kdtree.cpp:131-160); the order is ours only."""
import numpy as np
import pytest

from tests.golden.inputs import uniform
from tests.parity import assert_knn_equal

pytestmark = pytest.mark.gpu


@pytest.fixture
def knobs(gpu):
    names = ("self_order", "knn_seed_margin")
    saved = {n: gpu.get_tuning(n) for n in names}
    gpu.timing_enable(True)
    yield gpu
    gpu.timing_enable(False)
    for n, v in saved.items():
        gpu.set_tuning(n, v)


def _knn(gpu, t, dq, m, k, self_on):
    """kNN of the first m rows of device array dq; returns (d, i, self path taken)."""
    from nbodyhpc_amd import hip
    gpu.set_tuning("self_order", 1.0 if self_on else 0.0)
    od = hip.DeviceArray((m, k), np.float32)
    oi = hip.DeviceArray((m, k), np.uint32)
    s = hip.Stream()
    gpu.timing_reset()
    t.query_device(dq.ptr, m, k, od.ptr, oi.ptr, s.handle)
    s.synchronize()
    took = gpu.timing_read("self_order")[1] > 0
    return od.numpy(), oi.numpy(), took


def _lognormal(n, seed, L=1.0):
    from nbodyhpc_amd import synth
    return synth.lognormal(n, seed, L, grid=64)


@pytest.mark.parametrize("box,leaf,k", [(1.0, 64, 32), (None, 32, 16), (1.0, 32, 100)])
def test_self_order_matches_sorted_path(knobs, oracle, box, leaf, k):
    from nbodyhpc_amd import hip
    gpu = knobs
    pts = uniform(300_000, 71, L=box or 1.0)
    dp = hip.DeviceArray.from_numpy(pts)
    t = gpu.Tree(n=len(pts), dev_ptr=dp.ptr, leafsize=leaf, boxsize=box)
    d1, i1, took = _knn(gpu, t, dp, len(pts), k, True)
    assert took
    d0, i0, took0 = _knn(gpu, t, dp, len(pts), k, False)
    assert not took0
    assert np.array_equal(d1.view(np.uint32), d0.view(np.uint32))
    assert_knn_equal(d1, i1, d0, i0, pts, pts, box)
    assert np.all(d1[:, 0] == 0.0)
    sel = np.arange(0, len(pts), 37)
    dr, ir = oracle.tree(pts, leaf, box).query(pts[sel], k, workers=8)
    assert_knn_equal(d1[sel], i1[sel], dr, ir, pts, pts[sel], box)


@pytest.mark.parametrize("box", [None, 1.0])
def test_self_order_prefix_and_set_ids(knobs, oracle, box):
    """A slab tree: owned rows first, then halo rows; the owned rows are the
    queries (a prefix of the build array) and the ids are remapped
    (nbkd_set_ids), so the order comes from the build's permutation."""
    from nbodyhpc_amd import hip
    gpu = knobs
    pts = uniform(250_000, 72, L=box or 1.0)
    own = 170_001
    dp = hip.DeviceArray.from_numpy(pts)
    t = gpu.Tree(n=len(pts), dev_ptr=dp.ptr, leafsize=64, boxsize=box)
    gids = (np.arange(len(pts), dtype=np.uint32) * 3 + 1000).astype(np.uint32)
    t.set_ids(gids)
    k = 32
    d1, i1, took = _knn(gpu, t, dp, own, k, True)
    assert took
    d0, i0, _ = _knn(gpu, t, dp, own, k, False)
    assert np.array_equal(d1.view(np.uint32), d0.view(np.uint32))
    inv = np.full(gids.max() + 1, 0xFFFFFFFF, np.uint32)
    inv[gids] = np.arange(len(pts), dtype=np.uint32)
    assert_knn_equal(d1, inv[i1], d0, inv[i0], pts, pts[:own], box)
    sel = np.arange(0, own, 29)
    dr, ir = oracle.tree(pts, 64, box).query(pts[sel], k, workers=8)
    assert_knn_equal(d1[sel], inv[i1[sel]], dr, ir, pts, pts[sel], box)


def test_self_order_after_the_array_changed(knobs, oracle):
    """The same pointer, other contents: the order and seeds no longer fit the
    queries, and the results are still those of the queries as given."""
    from nbodyhpc_amd import hip
    gpu = knobs
    pts = uniform(200_000, 73)
    dp = hip.DeviceArray.from_numpy(pts)
    t = gpu.Tree(n=len(pts), dev_ptr=dp.ptr, leafsize=64, boxsize=1.0)
    q = _lognormal(len(pts), 74)
    hip.memcpy(dp.ptr, q.ctypes.data, q.nbytes, hip.H2D)
    d1, i1, took = _knn(gpu, t, dp, len(pts), 32, True)
    assert took
    d0, i0, _ = _knn(gpu, t, dp, len(pts), 32, False)
    assert np.array_equal(d1.view(np.uint32), d0.view(np.uint32))
    assert_knn_equal(d1, i1, d0, i0, pts, q, 1.0)
    sel = np.arange(0, len(q), 41)
    dr, ir = oracle.tree(pts, 64, 1.0).query(q[sel], 32, workers=8)
    assert_knn_equal(d1[sel], i1[sel], dr, ir, pts, q[sel], 1.0)


@pytest.mark.parametrize("margin", [0.05, 3.5])
def test_self_order_seed_failures_and_kth(knobs, oracle, margin):
    """Seed failures of the first pass (a tiny margin fails most queries):
    their seeds move from the per-position array to the per-id one for the
    re-walk rounds; k <= 64 (lane select) and k > 64 (wave select); the k-th
    distance alone (query_kth) and radius counts take the self order too."""
    from nbodyhpc_amd import hip
    gpu = knobs
    gpu.set_tuning("knn_seed_margin", margin)
    pts = _lognormal(150_000, 75)
    dp = hip.DeviceArray.from_numpy(pts)
    t = gpu.Tree(n=len(pts), dev_ptr=dp.ptr, leafsize=64, boxsize=1.0)
    for k in (32, 80):
        d1, i1, took = _knn(gpu, t, dp, len(pts), k, True)
        assert took
        d0, i0, _ = _knn(gpu, t, dp, len(pts), k, False)
        assert np.array_equal(d1.view(np.uint32), d0.view(np.uint32))
        assert_knn_equal(d1, i1, d0, i0, pts, pts, 1.0)
    sel = np.arange(0, len(pts), 53)
    dr, ir = oracle.tree(pts, 64, 1.0).query(pts[sel], 80, workers=8)
    assert_knn_equal(d1[sel], i1[sel], dr, ir, pts, pts[sel], 1.0)
    s = hip.Stream()
    kth = {}
    cnt = {}
    for on in (True, False):
        gpu.set_tuning("self_order", 1.0 if on else 0.0)
        od = hip.DeviceArray((len(pts),), np.float32)
        oc = hip.DeviceArray((len(pts),), np.uint32)
        gpu.timing_reset()
        t.query_kth_device(dp.ptr, len(pts), 32, od.ptr, s.handle)
        t.ball_count_device(dp.ptr, len(pts), 0.01, oc.ptr, s.handle)
        s.synchronize()
        assert (gpu.timing_read("self_order")[1] == 2) == on
        kth[on], cnt[on] = od.numpy(), oc.numpy()
    assert np.array_equal(kth[True].view(np.uint32), kth[False].view(np.uint32))
    assert np.array_equal(cnt[True], cnt[False])
    assert np.array_equal(cnt[True][sel], t.ball_count(pts[sel], 0.01))


def test_host_queries_do_not_take_the_self_order(knobs):
    """Host arrays stream through device slots: never the build array."""
    gpu = knobs
    pts = uniform(50_000, 76)
    t = gpu.Tree(pts, leafsize=64, boxsize=1.0)
    gpu.timing_reset()
    d, _ = t.query(pts, 8)
    assert gpu.timing_read("self_order")[1] == 0
    assert np.all(d[:, 0] == 0.0)


@pytest.mark.parametrize("box,k,margin", [(1.0, 32, 3.5), (1.0, 32, 0.05), (None, 16, 0.05),
                                          (1.0, 80, 3.5)])
def test_kth_out_beside_the_rows(knobs, box, k, margin):
    """nbkd_set_kth_out: a query of the tree's own rows with device rows leaves
    each row's last column in the attached array, bit for bit, whichever path
    wrote the row (lane select, re-walk rounds at a tiny seed margin, the exact
    kernel, the wave select at k > 64) and whichever order it took (the self
    order or, with self_order = 0, the sorted one: ADVICE r05); queries of
    other arrays, host-output and k-th-only calls leave it untouched."""
    from nbodyhpc_amd import hip
    gpu = knobs
    gpu.set_tuning("knn_seed_margin", margin)
    pts = _lognormal(120_000, 77, box or 1.0)
    dp = hip.DeviceArray.from_numpy(pts)
    t = gpu.Tree(n=len(pts), dev_ptr=dp.ptr, leafsize=64, boxsize=box)
    m = 100_001
    side = hip.DeviceArray((m,), np.float32)

    def reset():
        hip.memcpy(side.ptr, np.full(m, -1.0, np.float32).ctypes.data, 4 * m, hip.H2D)

    reset()
    t.set_kth_out(side.ptr, m)
    d, _, took = _knn(gpu, t, dp, m, k, True)
    assert took
    assert np.array_equal(side.numpy().view(np.uint32), d[:, k - 1].view(np.uint32))
    # the sorted path (self_order = 0) writes it too: a slab's forward test
    # must never read a stale array
    reset()
    d0, _, took0 = _knn(gpu, t, dp, m, k, False)
    assert not took0
    assert np.array_equal(side.numpy().view(np.uint32), d0[:, k - 1].view(np.uint32))
    before = side.numpy().copy()
    other = hip.DeviceArray.from_numpy(uniform(m, 78, L=box or 1.0))
    _knn(gpu, t, other, m, k, True)  # not the build array: no side write
    # device queries of the build array, host rows: no side write
    s = hip.Stream()
    od = hip.DeviceArray((m,), np.float32)
    t.query_kth_device(dp.ptr, m, k, od.ptr, s.handle)  # k-th only: untouched
    s.synchronize()
    assert np.array_equal(side.numpy().view(np.uint32), before.view(np.uint32))
    t.set_kth_out(None)
    _knn(gpu, t, dp, 50_000, k, True)
    assert np.array_equal(side.numpy().view(np.uint32), before.view(np.uint32))


def test_kth_out_beyond_the_packet_path(knobs):
    """k > 1024 (no collect/select: the exact kernel writes every row) fills
    the nbkd_set_kth_out array as well."""
    from nbodyhpc_amd import hip
    gpu = knobs
    pts = uniform(6_000, 79)
    dp = hip.DeviceArray.from_numpy(pts)
    t = gpu.Tree(n=len(pts), dev_ptr=dp.ptr, leafsize=32, boxsize=1.0)
    m, k = 700, 1100
    side = hip.DeviceArray((m,), np.float32)
    hip.memcpy(side.ptr, np.full(m, -1.0, np.float32).ctypes.data, 4 * m, hip.H2D)
    t.set_kth_out(side.ptr, m)
    d, _, _ = _knn(gpu, t, dp, m, k, True)
    assert np.array_equal(side.numpy().view(np.uint32), d[:, k - 1].view(np.uint32))
    t.set_kth_out(None)
