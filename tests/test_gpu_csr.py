"""Batched CSR radius query with rows sorted on the device.

nbkd_query_ball_csr streams: the counts through the host-buffer pipeline,
the fill in batches bounded in ids and queries, each batch's rows sorted on
the device (NBKD_SORTED: one wave per row in LDS, the radix sort for rows
past the LDS capacity) and copied out while the next batch fills.  NEW
capability (the reference has no radius search): the rows are checked against
brute force over the same f32 metric (d2 <= r*r, tests/parity.py d2_ref) and
the counts against the C oracle.
"""
import numpy as np
import pytest

from tests.parity import d2_ref

pytestmark = pytest.mark.gpu


def _brute_row(pts, qj, r, box):
    d2 = d2_ref(qj, pts, box)
    return np.nonzero(d2 <= np.float32(r) * np.float32(r))[0].astype(np.uint32)


@pytest.fixture
def small_batches(gpu):
    gpu.set_tuning("host_batch", 4096)
    yield 4096
    gpu.set_tuning("host_batch", 0)


@pytest.mark.parametrize("box", [1.0, None])
def test_csr_batches_sorted_rows_match_brute_force(gpu, oracle, small_batches, box):
    from nbodyhpc_amd import synth
    pts = synth.uniform(300_000, 81, 1.0)
    q = synth.uniform(40_000 + 17, 82, 1.0)  # ~10 batches, the last one ragged
    if box is not None:
        q[:5] += np.float32(1.5)  # periodic queries outside [0, L]^3: every point tested
    r = 0.02
    t = gpu.Tree(pts, leafsize=64, boxsize=box)
    off, idx = t.ball_csr(q, r, sorted=True)
    o = oracle.tree(pts, 64, box)
    cnt = oracle.ball_count(o, q, r).astype(np.int64)
    cnt[:5] = [len(_brute_row(pts, q[j], r, box)) for j in range(5)]  # outside the box
    assert np.array_equal(np.diff(off.astype(np.int64)), cnt.astype(np.int64))
    assert off[-1] == cnt.sum()
    # every row strictly ascending
    d = np.diff(idx.astype(np.int64))
    starts = off[1:-1].astype(np.int64)
    inner = np.ones(len(d), bool)
    inner[starts[(starts > 0) & (starts <= len(d))] - 1] = False
    assert np.all(d[inner] > 0)
    for j in list(range(0, len(q), 997)) + [0, 1, 2, 3, 4, len(q) - 1]:
        assert np.array_equal(idx[off[j]:off[j + 1]], _brute_row(pts, q[j], r, box)), j
    # unsorted rows: the same sets
    off2, idx2 = t.ball_csr(q, r, sorted=False)
    assert np.array_equal(off2, off)
    for j in range(0, len(q), 1499):
        assert np.array_equal(np.sort(idx2[off2[j]:off2[j + 1]]), idx[off[j]:off[j + 1]])
    t.close()


def test_csr_rows_past_the_lds_sort(gpu):
    """Rows longer than the one-wave LDS sort (2048 ids) go through the radix
    sort one by one: sorted and complete."""
    from nbodyhpc_amd import synth
    pts = synth.uniform(40_000, 83, 1.0)
    q = synth.uniform(300, 84, 1.0)
    r = 0.27  # ~3300 points per row on average; rows on both sides of 2048
    t = gpu.Tree(pts, leafsize=32, boxsize=1.0)
    off, idx = t.ball_csr(q, r, sorted=True)
    lens = np.diff(off.astype(np.int64))
    assert lens.max() > 2048 and lens.min() > 0
    for j in range(len(q)):
        assert np.array_equal(idx[off[j]:off[j + 1]], _brute_row(pts, q[j], r, 1.0)), j
    t.close()


def test_csr_device_io_and_python_surface(gpu, small_batches):
    """Device queries into device ids equal the host path; the Python
    surface returns sorted CSR rows and scipy-style row arrays without any
    per-row sort on the host."""
    from nbodyhpc import kdtree
    from nbodyhpc_amd import hip, synth
    pts = synth.uniform(200_000, 85, 1.0)
    q = synth.uniform(20_000, 86, 1.0)
    r = 0.03
    t = gpu.Tree(pts, leafsize=64, boxsize=1.0)
    off, idx = t.ball_csr(q, r, sorted=True)
    dq = hip.DeviceArray.from_numpy(q)
    doff = np.empty(len(q) + 1, np.uint64)
    t.ball_csr_device(dq.ptr, len(q), r, doff, None, 0, sorted=True)
    assert np.array_equal(doff, off)
    di = hip.DeviceArray((int(doff[-1]),), np.uint32)
    t.ball_csr_device(dq.ptr, len(q), r, doff, di.ptr, int(doff[-1]), sorted=True)
    assert np.array_equal(di.numpy(), idx)
    t.close()
    kt = kdtree.KDTree(pts, leafsize=64, boxsize=1.0)
    o2, i2 = kt.query_ball(q, r, return_csr=True)
    assert np.array_equal(o2, off) and np.array_equal(i2, idx)
    rows = kt.query_ball(q[:50].reshape(5, 10, 3), r)
    assert rows.shape == (5, 10)
    for j in range(50):
        assert np.array_equal(rows.reshape(-1)[j], idx[off[j]:off[j + 1]])


def test_csr_device_scratch_bounded(gpu):
    """3e6 host queries at ~113 neighbours each (~3.4e8 ids, 1.4 GB of
    output) grow device memory by what two fill batches need, not by the
    whole id array."""
    from nbodyhpc_amd import hip, synth
    pts = synth.uniform(1_000_000, 87, 1.0)
    q = synth.uniform(3_000_000, 88, 1.0)
    r = 0.03
    t = gpu.Tree(pts, leafsize=64, boxsize=1.0)
    gpu.set_tuning("host_batch", 1 << 18)
    try:
        t.ball_csr(q[:1000], r, sorted=True)  # the tree's fixed scratch
        hip.synchronize()
        free0, _ = hip.mem_info()
        off, idx = t.ball_csr(q, r, sorted=True)
        hip.synchronize()
        free1, _ = hip.mem_info()
    finally:
        gpu.set_tuning("host_batch", 0)
    nnz = int(off[-1])
    assert nnz > 3e8
    assert free0 - free1 < (nnz * 4) // 2, f"grew by {(free0 - free1) >> 20} MiB for {nnz} ids"
    for j in range(0, len(q), 150_001):
        assert np.array_equal(idx[off[j]:off[j + 1]], _brute_row(pts, q[j], r, 1.0)), j
    t.close()
