"""The drop-in surface with host buffers of any size (VERDICT r03 missing #1-3):

* M > host_batch rows through the pybind surface (nbodyhpc.kdtree) and the C
  ABI stream through two bounded device slots: rows, k-th distances and radius
  counts equal the oracle's (a small host_batch forces many batches here;
  the default is ~1 GiB of queries + results per batch);
* mixed placements: device queries with host outputs, host queries with
  device outputs;
* Ctrl-C: a long host query raises KeyboardInterrupt between batches (the
  reference polls PyErr_CheckSignals every 1000 queries,
  kdtree/src/cpp/pybind.cpp:128-133);
* concurrent queries from several Python threads on one const tree
  (pybind.cpp:90) give the serial results.
"""
import signal
import threading
import time

import numpy as np
import pytest

from tests.parity import assert_knn_equal

pytestmark = pytest.mark.gpu


@pytest.fixture
def small_host_batch(gpu):
    gpu.set_tuning("host_batch", 4096)
    yield 4096
    gpu.set_tuning("host_batch", 0)


def test_host_rows_stream_in_batches(gpu, oracle, small_host_batch):
    from nbodyhpc import kdtree
    from nbodyhpc_amd import synth
    pts = synth.uniform(300_000, 61, 1.0)
    q = synth.uniform(50_000 + 123, 62, 1.0)  # 13 batches, the last one ragged
    t = kdtree.KDTree(pts, boxsize=1.0)
    d, i = t.query(q, k=16)
    o = oracle.tree(pts, 128, 1.0)
    dr, ir = o.query(q, 16, workers=16)
    assert_knn_equal(d, i, dr, ir, pts, q, 1.0)
    kth = t.kth_distance(q, 16)
    assert np.array_equal(kth.view(np.uint32), dr[:, 15].view(np.uint32))
    c = t.query_ball(q, 0.02, return_length=True)
    assert np.array_equal(c, oracle.ball_count(o, q, 0.02))
    # k > 64 (wave select) through the same batches
    d2, i2 = t.query(q[:9000], k=100)
    dr2, ir2 = o.query(q[:9000], 100, workers=16)
    assert_knn_equal(d2, i2, dr2, ir2, pts, q[:9000], 1.0)


def test_mixed_placements_stream(gpu, oracle, small_host_batch):
    from nbodyhpc_amd import hip, synth
    pts = synth.uniform(200_000, 63, 1.0)
    m, k = 20_000, 8
    q = synth.uniform(m, 64, 1.0)
    t = gpu.Tree(pts, leafsize=64, boxsize=1.0)
    dr, ir = oracle.tree(pts, 64, 1.0).query(q, k, workers=16)
    # device queries, host outputs
    dq = hip.DeviceArray.from_numpy(q)
    d = np.empty((m, k), np.float32)
    i = np.empty((m, k), np.uint32)
    from nbodyhpc_amd import capi
    capi._check(capi.lib().nbkd_query_knn(t.h, dq.ptr, m, k, d.ctypes.data, i.ctypes.data,
                                          capi.NBKD_INPUT_DEVICE, None))
    assert_knn_equal(d, i, dr, ir, pts, q, 1.0)
    # host queries, device outputs
    od = hip.DeviceArray((m, k), np.float32)
    oi = hip.DeviceArray((m, k), np.uint32)
    t.query_device(q.ctypes.data, m, k, od.ptr, oi.ptr, input_device=False)
    hip.synchronize()
    assert_knn_equal(od.numpy(), oi.numpy(), dr, ir, pts, q, 1.0)
    t.close()


def test_device_scratch_bounded_for_large_host_query(gpu, oracle):
    """A host query of 4e6 rows with host_batch 2^18 grows the device scratch by
    what two batches need, not by the (m, k) rows (4e6 x 32 x 8 B = 1 GB)."""
    from nbodyhpc_amd import hip, synth
    pts = synth.uniform(1_000_000, 65, 1.0)
    t = gpu.Tree(pts, leafsize=64, boxsize=1.0)
    m, k = 4_000_000, 32
    q = synth.uniform(m, 66, 1.0)
    gpu.set_tuning("host_batch", 1 << 18)
    try:
        t.query(q[:1000], k)  # first call: the tree's fixed scratch
        hip.synchronize()
        free0, _ = hip.mem_info()
        d, i = t.query(q, k)
        hip.synchronize()
        free1, _ = hip.mem_info()
    finally:
        gpu.set_tuning("host_batch", 0)
    assert free0 - free1 < (600 << 20), f"grew by {(free0 - free1) >> 20} MiB"
    sel = np.arange(0, m, 401)
    dr, ir = oracle.tree(pts, 64, 1.0).query(q[sel], k, workers=16)
    assert_knn_equal(d[sel], i[sel], dr, ir, pts, q[sel], 1.0)
    t.close()


def test_ctrl_c_interrupts_a_long_host_query(gpu):
    from nbodyhpc import kdtree
    from nbodyhpc_amd import synth
    pts = synth.uniform(500_000, 67, 1.0)
    q = synth.uniform(4_000_000, 68, 1.0)
    t = kdtree.KDTree(pts, boxsize=1.0)
    gpu.set_tuning("host_batch", 1024)  # ~4000 batches: seconds of work

    def on_alarm(signum, frame):
        raise KeyboardInterrupt

    old = signal.signal(signal.SIGALRM, on_alarm)
    try:
        signal.setitimer(signal.ITIMER_REAL, 0.3)
        t0 = time.perf_counter()
        with pytest.raises(KeyboardInterrupt):
            t.query(q, k=32)
        waited = time.perf_counter() - t0
    finally:
        signal.setitimer(signal.ITIMER_REAL, 0)
        signal.signal(signal.SIGALRM, old)
        gpu.set_tuning("host_batch", 0)
    assert waited < 5.0
    # the tree is still usable afterwards
    d, i = t.query(q[:100], k=4)
    assert np.all(d[:, 0] >= 0)


def test_concurrent_queries_on_one_tree(gpu):
    from nbodyhpc import kdtree
    from nbodyhpc_amd import synth
    pts = synth.uniform(400_000, 69, 1.0)
    t = kdtree.KDTree(pts, boxsize=1.0)
    qs = [synth.uniform(150_000, 70 + j, 1.0) for j in range(6)]
    serial = [t.query(q, k=16) for q in qs]
    out = [None] * len(qs)
    errs = []

    def work(j):
        try:
            for _ in range(3):
                out[j] = t.query(qs[j], k=16)
        except Exception as e:  # reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(j,)) for j in range(len(qs))]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not errs, errs
    for j in range(len(qs)):
        assert_knn_equal(out[j][0], out[j][1], serial[j][0], serial[j][1], pts, qs[j], 1.0)


def test_stats_sum_over_host_batches(gpu, small_host_batch):
    """A host-buffer call's work counters cover every batch (each
    batch used to overwrite the last), equal to one device-buffer call's."""
    from nbodyhpc_amd import hip, synth
    pts = synth.uniform(200_000, 71, 1.0)
    m, k = 40_000, 16  # 10 batches of 4096
    q = synth.uniform(m, 72, 1.0)
    t = gpu.Tree(pts, leafsize=64, boxsize=1.0)
    gpu.stats_enable(True)
    try:
        t.query(q, k)
        host = gpu.stats_read_all()
        dq = hip.DeviceArray.from_numpy(q)
        od = hip.DeviceArray((m, k), np.float32)
        oi = hip.DeviceArray((m, k), np.uint32)
        gpu.set_tuning("host_batch", 0)
        t.query_device(dq.ptr, m, k, od.ptr, oi.ptr)
        hip.synchronize()
        dev = gpu.stats_read_all()
    finally:
        gpu.stats_enable(False)
    # packets of 64 kd-ordered queries: every batch's, at least m / 64 in all
    assert host["packets"] >= m // 64 and dev["packets"] >= m // 64
    assert abs(host["candidates"] - dev["candidates"]) < 0.1 * dev["candidates"]
    t.close()


def test_pageable_streaming_when_pinning_is_refused(gpu, oracle, small_host_batch):
    """a host-buffer call whose pinned staging would pass the
    process cap ("pinned_bytes"), or whose hipHostMalloc fails, streams
    between the caller's pageable arrays and the device instead of failing
    with NBKD_ENOMEM: same rows, k-th distances and counts."""
    from nbodyhpc_amd import synth
    pts = synth.uniform(200_000, 65, 1.0)
    q = synth.uniform(30_000 + 77, 66, 1.0)
    o = oracle.tree(pts, 64, 1.0)
    dr, ir = o.query(q, 16, workers=16)
    try:
        gpu.set_tuning("pinned_bytes", 1)  # nothing may be pinned
        t = gpu.Tree(pts, leafsize=64, boxsize=1.0)
        d, i = t.query(q, 16)
        assert_knn_equal(d, i, dr, ir, pts, q, 1.0)
        c = t.ball_count(q, 0.02)
        assert np.array_equal(c, oracle.ball_count(o, q, 0.02))
        t.close()
    finally:
        gpu.set_tuning("pinned_bytes", 0)
