"""Out-of-memory retry (api.cpp malloc_or_release): with the device filled to
the last allocation, a build and a query still succeed because what the device
holds idle -- cached tree blocks, the build scratch and the scratch of trees no
call is using -- goes back to the driver before one retry.  Results are checked
against the oracle, so a trimmed workspace regrowing stays correct."""
import numpy as np
import pytest

from tests.parity import assert_knn_equal

pytestmark = pytest.mark.gpu


def _fill_device(keep_mib=0):
    """allocate until hipMalloc fails; returns the blocks (free them!)"""
    from nbodyhpc_amd import hip
    blocks = []
    free, _ = hip.mem_info()
    big = free - (512 << 20)
    if big > 0:
        blocks.append(hip.DeviceArray((big,), np.uint8))
    for _ in range(4096):  # then 2 MiB at a time, to the last one
        try:
            blocks.append(hip.DeviceArray((2 << 20,), np.uint8))
        except RuntimeError:
            break
    for _ in range(keep_mib // 2):
        blocks.pop().free()
    return blocks


def test_oom_retry_releases_idle_scratch(gpu, oracle):
    from nbodyhpc_amd import hip, synth
    rng = np.random.default_rng(5)
    pa = synth.uniform(1_000_000, 101, 1.0)
    qa = rng.random((1_000_000, 3), dtype=np.float32)
    ta = gpu.Tree(pa, leafsize=64, boxsize=1.0)
    da, ia = ta.query(qa, 32)  # host output: its scratch holds > 256 MB
    pb = synth.uniform(3_000_000, 102, 1.0)
    hog = _fill_device()
    try:
        with pytest.raises(RuntimeError):  # the device is really full
            hip.DeviceArray((64 << 20,), np.uint8)
        # needs ~100 MB of tree blocks and build scratch: only a trimmed
        # workspace of the idle tree `ta` can give them
        tb = gpu.Tree(pb, leafsize=64, boxsize=1.0)
        qb = qa[:20_000]
        db, ib = tb.query(qb, 16)
    finally:
        for b in hog:
            b.free()
    ob = oracle.tree(pb, 64, 1.0)
    dr, ir = ob.query(qb, 16, workers=8)
    assert_knn_equal(db, ib, dr, ir, pb, qb, 1.0)
    # the trimmed tree regrows its scratch and still answers the same
    d2, i2 = ta.query(qa, 32)
    assert np.array_equal(d2, da) and np.array_equal(i2, ia)
    sel = np.arange(0, 1_000_000, 97)
    oa = oracle.tree(pa, 64, 1.0)
    dr, ir = oa.query(qa[sel], 32, workers=8)
    assert_knn_equal(da[sel], ia[sel], dr, ir, pa, qa[sel], 1.0)


@pytest.mark.parametrize("k", [32, 200])
def test_small_query_scratch_is_bounded(gpu, oracle, k):
    """The query scratch of a small call is sized for that call: the retry
    rounds' columns cover ~10 % / ~1 % of its queries, not every query failing
    (a 1e5-query k = 32 call held ~5.7 GB)."""
    from nbodyhpc_amd import hip, synth
    pts = synth.uniform(1_000_000, 103, 1.0)
    t = gpu.Tree(pts, leafsize=64, boxsize=1.0)
    m = 100_000
    dq = hip.DeviceArray.from_numpy(pts[:m])
    od = hip.DeviceArray((m, k), np.float32)
    oi = hip.DeviceArray((m, k), np.uint32)
    hip.synchronize()
    free0, _ = hip.mem_info()
    t.query_device(dq.ptr, m, k, od.ptr, oi.ptr)
    hip.synchronize()
    free1, _ = hip.mem_info()
    grew = free0 - free1
    assert grew < (512 << 20), f"a {m}-query k={k} call grew the scratch by {grew >> 20} MiB"
    o = oracle.tree(pts, 64, 1.0)
    sel = np.arange(0, m, 13)
    dr, ir = o.query(pts[sel], k, workers=8)
    assert_knn_equal(od.numpy()[sel], oi.numpy()[sel], dr, ir, pts, pts[sel], 1.0)
    t.close()
