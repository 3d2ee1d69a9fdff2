"""Config C5 (BASELINE.json: log-normal clustering, radius query + local-density
estimate, count-quantile x-slabs) checked ROW BY ROW on the GPU against the C
oracle (oracle/kdtree_oracle.c, pinned to the compiled reference by
tests/test_oracle.py), through the C ABI (capi) with device-resident inputs:

* one tree over 4e6 log-normal points (synth.lognormal, GRF 128^3): the radius
  count of EVERY point at r = 0.01 L (sampled against oracle.ball_count), CSR
  rows of 1e3 queries as exact sets (every listed id inside the ball, no
  duplicates, as many as the oracle counts), the k = 32 k-th distance of
  every point (sampled against column 31 of the oracle's rows) and kNN rows;
* two ranks sharing the box's one GPU on synth.lognormal_slab's count-quantile
  cuts, one halo of width max(radius halo, r) over gloo, the k-th distances and
  rows that reach past it resolved by the second-round exchange
  (slab.second_round / DeviceRows): every sampled count, row and k-th
  distance equals the single-tree oracle over the union.

Reference semantics: find_closest (kdtree/src/cpp/kdtree.cpp:133-159), the a10
d2 formula (kdtree/src/cpp/kdtree_asm_systemv.asm:89-119); the radius count is
NEW: points with d2 <= r*r in the same f32 arithmetic.
"""
import os

import numpy as np
import pytest

from tests.parity import assert_knn_equal, d2_ref

pytestmark = pytest.mark.gpu


def test_c5_single_tree_rows(gpu, oracle):
    from nbodyhpc_amd import hip, synth
    n, k, r, grid = 4_000_000, 32, 0.01, 128
    pts = synth.lognormal(n, grid=grid)
    dp = hip.DeviceArray.from_numpy(pts)
    t = gpu.Tree(n=n, dev_ptr=dp.ptr, leafsize=64, boxsize=1.0)
    s = hip.Stream()
    cnt = hip.DeviceArray((n,), np.uint32)
    rk = hip.DeviceArray((n,), np.float32)
    t.ball_count_device(dp.ptr, n, r, cnt.ptr, s.handle)
    t.query_kth_device(dp.ptr, n, k, rk.ptr, s.handle)
    s.synchronize()
    c, kth = cnt.numpy(), rk.numpy()
    o = oracle.tree(pts, 64, 1.0)
    rng = np.random.Generator(np.random.PCG64(51))
    sel = np.sort(rng.choice(n, 10_000, replace=False))
    oc = oracle.ball_count(o, pts[sel], r)
    assert np.array_equal(c[sel], oc)
    assert oc.max() > 10 * np.median(oc)  # clustered: dense cores (oracle: median 27, max 649)
    dr, ir = o.query(pts[sel], k, workers=16)
    assert np.array_equal(kth[sel].view(np.uint32), dr[:, k - 1].view(np.uint32))
    # kNN rows of the same sample (host-in, host-out path of the same tree)
    d, i = t.query(pts[sel], k)
    assert_knn_equal(d, i, dr, ir, pts, pts[sel], 1.0)
    # CSR rows: 1e3 queries, half from the densest sampled points
    qsel = np.concatenate([sel[np.argsort(oc)[-500:]], sel[:500]])
    off, idx = t.ball_csr(pts[qsel], r)
    want = oracle.ball_count(o, pts[qsel], r).astype(np.int64)
    assert np.array_equal(np.diff(off.astype(np.int64)), want)
    r2 = np.float32(r) * np.float32(r)
    for j in range(len(qsel)):
        row = idx[off[j]:off[j + 1]]
        assert len(np.unique(row)) == len(row)
        assert np.all(d2_ref(pts[qsel[j]], pts[row], 1.0) <= r2)
    t.close()


def _c5_worker(rank, world, port, n_total, grid, k, r, nsample, outdir):
    from nbodyhpc_amd import hip

    hip.preload()  # the ROCm 7.2 runtime must load before torch's bundled one
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nbodyhpc_amd import capi, slab, synth
        hip.set_device(0)
        h = slab.ball_halo(r, 1.0)  # thin for kNN: leaves k-th rows to the second round
        xyz, ids, bounds = synth.lognormal_slab(n_total, rank, world, grid=grid,
                                                min_width=4 * h)
        own = len(xyz)
        ds = slab.DeviceSlab(xyz, ids, rank, world, 1.0, 0, dist, comm=None, bounds=bounds)
        ds.exchange(h)
        t = capi.Tree(n=ds.n_local, dev_ptr=ds.xyz.ptr, leafsize=64, boxsize=1.0, device=0)
        t.set_ids(dev_ptr=ds.ids.ptr)
        s = hip.Stream()
        cnt = hip.DeviceArray((own,), np.uint32)
        rk = hip.DeviceArray((own,), np.float32)
        od = hip.DeviceArray((own, k), np.float32)
        oi = hip.DeviceArray((own, k), np.uint32)
        t.ball_count_device(ds.xyz.ptr, own, r, cnt.ptr, s.handle)
        t.query_kth_device(ds.xyz.ptr, own, k, rk.ptr, s.handle)
        t.query_device(ds.xyz.ptr, own, k, od.ptr, oi.ptr, s.handle)
        s.synchronize()
        past = ds.violations(od.ptr, k)
        st_rows = slab.second_round(slab.DeviceRows(ds, t, k, od.ptr, oi.ptr, stream=s.handle),
                                    rank, world, bounds, 1.0, ds.h, k, dist)
        st_kth = slab.second_round(slab.DeviceRows(ds, t, k, kth_ptr=rk.ptr, stream=s.handle),
                                   rank, world, bounds, 1.0, ds.h, k, dist)
        s.synchronize()
        rng = np.random.Generator(np.random.PCG64(300 + rank))
        sel = np.sort(rng.choice(own, min(nsample, own), replace=False))
        np.savez(os.path.join(outdir, f"c5_{rank}.npz"), sel=sel, ids=ids[sel],
                 cnt=cnt.numpy()[sel], kth=rk.numpy(), d=od.numpy(), i=oi.numpy(),
                 past=past, fwd_rows=st_rows["rows_forwarded"], fwd_kth=st_kth["rows_forwarded"],
                 bounds=np.asarray(bounds), own=own, nloc=ds.n_local)
        t.close()
    finally:
        dist.destroy_process_group()


def test_c5_two_rank_quantile_slabs_on_one_gpu(gpu, oracle, tmp_path):
    import multiprocessing as mp

    from nbodyhpc_amd import slab, synth
    from tests.test_gpu_slab import _free_port

    world, n_total, grid, k, r = 2, 2_000_000, 128, 32, 0.004
    ctx = mp.get_context("spawn")  # plain multiprocessing: torch must not load first
    port = _free_port()
    procs = [ctx.Process(target=_c5_worker, args=(rk, world, port, n_total, grid, k, r, 20_000,
                                                  str(tmp_path)))
             for rk in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=400)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [np.load(os.path.join(tmp_path, f"c5_{rk}.npz")) for rk in range(world)]
    # the union in global-id order: rank 0's cells, then rank 1's (lognormal_slab ids)
    parts = [synth.lognormal_slab(n_total, rk, world, grid=grid,
                                  min_width=4 * slab.ball_halo(r, 1.0))[0] for rk in range(world)]
    allp = np.concatenate(parts)
    assert len(allp) == n_total
    b = res[0]["bounds"]
    assert 0.0 < b[1] < 1.0 and abs(int(res[0]["own"]) - int(res[1]["own"])) < 0.02 * n_total
    o = oracle.tree(allp, 64, 1.0)
    forwarded = 0
    for rk in range(world):
        x = res[rk]
        own = int(x["own"])
        assert int(x["nloc"]) > own
        assert int(x["fwd_rows"]) == int(x["past"])
        forwarded += int(x["fwd_rows"])
        q = parts[rk]
        # counts on the sample; rows and k-th distances of EVERY own point
        # (the rows the second round rewrote included)
        first = 0 if rk == 0 else len(parts[0])
        assert np.array_equal(x["ids"], first + x["sel"])
        assert np.array_equal(x["cnt"], oracle.ball_count(o, q[x["sel"]], r))
        dr, ir = o.query(q, k, workers=16)
        assert_knn_equal(x["d"], x["i"], dr, ir, allp, q, 1.0)
        assert np.array_equal(x["kth"].view(np.uint32), dr[:, k - 1].view(np.uint32))
    assert forwarded > 0  # the second round ran (thin kNN halo on clustered data)
