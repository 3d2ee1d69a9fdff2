"""SURVEY.md §8(f) rank 2 on the GPU: particle files -> x-slabs -> DeviceSlab ->
slab trees -> kNN rows, two ranks sharing the box's one GPU (halo and second
round over gloo), every row compared with the single-tree oracle over the
whole file:

* raw float32 (N, 3) rows, the format the reference's CLI reads
  (kdtree/src/cpp/main.cpp:103-114), each rank scanning the file for its slab
  (io.read_slab);
* the same rows redistributed: each rank reads a contiguous row chunk and the
  particles go to their slab owners by the all-to-all-v (slab.redistribute);
* a two-file, format-2, big-endian Gadget-2 snapshot with a box of 50, each
  rank streaming its slab from the memory-mapped POS blocks
  (io.read_gadget_slab).
Global ids are row numbers in file order (read_gadget's order for Gadget).
"""
import os

import numpy as np
import pytest

from tests.parity import assert_knn_equal

pytestmark = pytest.mark.gpu

N, K = 240_000, 16


def _worker(rank, world, port, mode, path, box, outdir):
    from nbodyhpc_amd import hip

    hip.preload()
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nbodyhpc_amd import capi, io, slab
        hip.set_device(0)
        if mode == "raw":
            xyz, ids = io.read_slab(path, rank, world, box, chunk_rows=50_000)
        elif mode == "redistribute":
            rows = io.read_positions(path)
            lo, hi = rank * len(rows) // world, (rank + 1) * len(rows) // world
            xyz, ids = slab.redistribute(np.array(rows[lo:hi]), np.arange(lo, hi, dtype=np.uint32),
                                         rank, world, box, dist, comm=None, device=0)
        else:
            xyz, ids, hdr = io.read_gadget_slab(path, rank, world, chunk_rows=50_000)
            assert float(hdr["BoxSize"]) == box
        own = len(xyz)
        ds = slab.DeviceSlab(xyz, ids, rank, world, box, 0, dist, comm=None)
        ds.exchange(slab.halo_width(N, K, box) * 0.3)  # thin: rows reach the second round
        t = capi.Tree(n=ds.n_local, dev_ptr=ds.xyz.ptr, leafsize=64, boxsize=box, device=0)
        t.set_ids(dev_ptr=ds.ids.ptr)
        od = hip.DeviceArray((max(own, 1), K), np.float32)
        oi = hip.DeviceArray((max(own, 1), K), np.uint32)
        t.query_device(ds.xyz.ptr, own, K, od.ptr, oi.ptr)
        hip.synchronize()
        st = slab.second_round(slab.DeviceRows(ds, t, K, od.ptr, oi.ptr), rank, world, ds.bounds,
                               box, ds.h, K, dist)
        hip.synchronize()
        np.savez(os.path.join(outdir, f"{mode}{rank}.npz"), ids=ids, xyz=xyz,
                 d=od.numpy_head(own), i=oi.numpy_head(own), fwd=st["rows_forwarded"])
        t.close()
    finally:
        dist.destroy_process_group()


def _run(tmp_path, mode, path, box):
    import multiprocessing as mp

    from tests.test_gpu_slab import _free_port
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, path, box, str(tmp_path)))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return [np.load(os.path.join(tmp_path, f"{mode}{r}.npz")) for r in range(2)]


def _check(parts, allp, box, oracle):
    o = oracle.tree(allp, 64, box)
    seen = np.concatenate([p["ids"] for p in parts])
    assert np.array_equal(np.sort(seen), np.arange(len(allp), dtype=np.uint32))  # a partition
    fwd = 0
    for p in parts:
        assert np.array_equal(p["xyz"], allp[p["ids"]])
        dr, ir = o.query(p["xyz"], K, workers=16)
        assert_knn_equal(p["d"], p["i"], dr, ir, allp, p["xyz"], box)
        fwd += int(p["fwd"])
    assert fwd > 0


@pytest.mark.parametrize("mode", ["raw", "redistribute"])
def test_raw_file_slabs_on_one_gpu(gpu, oracle, tmp_path, mode):
    from nbodyhpc_amd import io, synth
    pts = synth.lognormal(N, seed=77, grid=64)
    path = str(tmp_path / "particles.f32")
    io.write_positions(path, pts)
    parts = _run(tmp_path, mode, path, 1.0)
    _check(parts, pts, 1.0, oracle)


def test_gadget_two_file_snapshot_slabs_on_one_gpu(gpu, oracle, tmp_path):
    from nbodyhpc_amd import io, synth
    box = 50.0
    pts = (synth.uniform(N, 78, 1.0) * np.float32(box)).astype(np.float32)
    pts = np.minimum(pts, np.float32(box))
    path = str(tmp_path / "snap_010")
    io.write_gadget(path, pts, box, fmt=2, endian=">", num_files=2)
    allp, _, hdr = io.read_gadget(path)
    assert np.array_equal(allp, pts) and hdr["num_files"] == 2
    parts = _run(tmp_path, "gadget", path, box)
    _check(parts, allp, box, oracle)
