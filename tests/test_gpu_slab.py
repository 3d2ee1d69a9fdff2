"""Slab entry points of the C ABI on the GPU.

Single-GPU checks of strip selection, id remapping, the exactness check and
the RCCL exchange (a self-exchange on a world-size-1 communicator), plus a
world-size-2 slab kNN with both ranks on the one GPU of the box (halo staged
over gloo, since RCCL needs one GPU per rank) compared with the single-tree
oracle result.
"""
import os
import socket

import numpy as np
import pytest

from nbodyhpc_amd import slab

pytestmark = pytest.mark.gpu


def test_slab_select_stable(gpu):
    from nbodyhpc_amd import hip
    rng = np.random.default_rng(5)
    n = 50_001
    xyz = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    ids = rng.permutation(n).astype(np.uint32)
    dx, di = hip.DeviceArray.from_numpy(xyz), hip.DeviceArray.from_numpy(ids)
    lo, hi = 0.25, 0.3125
    c = gpu.slab_select(dx.ptr, di.ptr, n, lo, hi)
    m = (xyz[:, 0] >= np.float32(lo)) & (xyz[:, 0] < np.float32(hi))
    assert c == int(m.sum())
    ox, oi = hip.DeviceArray((c, 3), np.float32), hip.DeviceArray((c,), np.uint32)
    assert gpu.slab_select(dx.ptr, di.ptr, n, lo, hi, ox.ptr, oi.ptr, c) == c
    assert np.array_equal(ox.numpy(), xyz[m])
    assert np.array_equal(oi.numpy(), ids[m])
    with pytest.raises(gpu.NbkdError):
        gpu.slab_select(dx.ptr, di.ptr, n, lo, hi, ox.ptr, oi.ptr, c - 1)


def test_set_ids_maps_query_results(gpu):
    rng = np.random.default_rng(6)
    pts = rng.uniform(0, 1, (30_000, 3)).astype(np.float32)
    ids = (rng.permutation(30_000) + 1_000_000).astype(np.uint32)
    t = gpu.Tree(pts, leafsize=32, boxsize=1.0)
    d0, i0 = t.query(pts[:2000], 16)
    t.set_ids(ids)
    d1, i1 = t.query(pts[:2000], 16)
    assert np.array_equal(d0, d1)
    assert np.array_equal(i1, ids[i0])
    t.close()


def test_violations_kernel_matches_host(gpu):
    from nbodyhpc_amd import hip
    rng = np.random.default_rng(8)
    world, rank, box, k = 4, 1, 1.0, 4
    lo, hi = slab.slab_bounds(rank, world, box)
    m = 20_000
    q = rng.uniform(0, 1, (m, 3)).astype(np.float32)
    q[:, 0] = rng.uniform(lo, hi, m).astype(np.float32)
    dist = rng.uniform(0, 0.02, (m, k)).astype(np.float32)
    h = 0.01
    want = slab.violations_host(q, dist[:, -1], rank, world, box, h)
    assert 0 < want < m
    dq, dd = hip.DeviceArray.from_numpy(q), hip.DeviceArray.from_numpy(dist)
    got = gpu.slab_violations(dq.ptr, dd.ptr, m, k, lo, hi, h)
    assert got == want


def test_rccl_self_exchange(gpu):
    """dlopen of librccl, communicator init and a grouped send/recv (to self)."""
    from nbodyhpc_amd import hip
    uid = gpu.comm_unique_id()
    assert len(uid) == gpu.COMM_ID_BYTES
    comm = gpu.Comm(uid, 0, 1, 0)
    a = hip.DeviceArray.from_numpy(np.arange(1000, dtype=np.uint32))
    b = hip.DeviceArray((1000,), np.uint32)
    s = hip.Stream()
    comm.exchange([(a.ptr, 4000, 0, b.ptr, 4000, 0)], stream=s.handle)
    s.synchronize()
    assert np.array_equal(b.numpy(), np.arange(1000, dtype=np.uint32))
    comm.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_points(n_per, rank, world):
    """The last rank also owns particles exactly at x = L (slab_of,
    io.read_slab); periodically they sit at x = 0, in rank 0's domain."""
    xyz, ids = slab.gen_slab_points(n_per, 21, 1.0, rank, world)
    if rank == world - 1:
        xyz[:32, 0] = 1.0
    return xyz, ids


def _worker(rank, world, port, n_per, k, outdir, rccl=False, hscale=1.0, same_gpu=False):
    from nbodyhpc_amd import capi, hip

    hip.preload()  # the ROCm 7.2 runtime must load before torch's bundled one
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = rank if (rccl and not same_gpu) else 0
    try:
        hip.set_device(dev)
        xyz, ids = _rank_points(n_per, rank, world)
        comm = slab.init_comm(dist, rank, world, dev, log=slab.log_stderr) if rccl else None
        if rccl and comm is None:
            raise RuntimeError("RCCL communicator did not start")
        ds = slab.DeviceSlab(xyz, ids, rank, world, 1.0, dev, dist, comm=comm)
        h = slab.halo_width(n_per * world, k, 1.0) * hscale
        ds.exchange(h)
        # as the bench builds a rank's tree: split axes by the slab's extent,
        # the rows' k-th distances beside them for the forward test
        t = capi.Tree(n=ds.n_local, dev_ptr=ds.xyz.ptr, leafsize=32, boxsize=1.0, device=dev,
                      extent=ds.extent())
        t.set_ids(dev_ptr=ds.ids.ptr)
        side = hip.DeviceArray((n_per,), np.float32)
        t.set_kth_out(side.ptr, n_per)
        od = hip.DeviceArray((n_per, k), np.float32)
        oi = hip.DeviceArray((n_per, k), np.uint32)
        t.query_device(ds.xyz.ptr, n_per, k, od.ptr, oi.ptr)
        hip.synchronize()
        v = ds.violations(od.ptr, k)
        # second-round exchange (device forward test on the side array, as the
        # bench's pipelined step starts it; gather / scatter, RCCL or gloo)
        rows = slab.DeviceRows(ds, t, k, od.ptr, oi.ptr, side_ptr=side.ptr)
        rows.start(*slab.covered_range(ds.bounds, rank, ds.h))
        st = slab.second_round(rows, rank, world, ds.bounds, 1.0, ds.h, k, dist)
        hip.synchronize()
        # and the k-th-distance-only form of the same resolution
        rk = hip.DeviceArray((n_per,), np.float32)
        t.query_kth_device(ds.xyz.ptr, n_per, k, rk.ptr)
        slab.second_round(slab.DeviceRows(ds, t, k, kth_ptr=rk.ptr), rank, world, ds.bounds,
                          1.0, ds.h, k, dist)
        hip.synchronize()
        np.savez(os.path.join(outdir, f"r{rank}.npz"), d=od.numpy(), i=oi.numpy(), v=v,
                 nloc=ds.n_local, transport=ds.transport, fwd=st["rows_forwarded"],
                 sr_transport=rows.transport, rk=rk.numpy())
        t.close()
        if comm is not None:
            comm.close()
    finally:
        dist.destroy_process_group()


def _run_two_ranks(tmp_path, oracle, rccl, hscale=1.0, same_gpu=False):
    import multiprocessing as mp

    from tests.parity import assert_knn_equal
    world, n_per, k = 2, 60_000, 32
    ctx = mp.get_context("spawn")  # plain multiprocessing: torch must not load first
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_per, k, str(tmp_path), rccl,
                                               hscale, same_gpu))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    parts = [_rank_points(n_per, r, world)[0] for r in range(world)]
    allp = np.concatenate(parts)
    gd, gi = oracle.tree(allp, 32, 1.0).query(allp, k, workers=8)
    fwd = 0
    for r in range(world):
        res = np.load(os.path.join(tmp_path, f"r{r}.npz"))
        assert res["nloc"] > n_per
        assert int(res["fwd"]) == int(res["v"])
        fwd += int(res["fwd"])
        assert str(res["transport"]) == ("rccl" if rccl else "gloo-staged")
        assert str(res["sr_transport"]) == ("rccl" if rccl else "gloo")
        sl = slice(r * n_per, (r + 1) * n_per)
        assert_knn_equal(res["d"], res["i"], gd[sl], gi[sl], allp, parts[r], 1.0)
        assert np.array_equal(res["rk"], gd[sl][:, -1])
    assert (fwd > 0) == (hscale < 1.0)  # a thin halo leaves rows to the second round
    # the x = L particles of the last rank are rank 0's neighbours at x = 0
    assert np.isin(np.arange((world - 1) * n_per, (world - 1) * n_per + 32),
                   np.load(os.path.join(tmp_path, "r0.npz"))["i"]).any()


def test_two_rank_slab_knn_on_one_gpu(gpu, oracle, tmp_path):
    _run_two_ranks(tmp_path, oracle, rccl=False)


def test_two_rank_second_round_on_one_gpu(gpu, oracle, tmp_path):
    """SURVEY.md §8(e)(3) on the device path: a halo a tenth of the usual width
    leaves thousands of rows reaching past it; the second-round exchange
    (nbkd_slab_forward, the neighbour's NBKD_SQUARED kNN, merge, row scatter)
    makes every row and every k-th distance equal the single-tree result."""
    _run_two_ranks(tmp_path, oracle, rccl=False, hscale=0.1)


def test_two_rank_slab_knn_rccl(gpu, oracle, tmp_path):
    """The RCCL halo path proper: one GPU per rank, grouped ncclSend/ncclRecv
    with both ring neighbours being the same peer (W = 2), and the second round
    over RCCL.  Needs two GPUs."""
    if gpu.device_count() < 2:
        pytest.skip("the RCCL halo path needs two GPUs (one per rank)")
    _run_two_ranks(tmp_path, oracle, rccl=True)
    _run_two_ranks(tmp_path, oracle, rccl=True, hscale=0.1)


def _rccl_probe_worker(rank, world, port, outdir):
    from nbodyhpc_amd import hip

    hip.preload()  # as bench.py: the image's HIP runtime and RCCL before torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nbodyhpc_amd import capi

    msgs = []
    try:
        dev = rank if capi.device_count() >= world else 0
        hip.set_device(dev)
        comm = slab.init_comm(dist, rank, world, dev, log=msgs.append)
        maps = open("/proc/self/maps").read()
        rccl = sorted({ln.split()[-1] for ln in maps.splitlines() if "librccl" in ln})
        with open(os.path.join(outdir, f"p{rank}.txt"), "w") as f:
            f.write(f"comm={comm is not None}\n" + "\n".join(msgs) + "\nRCCL " + " ".join(rccl))
        if comm is not None:
            comm.close()
    finally:
        dist.destroy_process_group()


def test_rccl_starts_in_a_torch_process(gpu, tmp_path):
    """The RCCL the slab path drives must be the image's (bound to libnbkd's
    HIP runtime) even though torch, imported for gloo, brings its own librccl:
    that one calls torch's HIP runtime, which sees no device here, and
    ncclCommInitRank failed with 'unhandled cuda error' before any rank could
    meet.  On a one-GPU box two ranks then get past bootstrap and device
    detection to RCCL's duplicate-device check ('invalid usage'); with two
    GPUs the communicator starts."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rccl_probe_worker, args=(r, 2, port, str(tmp_path)))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for r in range(2):
        txt = open(os.path.join(tmp_path, f"p{r}.txt")).read()
        assert "/opt/rocm" in txt.split("RCCL", 1)[1], txt
        if gpu.device_count() >= 2:
            assert "comm=True" in txt, txt
        else:
            assert "comm=False" in txt and "invalid usage" in txt, txt


def test_forward_and_row_kernels_match_host(gpu):
    """nbkd_slab_forward == slab.side_needs (per side, f32); row gather / scatter."""
    from nbodyhpc_amd import hip
    rng = np.random.default_rng(9)
    m, k = 30_000, 8
    q = rng.uniform(0, 1, (m, 3)).astype(np.float32)
    q[:, 0] = rng.uniform(0.25, 0.5, m).astype(np.float32)
    dist = rng.uniform(0, 0.03, (m, k)).astype(np.float32)
    cl, ch = np.float32(0.24), np.float32(0.51)
    left, right = slab.side_needs(q[:, 0], dist[:, -1], cl, ch)
    want = np.nonzero(left | right)[0]
    dq, dd = hip.DeviceArray.from_numpy(q), hip.DeviceArray.from_numpy(dist)
    assert gpu.slab_forward(dq.ptr, dd.ptr, m, k, cl, ch) == len(want) > 0
    lst = hip.DeviceArray((len(want),), np.uint32)
    sides = hip.DeviceArray((len(want),), np.uint8)
    assert gpu.slab_forward(dq.ptr, dd.ptr, m, k, cl, ch, lst.ptr, sides.ptr, len(want)) == len(want)
    got, gs = lst.numpy(), sides.numpy()
    o = np.argsort(got)
    assert np.array_equal(got[o], want)
    assert np.array_equal(gs[o], (left[want] * 1 + right[want] * 2).astype(np.uint8))
    idx = rng.permutation(m)[:5000].astype(np.uint32)
    di = hip.DeviceArray.from_numpy(idx)
    g = hip.DeviceArray((5000, k), np.float32)
    gpu.rows_gather(dd.ptr, 4 * k, di.ptr, 5000, g.ptr)
    hip.synchronize()
    assert np.array_equal(g.numpy(), dist[idx])
    z = hip.DeviceArray.from_numpy(np.zeros((m, k), np.float32))
    gpu.rows_scatter(g.ptr, 4 * k, di.ptr, 5000, z.ptr)
    hip.synchronize()
    want_z = np.zeros((m, k), np.float32)
    want_z[idx] = dist[idx]
    assert np.array_equal(z.numpy(), want_z)


def test_bench_c5_line_small(gpu, oracle, monkeypatch, capsys):
    """bench.py --workload c5 in-process at a small size: the JSON line's
    radius counts and k-th densities agree with the oracle on the same
    log-normal set (synth.lognormal_slab, one rank)."""
    import json
    import sys

    import bench
    from nbodyhpc_amd import synth

    n, grid, r, k = 200_000, 32, 0.02, 8
    monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", "c5", "--particles", str(n),
                                      "--lognormal-grid", str(grid), "--radius", str(r),
                                      "--k", str(k), "--leafsize", "32", "--steps", "1",
                                      "--warmup", "0"])
    args = bench.parse()
    bench.run_c5(args, 0, 1, 0, None, False, lambda: None, lambda v: v, lambda v: v)
    line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["config"]["n_particles"] == n
    pts, _, _ = synth.lognormal_slab(n, 0, 1, grid=grid)
    t = oracle.tree(pts, 32, 1.0)
    cnt = oracle.ball_count(t, pts, r)
    assert abs(line["radius_count"]["mean_count"] - cnt.mean()) < 1e-6 * cnt.mean()
    d, _ = t.query(pts, k, workers=8)
    dens = k / (4.0 / 3.0 * np.pi * d[:, -1].astype(np.float64) ** 3) / n
    got = line["kth_density"]["mean_density_over_mean"]
    assert abs(got - dens.mean()) < 1e-6 * dens.mean()


def _deposit_worker(rank, world, port, n_per, grid, outdir):
    from nbodyhpc_amd import hip

    hip.preload()
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hip.set_device(0)
        xyz, w, r = _deposit_balls(n_per, rank, world)
        c0, part = slab.deposit_slab(xyz, w, r, rank, world, 1.0, grid, float(grid[0]), dist,
                                     device=0)
        np.savez(os.path.join(outdir, f"d{rank}.npz"), c0=c0, g=part)
    finally:
        dist.destroy_process_group()


def _deposit_balls(n_per, rank, world):
    xyz, _ = _rank_points(n_per, rank, world)
    rng = np.random.default_rng(200 + rank)
    r = rng.choice(np.array([0.003, 0.02, 0.06], np.float32), n_per)
    w = rng.uniform(0.5, 1.5, n_per).astype(np.float32)
    return xyz, w, r


def test_two_rank_slab_deposit_on_one_gpu(gpu, oracle, tmp_path):
    """SURVEY.md 8(f) rank 3 on the 8(e) slabs: two ranks (sharing the box's one
    GPU) deposit their balls plus the halo into their own grid columns with the
    HIP kernel; the two slabs tile the oracle's single deposit of all balls."""
    import multiprocessing as mp

    world, n_per, grid = 2, 3000, (64, 64, 64)
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_deposit_worker, args=(r, world, port, n_per, grid, str(tmp_path)))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    parts = [np.load(os.path.join(tmp_path, f"d{r}.npz")) for r in range(world)]
    assert [int(p["c0"]) for p in parts] == [0, 32]
    got = np.concatenate([p["g"] for p in parts], axis=0)
    balls = [_deposit_balls(n_per, r, world) for r in range(world)]
    xyz = np.concatenate([b[0] for b in balls])
    w = np.concatenate([b[1] for b in balls])
    r = np.concatenate([b[2] for b in balls])
    ref = oracle.deposit(xyz, w, r, grid, float(grid[0]), (1.0, 1.0, 1.0), 4)
    np.testing.assert_allclose(got, ref, rtol=2e-5, atol=1e-6 * float(ref.max()))


def _multihop_worker(rank, world, port, bounds, n, k, h, outdir):
    from nbodyhpc_amd import hip

    hip.preload()
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nbodyhpc_amd import capi, synth
        hip.set_device(0)
        allp = synth.uniform(n, 91, 1.0)
        mine = np.nonzero(slab.slab_of(allp[:, 0], bounds) == rank)[0]
        xyz, ids = allp[mine], mine.astype(np.uint32)
        own = len(xyz)
        ds = slab.DeviceSlab(xyz, ids, rank, world, 1.0, 0, dist, comm=None, bounds=bounds)
        ds.exchange(h)
        t = capi.Tree(n=ds.n_local, dev_ptr=ds.xyz.ptr, leafsize=32, boxsize=1.0, device=0)
        t.set_ids(dev_ptr=ds.ids.ptr)
        od = hip.DeviceArray((own, k), np.float32)
        oi = hip.DeviceArray((own, k), np.uint32)
        t.query_device(ds.xyz.ptr, own, k, od.ptr, oi.ptr)
        hip.synchronize()
        st = slab.second_round(slab.DeviceRows(ds, t, k, od.ptr, oi.ptr), rank, world, bounds,
                               1.0, ds.h, k, dist)
        rk = hip.DeviceArray((own,), np.float32)
        t.query_kth_device(ds.xyz.ptr, own, k, rk.ptr)
        hip.synchronize()
        slab.second_round(slab.DeviceRows(ds, t, k, kth_ptr=rk.ptr), rank, world, bounds, 1.0,
                          ds.h, k, dist)
        hip.synchronize()
        np.savez(os.path.join(outdir, f"m{rank}.npz"), ids=ids, d=od.numpy(), i=oi.numpy(),
                 rk=rk.numpy(), hops=st["hops"], fwd=st["rows_forwarded"])
        t.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bounds", [(3, [0.0, 0.45, 0.5, 1.0]),
                                          (4, [0.0, 0.3, 0.33, 0.36, 1.0])])
def test_multi_hop_second_round_on_one_gpu(gpu, oracle, tmp_path, world, bounds):
    """hops >= 2 of the second round on the device path
    (nbkd_slab_forward, rows gather / scatter, DeviceRows over gloo), W = 3
    and 4 ranks sharing the one GPU.  Slabs 0.03-0.05 wide and a halo of
    0.005 make rows near them reach two or three slabs away; every row and
    k-th distance equals the single-tree oracle."""
    import multiprocessing as mp

    from nbodyhpc_amd import synth
    from tests.parity import assert_knn_equal
    n, k, h = 30_000, 16, 0.005
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_multihop_worker, args=(r, world, port, bounds, n, k, h,
                                                        str(tmp_path)))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    allp = synth.uniform(n, 91, 1.0)
    gd, gi = oracle.tree(allp, 32, 1.0).query(allp, k, workers=16)
    hops = 0
    for r in range(world):
        x = np.load(os.path.join(tmp_path, f"m{r}.npz"))
        ids = x["ids"]
        assert_knn_equal(x["d"], x["i"], gd[ids], gi[ids], allp, allp[ids], 1.0)
        assert np.array_equal(x["rk"].view(np.uint32), gd[ids][:, -1].view(np.uint32))
        hops = max(hops, int(x["hops"]))
    assert hops >= 2


def _axes_for_extent(e, depth):
    """The greedy schedule of nbkd_build_ext (api.cpp axes_for_extent)."""
    x, out = [float(v) for v in e], []
    for _ in range(depth):
        k = 0
        if x[1] > x[k]:
            k = 1
        if x[2] > x[k]:
            k = 2
        out.append(k)
        x[k] *= 0.5
    return out


def _node_depths(nodes):
    depth = np.zeros(len(nodes), np.int64)
    for i, nd in enumerate(nodes):  # preorder: children after their parent
        if nd["dim"] >= 0:
            depth[nd["left"]] = depth[nd["right"]] = depth[i] + 1
    return depth


@pytest.mark.parametrize("box", [None, 1.0])
def test_extent_axes_slab_tree(gpu, oracle, box):
    """nbkd_build_ext (slab trees): every internal node splits the axis the
    extent schedule names for its depth, extent (1, 1, 1) reproduces
    nbkd_build's node table bit for bit, and kNN rows and radius counts equal
    those of the depth % 3 tree (and the oracle's) on a thin x-slab."""
    from nbodyhpc_amd import hip
    from tests.golden.inputs import uniform
    from tests.parity import assert_knn_equal
    rng = np.random.Generator(np.random.PCG64(95))
    pts = uniform(120_000, 94)
    pts[:, 0] = (0.30 + 0.15 * rng.random(len(pts))).astype(np.float32)
    ext = (0.15, 1.0, 1.0)
    t_ref = gpu.Tree(pts, leafsize=32, boxsize=box)
    t_ext = gpu.Tree(pts, leafsize=32, boxsize=box, extent=ext)
    t_cube = gpu.Tree(pts, leafsize=32, boxsize=box, extent=(1.0, 1.0, 1.0))
    n_ref, n_ext, n_cube = t_ref.export()[0], t_ext.export()[0], t_cube.export()[0]
    assert n_ref.tobytes() == n_cube.tobytes()
    depth = _node_depths(n_ext)
    sched = _axes_for_extent(ext, int(depth.max()) + 1)
    internal = n_ext["dim"] >= 0
    assert np.array_equal(n_ext["dim"][internal], np.array(sched)[depth[internal]])
    assert (n_ext["dim"][internal][:1] == 1).all()  # y first: the slab is thin in x
    leaves = ~internal
    assert np.array_equal(np.sort(n_ext["right"][leaves] - n_ext["left"][leaves]),
                          np.sort(n_ref["right"][~(n_ref["dim"] >= 0)]
                                  - n_ref["left"][~(n_ref["dim"] >= 0)]))
    k = 24
    dp = hip.DeviceArray.from_numpy(pts)
    t_dev = gpu.Tree(n=len(pts), dev_ptr=dp.ptr, leafsize=32, boxsize=box, extent=ext)
    od = hip.DeviceArray((len(pts), k), np.float32)
    oi = hip.DeviceArray((len(pts), k), np.uint32)
    s = hip.Stream()
    t_dev.query_device(dp.ptr, len(pts), k, od.ptr, oi.ptr, s.handle)  # self order
    s.synchronize()
    d0, i0 = t_ref.query(pts, k)
    for d, i in ((od.numpy(), oi.numpy()), t_ext.query(pts, k)):
        assert np.array_equal(d.view(np.uint32), d0.view(np.uint32))
        assert_knn_equal(d, i, d0, i0, pts, pts, box)
    q = uniform(20_000, 96)
    d1, i1 = t_ext.query(q, k)
    dr, ir = oracle.tree(pts, 32, box).query(q, k, workers=8)
    assert_knn_equal(d1, i1, dr, ir, pts, q, box)
    assert np.array_equal(t_ext.ball_count(pts, 0.01), t_ref.ball_count(pts, 0.01))


def test_extent_tree_rows_on_tie_heavy_lattice(gpu, oracle):
    """an extent-scheduled tree and the depth % 3 tree give
    identical distances on a lattice full of exact-distance ties; indices may
    differ only inside tied groups (assert_knn_equal checks them as sets)."""
    from tests.parity import assert_knn_equal
    g = np.arange(24, dtype=np.float32) / np.float32(24.0)
    xs, ys, zs = np.meshgrid(g * np.float32(0.25), g, g, indexing="ij")
    pts = np.stack([xs.ravel(), ys.ravel(), zs.ravel()], 1).astype(np.float32)
    k = 27
    t_ref = gpu.Tree(pts, leafsize=32, boxsize=1.0)
    t_ext = gpu.Tree(pts, leafsize=32, boxsize=1.0, extent=(0.25, 1.0, 1.0))
    q = pts[::7]
    d0, i0 = t_ref.query(q, k)
    d1, i1 = t_ext.query(q, k)
    assert np.array_equal(d1.view(np.uint32), d0.view(np.uint32))
    assert_knn_equal(d1, i1, d0, i0, pts, q, 1.0)
    dr, ir = oracle.tree(pts, 32, 1.0).query(q, k, workers=8)
    assert_knn_equal(d1, i1, dr, ir, pts, q, 1.0)
