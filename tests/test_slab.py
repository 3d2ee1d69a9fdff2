"""Slab decomposition (multi-GPU path) on the CPU.

World sizes 2 and 3 run as gloo process groups on 127.0.0.1: each rank
generates its slab, exchanges halo strips with exchange_host (the protocol the
RCCL path implements on device buffers), answers the kNN of its own particles
over own + halo with the C oracle (the checker), maps local rows to global ids
and must equal — tie-aware, bit-exact distances — the single-tree oracle
result over all particles.  A too-narrow halo must be flagged by the
exactness check.
"""
import os
import socket

import numpy as np
import pytest

from nbodyhpc_amd import slab


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _slab_points(n_per, seed, rank, world):
    """gen_slab_points, with a few particles of the last rank exactly at x = L:
    the last slab owns them (io.read_slab, slab_of), and periodically they sit
    at x = 0, inside rank 0's domain."""
    xyz, ids = slab.gen_slab_points(n_per, seed, 1.0, rank, world)
    if rank == world - 1:
        xyz[:5, 0] = 1.0
    return xyz, ids


def test_slab_bounds_partition_the_box():
    for world in (1, 2, 3, 8):
        bounds = [slab.slab_bounds(r, world, 1.0) for r in range(world)]
        assert bounds[0][0] == 0.0 and bounds[-1][1] == 1.0
        for (a, b), (c, d) in zip(bounds, bounds[1:]):
            assert b == c and a < b


def test_gen_slab_points_in_slab_and_ids():
    world = 4
    allids = []
    for r in range(world):
        xyz, ids = slab.gen_slab_points(5000, 3, 1.0, r, world)
        lo, hi = slab.slab_bounds(r, world, 1.0)
        assert xyz.dtype == np.float32 and xyz.shape == (5000, 3)
        assert (xyz[:, 0] >= np.float32(lo)).all() and (xyz[:, 0] < np.float32(hi)).all()
        assert (xyz[:, 1:] >= 0).all() and (xyz[:, 1:] < 1).all()
        allids.append(ids)
    allids = np.concatenate(allids)
    assert np.array_equal(allids, np.arange(world * 5000, dtype=np.uint32))


def test_halo_width_scales_with_density():
    h1 = slab.halo_width(1_000_000, 32, 1.0)
    h8 = slab.halo_width(8_000_000, 32, 1.0)
    assert abs(h1 / h8 - 2.0) < 1e-9


def _worker(rank, world, port, n_per, k, hscale, outdir):
    import torch.distributed as dist

    from oracle.oracle import Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        xyz, ids = _slab_points(n_per, 11, rank, world)
        h = slab.halo_width(n_per * world, k, 1.0) * hscale
        lx, li = slab.exchange_host(xyz, ids, rank, world, 1.0, h, dist)
        tree = Oracle().tree(lx, 16, 1.0)
        d, i = tree.query(xyz, k, workers=1)
        gi = li[i]
        v = slab.violations_host(xyz, d[:, -1], rank, world, 1.0, h)
        np.savez(os.path.join(outdir, f"r{rank}.npz"), d=d, i=gi, v=v, nloc=len(lx))
    finally:
        dist.destroy_process_group()


def _run_world(world, n_per, k, hscale, tmp_path):
    import torch.multiprocessing as mp

    port = _free_port()
    mp.start_processes(_worker, args=(world, port, n_per, k, hscale, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    res = [np.load(os.path.join(tmp_path, f"r{r}.npz")) for r in range(world)]
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_slab_knn_equals_single_tree(world, tmp_path, oracle):
    from tests.parity import assert_knn_equal

    n_per, k = 4000, 8
    # h = 1.5 x halo_width: inside the two-rank limit (2h <= slab width)
    res = _run_world(world, n_per, k, 1.5, tmp_path)
    parts = [_slab_points(n_per, 11, r, world)[0] for r in range(world)]
    allp = np.concatenate(parts)
    gd, gi = oracle.tree(allp, 16, 1.0).query(allp, k, workers=4)
    for r in range(world):
        assert int(res[r]["v"]) == 0
        assert res[r]["nloc"] > n_per  # received a halo
        sl = slice(r * n_per, (r + 1) * n_per)
        assert_knn_equal(res[r]["d"], res[r]["i"], gd[sl], gi[sl], allp, parts[r], 1.0)


def test_narrow_halo_is_flagged(tmp_path):
    res = _run_world(2, 4000, 8, 0.05, tmp_path)
    assert sum(int(r["v"]) for r in res) > 0


def _c5_worker(rank, world, port, n, grid, r, k, outdir):
    """Config C5 in miniature: log-normal slabs at count-quantile cuts, one
    halo of width max(ball_halo(r), kNN halo) serving the radius count and the
    k-th distance (widened until no row reaches past it)."""
    import torch.distributed as dist

    from nbodyhpc_amd import synth
    from oracle.oracle import Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        h_r = slab.ball_halo(r, 1.0)
        xyz, ids, bounds = synth.lognormal_slab(n, rank, world, grid=grid, min_width=4 * h_r)
        h = max(h_r, slab.halo_width(n, k, 1.0))
        orc = Oracle()
        for _ in range(6):
            lx, li = slab.exchange_host(xyz, ids, rank, world, 1.0, h, dist, bounds=bounds)
            tree = orc.tree(lx, 16, 1.0)
            d, i = tree.query(xyz, k, workers=1)
            v = slab.violations_host(xyz, d[:, -1], rank, world, 1.0, h, bounds=bounds)
            import torch
            t = torch.tensor([v], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            if int(t[0]) == 0:
                break
            try:
                slab.check_halo(2 * h, bounds)
            except ValueError:
                break
            h *= 2
        cnt = orc.ball_count(tree, xyz, r)
        np.savez(os.path.join(outdir, f"c5r{rank}.npz"), d=d, i=li[i], v=v, cnt=cnt, xyz=xyz,
                 ids=ids, h=h, nloc=len(lx))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_lognormal_slab_radius_and_knn_equal_single_tree(world, tmp_path, oracle):
    """Radius counts of every particle and its kNN rows, computed per slab over
    own + halo, equal the single-tree (brute-force for counts) results over
    the union of all slabs."""
    import torch.multiprocessing as mp

    from tests.parity import assert_knn_equal

    n, grid, r, k = 12_000, 16, 0.04, 8
    port = _free_port()
    mp.start_processes(_c5_worker, args=(world, port, n, grid, r, k, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    res = [np.load(os.path.join(tmp_path, f"c5r{q}.npz")) for q in range(world)]
    allp = np.concatenate([x["xyz"] for x in res])
    ids = np.concatenate([x["ids"] for x in res])
    assert np.array_equal(ids, np.arange(n, dtype=np.uint32))
    cnt = oracle.ball_count_brute(allp, allp, r, 1.0)
    gd, gi = oracle.tree(allp, 16, 1.0).query(allp, k, workers=4)
    o = 0
    for x in res:
        m = len(x["ids"])
        assert x["nloc"] > m  # received a halo
        assert np.array_equal(x["cnt"], cnt[o:o + m])
        assert int(x["v"]) == 0
        assert_knn_equal(x["d"], x["i"], gd[o:o + m], gi[o:o + m], allp, x["xyz"], 1.0)
        o += m


def test_halo_wider_than_a_slab_is_refused():
    with pytest.raises(ValueError):
        slab.check_halo(0.3, [0.0, 0.5, 1.0])  # two ranks: 2h > width
    slab.check_halo(0.25, [0.0, 0.5, 1.0])
    with pytest.raises(ValueError):
        slab.check_halo(0.2, [0.0, 0.1, 0.6, 1.0])


def _redist_worker(rank, world, port, n, outdir, quantile):
    import torch.distributed as dist

    from nbodyhpc_amd import synth

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pts = synth.uniform(n, 77, 1.0)
        pts[:7, 0] = 1.0  # points exactly at L belong to the last slab
        bounds = [0.0, 0.1, 0.75, 1.0] if quantile else None  # quantile: world 3
        # arbitrary (file-row) chunks, not slabs
        lo, hi = rank * n // world, (rank + 1) * n // world
        ids = np.arange(lo, hi, dtype=np.uint32)
        ox, oi = slab.redistribute(pts[lo:hi], ids, rank, world, 1.0, dist, bounds=bounds)
        np.savez(os.path.join(outdir, f"rd{rank}.npz"), x=ox, i=oi)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,quantile", [(2, False), (3, False), (3, True)])
def test_redistribute_to_slab_owners(world, quantile, tmp_path):
    """All-to-all-v of contiguous row chunks: every particle arrives at the
    owner of its x, exactly once, with its global id."""
    import torch.multiprocessing as mp

    from nbodyhpc_amd import synth

    n = 20_000
    port = _free_port()
    mp.start_processes(_redist_worker, args=(world, port, n, str(tmp_path), quantile),
                       nprocs=world, join=True, start_method="spawn")
    pts = synth.uniform(n, 77, 1.0)
    pts[:7, 0] = 1.0
    bounds = slab.bounds_list(world, 1.0) if not quantile else [0.0, 0.1, 0.75, 1.0]
    owner = slab.slab_of(pts[:, 0], bounds)
    seen = np.zeros(n, np.int64)
    for r in range(world):
        res = np.load(os.path.join(tmp_path, f"rd{r}.npz"))
        assert np.array_equal(res["x"], pts[res["i"]])
        assert (owner[res["i"]] == r).all()
        assert (res["x"][:, 0] >= np.float32(bounds[r])).all()
        seen[res["i"]] += 1
    assert (seen == 1).all()
    assert (owner[:7] == world - 1).all()


def _agree_worker(rank, world, port, fail_ranks, outdir):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def enqueue():
            if rank in fail_ranks:
                raise RuntimeError("enqueue failed")
        try:
            err = slab._enqueue_agreed(dist, rank, "test", enqueue)
            out = "ok" if err is None else "fallback"
        except RuntimeError:
            out = "raised"
        with open(os.path.join(outdir, f"a{rank}.txt"), "w") as f:
            f.write(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail_ranks,want", [((), "ok"), ((0, 1), "fallback"),
                                             ((1,), "raised")])
def test_rccl_fallback_is_agreed_by_every_rank(fail_ranks, want, tmp_path):
    """The RCCL -> gloo fallback is taken only when every rank failed to
    enqueue; a partial failure raises on every rank instead of mixing
    transports (a peer with queued sends would otherwise deadlock)."""
    import torch.multiprocessing as mp

    port = _free_port()
    mp.start_processes(_agree_worker, args=(2, port, fail_ranks, str(tmp_path)), nprocs=2,
                       join=True, start_method="spawn")
    got = [open(os.path.join(tmp_path, f"a{r}.txt")).read() for r in range(2)]
    assert got == [want, want]


def test_violations_absolute_slack_for_thin_halos():
    """When h << L the relative slack is below one ulp of x: a k-th distance
    within a few ulps of the domain face must still be flagged."""
    world, rank, box = 2, 1, 1.0
    lo, hi = slab.slab_bounds(rank, world, box)
    h = 1e-6
    x = np.float32(0.75)
    q = np.array([[x, 0.5, 0.5]], np.float32)
    face = np.float32(np.float32(hi) + np.float32(h)) - x
    near = np.float32(face) - np.float32(2.0) * np.spacing(np.float32(1.0))
    assert slab.violations_host(q, np.array([near], np.float32), rank, world, box, h) == 1
    ok = np.float32(face) * np.float32(0.5)
    assert slab.violations_host(q, np.array([ok], np.float32), rank, world, box, h) == 0


# ------------------------------------------------------------ deposit per slab
def _deposit_worker(rank, world, port, n_per, grid, outdir):
    """deposit_slab's decomposition (payload halo + column windows) with the
    oracle as the deposit (full grid, then this rank's columns): the checker
    stands in for nbkd_deposit here; tests/test_gpu_slab.py runs the HIP one."""
    import torch.distributed as dist

    from oracle.oracle import Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        xyz, w, r = _deposit_balls(n_per, rank, world)
        orc = Oracle()

        def engine(bx, bw, br, g, ppu, period, S, window):
            full = orc.deposit(bx, bw, br, g, ppu, period, S)
            return full[window[0]:window[0] + window[1]]
        c0, part = slab.deposit_slab(xyz, w, r, rank, world, 1.0, grid, float(grid[0]), dist,
                                     engine=engine)
        np.savez(os.path.join(outdir, f"d{rank}.npz"), c0=c0, g=part)
    finally:
        dist.destroy_process_group()


def _deposit_balls(n_per, rank, world):
    xyz, _ = _slab_points(n_per, 31, rank, world)
    rng = np.random.default_rng(100 + rank)
    r = rng.choice(np.array([0.01, 0.04, 0.09], np.float32), n_per)
    w = rng.uniform(0.5, 1.5, n_per).astype(np.float32)
    return xyz, w, r


@pytest.mark.parametrize("world", [2, 3])
def test_deposit_slabs_tile_the_single_deposit(world, tmp_path, oracle):
    """Each rank's column window, deposited from its own balls plus the halo,
    equals those columns of the single deposit of all balls; the windows tile
    the grid, so their concatenation is the whole grid."""
    import torch.multiprocessing as mp

    n_per, grid = 150, (24, 24, 24)
    port = _free_port()
    mp.start_processes(_deposit_worker, args=(world, port, n_per, grid, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    parts = [np.load(os.path.join(tmp_path, f"d{r}.npz")) for r in range(world)]
    got = np.concatenate([p["g"] for p in parts], axis=0)
    assert [int(p["c0"]) for p in parts] == slab.grid_columns(world, grid[0], grid[0],
                                                              slab.bounds_list(world, 1.0))[:-1]
    balls = [_deposit_balls(n_per, r, world) for r in range(world)]
    xyz = np.concatenate([b[0] for b in balls])
    w = np.concatenate([b[1] for b in balls])
    r = np.concatenate([b[2] for b in balls])
    ref = oracle.deposit(xyz, w, r, grid, float(grid[0]), (1.0, 1.0, 1.0), 4)
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-12)
    assert abs(got.sum() - w.sum()) < 0.01 * w.sum()


def _comm_worker(rank, world, port, fail_rank, fail_uid, outdir):
    import torch.distributed as dist

    from nbodyhpc_amd import capi

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls, uids = [], []
    try:
        def probe():
            if rank == fail_rank:
                raise RuntimeError("cannot load librccl.so.1 (test)")

        def uid():
            uids.append(rank)
            if fail_uid:
                raise RuntimeError("ncclGetUniqueId failed (test)")
            return bytes(capi.COMM_ID_BYTES)

        class NoInit:  # must never be reached when some rank lacks RCCL
            def __init__(self, *a):
                calls.append(a)
                raise AssertionError("ncclCommInitRank entered")

        capi.comm_probe, capi.comm_unique_id, capi.Comm = probe, uid, NoInit
        c = slab.init_comm(dist, rank, world, 0)
        np.savez(os.path.join(outdir, f"c{rank}.npz"), none=c is None, init_calls=len(calls),
                 uid_calls=len(uids))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_rank,fail_uid", [(2, 1, False), (3, 0, False), (3, -1, True)])
def test_init_comm_agrees_before_rccl_init(world, fail_rank, fail_uid, tmp_path):
    """slab.init_comm: ncclCommInitRank blocks until every rank joins, so a rank
    that cannot load RCCL (or a failed unique id on rank 0) must stop all ranks
    before any enters it (gloo, CPU).  Only rank 0 creates the unique id: each
    ncclGetUniqueId starts a bootstrap listener that only rank 0's id uses."""
    import torch.multiprocessing as mp

    port = _free_port()
    mp.start_processes(_comm_worker, args=(world, port, fail_rank, fail_uid, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    for r in range(world):
        res = np.load(os.path.join(tmp_path, f"c{r}.npz"))
        assert bool(res["none"]) and int(res["init_calls"]) == 0, r
        assert int(res["uid_calls"]) == (1 if (r == 0 and fail_rank < 0) else 0), r


# ------------------------------------------------ second-round exchange (§8(e)(3))
def _sr_worker(rank, world, port, n, k, hscale, kind, outdir):
    """A deliberately thin halo (h << the k-th neighbour radius): the slab-local
    rows reaching past the covered x-range are forwarded to the neighbours and
    merged (slab.second_round, gloo transport, the oracle as the local kNN)."""
    import torch.distributed as dist

    from nbodyhpc_amd import synth
    from oracle.oracle import Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if kind == "lognormal":
            xyz, ids, bounds = synth.lognormal_slab(n, rank, world, grid=16)
        elif kind == "strong":
            # bench.py's strong split: every rank draws the one-GPU set and
            # keeps its own slab (ids = row numbers of synth.uniform)
            xyz, ids = slab.gen_uniform_slab(n, 20261016, 1.0, rank, world)
            bounds = slab.bounds_list(world, 1.0)
        else:
            xyz, ids = _slab_points(n // world, 17, rank, world)
            bounds = slab.bounds_list(world, 1.0)
        h = slab.halo_width(n, k, 1.0) * hscale
        lx, li = slab.exchange_host(xyz, ids, rank, world, 1.0, h, dist, bounds=bounds)
        tree = Oracle().tree(lx, 16, 1.0)

        def gids(i):
            return np.where(i == 0xFFFFFFFF, np.uint32(0xFFFFFFFF),
                            li[np.minimum(i, len(li) - 1)]).astype(np.uint32)

        def knn_sq(q):
            d2, i = tree.query(q, k, sqrt=False)
            return d2, gids(i)

        d, i = tree.query(xyz, k)
        gi = gids(i)
        v0 = slab.violations_host(xyz, d[:, -1], rank, world, 1.0, h, bounds=bounds)
        be = slab.HostRows(xyz, d, gi, knn_sq, k, dist, rank, world)
        st = slab.second_round(be, rank, world, bounds, 1.0, h, k, dist)
        np.savez(os.path.join(outdir, f"sr{rank}.npz"), d=d, i=gi, xyz=xyz, ids=ids, v0=v0,
                 nloc=len(lx), fwd=st["rows_forwarded"], hops=st["hops"])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,k,hscale,kind", [
    (2, 8000, 8, 0.05, "uniform"), (3, 9000, 8, 0.05, "uniform"),
    (4, 400, 48, 0.02, "uniform"),  # k-th radii wider than a slab: hops to the 2nd neighbour
    (2, 12_000, 8, 0.1, "lognormal"), (3, 12_000, 16, 0.1, "lognormal"),
    (2, 20_000, 32, 1.0, "strong"), (3, 30_000, 32, 0.1, "strong")])
def test_second_round_exchange_equals_single_tree(world, n, k, hscale, kind, tmp_path, oracle):
    """with a thin halo many slab-local rows are not exact;
    after the second-round exchange every row equals the single-tree oracle
    over all particles (tie-aware, bit-exact distances) - no rebuild, no
    halo widening."""
    import torch.multiprocessing as mp

    from tests.parity import assert_knn_equal

    port = _free_port()
    mp.start_processes(_sr_worker, args=(world, port, n, k, hscale, kind, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    res = [np.load(os.path.join(tmp_path, f"sr{r}.npz")) for r in range(world)]
    allp = np.concatenate([x["xyz"] for x in res])
    ids = np.concatenate([x["ids"] for x in res])
    pts = np.empty_like(allp)
    pts[ids] = allp  # global id order
    gd, gi = oracle.tree(pts, 16, 1.0).query(pts, k, workers=4)
    if kind == "strong":
        # the ranks' rows tile the one-GPU problem: every row of synth.uniform once
        from nbodyhpc_amd import synth
        assert np.array_equal(np.sort(ids), np.arange(n, dtype=np.uint32))
        assert np.array_equal(pts, synth.uniform(n, 20261016, 1.0))
    if hscale < 1.0:
        assert sum(int(x["v0"]) for x in res) > 0  # the thin halo did leave rows inexact
    assert sum(int(x["fwd"]) for x in res) == sum(int(x["v0"]) for x in res)
    if world == 4:
        assert max(int(x["hops"]) for x in res) >= 2
    for x in res:
        assert_knn_equal(x["d"], x["i"], gd[x["ids"]], gi[x["ids"]], pts, x["xyz"], 1.0)


def test_merge_rows_dedups_and_pads():
    f = np.float32
    a_d = np.array([[0.0, 1.0, 4.0, f(np.finfo(f).max)]], f)
    a_i = np.array([[5, 7, 9, 0xFFFFFFFF]], np.uint32)
    b_d = np.array([[1.0, 2.0, 4.0, 9.0]], f)
    b_i = np.array([[7, 3, 8, 11]], np.uint32)  # 7 is the same particle as in a
    d, i = slab.merge_rows(a_d, a_i, b_d, b_i, 4)
    assert d.tolist() == [[0.0, 1.0, 2.0, 4.0]]
    assert i.tolist() == [[5, 7, 3, 8]]  # equal d2 4.0: the smaller id first
    d, i = slab.merge_rows(a_d[:, :2], a_i[:, :2], a_d[:, :1], a_i[:, :1], 4)
    assert i.tolist() == [[5, 7, 0xFFFFFFFF, 0xFFFFFFFF]]
    assert d[0, 2] == np.finfo(f).max


def test_side_needs_matches_violations_host():
    rng = np.random.default_rng(3)
    world, rank, box, h = 3, 1, 1.0, 0.02
    lo, hi = slab.slab_bounds(rank, world, box)
    x = rng.uniform(lo, hi, 5000).astype(np.float32)
    q = np.stack([x, x, x], 1)
    dk = rng.uniform(0, 0.1, 5000).astype(np.float32)
    f32 = np.float32
    left, right = slab.side_needs(x, dk, f32(f32(lo) - f32(h)), f32(f32(hi) + f32(h)))
    assert int((left | right).sum()) == slab.violations_host(q, dk, rank, world, box, h)


def test_merge_rows_dedupes_by_id_even_when_d2_differs():
    """One particle returned by two trees with d2 one ulp apart: only the
    smaller copy survives, so it cannot push the true k-th neighbour out."""
    k = 3
    d_a = np.array([[0.1, 0.2, 0.3]], np.float32)
    i_a = np.array([[7, 8, 9]], np.uint32)
    bump = np.nextafter(np.float32(0.2), np.float32(1.0))
    d_b = np.array([[bump, 0.25, 0.5]], np.float32)
    i_b = np.array([[8, 11, 12]], np.uint32)
    od, oi = slab.merge_rows(d_a, i_a, d_b, i_b, k)
    assert oi.tolist() == [[7, 8, 11]]
    assert od[0].tolist() == [np.float32(0.1), np.float32(0.2), np.float32(0.25)]
