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
        xyz, ids = slab.gen_slab_points(n_per, 11, 1.0, rank, world)
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
    res = _run_world(world, n_per, k, 2.5, tmp_path)
    parts = [slab.gen_slab_points(n_per, 11, 1.0, r, world)[0] for r in range(world)]
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
