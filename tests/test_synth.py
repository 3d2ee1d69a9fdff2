"""Synthetic input generators of SURVEY.md §8(d) (host only)."""
import numpy as np

from nbodyhpc_amd import synth


def test_uniform_matches_bench_recipe():
    a = synth.uniform(1000, 5, 2.0)
    rng = np.random.Generator(np.random.PCG64(5))
    assert np.array_equal(a, rng.uniform(0.0, 2.0, size=(1000, 3)).astype(np.float32))


def test_lognormal_counts_box_and_determinism():
    n = 50_000
    a = synth.lognormal(n, grid=32, box=2.0)
    b = synth.lognormal(n, grid=32, box=2.0)
    assert a.shape == (n, 3) and a.dtype == np.float32
    assert np.array_equal(a, b)
    assert a.min() >= 0.0 and a.max() <= 2.0
    # clustered: the occupancy of 32^3 cells is far from Poisson
    c = np.floor(a / 2.0 * 32).clip(0, 31).astype(np.int64)
    occ = np.bincount((c[:, 0] * 32 + c[:, 1]) * 32 + c[:, 2], minlength=32 ** 3)
    mean = n / 32 ** 3
    assert occ.var() > 3 * mean  # Poisson: var == mean


def test_lognormal_weights_normalised():
    rng = np.random.Generator(np.random.PCG64(1))
    w = synth.lognormal_weights(32, rng, sigma=1.0)
    g = np.log(w) + 0.5
    assert abs(g.mean()) < 1e-6 and abs(g.std() - 1.0) < 1e-4


def _cell_hist(p, grid, box):
    c = np.floor(p.astype(np.float64) / box * grid).clip(0, grid - 1).astype(np.int64)
    return np.bincount((c[:, 0] * grid + c[:, 1]) * grid + c[:, 2], minlength=grid ** 3)


def test_plane_cuts_balanced_and_wide_enough():
    counts = np.array([0, 0, 50, 50, 0, 0, 0, 100, 0, 0], np.int64)
    cuts = synth.plane_cuts(counts, 2)
    assert cuts[0] == 0 and cuts[-1] == 10
    assert counts[:cuts[1]].sum() == 100
    cuts = synth.plane_cuts(counts, 4, min_planes=2)
    assert (np.diff(cuts) >= 2).all() and cuts[-1] == 10
    try:
        synth.plane_cuts(counts, 6, min_planes=2)
    except ValueError:
        pass
    else:
        raise AssertionError("6 slabs of 2 planes cannot fit 10 planes")


def test_lognormal_slab_union_has_lognormal_cell_counts():
    n, grid, box = 30_000, 16, 2.0
    ref = _cell_hist(synth.lognormal(n, grid=grid, box=box), grid, box)
    for world in (1, 3):
        parts = [synth.lognormal_slab(n, r, world, grid=grid, box=box, min_width=0.3)
                 for r in range(world)]
        bounds = parts[0][2]
        assert len(bounds) == world + 1 and bounds[0] == 0.0 and bounds[-1] == box
        assert all(p[2] == bounds for p in parts)
        assert (np.diff(bounds) >= 0.3 - 1e-6).all()
        for r, (xyz, ids, _) in enumerate(parts):
            assert xyz.dtype == np.float32 and ids.dtype == np.uint32
            assert (xyz[:, 0] >= np.float32(bounds[r])).all()
            assert (xyz[:, 0] < np.float32(bounds[r + 1])).all()
            assert (xyz >= 0).all() and (xyz <= box).all()
        allp = np.concatenate([p[0] for p in parts])
        allids = np.concatenate([p[1] for p in parts])
        assert np.array_equal(allids, np.arange(n, dtype=np.uint32))
        assert np.array_equal(_cell_hist(allp, grid, box), ref)
    # count-quantile cuts: no slab holds more than half the points (W = 3)
    assert max(len(p[1]) for p in parts) < n // 2
