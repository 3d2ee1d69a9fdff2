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
