"""Synthetic particle sets of SURVEY.md §8(d) (host side, numpy).

* ``uniform``: numpy ``Generator(PCG64(seed))``, ``uniform(0, L, (N, 3))`` cast
  to float32 (headline workload; points seed 20261015, queries 20261016).
* ``lognormal`` (config C5): a Gaussian random field g on a G^3 grid with power
  spectrum P(k) ~ k^slope (slope -2), zeroed above half the Nyquist wavenumber,
  normalised to sigma_g; delta = exp(g - sigma_g^2/2) - 1, cell weights
  w ~ 1 + delta; multinomial cell counts summing exactly to N; points uniform
  inside their cell; rows shuffled (so input order carries no locality, like
  the uniform set).  Seed ``PCG64(20261017)``.

These are generators of test and benchmark inputs, not part of the query path.
"""
from __future__ import annotations

import numpy as np

SEED_POINTS = 20261015
SEED_QUERIES = 20261016
SEED_LOGNORMAL = 20261017


def uniform(n: int, seed: int = SEED_POINTS, box: float = 1.0) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.empty((n, 3), np.float32)
    chunk = 1 << 24
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        out[s:e] = rng.uniform(0.0, box, size=(e - s, 3))
    return out


def lognormal_weights(grid: int, rng: np.random.Generator, sigma: float = 1.0,
                      slope: float = -2.0) -> np.ndarray:
    """Cell weights exp(g - sigma^2/2) of a log-normal field, float64 (grid^3,)."""
    try:
        import scipy.fft as fft
        kw = {"workers": -1}
    except ImportError:  # pragma: no cover
        fft = np.fft
        kw = {}
    white = rng.standard_normal((grid, grid, grid), dtype=np.float32)
    f = fft.rfftn(white, **kw)
    del white
    kx = np.fft.fftfreq(grid) * grid
    kz = np.fft.rfftfreq(grid) * grid
    k2 = (kx[:, None, None] ** 2 + kx[None, :, None] ** 2 + kz[None, None, :] ** 2)
    kmax = grid / 4.0  # half the Nyquist wavenumber (grid/2)
    amp = np.zeros_like(k2, dtype=np.float32)
    ok = (k2 > 0) & (k2 <= kmax * kmax)
    amp[ok] = np.power(k2[ok], slope / 4.0)  # sqrt(P(k)) = k^(slope/2)
    del k2, ok
    f *= amp
    del amp
    g = fft.irfftn(f, s=(grid, grid, grid), **kw).astype(np.float32)
    del f
    g -= g.mean()
    g *= sigma / g.std(dtype=np.float64)
    w = np.exp(g.astype(np.float64).ravel() - 0.5 * sigma * sigma)
    return w


def lognormal(n: int, seed: int = SEED_LOGNORMAL, box: float = 1.0, grid: int = 512,
              sigma: float = 1.0, slope: float = -2.0) -> np.ndarray:
    """N float32 points of the log-normal set, in [0, box]^3, shuffled."""
    rng = np.random.Generator(np.random.PCG64(seed))
    w = lognormal_weights(grid, rng, sigma, slope)
    counts = rng.multinomial(n, w / w.sum())
    del w
    cells = np.repeat(np.arange(grid ** 3, dtype=np.int64), counts)
    del counts
    cells = cells[rng.permutation(n)]
    h = box / grid
    out = np.empty((n, 3), np.float32)
    chunk = 1 << 24
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        c = cells[s:e]
        ijk = np.stack((c // (grid * grid), (c // grid) % grid, c % grid), axis=1)
        p = (ijk + rng.uniform(0.0, 1.0, size=(e - s, 3))) * h
        out[s:e] = np.minimum(p, box)  # f32 rounding may not exceed the box
    return out
