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


def plane_cuts(plane_counts: np.ndarray, world: int, min_planes: int = 1) -> np.ndarray:
    """W + 1 grid-plane indices cutting the x planes into W slabs of nearly
    equal particle count (boundaries at count quantiles),
    each at least `min_planes` planes wide."""
    g = len(plane_counts)
    if world * min_planes > g:
        raise ValueError(f"{world} slabs of >= {min_planes} planes do not fit {g} planes")
    cum = np.concatenate([[0], np.cumsum(plane_counts, dtype=np.int64)])
    total = int(cum[-1])
    cuts = [0]
    for j in range(1, world):
        c = int(np.searchsorted(cum, total * j / world))
        c = max(c, cuts[-1] + min_planes)            # room behind
        c = min(c, g - (world - j) * min_planes)     # room ahead
        cuts.append(c)
    cuts.append(g)
    return np.asarray(cuts, np.int64)


def lognormal_slab(n: int, rank: int, world: int, seed: int = SEED_LOGNORMAL, box: float = 1.0,
                   grid: int = 512, sigma: float = 1.0, slope: float = -2.0,
                   min_width: float = 0.0):
    """Rank `rank`'s x-slab of the log-normal set of N points (config C5 on W
    GPUs).  Every rank draws the same field and the same multinomial cell
    counts as ``lognormal`` (same seed, same draws), cuts the x planes at count
    quantiles (``plane_cuts``), and places only the points of its own cells,
    uniformly inside each cell (placement stream PCG64([seed, 1 + rank])).  The
    union over ranks has exactly ``lognormal``'s per-cell counts.

    Returns (xyz float32 (n_own, 3), global ids uint32 (n_own,), bounds): ids
    are the cell-ordered positions of the points over all slabs; bounds are the
    W + 1 slab cuts in x (float32 values), for slab.DeviceSlab(bounds=...).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    w = lognormal_weights(grid, rng, sigma, slope)
    counts = rng.multinomial(n, w / w.sum())
    del w
    g2 = grid * grid
    h = box / grid
    plane = counts.reshape(grid, g2).sum(axis=1)
    min_planes = max(1, int(np.ceil(min_width / h)))
    cuts = plane_cuts(plane, world, min_planes)
    bounds = [float(np.float32(box * c / grid)) for c in cuts[:-1]] + [float(np.float32(box))]
    a, b = int(cuts[rank]), int(cuts[rank + 1])
    first = int(plane[:a].sum())
    n_own = int(plane[a:b].sum())
    if first + n_own > 0xFFFFFFFF:
        raise ValueError("global ids exceed uint32")
    cells = np.repeat(np.arange(a * g2, b * g2, dtype=np.int64), counts[a * g2:b * g2])
    del counts
    lo32 = np.float32(bounds[rank])
    top = np.nextafter(np.float32(bounds[rank + 1]), np.float32(-np.inf))
    prng = np.random.Generator(np.random.PCG64([seed, 1 + rank]))
    out = np.empty((n_own, 3), np.float32)
    chunk = 1 << 24
    for s in range(0, n_own, chunk):
        e = min(n_own, s + chunk)
        c = cells[s:e]
        ijk = np.stack((c // g2, (c // grid) % grid, c % grid), axis=1)
        p = ((ijk + prng.uniform(0.0, 1.0, size=(e - s, 3))) * h).astype(np.float32)
        out[s:e, 0] = np.clip(p[:, 0], lo32, top)
        out[s:e, 1:] = np.minimum(p[:, 1:], np.float32(box))
    ids = (np.uint64(first) + np.arange(n_own, dtype=np.uint64)).astype(np.uint32)
    return out, ids, bounds
