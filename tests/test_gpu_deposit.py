"""GPU parity of the sphere deposit (nbodyhpc.rasterizer on the HIP kernel,
nbodyhpc_amd/csrc/deposit.hip) against the oracle's restatement of the
reference's rasteriser (oracle/deposit_oracle.c).

Every per-voxel decision (sprite coverage, clip, snap, sub-sample count) is
exact, so a wrong decision shows up as at least weight / S^3 / volume in one
voxel; what remains is the order of the float32 atomic additions, bounded here
by rtol 2e-5 plus an absolute 1e-6 of the grid's largest value.  The
reference's own Vulkan output cannot be produced in this image (no Vulkan
device), so the oracle itself is "parity unpinned" against it
(tests/test_deposit_oracle.py pins it to a numpy restatement and to physical
properties).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

f32 = np.float32
RTOL, ATOL_FRAC = 2e-5, 1e-6


def _close(got, ref):
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL_FRAC * max(float(np.abs(ref).max()), 1e-30))


def _ras():
    from nbodyhpc import rasterizer
    return rasterizer


def _particles(rng, n, box, radii):
    xyz = (rng.uniform(0, 1, (n, 3)) * np.asarray(box)).astype(f32)
    r = rng.choice(np.asarray(radii, f32), n).astype(f32)
    w = rng.uniform(0.5, 2.0, n).astype(f32)
    return xyz, w, r


@pytest.mark.parametrize("periodic", [False, True])
def test_volume_mixed_radii(gpu, oracle, periodic):
    rng = np.random.default_rng(11 + periodic)
    grid, ppu = (40, 33, 29), 4.0
    box = np.array(grid) / ppu
    # sub-voxel, about a voxel, a few voxels, and balls half the box across
    xyz, w, r = _particles(rng, 400, box, [0.05, 0.2, 0.5, 1.3, 2.5])
    got = _ras().render_points_volume(xyz, w, r, ppu, grid, periodic=periodic)
    period = tuple(box) if periodic else (-1.0, -1.0, -1.0)
    _close(got, oracle.deposit(xyz, w, r, grid, ppu, period, 4, 0))


@pytest.mark.parametrize("S", [1, 2, 3, 5, 6])
def test_subsample_factors(gpu, oracle, S):
    """Templated S = 1..5 and the generic runtime-S kernel (S = 6)."""
    rng = np.random.default_rng(20 + S)
    grid, ppu = (24, 24, 24), 3.0
    box = np.array(grid) / ppu
    xyz, w, r = _particles(rng, 200, box, [0.1, 0.6, 1.5])
    got = _ras().render_points_volume(xyz, w, r, ppu, grid, periodic=True, subsample_factor=S)
    _close(got, oracle.deposit(xyz, w, r, grid, ppu, tuple(box), S, 0))


def test_render_points_plane(gpu, oracle):
    rng = np.random.default_rng(31)
    grid, ppu = (50, 37), 5.0
    n = 400
    xyz = np.empty((n, 3), f32)
    xyz[:, 0] = rng.uniform(0, grid[0] / ppu, n)
    xyz[:, 1] = rng.uniform(0, grid[1] / ppu, n)
    xyz[:, 2] = rng.uniform(-1.0, 1.0, n)
    r = rng.choice(np.array([0.05, 0.3, 0.9], f32), n)
    w = rng.uniform(0.5, 2.0, n).astype(f32)
    got = _ras().render_points(xyz, w, r, ppu, grid, periodic=True)
    assert got.shape == grid
    period = (grid[0] / ppu, grid[1] / ppu, -1.0)
    ref = oracle.deposit(xyz, w, r, (grid[0], grid[1], 1), ppu, period, 4, 1)[:, :, 0]
    _close(got, ref)


def test_edges_outside_and_boundaries(gpu, oracle):
    """Centres outside the grid, exactly on voxel faces and box faces, zero and
    negative radii, zero weights."""
    grid, ppu = (16, 12, 10), 2.0
    box = np.array(grid) / ppu
    pts = [[-1.0, 2.0, 2.0], [9.5, 3.0, 2.5], [8.0, 6.0, 5.0], [0.0, 0.0, 0.0], [0.5, 0.5, 0.5],
           [4.0, 3.0, 2.0], [8.0, 3.0, 4.75], [2.25, -0.3, 5.2], [3.0, 3.0, 3.0], [7.9, 5.9, 4.9]]
    xyz = np.array(pts, f32)
    r = np.array([1.0, 2.5, 0.3, 0.0, -0.2, 0.25, 3.0, 0.8, 1.0, 0.6], f32)
    w = np.array([1.0, 2.0, 0.5, 1.0, 1.0, 1.5, 1.0, 1.0, 0.0, 1.0], f32)
    for periodic in (False, True):
        got = _ras().render_points_volume(xyz, w, r, ppu, grid, periodic=periodic)
        period = tuple(box) if periodic else (-1.0, -1.0, -1.0)
        _close(got, oracle.deposit(xyz, w, r, grid, ppu, period, 4, 0))


@pytest.mark.parametrize("periodic", [False, True])
def test_balls_spanning_many_tiles(gpu, oracle, periodic):
    """Balls whose sprite box covers more than 64 of the 32 x 32 x 8 tiles are
    listed by the whole wave (deposit_pairs_kernel's cooperative path)."""
    grid, ppu = (96, 80, 48), 1.0
    box = np.array(grid, np.float64)
    xyz = np.array([[40.0, 30.0, 20.0], [90.0, 5.0, 45.0], [10.5, 70.2, 3.3]], f32)
    r = np.array([45.0, 30.0, 6.0], f32)
    w = np.array([1.0, 2.0, 0.5], f32)
    got = _ras().render_points_volume(xyz, w, r, ppu, grid, periodic=periodic)
    period = tuple(box) if periodic else (-1.0, -1.0, -1.0)
    _close(got, oracle.deposit(xyz, w, r, grid, ppu, period, 4, 0))


def test_column_windows(gpu, oracle):
    """nbkd_deposit's column window (one rank's x-slab): each window equals those
    columns of the whole periodic grid, balls wrapping across x = 0 included."""
    from nbodyhpc_amd import capi
    rng = np.random.default_rng(51)
    grid, ppu = (40, 24, 16), 4.0
    box = np.array(grid) / ppu
    xyz, w, r = _particles(rng, 300, box, [0.1, 0.6, 1.8])
    ref = oracle.deposit(xyz, w, r, grid, ppu, tuple(box), 4, 0)
    for x0, wx in ((0, 40), (0, 13), (13, 14), (27, 13), (39, 1)):
        got = capi.deposit(xyz, w, r, grid, ppu, period=tuple(box), window=(x0, wx))
        assert got.shape == (wx, 24, 16)
        _close(got, ref[x0:x0 + wx])


def test_empty_and_accumulate(gpu, oracle):
    from nbodyhpc_amd import capi
    e = np.zeros((0, 3), f32)
    g = _ras().render_points_volume(e, np.zeros(0, f32), np.zeros(0, f32), 1.0, 8)
    assert g.shape == (8, 8, 8) and not g.any()
    rng = np.random.default_rng(41)
    xyz, w, r = _particles(rng, 300, (4.0, 4.0, 4.0), [0.1, 0.7])
    a = capi.deposit(xyz, w, r, (16, 16, 16), 4.0)
    b = capi.deposit(xyz, w, r, (16, 16, 16), 4.0, out=a.copy(order="F"))
    _close(b, 2.0 * oracle.deposit(xyz, w, r, (16, 16, 16), 4.0))


def test_knn_smoothing_lengths_feed_the_deposit(gpu, oracle):
    """kNN radii from the GPU tree into the deposit; the
    radii equal the oracle's k-th distances and the periodic grid holds the
    total weight to the S^3 sampling error."""
    from tests.golden.inputs import uniform
    pts = uniform(20000, seed=5, L=1.0)
    w = np.full(len(pts), 1.0 / len(pts), f32)
    grid, radii = _ras().render_knn_volume(pts, w, 16, 32, 1.0)
    ref_d, _ = oracle.knn_brute(pts, pts[:500], 16, boxsize=1.0)
    np.testing.assert_array_equal(radii[:500], ref_d[:, -1])
    _close(grid, oracle.deposit(pts, w, radii, (32, 32, 32), 32.0, (1.0, 1.0, 1.0), 4, 0))
    assert abs(float(grid.sum(dtype=np.float64)) - 1.0) < 0.02


def test_non_finite_radii_and_centres_contribute_nothing(gpu, oracle):
    """kth_distance pads with inf when k > n; w / (4/3 pi R^3) is then 0 in the
    reference's shader, and a NaN vertex is not rasterised: such balls add
    nothing (and are not expanded into 27 images over the whole grid)."""
    from nbodyhpc_amd import capi
    rng = np.random.default_rng(71)
    grid, ppu = (32, 32, 32), 8.0
    box = (4.0, 4.0, 4.0)
    xyz, w, r = _particles(rng, 300, box, [0.05, 0.3, 0.8])
    r[:40] = np.inf
    xyz[40:50, 1] = np.nan
    r[50:60] = np.nan
    got = capi.deposit(xyz, w, r, grid, ppu, period=box, device=0)
    keep = np.arange(300) >= 60
    ref = oracle.deposit(xyz[keep], w[keep], r[keep], grid, ppu, box, 4, 0)
    _close(got, ref)
    assert np.all(np.isfinite(got))


def test_device_deposits_on_two_streams(gpu, oracle):
    """Two device-output deposits enqueued back to back on two streams share the
    device's deposit workspace: the second call waits for the first's kernels
    (stream-ordered reuse), so both grids equal the oracle's."""
    from nbodyhpc_amd import capi, hip
    rng = np.random.default_rng(72)
    grid, ppu = (48, 48, 48), 6.0
    box = tuple(np.array(grid) / ppu)
    sets = [_particles(rng, 3000, box, [0.1, 0.4, 1.0]) for _ in range(2)]
    streams = [hip.Stream(), hip.Stream()]
    outs = []
    keep = []
    for (xyz, w, r), s in zip(sets, streams):
        dx, dw, dr = (hip.DeviceArray.from_numpy(a) for a in (xyz, w, r))
        g = hip.DeviceArray(grid[::-1], np.float32)
        capi.deposit_device(dx.ptr, dw.ptr, dr.ptr, len(r), grid, ppu, g.ptr, period=box,
                            device=0, stream=s.handle)
        outs.append(g)
        keep.append((dx, dw, dr))
    hip.synchronize()
    for (xyz, w, r), g in zip(sets, outs):
        got = g.numpy().reshape(grid[::-1]).transpose(2, 1, 0)
        _close(np.asfortranarray(got), oracle.deposit(xyz, w, r, grid, ppu, box, 4, 0))
