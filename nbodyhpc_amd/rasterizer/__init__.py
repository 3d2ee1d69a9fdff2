"""Sphere deposit onto voxel grids: the drop-in for `nbodyhpc.rasterizer`.

Mirrors rasterization/src/python/nbodyhpc/rasterizer/__init__.py (same
functions, arguments, defaults, output shapes and error messages) with the
Vulkan point renderer replaced by one HIP kernel (nbodyhpc_amd/csrc/deposit.hip,
C ABI `nbkd_deposit`).  The semantics -- sprite coverage, S^3 sub-sampling,
sub-voxel snapping, periodic images, slice planes -- are restated in
oracle/deposit_oracle.c, against which tests/test_gpu_deposit.py checks the
kernel.  There is no CPU fallback: without libnbkd.so the import fails.

Typical use feeds kNN smoothing lengths::

    h = KDTree(pos, boxsize=L).kth_distance(pos, 32)
    rho = render_points_volume(pos, mass, h, pixels_per_unit=n / L, grid_size=n,
                               periodic=True)
"""
from __future__ import annotations

import functools
from typing import Tuple, Union

import numpy as np

from .. import capi

Extent2d = Union[int, Tuple[int, int]]
Extent3d = Union[int, Tuple[int, int, int]]
PeriodT = Union[bool, float, Tuple[float, float, float]]

__all__ = ["DeviceContainer", "VulkanContainer", "PointRenderer", "get_default_container",
           "get_point_renderer", "render_points", "render_points_volume", "render_knn_volume"]


def _normalize_extent_2d(extent: Extent2d) -> Tuple[int, int]:
    if isinstance(extent, (int, np.integer)):
        return int(extent), int(extent)
    return tuple(extent)


def _normalize_extent_3d(extent: Extent3d) -> Tuple[int, int, int]:
    if isinstance(extent, (int, np.integer)):
        return int(extent), int(extent), int(extent)
    return tuple(extent)


def _normalize_period(deduced, period: PeriodT) -> Tuple[float, float, float]:
    """rasterizer/__init__.py:27-38: True -> the grid's own box, False -> none,
    a float -> cubic, a 2-tuple -> (x, y) with z open, else per axis."""
    if isinstance(period, (bool, np.bool_)):
        return tuple(deduced) if period else (-1.0, -1.0, -1.0)
    if isinstance(period, (float, int, np.floating, np.integer)):
        return float(period), float(period), float(period)
    if len(period) == 2:
        return float(period[0]), float(period[1]), -1.0
    return tuple(float(p) for p in period)


class DeviceContainer:
    """The device the renderers run on (stands where the reference's
    VulkanContainer, rasterization/src/cpp/vulkan_support.h, holds the Vulkan
    instance and device).  `device` < 0: the calling thread's current device."""

    def __init__(self, enable_validation_layers: bool = False, device: int = -1):
        self.device = int(device)


VulkanContainer = DeviceContainer


class PointRenderer:
    """rasterization/src/cpp/pybind.cpp:132-167.  As in the reference the
    constructor's (width, height) are stored transposed: `height` is the x
    extent of the grid and `width` the y extent, and results are (height,
    width[, num_slices]) arrays indexed [x, y, slice]."""

    def __init__(self, container: DeviceContainer, width: int, height: int,
                 subsample_factor: int = 4):
        self.container = container if container is not None else get_default_container()
        self.width = int(width)
        self.height = int(height)
        self.subsample_factor = int(subsample_factor)

    def _vertices(self, positions, weight, radii):
        # assemble_vertices' checks, in order (pybind.cpp:28-46)
        pos = np.asarray(positions, dtype=np.float32)
        w = np.asarray(weight, dtype=np.float32)
        r = np.asarray(radii, dtype=np.float32)
        if pos.ndim != 2 or pos.shape[1] != 3:
            raise RuntimeError("positions must be a 2D array of shape (N, 3)")
        if w.ndim != 1:
            raise RuntimeError("weight must be a 1D array")
        if r.ndim != 1:
            raise RuntimeError("radii must be a 1D array")
        if r.shape[0] != pos.shape[0]:
            raise RuntimeError("radii must have the same length as positions")
        if w.shape[0] != pos.shape[0]:
            raise RuntimeError("weights must have the same length as positions")
        return pos, w, r

    def render_points(self, positions, weight, radii, pixels_per_unit: float = 1.0,
                      periodic=(-1.0, -1.0, -1.0)) -> np.ndarray:
        """One plane at z = 0 (point_renderer.cpp:606-657): (height, width) array."""
        pos, w, r = self._vertices(positions, weight, radii)
        out = capi.deposit(pos, w, r, (self.height, self.width, 1), pixels_per_unit,
                           period=periodic, subsample=self.subsample_factor, mode=1,
                           device=self.container.device)
        return out[:, :, 0]

    def render_points_volume(self, positions, weight, radii, num_slices: int,
                             pixels_per_unit: float = 1.0,
                             periodic=(-1.0, -1.0, -1.0)) -> np.ndarray:
        """Slices [s, s+1) / ppu (point_renderer.cpp:825-950): (height, width,
        num_slices) array."""
        pos, w, r = self._vertices(positions, weight, radii)
        return capi.deposit(pos, w, r, (self.height, self.width, int(num_slices)),
                            pixels_per_unit, period=periodic, subsample=self.subsample_factor,
                            mode=0, device=self.container.device)


@functools.lru_cache(maxsize=None)
def get_default_container() -> DeviceContainer:
    return DeviceContainer(enable_validation_layers=False)


@functools.lru_cache(maxsize=None)
def _get_point_renderer_impl(width: int, height: int, subsample_factor: int = 4,
                             container: DeviceContainer = None) -> PointRenderer:
    return PointRenderer(container, width, height, subsample_factor)


def get_point_renderer(grid_size: Extent2d, subsample_factor: int = 4,
                       container: DeviceContainer = None) -> PointRenderer:
    """rasterizer/__init__.py:59-84 (renderers are cached per parameters)."""
    if container is None:
        container = get_default_container()
    height, width = _normalize_extent_2d(grid_size)
    return _get_point_renderer_impl(width, height, subsample_factor, container)


def render_points(positions: np.ndarray, weights: np.ndarray, radii: np.ndarray,
                  pixels_per_unit: float, grid_size: Extent2d,
                  periodic: PeriodT = False) -> np.ndarray:
    """rasterizer/__init__.py:87-101: the plane z = 0 of a (grid_x, grid_y) grid."""
    grid_x, grid_y = _normalize_extent_2d(grid_size)
    renderer = get_point_renderer((grid_x, grid_y))
    deduced = grid_x / pixels_per_unit, grid_y / pixels_per_unit, -1.0
    period = _normalize_period(deduced, periodic)
    return renderer.render_points(positions, weights, radii, pixels_per_unit, period)


def render_points_volume(positions: np.ndarray, weights: np.ndarray, radii: np.ndarray,
                         pixels_per_unit: float, grid_size: Extent3d, periodic: PeriodT = False,
                         subsample_factor: int = 4) -> np.ndarray:
    """rasterizer/__init__.py:104-143: a (grid_x, grid_y, grid_z) float32 grid
    holding, per voxel, the weight of every ball times the fraction of its
    volume inside the voxel (S^3 sub-samples, S = subsample_factor)."""
    grid_x, grid_y, num_slices = _normalize_extent_3d(grid_size)
    deduced_box = grid_x / pixels_per_unit, grid_y / pixels_per_unit, num_slices / pixels_per_unit
    period = _normalize_period(deduced_box, periodic)
    renderer = get_point_renderer((grid_x, grid_y), subsample_factor)
    return renderer.render_points_volume(positions, weights, radii, num_slices, pixels_per_unit,
                                         period)


def render_knn_volume(positions: np.ndarray, weights: np.ndarray, k: int, grid_size: int,
                      boxsize: float, subsample_factor: int = 4, leafsize: int = 64):
    """kNN smoothing lengths feeding the deposit: each
    particle's radius is its distance to its k-th neighbour (itself included),
    from the GPU kd-tree; the grid covers the periodic box [0, boxsize)^3.
    Returns (grid, radii)."""
    from ..kdtree import KDTree

    pos = np.asarray(positions, dtype=np.float32)
    tree = KDTree(pos, leafsize=leafsize, boxsize=boxsize)
    radii = tree.kth_distance(pos, k)
    ppu = grid_size / boxsize
    grid = render_points_volume(pos, weights, radii, ppu, grid_size, periodic=True,
                                subsample_factor=subsample_factor)
    return grid, radii
