"""Particle files: the reference benchmark's raw
format, float32 (N, 3) row-major with no header
(kdtree/src/cpp/main.cpp:103-114 `read_array_from_file`: N = file size // 12,
trailing bytes ignored), memory-mapped so 1e9-particle files stream.

`read_slab` streams a file in chunks and keeps the rows of one rank's x-slab
(slab.slab_bounds; the last slab also takes x == box, which periodic inputs
allow), with their row numbers as global ids, for the one-process-per-GPU
path (nbodyhpc_amd/slab.py) without a full host copy per rank.
"""
from __future__ import annotations

import os

import numpy as np

ROW_BYTES = 12


def count_rows(path: str) -> int:
    return os.path.getsize(path) // ROW_BYTES


def read_positions(path: str, mmap: bool = True) -> np.ndarray:
    """(N, 3) float32 positions; a read-only memory map unless mmap=False."""
    n = count_rows(path)
    if n == 0:
        return np.empty((0, 3), np.float32)
    if mmap:
        return np.memmap(path, dtype=np.float32, mode="r", shape=(n, 3))
    out = np.empty((n, 3), np.float32)
    with open(path, "rb") as f:
        f.readinto(memoryview(out).cast("B"))
    return out


def write_positions(path: str, xyz) -> None:
    a = np.ascontiguousarray(xyz, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] != 3:
        raise ValueError("positions must be a 2D array of shape (N, 3)")
    with open(path, "wb") as f:
        a.tofile(f)


def iter_chunks(path: str, chunk_rows: int = 1 << 24):
    """(first row, float32 (rows, 3) view) over the file."""
    a = read_positions(path)
    for s in range(0, a.shape[0], chunk_rows):
        yield s, a[s:s + chunk_rows]


def read_slab(path: str, rank: int, world: int, box: float, chunk_rows: int = 1 << 24):
    """Rows of rank `rank`'s x-slab, in file order, and their row numbers
    (uint32 global ids)."""
    from .slab import slab_bounds
    lo, hi = slab_bounds(rank, world, box)
    lo32, hi32 = np.float32(lo), np.float32(hi)
    last = rank == world - 1
    if count_rows(path) > 0xFFFFFFFF:
        raise ValueError("More than uint32_t points are not supported.")
    xs, ids = [], []
    for s, c in iter_chunks(path, chunk_rows):
        x = c[:, 0]
        keep = (x >= lo32) & ((x <= hi32) if last else (x < hi32))
        sel = np.nonzero(keep)[0]
        xs.append(np.array(c[sel], dtype=np.float32))
        ids.append((sel + s).astype(np.uint32))
    if not xs:
        return np.empty((0, 3), np.float32), np.empty(0, np.uint32)
    return np.concatenate(xs), np.concatenate(ids)
