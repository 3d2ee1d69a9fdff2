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


# ------------------------------------------------------------------ Gadget snapshots
# N-body codes write Gadget-2 binary snapshots.  The
# published layout (Springel 2005, the Gadget-2 user guide §6): Fortran
# unformatted records [int32 nbytes][payload][int32 nbytes]; SnapFormat 1 is
# HEAD (256 B), POS (float32 [N, 3]), VEL, ID, ...; SnapFormat 2 puts an 8-byte
# label record ("POS " + int32 next-block size) before each block.  A
# snapshot may be split over files <base>.0, <base>.1, ... (num_files in the
# header).  The reference has no loader (it reads raw float32 rows,
# main.cpp:103-114); this one feeds the same (N, 3) float32 positions.
GADGET_HEADER = np.dtype([
    ("npart", "<u4", 6), ("massarr", "<f8", 6), ("time", "<f8"), ("redshift", "<f8"),
    ("flag_sfr", "<i4"), ("flag_feedback", "<i4"), ("npartTotal", "<u4", 6),
    ("flag_cooling", "<i4"), ("num_files", "<i4"), ("BoxSize", "<f8"), ("Omega0", "<f8"),
    ("OmegaLambda", "<f8"), ("HubbleParam", "<f8"), ("flag_stellarage", "<i4"),
    ("flag_metals", "<i4"), ("npartTotalHighWord", "<u4", 6),
    ("flag_entropy_instead_u", "<i4"), ("fill", "V60")])
assert GADGET_HEADER.itemsize == 256


class _Records:
    """Fortran records of one file: (offset of payload, nbytes), in order."""

    def __init__(self, path):
        self.path = path
        self.size = os.path.getsize(path)
        with open(path, "rb") as f:
            head = f.read(4)
        if len(head) < 4:
            raise ValueError(f"{path}: not a Gadget snapshot (empty)")
        le, be = int(np.frombuffer(head, "<i4")[0]), int(np.frombuffer(head, ">i4")[0])
        if le in (8, 256):
            self.endian = "<"
        elif be in (8, 256):
            self.endian = ">"
        else:
            raise ValueError(f"{path}: not a Gadget snapshot (first record marker {le})")
        self.format = 2 if (le if self.endian == "<" else be) == 8 else 1
        self.recs = []
        i32 = np.dtype(self.endian + "i4")
        with open(path, "rb") as f:
            off = 0
            while off + 4 <= self.size:
                f.seek(off)
                n = int(np.frombuffer(f.read(4), i32)[0])
                if n < 0 or off + 8 + n > self.size:
                    raise ValueError(f"{path}: truncated record at byte {off}")
                f.seek(off + 4 + n)
                if int(np.frombuffer(f.read(4), i32)[0]) != n:
                    raise ValueError(f"{path}: record markers differ at byte {off}")
                self.recs.append((off + 4, n))
                off += 8 + n

    def blocks(self):
        """(label or None, payload offset, nbytes) per data block."""
        if self.format == 1:
            return [(None, o, n) for o, n in self.recs]
        out = []
        with open(self.path, "rb") as f:
            for j in range(0, len(self.recs) - 1, 2):
                o, n = self.recs[j]
                f.seek(o)
                label = f.read(4).decode("ascii", "replace")
                out.append((label, *self.recs[j + 1]))
        return out


def _gadget_files(path):
    if os.path.exists(path):
        return [path]
    files = []
    while os.path.exists(f"{path}.{len(files)}"):
        files.append(f"{path}.{len(files)}")
    if not files:
        raise FileNotFoundError(path)
    return files


def read_gadget(path, ids=True):
    """Positions (N, 3) float32 of every particle type of a Gadget-2 snapshot
    (format 1 or 2, either byte order, single or multi-file), the particle
    ids (uint32 or uint64, when the ID block exists and `ids`), and the header
    of the first file as a dict (BoxSize: the periodic box)."""
    pos, idv, header = [], [], None
    for fp in _gadget_files(path):
        r = _Records(fp)
        blocks = r.blocks()
        if not blocks or blocks[0][2] != 256:
            raise ValueError(f"{fp}: first block is not a 256-byte header")
        with open(fp, "rb") as f:
            f.seek(blocks[0][1])
            h = np.frombuffer(f.read(256), GADGET_HEADER.newbyteorder(r.endian)
                              if r.endian == ">" else GADGET_HEADER)[0]
            n = int(np.asarray(h["npart"], np.uint64).sum())
            if header is None:
                header = {k: (h[k].tolist() if hasattr(h[k], "tolist") else h[k])
                          for k in GADGET_HEADER.names if k != "fill"}
            if r.format == 2:
                byname = {lab.strip(): (o, nb) for lab, o, nb in blocks[1:]}
                p_blk = byname.get("POS")
                i_blk = byname.get("ID")
            else:
                p_blk = blocks[1][1:] if len(blocks) > 1 else None
                i_blk = blocks[3][1:] if len(blocks) > 3 else None
            if p_blk is None or p_blk[1] != 12 * n:
                raise ValueError(f"{fp}: no float32 POS block of {n} particles")
            f.seek(p_blk[0])
            pos.append(np.fromfile(f, np.dtype(r.endian + "f4"), 3 * n).reshape(n, 3)
                       .astype(np.float32))
            if ids and i_blk is not None and i_blk[1] in (4 * n, 8 * n):
                f.seek(i_blk[0])
                w = "u4" if i_blk[1] == 4 * n else "u8"
                idv.append(np.fromfile(f, np.dtype(r.endian + w), n))
    xyz = np.concatenate(pos) if pos else np.empty((0, 3), np.float32)
    idall = np.concatenate(idv) if idv and len(idv) == len(pos) else None
    return xyz, idall, header


def _gadget_pos_blocks(path):
    """Per file: (path, endian, payload offset of POS, particle count), and
    the first file's header as a dict."""
    out, header = [], None
    for fp in _gadget_files(path):
        r = _Records(fp)
        blocks = r.blocks()
        if not blocks or blocks[0][2] != 256:
            raise ValueError(f"{fp}: first block is not a 256-byte header")
        with open(fp, "rb") as f:
            f.seek(blocks[0][1])
            h = np.frombuffer(f.read(256), GADGET_HEADER.newbyteorder(r.endian)
                              if r.endian == ">" else GADGET_HEADER)[0]
        n = int(np.asarray(h["npart"], np.uint64).sum())
        if header is None:
            header = {k: (h[k].tolist() if hasattr(h[k], "tolist") else h[k])
                      for k in GADGET_HEADER.names if k != "fill"}
        if r.format == 2:
            p_blk = {lab.strip(): (o, nb) for lab, o, nb in blocks[1:]}.get("POS")
        else:
            p_blk = blocks[1][1:] if len(blocks) > 1 else None
        if p_blk is None or p_blk[1] != 12 * n:
            raise ValueError(f"{fp}: no float32 POS block of {n} particles")
        out.append((fp, r.endian, p_blk[0], n))
    return out, header


def read_gadget_slab(path, rank, world, box=None, chunk_rows=1 << 24, bounds=None):
    """Rank `rank`'s x-slab of a Gadget-2 snapshot, streamed: each file's POS
    block is memory-mapped and scanned in chunks, so no rank holds the whole
    snapshot ("streams to slabs directly").  Returns
    (xyz float32 (m, 3), row numbers uint32 in read_gadget's order, header).
    `box`: the periodic box (default: the header's BoxSize); `bounds`: the
    W + 1 slab cuts (default: equal widths).  The last slab also owns x == box."""
    from .slab import bounds_list
    files, header = _gadget_pos_blocks(path)
    box = float(header["BoxSize"]) if box is None else float(box)
    cuts = bounds_list(world, box) if bounds is None else bounds
    lo32, hi32 = np.float32(cuts[rank]), np.float32(cuts[rank + 1])
    last = rank == world - 1
    if sum(f[3] for f in files) > 0xFFFFFFFF:
        raise ValueError("More than uint32_t points are not supported.")
    xs, ids, base = [], [], 0
    for fp, endian, off, n in files:
        if n == 0:
            continue
        a = np.memmap(fp, dtype=np.dtype(endian + "f4"), mode="r", offset=off, shape=(n, 3))
        for s in range(0, n, chunk_rows):
            c = a[s:s + chunk_rows]
            x = c[:, 0]
            keep = (x >= lo32) & ((x <= hi32) if last else (x < hi32))
            sel = np.nonzero(keep)[0]
            xs.append(np.asarray(c[sel], dtype=np.float32))
            ids.append((sel + base + s).astype(np.uint32))
        base += n
        del a
    if not xs:
        return np.empty((0, 3), np.float32), np.empty(0, np.uint32), header
    return np.concatenate(xs), np.concatenate(ids), header


def write_gadget(path, xyz, box, ids=None, fmt=1, endian="<", num_files=1):
    """A minimal Gadget-2 snapshot (all particles type 1, unit mass): the
    test-fixture writer for read_gadget.  num_files > 1 writes <path>.0 ...
    with the particles split evenly."""
    xyz = np.ascontiguousarray(xyz, np.float32)
    n_all = xyz.shape[0]
    ids = np.arange(1, n_all + 1, dtype=np.uint32) if ids is None else np.asarray(ids)
    cuts = np.linspace(0, n_all, num_files + 1).astype(np.int64)
    i32 = np.dtype(endian + "i4")

    def rec(f, payload, label=None):
        if fmt == 2 and label is not None:
            f.write(np.array([8], i32).tobytes() + label.ljust(4)[:4].encode()
                    + np.array([len(payload) + 8], i32).tobytes() + np.array([8], i32).tobytes())
        f.write(np.array([len(payload)], i32).tobytes() + payload
                + np.array([len(payload)], i32).tobytes())

    for j in range(num_files):
        a, b = int(cuts[j]), int(cuts[j + 1])
        h = np.zeros((), GADGET_HEADER)
        h["npart"][1] = b - a
        h["npartTotal"][1] = n_all & 0xFFFFFFFF
        h["npartTotalHighWord"][1] = n_all >> 32
        h["massarr"][1] = 1.0
        h["num_files"] = num_files
        h["BoxSize"] = box
        hb = h.tobytes() if endian == "<" else np.array(h).astype(
            GADGET_HEADER.newbyteorder(">")).tobytes()
        name = path if num_files == 1 else f"{path}.{j}"
        with open(name, "wb") as f:
            rec(f, hb, "HEAD")
            rec(f, xyz[a:b].astype(endian + "f4").tobytes(), "POS ")
            rec(f, np.zeros((b - a, 3), endian + "f4").tobytes(), "VEL ")
            rec(f, ids[a:b].astype(endian + ids.dtype.str[1:]).tobytes(), "ID  ")
