"""Raw particle files (reference main.cpp:103-114 format) and slab streaming."""
import numpy as np
import pytest

from nbodyhpc_amd import io, slab


def test_roundtrip_and_trailing_bytes(tmp_path):
    rng = np.random.Generator(np.random.PCG64(3))
    a = rng.uniform(0, 1, (1001, 3)).astype(np.float32)
    p = str(tmp_path / "p.bin")
    io.write_positions(p, a)
    with open(p, "ab") as f:
        f.write(b"\x01\x02\x03\x04\x05")  # a partial row is ignored, as in the reference
    assert io.count_rows(p) == 1001
    assert np.array_equal(np.asarray(io.read_positions(p)), a)
    assert np.array_equal(io.read_positions(p, mmap=False), a)


def test_read_slab_partitions_rows(tmp_path):
    rng = np.random.Generator(np.random.PCG64(4))
    a = rng.uniform(0, 2.0, (5000, 3)).astype(np.float32)
    a[:7, 0] = np.float32(2.0)  # x == L belongs to the last slab
    a[7:9, 0] = np.float32(0.0)
    p = str(tmp_path / "p.bin")
    io.write_positions(p, a)
    seen = []
    for world in (1, 3):
        seen = []
        for r in range(world):
            xyz, ids = io.read_slab(p, r, world, 2.0, chunk_rows=333)
            lo, hi = slab.slab_bounds(r, world, 2.0)
            assert np.array_equal(xyz, a[ids])
            assert np.all(xyz[:, 0] >= np.float32(lo))
            if r < world - 1:
                assert np.all(xyz[:, 0] < np.float32(hi))
            assert np.all(np.diff(ids.astype(np.int64)) > 0)  # file order
            seen.append(ids)
        allids = np.sort(np.concatenate(seen))
        assert np.array_equal(allids, np.arange(5000, dtype=np.uint32))
    assert set(range(7)) <= set(seen[-1].tolist())


def test_empty_file(tmp_path):
    p = str(tmp_path / "e.bin")
    open(p, "wb").close()
    assert io.read_positions(p).shape == (0, 3)
    xyz, ids = io.read_slab(p, 0, 2, 1.0)
    assert xyz.shape == (0, 3) and ids.shape == (0,)


@pytest.mark.parametrize("fmt,endian,nfiles,idt", [(1, "<", 1, np.uint32), (2, "<", 1, np.uint64),
                                                   (1, ">", 3, np.uint32), (2, ">", 2, np.uint32)])
def test_gadget_round_trip(tmp_path, fmt, endian, nfiles, idt):
    """Gadget-2 snapshots (format 1 and 2, both byte orders, multi-file):
    positions, ids and BoxSize come back exactly."""
    from nbodyhpc_amd import io as nio
    rng = np.random.default_rng(3)
    xyz = rng.uniform(0, 50.0, (1001, 3)).astype(np.float32)
    ids = (rng.permutation(1001) + 7).astype(idt)
    p = str(tmp_path / "snap_010")
    nio.write_gadget(p, xyz, 50.0, ids=ids, fmt=fmt, endian=endian, num_files=nfiles)
    got, gid, h = nio.read_gadget(p)
    assert np.array_equal(got, xyz)
    assert gid is not None and np.array_equal(gid, ids) and gid.dtype == idt
    assert h["BoxSize"] == 50.0 and h["num_files"] == nfiles
    assert int(np.sum(h["npartTotal"])) == 1001


def test_gadget_rejects_other_files(tmp_path):
    from nbodyhpc_amd import io as nio
    p = tmp_path / "raw.bin"
    nio.write_positions(str(p), np.ones((10, 3), np.float32))
    with pytest.raises(ValueError):
        nio.read_gadget(str(p))


@pytest.mark.parametrize("fmt,endian,nfiles,world", [(1, "<", 1, 2), (2, ">", 3, 3),
                                                     (1, ">", 2, 4)])
def test_gadget_slab_streaming_partitions_rows(tmp_path, fmt, endian, nfiles, world):
    """read_gadget_slab: the ranks' slabs partition the snapshot's rows (in
    read_gadget's order), each row in its x-slab, x == BoxSize on the last
    rank; small chunks exercise the chunked scan across file boundaries."""
    from nbodyhpc_amd import io as nio
    rng = np.random.default_rng(4)
    box = 20.0
    xyz = rng.uniform(0, box, (2003, 3)).astype(np.float32)
    xyz[:3, 0] = box
    xyz[3:6, 0] = 0.0
    p = str(tmp_path / "snap")
    nio.write_gadget(p, xyz, box, fmt=fmt, endian=endian, num_files=nfiles)
    cuts = slab.bounds_list(world, box)
    seen = []
    for r in range(world):
        part, rows, h = nio.read_gadget_slab(p, r, world, chunk_rows=97)
        assert h["BoxSize"] == box and rows.dtype == np.uint32
        assert np.array_equal(part, xyz[rows])
        x = part[:, 0]
        assert np.all(x >= np.float32(cuts[r]))
        assert np.all(x <= np.float32(box)) if r == world - 1 else np.all(x < np.float32(cuts[r + 1]))
        seen.append(rows)
    allr = np.sort(np.concatenate(seen))
    assert np.array_equal(allr, np.arange(2003, dtype=np.uint32))
