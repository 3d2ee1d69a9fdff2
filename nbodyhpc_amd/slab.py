"""Slab decomposition of the periodic box across ranks.

One process per GPU.  Rank r of W owns the particles with x in the slab
[lo, hi) = [r L / W, (r+1) L / W).  Its kd-tree is built over its own particles
plus two halo strips of width h received from its ring neighbours: the
right neighbour's particles with x in [lo', lo' + h) and the left neighbour's
with x in [hi' - h, hi').  Halo particles keep their periodic coordinates (the
tree is periodic over the whole box, so min-image distances between local
points are the true ones) and their global ids (`nbkd_set_ids`), so the local
kNN of an own particle returns global ids.  A row is exact (equal to the
single-tree result over all W slabs) iff its k-th distance stays strictly
inside [lo - h, hi + h) along x (`nbkd_slab_violations`); `knn_setup` widens
h and rebuilds until every row is exact.

The bulk transfer is RCCL point-to-point over xGMI (`nbkd_comm_exchange`, one
grouped send/recv set with each neighbour).  Strip sizes (8 bytes per
neighbour) go over torch.distributed/gloo, which also carries the RCCL unique
id.  `exchange_host` is the same protocol on host arrays over gloo: the path
the world-size-2 CPU tests run and the fallback when RCCL cannot start.
"""
from __future__ import annotations

import math
import sys

import numpy as np

_TAG_RIGHTWARD, _TAG_LEFTWARD = 17, 18
# device buffers a failed RCCL group may still touch: kept alive, never freed
_ABANDONED = []


def slab_bounds(rank: int, world: int, box: float):
    """[lo, hi) of `rank` as float32 values (the comparisons run in f32)."""
    lo = np.float32(box * rank / world)
    hi = np.float32(box) if rank == world - 1 else np.float32(box * (rank + 1) / world)
    return float(lo), float(hi)


def bounds_list(world: int, box: float):
    """The W + 1 slab cuts of the equal-width decomposition."""
    return [slab_bounds(r, world, box)[0] for r in range(world)] + [float(np.float32(box))]


def check_halo(h: float, bounds) -> None:
    """A halo strip comes from the adjacent slab only, so h may not exceed the
    narrowest slab; with two ranks both strips of a rank go to the same
    neighbour, so they may not overlap either (2h <= width), or its points
    would arrive twice."""
    w = np.diff(np.asarray(bounds, np.float64))
    world = len(w)
    if world < 2:
        return
    lim = float(w.min()) / (2.0 if world == 2 else 1.0)
    if h > lim:
        raise ValueError(f"halo width {h:.4g} exceeds the slab limit {lim:.4g} "
                         f"({world} slabs, narrowest {float(w.min()):.4g})")


def ball_halo(r: float, box: float) -> float:
    """Halo width that holds every point within r (periodic min-image) of an
    own particle: r plus a relative 1e-4 and a few box ulps, so that neither
    the f32 strip cut nor the f32 d2 <= r2 test at the edge can drop one."""
    return float(r) * (1.0 + 1e-4) + 4.0 * float(np.spacing(np.float32(box)))


def halo_width(n_total: int, k: int, box: float, factor: float = 1.3) -> float:
    """factor x the mean k-th neighbour radius of a uniform density.  1.3 since
    round 4 (2.5 before): the second-round exchange makes every row exact
    whatever the width, and at 1.3 a uniform row reaches past the halo only if
    its ball of 1.3 r_k (~70 expected points at k = 32) holds fewer than k
    points; at N = 8 strong scaling of 1e8 points the halo adds ~9 % points per
    rank instead of ~17 %."""
    rho = n_total / box ** 3
    r_k = (k / (4.0 / 3.0 * math.pi * rho)) ** (1.0 / 3.0)
    return float(factor * r_k)


def gen_slab_points(n_per: int, seed: int, box: float, rank: int, world: int):
    """Uniform particles of rank `rank`'s slab; the union over ranks is a
    uniform sample of the box.  Global ids are rank * n_per + i."""
    lo, hi = slab_bounds(rank, world, box)
    lo32, hi32 = np.float32(lo), np.float32(hi)
    top = np.nextafter(hi32, np.float32(-np.inf))
    rng = np.random.Generator(np.random.PCG64([seed, rank]))
    out = np.empty((n_per, 3), np.float32)
    chunk = 1 << 24
    for s in range(0, n_per, chunk):
        e = min(n_per, s + chunk)
        u = rng.uniform(0.0, 1.0, size=(e - s, 3))
        out[s:e, 0] = np.clip((lo + (hi - lo) * u[:, 0]).astype(np.float32), lo32, top)
        out[s:e, 1:] = (box * u[:, 1:]).astype(np.float32)
    out[:, 1:] = np.minimum(out[:, 1:], np.nextafter(np.float32(box), np.float32(-np.inf)))
    ids = (np.uint64(rank) * np.uint64(n_per) + np.arange(n_per, dtype=np.uint64))
    if n_per and ids[-1] > np.uint64(0xFFFFFFFE):
        raise ValueError("global ids exceed uint32")
    return out, ids.astype(np.uint32)


def gen_uniform_slab(n_total: int, seed: int, box: float, rank: int, world: int, bounds=None):
    """Rank `rank`'s slab of the SAME uniform set at every world size (strong
    scaling): the stream of synth.uniform(n_total, seed, box) - PCG64(seed),
    rows drawn in chunks of 2^24 - kept where slab_of(x) == rank.  Global ids
    are the row numbers, so the union over ranks is exactly the one-GPU set."""
    bounds = bounds_list(world, box) if bounds is None else bounds
    if n_total > 0xFFFFFFFF:
        raise ValueError("global ids exceed uint32")
    rng = np.random.Generator(np.random.PCG64(seed))
    xs, ids = [], []
    chunk = 1 << 24
    for s0 in range(0, n_total, chunk):
        e = min(n_total, s0 + chunk)
        c = rng.uniform(0.0, box, size=(e - s0, 3)).astype(np.float32)
        m = slab_of(c[:, 0], bounds) == rank
        xs.append(c[m])
        ids.append((s0 + np.nonzero(m)[0]).astype(np.uint32))
    if not xs:
        return np.zeros((0, 3), np.float32), np.zeros(0, np.uint32)
    return np.concatenate(xs), np.concatenate(ids)


def _enqueue_agreed(dist, rank, what, enqueue):
    """Run `enqueue` (an RCCL grouped send/recv, enqueue only) and agree over
    gloo whether it succeeded everywhere.  Returns None when every rank
    enqueued, the local error when every rank failed (the caller may then fall
    back to gloo on every rank), and raises when only some ranks failed: their
    peers' queued operations can never complete, and mixing transports could
    deliver the same range twice."""
    import torch

    err = None
    try:
        enqueue()
    except Exception as e:  # agreed on below
        err = e
    ok = 0 if err is not None else 1
    t = torch.tensor([ok, -ok], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    all_ok, any_ok = int(t[0]) == 1, -int(t[1]) == 1
    if all_ok:
        return None
    if any_ok:
        raise RuntimeError(f"rank {rank}: RCCL {what} failed on some ranks only "
                           f"(here: {err or 'ok'}); refusing to mix transports")
    return err


def neighbours(rank: int, world: int):
    return (rank - 1) % world, (rank + 1) % world


def _strip_counts(dist, rank, world, to_right: int, to_left: int):
    """all-gather of (to_right, to_left); returns (from_left, from_right)."""
    import torch

    left, right = neighbours(rank, world)
    mine = torch.tensor([to_right, to_left], dtype=torch.int64)
    allc = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allc, mine)
    return int(allc[left][0]), int(allc[right][1])


def _host_sendrecv(dist, rank, world, send_r, send_l, n_fl, n_fr, dtype, cols):
    """gloo point-to-point: send_r -> right, send_l -> left; receive from left
    (its rightward strip) and from right (its leftward strip)."""
    import torch

    left, right = neighbours(rank, world)
    shape = (lambda n: (n, cols)) if cols > 1 else (lambda n: (n,))
    rl = torch.empty(shape(n_fl), dtype=dtype)
    rr = torch.empty(shape(n_fr), dtype=dtype)
    reqs = []
    if len(send_r):
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(send_r)), right,
                               tag=_TAG_RIGHTWARD))
    if len(send_l):
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(send_l)), left,
                               tag=_TAG_LEFTWARD))
    if n_fl:
        reqs.append(dist.irecv(rl, left, tag=_TAG_RIGHTWARD))
    if n_fr:
        reqs.append(dist.irecv(rr, right, tag=_TAG_LEFTWARD))
    for r in reqs:
        r.wait()
    return rl.numpy(), rr.numpy()


def exchange_host(own_xyz, own_ids, rank, world, box, h, dist, bounds=None):
    """Host-array halo exchange over gloo.  Returns (local_xyz, local_ids) with
    the own particles first, then the strip from the left neighbour, then the
    strip from the right neighbour.  `bounds`: the W + 1 slab cuts (default:
    equal widths)."""
    if world == 1:
        return own_xyz, own_ids
    bounds = bounds_list(world, box) if bounds is None else bounds
    check_halo(h, bounds)
    lo, hi = float(bounds[rank]), float(bounds[rank + 1])
    x = own_xyz[:, 0]
    mr = x >= np.float32(hi - h)
    ml = x < np.float32(lo + h)
    n_fl, n_fr = _strip_counts(dist, rank, world, int(mr.sum()), int(ml.sum()))
    import torch

    fl_x, fr_x = _host_sendrecv(dist, rank, world, own_xyz[mr], own_xyz[ml], n_fl, n_fr,
                                torch.float32, 3)
    fl_i, fr_i = _host_sendrecv(dist, rank, world, own_ids[mr].astype(np.int32),
                                own_ids[ml].astype(np.int32), n_fl, n_fr, torch.int32, 1)
    xyz = np.concatenate([own_xyz, fl_x, fr_x])
    ids = np.concatenate([own_ids, fl_i.astype(np.uint32), fr_i.astype(np.uint32)])
    return xyz, ids


def violations_host(q_xyz, kth_dist, rank, world, box, h, bounds=None):
    """numpy statement of nbkd_slab_violations (slab.hip violations_kernel)."""
    if world == 1:
        return 0
    if bounds is None:
        lo, hi = slab_bounds(rank, world, box)
    else:
        lo, hi = float(bounds[rank]), float(bounds[rank + 1])
    x = q_xyz[:, 0].astype(np.float32)
    f32 = np.float32
    lo_h, hi_h = f32(f32(lo) - f32(h)), f32(f32(hi) + f32(h))
    margin = np.minimum(x - lo_h, hi_h - x)
    mag = np.maximum(np.abs(lo_h), np.abs(hi_h))
    slack = np.float32(4.0) * np.spacing(mag)
    ok = kth_dist.astype(np.float32) < margin * np.float32(1.0 - 4e-7) - slack
    return int((~ok).sum())


# ------------------------------------------------------ redistribution to owners
def slab_of(x, bounds):
    """Owner rank of each x (float32 compares against the f32 cuts): rank r
    owns [b_r, b_r+1); the last slab also owns x == L (periodic points lie in
    [0, L])."""
    inner = np.asarray(bounds[1:-1], np.float32)
    return np.searchsorted(inner, np.asarray(x, np.float32), side="right").astype(np.int64)


def _count_matrix(dist, world, send_counts):
    import torch

    mine = torch.as_tensor(np.asarray(send_counts, np.int64))
    allc = [torch.zeros(world, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allc, mine)
    return np.stack([a.numpy() for a in allc])  # [src, dst]


def redistribute(xyz, ids, rank, world, box, dist, comm=None, bounds=None, device=0, log=None):
    """all-to-all-v of arbitrary per-rank particle
    chunks (e.g. contiguous file rows) to their slab owners.

    Each rank orders its particles by owner (host, stable), the W x W count
    matrix goes over gloo, and the payload moves as one grouped RCCL
    send/recv set with every peer (`nbkd_comm_exchange` on device buffers)
    when `comm` is given, else as gloo point-to-point messages.  Returns
    (own_xyz, own_ids) as host arrays, in (source rank, source order) order;
    they feed DeviceSlab.  Exact: every particle lands on exactly one rank."""
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    ids = np.ascontiguousarray(ids, np.uint32).reshape(-1)
    if world == 1:
        return xyz, ids
    bounds = bounds_list(world, box) if bounds is None else bounds
    dest = slab_of(xyz[:, 0], bounds)
    order = np.argsort(dest, kind="stable")
    sx, si = xyz[order], ids[order]
    send = np.bincount(dest, minlength=world).astype(np.int64)
    mat = _count_matrix(dist, world, send)
    recv = mat[:, rank].astype(np.int64)
    soff = np.concatenate([[0], np.cumsum(send)])
    roff = np.concatenate([[0], np.cumsum(recv)])
    n_own = int(roff[-1])
    if comm is not None:
        out = _redistribute_rccl(sx, si, rank, world, comm, soff, roff, n_own, device, dist)
        if out is not None:
            return out
        (log or (lambda *a: None))(f"rank {rank}: RCCL redistribution failed on every rank; gloo")
    import torch

    out_x = np.empty((n_own, 3), np.float32)
    out_i = np.empty(n_own, np.uint32)
    out_x[roff[rank]:roff[rank + 1]] = sx[soff[rank]:soff[rank + 1]]
    out_i[roff[rank]:roff[rank + 1]] = si[soff[rank]:soff[rank + 1]]
    reqs, bufs = [], []
    for j in range(world):
        if j == rank:
            continue
        if send[j]:
            for a, tag in ((sx[soff[j]:soff[j + 1]], 31),
                           (si[soff[j]:soff[j + 1]].view(np.int32), 32)):
                reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(a)), j, tag=tag))
        if recv[j]:
            bx = torch.empty((int(recv[j]), 3), dtype=torch.float32)
            bi = torch.empty(int(recv[j]), dtype=torch.int32)
            reqs.append(dist.irecv(bx, j, tag=31))
            reqs.append(dist.irecv(bi, j, tag=32))
            bufs.append((j, bx, bi))
    for r in reqs:
        r.wait()
    for j, bx, bi in bufs:
        out_x[roff[j]:roff[j + 1]] = bx.numpy()
        out_i[roff[j]:roff[j + 1]] = bi.numpy().view(np.uint32)
    return out_x, out_i


def _redistribute_rccl(sx, si, rank, world, comm, soff, roff, n_own, device, dist):
    """None when the grouped send/recv failed to enqueue on every rank (the
    caller then moves the payload over gloo into its own host buffers)."""
    from . import hip

    dsx = hip.DeviceArray.from_numpy(sx if len(sx) else np.zeros((1, 3), np.float32))
    dsi = hip.DeviceArray.from_numpy(si if len(si) else np.zeros(1, np.uint32))
    drx = hip.DeviceArray((max(n_own, 1), 3), np.float32)
    dri = hip.DeviceArray((max(n_own, 1),), np.uint32)
    try:
        pairs = []
        for j in range(world):
            if j == rank:
                continue
            ns, nr = int(soff[j + 1] - soff[j]), int(roff[j + 1] - roff[j])
            # per peer: coordinates, then ids (matched in posting order)
            pairs.append((dsx.ptr + int(soff[j]) * 12, ns * 12, j,
                          drx.ptr + int(roff[j]) * 12, nr * 12, j))
            pairs.append((dsi.ptr + int(soff[j]) * 4, ns * 4, j,
                          dri.ptr + int(roff[j]) * 4, nr * 4, j))
        n_self = int(soff[rank + 1] - soff[rank])
        if n_self:
            hip.memcpy(drx.ptr + int(roff[rank]) * 12, dsx.ptr + int(soff[rank]) * 12, n_self * 12)
            hip.memcpy(dri.ptr + int(roff[rank]) * 4, dsi.ptr + int(soff[rank]) * 4, n_self * 4)
        err = _enqueue_agreed(dist, rank, "redistribution", lambda: comm.exchange(pairs))
        if err is not None:
            note_rccl_error(rank, "redistribution failed, moved over gloo", err)
            # a failed group may still read or write these: never free them
            _ABANDONED.extend((dsx, dsi, drx, dri))
            dsx = dsi = drx = dri = None
            return None
        hip.synchronize()
        return drx.numpy_head(n_own), dri.numpy_head(n_own)
    finally:
        for a in (dsx, dsi, drx, dri):
            if a is not None:
                a.free()


# ------------------------------------------------------------------ device path
class DeviceSlab:
    """Own particles + halo on the GPU for one rank (device arrays via hip.py)."""

    def __init__(self, own_xyz, own_ids, rank, world, box, device, dist=None, comm=None,
                 log=None, bounds=None):
        from . import hip

        self.rank, self.world, self.box, self.device = rank, world, box, device
        self.dist, self.comm = dist, comm
        self.log = log or (lambda *a: None)
        self.n_own = len(own_xyz)
        self.bounds = bounds_list(world, box) if bounds is None else [float(b) for b in bounds]
        self.lo, self.hi = self.bounds[rank], self.bounds[rank + 1]
        self.own_xyz = hip.DeviceArray.from_numpy(own_xyz)
        self.own_ids = hip.DeviceArray.from_numpy(own_ids)
        self.xyz = self.ids = None
        self.n_local = self.n_own
        self.h = 0.0
        self.transport = "none"

    def extent(self):
        """The local points' extent per axis, for the slab tree's split axes
        (nbkd_build_ext): the slab plus its two halo strips in x, the box in y
        and z.  With the reference's depth % 3 a thin slab's leaves are flat
        (35 % more leaves per query at 1/8 of the box)."""
        return (min(self.box, self.hi - self.lo + 2.0 * self.h), self.box, self.box)

    def exchange(self, h, stream=None):
        """(Re)build the local arrays with halo width h."""
        from . import capi, hip

        if self.world > 1:
            check_halo(float(h), self.bounds)
        self.h = float(h)
        if self.world == 1:
            self.xyz, self.ids, self.n_local = self.own_xyz, self.own_ids, self.n_own
            return
        lo, hi = self.lo, self.hi
        dev, s = self.device, stream
        sel = {}
        # open outer bounds, as exchange_host: the last rank owns x == L too
        # (slab_of, io.read_slab), and such a point sits at x = 0 for rank 0
        for name, (a, b) in (("r", (hi - h, math.inf)), ("l", (-math.inf, lo + h))):
            n = capi.slab_select(self.own_xyz.ptr, self.own_ids.ptr, self.n_own, a, b,
                                 device=dev, stream=s)
            bx = hip.DeviceArray((max(n, 1), 3), np.float32)
            bi = hip.DeviceArray((max(n, 1),), np.uint32)
            capi.slab_select(self.own_xyz.ptr, self.own_ids.ptr, self.n_own, a, b, bx.ptr, bi.ptr,
                             n, device=dev, stream=s)
            sel[name] = (n, bx, bi)
        n_fl, n_fr = _strip_counts(self.dist, self.rank, self.world, sel["r"][0], sel["l"][0])
        n_loc = self.n_own + n_fl + n_fr
        xyz = hip.DeviceArray((n_loc, 3), np.float32)
        ids = hip.DeviceArray((n_loc,), np.uint32)
        hip.memcpy(xyz.ptr, self.own_xyz.ptr, self.n_own * 12)
        hip.memcpy(ids.ptr, self.own_ids.ptr, self.n_own * 4)
        o_fl, o_fr = self.n_own, self.n_own + n_fl
        left, right = neighbours(self.rank, self.world)
        done = False
        if self.comm is not None:
            nr, rx, ri = sel["r"]
            nl, lx, li = sel["l"]
            pairs = [
                (rx.ptr, nr * 12, right, xyz.ptr + o_fl * 12, n_fl * 12, left),
                (lx.ptr, nl * 12, left, xyz.ptr + o_fr * 12, n_fr * 12, right),
                (ri.ptr, nr * 4, right, ids.ptr + o_fl * 4, n_fl * 4, left),
                (li.ptr, nl * 4, left, ids.ptr + o_fr * 4, n_fr * 4, right),
            ]
            err = _enqueue_agreed(self.dist, self.rank, "halo exchange",
                                  lambda: self.comm.exchange(pairs, stream=s))
            if err is None:
                hip.synchronize()
                done = True
                self.transport = "rccl"
            else:
                # every rank failed: the gloo path below is exact too.  RCCL may
                # have queued part of the group before failing, so the staged
                # strips go to fresh buffers and the old ones are never freed.
                note_rccl_error(self.rank, "halo exchange failed, staged over gloo", err,
                                self.log)
                _ABANDONED.extend((xyz, ids) + tuple(b for v in sel.values() for b in v[1:]))
                xyz = hip.DeviceArray((n_loc, 3), np.float32)
                ids = hip.DeviceArray((n_loc,), np.uint32)
                hip.memcpy(xyz.ptr, self.own_xyz.ptr, self.n_own * 12)
                hip.memcpy(ids.ptr, self.own_ids.ptr, self.n_own * 4)
        if not done:
            sr = (sel["r"][1].numpy_head(sel["r"][0]), sel["r"][2].numpy_head(sel["r"][0]))
            sl = (sel["l"][1].numpy_head(sel["l"][0]), sel["l"][2].numpy_head(sel["l"][0]))
            import torch

            fl_x, fr_x = _host_sendrecv(self.dist, self.rank, self.world, sr[0], sl[0], n_fl,
                                        n_fr, torch.float32, 3)
            fl_i, fr_i = _host_sendrecv(self.dist, self.rank, self.world,
                                        sr[1].astype(np.int32), sl[1].astype(np.int32), n_fl,
                                        n_fr, torch.int32, 1)
            for arr, off, item in ((fl_x, o_fl, 12), (fr_x, o_fr, 12)):
                a = np.ascontiguousarray(arr, np.float32)
                hip.memcpy(xyz.ptr + off * item, a.ctypes.data, a.nbytes, hip.H2D)
            for arr, off in ((fl_i, o_fl), (fr_i, o_fr)):
                a = np.ascontiguousarray(arr).view(np.uint32)
                hip.memcpy(ids.ptr + off * 4, a.ctypes.data, a.nbytes, hip.H2D)
            self.transport = "gloo-staged"
        if self.transport != "gloo-staged" or self.comm is None:
            for v in sel.values():
                v[1].free()
                v[2].free()
        self.xyz, self.ids, self.n_local = xyz, ids, n_loc

    def violations(self, dist_ptr, k, stream=None):
        from . import capi

        if self.world == 1:
            return 0
        return capi.slab_violations(self.xyz.ptr, dist_ptr, self.n_own, k, self.lo, self.hi,
                                    self.h, device=self.device, stream=stream)


# This process's RCCL failures ("rank r: what: message"), in order: every path
# that falls back to gloo (communicator start, halo exchange, second round,
# redistribution) notes why here, so the bench line can carry the reason
# (halo.rccl_error) instead of leaving it on stderr alone.
RCCL_ERRORS = []


def note_rccl_error(rank, what, err, log=None):
    msg = f"rank {rank}: {what}: {err}"
    RCCL_ERRORS.append(msg)
    if log is not None:
        log(msg)


def init_comm(dist, rank, world, device, log=None, probe=None):
    """RCCL communicator (unique id broadcast over gloo); None if it cannot
    start.  `probe` (tests: a forced failure) replaces nbkd_comm_probe."""
    from . import capi

    log = log or (lambda *a: None)
    if world == 1:
        return None
    import torch

    # every rank loads RCCL (nbkd_comm_probe: no bootstrap listener) before any
    # rank enters ncclCommInitRank, which blocks until all ranks join: a rank
    # that cannot load it would leave the others waiting there for ever
    ok = torch.zeros(1, dtype=torch.int64)
    try:
        (probe or capi.comm_probe)()
        ok[0] = 1
    except Exception as e:
        note_rccl_error(rank, "RCCL unavailable", e, log)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if not int(ok[0]):
        return None
    if probe is not None:  # a probe run (tests): no communicator is started
        return None
    # only rank 0 creates the unique id (ncclGetUniqueId starts the bootstrap
    # root); its last byte says whether that worked
    buf = torch.zeros(capi.COMM_ID_BYTES + 1, dtype=torch.uint8)
    if rank == 0:
        try:
            buf = torch.tensor(list(capi.comm_unique_id()) + [1], dtype=torch.uint8)
        except Exception as e:
            note_rccl_error(rank, "ncclGetUniqueId failed", e, log)
    dist.broadcast(buf, 0)
    if int(buf[-1]) != 1:
        return None
    try:
        c = capi.Comm(bytes(buf[:-1].numpy().tobytes()), rank, world, device)
    except Exception as e:
        note_rccl_error(rank, "ncclCommInitRank failed", e, log)
        c = None
    flag = torch.tensor([1 if c is not None else 0], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if not int(flag[0]):
        if c is not None:
            c.close()
        return None
    return c


def log_stderr(*a):
    print("[slab]", *a, file=sys.stderr, flush=True)


# ------------------------------------------------------- density deposit per slab
def grid_columns(world: int, gx: int, ppu: float, bounds):
    """The W + 1 grid column cuts: rank r holds columns [c_r, c_r+1), c_r the
    column nearest its slab's lower bound (c_0 = 0, c_W = gx)."""
    c = [min(max(int(round(float(b) * ppu)), 0), gx) for b in bounds]
    c[0], c[-1] = 0, gx
    for i in range(1, world + 1):
        c[i] = max(c[i], c[i - 1])
    return c


def deposit_halo(r_max: float, ppu: float) -> float:
    """Halo width for the deposit: a ball's sprite reaches ceil(r ppu) + 1
    voxels past its centre and a column cut sits within half a voxel of the
    slab bound, so r_max + 3 voxels covers every ball touching a rank's columns."""
    return float(r_max) + 3.0 / float(ppu)


def exchange_payload(payload, rank, world, box, h, dist, bounds=None):
    """exchange_host for (n, c) float32 rows whose column 0 is x: own rows,
    then the left neighbour's strip, then the right neighbour's."""
    import torch

    if world == 1:
        return payload
    bounds = bounds_list(world, box) if bounds is None else bounds
    check_halo(h, bounds)
    lo, hi = float(bounds[rank]), float(bounds[rank + 1])
    x = payload[:, 0]
    mr = x >= np.float32(hi - h)
    ml = x < np.float32(lo + h)
    n_fl, n_fr = _strip_counts(dist, rank, world, int(mr.sum()), int(ml.sum()))
    fl, fr = _host_sendrecv(dist, rank, world, payload[mr], payload[ml], n_fl, n_fr,
                            torch.float32, payload.shape[1])
    return np.concatenate([payload, fl.reshape(-1, payload.shape[1]),
                           fr.reshape(-1, payload.shape[1])])


def deposit_slab(own_xyz, own_w, own_r, rank, world, box, grid, ppu, dist, bounds=None,
                 subsample=4, device=-1, engine=None):
    """This rank's x-slab of the periodic sphere deposit over all ranks' balls
    (SURVEY.md 8(f) rank 3 on the 8(e) decomposition): the own balls plus a
    halo of the neighbours' balls within deposit_halo(max radius) are deposited
    into the rank's grid columns only (nbkd_deposit's column window).  No grid
    reduction is needed: the slabs of all ranks tile the grid.

    Returns (c0, slab): the first column and the (wx, gy, nz) float32 slab.
    `engine(xyz, w, r, grid, ppu, period, subsample, window)` defaults to the
    HIP deposit (capi.deposit)."""
    import torch

    gx = int(grid[0])
    bounds = bounds_list(world, box) if bounds is None else [float(b) for b in bounds]
    if engine is None:
        from . import capi

        def engine(xyz, w, r, grid, ppu, period, subsample, window):
            return capi.deposit(xyz, w, r, grid, ppu, period=period, subsample=subsample,
                                device=device, window=window)
    payload = np.column_stack([np.asarray(own_xyz, np.float32), np.asarray(own_w, np.float32),
                               np.asarray(own_r, np.float32)]).astype(np.float32)
    if world > 1:
        rmax = torch.tensor([float(np.max(own_r)) if len(own_r) else 0.0], dtype=torch.float64)
        dist.all_reduce(rmax, op=dist.ReduceOp.MAX)
        h = deposit_halo(float(rmax[0]), ppu)
        payload = exchange_payload(payload, rank, world, box, h, dist, bounds)
    cuts = grid_columns(world, gx, ppu, bounds)
    c0, wx = cuts[rank], cuts[rank + 1] - cuts[rank]
    if wx == 0:
        return c0, np.zeros((0, int(grid[1]), int(grid[2])), np.float32, order="F")
    slab_grid = engine(payload[:, :3], payload[:, 3], payload[:, 4], tuple(int(g) for g in grid),
                       float(ppu), (box, box, box), subsample, (c0, wx))
    return c0, slab_grid


# ------------------------------------------------ second-round exchange (§8(e)(3))
# A slab-local kNN row is exact iff its k-th distance stays inside the x-range
# the local tree covers (own slab +- h).  The rows that reach past a face are
# forwarded: the query goes to the neighbour that owns the far side, which
# answers with its own local kNN (in d2, NBKD_SQUARED), and the owner merges
# the two rows: the union deduplicated by global id (a particle held by both
# trees has the same coordinates, so the same d2), the k smallest by d2, then
# sqrtf (KDTree::find_closest, kdtree/src/cpp/kdtree.cpp:133-159: insertion of
# d2 < k-th, sorted by d2, sqrt last; tournament_tree.hpp:86-91).  The covered
# range then extends to that neighbour's range; a row still reaching past it
# goes one rank further, until every rank has been consulted (then the merge
# is over all particles).  No tree is rebuilt and the halo never widens.
LEFT, RIGHT = 1, 2
_PAD = np.uint32(0xFFFFFFFF)
_D2_PAD = np.float32(np.finfo(np.float32).max)
_TAG_Q_R, _TAG_Q_L, _TAG_A_R, _TAG_A_L = 41, 42, 43, 44


def unwrapped_bound(bounds, i: int, box: float) -> float:
    """Cut i of the periodic sequence of slabs (i may be < 0 or > W)."""
    world = len(bounds) - 1
    return float(bounds[i % world]) + box * (i // world)


def side_needs(x, dk, cl, ch):
    """(needs left, needs right): the f32 test of nbkd_slab_forward / violations_kernel
    (a k-th distance must stay strictly inside [cl, ch) with a relative gap of 4e-7
    and 4 ulps of the larger face)."""
    f32 = np.float32
    x = np.asarray(x, f32)
    dk = np.asarray(dk, f32)
    cl, ch = f32(cl), f32(ch)
    mag = max(abs(cl), abs(ch))
    slack = f32(4.0) * np.spacing(f32(mag))
    rel = f32(1.0 - 4e-7)
    left = ~(dk < (x - cl) * rel - slack)
    right = ~(dk < (ch - x) * rel - slack)
    return left, right


def merge_rows(d2a, ia, d2b, ib, k):
    """Row-wise merge of two (n, k) d2-row sets: the k smallest d2 of the union,
    deduplicated by id, sorted by (d2, id); padding entries (id 0xFFFFFFFF) fill
    the rows that hold fewer than k particles, with d2 = FLT_MAX (the
    reference's k > n rows, sqrtf(FLT_MAX))."""
    d2 = np.concatenate([np.asarray(d2a, np.float32), np.asarray(d2b, np.float32)], axis=1)
    ii = np.concatenate([np.asarray(ia, np.uint32), np.asarray(ib, np.uint32)], axis=1)
    n = d2.shape[0]
    od = np.full((n, k), _D2_PAD, np.float32)
    oi = np.full((n, k), _PAD, np.uint32)
    if n == 0:
        return od, oi
    o = np.lexsort((ii, d2), axis=-1)
    d2 = np.take_along_axis(d2, o, axis=1)
    ii = np.take_along_axis(ii, o, axis=1)
    keep = ii != _PAD
    # deduplicate by id alone: of each id's copies keep the first in (d2, id)
    # order (a stable sort by id keeps that order inside a run of one id), so
    # two trees' copies of one particle never both survive, even if their d2
    # differed in the last bit
    o2 = np.argsort(ii, axis=1, kind="stable")
    s2 = np.take_along_axis(ii, o2, axis=1)
    first = np.ones_like(keep)
    first[:, 1:] = s2[:, 1:] != s2[:, :-1]
    dup = np.empty_like(keep)
    np.put_along_axis(dup, o2, ~first, axis=1)
    keep &= ~dup
    rank = np.cumsum(keep, axis=1) - 1
    sel = keep & (rank < k)
    r, c = np.nonzero(sel)
    od[r, rank[r, c]] = d2[r, c]
    oi[r, rank[r, c]] = ii[r, c]
    return od, oi


def _bytes_sendrecv(dist, right, left, send_r, send_l, n_fl, n_fr, row_shape, dtype, tags):
    """gloo point-to-point of row arrays with explicit peers: send_r -> right,
    send_l -> left; receive n_fl rows from left (its rightward message) and n_fr
    from right (its leftward message).  Distinct tags keep the two directions
    apart when left == right."""
    import torch

    itemsize = int(np.prod(row_shape)) * np.dtype(dtype).itemsize
    rl = torch.empty(max(n_fl, 0) * itemsize, dtype=torch.uint8)
    rr = torch.empty(max(n_fr, 0) * itemsize, dtype=torch.uint8)
    reqs = []
    for arr, peer, tag in ((send_r, right, tags[0]), (send_l, left, tags[1])):
        a = np.ascontiguousarray(arr, dtype)
        if a.size:
            reqs.append(dist.isend(torch.from_numpy(a.reshape(-1).view(np.uint8).copy()), peer,
                                   tag=tag))
    if n_fl:
        reqs.append(dist.irecv(rl, left, tag=tags[0]))
    if n_fr:
        reqs.append(dist.irecv(rr, right, tag=tags[1]))
    for r in reqs:
        r.wait()
    shape = lambda n: (n,) + tuple(row_shape)
    return (rl.numpy().view(dtype).reshape(shape(n_fl)),
            rr.numpy().view(dtype).reshape(shape(n_fr)))


class HostRows:
    """Second-round backend over host arrays (the CPU tests: the oracle is the
    local kNN engine).  knn_sq(q) -> (d2 (n, k) f32, global ids (n, k) u32)."""

    def __init__(self, own_xyz, rows_d, rows_i, knn_sq, k, dist=None, rank=0, world=1):
        self.own_xyz = np.asarray(own_xyz, np.float32)
        self.rows_d, self.rows_i = rows_d, rows_i
        self.knn_sq, self.k = knn_sq, k
        self.dist, self.rank, self.world = dist, rank, world
        self.transport = "gloo"

    def forward(self, cl, ch):
        left, right = side_needs(self.own_xyz[:, 0], self.rows_d[:, self.k - 1], cl, ch)
        sides = left.astype(np.uint8) * LEFT + right.astype(np.uint8) * RIGHT
        u = np.nonzero(sides)[0].astype(np.uint32)
        return u, sides[u]

    def coords(self, u):
        return self.own_xyz[u]

    def exchange(self, right, left, send_r, send_l, n_fl, n_fr, row_shape, dtype, tags):
        return _bytes_sendrecv(self.dist, right, left, send_r, send_l, n_fl, n_fr, row_shape,
                               dtype, tags)

    def write(self, u, d2, ids):
        self.rows_d[u] = np.sqrt(d2)
        self.rows_i[u] = ids


def covered_range(bounds, rank, h):
    """(cl, ch): the x-range a rank's local tree covers, [b_r - h, b_r+1 + h),
    as the f32 values the forward test compares with."""
    f32 = np.float32
    return f32(f32(bounds[rank]) - f32(h)), f32(f32(bounds[rank + 1]) + f32(h))


def second_round(be, rank, world, bounds, box, h, k, dist, log=None):
    """Resolve every own row whose k-th distance reaches past the covered
    x-range; all ranks call it together (it holds
    collectives).  `be`: HostRows or DeviceRows.  Returns counters: the rows
    forwarded at the first hop, the (query, hop) forwards, the hops run."""
    import torch

    st = {"rows_forwarded": 0, "forwards": 0, "hops": 0}
    if world == 1:
        return st
    f32 = np.float32
    cl0, ch0 = covered_range(bounds, rank, h)
    u, sides = be.forward(cl0, ch0)
    t = torch.tensor([len(u)], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    st["rows_forwarded"] = len(u)
    if int(t[0]) == 0:
        return st
    qc = np.ascontiguousarray(be.coords(u), np.float32).reshape(-1, 3)
    s_d2, s_id = be.knn_sq(qc)
    s_d2 = np.array(s_d2, np.float32).reshape(len(u), k)
    s_id = np.array(s_id, np.uint32).reshape(len(u), k)
    rs = np.nonzero(sides & RIGHT)[0]
    ls = np.nonzero(sides & LEFT)[0]
    for j in range(1, world):
        mine = torch.tensor([len(rs), len(ls)], dtype=torch.int64)
        allc = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allc, mine)
        if sum(int(c.sum()) for c in allc) == 0:
            break
        st["hops"] = j
        st["forwards"] += len(rs) + len(ls)
        right, left = (rank + j) % world, (rank - j) % world
        n_fl, n_fr = int(allc[left][0]), int(allc[right][1])
        ql, qr = be.exchange(right, left, qc[rs], qc[ls], n_fl, n_fr, (3,), np.float32,
                             (_TAG_Q_R, _TAG_Q_L))
        a_d2, a_id = be.knn_sq(np.concatenate([ql.reshape(-1, 3), qr.reshape(-1, 3)]))
        a_d2 = np.asarray(a_d2, np.float32).reshape(-1, k)
        a_id = np.asarray(a_id, np.uint32).reshape(-1, k)
        # answers go back the way their queries came: to the right for the
        # queries that came from the right (their left-going rows), and so on
        l_d2, r_d2 = be.exchange(right, left, a_d2[n_fl:], a_d2[:n_fl], len(ls), len(rs), (k,),
                                 np.float32, (_TAG_A_R, _TAG_A_L))
        l_id, r_id = be.exchange(right, left, a_id[n_fl:], a_id[:n_fl], len(ls), len(rs), (k,),
                                 np.uint32, (_TAG_A_R + 10, _TAG_A_L + 10))
        if len(rs):
            s_d2[rs], s_id[rs] = merge_rows(s_d2[rs], s_id[rs], r_d2, r_id, k)
        if len(ls):
            s_d2[ls], s_id[ls] = merge_rows(s_d2[ls], s_id[ls], l_d2, l_id, k)
        dk = np.sqrt(s_d2[:, k - 1])
        ch = f32(f32(unwrapped_bound(bounds, rank + j + 1, box)) + f32(h))
        cl = f32(f32(unwrapped_bound(bounds, rank - j, box)) - f32(h))
        if len(rs):
            rs = rs[side_needs(qc[rs, 0], dk[rs], cl, ch)[1]]
        if len(ls):
            ls = ls[side_needs(qc[ls, 0], dk[ls], cl, ch)[0]]
    be.write(u, s_d2, s_id)
    if log is not None and st["rows_forwarded"]:
        log(f"rank {rank}: {st['rows_forwarded']} rows forwarded, {st['forwards']} forwards "
            f"over {st['hops']} hop(s)")
    return st


class DeviceRows:
    """Second-round backend over a DeviceSlab: the own queries are the first
    n_own rows of ds.xyz, their rows (od, oi device pointers) or their k-th
    distances only (kth device pointer) were written by the local tree, whose
    ids are global (nbkd_set_ids).  The forward test runs on the device
    (nbkd_slab_forward); the few forwarded rows travel over RCCL (device
    buffers, grouped send/recv) when the slab has a communicator, else over
    gloo; the neighbour's answer is its tree's NBKD_SQUARED kNN."""

    def __init__(self, ds, tree, k, od_ptr=None, oi_ptr=None, kth_ptr=None, stream=None,
                 side_ptr=None):
        self.ds, self.tree, self.k = ds, tree, int(k)
        self.od_ptr, self.oi_ptr, self.kth_ptr = od_ptr, oi_ptr, kth_ptr
        # side_ptr: the tree's nbkd_set_kth_out array, holding the last
        # column of the rows the latest kNN wrote: start()'s forward test
        # reads 4 B per row there instead of each row's last line
        self.side_ptr = side_ptr
        self.stream = stream
        self._cap = 0
        self._list = self._sides = None
        self._bufs = {}  # grow-only device buffers, reused across calls
        self.transport = "rccl" if ds.comm is not None else "gloo"
        # start(): the forward test enqueued ahead, its count copied into
        # pinned memory behind an event (no device synchronisation, no hipFree)
        self._dcount = self._hcount = self._ev = None
        self._pending = None

    def _buf(self, key, nbytes):
        from . import hip

        b = self._bufs.get(key)
        if b is None or b.nbytes < nbytes:
            old = 0 if b is None else b.nbytes
            b = hip.DeviceArray((max(int(nbytes), 2 * old, 4096),), np.uint8)
            self._bufs[key] = b
        return b

    def _put(self, key, a):
        """host array -> the reused device buffer `key` (synchronous copy)"""
        from . import hip

        a = np.ascontiguousarray(a)
        b = self._buf(key, a.nbytes)
        hip.memcpy(b.ptr, a.ctypes.data, a.nbytes, hip.H2D)
        return b

    def _sync(self):
        from . import hip

        hip.stream_synchronize(self.stream)

    def _grow(self, n):
        from . import hip

        self._cap = max(n, 2 * self._cap, 1024)
        self._list = hip.DeviceArray((self._cap,), np.uint32)
        self._sides = hip.DeviceArray((self._cap,), np.uint8)

    def start(self, cl, ch):
        """Enqueue the forward test of the current rows (nbkd_slab_forward_async)
        and the copy of its count into pinned host memory, behind an event, on
        the rows' stream.  The following forward(cl, ch) waits for that event
        only: a caller that has queued its next kNN meanwhile (the bench's N > 1
        step) keeps the device busy while it agrees on the count."""
        from . import capi, hip

        ds = self.ds
        if self._cap == 0:
            self._grow(1024)
        if self._dcount is None:
            self._dcount = hip.DeviceArray((1,), np.uint64)
            self._hcount = hip.HostBuffer((1,), np.uint64)
            self._ev = hip.Event()
        if self.kth_ptr is not None:
            dptr, kk = self.kth_ptr, 1
        elif self.side_ptr is not None:
            dptr, kk = self.side_ptr, 1
        else:
            dptr, kk = self.od_ptr, self.k
        capi.slab_forward_async(ds.xyz.ptr, dptr, ds.n_own, kk, cl, ch, self._dcount.ptr,
                                self._list.ptr, self._sides.ptr, self._cap, device=ds.device,
                                stream=self.stream)
        hip.memcpy_async(self._hcount.ptr, self._dcount.ptr, 8, hip.D2H, self.stream)
        self._ev.record(self.stream)
        self._pending = (float(np.float32(cl)), float(np.float32(ch)))

    def wait(self):
        """Block until the count of the last start() is in host memory."""
        if self._pending is not None:
            self._ev.synchronize()

    def forward(self, cl, ch):
        from . import capi

        ds = self.ds
        # the rows themselves here, not side_ptr: a later kNN may have
        # rewritten that array by now (the bench queues its next step first)
        dptr, kk = (self.kth_ptr, 1) if self.kth_ptr is not None else (self.od_ptr, self.k)
        if self._pending == (float(np.float32(cl)), float(np.float32(ch))):
            self._pending = None
            self._ev.synchronize()
            n = int(self._hcount.array[0])
            if n == 0:
                return np.zeros(0, np.uint32), np.zeros(0, np.uint8)
            if n <= self._cap:
                return self._listed(n)
        self._pending = None
        for _ in range(2):
            n = capi.slab_forward(ds.xyz.ptr, dptr, ds.n_own, kk, cl, ch,
                                  self._list.ptr if self._cap else None,
                                  self._sides.ptr if self._cap else None, self._cap,
                                  device=ds.device, stream=self.stream)
            if n <= self._cap:
                break
            self._grow(n)
        if n == 0:
            return np.zeros(0, np.uint32), np.zeros(0, np.uint8)
        return self._listed(n)

    def _listed(self, n):
        u = self._list.numpy_head(n)
        sides = self._sides.numpy_head(n)
        o = np.argsort(u, kind="stable")  # the device list is in completion order
        return u[o], sides[o]

    def coords(self, u):
        from . import capi, hip

        if len(u) == 0:
            return np.zeros((0, 3), np.float32)
        du = self._put("u", np.ascontiguousarray(u, np.uint32))
        dq = self._buf("q", 12 * len(u))
        capi.rows_gather(self.ds.xyz.ptr, 12, du.ptr, len(u), dq.ptr, self.ds.device,
                         self.stream)
        self._sync()
        out = np.empty((len(u), 3), np.float32)
        hip.memcpy(out.ctypes.data, dq.ptr, out.nbytes, hip.D2H)
        return out

    def knn_sq(self, q):
        q = np.ascontiguousarray(q, np.float32).reshape(-1, 3)
        if len(q) == 0:
            return np.zeros((0, self.k), np.float32), np.zeros((0, self.k), np.uint32)
        return self.tree.query(q, self.k, squared=True)

    def exchange(self, right, left, send_r, send_l, n_fl, n_fr, row_shape, dtype, tags):
        if self.ds.comm is None:
            return _bytes_sendrecv(self.ds.dist, right, left, send_r, send_l, n_fl, n_fr,
                                   row_shape, dtype, tags)
        from . import hip

        rb = int(np.prod(row_shape)) * np.dtype(dtype).itemsize
        sr = np.ascontiguousarray(send_r, dtype)
        sl = np.ascontiguousarray(send_l, dtype)
        bs_r, bs_l = self._put("xs_r", sr), self._put("xs_l", sl)
        rl, rr = self._buf("xr_l", n_fl * rb), self._buf("xr_r", n_fr * rb)
        pairs = [(bs_r.ptr, sr.nbytes, right, rl.ptr, n_fl * rb, left),
                 (bs_l.ptr, sl.nbytes, left, rr.ptr, n_fr * rb, right)]
        err = _enqueue_agreed(self.ds.dist, self.ds.rank, "second-round exchange",
                              lambda: self.ds.comm.exchange(pairs, stream=self.stream))
        if err is not None:
            # every rank failed to enqueue: the buffers may still be touched, so
            # they leave the reuse cache and are never freed
            for key in ("xs_r", "xs_l", "xr_l", "xr_r"):
                _ABANDONED.append(self._bufs.pop(key))
            if self.transport != "gloo":  # once per rows object
                note_rccl_error(self.ds.rank, "second-round exchange failed, moved over gloo", err)
            self.transport = "gloo"
            return _bytes_sendrecv(self.ds.dist, right, left, send_r, send_l, n_fl, n_fr,
                                   row_shape, dtype, tags)
        self._sync()
        shape = lambda n: (n,) + tuple(row_shape)
        out_l = np.empty(shape(n_fl), dtype)
        out_r = np.empty(shape(n_fr), dtype)
        hip.memcpy(out_l.ctypes.data, rl.ptr, out_l.nbytes, hip.D2H)
        hip.memcpy(out_r.ctypes.data, rr.ptr, out_r.nbytes, hip.D2H)
        return out_l, out_r

    def write(self, u, d2, ids):
        from . import capi

        if len(u) == 0:
            return
        du = self._put("u", np.ascontiguousarray(u, np.uint32))
        dev, s = self.ds.device, self.stream
        if self.kth_ptr is not None:
            col = self._put("d", np.sqrt(np.ascontiguousarray(d2[:, self.k - 1])))
            capi.rows_scatter(col.ptr, 4, du.ptr, len(u), self.kth_ptr, dev, s)
        else:
            dd = self._put("d", np.sqrt(np.asarray(d2, np.float32)))
            di = self._put("i", np.ascontiguousarray(ids, np.uint32))
            capi.rows_scatter(dd.ptr, 4 * self.k, du.ptr, len(u), self.od_ptr, dev, s)
            capi.rows_scatter(di.ptr, 4 * self.k, du.ptr, len(u), self.oi_ptr, dev, s)
        self._sync()
