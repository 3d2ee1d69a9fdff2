/*
 * nbkd.h — C ABI of the MI355X-native kd-tree (libnbkd.so).
 *
 * Drop-in boundary for the reference's kd-tree hot path (wendazhou/nbodyhpc,
 * kdtree/ subsystem).  Plain pointers and sizes; no exceptions and no C++ or
 * torch types cross this boundary.  The pybind11 module nbodyhpc_amd.kdtree._impl
 * (mirror of kdtree/src/cpp/pybind.cpp) is one caller; a ctypes / cffi / JNI /
 * cgo stub is another.
 *
 * Ownership: the caller owns every input and output buffer; the library owns
 * the tree handle and everything on the device behind it.  Buffers are host
 * memory unless the matching NBKD_*_DEVICE flag is set, in which case they are
 * device pointers on the tree's device.  `stream` is a hipStream_t (NULL = the
 * null stream).  With host outputs a call returns after the results are
 * copied back.  With device outputs nbkd_query_knn / nbkd_query_kth return once
 * the work is enqueued (the re-walk of the queries whose seed ball held fewer
 * than k points runs on grids that read the failure count on the device), and
 * so does nbkd_query_ball_count.  nbkd_query_ball_csr waits (its offsets are
 * host memory), and the first call of a tree, or one needing more scratch than
 * any before it, may also wait while the scratch grows.  Calls on one tree
 * from several host threads run concurrently (the reference's query is const,
 * kdtree/src/cpp/pybind.cpp:90): a tree keeps up to 4 scratch workspaces and
 * each call holds one; a call reusing a workspace from another stream first
 * waits for that workspace's previous call on the device.
 *
 * Host buffers of any size: a kNN, k-th distance or radius-count call with
 * host queries or host outputs runs in batches of "host_batch" queries
 * (nbkd_set_tuning; default ~1 GiB of queries, results and unbudgeted device
 * scratch per batch) through two device slots and two pinned host staging
 * slots: the next batch's queries are copied in and the previous batch's
 * results copied out (DMA on a second stream, host copies on the library's
 * copy threads, "host_threads") while one batch computes, so device scratch
 * stays bounded for any m (the reference streams any m its host memory holds,
 * pybind.cpp:103-104,164-172).
 * Between batches the call runs the thread's interrupt check
 * (nbkd_set_interrupt; the reference polls PyErr_CheckSignals every 1000
 * queries, pybind.cpp:128-133) and returns NBKD_EINTR when it asks to stop.
 *
 * Every entry point returns an nbkd_status; on failure nbkd_last_error()
 * (thread-local) holds a message.  Statuses NBKD_EINVAL / NBKD_EBOX /
 * NBKD_ETOOMANY carry the reference's exact messages (kdtree/src/cpp/pybind.cpp:17,43-45,93;
 * kdtree/src/cpp/kdtree.cpp:99).
 */
#ifndef NBKD_H
#define NBKD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t nbkd_status;

enum {
    NBKD_OK = 0,
    NBKD_EINVAL = 1,   /* bad argument: shape, k <= 0, NULL pointer, ...              */
    NBKD_EBOX = 2,     /* periodic build: a coordinate outside [0, box_size]           */
    NBKD_ETOOMANY = 3, /* more than UINT32_MAX (padded) points                         */
    NBKD_ENOMEM = 4,   /* host or device allocation failed                             */
    NBKD_EDEVICE = 5,  /* HIP runtime error, no device, or kernel failure              */
    NBKD_EINTR = 6     /* the calling thread's interrupt check asked to stop (nbkd_set_interrupt) */
};

/* flags */
#define NBKD_INPUT_DEVICE 0x1u  /* point / query arrays are device pointers */
#define NBKD_OUTPUT_DEVICE 0x2u /* output arrays are device pointers        */
#define NBKD_ACCUMULATE 0x4u    /* nbkd_deposit: add into `out` instead of overwriting it */
#define NBKD_SQUARED 0x8u       /* nbkd_query_knn / _kth: output d2 (no sqrtf), the values
                                   the reference sorts by (kdtree.cpp:149-151) */
#define NBKD_SORTED 0x10u       /* nbkd_query_ball_csr: each row sorted ascending (on the device) */

typedef struct nbkd_tree nbkd_tree;

/* Node record, bit-identical to KDTree::KDTreeNode (kdtree/src/cpp/include/kdtree/kdtree.hpp:149-163). */
typedef struct {
    int32_t dimension; /* split axis, -1 = leaf                               */
    float split;       /* split value (internal nodes), 0.0f for leaves       */
    uint32_t left;     /* internal: left child id;  leaf: first point (tree order) */
    uint32_t right;    /* internal: right child id; leaf: one past the last point  */
} nbkd_node;

/*
 * Build a tree over n points given as an (n, 3) row-major float32 array.
 * Replaces: PyKDTree::PyKDTree / make_positions_and_indices (kdtree/src/cpp/pybind.cpp:14-56,76-88)
 *           and KDTree::KDTree (kdtree/src/cpp/kdtree.cpp:95-131).
 *   leaf_size  as the caller passes it; the reference clamps to >= 16
 *              (kdtree/src/cpp/include/kdtree/kdtree_impl.hpp:88-92).
 *   periodic   0 or 1; when 1 every coordinate must lie in [0, box_size].
 *   device     HIP device ordinal (< 0: the calling thread's current device).
 * The node table equals the reference's for the same (points, leaf_size):
 * preorder, left child = id + 1, split = the m-th order statistic with
 * m = (count/2)/8*8, leaves <= max(leaf_size, 16) points, padded to a multiple
 * of 8 with FLT_MAX coordinates and indices n..n8-1.
 */
nbkd_status nbkd_build(const float *xyz, uint64_t n, int32_t leaf_size, int32_t periodic,
                       float box_size, int32_t device, uint32_t flags, void *stream,
                       nbkd_tree **out);

/* NEW (slab trees): nbkd_build with extent = the points'
 * extent per axis (3 positive floats, host memory; NULL = nbkd_build).  Each
 * depth then splits the axis with the largest remaining extent (halved per
 * split, ties to the lower axis) instead of depth % 3, so a thin slab's
 * leaves are not flat: an x-slab of 1/8 of the box took 35 % more leaves
 * per query with depth % 3.  Same median rule, leaves and padding; the node
 * table differs from the reference's when the schedule does (extent (1, 1, 1)
 * gives depth % 3).  Query results: distances identical; indices identical up
 * to exact-distance ties (the traversal order differs, so which member of a
 * tied group a row holds may too). */
nbkd_status nbkd_build_ext(const float *xyz, uint64_t n, int32_t leaf_size, int32_t periodic,
                           float box_size, const float *extent, int32_t device, uint32_t flags,
                           void *stream, nbkd_tree **out);

/*
 * k nearest neighbours of m query points (row-major (m, 3) float32).
 * Replaces: PyKDTree::query (kdtree/src/cpp/pybind.cpp:90-189) and
 *           KDTree::find_closest (kdtree/src/cpp/kdtree.cpp:133-159).
 * out_dist / out_idx are (m, k) row-major: rows sorted by squared distance,
 * distances = sqrtf(d2); slots beyond the number of points hold
 * (sqrtf(FLT_MAX), 0xFFFFFFFF) as in the reference.
 */
nbkd_status nbkd_query_knn(const nbkd_tree *tree, const float *q, uint64_t m, int32_t k,
                           float *out_dist, uint32_t *out_idx, uint32_t flags, void *stream);

/*
 * Distance to the k-th nearest neighbour of each query (m floats): exactly
 * column k-1 of nbkd_query_knn's out_dist, without writing the (m, k) rows.
 * For local densities k / (4/3 pi r_k^3) and SPH-style smoothing lengths
 * (the per-point radii the reference's rasterizer consumes:
 * rasterization/src/python/nbodyhpc/rasterizer/__init__.py:104-143).
 * Replaces: row[k-1] of PyKDTree::query (pybind.cpp:90-189).  NEW.
 */
nbkd_status nbkd_query_kth(const nbkd_tree *tree, const float *q, uint64_t m, int32_t k,
                           float *out_dist, uint32_t flags, void *stream);

/*
 * NEW (no reference counterpart): number of points with d2 <= r*r of each
 * query (periodic metric when the tree is periodic).  out_count is (m,) uint32.
 */
nbkd_status nbkd_query_ball_count(const nbkd_tree *tree, const float *q, uint64_t m, float r,
                                  uint32_t *out_count, uint32_t flags, void *stream);

/*
 * NEW: neighbour lists within r in CSR form.  out_offsets is (m+1,) uint64
 * (always host memory); out_idx receives offsets[m] original point indices,
 * each row in tree traversal order, or ascending with NBKD_SORTED (a per-row
 * sort on the device).  Call with out_idx == NULL first to get offsets[m]
 * (the required capacity), then again with a buffer of that size.
 * Batched (round 6): the counts stream through the host-buffer pipeline; the
 * fill runs in batches of at most ~64 M ids (a row longer than that is a batch
 * of its own) whose ids are sorted and copied out while the next batch is
 * computed, so device scratch is bounded by the batch, not by m or offsets[m]
 * (the reference streams any m its host memory holds, pybind.cpp:103-104,164-172).
 * Queries and out_idx may be host or device memory (NBKD_INPUT_DEVICE /
 * NBKD_OUTPUT_DEVICE); the call returns when out_idx is complete.  Between
 * batches it runs the thread's interrupt check.
 */
nbkd_status nbkd_query_ball_csr(const nbkd_tree *tree, const float *q, uint64_t m, float r,
                                uint64_t *out_offsets, uint32_t *out_idx, uint64_t capacity,
                                uint32_t flags, void *stream);

/* n8 = padded point count (the reference's `n`), nodes = node count (`size`). */
nbkd_status nbkd_tree_info(const nbkd_tree *tree, uint64_t *n8, uint64_t *nodes,
                           int32_t *periodic, float *box_size, int32_t *device);

/* Copy the node table (nodes entries) and the tree-ordered SoA points and
 * original indices (n8 entries each) to host buffers; any may be NULL. */
nbkd_status nbkd_export(const nbkd_tree *tree, nbkd_node *nodes, float *x, float *y, float *z,
                        uint32_t *idx);

void nbkd_free(nbkd_tree *tree);

/* Process-wide tuning knobs (the library reads no environment variable):
 *   "knn_seed_margin"  a in the seed ball's expected count mu = k + a sqrt(k) + a
 *                      (default 3.0; > 0).  Results never depend on it: a query
 *                      whose seed ball holds fewer than k points is re-walked.
 *   "candidate_bytes"  HBM budget of one collect / select batch's candidate
 *                      columns (default 0 = min(96 GiB, free / 3)).
 *   "host_batch"       queries per batch of a host-buffer call (default 0 =
 *                      about 1 GiB of queries plus results per batch).
 *   "host_threads"     threads copying between the caller's host arrays and
 *                      pinned staging (default 0 = the usable cores, <= 16).
 *   "self_order"       1 (default): a kNN / k-th query whose queries are the
 *                      first m rows of the device array the tree was built from
 *                      (same pointer, NBKD_INPUT_DEVICE) runs in tree order
 *                      instead of bucketing and sorting the queries; 0: always
 *                      bucket and sort.  Results never depend on it (the order
 *                      and the seeds only steer the work).
 *   "pinned_bytes"     process-wide cap on the host-buffer pipeline's pinned
 *                      staging (default 0 = 8 GiB).  A call whose staging would
 *                      pass it, or whose hipHostMalloc fails, streams between
 *                      the caller's pageable arrays and the device instead
 *                      (same results, lower rate).  Idle workspaces release
 *                      their staging when a device allocation needs memory.
 * NEW (no reference counterpart: kdtree/src/cpp/pybind.cpp:196-216 has no knobs). */
nbkd_status nbkd_set_tuning(const char *name, double value);
nbkd_status nbkd_get_tuning(const char *name, double *value);

/* The calling thread's interrupt check: host-buffer query calls (kNN, k-th
 * distance, radius count) call fn(user) between batches and stop with
 * NBKD_EINTR when it returns nonzero (results of that call are then
 * undefined).  NULL removes it.  Replaces the reference's
 * PyErr_CheckSignals poll (kdtree/src/cpp/pybind.cpp:128-133).  NEW. */
typedef int (*nbkd_interrupt_fn)(void *user);
nbkd_status nbkd_set_interrupt(nbkd_interrupt_fn fn, void *user);

/* thread-local message of the last failure on this thread ("" if none) */
const char *nbkd_last_error(void);

/* number of visible HIP devices (0 and NBKD_OK when there are none) */
nbkd_status nbkd_device_count(int32_t *count);

/* Kernel timing with HIP events recorded on the launch stream.  While enabled,
 * each launch of a named kernel is bracketed by events; nbkd_timing_read
 * synchronises them and returns the summed milliseconds and launch count of
 * every launch of `name` since the last reset. */
nbkd_status nbkd_timing_enable(int32_t enable);
nbkd_status nbkd_timing_reset(void);
nbkd_status nbkd_timing_read(const char *name, double *ms, uint64_t *launches);

/* per-query work counters of the last kNN call on this thread (debug builds of
 * the statistics, KDTreeQueryStatistics kdtree/src/cpp/include/kdtree/kdtree.hpp:124-131):
 * sums over all queries of nodes visited and points scanned by the packet
 * traversal.  Enabled with nbkd_stats_enable(1); costs a few % when on. */
nbkd_status nbkd_stats_enable(int32_t enable);
nbkd_status nbkd_stats_read(uint64_t *nodes_visited, uint64_t *points_scanned);
/* all counters of the last kNN call: [0] nodes entered x packet lanes,
 * [1] (query, point) distance evaluations, [2] dense leaf rounds, [3] sparse
 * (lane-compacted) iterations, [4] top-k merges, [5] packets (waves),
 * [6] candidates merged (all lanes), [7] merges while some lane was still filling */
nbkd_status nbkd_stats_read_all(uint64_t *out, int32_t n);

/* ------------------------------------------------------------------ slabs (multi-GPU)
 * NEW (the reference is single-node CPU only).  One process per
 * GPU; the particles are cut into x-slabs [lo, hi) of the periodic box and each
 * rank builds its tree over its own particles plus halo strips of width h
 * received from its two ring neighbours.  All pointers here are device
 * pointers on `device`; xyz arrays are (n, 3) row-major float32. */

/* Replace the tree's point ids: idx[j] <- ids[idx[j]] for the n real points
 * (ids has n entries; host memory unless NBKD_INPUT_DEVICE).  kNN and ball
 * queries then return these ids (e.g. global particle ids of a slab tree). */
nbkd_status nbkd_set_ids(nbkd_tree *tree, const uint32_t *ids, uint32_t flags, void *stream);

/* A device array of `capacity` floats beside the tree's kNN rows: each later
 * nbkd_query_knn of the tree's own points (the first m <= capacity rows of
 * the device array it was built from) with NBKD_OUTPUT_DEVICE also writes
 * every row's last column (its k-th distance, as the row holds it) to
 * kth[row].  A slab's exactness test then reads 4 B per row instead of a
 * row's last line (nbkd_slab_forward_async with dist = kth, k = 1).  kth =
 * NULL or capacity = 0 detaches it; other calls leave it untouched.  The call
 * waits for every kNN of the tree already enqueued (on any stream), so the
 * previously attached array may be freed once it returns. */
nbkd_status nbkd_set_kth_out(nbkd_tree *tree, float *kth, uint64_t capacity);

/* Stable compaction of the points with lo <= x < hi into out_xyz / out_ids
 * (ids may be NULL: then the row number is stored).  *count receives the
 * number selected; with out_xyz or out_ids NULL only the count is computed. */
nbkd_status nbkd_slab_select(const float *xyz, const uint32_t *ids, uint64_t n, float lo, float hi,
                             float *out_xyz, uint32_t *out_ids, uint64_t capacity,
                             uint64_t *count, int32_t device, void *stream);

/* Exactness check of a slab-local kNN result: counts the queries (x in
 * [lo, hi)) whose k-th distance (column k-1 of the (m, k) dist rows) is not
 * strictly inside the local domain [lo - h, hi + h) along x.  Zero means every
 * row equals the single-tree result over all particles. */
nbkd_status nbkd_slab_violations(const float *q, const float *dist, uint64_t m, int32_t k,
                                 float lo, float hi, float h, uint64_t *count, int32_t device,
                                 void *stream);

/* Second-round exchange of a slab-local kNN result: the
 * own queries whose k-th distance (column k-1 of the (m, k) rows `dist`, or
 * the m distances with k = 1) reaches past the left face cl or the right face
 * ch of the covered x-range: bit 0 of out_sides = left, bit 1 = right (the
 * same f32 test as nbkd_slab_violations, split by side).  Up to `capacity`
 * query indices go to out_list (in no particular order); *count receives the
 * total, which may exceed the capacity (call again with a larger buffer). */
nbkd_status nbkd_slab_forward(const float *q, const float *dist, uint64_t m, int32_t k, float cl,
                              float ch, uint32_t *out_list, uint8_t *out_sides, uint64_t capacity,
                              uint64_t *count, int32_t device, void *stream);

/* nbkd_slab_forward without waiting: `count` is a device word (8 B) that the
 * call zeroes and the kernel fills on `stream`; nothing is read back, so a
 * caller can queue its next work before it copies the count out (the bench's
 * N > 1 step overlaps the second round's agreement with the next step). */
nbkd_status nbkd_slab_forward_async(const float *q, const float *dist, uint64_t m, int32_t k,
                                    float cl, float ch, uint32_t *out_list, uint8_t *out_sides,
                                    uint64_t capacity, uint64_t *count, int32_t device,
                                    void *stream);

/* Row gather / scatter of device arrays: dst[i] = src[idx[i]] (gather) or
 * dst[idx[i]] = src[i] (scatter) for n rows of row_bytes (a multiple of 4)
 * bytes; idx is a device array of uint32 row numbers. */
nbkd_status nbkd_rows_gather(const void *src, uint64_t row_bytes, const uint32_t *idx, uint64_t n,
                             void *dst, int32_t device, void *stream);
nbkd_status nbkd_rows_scatter(const void *src, uint64_t row_bytes, const uint32_t *idx, uint64_t n,
                              void *dst, int32_t device, void *stream);

/* RCCL communicator (librccl.so.1 loaded on first use).  Rank 0 calls
 * nbkd_comm_unique_id and distributes the NBKD_COMM_ID_BYTES bytes out of band
 * (e.g. torch.distributed over gloo); every rank then calls nbkd_comm_init. */
#define NBKD_COMM_ID_BYTES 128
typedef struct nbkd_comm nbkd_comm;
nbkd_status nbkd_comm_unique_id(uint8_t *out);
/* NBKD_OK iff librccl.so.1 loads with every symbol the exchange uses; unlike
 * nbkd_comm_unique_id it starts no bootstrap listener (every rank may call it). */
nbkd_status nbkd_comm_probe(void);
nbkd_status nbkd_comm_init(const uint8_t *id, int32_t rank, int32_t world, int32_t device,
                           nbkd_comm **out);
/* One grouped set of point-to-point byte transfers: for each i, send
 * send_bytes[i] from send[i] to rank send_peer[i] and receive recv_bytes[i]
 * into recv[i] from rank recv_peer[i] (zero sizes skip).  Transfers between
 * one pair of ranks are matched in posting order.  Enqueued on `stream`. */
nbkd_status nbkd_comm_exchange(nbkd_comm *comm, int32_t npairs, const void *const *send,
                               const uint64_t *send_bytes, const int32_t *send_peer,
                               void *const *recv, const uint64_t *recv_bytes,
                               const int32_t *recv_peer, void *stream);
void nbkd_comm_free(nbkd_comm *comm);

/*
 * Deposit n spheres (centres xyz row-major (n, 3), weight[n], radius[n]) onto a
 * voxel grid, with the semantics of the reference's point rasteriser:
 * replaces PointRenderer::render_points_volume / render_points
 * (rasterization/src/cpp/point_renderer.cpp:606-657,825-950), assemble_vertices
 * (rasterization/src/cpp/pybind.cpp:25-71), augment_vertices_periodic
 * (rasterization/src/cpp/vertex_utilities.cpp:15-42) and the vertex / fragment
 * shaders (rasterization/shaders/triangle.vert, triangle.frag).
 *   out        gx * gy * nz float32, element (px, py, s) at px + gx * (py + gy * s)
 *              (the reference's column-major (gx, gy, nz) array); zeroed first
 *              unless NBKD_ACCUMULATE is set.
 *   pixels_per_unit  voxels per unit length (> 0).
 *   period     3 floats (NULL = none); period[d] > 0 wraps axis d with that length.
 *   subsample  S: each straddled voxel is sampled at S^3 points (1..16).
 *   mode       0: nz slices [s, s+1) / ppu (render_points_volume);
 *              1: one plane at z = 0 (render_points; nz must be 1).
 *   x0, wx     `out` holds only the columns [x0, x0 + wx) of the gx-wide grid,
 *              element (px, py, s) at (px - x0) + wx * (py + gy * s); sprites,
 *              periodic images and clipping are those of the whole grid
 *              (0, gx: the whole grid).  One rank's x-slab (nbodyhpc_amd/slab.py).
 * A voxel receives weight * (sub-samples inside the ball) / S^3 / (4/3 pi R^3)
 * (R the radius in voxels); a ball under half a voxel across deposits its whole
 * weight in the voxel holding its centre.
 */
nbkd_status nbkd_deposit(const float *xyz, const float *weight, const float *radius, uint64_t n,
                         int32_t gx, int32_t gy, int32_t nz, float pixels_per_unit,
                         const float *period, int32_t subsample, int32_t mode, int32_t x0,
                         int32_t wx, float *out, int32_t device, uint32_t flags, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* NBKD_H */
