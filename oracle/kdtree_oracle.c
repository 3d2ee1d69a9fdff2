/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product (nbodyhpc_amd / libnbkd.so).  Only tests/, the smoke() check
 * in __graft_entry__.py and bench.py's cpu_baseline leg may use it, and only as
 * the checker / CPU baseline, never as the thing measured or shipped.
 *
 * Plain-C restatement of the reference kd-tree hot path
 * (wendazhou/nbodyhpc, kdtree/ subsystem; paths relative to /root/reference):
 *
 *   padding / SoA / box check   kdtree/src/cpp/pybind.cpp:14-56
 *   build (median split)        kdtree/src/cpp/include/kdtree/kdtree_impl.hpp:78-146
 *                               (leaf_size_ = max(leaf, 2*block) :88-92, m = (count/2)/8*8 :108-109)
 *   constructor checks          kdtree/src/cpp/kdtree.cpp:95-131
 *   distance metrics            kdtree/src/cpp/include/kdtree/kdtree.hpp:20-121
 *   traversal                   kdtree/src/cpp/include/kdtree/kdtree_impl.hpp:226-268
 *   loser (tournament) tree     kdtree/src/cpp/include/kdtree/tournament_tree.hpp:18-105
 *   leaf scan (asm semantics)   kdtree/src/cpp/kdtree_asm_systemv.asm:3-61,76-188
 *                               kdtree/src/cpp/include/kdtree/kdtree_opt.hpp:20-44 (Vanilla)
 *   finalisation (sort, sqrt)   kdtree/src/cpp/kdtree.cpp:133-159
 *   query batch / threads       kdtree/src/cpp/pybind.cpp:90-172,
 *                               kdtree/third_party/misc/thread_pool.hpp:148-183
 *   naive kNN (house KAT)       kdtree/src/cpp/tests/test.cpp:14-37
 *
 * Selection: the reference selects with Floyd-Rivest (kdtree_selection.cpp:
 * 322-368) over an AVX2 vectorised partition; fr_select below restates the same
 * sample-window recursion (integer pivot-side test, truncating window bounds)
 * over a scalar Hoare partition.  Only the order statistic, i.e. the split
 * value, is pinned: where several points tie at a split value, which of them
 * land left depends on the partition, so leaf membership and the descendants'
 * splits under such ties can differ from the reference.
 *
 * Radius query (query_ball) is NEW capability (no reference code): brute-force
 * semantics are "count points with d2 <= r*r", d2 computed with the same f32
 * formula as the kNN path.
 *
 * Build with -ffp-contract=off: the reference is compiled with -mavx2 and no
 * -mfma (kdtree/CMakeLists.txt:74), so no product is fused into an add.
 */
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_EXPORT __attribute__((visibility("default")))

typedef struct {
    int32_t dim; /* -1 = leaf */
    float split;
    uint32_t left;
    uint32_t right;
} orc_node; /* KDTree::KDTreeNode, kdtree.hpp:149-163 (16 B) */

typedef struct {
    int64_t n8;
    int64_t nnodes;
    int64_t cap_nodes;
    float *x, *y, *z;
    uint32_t *idx;
    orc_node *nodes;
    int periodic;
    float box;
} orc_tree;

/* status codes mirror include/nbkd.h */
enum { ORC_OK = 0, ORC_EINVAL = 1, ORC_EBOX = 2, ORC_ETOOMANY = 3, ORC_ENOMEM = 4 };

/* ------------------------------------------------------------------ metrics */

/* L2Distance::operator() kdtree.hpp:23-31 == asm compute_distance_l2 :76-87 */
static inline float d2_l2(float qx, float qy, float qz, float px, float py, float pz) {
    float dx = px - qx, dy = py - qy, dz = pz - qz;
    float a = dx * dx, b = dy * dy, c = dz * dz;
    return (a + b) + c;
}

static inline float min3f(float a, float b, float c) {
    float m = a < b ? a : b;
    return m < c ? m : c;
}

/* L2PeriodicDistance::operator() kdtree.hpp:72-84 == asm :89-119 */
static inline float d2_per(float qx, float qy, float qz, float px, float py, float pz, float L) {
    float dx = px - qx, dy = py - qy, dz = pz - qz;
    float xm = dx - L, xp = dx + L, ym = dy - L, yp = dy + L, zm = dz - L, zp = dz + L;
    float a = min3f(dx * dx, xm * xm, xp * xp);
    float b = min3f(dy * dy, ym * ym, yp * yp);
    float c = min3f(dz * dz, zm * zm, zp * zp);
    return (a + b) + c;
}

/* L2Distance::box_distance kdtree.hpp:35-45 */
static inline float box_l2(const float q[3], const float box[6]) {
    float r = 0.0f;
    for (int i = 0; i < 3; ++i) {
        float dl = box[2 * i] - q[i];
        dl = dl > 0.0f ? dl : 0.0f;
        float dr = q[i] - box[2 * i + 1];
        dr = dr > 0.0f ? dr : 0.0f;
        float s = dl * dl;
        float t = dr * dr;
        r += s + t;
    }
    return r;
}

/* L2PeriodicDistance::box_distance kdtree.hpp:89-107 */
static inline float box_per(const float q[3], const float box[6], float L) {
    float r = 0.0f;
    for (int i = 0; i < 3; ++i) {
        float lo = box[2 * i], hi = box[2 * i + 1];
        if (q[i] < lo) {
            float d = lo - q[i];
            float w = (q[i] + L) - hi;
            float m = w < d ? w : d;
            r += m * m;
        } else if (q[i] > hi) {
            float d = q[i] - hi;
            float w = (lo + L) - q[i];
            float m = w < d ? w : d;
            r += m * m;
        }
    }
    return r;
}

ORC_EXPORT float orc_point_d2(const float q[3], const float p[3], int periodic, float L) {
    return periodic ? d2_per(q[0], q[1], q[2], p[0], p[1], p[2], L)
                    : d2_l2(q[0], q[1], q[2], p[0], p[1], p[2]);
}

ORC_EXPORT float orc_box_d2(const float q[3], const float box[6], int periodic, float L) {
    return periodic ? box_per(q, box, L) : box_l2(q, box);
}

/* ------------------------------------------------------------------ build */

/* pybind.cpp:14-56: AoS -> SoA, periodic range check, pad to multiple of 8 with
 * FLT_MAX coordinates and iota indices. */
static int make_positions(orc_tree *t, const float *aos, int64_t n) {
    int64_t n8 = (n + 7) / 8 * 8;
    if (n8 > (int64_t)UINT32_MAX) return ORC_ETOOMANY; /* kdtree.cpp:98-100 */
    t->n8 = n8;
    size_t bytes = (size_t)(n8 ? n8 : 1) * sizeof(float);
    t->x = (float *)malloc(bytes);
    t->y = (float *)malloc(bytes);
    t->z = (float *)malloc(bytes);
    t->idx = (uint32_t *)malloc((size_t)(n8 ? n8 : 1) * sizeof(uint32_t));
    if (!t->x || !t->y || !t->z || !t->idx) return ORC_ENOMEM;
    float *c[3] = {t->x, t->y, t->z};
    for (int64_t i = 0; i < n8; ++i) t->idx[i] = (uint32_t)i;
    for (int d = 0; d < 3; ++d) {
        for (int64_t i = 0; i < n; ++i) c[d][i] = aos[3 * i + d];
        if (t->periodic) {
            for (int64_t i = 0; i < n; ++i) {
                float v = c[d][i];
                if (!(v >= 0.0f && v <= t->box)) return ORC_EBOX;
            }
        }
        for (int64_t i = n; i < n8; ++i) c[d][i] = FLT_MAX;
    }
    return ORC_OK;
}

typedef struct {
    float k;
    float x, y, z;
    uint32_t id;
} orc_pt;

static inline void swap_pt(orc_pt *a, orc_pt *b) {
    orc_pt t = *a;
    *a = *b;
    *b = t;
}

/* Floyd-Rivest selection (the recursion of kdtree_selection.cpp:322-368: a
 * sample window when the range exceeds 600 elements, the pivot side flipped by
 * the integer test i < n / 2, window bounds truncated to integers), then a
 * scalar Hoare partition around the sampled pivot where the reference runs its
 * AVX2 partition (pivot at the right end).  Afterwards p[m].k is the m-th order
 * statistic of p[0..n) and p[0..m) <= p[m] <= p[m+1..n).  Only that order
 * statistic (the split value) is pinned to the reference; the order of the
 * other elements, and so which of several points tied at the split land left,
 * is this partition's own. */
static void fr_select(orc_pt *p, int64_t left, int64_t right, int64_t m) {
    while (right > left) {
        if (right - left > 600) {
            const int64_t ni = right - left + 1, ii = m - left + 1;
            const double n = (double)ni, i = (double)ii;
            const double z = log(n);
            const double sz = 0.5 * exp(2.0 * z / 3.0);
            /* the reference's ptrdiff_t test (kdtree_selection.cpp:340) */
            const double sd = 0.5 * sqrt(z * sz * (n - sz) / n) * (ii < ni / 2 ? -1.0 : 1.0);
            /* static_cast<ptrdiff_t>: truncation toward zero (kdtree_selection.cpp:343-344) */
            int64_t nl = (int64_t)((double)m - i * sz / n + sd);
            int64_t nr = (int64_t)((double)m + (n - i) * sz / n + sd);
            if (nl < left) nl = left;
            if (nr > right) nr = right;
            fr_select(p, nl, nr, m);
        }
        const float t = p[m].k;
        int64_t i = left, j = right;
        swap_pt(&p[left], &p[m]);
        if (p[right].k > t) swap_pt(&p[right], &p[left]);
        while (i < j) {
            swap_pt(&p[i], &p[j]);
            ++i;
            --j;
            while (p[i].k < t) ++i;
            while (p[j].k > t) --j;
        }
        if (p[left].k == t) {
            swap_pt(&p[left], &p[j]);
        } else {
            ++j;
            swap_pt(&p[j], &p[right]);
        }
        if (j <= m) left = j + 1;
        if (m <= j) right = j - 1;
    }
}

static void quickselect(orc_pt *p, int64_t n, int64_t m) { fr_select(p, 0, n - 1, m); }

static int push_node(orc_tree *t, orc_node nd) {
    if (t->nnodes == t->cap_nodes) {
        int64_t cap = t->cap_nodes ? 2 * t->cap_nodes : 64;
        orc_node *nn = (orc_node *)realloc(t->nodes, (size_t)cap * sizeof(orc_node));
        if (!nn) return -1;
        t->nodes = nn;
        t->cap_nodes = cap;
    }
    t->nodes[t->nnodes] = nd;
    return (int)(t->nnodes++);
}

/* KDTreeBuilder::build_node, kdtree_impl.hpp:98-146 (non-threaded branch :148-157) */
static int64_t build_node(orc_tree *t, orc_pt *pts, int dim, uint32_t left, uint32_t count,
                          uint32_t leaf) {
    if (count <= leaf) {
        orc_node nd = {-1, 0.0f, left, left + count};
        return push_node(t, nd);
    }
    uint32_t m = count / 2;
    m = (m / 8) * 8;
    orc_pt *seg = pts + left;
    for (uint32_t i = 0; i < count; ++i) seg[i].k = dim == 0 ? seg[i].x : (dim == 1 ? seg[i].y : seg[i].z);
    quickselect(seg, count, m);
    float split = seg[m].k;
    orc_node nd = {dim, split, 0u, 0u};
    int64_t cur = push_node(t, nd);
    if (cur < 0) return -1;
    int64_t l = build_node(t, pts, (dim + 1) % 3, left, m, leaf);
    int64_t r = build_node(t, pts, (dim + 1) % 3, left + m, count - m, leaf);
    if (l < 0 || r < 0) return -1;
    t->nodes[cur].left = (uint32_t)l;
    t->nodes[cur].right = (uint32_t)r;
    return cur;
}

ORC_EXPORT void orc_free(orc_tree *t) {
    if (!t) return;
    free(t->x);
    free(t->y);
    free(t->z);
    free(t->idx);
    free(t->nodes);
    free(t);
}

/* box <= 0 or periodic == 0 -> non-periodic */
ORC_EXPORT int orc_build(const float *aos, int64_t n, int32_t leafsize, int32_t periodic, float box,
                         orc_tree **out) {
    *out = NULL;
    if (n < 0) return ORC_EINVAL;
    orc_tree *t = (orc_tree *)calloc(1, sizeof(orc_tree));
    if (!t) return ORC_ENOMEM;
    t->periodic = periodic ? 1 : 0;
    t->box = periodic ? box : 0.0f;
    int st = make_positions(t, aos, n);
    if (st) {
        orc_free(t);
        return st;
    }
    /* leaf_size_ = max(leaf_size, 2 * block_size) with block_size 8, kdtree_impl.hpp:88-92.
     * The int -> size_t conversion there makes negative leaf sizes huge. */
    uint64_t leaf = leafsize < 0 ? (uint64_t)(int64_t)leafsize : (uint64_t)leafsize;
    if (leaf < 16) leaf = 16;
    if (leaf > UINT32_MAX) leaf = UINT32_MAX;
    orc_pt *pts = (orc_pt *)malloc((size_t)(t->n8 ? t->n8 : 1) * sizeof(orc_pt));
    if (!pts) {
        orc_free(t);
        return ORC_ENOMEM;
    }
    for (int64_t i = 0; i < t->n8; ++i) {
        pts[i].x = t->x[i];
        pts[i].y = t->y[i];
        pts[i].z = t->z[i];
        pts[i].id = t->idx[i];
    }
    if (build_node(t, pts, 0, 0, (uint32_t)t->n8, (uint32_t)leaf) < 0) {
        free(pts);
        orc_free(t);
        return ORC_ENOMEM;
    }
    for (int64_t i = 0; i < t->n8; ++i) {
        t->x[i] = pts[i].x;
        t->y[i] = pts[i].y;
        t->z[i] = pts[i].z;
        t->idx[i] = pts[i].id;
    }
    free(pts);
    *out = t;
    return ORC_OK;
}

ORC_EXPORT int64_t orc_n8(const orc_tree *t) { return t->n8; }
ORC_EXPORT int64_t orc_num_nodes(const orc_tree *t) { return t->nnodes; }

ORC_EXPORT void orc_export(const orc_tree *t, orc_node *nodes, float *x, float *y, float *z,
                           uint32_t *idx) {
    if (nodes) memcpy(nodes, t->nodes, (size_t)t->nnodes * sizeof(orc_node));
    if (x) memcpy(x, t->x, (size_t)t->n8 * sizeof(float));
    if (y) memcpy(y, t->y, (size_t)t->n8 * sizeof(float));
    if (z) memcpy(z, t->z, (size_t)t->n8 * sizeof(float));
    if (idx) memcpy(idx, t->idx, (size_t)t->n8 * sizeof(uint32_t));
}

/* ------------------------------------------------------------------ loser tree */

typedef struct {
    float d;
    uint32_t id;
    uint32_t slot;
} orc_entry; /* pair<pair<float,uint32>,uint32>: 12 B, as the asm addresses it */

/* TournamentTree(n, val), tournament_tree.hpp:18-36,70-77 */
static void lt_init(orc_entry *data, uint32_t n, uint32_t *wtmp) {
    /* wtmp: 2n winners; loser of internal node i = min(child winners) */
    for (uint32_t i = 0; i < n; ++i) wtmp[i + n] = i;
    for (uint32_t i = 0; i < 2 * n; ++i) {
        data[i].d = FLT_MAX;
        data[i].id = 0xFFFFFFFFu;
    }
    for (uint32_t i = n - 1; i > 0; --i) {
        uint32_t a = wtmp[2 * i], b = wtmp[2 * i + 1];
        wtmp[i] = a > b ? a : b;
        data[i].slot = (a < b ? a : b) + n;
    }
    for (uint32_t i = n; i < 2 * n; ++i) data[i].slot = i;
    data[0].slot = 2 * n - 1;
}

/* replace_top + update_root_from_index, tournament_tree.hpp:49-64,86-91 */
static inline void lt_replace_top(orc_entry *data, float d, uint32_t id) {
    uint32_t s = data[0].slot;
    data[s].d = d;
    data[s].id = id;
    data[s].slot = s;
    orc_entry w = data[s];
    uint32_t i = s;
    while (i > 1) {
        i >>= 1;
        if (w.d < data[i].d) { /* PairLessFirst: previous winner lost */
            orc_entry t = data[i];
            data[i] = w;
            w = t;
        }
    }
    data[0] = w;
}

/* ------------------------------------------------------------------ query */

typedef struct {
    const orc_tree *t;
    float q[3];
    orc_entry *lt;
    uint64_t visited, pruned, points;
} orc_query;

/* process_leaf + insert semantics: kdtree_impl.hpp:212-220, asm :148-188.
 * Like the asm, a block of 8 distances is computed first (a loop gcc turns into
 * AVX2 at -O3 -mavx2; no FMA, -ffp-contract=off), then each lane is re-checked
 * against the current top in order (asm :168-169).  Leaves hold multiples of 8
 * points (splits at multiples of 8, n padded to n8). */
static void process_leaf(orc_query *Q, const orc_node *nd) {
    const orc_tree *t = Q->t;
    const float qx = Q->q[0], qy = Q->q[1], qz = Q->q[2], L = t->box;
    float top = Q->lt[0].d;
    float d[8];
    for (uint32_t i = nd->left; i < nd->right; i += 8) {
        const float *px = t->x + i, *py = t->y + i, *pz = t->z + i;
        if (t->periodic) {
            for (int j = 0; j < 8; ++j) d[j] = d2_per(qx, qy, qz, px[j], py[j], pz[j], L);
        } else {
            for (int j = 0; j < 8; ++j) d[j] = d2_l2(qx, qy, qz, px[j], py[j], pz[j]);
        }
        for (int j = 0; j < 8; ++j) {
            if (d[j] < top) {
                lt_replace_top(Q->lt, d[j], t->idx[i + j]);
                top = Q->lt[0].d;
            }
        }
    }
    Q->points += nd->right - nd->left;
}

/* KDTreeQuery::compute, kdtree_impl.hpp:226-268 */
static void compute(orc_query *Q, const orc_node *node, const float bounds[6]) {
    const orc_tree *t = Q->t;
    Q->visited += 1;
    if (node->dim == -1) {
        process_leaf(Q, node);
        return;
    }
    const orc_node *closer = t->nodes + node->left;
    const orc_node *further = t->nodes + node->right;
    int cbd = 2 * node->dim + 1, fbd = 2 * node->dim;
    if (Q->q[node->dim] > node->split) {
        const orc_node *tmp = closer;
        closer = further;
        further = tmp;
        int ti = cbd;
        cbd = fbd;
        fbd = ti;
    }
    {
        float cb[6];
        memcpy(cb, bounds, sizeof(cb));
        cb[cbd] = node->split;
        float d = t->periodic ? box_per(Q->q, cb, t->box) : box_l2(Q->q, cb);
        if (d < Q->lt[0].d)
            compute(Q, closer, cb);
        else
            Q->pruned += 1;
    }
    float fb[6];
    memcpy(fb, bounds, sizeof(fb));
    fb[fbd] = node->split;
    float d = t->periodic ? box_per(Q->q, fb, t->box) : box_l2(Q->q, fb);
    if (Q->lt[0].d < d) {
        Q->pruned += 1;
        return;
    }
    compute(Q, further, fb);
}

/* stable sort of k results by d (ties keep loser-tree leaf order) */
static void sort_results(orc_entry *r, uint32_t k) {
    for (uint32_t i = 1; i < k; ++i) {
        orc_entry v = r[i];
        uint32_t j = i;
        while (j > 0 && v.d < r[j - 1].d) {
            r[j] = r[j - 1];
            --j;
        }
        r[j] = v;
    }
}

/* KDTree::find_closest, kdtree.cpp:133-159.  want_sqrt = 0 returns d2. */
static void find_closest(const orc_tree *t, const float q[3], uint32_t k, orc_entry *lt,
                         uint32_t *wtmp, float *out_d, uint32_t *out_i, int want_sqrt,
                         uint64_t stats[3]) {
    orc_query Q;
    Q.t = t;
    Q.q[0] = q[0];
    Q.q[1] = q[1];
    Q.q[2] = q[2];
    Q.lt = lt;
    Q.visited = Q.pruned = Q.points = 0;
    lt_init(lt, k, wtmp);
    float bounds[6];
    for (int i = 0; i < 3; ++i) { /* initial_box kdtree.hpp:52-61, :111-120 */
        bounds[2 * i] = t->periodic ? 0.0f : -FLT_MAX;
        bounds[2 * i + 1] = t->periodic ? t->box : FLT_MAX;
    }
    if (t->nnodes > 0) compute(&Q, t->nodes, bounds);
    orc_entry *res = lt + k; /* copy_values: leaves data[k..2k) */
    sort_results(res, k);
    for (uint32_t j = 0; j < k; ++j) {
        out_d[j] = want_sqrt ? sqrtf(res[j].d) : res[j].d;
        out_i[j] = res[j].id;
    }
    if (stats) {
        stats[0] += Q.visited;
        stats[1] += Q.pruned;
        stats[2] += Q.points;
    }
}

typedef struct {
    const orc_tree *t;
    const float *q;
    int64_t begin, end;
    uint32_t k;
    float *out_d;
    uint32_t *out_i;
    int want_sqrt;
    uint64_t stats[3];
    int err;
} knn_job;

static void *knn_worker(void *arg) {
    knn_job *J = (knn_job *)arg;
    orc_entry *lt = (orc_entry *)malloc(2 * (size_t)J->k * sizeof(orc_entry));
    uint32_t *wtmp = (uint32_t *)malloc(2 * (size_t)J->k * sizeof(uint32_t));
    if (!lt || !wtmp) {
        J->err = ORC_ENOMEM;
        free(lt);
        free(wtmp);
        return NULL;
    }
    uint64_t st[3] = {0, 0, 0}; /* local: adjacent jobs' counters would share lines */
    for (int64_t i = J->begin; i < J->end; ++i)
        find_closest(J->t, J->q + 3 * i, J->k, lt, wtmp, J->out_d + (size_t)i * J->k,
                     J->out_i + (size_t)i * J->k, J->want_sqrt, st);
    J->stats[0] = st[0];
    J->stats[1] = st[1];
    J->stats[2] = st[2];
    free(lt);
    free(wtmp);
    return NULL;
}

/* PyKDTree::query, pybind.cpp:90-172: workers contiguous blocks
 * (thread_pool::parallelize_loop, thread_pool.hpp:148-183).
 * stats (optional): sums of nodes_visited, nodes_pruned, points_visited. */
ORC_EXPORT int orc_knn(const orc_tree *t, const float *q, int64_t m, int32_t k, int32_t workers,
                       int32_t want_sqrt, float *out_d, uint32_t *out_i, uint64_t *stats) {
    if (k <= 0) return ORC_EINVAL;
    if (workers < 1) workers = 1;
    if (workers > 256) workers = 256;
    if ((int64_t)workers > m) workers = m > 0 ? (int32_t)m : 1;
    knn_job jobs[256];
    pthread_t th[256];
    int64_t blk = m / workers, rem = m % workers, pos = 0;
    for (int w = 0; w < workers; ++w) {
        int64_t cnt = blk + (w < rem ? 1 : 0);
        jobs[w] = (knn_job){t, q, pos, pos + cnt, (uint32_t)k, out_d, out_i, want_sqrt, {0, 0, 0}, 0};
        pos += cnt;
    }
    if (workers == 1) {
        knn_worker(&jobs[0]);
    } else {
        for (int w = 0; w < workers; ++w) pthread_create(&th[w], NULL, knn_worker, &jobs[w]);
        for (int w = 0; w < workers; ++w) pthread_join(th[w], NULL);
    }
    int err = 0;
    for (int w = 0; w < workers; ++w) {
        if (jobs[w].err) err = jobs[w].err;
        if (stats) {
            stats[0] += jobs[w].stats[0];
            stats[1] += jobs[w].stats[1];
            stats[2] += jobs[w].stats[2];
        }
    }
    return err;
}

/* ------------------------------------------------------------------ brute force */

/* find_nearest_naive, tests/test.cpp:14-37: priority queue with `dist < top`
 * insertion, then sort, then sqrt.  Here the queue is the same loser tree. */
ORC_EXPORT int orc_knn_brute(const float *aos, int64_t n, int32_t periodic, float box,
                             const float *q, int64_t m, int32_t k, int32_t want_sqrt, float *out_d,
                             uint32_t *out_i) {
    if (k <= 0) return ORC_EINVAL;
    orc_entry *lt = (orc_entry *)malloc(2 * (size_t)k * sizeof(orc_entry));
    uint32_t *wtmp = (uint32_t *)malloc(2 * (size_t)k * sizeof(uint32_t));
    if (!lt || !wtmp) {
        free(lt);
        free(wtmp);
        return ORC_ENOMEM;
    }
    for (int64_t j = 0; j < m; ++j) {
        const float *qq = q + 3 * j;
        lt_init(lt, (uint32_t)k, wtmp);
        float top = lt[0].d;
        for (int64_t i = 0; i < n; ++i) {
            const float *p = aos + 3 * i;
            float d = periodic ? d2_per(qq[0], qq[1], qq[2], p[0], p[1], p[2], box)
                               : d2_l2(qq[0], qq[1], qq[2], p[0], p[1], p[2]);
            if (d < top) {
                lt_replace_top(lt, d, (uint32_t)i);
                top = lt[0].d;
            }
        }
        orc_entry *res = lt + k;
        sort_results(res, (uint32_t)k);
        for (int32_t i = 0; i < k; ++i) {
            out_d[j * k + i] = want_sqrt ? sqrtf(res[i].d) : res[i].d;
            out_i[j * k + i] = res[i].id;
        }
    }
    free(lt);
    free(wtmp);
    return ORC_OK;
}

/* NEW (no reference): radius count, brute force.  d2 <= r*r, same d2 formula. */
ORC_EXPORT int orc_ball_count_brute(const float *aos, int64_t n, int32_t periodic, float box,
                                    const float *q, int64_t m, float r, uint32_t *out_count) {
    float r2 = r * r;
    for (int64_t j = 0; j < m; ++j) {
        const float *qq = q + 3 * j;
        uint32_t c = 0;
        for (int64_t i = 0; i < n; ++i) {
            const float *p = aos + 3 * i;
            float d = periodic ? d2_per(qq[0], qq[1], qq[2], p[0], p[1], p[2], box)
                               : d2_l2(qq[0], qq[1], qq[2], p[0], p[1], p[2]);
            c += d <= r2;
        }
        out_count[j] = c;
    }
    return ORC_OK;
}

/* NEW (no reference): radius count through the tree.  Same DFS, pruning by
 * box distance > r*r. Used as the CPU baseline of the ball path. */
static uint64_t g_ball_nodes, g_ball_points; /* orc_ball_count_stats (single thread) */

static uint32_t ball_rec(const orc_tree *t, const orc_node *node, const float q[3], float bounds[6],
                         float r2) {
    ++g_ball_nodes;
    if (node->dim == -1) {
        uint32_t c = 0;
        g_ball_points += node->right - node->left;
        for (uint32_t i = node->left; i < node->right; ++i) {
            float d = t->periodic ? d2_per(q[0], q[1], q[2], t->x[i], t->y[i], t->z[i], t->box)
                                  : d2_l2(q[0], q[1], q[2], t->x[i], t->y[i], t->z[i]);
            c += d <= r2;
        }
        return c;
    }
    uint32_t c = 0;
    float lb[6], rb[6];
    memcpy(lb, bounds, sizeof(lb));
    memcpy(rb, bounds, sizeof(rb));
    lb[2 * node->dim + 1] = node->split;
    rb[2 * node->dim] = node->split;
    float dl = t->periodic ? box_per(q, lb, t->box) : box_l2(q, lb);
    float dr = t->periodic ? box_per(q, rb, t->box) : box_l2(q, rb);
    if (dl <= r2) c += ball_rec(t, t->nodes + node->left, q, lb, r2);
    if (dr <= r2) c += ball_rec(t, t->nodes + node->right, q, rb, r2);
    return c;
}

ORC_EXPORT int orc_ball_count(const orc_tree *t, const float *q, int64_t m, float r,
                              uint32_t *out_count) {
    float r2 = r * r;
    for (int64_t j = 0; j < m; ++j) {
        float bounds[6];
        for (int i = 0; i < 3; ++i) {
            bounds[2 * i] = t->periodic ? 0.0f : -FLT_MAX;
            bounds[2 * i + 1] = t->periodic ? t->box : FLT_MAX;
        }
        out_count[j] = t->nnodes ? ball_rec(t, t->nodes, q + 3 * j, bounds, r2) : 0;
    }
    return ORC_OK;
}

/* The counters SURVEY.md §8(d) prices the radius query with (B_r = 16 N + 12 P
 * + 16): nodes visited and points scanned by the one-query-at-a-time DFS
 * above, summed over the m queries.  Not thread-safe (file-static counters). */
ORC_EXPORT int orc_ball_count_stats(const orc_tree *t, const float *q, int64_t m, float r,
                                    uint32_t *out_count, uint64_t *nodes, uint64_t *points) {
    g_ball_nodes = 0;
    g_ball_points = 0;
    int rc = orc_ball_count(t, q, m, r, out_count);
    *nodes = g_ball_nodes;
    *points = g_ball_points;
    return rc;
}
