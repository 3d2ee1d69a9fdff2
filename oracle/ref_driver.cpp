// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/kdtree_oracle.c header).
//
// A thin extern "C" driver over the REFERENCE's own sources, compiled where
// they lie under /root/reference by oracle/Makefile into oracle/_ref/.  No
// reference source is copied into this repository; nothing here replaces a
// reference component.  What the driver does:
//
//   * ref_build: the pybind PyKDTree constructor path (kdtree/src/cpp/pybind.cpp:14-56,76-88)
//     — AoS -> padded SoA with iota indices and the periodic range check —
//     then the reference KDTree constructor itself (kdtree/src/cpp/kdtree.cpp:95-131,
//     FloydRivestAvxSelectionPolicy), compiled from kdtree.cpp + kdtree_selection.cpp.
//   * ref_knn: KDTree::find_closest's body (kdtree/src/cpp/kdtree.cpp:133-159) with the
//     reference's own InsertShorterDistanceAVX leaf inserter
//     (kdtree/src/cpp/include/kdtree/kdtree_opt.hpp) instead of the NASM one:
//     the .asm file needs `nasm`, absent from this image, so the asm TU is
//     unbuildable here.  The reference's test_inserters.cpp / test_asm.cpp pin
//     the AVX and asm inserters to the same results.  The asm-bound
//     find_closest instantiations of kdtree.cpp are never referenced and are
//     discarded by the linker (--gc-sections, hidden visibility).
//   * the batch loop runs on the reference's own thread pool
//     (kdtree/third_party/misc/thread_pool.hpp:148-183) exactly as pybind.cpp:164-172.
#include <kdtree/kdtree.hpp>
#include <kdtree/kdtree_impl.hpp>
#include <kdtree/kdtree_opt.hpp>
#include <kdtree/tournament_tree.hpp>
#include <thread_pool.hpp>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <numeric>
#include <optional>
#include <stdexcept>

#define REF_EXPORT extern "C" __attribute__((visibility("default")))

using wenda::kdtree::KDTree;
using wenda::kdtree::PositionAndIndexArray;

namespace {

struct RefTree {
    KDTree tree;
    bool periodic;
    float box;
};

PositionAndIndexArray<3, float, uint32_t> make_positions(const float *aos, int64_t n,
                                                         std::optional<float> box) {
    const int block_size = 8;
    int64_t size_up = (n + block_size - 1) / block_size * block_size;
    PositionAndIndexArray<3, float, uint32_t> pos(size_up);
    std::iota(pos.indices_.begin(), pos.indices_.end(), 0);
    for (size_t dim = 0; dim < 3; ++dim) {
        for (int64_t i = 0; i < n; ++i) pos.positions_[dim][i] = aos[3 * i + dim];
        if (box) {
            float L = *box;
            bool ok = std::all_of(pos.positions_[dim], pos.positions_[dim] + n,
                                  [&](float x) { return x >= 0.0f && x <= L; });
            if (!ok) throw std::runtime_error("box");
        }
        std::fill(pos.positions_[dim] + n, pos.positions_[dim] + size_up,
                  std::numeric_limits<float>::max());
    }
    return pos;
}

template <typename Dist>
void find_closest_avx(const KDTree &tree, const std::array<float, 3> &q, size_t k,
                      const Dist &dist, float *out_d, uint32_t *out_i, bool want_sqrt,
                      wenda::kdtree::KDTreeQueryStatistics *st) {
    typedef std::pair<float, uint32_t> result_t;
    wenda::kdtree::detail::KDTreeQuery<
        Dist, wenda::kdtree::TournamentTree<result_t, wenda::kdtree::PairLessFirst>,
        wenda::kdtree::InsertShorterDistanceAVX>
        query(tree.nodes(), tree.positions(), dist, q, k);
    query.compute(&tree.nodes()[0]);
    if (st) {
        st->nodes_visited = query.num_nodes_visited;
        st->nodes_pruned = query.num_nodes_pruned;
        st->points_visited = query.num_points_visited;
    }
    std::vector<result_t> result(k);
    query.distances_.copy_values(result.begin());
    std::sort(result.begin(), result.end(), wenda::kdtree::PairLessFirst{});
    for (size_t j = 0; j < k; ++j) {
        out_d[j] = want_sqrt ? dist.postprocess(result[j].first) : result[j].first;
        out_i[j] = result[j].second;
    }
}

} // namespace

// status: 0 ok, 2 box violation, 3 too many points, 5 other
REF_EXPORT int ref_build(const float *aos, int64_t n, int32_t leafsize, int32_t periodic,
                         float box, void **out) {
    *out = nullptr;
    try {
        std::optional<float> b;
        if (periodic) b = box;
        auto pos = make_positions(aos, n, b);
        auto *t = new RefTree{KDTree(std::move(pos), {.leaf_size = leafsize, .max_threads = -1,
                                                      .block_size = 8}),
                              periodic != 0, periodic ? box : 0.0f};
        *out = t;
        return 0;
    } catch (std::runtime_error const &e) {
        if (std::strcmp(e.what(), "box") == 0) return 2;
        if (std::strstr(e.what(), "uint32_t")) return 3;
        return 5;
    } catch (...) {
        return 5;
    }
}

REF_EXPORT void ref_free(void *t) { delete static_cast<RefTree *>(t); }

REF_EXPORT int64_t ref_n8(void *t) {
    return (int64_t) static_cast<RefTree *>(t)->tree.positions().size();
}

REF_EXPORT int64_t ref_num_nodes(void *t) {
    return (int64_t) static_cast<RefTree *>(t)->tree.nodes().size();
}

REF_EXPORT void ref_export(void *tp, void *nodes, float *x, float *y, float *z, uint32_t *idx) {
    auto *t = static_cast<RefTree *>(tp);
    auto nd = t->tree.nodes();
    static_assert(sizeof(KDTree::KDTreeNode) == 16, "node layout");
    if (nodes) std::memcpy(nodes, nd.data(), nd.size() * sizeof(KDTree::KDTreeNode));
    auto const &p = t->tree.positions();
    size_t n = p.size();
    if (x) std::memcpy(x, p.positions_[0], n * sizeof(float));
    if (y) std::memcpy(y, p.positions_[1], n * sizeof(float));
    if (z) std::memcpy(z, p.positions_[2], n * sizeof(float));
    if (idx) std::memcpy(idx, p.indices_.data(), n * sizeof(uint32_t));
}

// PyKDTree::query (pybind.cpp:90-172) minus the Python plumbing.
// stats (optional, 3 x uint64): sums of nodes_visited, nodes_pruned, points_visited.
REF_EXPORT int ref_knn(void *tp, const float *q, int64_t m, int32_t k, int32_t workers,
                       int32_t want_sqrt, float *out_d, uint32_t *out_i, uint64_t *stats) {
    if (k <= 0) return 1;
    auto *t = static_cast<RefTree *>(tp);
    std::atomic<uint64_t> sv{0}, sp{0}, spts{0};
    auto run = [&](auto const &dist) {
        auto loop_fn = [&](size_t start, size_t end) {
            uint64_t a = 0, b = 0, c = 0;
            for (size_t i = start; i < end; ++i) {
                wenda::kdtree::KDTreeQueryStatistics st{};
                find_closest_avx(t->tree, {q[3 * i], q[3 * i + 1], q[3 * i + 2]}, (size_t)k, dist,
                                 out_d + i * k, out_i + i * k, want_sqrt != 0,
                                 stats ? &st : nullptr);
                a += st.nodes_visited;
                b += st.nodes_pruned;
                c += st.points_visited;
            }
            sv += a;
            sp += b;
            spts += c;
        };
        if (workers == 1) {
            loop_fn(0, (size_t)m);
        } else {
            wenda::thread_pool pool(workers > 0 ? workers : std::thread::hardware_concurrency());
            pool.parallelize_loop((size_t)0, (size_t)m, loop_fn);
        }
    };
    if (t->periodic)
        run(wenda::kdtree::L2PeriodicDistance<float>{t->box});
    else
        run(wenda::kdtree::L2Distance{});
    if (stats) {
        stats[0] += sv;
        stats[1] += sp;
        stats[2] += spts;
    }
    return 0;
}
