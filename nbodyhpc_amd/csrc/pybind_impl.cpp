// nbodyhpc_amd.kdtree._impl — pybind11 mirror of the reference binding
// kdtree/src/cpp/pybind.cpp:60-216 over the C ABI (include/nbkd.h).
//
// Same class name, constructor / method signatures and defaults
// (KDTree(points, leafsize=64, max_threads=-1, boxsize=None); query(points,
// k=1, workers=1)), same properties (n = padded count, size = node count,
// periodic, boxsize) and the same RuntimeError messages.  Differences, all
// additive: a trailing `device` constructor argument, radius queries
// (query_ball_count / query_ball_csr) and export() for parity tests.
// `max_threads` and `workers` are accepted and ignored: the build and the
// queries run on the GPU (the reference ignores max_threads too,
// kdtree/src/cpp/kdtree.cpp:116).  Queries release the GIL, may be called from
// several Python threads on one tree at once (the library gives each call its
// own scratch), accept any number of rows (host buffers stream through bounded
// device memory) and stop with KeyboardInterrupt on Ctrl-C: the library polls
// PyErr_CheckSignals between batches, as the reference does every 1000 queries
// (kdtree/src/cpp/pybind.cpp:128-133).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <new>
#include <optional>
#include <stdexcept>
#include <string>

#include "../../include/nbkd.h"

namespace py = pybind11;

namespace {

using farray = py::array_t<float, py::array::c_style | py::array::forcecast>;

[[noreturn]] void raise(nbkd_status st) {
    if (st == NBKD_ENOMEM) throw std::bad_alloc();
    throw std::runtime_error(nbkd_last_error());
}

// nbkd_set_interrupt callback: runs on the calling thread between batches of a
// host-buffer query, with the GIL released around it
int check_signals(void *hit) {
    py::gil_scoped_acquire gil;
    if (PyErr_CheckSignals() != 0) { // pybind.cpp:128-133
        *static_cast<bool *>(hit) = true;
        return 1;
    }
    return 0;
}

// one query call: the interrupt check installed for its duration (GIL held
// when constructed and when finish() runs)
struct Interruptible {
    bool hit = false;
    Interruptible() { nbkd_set_interrupt(check_signals, &hit); }
    ~Interruptible() { nbkd_set_interrupt(nullptr, nullptr); }
    void finish(nbkd_status st) {
        if (st == NBKD_EINTR && hit) throw py::error_already_set(); // KeyboardInterrupt
        if (st != NBKD_OK) raise(st);
    }
};

void check(nbkd_status st) {
    if (st != NBKD_OK) raise(st);
}

void check_shape(const farray &points) {
    if (points.ndim() != 2 || points.shape(1) != 3)
        throw std::runtime_error("positions must be a 2D array of shape (N, 3)"); // pybind.cpp:17,97
}

class PyKDTree {
    nbkd_tree *h_ = nullptr;
    bool periodic_ = false;
    float box_ = 0.0f;
    int device_ = 0;
    uint64_t n8_ = 0, nodes_ = 0;

  public:
    PyKDTree(farray points, int leaf_size, int /*max_threads*/, std::optional<float> box_size,
             int device) {
        check_shape(points);
        periodic_ = box_size.has_value();
        box_ = box_size.value_or(0.0f);
        const float *ptr = points.data();
        const uint64_t n = (uint64_t)points.shape(0);
        nbkd_status st;
        {
            py::gil_scoped_release nogil; // pybind.cpp:86
            st = nbkd_build(ptr, n, leaf_size, periodic_ ? 1 : 0, box_, device, 0u, nullptr, &h_);
        }
        check(st);
        int32_t dev = 0;
        check(nbkd_tree_info(h_, &n8_, &nodes_, nullptr, nullptr, &dev));
        device_ = dev;
    }
    PyKDTree(const PyKDTree &) = delete;
    PyKDTree &operator=(const PyKDTree &) = delete;
    ~PyKDTree() {
        if (h_) nbkd_free(h_);
    }

    size_t num_points() const { return (size_t)n8_; }
    size_t num_nodes() const { return (size_t)nodes_; }
    bool periodic() const { return periodic_; }
    float box_size() const { return box_; }
    int device() const { return device_; }

    // pybind.cpp:90-189
    std::pair<py::array_t<float>, py::array_t<uint32_t>> query(farray points, int k, int workers) {
        (void)workers;
        if (k <= 0) throw std::runtime_error("k must be positive integer");
        check_shape(points);
        const py::ssize_t m = points.shape(0);
        py::array_t<float> dist({m, (py::ssize_t)k});
        py::array_t<uint32_t> idx({m, (py::ssize_t)k});
        const float *q = points.data();
        float *d = dist.mutable_data();
        uint32_t *i = idx.mutable_data();
        nbkd_status st;
        Interruptible intr;
        {
            py::gil_scoped_release nogil;
            st = nbkd_query_knn(h_, q, (uint64_t)m, k, d, i, 0u, nullptr);
        }
        intr.finish(st);
        return {dist, idx};
    }

    // distance to the k-th neighbour only (nbkd_query_kth), float32 (m,)
    py::array_t<float> query_kth(farray points, int k) {
        if (k <= 0) throw std::runtime_error("k must be positive integer");
        check_shape(points);
        const py::ssize_t m = points.shape(0);
        py::array_t<float> out(m);
        const float *q = points.data();
        float *o = out.mutable_data();
        nbkd_status st;
        Interruptible intr;
        {
            py::gil_scoped_release nogil;
            st = nbkd_query_kth(h_, q, (uint64_t)m, k, o, 0u, nullptr);
        }
        intr.finish(st);
        return out;
    }

    py::array_t<uint32_t> query_ball_count(farray points, float r) {
        check_shape(points);
        const py::ssize_t m = points.shape(0);
        py::array_t<uint32_t> out(m);
        const float *q = points.data();
        uint32_t *o = out.mutable_data();
        nbkd_status st;
        Interruptible intr;
        {
            py::gil_scoped_release nogil;
            st = nbkd_query_ball_count(h_, q, (uint64_t)m, r, o, 0u, nullptr);
        }
        intr.finish(st);
        return out;
    }

    // rows sorted ascending on the device unless sorted=false (NBKD_SORTED);
    // both passes stream in batches and poll Ctrl-C between them
    std::pair<py::array_t<uint64_t>, py::array_t<uint32_t>> query_ball_csr(farray points, float r,
                                                                           bool sorted) {
        check_shape(points);
        const py::ssize_t m = points.shape(0);
        py::array_t<uint64_t> off(m + 1);
        const float *q = points.data();
        uint64_t *o = off.mutable_data();
        const uint32_t fl = sorted ? NBKD_SORTED : 0u;
        nbkd_status st;
        {
            Interruptible intr;
            {
                py::gil_scoped_release nogil;
                st = nbkd_query_ball_csr(h_, q, (uint64_t)m, r, o, nullptr, 0, fl, nullptr);
            }
            intr.finish(st);
        }
        const uint64_t nnz = o[m];
        py::array_t<uint32_t> idx((py::ssize_t)nnz);
        uint32_t *ip = idx.mutable_data();
        {
            Interruptible intr;
            {
                py::gil_scoped_release nogil;
                st = nbkd_query_ball_csr(h_, q, (uint64_t)m, r, o, ip, nnz, fl, nullptr);
            }
            intr.finish(st);
        }
        return {off, idx};
    }

    // node table (n, 4) as raw 32-bit words + tree-ordered SoA, for parity tests
    py::tuple export_tree() const {
        py::array_t<uint32_t> nodes({(py::ssize_t)nodes_, (py::ssize_t)4});
        py::array_t<float> x((py::ssize_t)n8_), y((py::ssize_t)n8_), z((py::ssize_t)n8_);
        py::array_t<uint32_t> idx((py::ssize_t)n8_);
        check(nbkd_export(h_, reinterpret_cast<nbkd_node *>(nodes.mutable_data()),
                          x.mutable_data(), y.mutable_data(), z.mutable_data(),
                          idx.mutable_data()));
        return py::make_tuple(nodes, x, y, z, idx);
    }
};

} // namespace

PYBIND11_MODULE(_impl, m) {
    m.doc() = "MI355X-native KD-tree for spatial data, including periodic boundary conditions.";

    py::class_<PyKDTree>(m, "KDTree")
        .def(py::init<farray, int, int, std::optional<float>, int>(), py::arg("points"),
             py::arg("leafsize") = 64, py::arg("max_threads") = -1,
             py::arg("boxsize") = std::nullopt, py::arg("device") = -1)
        .def("query", &PyKDTree::query, py::arg("points"), py::arg("k") = 1,
             py::arg("workers") = 1)
        .def("query_kth", &PyKDTree::query_kth, py::arg("points"), py::arg("k"))
        .def("query_ball_count", &PyKDTree::query_ball_count, py::arg("points"), py::arg("r"))
        .def("query_ball_csr", &PyKDTree::query_ball_csr, py::arg("points"), py::arg("r"),
             py::arg("sorted") = true)
        .def("export", &PyKDTree::export_tree)
        .def_property_readonly("n", &PyKDTree::num_points)
        .def_property_readonly("size", &PyKDTree::num_nodes)
        .def_property_readonly("periodic", &PyKDTree::periodic)
        .def_property_readonly("boxsize", &PyKDTree::box_size)
        .def_property_readonly("device", &PyKDTree::device);

    m.def("device_count", []() {
        int32_t c = 0;
        nbkd_device_count(&c);
        return c;
    });
}
