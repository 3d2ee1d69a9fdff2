// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// A C entry point over the reference rasteriser's own periodic vertex
// augmentation, wenda::augment_vertices_periodic
// (rasterization/src/cpp/vertex_utilities.cpp:13-42), compiled from the
// reference sources where they lie under /root/reference by oracle/Makefile
// (target `ref`).  It pins the periodic-image stage of oracle/deposit_oracle.c
// (orc_deposit_images) and so of the GPU deposit (nbkd_deposit), whose grids
// are checked against that oracle.  The shader stage has no CPU counterpart in
// the reference (Vulkan), so it stays parity unpinned.
#include <array>
#include <cstdint>
#include <vector>

#include "vertex_utilities.h"

extern "C" __attribute__((visibility("default"))) int64_t
ref_augment_vertices_periodic(const float *xyz, const float *weight, const float *radius,
                              int64_t n, const float *box, float *out, int64_t capacity) {
    std::vector<wenda::Vertex> v((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        v[i].position[0] = xyz[3 * i];
        v[i].position[1] = xyz[3 * i + 1];
        v[i].position[2] = xyz[3 * i + 2];
        v[i].weight = weight[i];
        v[i].radius = radius[i];
    }
    wenda::augment_vertices_periodic(v, std::array<float, 3>{box[0], box[1], box[2]});
    const int64_t m = (int64_t)v.size();
    for (int64_t j = 0; j < m && j < capacity; ++j) {
        out[5 * j] = v[j].position[0];
        out[5 * j + 1] = v[j].position[1];
        out[5 * j + 2] = v[j].position[2];
        out[5 * j + 3] = v[j].weight;
        out[5 * j + 4] = v[j].radius;
    }
    return m;
}
