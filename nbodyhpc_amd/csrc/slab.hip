// Slab decomposition support for multi-GPU runs: strip
// selection, id remapping, the exactness check of a slab-local kNN result and
// the RCCL point-to-point exchange of halo strips.  The reference has no
// multi-GPU path; these entry points sit beside the single-tree ABI.
//
// RCCL is loaded with dlopen on first use (librccl.so.1 from /opt/rocm/lib),
// so single-GPU users never pay for it and libnbkd.so has no link-time
// dependency on it.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "internal.hpp"

namespace nbkd {
namespace {

constexpr int SEL_TB = 256;
constexpr int SEL_ITEMS = 16; // points per thread per tile
constexpr int SEL_TILE = SEL_TB * SEL_ITEMS;

__device__ __forceinline__ bool in_band(const float *__restrict__ xyz, uint64_t i, float lo,
                                        float hi) {
    const float x = xyz[3 * i];
    return x >= lo && x < hi;
}

__global__ void __launch_bounds__(SEL_TB) band_count_kernel(const float *__restrict__ xyz,
                                                            uint64_t n, float lo, float hi,
                                                            uint32_t *__restrict__ counts) {
    __shared__ uint32_t wsum[SEL_TB / 64];
    const uint64_t base = (uint64_t)blockIdx.x * SEL_TILE;
    uint32_t c = 0;
#pragma unroll 4
    for (int it = 0; it < SEL_ITEMS; ++it) {
        const uint64_t i = base + (uint64_t)it * SEL_TB + threadIdx.x;
        c += (i < n && in_band(xyz, i, lo, hi)) ? 1u : 0u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < SEL_TB / 64; ++w) t += wsum[w];
        counts[blockIdx.x] = t;
    }
}

// stable compaction: output order = input order
__global__ void __launch_bounds__(SEL_TB)
band_scatter_kernel(const float *__restrict__ xyz, const uint32_t *__restrict__ ids, uint64_t n,
                    float lo, float hi, const uint64_t *__restrict__ offsets,
                    float *__restrict__ out_xyz, uint32_t *__restrict__ out_ids) {
    __shared__ uint32_t wsum[SEL_TB / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * SEL_TILE;
    uint64_t run = offsets[blockIdx.x];
    for (int it = 0; it < SEL_ITEMS; ++it) {
        const uint64_t i = base + (uint64_t)it * SEL_TB + threadIdx.x;
        const bool hit = i < n && in_band(xyz, i, lo, hi);
        const uint64_t bal = __ballot(hit);
        const uint32_t below = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wave] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t before = 0, total = 0;
#pragma unroll
        for (int w = 0; w < SEL_TB / 64; ++w) {
            before += w < wave ? wsum[w] : 0u;
            total += wsum[w];
        }
        if (hit) {
            const uint64_t o = run + before + below;
            out_xyz[3 * o] = xyz[3 * i];
            out_xyz[3 * o + 1] = xyz[3 * i + 1];
            out_xyz[3 * o + 2] = xyz[3 * i + 2];
            out_ids[o] = ids ? ids[i] : (uint32_t)i;
        }
        run += total;
        __syncthreads();
    }
}

__global__ void remap_ids_kernel(uint32_t *__restrict__ idx, float4 *__restrict__ p4, uint64_t n8,
                                 uint64_t n, const uint32_t *__restrict__ ids) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n8) return;
    const uint32_t p = idx[j];
    if (p < n) {
        idx[j] = ids[p];
        if (p4) p4[j].w = __uint_as_float(ids[p]); // the packed copy carries the id too
    }
}

// a query's result is exact iff its k-th distance does not reach past the
// x-faces of the local domain [lo - h, hi + h): every point outside is then
// strictly farther than the k-th neighbour found
__global__ void violations_kernel(const float *__restrict__ q, const float *__restrict__ dist,
                                  uint64_t m, int k, float lo, float hi, float h, float slack,
                                  unsigned long long *__restrict__ count) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool bad = false;
    if (i < m) {
        const float x = q[3 * i];
        const float dk = dist[i * (uint64_t)k + (uint64_t)(k - 1)];
        const float margin = fminf(x - (lo - h), (hi + h) - x);
        // the f32 margin may be rounded up by an ulp or two, relative to the margin
        // and to x itself: demand a relative gap plus a few ulps of the domain
        bad = !(dk < margin * (1.0f - 4e-7f) - slack);
    }
    const uint64_t bal = __ballot(bad);
    if ((threadIdx.x & 63) == 0 && bal) atomicAdd(count, (unsigned long long)__popcll(bal));
}

// Second-round forwarding: the queries whose k-th
// distance reaches past the left face cl (bit 0) or the right face ch (bit 1)
// of the x-range the local result covers.  Per side the same f32 test as
// violations_kernel (whose margin is the min of the two sides' gaps).
__global__ void forward_kernel(const float *__restrict__ q, const float *__restrict__ dist,
                               uint64_t m, int k, float cl, float ch, float slack,
                               uint32_t *__restrict__ list, uint8_t *__restrict__ sides,
                               uint64_t cap, unsigned long long *__restrict__ count) {
    const int lane = threadIdx.x & 63;
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < m;
         i0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = i0 + threadIdx.x;
        uint32_t side = 0;
        if (i < m) {
            const float x = q[3 * i];
            const float dk = dist[i * (uint64_t)k + (uint64_t)(k - 1)];
            const float rel = 1.0f - 4e-7f;
            if (!(dk < (x - cl) * rel - slack)) side |= 1u;
            if (!(dk < (ch - x) * rel - slack)) side |= 2u;
        }
        const uint64_t bal = __ballot(side != 0u);
        if (bal == 0) continue;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(count, (unsigned long long)__popcll(bal));
        base = __shfl(base, 0, 64);
        if (side) {
            const uint64_t pos = base + (uint64_t)__popcll(bal & ((1ull << lane) - 1ull));
            if (pos < cap) {
                list[pos] = (uint32_t)i;
                sides[pos] = (uint8_t)side;
            }
        }
    }
}

// rows of `words` 32-bit words: gather dst[i] = src[idx[i]], scatter dst[idx[i]] = src[i]
template <bool SCATTER>
__global__ void rows_kernel(const uint32_t *__restrict__ src, uint32_t words,
                            const uint32_t *__restrict__ idx, uint64_t n, uint32_t *__restrict__ dst) {
    const uint64_t total = n * words;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = t / words, w = t - r * words;
        const uint64_t j = idx[r];
        if (SCATTER)
            dst[j * words + w] = src[t];
        else
            dst[t] = src[j * words + w];
    }
}

// ------------------------------------------------------------------ RCCL (dlopen)
struct Rccl {
    bool tried = false, ok = false;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) =
        nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char *(*ErrorString)(ncclResult_t) = nullptr;
};

std::mutex g_rccl_mu;
Rccl g_rccl;

const Rccl *rccl() {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    Rccl &r = g_rccl;
    if (r.tried) return r.ok ? &r : nullptr;
    r.tried = true;
    // the image's RCCL first, by path: it is built against the HIP runtime this
    // library links (ROCm 7.2).  By soname a process that has imported torch
    // gets torch's bundled librccl, which calls torch's own HIP runtime: that
    // one sees no device once ours owns it, and ncclCommInitRank fails with
    // "no ROCm-capable device is detected" (profiles/r03_rccl_probe_*.log).
    // hip.preload() loads it before torch for the same reason.
    void *h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        const char *e = dlerror();
        r.err = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
        return nullptr;
    }
    bool all = true;
    auto sym = [&](const char *name) {
        void *p = dlsym(h, name);
        all = all && p != nullptr;
        return p;
    };
    r.GetUniqueId = (decltype(r.GetUniqueId))sym("ncclGetUniqueId");
    r.CommInitRank = (decltype(r.CommInitRank))sym("ncclCommInitRank");
    r.CommDestroy = (decltype(r.CommDestroy))sym("ncclCommDestroy");
    r.Send = (decltype(r.Send))sym("ncclSend");
    r.Recv = (decltype(r.Recv))sym("ncclRecv");
    r.GroupStart = (decltype(r.GroupStart))sym("ncclGroupStart");
    r.GroupEnd = (decltype(r.GroupEnd))sym("ncclGroupEnd");
    r.ErrorString = (decltype(r.ErrorString))sym("ncclGetErrorString");
    if (!all) {
        r.err = "librccl.so.1 lacks a required symbol";
        return nullptr;
    }
    r.ok = true;
    return &r;
}

nbkd_status rccl_fail(const Rccl *r, ncclResult_t e, const char *what) {
    set_error(std::string("RCCL error in ") + what + ": " +
              (r && r->ErrorString ? r->ErrorString(e) : "?"));
    return NBKD_EDEVICE;
}

struct DevGuard {
    int prev = -1;
    bool ok = true;
    explicit DevGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DevGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

} // namespace
} // namespace nbkd

struct nbkd_comm {
    ncclComm_t c = nullptr;
    int rank = 0, world = 1, device = 0;
};

using namespace nbkd;

#define SLAB_TRY try {
#define SLAB_CATCH                                                                                 \
    }                                                                                              \
    catch (std::bad_alloc const &) {                                                               \
        set_error("host allocation failed");                                                       \
        return NBKD_ENOMEM;                                                                        \
    }                                                                                              \
    catch (std::exception const &e) {                                                              \
        set_error(e.what());                                                                       \
        return NBKD_EDEVICE;                                                                       \
    }

extern "C" {

nbkd_status nbkd_set_ids(nbkd_tree *tree, const uint32_t *ids, uint32_t flags, void *stream) {
    SLAB_TRY
    if (!tree || (!ids && tree->t.n > 0)) {
        set_error("nbkd_set_ids: NULL argument");
        return NBKD_EINVAL;
    }
    Tree &t = tree->t;
    if (t.n8 == 0) return NBKD_OK;
    DevGuard g(t.device);
    hipStream_t s = (hipStream_t)stream;
    AllWs all(t, s); // no query of this tree runs while its ids change
    const uint32_t *dids = ids;
    DevBuf tmp;
    if (!(flags & NBKD_INPUT_DEVICE)) {
        NBKD_HIP(tmp.alloc(t.n * 4, s));
        NBKD_HIP(hipMemcpyAsync(tmp.p, ids, t.n * 4, hipMemcpyHostToDevice, s));
        NBKD_HIP(hipStreamSynchronize(s));
        dids = tmp.as<uint32_t>();
    }
    // the self-query order (query.hip self_order) keeps the build's permutation
    if (!t.sidx) {
        NBKD_HIP(tree_malloc((void **)&t.sidx, t.n8 * 4));
        NBKD_HIP(hipMemcpyAsync(t.sidx, t.idx, t.n8 * 4, hipMemcpyDeviceToDevice, s));
    }
    const unsigned blocks = (unsigned)((t.n8 + 255) / 256);
    remap_ids_kernel<<<blocks, 256, 0, s>>>(t.idx, t.p4, t.n8, t.n, dids);
    NBKD_HIP(hipGetLastError());
    // every later call on any workspace (any stream) sees the new ids
    NBKD_HIP(hipStreamSynchronize(s));
    return NBKD_OK;
    SLAB_CATCH
}

nbkd_status nbkd_set_kth_out(nbkd_tree *tree, float *kth, uint64_t capacity) {
    SLAB_TRY
    if (!tree) {
        set_error("nbkd_set_kth_out: NULL tree");
        return NBKD_EINVAL;
    }
    Tree &t = tree->t;
    DevGuard g(t.device);
    AllWs all(t, nullptr); // no query of this tree runs while the target changes
    // a kNN already queued on another stream may still write the
    // old array; the host waits for every workspace's last call, so the
    // caller may free the old array once this returns
    auto drain = [](Workspace &w) {
        if (w.used && w.done) (void)hipEventSynchronize(w.done);
    };
    drain(t.ws);
    for (auto &w : t.ws_extra) drain(*w);
    t.kth_side = capacity ? kth : nullptr;
    t.kth_side_cap = kth ? capacity : 0;
    return NBKD_OK;
    SLAB_CATCH
}

nbkd_status nbkd_slab_select(const float *xyz, const uint32_t *ids, uint64_t n, float lo, float hi,
                             float *out_xyz, uint32_t *out_ids, uint64_t capacity,
                             uint64_t *count, int32_t device, void *stream) {
    SLAB_TRY
    if (!count || (n > 0 && !xyz)) {
        set_error("nbkd_slab_select: NULL argument");
        return NBKD_EINVAL;
    }
    *count = 0;
    if (n == 0) return NBKD_OK;
    DevGuard g(device);
    hipStream_t s = (hipStream_t)stream;
    const uint64_t tiles = (n + SEL_TILE - 1) / SEL_TILE;
    if (tiles > 0x7FFFFFFFull) {
        set_error("nbkd_slab_select: too many points");
        return NBKD_EINVAL;
    }
    DevBuf dcounts, doffs;
    NBKD_HIP(dcounts.alloc(tiles * 4, s));
    band_count_kernel<<<(unsigned)tiles, SEL_TB, 0, s>>>(xyz, n, lo, hi, dcounts.as<uint32_t>());
    NBKD_HIP(hipGetLastError());
    std::vector<uint32_t> hc(tiles);
    NBKD_HIP(hipMemcpyAsync(hc.data(), dcounts.p, tiles * 4, hipMemcpyDeviceToHost, s));
    NBKD_HIP(hipStreamSynchronize(s));
    std::vector<uint64_t> ho(tiles);
    uint64_t tot = 0;
    for (uint64_t b = 0; b < tiles; ++b) {
        ho[b] = tot;
        tot += hc[b];
    }
    *count = tot;
    if (!out_xyz || !out_ids) return NBKD_OK; // count only
    if (capacity < tot) {
        set_error("nbkd_slab_select: output capacity too small");
        return NBKD_EINVAL;
    }
    NBKD_HIP(doffs.alloc(tiles * 8, s));
    NBKD_HIP(hipMemcpyAsync(doffs.p, ho.data(), tiles * 8, hipMemcpyHostToDevice, s));
    band_scatter_kernel<<<(unsigned)tiles, SEL_TB, 0, s>>>(xyz, ids, n, lo, hi,
                                                          doffs.as<uint64_t>(), out_xyz, out_ids);
    NBKD_HIP(hipGetLastError());
    NBKD_HIP(hipStreamSynchronize(s));
    return NBKD_OK;
    SLAB_CATCH
}

nbkd_status nbkd_slab_violations(const float *q, const float *dist, uint64_t m, int32_t k,
                                 float lo, float hi, float h, uint64_t *count, int32_t device,
                                 void *stream) {
    SLAB_TRY
    if (!count || k <= 0 || (m > 0 && (!q || !dist))) {
        set_error("nbkd_slab_violations: bad argument");
        return NBKD_EINVAL;
    }
    *count = 0;
    if (m == 0) return NBKD_OK;
    DevGuard g(device);
    hipStream_t s = (hipStream_t)stream;
    DevBuf dc;
    NBKD_HIP(dc.alloc(8, s));
    NBKD_HIP(hipMemsetAsync(dc.p, 0, 8, s));
    // absolute slack: 4 ulps of the largest |x| of the local domain, so a k-th
    // distance within an ulp of the face is flagged even when h << the box
    const float mag = std::fmax(std::fabs(lo - h), std::fabs(hi + h));
    const float slack = 4.0f * (std::nextafter(mag, INFINITY) - mag);
    violations_kernel<<<(unsigned)((m + 255) / 256), 256, 0, s>>>(
        q, dist, m, k, lo, hi, h, slack, dc.as<unsigned long long>());
    NBKD_HIP(hipGetLastError());
    NBKD_HIP(hipMemcpyAsync(count, dc.p, 8, hipMemcpyDeviceToHost, s));
    NBKD_HIP(hipStreamSynchronize(s));
    return NBKD_OK;
    SLAB_CATCH
}

nbkd_status nbkd_slab_forward(const float *q, const float *dist, uint64_t m, int32_t k, float cl,
                              float ch, uint32_t *out_list, uint8_t *out_sides, uint64_t capacity,
                              uint64_t *count, int32_t device, void *stream) {
    SLAB_TRY
    if (!count || k <= 0 || (m > 0 && (!q || !dist)) || (capacity > 0 && (!out_list || !out_sides))) {
        set_error("nbkd_slab_forward: bad argument");
        return NBKD_EINVAL;
    }
    *count = 0;
    if (m == 0) return NBKD_OK;
    DevGuard g(device);
    hipStream_t s = (hipStream_t)stream;
    DevBuf dc;
    NBKD_HIP(dc.alloc(8, s));
    NBKD_HIP(hipMemsetAsync(dc.p, 0, 8, s));
    const float mag = std::fmax(std::fabs(cl), std::fabs(ch));
    const float slack = 4.0f * (std::nextafter(mag, INFINITY) - mag);
    const unsigned blocks = (unsigned)std::min<uint64_t>((m + 255) / 256, 65536);
    forward_kernel<<<blocks, 256, 0, s>>>(q, dist, m, k, cl, ch, slack, out_list, out_sides,
                                          capacity, dc.as<unsigned long long>());
    NBKD_HIP(hipGetLastError());
    NBKD_HIP(hipMemcpyAsync(count, dc.p, 8, hipMemcpyDeviceToHost, s));
    NBKD_HIP(hipStreamSynchronize(s));
    return NBKD_OK;
    SLAB_CATCH
}

nbkd_status nbkd_slab_forward_async(const float *q, const float *dist, uint64_t m, int32_t k,
                                    float cl, float ch, uint32_t *out_list, uint8_t *out_sides,
                                    uint64_t capacity, uint64_t *count, int32_t device,
                                    void *stream) {
    SLAB_TRY
    if (!count || k <= 0 || (m > 0 && (!q || !dist)) || (capacity > 0 && (!out_list || !out_sides))) {
        set_error("nbkd_slab_forward_async: bad argument");
        return NBKD_EINVAL;
    }
    DevGuard g(device);
    hipStream_t s = (hipStream_t)stream;
    // the count lives in device memory the caller owns: no allocation, no
    // wait (nbkd_slab_forward's scratch word costs a hipFree, a device sync)
    NBKD_HIP(hipMemsetAsync(count, 0, 8, s));
    if (m == 0) return NBKD_OK;
    const float mag = std::fmax(std::fabs(cl), std::fabs(ch));
    const float slack = 4.0f * (std::nextafter(mag, INFINITY) - mag);
    const unsigned blocks = (unsigned)std::min<uint64_t>((m + 255) / 256, 65536);
    forward_kernel<<<blocks, 256, 0, s>>>(q, dist, m, k, cl, ch, slack, out_list, out_sides,
                                          capacity, (unsigned long long *)count);
    NBKD_HIP(hipGetLastError());
    return NBKD_OK;
    SLAB_CATCH
}

static nbkd_status rows_common(const void *src, uint64_t row_bytes, const uint32_t *idx, uint64_t n,
                               void *dst, int32_t device, void *stream, bool scatter) {
    if (row_bytes == 0 || row_bytes % 4 != 0 || (n > 0 && (!src || !idx || !dst))) {
        set_error("nbkd_rows_gather / nbkd_rows_scatter: bad argument");
        return NBKD_EINVAL;
    }
    if (n == 0) return NBKD_OK;
    DevGuard g(device);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t words = (uint32_t)(row_bytes / 4);
    const unsigned blocks = (unsigned)std::min<uint64_t>((n * words + 255) / 256, 65536);
    if (scatter)
        rows_kernel<true><<<blocks, 256, 0, s>>>((const uint32_t *)src, words, idx, n, (uint32_t *)dst);
    else
        rows_kernel<false><<<blocks, 256, 0, s>>>((const uint32_t *)src, words, idx, n, (uint32_t *)dst);
    NBKD_HIP(hipGetLastError());
    return NBKD_OK;
}

nbkd_status nbkd_rows_gather(const void *src, uint64_t row_bytes, const uint32_t *idx, uint64_t n,
                             void *dst, int32_t device, void *stream) {
    SLAB_TRY
    return rows_common(src, row_bytes, idx, n, dst, device, stream, false);
    SLAB_CATCH
}

nbkd_status nbkd_rows_scatter(const void *src, uint64_t row_bytes, const uint32_t *idx, uint64_t n,
                              void *dst, int32_t device, void *stream) {
    SLAB_TRY
    return rows_common(src, row_bytes, idx, n, dst, device, stream, true);
    SLAB_CATCH
}

nbkd_status nbkd_comm_probe(void) {
    if (!rccl()) {
        set_error(g_rccl.err);
        return NBKD_EDEVICE;
    }
    return NBKD_OK;
}

nbkd_status nbkd_comm_unique_id(uint8_t *out) {
    if (!out) return NBKD_EINVAL;
    const Rccl *r = rccl();
    if (!r) {
        set_error(g_rccl.err);
        return NBKD_EDEVICE;
    }
    ncclUniqueId id;
    ncclResult_t e = r->GetUniqueId(&id);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclGetUniqueId");
    std::memcpy(out, id.internal, NBKD_COMM_ID_BYTES);
    return NBKD_OK;
}

nbkd_status nbkd_comm_init(const uint8_t *id, int32_t rank, int32_t world, int32_t device,
                           nbkd_comm **out) {
    SLAB_TRY
    if (!id || !out || world < 1 || rank < 0 || rank >= world) {
        set_error("nbkd_comm_init: bad argument");
        return NBKD_EINVAL;
    }
    *out = nullptr;
    const Rccl *r = rccl();
    if (!r) {
        set_error(g_rccl.err);
        return NBKD_EDEVICE;
    }
    DevGuard g(device);
    if (!g.ok) {
        set_error("hipSetDevice failed");
        return NBKD_EDEVICE;
    }
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, NBKD_COMM_ID_BYTES);
    auto *c = new nbkd_comm();
    c->rank = rank;
    c->world = world;
    c->device = device;
    ncclResult_t e = r->CommInitRank(&c->c, world, uid, rank);
    if (e != ncclSuccess) {
        delete c;
        return rccl_fail(r, e, "ncclCommInitRank");
    }
    *out = c;
    return NBKD_OK;
    SLAB_CATCH
}

nbkd_status nbkd_comm_exchange(nbkd_comm *c, int32_t npairs, const void *const *send,
                               const uint64_t *send_bytes, const int32_t *send_peer,
                               void *const *recv, const uint64_t *recv_bytes,
                               const int32_t *recv_peer, void *stream) {
    if (!c || npairs < 0 || (npairs > 0 && (!send || !send_bytes || !send_peer || !recv ||
                                            !recv_bytes || !recv_peer))) {
        set_error("nbkd_comm_exchange: bad argument");
        return NBKD_EINVAL;
    }
    const Rccl *r = rccl();
    if (!r) {
        set_error(g_rccl.err);
        return NBKD_EDEVICE;
    }
    DevGuard g(c->device);
    hipStream_t s = (hipStream_t)stream;
    ncclResult_t e = r->GroupStart();
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclGroupStart");
    // messages to / from one peer are matched in posting order
    for (int i = 0; i < npairs; ++i) {
        if (send_bytes[i] > 0) {
            e = r->Send(send[i], send_bytes[i], ncclUint8, send_peer[i], c->c, s);
            if (e != ncclSuccess) {
                (void)r->GroupEnd();
                return rccl_fail(r, e, "ncclSend");
            }
        }
        if (recv_bytes[i] > 0) {
            e = r->Recv(recv[i], recv_bytes[i], ncclUint8, recv_peer[i], c->c, s);
            if (e != ncclSuccess) {
                (void)r->GroupEnd();
                return rccl_fail(r, e, "ncclRecv");
            }
        }
    }
    e = r->GroupEnd();
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclGroupEnd");
    return NBKD_OK;
}

void nbkd_comm_free(nbkd_comm *c) {
    if (!c) return;
    const Rccl *r = rccl();
    if (r && c->c) {
        DevGuard g(c->device);
        (void)r->CommDestroy(c->c);
    }
    delete c;
}

} // extern "C"
