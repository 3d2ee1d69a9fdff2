// Probe of CU-masked streams on MI355X (hipExtStreamCreateWithCUMask): which
// hardware XCD / SE / CU each mask bit selects, and the HBM read bandwidth a
// streaming kernel reaches on a masked subset of CUs.  Measurement tooling
// for the collect / select overlap, not product code.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/calib/cumask_probe scripts/calib/cumask_probe.hip
//   ./scripts/calib/cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <tuple>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

// s_getreg: HW_ID (hwreg 4) and XCC_ID (hwreg 20, gfx940+)
__global__ void where_kernel(uint32_t *out) {
    if (threadIdx.x == 0) {
        const uint32_t hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
        const uint32_t xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
}

__global__ void stream_kernel(const float4 *__restrict__ a, size_t n, float *__restrict__ sink) {
    float acc = 0.0f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.678f) sink[0] = acc; // keeps the loads
}

static void placement(const char *name, const std::vector<uint32_t> &mask) {
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    const int blocks = 4096;
    uint32_t *d;
    CK(hipMalloc(&d, blocks * 8));
    where_kernel<<<blocks, 64, 0, s>>>(d);
    CK(hipStreamSynchronize(s));
    std::vector<uint32_t> h(blocks * 2);
    CK(hipMemcpy(h.data(), d, blocks * 8, hipMemcpyDeviceToHost));
    std::set<std::tuple<uint32_t, uint32_t, uint32_t>> cus; // (xcc, se, cu)
    std::vector<int> per_xcc(16, 0);
    for (int b = 0; b < blocks; ++b) {
        const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 0xF;
        const uint32_t cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
        cus.insert({xcc, se * 2 + sh, cu});
        per_xcc[xcc]++;
    }
    std::printf("%s: %zu distinct (xcc, se/sh, cu); blocks per xcc:", name, cus.size());
    for (int x = 0; x < 8; ++x) std::printf(" %d", per_xcc[x]);
    std::printf("\n   cus:");
    int shown = 0;
    for (auto &c : cus) {
        if (shown++ < 40) std::printf(" %u/%u/%u", std::get<0>(c), std::get<1>(c), std::get<2>(c));
    }
    std::printf("\n");
    CK(hipFree(d));
    CK(hipStreamDestroy(s));
}

static void bandwidth(const char *name, const std::vector<uint32_t> &mask, const float4 *a,
                      size_t n, float *sink) {
    hipStream_t s;
    if (mask.empty())
        CK(hipStreamCreate(&s));
    else
        CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    stream_kernel<<<8192, 256, 0, s>>>(a, n, sink);
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < 5; ++r) stream_kernel<<<8192, 256, 0, s>>>(a, n, sink);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("%s: %.1f GB/s\n", name, 5.0 * n * 16 / (ms * 1e-3) / 1e9);
    CK(hipStreamDestroy(s));
}

int main() {
    int dev = 0, cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    std::printf("CUs: %d\n", cus);
    const int words = (cus + 31) / 32;
    auto mk = [&](auto pred) {
        std::vector<uint32_t> m(words, 0u);
        for (int i = 0; i < cus; ++i)
            if (pred(i)) m[i / 32] |= 1u << (i % 32);
        return m;
    };
    placement("bits 0..31", mk([](int i) { return i < 32; }));
    placement("bits 0..7", mk([](int i) { return i < 8; }));
    placement("every 8th bit", mk([](int i) { return i % 8 == 0; }));
    placement("bits i%32<4", mk([](int i) { return i % 32 < 4; }));
    placement("all", mk([](int) { return true; }));

    const size_t n = (4ull << 30) / 16;
    float4 *a;
    float *sink;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(a, 0, n * 16));
    bandwidth("all CUs (plain stream)", {}, a, n, sink);
    bandwidth("bits 0..31", mk([](int i) { return i < 32; }), a, n, sink);
    bandwidth("bits 0..63", mk([](int i) { return i < 64; }), a, n, sink);
    bandwidth("every 8th bit (32)", mk([](int i) { return i % 8 == 0; }), a, n, sink);
    bandwidth("every 4th bit (64)", mk([](int i) { return i % 4 == 0; }), a, n, sink);
    bandwidth("i%32<4 (32)", mk([](int i) { return i % 32 < 4; }), a, n, sink);
    bandwidth("all but every 8th (224)", mk([](int i) { return i % 8 != 0; }), a, n, sink);
    CK(hipFree(a));
    CK(hipFree(sink));
    return 0;
}
