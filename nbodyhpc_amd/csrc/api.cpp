// C ABI of libnbkd.so (include/nbkd.h).  Host code only; kernels live in
// build.hip / query.hip.  No exception crosses the boundary.
#include <hip/hip_runtime.h>

#include <sched.h>

#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "internal.hpp"

namespace nbkd {

namespace {
thread_local std::string g_err;
thread_local uint64_t g_stats[NBKD_NSTATS] = {};

std::mutex g_tmu;
bool g_timing = false;
bool g_stats_on = false;
struct TimedLaunch {
    const char *name; // a string literal (TimedScope's)
    hipEvent_t a, b;
    int dev;
};
std::vector<TimedLaunch> g_pending;
// harvested events go back to a per-device pool: creating two events per
// timed scope cost ~0.4 ms per step of an N = 8 slab (the re-walk rounds'
// ~40 launches; profiles/r05ak_timing_overhead.txt)
std::map<int, std::vector<hipEvent_t>> g_free_events;
hipEvent_t take_event(int dev) {
    {
        std::lock_guard<std::mutex> lk(g_tmu);
        auto &v = g_free_events[dev];
        if (!v.empty()) {
            hipEvent_t e = v.back();
            v.pop_back();
            return e;
        }
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return e;
}
// g_tmu held
void give_events(const TimedLaunch &p) {
    auto &v = g_free_events[p.dev];
    v.push_back(p.a);
    v.push_back(p.b);
}
std::map<std::string, std::pair<double, uint64_t>> g_acc;

struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

} // namespace

uint64_t axes_for_extent(const float e[3]) {
    double x[3] = {e[0], e[1], e[2]};
    uint64_t a = 0;
    for (int d = 0; d < 32; ++d) {
        int k = 0;
        if (x[1] > x[k]) k = 1;
        if (x[2] > x[k]) k = 2;
        a |= (uint64_t)k << (2 * d);
        x[k] *= 0.5;
    }
    return a;
}

namespace {

void free_tree(Tree &t) {
    // no kernel of this tree may still run when its blocks are reused
    if (t.x || t.nodes) (void)hipDeviceSynchronize();
    tree_free(t.x);
    tree_free(t.y);
    tree_free(t.z);
    tree_free(t.idx);
    tree_free(t.sidx);
    t.sidx = nullptr;
    t.src = nullptr;
    tree_free(t.p4);
    t.p4 = nullptr;
    tree_free(t.nodes);
    tree_free(t.splits);
    tree_free(t.shape_c);
    tree_free(t.shape_n);
    tree_free(t.leafinfo);
    tree_free(t.hsplit);
    tree_free(t.ginfo);
    tree_free(t.hinfo);
    tree_free(t.nbox);
    t.nbox = nullptr;
    t.ginfo = t.hinfo = nullptr;
    t.leafinfo = nullptr;
    t.hsplit = nullptr;
    t.splits = nullptr;
    t.shape_c = t.shape_n = nullptr;
    t.x = t.y = t.z = nullptr;
    t.idx = nullptr;
    t.nodes = nullptr;
    t.ws.release();
    for (auto &w : t.ws_extra) w->release();
    t.ws_extra.clear();
}
} // namespace

namespace {
struct BlockCache {
    std::mutex mu;
    std::map<void *, std::pair<int, size_t>> live;             // block -> (device, bytes)
    std::multimap<std::pair<int, size_t>, void *> idle;         // (device, bytes) -> block
    size_t idle_bytes = 0;
    static constexpr size_t CAP = 64ull << 30;                  // idle bytes kept, all devices
};
BlockCache &block_cache() {
    static BlockCache c;
    return c;
}
} // namespace

void release_idle_blocks(int dev) {
    BlockCache &c = block_cache();
    std::lock_guard<std::mutex> g(c.mu);
    for (auto it = c.idle.begin(); it != c.idle.end();) {
        if (it->first.first == dev) {
            (void)hipFree(it->second);
            c.idle_bytes -= it->first.second;
            it = c.idle.erase(it);
        } else {
            ++it;
        }
    }
}

namespace {
thread_local std::vector<const void *> t_held;
struct WsList {
    std::mutex mu;
    std::vector<Workspace *> all;
};
WsList &ws_list() {
    static WsList *l = new WsList(); // never destroyed: workspaces outlive statics
    return *l;
}
} // namespace

void hold_mark(const void *p) { t_held.push_back(p); }
void hold_unmark(const void *p) {
    for (size_t i = t_held.size(); i-- > 0;)
        if (t_held[i] == p) {
            t_held.erase(t_held.begin() + (std::ptrdiff_t)i);
            return;
        }
}
bool held_here(const void *p) {
    for (const void *h : t_held)
        if (h == p) return true;
    return false;
}

Workspace::Workspace() {
    WsList &l = ws_list();
    std::lock_guard<std::mutex> g(l.mu);
    l.all.push_back(this);
}

Workspace::~Workspace() {
    WsList &l = ws_list();
    std::lock_guard<std::mutex> g(l.mu);
    for (size_t i = 0; i < l.all.size(); ++i)
        if (l.all[i] == this) {
            l.all[i] = l.all.back();
            l.all.pop_back();
            break;
        }
}

// the idle workspaces of `dev` (no call holds them) give their slots back;
// try_lock only, so a call in flight on another thread is never waited for
static void trim_idle_workspaces(int dev) {
    WsList &l = ws_list();
    std::lock_guard<std::mutex> g(l.mu);
    for (Workspace *w : l.all) {
        if (w->dev != dev || held_here(w) || !w->mu.try_lock()) continue;
        w->trim();
        w->mu.unlock();
    }
}

hipError_t malloc_or_release(void **p, size_t bytes) {
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipErrorOutOfMemory) return e;
    // what the device holds idle goes back to the driver, then one retry
    (void)hipGetLastError();
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return e;
    release_idle_blocks(dev);
    release_idle_build_scratch(dev);
    trim_idle_workspaces(dev);
    return hipMalloc(p, bytes);
}

hipError_t tree_malloc(void **p, size_t bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    bytes = bytes ? bytes : 16;
    BlockCache &c = block_cache();
    {
        std::lock_guard<std::mutex> g(c.mu);
        auto it = c.idle.find({dev, bytes});
        if (it != c.idle.end()) {
            *p = it->second;
            c.idle.erase(it);
            c.idle_bytes -= bytes;
            c.live[*p] = {dev, bytes};
            return hipSuccess;
        }
    }
    e = malloc_or_release(p, bytes);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> g(c.mu);
    c.live[*p] = {dev, bytes};
    return hipSuccess;
}

void tree_free(void *p) {
    if (!p) return;
    BlockCache &c = block_cache();
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.live.find(p);
    if (it == c.live.end()) {
        (void)hipFree(p);
        return;
    }
    const auto key = it->second;
    c.live.erase(it);
    if (c.idle_bytes + key.second <= BlockCache::CAP) {
        c.idle.insert({key, p});
        c.idle_bytes += key.second;
    } else {
        (void)hipFree(p);
    }
}


namespace {
// nbkd_set_tuning knobs (process-wide); defaults are the measured optima
std::atomic<double> g_tune[TUNE_N] = {{3.0}, {0.0}, {0.0}, {0.0}, {1.0}, {0.0}};
const char *const g_tune_names[TUNE_N] = {"knn_seed_margin", "candidate_bytes", "host_batch",
                                          "host_threads", "self_order", "pinned_bytes"};
thread_local nbkd_interrupt_fn t_intr = nullptr;
thread_local void *t_intr_user = nullptr;
} // namespace

double tuning(int id) { return g_tune[id].load(std::memory_order_relaxed); }

bool interrupted() { return t_intr != nullptr && t_intr(t_intr_user) != 0; }

Workspace &acquire_ws(const Tree &t) {
    if (t.ws.mu.try_lock()) return t.ws;
    {
        std::lock_guard<std::mutex> g(t.ws_mu);
        for (auto &w : t.ws_extra)
            if (w->mu.try_lock()) return *w;
        if ((int)t.ws_extra.size() < NBKD_MAX_WS - 1) {
            t.ws_extra.emplace_back(new Workspace());
            Workspace &w = *t.ws_extra.back();
            w.mu.lock();
            return w;
        }
    }
    t.ws.mu.lock();
    return t.ws;
}

AllWs::AllWs(const Tree &t_, hipStream_t s) : t(t_), pool(t_.ws_mu) {
    locks.emplace_back(t.ws.mu);
    for (auto &w : t.ws_extra) locks.emplace_back(w->mu);
    // held by this thread: an out-of-memory retry under this lock (malloc_or_release
    // -> trim_idle_workspaces) must not try_lock them
    hold_mark(&t.ws);
    for (auto &w : t.ws_extra) hold_mark(w.get());
    // the stream waits for every workspace's last call
    auto wait = [&](Workspace &w) {
        if (w.used && w.done) (void)hipStreamWaitEvent(s, w.done, 0);
    };
    wait(t.ws);
    for (auto &w : t.ws_extra) wait(*w);
}

AllWs::~AllWs() {
    for (auto &w : t.ws_extra) hold_unmark(w.get());
    hold_unmark(&t.ws);
}

// ------------------------------------------------------------ host copy threads
// The host-buffer pipeline moves every batch between the caller's (pageable)
// arrays and pinned staging: a ~1 GiB batch of k = 32 rows is one memcpy per
// output, and its first touch of fresh numpy pages faults them in.  With one
// copy thread the whole 1e8-query host call ran at 4.6e7 queries/s (12 GB/s of
// rows), with 4 at 1.53e8 and with 16 at 1.56e8 (40 GB/s, the DMA's rate:
// profiles/r05c_probes.txt), so the copy is split into 8 MiB chunks over the
// usable cores (the affinity mask capped by the cgroup quota, at most 16;
// nbkd_set_tuning("host_threads")).
namespace {
int usable_cpus() {
    int n = 1;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
    if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        double period = 0.0;
        if (std::fscanf(f, "%31s %lf", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0)
            n = std::min(n, std::max(1, (int)std::ceil(std::atof(q) / period)));
        std::fclose(f);
    }
    return std::max(n, 1);
}

struct CopyPool {
    std::mutex job_mu; // one job at a time
    std::mutex mu;
    std::condition_variable cv, done_cv;
    int nthreads = 0;
    char *dst = nullptr;
    const char *src = nullptr;
    size_t bytes = 0;
    std::atomic<size_t> next{0};
    int busy = 0;
    uint64_t gen = 0;
    static constexpr size_t CHUNK = 8u << 20;

    void work() {
        for (size_t i; (i = next.fetch_add(1)) * CHUNK < bytes;) {
            const size_t o = i * CHUNK;
            std::memcpy(dst + o, src + o, std::min(CHUNK, bytes - o));
        }
    }
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return gen != seen; });
            seen = gen;
            lk.unlock();
            work();
            lk.lock();
            if (--busy == 0) done_cv.notify_all();
        }
    }
    // workers are created on first use and never joined (detached, the pool
    // is never destroyed): a process may exit with them waiting
    void grow(int want) {
        while (nthreads < want) {
            std::thread(&CopyPool::loop, this).detach();
            ++nthreads;
        }
    }
    void run(void *d, const void *s, size_t n, int workers) {
        std::lock_guard<std::mutex> job(job_mu);
        {
            std::lock_guard<std::mutex> lk(mu);
            grow(workers - 1);
            dst = (char *)d;
            src = (const char *)s;
            bytes = n;
            next.store(0);
            busy = nthreads;
            ++gen;
        }
        cv.notify_all();
        work(); // the calling thread takes chunks too
        std::unique_lock<std::mutex> lk(mu);
        done_cv.wait(lk, [&] { return busy == 0; });
    }
};
CopyPool &copy_pool() {
    static CopyPool *p = new CopyPool(); // never destroyed (see grow)
    return *p;
}
} // namespace

void host_copy(void *dst, const void *src, size_t bytes) {
    if (bytes == 0) return;
    static const int cpus = usable_cpus();
    const double tw = tuning(TUNE_HOST_THREADS);
    const int workers = tw >= 1.0 ? (int)std::min(tw, 256.0) : std::min(cpus, 16);
    if (workers <= 1 || bytes < (16u << 20)) {
        std::memcpy(dst, src, bytes);
        return;
    }
    copy_pool().run(dst, src, bytes, workers);
}

void set_error(const std::string &msg) { g_err = msg; }

nbkd_status hip_fail(hipError_t e, const char *what) {
    g_err = std::string("HIP error ") + hipGetErrorName(e) + " (" + hipGetErrorString(e) +
            ") in " + what;
    (void)hipGetLastError();
    return e == hipErrorOutOfMemory ? NBKD_ENOMEM : NBKD_EDEVICE;
}

bool timing_enabled() { return g_timing; }
bool stats_enabled() { return g_stats_on; }
void stats_reset() {
    for (int i = 0; i < NBKD_NSTATS; ++i) g_stats[i] = 0;
}
void stats_add(const uint64_t *v) {
    for (int i = 0; i < NBKD_NSTATS; ++i) g_stats[i] += v[i];
}

TimedScope::TimedScope(const char *name, hipStream_t s, bool on) : name_(name), s_(s) {
    if (!g_timing || !on) return;
    if (hipGetDevice(&dev_) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    a_ = take_event(dev_);
    if (a_) (void)hipEventRecord(a_, s_);
}

TimedScope::~TimedScope() {
    if (!a_) return;
    hipEvent_t b = take_event(dev_);
    std::lock_guard<std::mutex> lk(g_tmu);
    if (!b) {
        g_free_events[dev_].push_back(a_);
        return;
    }
    (void)hipEventRecord(b, s_);
    g_pending.push_back(TimedLaunch{name_, a_, b, dev_});
}

} // namespace nbkd

using namespace nbkd;

#define NBKD_GUARD_BEGIN try {
#define NBKD_GUARD_END                                                                             \
    }                                                                                              \
    catch (std::bad_alloc const &) {                                                               \
        set_error("host allocation failed");                                                       \
        return NBKD_ENOMEM;                                                                        \
    }                                                                                              \
    catch (std::exception const &e) {                                                              \
        set_error(e.what());                                                                       \
        return NBKD_EDEVICE;                                                                       \
    }                                                                                              \
    catch (...) {                                                                                  \
        set_error("unknown error");                                                                \
        return NBKD_EDEVICE;                                                                       \
    }

extern "C" {

const char *nbkd_last_error(void) { return g_err.c_str(); }

nbkd_status nbkd_device_count(int32_t *count) {
    if (!count) return NBKD_EINVAL;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    (void)hipGetLastError();
    *count = c;
    return NBKD_OK;
}

nbkd_status nbkd_build(const float *xyz, uint64_t n, int32_t leaf_size, int32_t periodic,
                       float box_size, int32_t device, uint32_t flags, void *stream,
                       nbkd_tree **out) {
    return nbkd_build_ext(xyz, n, leaf_size, periodic, box_size, nullptr, device, flags, stream,
                          out);
}

nbkd_status nbkd_build_ext(const float *xyz, uint64_t n, int32_t leaf_size, int32_t periodic,
                           float box_size, const float *extent, int32_t device, uint32_t flags,
                           void *stream, nbkd_tree **out) {
    NBKD_GUARD_BEGIN
    g_err.clear();
    if (!out || (n > 0 && !xyz)) {
        set_error("nbkd_build: NULL argument");
        return NBKD_EINVAL;
    }
    if (extent && !(extent[0] > 0.0f && extent[1] > 0.0f && extent[2] > 0.0f &&
                    std::isfinite(extent[0]) && std::isfinite(extent[1]) &&
                    std::isfinite(extent[2]))) {
        set_error("nbkd_build_ext: extents must be positive and finite");
        return NBKD_EINVAL;
    }
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        (void)hipGetLastError();
        set_error("no HIP device available: the MI355X kd-tree requires a GPU");
        return NBKD_EDEVICE;
    }
    int dev = device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (dev >= ndev) {
        set_error("nbkd_build: device ordinal out of range");
        return NBKD_EINVAL;
    }
    DeviceGuard g(dev);
    if (!g.ok) {
        set_error("hipSetDevice failed");
        return NBKD_EDEVICE;
    }
    auto *h = new nbkd_tree();
    h->t.device = dev;
    h->t.periodic = periodic ? 1 : 0;
    h->t.box = periodic ? box_size : 0.0f;
    h->t.axes = extent ? axes_for_extent(extent) : AXES_REF;
    nbkd_status st = build_tree(h->t, xyz, n, leaf_size, (flags & NBKD_INPUT_DEVICE) != 0,
                                (hipStream_t)stream);
    if (st != NBKD_OK) {
        (void)hipStreamSynchronize((hipStream_t)stream);
        free_tree(h->t);
        delete h;
        return st;
    }
    if (flags & NBKD_INPUT_DEVICE) h->t.src = xyz;
    *out = h;
    return NBKD_OK;
    NBKD_GUARD_END
}

nbkd_status nbkd_query_knn(const nbkd_tree *tree, const float *q, uint64_t m, int32_t k,
                           float *out_dist, uint32_t *out_idx, uint32_t flags, void *stream) {
    NBKD_GUARD_BEGIN
    g_err.clear();
    if (!tree) {
        set_error("nbkd_query_knn: NULL tree");
        return NBKD_EINVAL;
    }
    if (k <= 0) {
        set_error("k must be positive integer");
        return NBKD_EINVAL;
    }
    if (m > 0 && (!q || !out_dist || !out_idx)) {
        set_error("nbkd_query_knn: NULL argument");
        return NBKD_EINVAL;
    }
    DeviceGuard g(tree->t.device);
    return query_knn(tree->t, q, m, k, out_dist, out_idx, flags, (hipStream_t)stream);
    NBKD_GUARD_END
}

nbkd_status nbkd_query_kth(const nbkd_tree *tree, const float *q, uint64_t m, int32_t k,
                           float *out_dist, uint32_t flags, void *stream) {
    NBKD_GUARD_BEGIN
    g_err.clear();
    if (!tree) {
        set_error("nbkd_query_kth: NULL tree");
        return NBKD_EINVAL;
    }
    if (k <= 0) {
        set_error("k must be positive integer");
        return NBKD_EINVAL;
    }
    if (m > 0 && (!q || !out_dist)) {
        set_error("nbkd_query_kth: NULL argument");
        return NBKD_EINVAL;
    }
    DeviceGuard g(tree->t.device);
    return query_kth(tree->t, q, m, k, out_dist, flags, (hipStream_t)stream);
    NBKD_GUARD_END
}

nbkd_status nbkd_query_ball_count(const nbkd_tree *tree, const float *q, uint64_t m, float r,
                                  uint32_t *out_count, uint32_t flags, void *stream) {
    NBKD_GUARD_BEGIN
    g_err.clear();
    if (!tree || (m > 0 && (!q || !out_count))) {
        set_error("nbkd_query_ball_count: NULL argument");
        return NBKD_EINVAL;
    }
    DeviceGuard g(tree->t.device);
    return query_ball_count(tree->t, q, m, r, out_count, flags, (hipStream_t)stream);
    NBKD_GUARD_END
}

nbkd_status nbkd_query_ball_csr(const nbkd_tree *tree, const float *q, uint64_t m, float r,
                                uint64_t *out_offsets, uint32_t *out_idx, uint64_t capacity,
                                uint32_t flags, void *stream) {
    NBKD_GUARD_BEGIN
    g_err.clear();
    if (!tree || !out_offsets || (m > 0 && !q)) {
        set_error("nbkd_query_ball_csr: NULL argument");
        return NBKD_EINVAL;
    }
    DeviceGuard g(tree->t.device);
    return query_ball_csr(tree->t, q, m, r, out_offsets, out_idx, capacity, flags,
                          (hipStream_t)stream);
    NBKD_GUARD_END
}

nbkd_status nbkd_deposit(const float *xyz, const float *weight, const float *radius, uint64_t n,
                         int32_t gx, int32_t gy, int32_t nz, float ppu, const float *period,
                         int32_t subsample, int32_t mode, int32_t x0, int32_t wx, float *out,
                         int32_t device, uint32_t flags, void *stream) {
    NBKD_GUARD_BEGIN
    g_err.clear();
    if (!out || (n > 0 && (!xyz || !weight || !radius))) {
        set_error("nbkd_deposit: NULL argument");
        return NBKD_EINVAL;
    }
    if (gx < 1 || gy < 1 || nz < 1 || (uint64_t)gx * (uint64_t)gy >= (1ull << 31)) {
        set_error("nbkd_deposit: grid extents must be >= 1 with gx * gy < 2^31");
        return NBKD_EINVAL;
    }
    if (!(ppu > 0.0f) || !std::isfinite(ppu)) {
        set_error("nbkd_deposit: pixels_per_unit must be positive and finite");
        return NBKD_EINVAL;
    }
    if (subsample < 1 || subsample > 16) {
        set_error("nbkd_deposit: subsample must be in [1, 16]");
        return NBKD_EINVAL;
    }
    if (x0 < 0 || wx < 1 || (int64_t)x0 + wx > gx) {
        set_error("nbkd_deposit: the column window [x0, x0 + wx) must lie inside [0, gx)");
        return NBKD_EINVAL;
    }
    if (mode != 0 && !(mode == 1 && nz == 1)) {
        set_error("nbkd_deposit: mode must be 0 (volume) or 1 (one plane, nz = 1)");
        return NBKD_EINVAL;
    }
    DeviceGuard g(device);
    if (!g.ok) {
        set_error("nbkd_deposit: cannot select the device");
        return NBKD_EDEVICE;
    }
    return deposit(xyz, weight, radius, n, gx, gy, nz, ppu, period, subsample, mode, x0, wx, out,
                   flags, (hipStream_t)stream);
    NBKD_GUARD_END
}

nbkd_status nbkd_tree_info(const nbkd_tree *tree, uint64_t *n8, uint64_t *nodes, int32_t *periodic,
                           float *box_size, int32_t *device) {
    if (!tree) {
        set_error("nbkd_tree_info: NULL tree");
        return NBKD_EINVAL;
    }
    if (n8) *n8 = tree->t.n8;
    if (nodes) *nodes = tree->t.nnodes;
    if (periodic) *periodic = tree->t.periodic;
    if (box_size) *box_size = tree->t.box;
    if (device) *device = tree->t.device;
    return NBKD_OK;
}

nbkd_status nbkd_export(const nbkd_tree *tree, nbkd_node *nodes, float *x, float *y, float *z,
                        uint32_t *idx) {
    NBKD_GUARD_BEGIN
    if (!tree) {
        set_error("nbkd_export: NULL tree");
        return NBKD_EINVAL;
    }
    const Tree &t = tree->t;
    DeviceGuard g(t.device);
    if (nodes)
        NBKD_HIP(hipMemcpy(nodes, t.nodes, t.nnodes * sizeof(nbkd_node), hipMemcpyDeviceToHost));
    if (x) NBKD_HIP(hipMemcpy(x, t.x, t.n8 * 4, hipMemcpyDeviceToHost));
    if (y) NBKD_HIP(hipMemcpy(y, t.y, t.n8 * 4, hipMemcpyDeviceToHost));
    if (z) NBKD_HIP(hipMemcpy(z, t.z, t.n8 * 4, hipMemcpyDeviceToHost));
    if (idx) NBKD_HIP(hipMemcpy(idx, t.idx, t.n8 * 4, hipMemcpyDeviceToHost));
    return NBKD_OK;
    NBKD_GUARD_END
}

void nbkd_free(nbkd_tree *tree) {
    if (!tree) return;
    DeviceGuard g(tree->t.device);
    (void)hipDeviceSynchronize();
    free_tree(tree->t);
    delete tree;
}

nbkd_status nbkd_set_tuning(const char *name, double value) {
    if (!name) {
        set_error("nbkd_set_tuning: NULL name");
        return NBKD_EINVAL;
    }
    for (int i = 0; i < TUNE_N; ++i) {
        if (std::strcmp(name, g_tune_names[i]) != 0) continue;
        const bool ok = i == TUNE_KNN_SEED ? (value > 0.0 && value <= 1e3)
                                           : (value >= 0.0 && value < 1e15);
        if (!ok || !std::isfinite(value)) {
            set_error(std::string("nbkd_set_tuning: value out of range for ") + name);
            return NBKD_EINVAL;
        }
        g_tune[i].store(value, std::memory_order_relaxed);
        return NBKD_OK;
    }
    set_error(std::string("nbkd_set_tuning: unknown knob ") + name);
    return NBKD_EINVAL;
}

nbkd_status nbkd_get_tuning(const char *name, double *value) {
    if (!name || !value) {
        set_error("nbkd_get_tuning: NULL argument");
        return NBKD_EINVAL;
    }
    for (int i = 0; i < TUNE_N; ++i)
        if (std::strcmp(name, g_tune_names[i]) == 0) {
            *value = tuning(i);
            return NBKD_OK;
        }
    set_error(std::string("nbkd_get_tuning: unknown knob ") + name);
    return NBKD_EINVAL;
}

nbkd_status nbkd_set_interrupt(nbkd_interrupt_fn fn, void *user) {
    t_intr = fn;
    t_intr_user = user;
    return NBKD_OK;
}

nbkd_status nbkd_timing_enable(int32_t enable) {
    g_timing = enable != 0;
    return NBKD_OK;
}

nbkd_status nbkd_timing_reset(void) {
    std::lock_guard<std::mutex> lk(g_tmu);
    for (auto &p : g_pending) {
        (void)hipEventSynchronize(p.b);
        give_events(p);
    }
    g_pending.clear();
    g_acc.clear();
    return NBKD_OK;
}

nbkd_status nbkd_timing_read(const char *name, double *ms, uint64_t *launches) {
    if (!name) return NBKD_EINVAL;
    std::lock_guard<std::mutex> lk(g_tmu);
    for (auto &p : g_pending) {
        if (hipEventSynchronize(p.b) != hipSuccess) return hip_fail(hipGetLastError(), "timing");
        float t = 0.0f;
        (void)hipEventElapsedTime(&t, p.a, p.b);
        auto &acc = g_acc[p.name];
        acc.first += t;
        acc.second += 1;
        give_events(p);
    }
    g_pending.clear();
    auto it = g_acc.find(name);
    if (ms) *ms = it == g_acc.end() ? 0.0 : it->second.first;
    if (launches) *launches = it == g_acc.end() ? 0 : it->second.second;
    return NBKD_OK;
}

nbkd_status nbkd_stats_enable(int32_t enable) {
    g_stats_on = enable != 0;
    return NBKD_OK;
}

nbkd_status nbkd_stats_read(uint64_t *nodes_visited, uint64_t *points_scanned) {
    if (nodes_visited) *nodes_visited = g_stats[0];
    if (points_scanned) *points_scanned = g_stats[1];
    return NBKD_OK;
}

nbkd_status nbkd_stats_read_all(uint64_t *out, int32_t n) {
    if (!out || n < 0) return NBKD_EINVAL;
    for (int i = 0; i < n && i < NBKD_NSTATS; ++i) out[i] = g_stats[i];
    return NBKD_OK;
}

} // extern "C"

namespace nbkd {

void *Workspace::get(int slot, size_t bytes, hipStream_t s) {
    if (bytes == 0) bytes = 16;
    if (cap[slot] >= bytes) return p[slot];
    if (p[slot]) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(p[slot]);
        p[slot] = nullptr;
        cap[slot] = 0;
    }
    size_t want = bytes + bytes / 8; // some headroom for the next, slightly larger call
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        dev = -1;
    }
    hipError_t e = malloc_or_release(&p[slot], want);
    if (e != hipSuccess) {
        (void)hip_fail(e, "hipMalloc(workspace)");
        p[slot] = nullptr;
        return nullptr;
    }
    cap[slot] = want;
    return p[slot];
}

void Workspace::release() {
    for (int i = 0; i < WS_NSLOTS; ++i) {
        if (p[i]) (void)hipFree(p[i]);
        p[i] = nullptr;
        cap[i] = 0;
    }
    if (done) (void)hipEventDestroy(done);
    done = nullptr;
    used = false;
    for (hipEvent_t &e : pev) {
        if (e) (void)hipEventDestroy(e);
        e = nullptr;
    }
    if (copy) (void)hipStreamDestroy(copy);
    copy = nullptr;
    free_pinned();
}

// Pinned staging over every workspace of the process is capped (ADVICE r05:
// several trees or workspaces could each keep ~2 GiB pinned): past the cap,
// or when hipHostMalloc fails, host_pinned returns nullptr and the pipeline
// streams through pageable memory instead (the runtime stages those copies).
static std::atomic<uint64_t> g_pinned_bytes{0};
static uint64_t pinned_cap() { // nbkd_set_tuning("pinned_bytes"), 0 = 8 GiB
    const double v = tuning(TUNE_PINNED_BYTES);
    return v > 0.0 ? (uint64_t)v : (8ull << 30);
}

void Workspace::free_pinned() {
    for (int b = 0; b < 2; ++b) {
        if (hpin[b]) {
            (void)hipHostFree(hpin[b]);
            g_pinned_bytes -= hpin_cap[b];
        }
        hpin[b] = nullptr;
        hpin_cap[b] = 0;
    }
}

void *Workspace::host_pinned(int slot, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (hpin_cap[slot] >= bytes) return hpin[slot];
    if (hpin[slot]) {
        // the slot's last DMA belongs to a finished call (every call drains
        // its copies before returning)
        (void)hipHostFree(hpin[slot]);
        g_pinned_bytes -= hpin_cap[slot];
        hpin[slot] = nullptr;
        hpin_cap[slot] = 0;
    }
    if (g_pinned_bytes.fetch_add(bytes) + bytes > pinned_cap()) {
        g_pinned_bytes -= bytes;
        return nullptr; // over the process cap: pageable streaming
    }
    hipError_t e = hipHostMalloc(&hpin[slot], bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError(); // not an error of the call: pageable streaming
        g_pinned_bytes -= bytes;
        hpin[slot] = nullptr;
        return nullptr;
    }
    hpin_cap[slot] = bytes;
    return hpin[slot];
}

hipError_t Workspace::pipe_init() {
    if (!copy) {
        hipError_t e = hipStreamCreateWithFlags(&copy, hipStreamNonBlocking);
        if (e != hipSuccess) {
            copy = nullptr;
            return e;
        }
    }
    for (hipEvent_t &ev : pev)
        if (!ev) {
            hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
            if (e != hipSuccess) {
                ev = nullptr;
                return e;
            }
        }
    return hipSuccess;
}

void Workspace::trim() {
    if (used && done) (void)hipEventSynchronize(done);
    for (int i = 0; i < WS_NSLOTS; ++i) {
        if (p[i]) (void)hipFree(p[i]);
        p[i] = nullptr;
        cap[i] = 0;
    }
    // an idle workspace's pinned staging goes back too (every call drains its
    // copies before returning, so no DMA can still use it)
    free_pinned();
    (void)hipGetLastError();
}

hipError_t Workspace::enter(hipStream_t s) {
    if (used && s != last && done) return hipStreamWaitEvent(s, done, 0);
    return hipSuccess;
}

void Workspace::leave(hipStream_t s) {
    if (!done && hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        done = nullptr;
        (void)hipStreamSynchronize(s); // no event: drain instead
        used = false;
        return;
    }
    if (hipEventRecord(done, s) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipStreamSynchronize(s);
        used = false;
        return;
    }
    last = s;
    used = true;
}

} // namespace nbkd
