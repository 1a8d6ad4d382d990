// Host-buffer witness commit (bj_lde_commit_h): what a Rust prover handing over host Vecs calls
// (prover.rs:313-353 over Vec<GoldilocksField> storages).  The trace comes in over PCIe, every
// output goes back.  DESIGN.md section 6 ("Host-resident boundary").
//
// Column-chunked pipeline: the trace of chunk k+1 goes in (calling thread) while chunk k is
// transformed and absorbed into the leaf sponges (compute stream) and the LDE of chunk k-1 comes
// out (a copy-out thread), so both PCIe directions and the GPU work at once.  Chunks are 8, 8,
// 16, then 32 columns (multiples of the sponge rate); the leaf sponges carry their capacity words
// between chunks (bj_merkle_leaves_partial_d), so outputs equal the one-shot commit.
//
// The trace goes in on the copy engine (the runtime's pageable path).  The outputs come back
// through a small ring of pinned slots: CU store kernels write a slot (store_to_host) while a
// pool of host threads copies the previous one into the caller's buffer (130 GB/s on 8
// threads).  Memory the caller has page-locked itself is written directly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/boojum_mi355x.h"
#include "bj_internal.hpp"

namespace {

int err(int code, const std::string& msg) { return bj::set_error(code, msg.c_str()); }
int hip_err(hipError_t e, const char* what) { return err(BJ_EHIP, std::string(what) + ": " + hipGetErrorString(e)); }

#define HIP_CHECK(expr, what)                         \
    do {                                              \
        hipError_t e_ = (expr);                       \
        if (e_ != hipSuccess) return hip_err(e_, what); \
    } while (0)

// Persistent host threads for parallel memcpy (never destroyed: they sleep between calls).
class CopyPool {
  public:
    explicit CopyPool(unsigned workers) {
        for (unsigned i = 0; i < workers; i++) th_.emplace_back([this] { loop(); });
        parts_ = workers + 1;
    }
    // dst <- src over the workers and the calling thread; returns when every part is done
    void copy(void* dst, const void* src, size_t bytes) {
        const unsigned parts = bytes < ((size_t)4 << 20) ? 1 : parts_;
        const size_t per = ((bytes + parts - 1) / parts + 4095) & ~(size_t)4095;
        std::atomic<unsigned> left{0};
        std::mutex m;
        std::condition_variable cv;
        {
            std::lock_guard<std::mutex> lk(mu_);
            unsigned queued = 0;
            for (size_t off = per; off < bytes; off += per) {
                char* d = static_cast<char*>(dst) + off;
                const char* s = static_cast<const char*>(src) + off;
                const size_t len = std::min(per, bytes - off);
                q_.push_back([d, s, len, &left, &m, &cv] {
                    std::memcpy(d, s, len);
                    if (left.fetch_sub(1) == 1) {
                        std::lock_guard<std::mutex> l(m);
                        cv.notify_one();
                    }
                });
                queued++;
            }
            left.store(queued);  // before any worker can pop (they pop under mu_)
        }
        cv_.notify_all();
        std::memcpy(dst, src, std::min(per, bytes));
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return left.load() == 0; });
    }

  private:
    void loop() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return !q_.empty(); });
                f = std::move(q_.front());
                q_.pop_front();
            }
            f();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    unsigned parts_ = 1;
};

// BJ_COPY_THREADS (default 6) threads share each copy-out, counting the calling thread.
CopyPool& copy_pool() {
    static CopyPool* p = [] {
        const char* e = std::getenv("BJ_COPY_THREADS");
        const int t = e ? std::atoi(e) : 6;
        return new CopyPool((unsigned)std::max(0, std::min(t, 64) - 1));
    }();
    return *p;
}

constexpr size_t SLOT = (size_t)64 << 20;  // bytes per pinned slot
constexpr int RING = 3;                    // copy-out slots

// A staging set: pinned slots, their reuse events, and the three streams (created once:
// stream creation and pinning cost milliseconds).  The sets live in a bounded per-device pool
// shared by every calling thread: a call takes a free set (or makes one while fewer than
// kMaxStaging exist, else waits for one) and returns it when done, so a rayon-style pool of
// callers holds at most kMaxStaging x 192 MiB of pinned memory per device, not one set per
// thread.  The sets are kept for the life of the process.
struct Staging {
    char* out[RING] = {};
    hipEvent_t out_ev[RING] = {};
    hipStream_t s_in = nullptr, s_cmp = nullptr, s_out = nullptr;
};
constexpr size_t kMaxStaging = 4;

struct StagingPool {
    std::mutex mu;
    std::condition_variable cv;
    std::map<int, std::vector<Staging*>> free_, all_;
};
StagingPool& staging_pool() {
    static StagingPool* p = new StagingPool();
    return *p;
}

int make_staging(Staging* sg) {
    for (int i = 0; i < RING; i++) {
        HIP_CHECK(hipHostMalloc((void**)&sg->out[i], SLOT, hipHostMallocDefault), "hipHostMalloc");
        HIP_CHECK(hipEventCreateWithFlags(&sg->out_ev[i], hipEventDisableTiming), "hipEventCreate");
    }
    HIP_CHECK(hipStreamCreateWithFlags(&sg->s_in, hipStreamNonBlocking), "hipStreamCreate");
    HIP_CHECK(hipStreamCreateWithFlags(&sg->s_cmp, hipStreamNonBlocking), "hipStreamCreate");
    HIP_CHECK(hipStreamCreateWithFlags(&sg->s_out, hipStreamNonBlocking), "hipStreamCreate");
    return BJ_OK;
}

// Takes a staging set of the current device for the duration of one call.
struct StagingLease {
    Staging* sg = nullptr;
    int dev = 0;
    int acquire() {
        HIP_CHECK(hipGetDevice(&dev), "hipGetDevice");
        StagingPool& p = staging_pool();
        std::unique_lock<std::mutex> lk(p.mu);
        for (;;) {
            auto& fr = p.free_[dev];
            if (!fr.empty()) {
                sg = fr.back();
                fr.pop_back();
                return BJ_OK;
            }
            if (p.all_[dev].size() < kMaxStaging) break;
            p.cv.wait(lk);
        }
        Staging* s = new Staging();
        p.all_[dev].push_back(s);  // reserve the slot before dropping the lock
        lk.unlock();
        if (int r = make_staging(s)) {
            // give the slot back; the half-made set's resources are released
            for (int i = 0; i < RING; i++) {
                if (s->out[i]) (void)hipHostFree(s->out[i]);
                if (s->out_ev[i]) (void)hipEventDestroy(s->out_ev[i]);
            }
            for (hipStream_t q : {s->s_in, s->s_cmp, s->s_out})
                if (q) (void)hipStreamDestroy(q);
            {
                std::lock_guard<std::mutex> g(p.mu);
                auto& a = p.all_[dev];
                a.erase(std::find(a.begin(), a.end(), s));
            }
            p.cv.notify_one();
            delete s;
            return r;
        }
        sg = s;
        return BJ_OK;
    }
    ~StagingLease() {
        if (!sg) return;
        StagingPool& p = staging_pool();
        {
            std::lock_guard<std::mutex> lk(p.mu);
            p.free_[dev].push_back(sg);
        }
        p.cv.notify_one();
    }
};

// Page-locked by the caller (hipHostRegister / hipHostMalloc): DMA it directly.
bool is_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Device-to-host copies are CU stores straight into pinned host memory.  The copy engines' own
// device-to-host rate falls to ~30 GB/s once the GPU has been computing (and recovers only after
// about a second idle), while a store kernel keeps ~55 GB/s (tools/d2h_after_compute_probe.cpp).
// Its waves need few VGPRs, so they co-run with the VGPR-limited hashing kernels.
__global__ __launch_bounds__(256) void store_to_host_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                            size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
__global__ __launch_bounds__(256) void store_to_host_kernel8(uint2* __restrict__ dst, const uint2* __restrict__ src,
                                                             size_t n8) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// dst_host (pinned, device-visible) <- src_dev, asynchronous on s; falls back to the copy engine
// for memory the device cannot address or sizes off the 8-byte grid
hipError_t store_to_host(void* dst_host, const void* src_dev, size_t bytes, hipStream_t s) {
    void* dp = nullptr;
    if (bytes % 8 || hipHostGetDevicePointer(&dp, dst_host, 0) != hipSuccess || !dp) {
        (void)hipGetLastError();
        return hipMemcpyAsync(dst_host, src_dev, bytes, hipMemcpyDeviceToHost, s);
    }
    const unsigned blocks = 128;
    if (((uintptr_t)dp | (uintptr_t)src_dev | bytes) % 16 == 0)
        store_to_host_kernel<<<blocks, 256, 0, s>>>(static_cast<uint4*>(dp), static_cast<const uint4*>(src_dev),
                                                    bytes / 16);
    else
        store_to_host_kernel8<<<blocks, 256, 0, s>>>(static_cast<uint2*>(dp), static_cast<const uint2*>(src_dev),
                                                     bytes / 8);
    return hipGetLastError();
}

// host <- device over s_out, synchronous; up to RING pieces in flight, the host copy of piece i
// overlapping the device stores of the next ones.
hipError_t d2h(Staging& sg, void* host, const void* dev, size_t bytes, bool pinned) {
    if (bytes == 0) return hipSuccess;
    if (pinned) {
        hipError_t e = store_to_host(host, dev, bytes, sg.s_out);
        return e == hipSuccess ? hipStreamSynchronize(sg.s_out) : e;
    }
    const size_t pieces = (bytes + SLOT - 1) / SLOT;
    size_t issued = 0, done = 0;
    while (done < pieces) {
        while (issued < pieces && issued - done < (size_t)RING) {
            const size_t off = issued * SLOT, len = std::min(SLOT, bytes - off);
            const unsigned k = issued % RING;
            hipError_t e = store_to_host(sg.out[k], static_cast<const char*>(dev) + off, len, sg.s_out);
            if (e == hipSuccess) e = hipEventRecord(sg.out_ev[k], sg.s_out);
            if (e != hipSuccess) return e;
            issued++;
        }
        const size_t off = done * SLOT, len = std::min(SLOT, bytes - off);
        const unsigned k = done % RING;
        hipError_t e = hipEventSynchronize(sg.out_ev[k]);
        if (e != hipSuccess) return e;
        copy_pool().copy(static_cast<char*>(host) + off, sg.out[k], len);
        done++;
    }
    return hipSuccess;
}

}  // namespace

extern "C" int bj_lde_commit_h(const uint64_t* trace_h, uint32_t n_cols, uint32_t log_n, uint32_t log_lde,
                               uint32_t log_commit_cosets, uint32_t cap_size, uint64_t* lde_h, uint64_t* leaves_h,
                               uint64_t* nodes_h, uint64_t* cap_h) {
    if (log_n + log_lde > 32) return err(BJ_EINVAL, "log_n exceeds the 2-adicity (32) of the field");
    if (log_commit_cosets > log_lde)
        return err(BJ_EINVAL, "committed cosets exceed the lde degree (prover.rs:313, lde.rs:298-308)");
    // nd: LDE length per column (all D cosets); nl: leaves, the first k cosets (subset_for_degree)
    const size_t n = (size_t)1 << log_n, nd = n << log_lde, nl = n << log_commit_cosets;
    if (!cap_size || (cap_size & (cap_size - 1)) || nl <= cap_size)
        return err(BJ_EINVAL, "need power-of-two cap_size < n * k");
    if (log_lde == 0) return err(BJ_EINVAL, "lde degree must be > 1 (utils.rs:283)");
    if (n_cols && !trace_h) return err(BJ_EINVAL, "null trace");
    // chunk k covers columns [c_first[k], c_first[k + 1]): 8, 8, 16, then 32 at a time (every
    // chunk but the last a multiple of the sponge rate), so the first LDE columns start back
    // across PCIe early and the later chunks amortise their launches
    std::vector<uint32_t> c_first{0};
    for (uint32_t w = 8; c_first.back() < n_cols; w = std::min(2 * w, 32u)) {
        c_first.push_back(std::min(n_cols, c_first.back() + w));
        if (c_first.size() == 2) w = 4;  // second chunk 8 as well
    }
    const uint32_t n_chunks = (uint32_t)c_first.size() - 1;
    StagingLease lease;
    if (int r = lease.acquire()) return r;
    Staging& sg = *lease.sg;
    hipStream_t s_in = sg.s_in, s_cmp = sg.s_cmp, s_out = sg.s_out;
    const int dev = lease.dev;
    const bool pin_lde = lde_h && is_pinned(lde_h);
    const size_t tn = n * n_cols;
    uint64_t *tr = nullptr, *mono = nullptr, *lde = nullptr, *lv = nullptr, *nodes = nullptr, *st = nullptr;
    // the library's own stream-ordered pool keeps this workspace mapped between calls
    HIP_CHECK(bj::pool_alloc((void**)&tr, tn * 8, s_cmp), "pool_alloc");
    HIP_CHECK(bj::pool_alloc((void**)&mono, tn * 8, s_cmp), "pool_alloc");
    HIP_CHECK(bj::pool_alloc((void**)&lde, (tn << log_lde) * 8, s_cmp), "pool_alloc");
    HIP_CHECK(bj::pool_alloc((void**)&lv, nl * 32, s_cmp), "pool_alloc");
    HIP_CHECK(bj::pool_alloc((void**)&nodes, (nl - cap_size) * 32, s_cmp), "pool_alloc");
    HIP_CHECK(bj::pool_alloc((void**)&st, nl * 32, s_cmp), "pool_alloc");
    HIP_CHECK(hipStreamSynchronize(s_cmp), "sync");
    struct Frees {
        uint64_t** p[6];
        hipStream_t s, s_in, s_out;
        ~Frees() {
            // copies still in flight on an error path finish before the buffers go back
            (void)hipStreamSynchronize(s_in);
            (void)hipStreamSynchronize(s_out);
            for (auto q : p)
                if (*q) (void)hipFreeAsync(*q, s);
            (void)hipStreamSynchronize(s);
        }
    } frees{{&tr, &mono, &lde, &lv, &nodes, &st}, s_cmp, s_in, s_out};
    std::vector<hipEvent_t> ev_in(n_chunks, nullptr), ev_cmp(n_chunks, nullptr);
    struct Events {
        std::vector<hipEvent_t>* v[2];
        ~Events() {
            for (auto e : v)
                for (auto x : *e)
                    if (x) (void)hipEventDestroy(x);
        }
    } evg{{&ev_in, &ev_cmp}};
    for (uint32_t k = 0; k < n_chunks; k++) {
        HIP_CHECK(hipEventCreateWithFlags(&ev_in[k], hipEventDisableTiming), "hipEventCreate");
        HIP_CHECK(hipEventCreateWithFlags(&ev_cmp[k], hipEventDisableTiming), "hipEventCreate");
    }
    // copy-out thread: the LDE rows of chunk k as soon as its compute is done.  It waits on the
    // host until this thread has recorded ev_cmp[k], and stops early when the issuing side fails.
    hipError_t out_err = hipSuccess;
    std::mutex mu;
    std::condition_variable cv;
    uint32_t recorded = 0;
    bool abort_out = false;
    std::thread out_thread([&]() {
        (void)hipSetDevice(dev);
        for (uint32_t k = 0; k < n_chunks && out_err == hipSuccess && lde_h; k++) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return recorded > k || abort_out; });
                if (recorded <= k) return;
            }
            const uint32_t c0 = c_first[k], c = c_first[k + 1] - c0;
            hipError_t e = hipStreamWaitEvent(s_out, ev_cmp[k], 0);
            if (e == hipSuccess) e = d2h(sg, lde_h + (size_t)c0 * nd, lde + (size_t)c0 * nd, (size_t)c * nd * 8, pin_lde);
            if (e != hipSuccess) out_err = e;
        }
    });
    struct Join {
        std::thread* t;
        std::mutex* mu;
        std::condition_variable* cv;
        bool* abort_out;
        ~Join() {
            {
                std::lock_guard<std::mutex> lk(*mu);
                *abort_out = true;
            }
            cv->notify_all();
            if (t->joinable()) t->join();
        }
    } join{&out_thread, &mu, &cv, &abort_out};
    for (uint32_t k = 0; k < n_chunks; k++) {
        const uint32_t c0 = c_first[k], c = c_first[k + 1] - c0;
        const bool last = k + 1 == n_chunks;
        // host-to-device stays on the copy engine: the runtime's own path for pageable memory
        // keeps ~56 GB/s here beside the store kernels (staging it through our slots was slower)
        HIP_CHECK(hipMemcpyAsync(tr + (size_t)c0 * n, trace_h + (size_t)c0 * n, (size_t)c * n * 8,
                                 hipMemcpyHostToDevice, s_in),
                  "memcpy trace");
        HIP_CHECK(hipEventRecord(ev_in[k], s_in), "hipEventRecord");
        HIP_CHECK(hipStreamWaitEvent(s_cmp, ev_in[k], 0), "hipStreamWaitEvent");
        if (int r = bj_lde_d(tr + (size_t)c0 * n, c, n, log_n, log_lde, mono + (size_t)c0 * n, lde + (size_t)c0 * nd,
                             s_cmp))
            return r;
        // the sponges absorb the chunk's first k cosets (leaf L < k * n of column c at c * nd + L)
        if (int r = bj_merkle_leaves_partial_d(lde + (size_t)c0 * nd, c, nd, nl, k ? st : nullptr, last ? lv : st,
                                               last ? 1 : 0, s_cmp))
            return r;
        HIP_CHECK(hipEventRecord(ev_cmp[k], s_cmp), "hipEventRecord");
        {
            std::lock_guard<std::mutex> lk(mu);
            recorded = k + 1;
        }
        cv.notify_all();
    }
    if (n_chunks == 0)
        if (int r = bj_merkle_leaves_d(lde, 0, nd, nl, lv, s_cmp)) return r;
    hipEvent_t ev_leaves = nullptr, ev_nodes = nullptr;
    HIP_CHECK(hipEventCreateWithFlags(&ev_leaves, hipEventDisableTiming), "hipEventCreate");
    struct Ev {
        hipEvent_t* e;
        ~Ev() {
            if (*e) (void)hipEventDestroy(*e);
        }
    } evl{&ev_leaves}, evn{&ev_nodes};
    HIP_CHECK(hipEventCreateWithFlags(&ev_nodes, hipEventDisableTiming), "hipEventCreate");
    HIP_CHECK(hipEventRecord(ev_leaves, s_cmp), "hipEventRecord");
    if (int r = bj_merkle_nodes_d(lv, nl, cap_size, nodes, s_cmp)) return r;
    HIP_CHECK(hipEventRecord(ev_nodes, s_cmp), "hipEventRecord");
    out_thread.join();
    if (out_err != hipSuccess) return hip_err(out_err, "memcpy lde");
    // the leaf digests go out while the node levels are hashed
    if (leaves_h) {
        HIP_CHECK(hipStreamWaitEvent(s_out, ev_leaves, 0), "hipStreamWaitEvent");
        HIP_CHECK(d2h(sg, leaves_h, lv, nl * 32, is_pinned(leaves_h)), "memcpy leaves");
    }
    HIP_CHECK(hipStreamWaitEvent(s_out, ev_nodes, 0), "hipStreamWaitEvent");
    if (nodes_h) HIP_CHECK(d2h(sg, nodes_h, nodes, (nl - cap_size) * 32, is_pinned(nodes_h)), "memcpy nodes");
    if (cap_h) {
        HIP_CHECK(hipMemcpyAsync(cap_h, nodes + 4 * (nl - 2 * (size_t)cap_size), (size_t)cap_size * 32,
                                 hipMemcpyDeviceToHost, s_out),
                  "memcpy cap");
    }
    HIP_CHECK(hipStreamSynchronize(s_out), "sync");
    HIP_CHECK(hipStreamSynchronize(s_in), "sync");
    return BJ_OK;
}
