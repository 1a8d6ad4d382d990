// Collective sharded witness commit: the multi-GPU split of the commitment as one native call
// per rank (include/boojum_mi355x.h, "collective sharded commit").
//
// The reference commits on one host (transform_raw_storages_to_lde, utils.rs:270-403, then
// MerkleTreeWithCap::construct, merkle_tree.rs:78-172, driven by prover.rs:313-353).  Here the
// flat leaf domain (coset * n + row) is cut into G contiguous ranges, one per rank, and every
// rank hashes a subtree of the reference's tree.  The only data exchange is per column chunk:
//   G <= D  all-gather of the chunk's coefficients (bj_lde_coeffs_d format), then this rank's
//           whole cosets (bj_lde_shard_d);
//   G >  D  the sender folds its own columns for every rank (bj_lde_fold_shards_d), one
//           all-to-all delivers them, then this rank's sub-coset (bj_lde_shard_folded_d).
// Chunk k's exchange runs on a high-priority stream while the compute stream transforms and
// absorbs the chunks that have already arrived; the leaf sponge carries its capacity words
// (Poseidon2) or chaining value (Blake2s) between chunks.  The cap is all-gathered at the end.
//
// Transports behind bj_comm: RCCL (resolved with dlopen, so the library loads without it) and
// an in-process "local" group of ranks sharing one device (device-to-device copies ordered by
// events through a host barrier), which runs the same pipeline multi-rank on a single GPU.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/boojum_mi355x.h"
#include "bj_internal.hpp"
#include "gl.hpp"

namespace {

int err(int code, const std::string& msg) { return bj::set_error(code, msg.c_str()); }

#define HIP_CHECK(expr, what)                                                            \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) return err(BJ_EHIP, std::string(what) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define BJ_CHECK(expr)               \
    do {                             \
        if (int r_ = (expr)) return r_; \
    } while (0)

// ------------------------------------------------------------------ RCCL, at run time
struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    // what the communicator itself reports (bj_comm_info); optional: a librccl without them
    // still runs commits, and bj_comm_info then fails for RCCL communicators
    decltype(&ncclCommCount) comm_count = nullptr;
    decltype(&ncclCommUserRank) comm_user_rank = nullptr;
    decltype(&ncclCommCuDevice) comm_cu_device = nullptr;
    bool ok = false;
    std::string why;
};

// The process's RCCL: the copy already loaded (torch's, say) when there is one, so a
// communicator made by the caller and our calls on it use the same library.
const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
        if (!h) {
            const char* e = dlerror();
            r.why = std::string("cannot load librccl.so.1: ") + (e ? e : "");
            return;
        }
#define RCCL_SYM(field, name)                                             \
    r.field = reinterpret_cast<decltype(r.field)>(dlsym(h, name));       \
    if (!r.field) {                                                       \
        r.why = "librccl.so.1 does not export " name;                     \
        return;                                                           \
    }
        RCCL_SYM(get_unique_id, "ncclGetUniqueId")
        RCCL_SYM(init_rank, "ncclCommInitRank")
        RCCL_SYM(destroy, "ncclCommDestroy")
        RCCL_SYM(all_gather, "ncclAllGather")
        RCCL_SYM(send, "ncclSend")
        RCCL_SYM(recv, "ncclRecv")
        RCCL_SYM(group_start, "ncclGroupStart")
        RCCL_SYM(group_end, "ncclGroupEnd")
        RCCL_SYM(error_string, "ncclGetErrorString")
#undef RCCL_SYM
        r.comm_count = reinterpret_cast<decltype(r.comm_count)>(dlsym(h, "ncclCommCount"));
        r.comm_user_rank = reinterpret_cast<decltype(r.comm_user_rank)>(dlsym(h, "ncclCommUserRank"));
        r.comm_cu_device = reinterpret_cast<decltype(r.comm_cu_device)>(dlsym(h, "ncclCommCuDevice"));
        r.ok = true;
    });
    return r;
}

int rccl_fail(const Rccl& r, ncclResult_t e, const char* what) {
    return err(BJ_EHIP, std::string(what) + ": " + r.error_string(e));
}

#define RCCL_CHECK(R, expr, what)                                   \
    do {                                                            \
        ncclResult_t e_ = (expr);                                   \
        if (e_ != ncclSuccess) return rccl_fail(R, e_, what);       \
    } while (0)

// ----------------------------------------------------- in-process rank group (one device)
struct LocalGroup {
    int world = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    bool aborted = false;  // a rank failed mid-collective: the group is unusable from then on
    std::vector<const void*> slot;
    std::vector<hipEvent_t> ready, done;

    // false when a peer aborted (instead of waiting for it forever)
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) return false;
        const uint64_t g = generation;
        if (++arrived == world) {
            arrived = 0;
            generation++;
            cv.notify_all();
            return true;
        }
        cv.wait(lk, [&] { return generation != g || aborted; });
        return generation != g;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
};

}  // namespace

struct bj_comm {
    enum Kind { RCCL_OWNED, RCCL_WRAPPED, LOCAL, CALLBACK } kind;
    int world = 1, rank = 0;
    int device = -1;  // the device current when the communicator was made (bj_comm_info)
    ncclComm_t nccl = nullptr;
    LocalGroup* group = nullptr;
    bj_exchange_fn fn = nullptr;  // CALLBACK: the caller's exchange
    void* user = nullptr;
    int host_staged = 1;
    hipStream_t xs = nullptr;  // exchange stream, high priority, created on first use
    int xs_dev = -1;
    // bj_comm_set_timing: (start, end, phase) event triples of the calls not yet read
    bool timing = false;
    struct Interval {
        hipEvent_t a, b;
        int phase;
    };
    std::vector<Interval> intervals;
    float folded_ms[4] = {0, 0, 0, 0};  // intervals already completed and summed
    std::string timing_error;           // first failure to read an interval, reported by bj_comm_phase_ms
    int timed_calls = 0;
};

namespace {

// Sum the intervals whose end event has completed into folded_ms and free their events (all of
// them when `wait`).  Called at the start of every commit, so a caller that times calls and never
// reads the totals holds the events of its in-flight calls only.  Timing is bookkeeping: an event
// that cannot be read is kept as timing_error for bj_comm_phase_ms, never a failure of the commit.
void fold_intervals(bj_comm* c, bool wait) {
    size_t keep = 0;
    for (size_t i = 0; i < c->intervals.size(); i++) {
        const bj_comm::Interval iv = c->intervals[i];
        hipError_t e = wait ? hipEventSynchronize(iv.b) : hipEventQuery(iv.b);
        if (e == hipErrorNotReady) {
            c->intervals[keep++] = iv;
            continue;
        }
        float ms = 0;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, iv.a, iv.b);
        if (e != hipSuccess && c->timing_error.empty())
            c->timing_error = std::string("phase timing: ") + hipGetErrorString(e);
        if (iv.phase >= 0 && iv.phase < 4) c->folded_ms[iv.phase] += ms;
        (void)hipEventDestroy(iv.a);
        (void)hipEventDestroy(iv.b);
    }
    c->intervals.resize(keep);
}

// Phase intervals of one timed call (bj_comm_set_timing); a no-op when timing is off.
struct PhaseTimer {
    bj_comm* c;
    hipStream_t st;
    hipEvent_t open = nullptr;
    int phase = -1;
    PhaseTimer(bj_comm* comm, hipStream_t s) : c(comm), st(s) {}
    int begin(int ph) {
        if (!c->timing) return BJ_OK;
        HIP_CHECK(hipEventCreate(&open), "hipEventCreate");
        phase = ph;
        HIP_CHECK(hipEventRecord(open, st), "hipEventRecord");
        return BJ_OK;
    }
    int end() {
        if (!c->timing || !open) return BJ_OK;
        hipEvent_t e;
        HIP_CHECK(hipEventCreate(&e), "hipEventCreate");
        HIP_CHECK(hipEventRecord(e, st), "hipEventRecord");
        c->intervals.push_back({open, e, phase});
        open = nullptr;
        return BJ_OK;
    }
    ~PhaseTimer() {
        if (open) (void)hipEventDestroy(open);
    }
};

int exchange_stream(bj_comm* c, hipStream_t* out) {
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev), "hipGetDevice");
    if (c->xs && c->xs_dev != dev) return err(BJ_EINVAL, "communicator used from another device");
    if (!c->xs) {
        int least = 0, greatest = 0;
        HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest), "stream priority range");
        HIP_CHECK(hipStreamCreateWithPriority(&c->xs, hipStreamNonBlocking, greatest), "hipStreamCreate");
        c->xs_dev = dev;
    }
    *out = c->xs;
    return BJ_OK;
}

// recv block p <- rank p's send block (all-to-all: its block `rank`; all-gather: its only one)
int local_exchange(bj_comm* c, const void* send, void* recv, size_t bytes, bool all_to_all, hipStream_t st) {
    LocalGroup& g = *c->group;
    const int me = c->rank;
    HIP_CHECK(hipEventRecord(g.ready[me], st), "hipEventRecord");
    g.slot[me] = send;
    // every rank's send buffer and ready event are published
    if (!g.barrier()) return err(BJ_EINVAL, "a peer rank of the local group failed");
    for (int p = 0; p < g.world; p++) {
        HIP_CHECK(hipStreamWaitEvent(st, g.ready[p], 0), "hipStreamWaitEvent");
        const char* src = static_cast<const char*>(g.slot[p]) + (all_to_all ? (size_t)me * bytes : 0);
        char* dst = static_cast<char*>(recv) + (size_t)p * bytes;
        if (src != dst && bytes) HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st), "memcpy");
    }
    HIP_CHECK(hipEventRecord(g.done[me], st), "hipEventRecord");
    // every rank has queued its reads of the others' buffers
    if (!g.barrier()) return err(BJ_EINVAL, "a peer rank of the local group failed");
    for (int p = 0; p < g.world; p++) HIP_CHECK(hipStreamWaitEvent(st, g.done[p], 0), "hipStreamWaitEvent");
    // nobody re-records this round's events before all waits are queued
    if (!g.barrier()) return err(BJ_EINVAL, "a peer rank of the local group failed");
    return BJ_OK;
}

// The caller's exchange (bj_comm_init_callback).  Host-staged: the device data goes to host
// memory, the callback exchanges host buffers (gloo, MPI, ...), the result comes back; every
// step synchronises, so this transport is for rehearsal and tests, not for overlap.  Device
// mode hands the callback device pointers and the stream to order its work on.
int callback_exchange(bj_comm* c, int kind, const void* send, void* recv, size_t bytes, hipStream_t st) {
    const size_t world = (size_t)c->world;
    const size_t send_bytes = kind == BJ_XCHG_ALL_TO_ALL ? world * bytes : bytes, recv_bytes = world * bytes;
    if (!c->host_staged) {
        if (int r = c->fn(c->user, kind, send, recv, bytes, st))
            return err(BJ_EINVAL, "exchange callback failed (" + std::to_string(r) + ")");
        return BJ_OK;
    }
    std::vector<uint8_t> hs(send_bytes), hr(recv_bytes);
    HIP_CHECK(hipStreamSynchronize(st), "sync");
    if (send_bytes) HIP_CHECK(hipMemcpyAsync(hs.data(), send, send_bytes, hipMemcpyDeviceToHost, st), "memcpy");
    HIP_CHECK(hipStreamSynchronize(st), "sync");
    if (int r = c->fn(c->user, kind, hs.data(), hr.data(), bytes, nullptr))
        return err(BJ_EINVAL, "exchange callback failed (" + std::to_string(r) + ")");
    if (recv_bytes) HIP_CHECK(hipMemcpyAsync(recv, hr.data(), recv_bytes, hipMemcpyHostToDevice, st), "memcpy");
    HIP_CHECK(hipStreamSynchronize(st), "sync");
    return BJ_OK;
}

// recv (world x bytes) <- concat over ranks of send (bytes); send may be recv + rank * bytes
// A one-rank RCCL communicator still runs the RCCL call (a copy inside RCCL), so the calls the
// multi-GPU run depends on are exercised on a one-GPU box (tests/test_gpu_rccl.py).
bool is_rccl(const bj_comm* c) { return c->kind == bj_comm::RCCL_OWNED || c->kind == bj_comm::RCCL_WRAPPED; }

int all_gather(bj_comm* c, const void* send, void* recv, size_t bytes, hipStream_t st) {
    if (c->world == 1 && !is_rccl(c)) {
        if (send != recv && bytes) HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, st), "memcpy");
        return BJ_OK;
    }
    if (c->kind == bj_comm::LOCAL) return local_exchange(c, send, recv, bytes, false, st);
    if (c->kind == bj_comm::CALLBACK) return callback_exchange(c, BJ_XCHG_ALL_GATHER, send, recv, bytes, st);
    const Rccl& R = rccl();
    RCCL_CHECK(R, R.all_gather(send, recv, bytes / 8, ncclUint64, c->nccl, st), "ncclAllGather");
    return BJ_OK;
}

// recv block p (bytes) <- block `rank` of rank p's send (world x bytes)
int all_to_all(bj_comm* c, const void* send, void* recv, size_t bytes, hipStream_t st) {
    if (c->world == 1 && !is_rccl(c)) {
        if (send != recv && bytes) HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, st), "memcpy");
        return BJ_OK;
    }
    if (c->kind == bj_comm::LOCAL) return local_exchange(c, send, recv, bytes, true, st);
    if (c->kind == bj_comm::CALLBACK) return callback_exchange(c, BJ_XCHG_ALL_TO_ALL, send, recv, bytes, st);
    const Rccl& R = rccl();
    RCCL_CHECK(R, R.group_start(), "ncclGroupStart");
    for (int p = 0; p < c->world; p++) {
        const char* s = static_cast<const char*>(send) + (size_t)p * bytes;
        char* d = static_cast<char*>(recv) + (size_t)p * bytes;
        RCCL_CHECK(R, R.send(s, bytes / 8, ncclUint64, p, c->nccl, st), "ncclSend");
        RCCL_CHECK(R, R.recv(d, bytes / 8, ncclUint64, p, c->nccl, st), "ncclRecv");
    }
    RCCL_CHECK(R, R.group_end(), "ncclGroupEnd");
    return BJ_OK;
}

// ------------------------------------------------------------------ column pipeline plan
bool is_pow2(uint64_t x) { return x && !(x & (x - 1)); }

uint32_t log2u(uint64_t x) {
    uint32_t l = 0;
    while ((1ull << l) < x) l++;
    return l;
}

// BJ_LEAVES_DEFER=d (an experiment knob, bj_internal.hpp; tools/shard_compute_probe.py): chunk
// k's leaves are issued after chunk k + d's LDE instead of right after its own (d = 0), so fewer
// LDE -> leaf switches happen on the compute stream; larger d needs the later chunks' exchanges
// earlier.
size_t leaves_defer() { return (size_t)bj::knobs().leaves_defer; }

// Chunks per leaf grid (BJ_LEAVES_GROUP, an experiment knob; 1 in production).  Two chunks per
// grid halve the LDE -> leaves switches while every chunk's LDE still waits only for its own
// arrival, but measured 0.1-0.7 ms per rank slower at C3 G = 4 and 8 with the exchange stubbed
// (profiles/r6c_group_*.log), so each chunk keeps its own grid.
size_t leaves_group() {
    const uint64_t g = bj::knobs().leaves_group;
    return g ? (size_t)g : 1;
}

struct Run {
    uint32_t lo, global, count;  // local first row, global first column, columns
    uint32_t c0, c1;             // the chunk's global column range
};

// The column deal (bj_sharded_columns; the CPU model of it is tests/sharded_model.py): chunk k is
// G * c_k consecutive columns, rank P holding the P-th run of c_k, u = 8/gcd(8, G): c = u, u,
// then each chunk 3/2 of the previous (G <= 4) or twice it (G >= 8), rounded down to u but at
// least u more, capped at 32 rounded to u.  One chunk (contiguous ownership) when C/G is not a
// multiple of u, for a hasher without column continuation, or at G = 1 (nothing to overlap).
// The growth keeps each chunk's exchange behind the previous chunk's compute and the last
// chunk, whose compute follows the last arrival, small: at G <= 4 the all-gather moves ~0.5 ms
// per own column at 64 GB/s per xGMI link against ~0.73 ms of compute (C3), so doubling left the
// final 32-column chunk's transfer exposed; at G = 8 the fold halves the bytes and 7 links carry
// them.
std::vector<Run> column_runs(uint32_t n_cols, uint32_t world, uint32_t rank, int hasher) {
    const uint32_t cpr = n_cols / world;
    uint32_t gcd = 8, w = world;
    while (w) {
        uint32_t t = gcd % w;
        gcd = w;
        w = t;
    }
    const uint32_t unit = 8 / gcd;
    const bool partial = hasher == BJ_HASHER_POSEIDON2 || hasher == BJ_HASHER_BLAKE2S;
    std::vector<Run> runs;
    if (world == 1 || cpr % unit != 0 || !partial) {
        runs.push_back({0, rank * cpr, cpr, 0, n_cols});
        return runs;
    }
    const uint32_t max_cols = std::max(unit, 32 / unit * unit);
    uint32_t done = 0, b = unit;
    while (done < cpr) {
        const uint32_t take = std::min(b, cpr - done);
        runs.push_back({done, done * world + rank * take, take, done * world, (done + take) * world});
        done += take;
        if (runs.size() >= 2) b = std::min(world <= 4 ? std::max(b + unit, b * 3 / 2 / unit * unit) : 2 * b, max_cols);
    }
    return runs;
}

// Stream-ordered workspace, freed on the stream at scope exit.
struct Workspace {
    hipStream_t st;
    std::vector<void*> ptrs;
    explicit Workspace(hipStream_t s) : st(s) {}
    hipError_t alloc(uint64_t** p, size_t elems) {
        hipError_t e = bj::pool_alloc(reinterpret_cast<void**>(p), elems * 8, st);
        if (e == hipSuccess) ptrs.push_back(*p);
        return e;
    }
    ~Workspace() {
        for (void* p : ptrs) (void)hipFreeAsync(p, st);
    }
};

struct Events {
    std::vector<hipEvent_t> ev;
    hipError_t make(size_t n) {
        for (size_t i = 0; i < n; i++) {
            hipEvent_t e;
            hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
            if (r != hipSuccess) return r;
            ev.push_back(e);
        }
        return hipSuccess;
    }
    ~Events() {
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    }
};

// Error paths of a collective.  GroupAbort (armed from the first line): unless the call
// completes, an in-process group is aborted so its peers fail instead of blocking in a barrier
// (a rank that rejects its arguments aborts them too).  XsJoin (declared after the workspace,
// so it runs before the workspace frees on the compute stream): unless the call completes, the
// compute stream first waits for everything already queued on the exchange stream.
struct GroupAbort {
    bj_comm* c;
    bool ok = false;
    explicit GroupAbort(bj_comm* c_) : c(c_) {}
    ~GroupAbort() {
        if (!ok && c && c->kind == bj_comm::LOCAL) c->group->abort();
    }
};
struct XsJoin {
    hipStream_t st, xs;
    bool ok = false;
    XsJoin(hipStream_t st_, hipStream_t xs_) : st(st_), xs(xs_) {}
    ~XsJoin() {
        if (ok || !xs) return;
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) {
            if (hipEventRecord(e, xs) == hipSuccess) (void)hipStreamWaitEvent(st, e, 0);
            (void)hipEventDestroy(e);
        } else {
            (void)hipStreamSynchronize(xs);
        }
    }
};

int nodes_for(int hasher, const uint64_t* leaves, size_t n, uint32_t cap, uint64_t* nodes, void* st) {
    switch (hasher) {
        case BJ_HASHER_POSEIDON2: return bj_merkle_nodes_d(leaves, n, cap, nodes, st);
        case BJ_HASHER_BLAKE2S: return bj_blake2s_nodes_d(leaves, n, cap, nodes, st);
        default: return bj_keccak256_nodes_d(leaves, n, cap, nodes, st);
    }
}

}  // namespace

extern "C" {

int bj_comm_rccl_unique_id(uint8_t* id_out128) {
    if (!id_out128) return err(BJ_EINVAL, "null id buffer");
    const Rccl& R = rccl();
    if (!R.ok) return err(BJ_EHIP, R.why);
    ncclUniqueId id;
    RCCL_CHECK(R, R.get_unique_id(&id), "ncclGetUniqueId");
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(id_out128, &id, sizeof(id));
    return BJ_OK;
}

int bj_comm_init_rccl(const uint8_t* id128, int world, int rank, bj_comm** out) {
    if (!id128 || !out) return err(BJ_EINVAL, "null argument");
    if (world < 1 || !is_pow2((uint64_t)world) || rank < 0 || rank >= world)
        return err(BJ_EINVAL, "world must be a power of two and 0 <= rank < world");
    const Rccl& R = rccl();
    if (!R.ok) return err(BJ_EHIP, R.why);
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof(id));
    ncclComm_t comm = nullptr;
    RCCL_CHECK(R, R.init_rank(&comm, world, id, rank), "ncclCommInitRank");
    bj_comm* c = new bj_comm();
    (void)hipGetDevice(&c->device);
    c->kind = bj_comm::RCCL_OWNED;
    c->world = world;
    c->rank = rank;
    c->nccl = comm;
    *out = c;
    return BJ_OK;
}

int bj_comm_wrap_rccl(void* nccl_comm, int world, int rank, bj_comm** out) {
    if (!nccl_comm || !out) return err(BJ_EINVAL, "null argument");
    if (world < 1 || !is_pow2((uint64_t)world) || rank < 0 || rank >= world)
        return err(BJ_EINVAL, "world must be a power of two and 0 <= rank < world");
    const Rccl& R = rccl();
    if (!R.ok) return err(BJ_EHIP, R.why);
    bj_comm* c = new bj_comm();
    (void)hipGetDevice(&c->device);
    c->kind = bj_comm::RCCL_WRAPPED;
    c->world = world;
    c->rank = rank;
    c->nccl = static_cast<ncclComm_t>(nccl_comm);
    *out = c;
    return BJ_OK;
}

int bj_comm_local_group_create(int world, void** group_out) {
    if (!group_out) return err(BJ_EINVAL, "null argument");
    if (world < 1 || !is_pow2((uint64_t)world) || world > 64) return err(BJ_EINVAL, "world must be a power of two <= 64");
    LocalGroup* g = new LocalGroup();
    g->world = world;
    g->slot.assign(world, nullptr);
    for (int i = 0; i < 2 * world; i++) {
        hipEvent_t e;
        hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
        if (r != hipSuccess) {
            for (hipEvent_t x : g->ready) (void)hipEventDestroy(x);
            for (hipEvent_t x : g->done) (void)hipEventDestroy(x);
            delete g;
            return err(BJ_EHIP, std::string("hipEventCreate: ") + hipGetErrorString(r));
        }
        (i < world ? g->ready : g->done).push_back(e);
    }
    *group_out = g;
    return BJ_OK;
}

int bj_comm_local_group_destroy(void* group) {
    LocalGroup* g = static_cast<LocalGroup*>(group);
    if (!g) return BJ_OK;
    for (hipEvent_t e : g->ready) (void)hipEventDestroy(e);
    for (hipEvent_t e : g->done) (void)hipEventDestroy(e);
    delete g;
    return BJ_OK;
}

int bj_comm_init_local(void* group, int rank, bj_comm** out) {
    LocalGroup* g = static_cast<LocalGroup*>(group);
    if (!g || !out) return err(BJ_EINVAL, "null argument");
    if (rank < 0 || rank >= g->world) return err(BJ_EINVAL, "rank out of range");
    bj_comm* c = new bj_comm();
    (void)hipGetDevice(&c->device);
    c->kind = bj_comm::LOCAL;
    c->world = g->world;
    c->rank = rank;
    c->group = g;
    *out = c;
    return BJ_OK;
}

int bj_comm_init_callback(int world, int rank, bj_exchange_fn fn, void* user, int host_staged, bj_comm** out) {
    if (!fn || !out) return err(BJ_EINVAL, "null argument");
    if (world < 1 || !is_pow2((uint64_t)world) || rank < 0 || rank >= world)
        return err(BJ_EINVAL, "world must be a power of two and 0 <= rank < world");
    bj_comm* c = new bj_comm();
    (void)hipGetDevice(&c->device);
    c->kind = bj_comm::CALLBACK;
    c->world = world;
    c->rank = rank;
    c->fn = fn;
    c->user = user;
    c->host_staged = host_staged ? 1 : 0;
    *out = c;
    return BJ_OK;
}

int bj_comm_set_timing(bj_comm* c, int on) {
    if (!c) return err(BJ_EINVAL, "null communicator");
    c->timing = on != 0;
    return BJ_OK;
}

int bj_comm_phase_ms(bj_comm* c, float* ms_out4, int* calls_out) {
    if (!c || !ms_out4) return err(BJ_EINVAL, "null argument");
    fold_intervals(c, true);
    int rc = BJ_OK;
    if (!c->timing_error.empty()) {
        rc = err(BJ_EHIP, c->timing_error);
        c->timing_error.clear();
    }
    for (int i = 0; i < 4; i++) {
        ms_out4[i] = c->folded_ms[i];
        c->folded_ms[i] = 0;
    }
    if (calls_out) *calls_out = c->timed_calls;
    c->timed_calls = 0;
    return rc;
}

int bj_comm_exchange_d(bj_comm* c, int kind, const void* send, void* recv, size_t bytes, void* stream) {
    if (!c) return err(BJ_EINVAL, "null communicator");
    if (kind != BJ_XCHG_ALL_GATHER && kind != BJ_XCHG_ALL_TO_ALL) return err(BJ_EINVAL, "unknown exchange kind");
    if (bytes % 8) return err(BJ_EINVAL, "bytes must be a multiple of 8");
    if (bytes && (!send || !recv)) return err(BJ_EINVAL, "null buffer");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    return kind == BJ_XCHG_ALL_GATHER ? all_gather(c, send, recv, bytes, st) : all_to_all(c, send, recv, bytes, st);
}

int bj_comm_info(bj_comm* c, bj_comm_info_t* out) {
    if (!c || !out) return err(BJ_EINVAL, "null argument");
    std::memset(out, 0, sizeof(*out));
    out->world = c->world;
    out->rank = c->rank;
    out->transport_count = c->world;
    out->transport_rank = c->rank;
    out->device = c->device;
    if (is_rccl(c)) {
        out->kind = BJ_COMM_RCCL;
        const Rccl& R = rccl();
        if (!R.comm_count || !R.comm_user_rank || !R.comm_cu_device)
            return err(BJ_EHIP, "librccl.so.1 does not export ncclCommCount / ncclCommUserRank / ncclCommCuDevice");
        RCCL_CHECK(R, R.comm_count(c->nccl, &out->transport_count), "ncclCommCount");
        RCCL_CHECK(R, R.comm_user_rank(c->nccl, &out->transport_rank), "ncclCommUserRank");
        RCCL_CHECK(R, R.comm_cu_device(c->nccl, &out->device), "ncclCommCuDevice");
    } else {
        out->kind = c->kind == bj_comm::LOCAL ? BJ_COMM_LOCAL : BJ_COMM_CALLBACK;
    }
    // the bus id names the physical device; a device number this process cannot open (a stand-in
    // transport's) leaves it empty
    if (hipDeviceGetPCIBusId(out->pci_bus_id, (int)sizeof(out->pci_bus_id) - 1, out->device) != hipSuccess) {
        out->pci_bus_id[0] = 0;
        (void)hipGetLastError();
    }
    if (gethostname(out->host, sizeof(out->host) - 1) != 0) out->host[0] = 0;
    return BJ_OK;
}

int bj_comm_check_world(bj_comm* c, bj_comm_info_t* all_out, void* stream) {
    if (!c || !all_out) return err(BJ_EINVAL, "null argument");
    static_assert(sizeof(bj_comm_info_t) == 128, "bj_comm_info_t is 128 bytes");
    // every rank enters the gather, also one whose own record failed: it sends a
    // record marked invalid, so its peers fail with the same BJ_EINVAL instead of waiting in the
    // collective for a rank that returned early
    bj_comm_info_t mine;
    const int info_rc = bj_comm_info(c, &mine);
    std::string info_err;
    if (info_rc != BJ_OK) {
        info_err = bj_last_error();
        std::memset(&mine, 0, sizeof(mine));
        mine.kind = BJ_COMM_INVALID;
        mine.world = c->world;
        mine.rank = c->rank;
        mine.transport_count = c->world;
        mine.transport_rank = c->rank;
        mine.reserved[0] = info_rc;
        if (gethostname(mine.host, sizeof(mine.host) - 1) != 0) mine.host[0] = 0;
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const size_t rec = sizeof(bj_comm_info_t);
    void* dev = nullptr;
    // the one local failure that cannot enter the gather (no buffer to gather into)
    HIP_CHECK(hipMalloc(&dev, rec * (c->world + 1)), "hipMalloc");
    char* send = static_cast<char*>(dev) + rec * c->world;
    // a failed copy still enters the gather: the peers then see a slot that does not match
    hipError_t e = hipMemcpyAsync(send, &mine, rec, hipMemcpyHostToDevice, st);
    int rc = all_gather(c, send, dev, rec, st);
    if (rc == BJ_OK) {
        const hipError_t e2 = hipMemcpyAsync(all_out, dev, rec * c->world, hipMemcpyDeviceToHost, st);
        const hipError_t e3 = hipStreamSynchronize(st);
        if (e == hipSuccess) e = e2 != hipSuccess ? e2 : e3;
    }
    (void)hipFree(dev);
    if (rc) return rc;
    if (e != hipSuccess) return err(BJ_EHIP, std::string("bj_comm_check_world: ") + hipGetErrorString(e));
    for (int p = 0; p < c->world; p++)
        if (all_out[p].kind == BJ_COMM_INVALID)
            return err(BJ_EINVAL, "bj_comm_check_world: rank " + std::to_string(all_out[p].rank) +
                                      " could not read its transport record (code " +
                                      std::to_string(all_out[p].reserved[0]) + ")" +
                                      (p == c->rank && !info_err.empty() ? ": " + info_err : std::string()));
    // what the transport saw: every rank in its own slot, the transport's count and rank equal to
    // the communicator's; an RCCL world with one device per rank (the local and callback
    // transports may share a device by design: ranks as threads, a rehearsal over gloo)
    for (int p = 0; p < c->world; p++) {
        const bj_comm_info_t& r = all_out[p];
        if (r.world != c->world || r.rank != p || r.transport_count != c->world || r.transport_rank != p)
            return err(BJ_EINVAL, "bj_comm_check_world: slot " + std::to_string(p) + " holds rank " +
                                      std::to_string(r.rank) + " of " + std::to_string(r.world) + ", transport rank " +
                                      std::to_string(r.transport_rank) + " of " + std::to_string(r.transport_count) +
                                      " (expected rank " + std::to_string(p) + " of " + std::to_string(c->world) + ")");
    }
    if (mine.kind == BJ_COMM_RCCL) {
        for (int p = 0; p < c->world; p++)
            for (int q = 0; q < p; q++) {
                const bj_comm_info_t &a = all_out[q], &b = all_out[p];
                const bool same_host = std::strncmp(a.host, b.host, sizeof(a.host)) == 0;
                const bool same_dev = a.pci_bus_id[0] && b.pci_bus_id[0]
                                          ? std::strncmp(a.pci_bus_id, b.pci_bus_id, sizeof(a.pci_bus_id)) == 0
                                          : a.device == b.device;
                if (same_host && same_dev)
                    return err(BJ_EINVAL, "bj_comm_check_world: ranks " + std::to_string(q) + " and " +
                                              std::to_string(p) + " share device " + std::to_string(a.device) +
                                              (a.pci_bus_id[0] ? std::string(" (") + a.pci_bus_id + ")" : std::string()) +
                                              " on " + a.host);
            }
    }
    return BJ_OK;
}

int bj_comm_destroy(bj_comm* c) {
    if (!c) return BJ_OK;
    for (const bj_comm::Interval& iv : c->intervals) {
        (void)hipEventDestroy(iv.a);
        (void)hipEventDestroy(iv.b);
    }
    int rc = BJ_OK;
    if (c->xs) (void)hipStreamDestroy(c->xs);
    if (c->kind == bj_comm::RCCL_OWNED && c->nccl) {
        const Rccl& R = rccl();
        ncclResult_t e = R.destroy(c->nccl);
        if (e != ncclSuccess) rc = rccl_fail(R, e, "ncclCommDestroy");
    }
    delete c;
    return rc;
}

int bj_sharded_columns(uint32_t n_cols, uint32_t log_shards, uint32_t shard, int hasher, uint32_t* cols_out) {
    if (log_shards > 16) return err(BJ_EINVAL, "too many shards");
    const uint32_t world = 1u << log_shards;
    if (!cols_out || shard >= world || n_cols % world)
        return err(BJ_EINVAL, "need n_cols a multiple of the shard count and shard < G");
    if (hasher < BJ_HASHER_POSEIDON2 || hasher > BJ_HASHER_KECCAK256) return err(BJ_EINVAL, "unknown hasher");
    size_t j = 0;
    for (const Run& r : column_runs(n_cols, world, shard, hasher))
        for (uint32_t i = 0; i < r.count; i++) cols_out[j++] = r.global + i;
    return BJ_OK;
}

int bj_sharded_commit_d(bj_comm* comm, const uint64_t* trace_shard, size_t trace_stride, uint32_t n_cols,
                        uint32_t log_n, uint32_t log_lde, uint32_t log_commit_cosets, uint32_t cap_size, int hasher,
                        uint64_t* lde, uint64_t* leaves, uint64_t* nodes, uint64_t* cap, void* stream) {
    if (!comm) return err(BJ_EINVAL, "null communicator");
    GroupAbort abort_guard(comm);
    if (hasher < BJ_HASHER_POSEIDON2 || hasher > BJ_HASHER_KECCAK256) return err(BJ_EINVAL, "unknown hasher");
    const uint32_t world = (uint32_t)comm->world, rank = (uint32_t)comm->rank;
    const uint32_t log_g = log2u(world), log_k = log_commit_cosets;
    if (n_cols == 0 || n_cols % world) return err(BJ_EINVAL, "n_cols must be a positive multiple of the world size");
    if (log_lde == 0) return err(BJ_EINVAL, "lde degree must be > 1 (utils.rs:283)");
    if (log_k > log_lde) return err(BJ_EINVAL, "committed cosets exceed the lde degree (prover.rs:313, lde.rs:298-308)");
    if (log_n > 30 || log_g > log_n + log_k) return err(BJ_EINVAL, "more shards than committed leaves");
    if (log_g > log_k && log_g - log_k > 6) return err(BJ_EINVAL, "G / k exceeds 64");
    // m: this rank's leaves (and its share of each k-coset block of the LDE); B blocks of k cosets
    const size_t n = (size_t)1 << log_n, nk = n << log_k, m = nk >> log_g;
    const uint32_t B = 1u << (log_lde - log_k);
    // rank P's part of block j is leaf range j * G + P of the D-coset domain cut into 2^ls ranges
    const uint32_t ls = log_g + log_lde - log_k;
    if (!is_pow2(cap_size) || nk <= cap_size)
        return err(BJ_EINVAL, "need power-of-two cap_size < n * k (merkle_tree.rs:83-96)");
    const uint32_t cap_local = std::max<uint32_t>(1, cap_size / world);
    if (m <= cap_local) return err(BJ_EINVAL, "each shard needs more leaves than its cap slice");
    if (trace_stride < n) return err(BJ_EINVAL, "trace_stride < n");
    if (!trace_shard || !lde || !leaves || !nodes || !cap) return err(BJ_EINVAL, "null buffer");

    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipStream_t xs = nullptr;
    if (world > 1) BJ_CHECK(exchange_stream(comm, &xs));
    const uint32_t cpr = n_cols / world;
    // G > D: the sender folds (m < n values per column and block); else all-gather n per column
    const bool fold = log_g > log_lde;
    const uint32_t log_f = ls > log_lde ? ls - log_lde : 0;  // folding factor per transform
    const std::vector<Run> runs = column_runs(n_cols, world, rank, hasher);
    // world 1: no exchange, so no monomials need to reach memory (one run of every column)
    const bool fused = world == 1 && runs.size() == 1 && bj::lde_fused_supported(log_n);
    // G <= D, every coset committed: a rank's own columns of a chunk take the inverse tail fused
    // with the forward stages 0..12 of its cosets (bj::lde_own_shard), writing the monomials for
    // the all-gather once; only the other ranks' columns are transformed from arrived monomials
    const bool own_fused =
        world > 1 && !fold && B == 1 && bj::lde_fused_supported(log_n) && bj::knobs().lde_own_fused;
    const size_t K = runs.size();
    uint32_t max_cc = 0;
    for (const Run& r : runs) max_cc = std::max(max_cc, r.c1 - r.c0);

    Workspace ws(st);
    XsJoin xs_join(st, xs);
    uint64_t *coeffs = nullptr, *own = nullptr, *send = nullptr, *folded = nullptr, *state = nullptr, *work = nullptr;
    if (fold) {
        HIP_CHECK(ws.alloc(&own, (size_t)cpr * n), "pool_alloc");
        HIP_CHECK(ws.alloc(&send, (size_t)cpr * world * B * m), "pool_alloc");
        HIP_CHECK(ws.alloc(&folded, (size_t)B * n_cols * m), "pool_alloc");
    } else {
        HIP_CHECK(ws.alloc(&coeffs, (size_t)n_cols * n), "pool_alloc");
        if (log_f) HIP_CHECK(ws.alloc(&work, (size_t)max_cc * m), "pool_alloc");
    }
    if (K > 1) HIP_CHECK(ws.alloc(&state, m * 4), "pool_alloc");
    Events in, arrived;
    if (world > 1) {
        HIP_CHECK(in.make(K), "hipEventCreate");
        HIP_CHECK(arrived.make(K), "hipEventCreate");
    }
    std::vector<uint64_t> spm((size_t)B * world);
    // phases 0 inverse (+ fold), 1 lde, 2 leaves, 3 nodes (bj_comm_set_timing)
    if (!comm->intervals.empty()) fold_intervals(comm, false);
    PhaseTimer pt(comm, st);

    // 1. local inverse transforms (and folds), each chunk's exchange issued as soon as its
    //    part is ready
    for (size_t k = 0; k < K; k++) {
        const Run& r = runs[k];
        const uint64_t* tr = trace_shard + (size_t)r.lo * trace_stride;
        hipStream_t xst = world > 1 ? xs : st;
        if (fold) {
            // send layout per run: [block j][rank p][c][m], so block j's all-to-all is contiguous
            uint64_t* snd = send + (size_t)world * B * m * r.lo;
            uint64_t* mine = own + (size_t)r.lo * n;
            BJ_CHECK(pt.begin(0));
            // targets T = j G + p (block j, rank p) sit at snd + T r.count m: one stride
            for (uint32_t T = 0; T < B * world; T++) spm[T] = gl::pow(bj::shard_shift(log_n, log_lde, ls, T), m);
            if (bj::inverse_fold_supported(log_n, log_f, B * world)) {
                // the inverse tail folds for every target straight from registers (ntt_lde3.hip)
                BJ_CHECK(bj::inverse_fold_all(tr, r.count, trace_stride, log_n, log_f, B * world, spm.data(), mine, n,
                                              snd, m, (size_t)r.count * m, st));
            } else {
                BJ_CHECK(bj_lde_coeffs_d(tr, r.count, trace_stride, log_n, mine, n, st));
                for (uint32_t j = 0; j < B; j++)
                    HIP_CHECK(bj::launch_fold_all(snd + (size_t)j * world * r.count * m, m, (size_t)r.count * m, mine,
                                                  n, r.count, log2u(m), log_f, world, spm.data() + (size_t)j * world,
                                                  st),
                              "fold");
            }
            BJ_CHECK(pt.end());
            if (world > 1) {
                HIP_CHECK(hipEventRecord(in.ev[k], st), "hipEventRecord");
                HIP_CHECK(hipStreamWaitEvent(xs, in.ev[k], 0), "hipStreamWaitEvent");
            }
            for (uint32_t j = 0; j < B; j++)
                BJ_CHECK(all_to_all(comm, snd + (size_t)j * world * r.count * m,
                                    folded + ((size_t)j * n_cols + r.c0) * m, (size_t)r.count * m * 8, xst));
            if (world > 1) HIP_CHECK(hipEventRecord(arrived.ev[k], xs), "hipEventRecord");
        } else {
            if (fused) continue;  // the inverse runs inside the fused LDE (step 2)
            uint64_t* mine = coeffs + (size_t)r.global * n;
            BJ_CHECK(pt.begin(0));
            if (own_fused)
                BJ_CHECK(bj::lde_own_shard(tr, r.count, trace_stride, log_n, log_lde, ls, rank, mine, n,
                                           lde + (size_t)r.global * m, m, bj::LDE3_MID, st));
            else
                BJ_CHECK(bj_lde_coeffs_d(tr, r.count, trace_stride, log_n, mine, n, st));
            BJ_CHECK(pt.end());
            if (world > 1) {
                HIP_CHECK(hipEventRecord(in.ev[k], st), "hipEventRecord");
                HIP_CHECK(hipStreamWaitEvent(xs, in.ev[k], 0), "hipStreamWaitEvent");
                BJ_CHECK(all_gather(comm, mine, coeffs + (size_t)r.c0 * n, (size_t)r.count * n * 8, xs));
                HIP_CHECK(hipEventRecord(arrived.ev[k], xs), "hipEventRecord");
            }
        }
    }
    // 2. per arrived chunk: this rank's part of the committed block (block 0) of its columns'
    //    LDE, absorbed into the sponges, then its part of the other blocks (LDE only).  Chunk k's
    //    leaves follow chunk k + defer's LDE (leaves_defer(); 0 in production).
    // chunks [k0, k1) in one leaf grid: their block-0 columns are contiguous (chunk k + 1's
    // global columns follow chunk k's), so one sponge pass absorbs them
    auto absorb = [&](size_t k0, size_t k1) -> int {
        const uint32_t c0 = runs[k0].c0, cc = runs[k1 - 1].c1 - c0;
        const uint64_t* out = lde + (size_t)c0 * m;  // block 0
        const bool last = k1 == K;
        const uint64_t* cin = k0 == 0 ? nullptr : state;
        uint64_t* dst = last ? leaves : state;
        BJ_CHECK(pt.begin(2));
        if (hasher == BJ_HASHER_POSEIDON2)
            BJ_CHECK(bj_merkle_leaves_partial_d(out, cc, m, m, cin, dst, last ? 1 : 0, st));
        else if (hasher == BJ_HASHER_BLAKE2S)
            BJ_CHECK(bj_blake2s_leaves_partial_d(out, cc, m, m, c0, cin, dst, last ? 1 : 0, st));
        else
            BJ_CHECK(bj_keccak256_leaves_d(out, cc, m, m, dst, st));
        return pt.end();
    };
    // chunk k's leaves follow chunk k + defer's LDE (leaves_defer(), 0 in production), `group`
    // chunks per leaf grid (leaves_group(), 1 in production)
    const size_t defer = leaves_defer(), group = leaves_group();
    size_t absorbed = 0;
    auto absorb_ready = [&](size_t ready, bool flush) -> int {
        while (ready > absorbed && (flush || ready - absorbed >= group)) {
            const size_t hi = std::min(ready, absorbed + group);
            BJ_CHECK(absorb(absorbed, hi));
            absorbed = hi;
        }
        return BJ_OK;
    };
    for (size_t k = 0; k < K; k++) {
        const Run& r = runs[k];
        const uint32_t cc = r.c1 - r.c0;
        if (own_fused) {
            // the rank's own columns need no arrival: their last stages first
            BJ_CHECK(pt.begin(1));
            BJ_CHECK(bj::lde_own_shard(trace_shard + (size_t)r.lo * trace_stride, r.count, trace_stride, log_n,
                                       log_lde, ls, rank, coeffs + (size_t)r.global * n, n, lde + (size_t)r.global * m,
                                       m, bj::LDE3_FINAL, st));
            BJ_CHECK(pt.end());
        }
        if (world > 1) HIP_CHECK(hipStreamWaitEvent(st, arrived.ev[k], 0), "hipStreamWaitEvent");
        for (uint32_t j = 0; j < B; j++) {
            uint64_t* out = lde + ((size_t)j * n_cols + r.c0) * m;
            const uint32_t shard = j * world + rank;
            BJ_CHECK(pt.begin(1));
            if (fused) {
                // one rank, nothing to exchange: bj_lde_ex_d's three passes straight from the trace
                // (the inverse head, then the inverse tail fused with every coset's first 13 stages),
                // all B blocks at once
                if (j == 0)
                    BJ_CHECK(bj::lde_fused_blocks(trace_shard + (size_t)r.lo * trace_stride, r.count, trace_stride,
                                                  log_n, log_lde, log_k, coeffs, out, m, (size_t)n_cols * m, st));
            } else if (fold)
                BJ_CHECK(bj_lde_shard_folded_d(folded + ((size_t)j * n_cols + r.c0) * m, cc, m, log_n, log_lde, ls,
                                               shard, out, st));
            else if (own_fused) {
                // the other ranks' columns of the chunk: before and after this rank's run
                const uint32_t before = r.global - r.c0, own_end = r.global + r.count, after = r.c1 - own_end;
                if (before)
                    BJ_CHECK(bj_lde_shard_d(coeffs + (size_t)r.c0 * n, before, n, log_n, log_lde, ls, shard, work, out,
                                            st));
                if (after)
                    BJ_CHECK(bj_lde_shard_d(coeffs + (size_t)own_end * n, after, n, log_n, log_lde, ls, shard, work,
                                            lde + (size_t)own_end * m, st));
            } else
                BJ_CHECK(bj_lde_shard_d(coeffs + (size_t)r.c0 * n, cc, n, log_n, log_lde, ls, shard, work, out, st));
            BJ_CHECK(pt.end());
            if (j == 0 && k + 1 > defer) BJ_CHECK(absorb_ready(k + 1 - defer, k + 1 == K));
        }
    }
    BJ_CHECK(absorb_ready(K, true));
    // 3. this rank's subtree, then the cap
    BJ_CHECK(pt.begin(3));
    BJ_CHECK(nodes_for(hasher, leaves, m, cap_local, nodes, st));
    BJ_CHECK(pt.end());
    const uint64_t* local_cap = nodes + (m - 2 * (size_t)cap_local) * 4;
    if (cap_size >= world) {
        BJ_CHECK(all_gather(comm, local_cap, cap, (size_t)cap_local * 32, st));
    } else {
        // fewer cap digests than ranks: gather the subtree roots, hash the top levels everywhere
        uint64_t *roots = nullptr, *top = nullptr;
        HIP_CHECK(ws.alloc(&roots, (size_t)world * 4), "pool_alloc");
        HIP_CHECK(ws.alloc(&top, (size_t)(world - cap_size) * 4), "pool_alloc");
        BJ_CHECK(all_gather(comm, local_cap, roots, 32, st));
        BJ_CHECK(nodes_for(hasher, roots, world, cap_size, top, st));
        HIP_CHECK(hipMemcpyAsync(cap, top + (size_t)(world - 2 * cap_size) * 4, (size_t)cap_size * 32,
                                 hipMemcpyDeviceToDevice, st),
                  "memcpy cap");
    }
    if (comm->timing) comm->timed_calls++;
    xs_join.ok = abort_guard.ok = true;
    return BJ_OK;
}

int bj_sharded_query_h(bj_comm* comm, const uint64_t* lde, const uint64_t* leaves, const uint64_t* nodes,
                       uint32_t n_cols, uint32_t log_n, uint32_t log_lde, uint32_t log_commit_cosets, uint32_t cap_size,
                       int hasher, uint64_t idx, uint64_t* leaf_elements_h, uint64_t* leaf_hash_h, uint64_t* proof_h,
                       void* stream) {
    if (!comm) return err(BJ_EINVAL, "null communicator");
    GroupAbort abort_guard(comm);
    if (hasher < BJ_HASHER_POSEIDON2 || hasher > BJ_HASHER_KECCAK256) return err(BJ_EINVAL, "unknown hasher");
    const uint32_t world = (uint32_t)comm->world, rank = (uint32_t)comm->rank;
    const uint32_t log_g = log2u(world);
    if (log_commit_cosets > log_lde) return err(BJ_EINVAL, "committed cosets exceed the lde degree");
    if (log_n > 30 || log_g > log_n + log_commit_cosets || n_cols == 0) return err(BJ_EINVAL, "bad geometry");
    // the tree is over the first k cosets; this rank's block-0 slice (its leaves) is lde[c * m + i]
    const size_t nl = (size_t)1 << (log_n + log_commit_cosets), m = nl >> log_g;
    if (!is_pow2(cap_size) || nl <= cap_size) return err(BJ_EINVAL, "need power-of-two cap_size < n * k");
    const uint32_t cap_local = std::max<uint32_t>(1, cap_size / world);
    if (m <= cap_local) return err(BJ_EINVAL, "each shard needs more leaves than its cap slice");
    if (idx >= nl) return err(BJ_EINVAL, "tree index out of range");
    if (!lde || !leaves || !nodes || !leaf_elements_h || !leaf_hash_h || !proof_h) return err(BJ_EINVAL, "null buffer");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const uint32_t owner = (uint32_t)(idx / m);
    const size_t local = idx % m;
    const uint32_t local_depth = log2u(m) - log2u(cap_local);
    const uint32_t top_depth = cap_size < world ? log_g - log2u(cap_size) : 0;
    const size_t words = (size_t)n_cols + 4 + 4 * ((size_t)local_depth + top_depth);
    Workspace ws(st);
    uint64_t *buf = nullptr, *all = nullptr;
    HIP_CHECK(ws.alloc(&buf, words), "pool_alloc");
    HIP_CHECK(ws.alloc(&all, words * world), "pool_alloc");
    HIP_CHECK(hipMemsetAsync(buf, 0, words * 8, st), "memset");
    if (rank == owner) {
        // leaf_elements: every column's LDE value at the row (a strided gather), then the leaf
        HIP_CHECK(hipMemcpy2DAsync(buf, 8, lde + local, m * 8, 8, n_cols, hipMemcpyDeviceToDevice, st), "gather row");
        HIP_CHECK(hipMemcpyAsync(buf + n_cols, leaves + 4 * local, 32, hipMemcpyDeviceToDevice, st), "leaf");
        // siblings up the subtree (MerkleTreeWithCap::get_proof, merkle_tree.rs:462-480); node
        // level l >= 1 holds m >> l digests after the lower levels
        size_t at = local, level_off = 0, level_len = m;
        for (uint32_t l = 0; l < local_depth; l++) {
            const uint64_t* src = l == 0 ? leaves + 4 * (at ^ 1) : nodes + 4 * (level_off + (at ^ 1));
            HIP_CHECK(hipMemcpyAsync(buf + n_cols + 4 + 4 * l, src, 32, hipMemcpyDeviceToDevice, st), "sibling");
            if (l > 0) level_off += level_len;
            level_len >>= 1;
            at >>= 1;
        }
    }
    if (top_depth) {
        // cap < G: the top levels over the G subtree roots, hashed on every rank
        uint64_t *roots = nullptr, *top = nullptr;
        HIP_CHECK(ws.alloc(&roots, (size_t)world * 4), "pool_alloc");
        HIP_CHECK(ws.alloc(&top, (size_t)(world - cap_size) * 4), "pool_alloc");
        BJ_CHECK(all_gather(comm, nodes + (m - 2 * (size_t)cap_local) * 4, roots, 32, st));
        BJ_CHECK(nodes_for(hasher, roots, world, cap_size, top, st));
        size_t at = owner, level_off = 0, level_len = world;
        for (uint32_t l = 0; l < top_depth; l++) {
            const uint64_t* src = l == 0 ? roots + 4 * (at ^ 1) : top + 4 * (level_off + (at ^ 1));
            HIP_CHECK(hipMemcpyAsync(buf + n_cols + 4 + 4 * ((size_t)local_depth + l), src, 32,
                                     hipMemcpyDeviceToDevice, st),
                      "top sibling");
            if (l > 0) level_off += level_len;
            level_len >>= 1;
            at >>= 1;
        }
    }
    // every rank gets the owner's row and path (the other ranks contributed zeros)
    BJ_CHECK(all_gather(comm, buf, all, words * 8, st));
    const uint64_t* mine = all + (size_t)owner * words;
    HIP_CHECK(hipMemcpyAsync(leaf_elements_h, mine, (size_t)n_cols * 8, hipMemcpyDeviceToHost, st), "memcpy");
    HIP_CHECK(hipMemcpyAsync(leaf_hash_h, mine + n_cols, 32, hipMemcpyDeviceToHost, st), "memcpy");
    HIP_CHECK(hipMemcpyAsync(proof_h, mine + n_cols + 4, 32 * ((size_t)local_depth + top_depth), hipMemcpyDeviceToHost,
                             st),
              "memcpy");
    HIP_CHECK(hipStreamSynchronize(st), "sync");
    abort_guard.ok = true;
    return BJ_OK;
}

}  // extern "C"
