// Test infrastructure, not product: a stand-in for librccl.so.1 with RCCL's API semantics for
// ranks that are threads of one process sharing one GPU.  RCCL itself refuses two ranks on one
// device ("Duplicate GPU detected", profiles/r3j_rccl_two_ranks_one_gpu.log), so on a one-GPU
// box this is how the library's RCCL code path (collective.hip: ncclAllGather in place and not,
// grouped ncclSend/ncclRecv, all on the exchange stream) runs at world > 1 -- the calls, counts,
// offsets and peer pairing it issues are checked here, and the data they move ends up in a
// commit that c_caller compares with the oracle.
//
// Semantics followed (NCCL/RCCL documentation):
// * ncclAllGather(send, recv, count, type, comm, stream): recv[p * count ..] = rank p's send;
//   in place when send == recv + rank * count.  Every rank must pass the same count and type.
// * ncclSend / ncclRecv between ncclGroupStart / ncclGroupEnd: the i-th send from rank a to b
//   pairs with the i-th receive on b from a; both sides must name the same count and type.
// * Completion is stream-ordered on each rank's stream; a send buffer is free once the rank's
//   stream passes the collective.
// A mismatch returns ncclInvalidUsage and prints what was wrong (the test then fails).
// Built as librccl.so.1 (soname) by tests/c/Makefile; c_caller dlopens it first when
// BJ_TEST_MOCK_RCCL names it, so the product library's dlopen("librccl.so.1", RTLD_NOLOAD)
// finds it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct P2p {
    bool send;
    void* buf;
    size_t bytes;
    int peer;
};

struct Op {
    int kind = 0;  // 1 all-gather, 2 point-to-point group
    const void* send = nullptr;
    void* recv = nullptr;
    size_t bytes = 0;
    std::vector<P2p> p2p;
    hipEvent_t ready = nullptr, done = nullptr;
};

struct Group {
    int world = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    std::vector<Op> ops;
    bool bad = false;

    // every rank reaches the same step
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t g = generation;
        if (++arrived == world) {
            arrived = 0;
            generation++;
            cv.notify_all();
            return;
        }
        cv.wait(lk, [&] { return generation != g; });
    }
};

std::mutex g_mu;
std::map<std::string, Group*>* g_groups = new std::map<std::string, Group*>();
uint64_t g_next = 1;

size_t type_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

thread_local int t_depth = 0;
thread_local std::vector<P2p> t_pending;
thread_local ncclComm_t t_comm = nullptr;
thread_local hipStream_t t_stream = nullptr;

}  // namespace

struct ncclComm {
    Group* g;
    int rank;
    int device;  // ncclCommCuDevice: the calling thread's device, or the rank with MOCK_RCCL_FAKE_DEVICES=1
};

namespace {

// Publish this rank's op, wait for all ranks, queue this rank's copies on its stream, then make
// every rank's stream wait until all ranks have queued their reads.
ncclResult_t run(ncclComm_t c, Op op, hipStream_t st) {
    Group& g = *c->g;
    const int me = c->rank;
    if (hipEventCreateWithFlags(&op.ready, hipEventDisableTiming) != hipSuccess) return ncclUnhandledCudaError;
    if (hipEventCreateWithFlags(&op.done, hipEventDisableTiming) != hipSuccess) return ncclUnhandledCudaError;
    if (hipEventRecord(op.ready, st) != hipSuccess) return ncclUnhandledCudaError;
    {
        std::lock_guard<std::mutex> lk(g.mu);
        g.ops[me] = op;
    }
    g.barrier();
    bool ok = true;
    const Op& mine = g.ops[me];
    for (int p = 0; p < g.world; p++) {
        const Op& o = g.ops[p];
        if (o.kind != mine.kind) {
            fprintf(stderr, "mock rccl: rank %d runs op kind %d while rank %d runs %d\n", me, mine.kind, p, o.kind);
            ok = false;
        }
    }
    if (ok && mine.kind == 1) {
        for (int p = 0; p < g.world; p++) {
            const Op& o = g.ops[p];
            if (o.bytes != mine.bytes) {
                fprintf(stderr, "mock rccl: all-gather of %zu bytes on rank %d, %zu on rank %d\n", mine.bytes, me,
                        o.bytes, p);
                ok = false;
                continue;
            }
            (void)hipStreamWaitEvent(st, o.ready, 0);
            char* dst = static_cast<char*>(mine.recv) + (size_t)p * mine.bytes;
            if (p == me && mine.send == dst) continue;  // in place
            if (mine.bytes) (void)hipMemcpyAsync(dst, o.send, mine.bytes, hipMemcpyDeviceToDevice, st);
        }
    } else if (ok && mine.kind == 2) {
        // the i-th receive from p pairs with p's i-th send to me
        std::map<int, int> nth;
        for (const P2p& r : mine.p2p) {
            if (r.send) continue;
            const int p = r.peer, i = nth[p]++;
            const P2p* s = nullptr;
            int seen = 0;
            for (const P2p& x : g.ops[p].p2p)
                if (x.send && x.peer == me && seen++ == i) { s = &x; break; }
            if (!s) {
                fprintf(stderr, "mock rccl: rank %d's receive #%d from %d has no matching send\n", me, i, p);
                ok = false;
                continue;
            }
            if (s->bytes != r.bytes) {
                fprintf(stderr, "mock rccl: rank %d receives %zu bytes from %d, which sends %zu\n", me, r.bytes, p,
                        s->bytes);
                ok = false;
                continue;
            }
            (void)hipStreamWaitEvent(st, g.ops[p].ready, 0);
            if (r.bytes) (void)hipMemcpyAsync(r.buf, s->buf, r.bytes, hipMemcpyDeviceToDevice, st);
        }
        // every send must be received
        std::map<int, int> sends_to;
        for (const P2p& s : mine.p2p)
            if (s.send) sends_to[s.peer]++;
        for (auto& kv : sends_to) {
            int recvs = 0;
            for (const P2p& x : g.ops[kv.first].p2p)
                if (!x.send && x.peer == me) recvs++;
            if (recvs != kv.second) {
                fprintf(stderr, "mock rccl: rank %d sends %d to %d, which receives %d\n", me, kv.second, kv.first, recvs);
                ok = false;
            }
        }
    }
    (void)hipEventRecord(mine.done, st);
    if (!ok) {
        std::lock_guard<std::mutex> lk(g.mu);
        g.bad = true;
    }
    g.barrier();
    for (int p = 0; p < g.world; p++) (void)hipStreamWaitEvent(st, g.ops[p].done, 0);
    const bool bad = g.bad;
    g.barrier();  // every wait is queued before anyone frees or re-publishes
    (void)hipEventDestroy(g.ops[me].ready);
    (void)hipEventDestroy(g.ops[me].done);
    if (bad) {
        g.barrier();
        std::lock_guard<std::mutex> lk(g.mu);
        g.bad = false;
        return ncclInvalidUsage;
    }
    return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    std::lock_guard<std::mutex> lk(g_mu);
    std::memset(id, 0, sizeof(*id));
    snprintf(id->internal, sizeof(id->internal), "mock-rccl-%llu", (unsigned long long)g_next++);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    std::string key(id.internal, strnlen(id.internal, sizeof(id.internal)));
    Group* g;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_groups->find(key);
        if (it == g_groups->end()) {
            g = new Group();
            g->world = nranks;
            g->ops.resize(nranks);
            (*g_groups)[key] = g;
        } else {
            g = it->second;
        }
    }
    if (g->world != nranks) return ncclInvalidUsage;
    g->barrier();  // ncclCommInitRank is collective
    // The ranks of this stand-in are threads on one GPU, so ncclCommCuDevice reports that device
    // for all of them (what bj_comm_check_world must reject as a duplicated device); with
    // MOCK_RCCL_FAKE_DEVICES=1 at init it reports device = rank instead, a world of distinct
    // devices as a real one-process-per-GPU run has.
    int dev = 0;
    (void)hipGetDevice(&dev);
    const char* fake = getenv("MOCK_RCCL_FAKE_DEVICES");
    if (fake && fake[0] == '1') dev = rank;
    *comm = new ncclComm{g, rank, dev};
    return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
    if (!comm || !count) return ncclInvalidArgument;
    *count = comm->g->world;
    return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
    if (!comm || !rank) return ncclInvalidArgument;
    *rank = comm->rank;
    return ncclSuccess;
}

ncclResult_t ncclCommCuDevice(const ncclComm_t comm, int* device) {
    if (!comm || !device) return ncclInvalidArgument;
    // MOCK_RCCL_FAIL_INFO_RANK=r: rank r cannot report its device (bj_comm_check_world must still
    // enter the gather, and every rank must get the same rejection)
    const char* f = getenv("MOCK_RCCL_FAIL_INFO_RANK");
    if (f && atoi(f) == comm->rank) return ncclInternalError;
    *device = comm->device;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    delete comm;
    return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype,
                           ncclComm_t comm, hipStream_t stream) {
    const size_t ts = type_size(datatype);
    if (!comm || !ts) return ncclInvalidArgument;
    if (t_depth) {
        fprintf(stderr, "mock rccl: all-gather inside a group is not used by this library\n");
        return ncclInvalidUsage;
    }
    Op op;
    op.kind = 1;
    op.send = sendbuff;
    op.recv = recvbuff;
    op.bytes = sendcount * ts;
    return run(comm, op, stream);
}

ncclResult_t ncclGroupStart() {
    t_depth++;
    return ncclSuccess;
}

static ncclResult_t p2p(bool send, void* buf, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                        hipStream_t stream) {
    const size_t ts = type_size(datatype);
    if (!comm || !ts || peer < 0 || peer >= comm->g->world) return ncclInvalidArgument;
    if (!t_depth) {
        // outside a group: a group of one
        t_pending.assign(1, P2p{send, buf, count * ts, peer});
        Op op;
        op.kind = 2;
        op.p2p = t_pending;
        t_pending.clear();
        return run(comm, op, stream);
    }
    if ((t_comm && t_comm != comm) || (t_stream && t_stream != stream)) {
        fprintf(stderr, "mock rccl: one group spans two communicators or streams\n");
        return ncclInvalidUsage;
    }
    t_comm = comm;
    t_stream = stream;
    t_pending.push_back(P2p{send, buf, count * ts, peer});
    return ncclSuccess;
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    return p2p(true, const_cast<void*>(sendbuff), count, datatype, peer, comm, stream);
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    return p2p(false, recvbuff, count, datatype, peer, comm, stream);
}

ncclResult_t ncclGroupEnd() {
    if (t_depth <= 0) return ncclInvalidUsage;
    if (--t_depth) return ncclSuccess;
    if (t_pending.empty()) return ncclSuccess;
    Op op;
    op.kind = 2;
    op.p2p = t_pending;
    ncclComm_t c = t_comm;
    hipStream_t st = t_stream;
    t_pending.clear();
    t_comm = nullptr;
    t_stream = nullptr;
    return run(c, op, st);
}

const char* ncclGetErrorString(ncclResult_t result) {
    switch (result) {
        case ncclSuccess: return "no error (mock rccl)";
        case ncclInvalidArgument: return "invalid argument (mock rccl)";
        case ncclInvalidUsage: return "invalid usage (mock rccl)";
        default: return "error (mock rccl)";
    }
}

}  // extern "C"
