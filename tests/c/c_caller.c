/*
 * c_caller.c -- a plain-C caller of the C ABI (include/boojum_mi355x.h), as a Rust prover's
 * FFI would bind it: host Vecs in, no torch, no Python.  Test infrastructure (it also links the
 * CPU oracle, oracle/liboracle.so, as the checker); built by tests/c/Makefile, run by
 * tests/test_c_caller.py on the GPU box.
 *
 * Checks, each against the oracle restatement of the reference:
 *   1. the per-column FFT seam the reference calls from rayon workers
 *      (PrimeFieldLikeVectorized, field/traits/field_like.rs:111-162; fft/mod.rs:398-411,
 *      464-491): twiddles, ifft_natural_to_natural, fft_natural_to_bitreversed with a coset,
 *      distribute_powers -- called concurrently from T threads on distinct columns, three rounds
 *      (an earlier null-stream version of the seam returned a stale column about every other run);
 *   2. TreeHasher leaf/node (cs/oracle/mod.rs:141-168);
 *   3. the whole witness commit through the host-buffer entry point bj_lde_commit_h, and
 *      through the device-resident one-call bj_lde_commit_ex_d (flags 0) on hipMalloc buffers
 *      (prover.rs:313-353): LDE at D, tree over the first k cosets (subset_for_degree,
 *      prover.rs:325-347); LDE, leaves, nodes and cap bit-exact;
 *   4. the collective sharded commit (bj_sharded_commit_d) at G = 2, 4, 8 ranks as threads on
 *      one device, with the same D / k split;
 *   5. the error contract: a violated precondition (fft/mod.rs:399-402 asserts a power-of-two
 *      length) returns BJ_EINVAL with a message, and the library keeps working;
 *   6. (c_caller release) commits of three sizes, then bj_release_tables + bj_release_workspace
 *      return the device memory to its baseline.
 *
 * usage: c_caller LOG_N N_COLS LOG_LDE CAP THREADS [LOG_K]   prints "c_caller ok ..." on success
 *        c_caller release                                    prints "c_caller release ok ..." 
 *        (LOG_K = log2 of the committed cosets, default LOG_LDE)
 */
#include <pthread.h>
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "boojum_mi355x.h"
#include <hip/hip_runtime_api.h> /* device buffers for the *_d family (a Rust host: hip-sys) */

typedef uint64_t u64;
#define GL_P 0xFFFFFFFF00000001ull

/* oracle/boojum_oracle.c (the checker) */
u64 bjo_domain_generator(uint32_t log_n);
u64 bjo_gl_pow(u64 b, u64 e);
void bjo_precompute_twiddles(uint32_t log_n, int inverse, u64* out);
void bjo_distribute_powers(u64* a, size_t n, u64 element);
void bjo_fft_natural_to_bitreversed(u64* a, size_t n, u64 coset, const u64* tw);
void bjo_ifft_natural_to_natural(u64* a, size_t n, u64 coset, const u64* inv_tw);
void bjo_hash_into_leaf(const u64* elems, size_t count, u64* out4);
void bjo_hash_into_node(const u64* l, const u64* r, u64* out4);
int bjo_lde_commit_subset(u64* trace, uint32_t n_cols, uint32_t log_n, uint32_t log_d, uint32_t log_k,
                          uint32_t cap_size, u64* lde, u64* leaves, u64* nodes, u64* cap_out, int threads);

static int failures = 0;
#define CHECK(cond, ...)                      \
    do {                                      \
        if (!(cond)) {                        \
            fprintf(stderr, "FAIL: " __VA_ARGS__); \
            fprintf(stderr, "\n");            \
            failures++;                       \
        }                                     \
    } while (0)

/* SURVEY 8(d) synthetic trace: splitmix64(seed = 42 + c*n + r), reduced below p */
static u64 splitmix64(u64 x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static u64 canon(u64 x) { return x >= GL_P ? x - GL_P : x; }

static int eq_canon(const u64* a, const u64* b, size_t n, size_t* where) {
    for (size_t i = 0; i < n; i++)
        if (canon(a[i]) != canon(b[i])) {
            *where = i;
            return 0;
        }
    return 1;
}

static void* xmalloc(size_t bytes) {
    void* p = malloc(bytes ? bytes : 1);
    if (!p) {
        fprintf(stderr, "out of host memory\n");
        exit(2);
    }
    return p;
}

/* ------------------------------------------------ 1. concurrent per-column FFT seam */

typedef struct {
    u64* cols;          /* n_cols x n, in place */
    size_t n;
    uint32_t first, count;
    u64 coset;
    int rc;
} seam_job_t;

/* utils.rs:295-304,363-379: one column per call from a worker thread, in place */
static void* seam_worker(void* p) {
    seam_job_t* j = (seam_job_t*)p;
    j->rc = 0;
    for (uint32_t c = j->first; c < j->first + j->count && j->rc == 0; c++) {
        u64* col = j->cols + (size_t)c * j->n;
        j->rc = bj_ifft_natural_to_natural_h(col, j->n, 1);
        if (j->rc == 0) j->rc = bj_fft_natural_to_bitreversed_h(col, j->n, j->coset);
    }
    return NULL;
}

static void check_fft_seam(uint32_t log_n, uint32_t n_cols, int threads) {
    size_t n = (size_t)1 << log_n;
    u64* tw = xmalloc(8 * (n / 2));
    u64* tw_ref = xmalloc(8 * (n / 2));
    for (int inv = 0; inv < 2; inv++) {
        CHECK(bj_precompute_twiddles_h(log_n, inv, tw) == BJ_OK, "bj_precompute_twiddles_h: %s", bj_last_error());
        bjo_precompute_twiddles(log_n, inv, tw_ref);
        size_t w = 0;
        CHECK(eq_canon(tw, tw_ref, n / 2, &w), "twiddles (inverse=%d) differ at %zu", inv, w);
    }
    u64* cols = xmalloc(8 * n * n_cols);
    u64* ref = xmalloc(8 * n * n_cols);
    for (size_t i = 0; i < n * n_cols; i++) cols[i] = ref[i] = splitmix64(7 + i); /* non-canonical inputs too */
    /* the LDE's coset for i = 1 of D = 2: 7 * w_{2n} (utils.rs:334-347) */
    u64 coset = canon((u64)(((unsigned __int128)7 * bjo_gl_pow(bjo_domain_generator(log_n + 1), 1)) % GL_P));
    pthread_t* th = xmalloc(sizeof(pthread_t) * threads);
    seam_job_t* jobs = xmalloc(sizeof(seam_job_t) * threads);
    uint32_t per = (n_cols + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        uint32_t first = t * per < n_cols ? t * per : n_cols;
        uint32_t count = first + per <= n_cols ? per : n_cols - first;
        jobs[t] = (seam_job_t){cols, n, first, count, coset, 0};
        pthread_create(&th[t], NULL, seam_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        CHECK(jobs[t].rc == BJ_OK, "seam thread %d: rc %d (%s)", t, jobs[t].rc, bj_last_error());
    }
    bjo_precompute_twiddles(log_n, 1, tw_ref);
    bjo_precompute_twiddles(log_n, 0, tw);
    for (uint32_t c = 0; c < n_cols; c++) {
        bjo_ifft_natural_to_natural(ref + (size_t)c * n, n, 1, tw_ref);
        bjo_fft_natural_to_bitreversed(ref + (size_t)c * n, n, coset, tw);
    }
    size_t w = 0;
    CHECK(eq_canon(cols, ref, n * n_cols, &w), "concurrent ifft+fft seam differs at %zu", w);
    /* distribute_powers (fft/mod.rs:308-317) */
    memcpy(cols, ref, 8 * n);
    CHECK(bj_distribute_powers_h(cols, n, coset) == BJ_OK, "bj_distribute_powers_h: %s", bj_last_error());
    bjo_distribute_powers(ref, n, coset);
    CHECK(eq_canon(cols, ref, n, &w), "distribute_powers differs at %zu", w);
    free(th); free(jobs); free(cols); free(ref); free(tw); free(tw_ref);
}

/* -------------------------------------------------------------- 2. TreeHasher */

static void check_tree_hasher(void) {
    u64 elems[19], got[4], want[4];
    for (int i = 0; i < 19; i++) elems[i] = splitmix64(100 + i);
    for (size_t len = 0; len <= 19; len++) {  /* every sponge padding case up to 2 blocks + 3 */
        CHECK(bj_hash_into_leaf_h(elems, len, got) == BJ_OK, "bj_hash_into_leaf_h: %s", bj_last_error());
        bjo_hash_into_leaf(elems, len, want);
        size_t w = 0;
        CHECK(eq_canon(got, want, 4, &w), "leaf of %zu elements differs", len);
    }
    CHECK(bj_hash_into_node_h(elems, elems + 4, got) == BJ_OK, "bj_hash_into_node_h: %s", bj_last_error());
    bjo_hash_into_node(elems, elems + 4, want);
    size_t w = 0;
    CHECK(eq_canon(got, want, 4, &w), "node hash differs");
}

/* ------------------------------------------------------ 3. whole witness commit */

static void check_commit(uint32_t log_n, uint32_t n_cols, uint32_t log_lde, uint32_t log_k, uint32_t cap, int threads,
                         u64* cap_out) {
    size_t n = (size_t)1 << log_n, nd = n << log_lde, nl = n << log_k, n_nodes = nl - cap;
    u64* trace = xmalloc(8 * n * n_cols);
    for (uint32_t c = 0; c < n_cols; c++)
        for (size_t r = 0; r < n; r++) trace[(size_t)c * n + r] = canon(splitmix64(42 + (u64)c * n + r));
    u64* lde = xmalloc(8 * nd * n_cols), *leaves = xmalloc(32 * nl), *nodes = xmalloc(32 * n_nodes);
    /* the trace into HBM for the device-resident call below, now: the oracle transforms its
     * input in place */
    u64 *d_tr = NULL, *d_scr = NULL, *d_lde = NULL, *d_lv = NULL, *d_nd = NULL;
    int ok = hipMalloc((void**)&d_tr, 8 * n * n_cols) == hipSuccess &&
             hipMemcpy(d_tr, trace, 8 * n * n_cols, hipMemcpyHostToDevice) == hipSuccess;
    int rc = bj_lde_commit_h(trace, n_cols, log_n, log_lde, log_k, cap, lde, leaves, nodes, cap_out);
    CHECK(rc == BJ_OK, "bj_lde_commit_h: rc %d (%s)", rc, bj_last_error());
    u64* r_lde = xmalloc(8 * nd * n_cols), *r_leaves = xmalloc(32 * nl), *r_nodes = xmalloc(32 * n_nodes);
    u64 r_cap[4 * 4096];
    bjo_lde_commit_subset(trace, n_cols, log_n, log_lde, log_k, cap, r_lde, r_leaves, r_nodes, r_cap, threads);
    size_t w = 0;
    CHECK(eq_canon(lde, r_lde, nd * n_cols, &w), "LDE differs at %zu", w);
    CHECK(eq_canon(leaves, r_leaves, 4 * nl, &w), "leaves differ at %zu", w);
    CHECK(eq_canon(nodes, r_nodes, 4 * n_nodes, &w), "nodes differ at %zu", w);
    CHECK(eq_canon(cap_out, r_cap, 4 * cap, &w), "cap differs at %zu", w);
    /* the device-resident one-call commit (ABI 2.4, flags 0: no monomial write-back), HBM buffers
     * from hipMalloc, the legacy stream: the mode a GPU-resident Rust prover uses */
    u64 d_cap[4 * 4096];
    ok = ok && hipMalloc((void**)&d_scr, 8 * n * n_cols) == hipSuccess &&
         hipMalloc((void**)&d_lde, 8 * nd * n_cols) == hipSuccess && hipMalloc((void**)&d_lv, 32 * nl) == hipSuccess &&
         hipMalloc((void**)&d_nd, 32 * n_nodes) == hipSuccess;
    CHECK(ok, "device buffers for bj_lde_commit_ex_d");
    if (ok) {
        rc = bj_lde_commit_ex_d(d_tr, n_cols, n, log_n, log_lde, log_k, cap, d_scr, d_lde, d_lv, d_nd, d_cap, 0, NULL);
        CHECK(rc == BJ_OK, "bj_lde_commit_ex_d: rc %d (%s)", rc, bj_last_error());
        CHECK(hipMemcpy(lde, d_lde, 8 * nd * n_cols, hipMemcpyDeviceToHost) == hipSuccess &&
                  hipMemcpy(leaves, d_lv, 32 * nl, hipMemcpyDeviceToHost) == hipSuccess &&
                  hipMemcpy(nodes, d_nd, 32 * n_nodes, hipMemcpyDeviceToHost) == hipSuccess,
              "copy back");
        CHECK(eq_canon(lde, r_lde, nd * n_cols, &w), "device commit: LDE differs at %zu", w);
        CHECK(eq_canon(leaves, r_leaves, 4 * nl, &w), "device commit: leaves differ at %zu", w);
        CHECK(eq_canon(nodes, r_nodes, 4 * n_nodes, &w), "device commit: nodes differ at %zu", w);
        CHECK(eq_canon(d_cap, r_cap, 4 * cap, &w), "device commit: cap differs at %zu", w);
    }
    hipFree(d_tr); hipFree(d_scr); hipFree(d_lde); hipFree(d_lv); hipFree(d_nd);
    free(trace); free(lde); free(leaves); free(nodes); free(r_lde); free(r_leaves); free(r_nodes);
}

/* ------------------------------- 4. collective sharded commit, one thread per rank */

typedef struct {
    void* group;            /* in-process transport (bj_comm_init_local), or NULL: */
    const uint8_t* uid;     /* RCCL (bj_comm_init_rccl) over this unique id */
    int rank, world;
    uint32_t n_cols, log_n, log_lde, log_k, cap;
    int check_world;        /* RCCL: 1 expect bj_comm_check_world to pass (then time one exchange of the
                             * run's kind and size, as bench.py's "link" does), -1 to reject a shared
                             * device, 2 to reject a rank whose own record failed (the mock's
                             * MOCK_RCCL_FAIL_INFO_RANK) on every rank */
    const u64* trace; /* all columns, host */
    u64* leaves;      /* all leaves, host: rank P writes its range */
    u64* cap_out;     /* this rank's gathered cap */
    int rc;
} rank_job_t;

#define HIPC(expr)                                     \
    do {                                               \
        if ((expr) != hipSuccess) {                    \
            fprintf(stderr, "HIP error: %s\n", #expr); \
            j->rc = -1;                                \
            return NULL;                               \
        }                                              \
    } while (0)

/* What one rank of a multi-GPU prover does: its columns (bj_sharded_columns order) into HBM,
 * then one collective bj_sharded_commit_d.  Ranks share one device through the in-process
 * transport here; with RCCL each would own a GPU (bj_comm_init_rccl). */
static void* rank_worker(void* p) {
    rank_job_t* j = (rank_job_t*)p;
    /* m leaves per rank over the first k cosets; its LDE is D / k blocks of m per column */
    const size_t n = (size_t)1 << j->log_n, nl = n << j->log_k, m = nl / j->world;
    const size_t blocks = (size_t)1 << (j->log_lde - j->log_k);
    const uint32_t cpr = j->n_cols / j->world, cap_local = j->cap / j->world ? j->cap / j->world : 1;
    uint32_t log_g = 0;
    while ((1 << log_g) < j->world) log_g++;
    uint32_t* cols = xmalloc(4 * cpr);
    j->rc = bj_sharded_columns(j->n_cols, log_g, j->rank, BJ_HASHER_POSEIDON2, cols);
    if (j->rc) return NULL;
    HIPC(hipSetDevice(0));
    hipStream_t st;
    HIPC(hipStreamCreate(&st));
    u64 *tr, *lde, *leaves, *nodes, *cap;
    HIPC(hipMalloc((void**)&tr, 8 * n * cpr));
    HIPC(hipMalloc((void**)&lde, 8 * m * j->n_cols * blocks));
    HIPC(hipMalloc((void**)&leaves, 32 * m));
    HIPC(hipMalloc((void**)&nodes, 32 * (m - cap_local)));
    HIPC(hipMalloc((void**)&cap, 32 * j->cap));
    for (uint32_t c = 0; c < cpr; c++) HIPC(hipMemcpy(tr + c * n, j->trace + (size_t)cols[c] * n, 8 * n, hipMemcpyHostToDevice));
    bj_comm* comm = NULL;
    j->rc = j->group ? bj_comm_init_local(j->group, j->rank, &comm) : bj_comm_init_rccl(j->uid, j->world, j->rank, &comm);
    if (j->rc) return NULL;
    if (j->check_world == 2) {
        /* one rank cannot read its transport record: it still enters the gather, so every rank
         * returns BJ_EINVAL instead of its peers waiting for it */
        bj_comm_info_t all[64];
        int rc = bj_comm_check_world(comm, all, st);
        if (rc != BJ_EINVAL || !strstr(bj_last_error(), "could not read its transport record")) {
            fprintf(stderr, "rank %d: bj_comm_check_world rc %d (%s), expected an invalid-record rejection\n",
                    j->rank, rc, bj_last_error());
            j->rc = -1;
            return NULL;
        }
    } else if (j->check_world) {
        /* what RCCL's API reports for this rank (ncclCommCount / UserRank / CuDevice), then the
         * collective world check: a shared device must be rejected, distinct ones accepted */
        bj_comm_info_t info, all[64];
        j->rc = bj_comm_info(comm, &info);
        if (j->rc) return NULL;
        if (info.kind != BJ_COMM_RCCL || info.transport_count != j->world || info.transport_rank != j->rank ||
            info.world != j->world || info.rank != j->rank) {
            fprintf(stderr, "rank %d: bj_comm_info kind %d world %d rank %d transport %d of %d\n", j->rank, info.kind,
                    info.world, info.rank, info.transport_rank, info.transport_count);
            j->rc = -1;
            return NULL;
        }
        int rc = bj_comm_check_world(comm, all, st);
        if (j->check_world > 0 ? rc != BJ_OK : rc != BJ_EINVAL || !strstr(bj_last_error(), "share device")) {
            fprintf(stderr, "rank %d: bj_comm_check_world rc %d (%s), expected %s\n", j->rank, rc, bj_last_error(),
                    j->check_world > 0 ? "success" : "a shared-device rejection");
            j->rc = -1;
            return NULL;
        }
        for (int p = 0; p < j->world; p++)
            if (all[p].rank != p || all[p].transport_count != j->world) {
                fprintf(stderr, "rank %d: gathered slot %d holds rank %d of %d\n", j->rank, p, all[p].rank,
                        all[p].transport_count);
                j->rc = -1;
                return NULL;
            }
        if (j->check_world > 0) {
            /* the link probe bench.py runs before an N > 1 line's timed region (its "link"
             * object): one bj_comm_exchange_d of the commit's kind and size -- G <= D the
             * all-gather of 8 n C/G bytes per rank, G > D the all-to-all of 8 m C/G per
             * destination and block -- after a small exchange that sets up the transport */
            const int a2a = j->world > (1 << j->log_lde);
            const size_t block = a2a ? 8 * m * cpr * blocks : 8 * n * cpr;
            const int kind = a2a ? BJ_XCHG_ALL_TO_ALL : BJ_XCHG_ALL_GATHER;
            void *snd, *rcv;
            HIPC(hipMalloc(&snd, a2a ? block * j->world : block));
            HIPC(hipMalloc(&rcv, block * j->world));
            HIPC(hipMemsetAsync(snd, 0, a2a ? block * j->world : block, st));
            hipEvent_t e0, e1;
            HIPC(hipEventCreate(&e0));
            HIPC(hipEventCreate(&e1));
            j->rc = bj_comm_exchange_d(comm, kind, snd, rcv, 8, st);
            if (j->rc == 0) {
                HIPC(hipStreamSynchronize(st));
                HIPC(hipEventRecord(e0, st));
                j->rc = bj_comm_exchange_d(comm, kind, snd, rcv, block, st);
                HIPC(hipEventRecord(e1, st));
                HIPC(hipStreamSynchronize(st));
            }
            float ms = 0;
            HIPC(hipEventElapsedTime(&ms, e0, e1));
            hipEventDestroy(e0); hipEventDestroy(e1); hipFree(snd); hipFree(rcv);
            if (j->rc) return NULL;
            const size_t peer_bytes = (size_t)(j->world - 1) * block;
            printf("link world %d rank %d kind %s bytes_per_rank %zu ms %.3f gbs_per_rank %.2f\n", j->world, j->rank,
                   a2a ? "all_to_all" : "all_gather", peer_bytes, ms, ms > 0 ? peer_bytes / ms / 1e6 : 0.0);
        }
    }
    j->rc = bj_sharded_commit_d(comm, tr, n, j->n_cols, j->log_n, j->log_lde, j->log_k, j->cap, BJ_HASHER_POSEIDON2,
                                lde, leaves, nodes, cap, st);
    if (j->rc == 0) {
        HIPC(hipStreamSynchronize(st));
        HIPC(hipMemcpy(j->leaves + 4 * m * j->rank, leaves, 32 * m, hipMemcpyDeviceToHost));
        HIPC(hipMemcpy(j->cap_out, cap, 32 * j->cap, hipMemcpyDeviceToHost));
    }
    bj_comm_destroy(comm);
    hipFree(tr); hipFree(lde); hipFree(leaves); hipFree(nodes); hipFree(cap);
    hipStreamDestroy(st);
    free(cols);
    return NULL;
}

/* use_rccl: the ranks talk through RCCL's API (bj_comm_init_rccl) -- on a one-GPU box only with
 * the mock librccl.so.1 (tests/c/mock_rccl.cpp, BJ_TEST_MOCK_RCCL), since RCCL refuses two ranks
 * on one device */
static void check_sharded(uint32_t log_n, uint32_t n_cols, uint32_t log_lde, uint32_t log_k, uint32_t cap, int world,
                          int use_rccl, int check_world) {
    size_t n = (size_t)1 << log_n, nd = n << log_lde, nl = n << log_k, n_nodes = nl - cap;
    u64* trace = xmalloc(8 * n * n_cols);
    for (uint32_t c = 0; c < n_cols; c++)
        for (size_t r = 0; r < n; r++) trace[(size_t)c * n + r] = canon(splitmix64(42 + (u64)c * n + r));
    u64* leaves = xmalloc(32 * nl), *caps = xmalloc(32 * (size_t)cap * world);
    void* group = NULL;
    uint8_t uid[128];
    int rc = use_rccl ? bj_comm_rccl_unique_id(uid) : bj_comm_local_group_create(world, &group);
    CHECK(rc == BJ_OK, "%s: %s", use_rccl ? "bj_comm_rccl_unique_id" : "bj_comm_local_group_create", bj_last_error());
    if (rc) return;
    pthread_t th[64];
    rank_job_t jobs[64];
    for (int P = 0; P < world; P++) {
        jobs[P] = (rank_job_t){group, uid, P, world, n_cols, log_n, log_lde, log_k, cap, check_world, trace, leaves,
                               caps + 4 * (size_t)cap * P, 0};
        pthread_create(&th[P], NULL, rank_worker, &jobs[P]);
    }
    for (int P = 0; P < world; P++) {
        pthread_join(th[P], NULL);
        CHECK(jobs[P].rc == 0, "rank %d of %d%s: rc %d (%s)", P, world, use_rccl ? " (rccl)" : "", jobs[P].rc,
              bj_last_error());
    }
    if (group) bj_comm_local_group_destroy(group);
    u64* r_lde = xmalloc(8 * nd * n_cols), *r_leaves = xmalloc(32 * nl), *r_nodes = xmalloc(32 * n_nodes);
    u64 r_cap[4 * 4096];
    bjo_lde_commit_subset(trace, n_cols, log_n, log_lde, log_k, cap, r_lde, r_leaves, r_nodes, r_cap, 4);
    size_t w = 0;
    CHECK(eq_canon(leaves, r_leaves, 4 * nl, &w), "sharded x%d leaves differ at %zu", world, w);
    for (int P = 0; P < world; P++)
        CHECK(eq_canon(caps + 4 * (size_t)cap * P, r_cap, 4 * cap, &w), "sharded x%d: rank %d cap differs", world, P);
    free(trace); free(leaves); free(caps); free(r_lde); free(r_leaves); free(r_nodes);
}

/* ------------------------------------------------------------ 5. error contract */

static void check_errors(void) {
    u64 col[12] = {0};
    CHECK(bj_fft_natural_to_bitreversed_h(col, 12, 1) == BJ_EINVAL, "length 12 must be rejected");
    CHECK(strlen(bj_last_error()) > 0, "no error message after BJ_EINVAL");
    u64 st[12] = {0};
    CHECK(bj_poseidon2_permute_h(st) == BJ_OK, "library unusable after an error: %s", bj_last_error());
}

/* ------------------- 6. memory returns after the caches are released (ABI 2.1 / 2.3) */

/* Three commits of different sizes leave their tables (per size) and pooled workspace cached;
 * bj_release_tables + bj_release_workspace (what the Rust shim's BjTables guard runs in its Drop,
 * INTEGRATION.md) must give the device memory back: free memory returns to its baseline within
 * `slack` bytes (the runtime's own small allocations).  The reference drops its twiddle Vecs at
 * scope end (prover.rs:313-353); this is that drop for the library's caches. */
static void commit_three_sizes(void) {
    const uint32_t sizes[3][3] = {{16, 16, 1}, {18, 8, 2}, {20, 8, 1}}; /* log_n, cols, log_lde */
    for (int i = 0; i < 3; i++) {
        const uint32_t log_n = sizes[i][0], n_cols = sizes[i][1], log_lde = sizes[i][2], cap = 16;
        const size_t n = (size_t)1 << log_n;
        u64* trace = xmalloc(8 * n * n_cols);
        for (size_t j = 0; j < n * n_cols; j++) trace[j] = canon(splitmix64(7 + j));
        u64 cap_out[4 * 16];
        int rc = bj_lde_commit_h(trace, n_cols, log_n, log_lde, log_lde, cap, NULL, NULL, NULL, cap_out);
        CHECK(rc == BJ_OK, "commit 2^%u: rc %d (%s)", log_n, rc, bj_last_error());
        free(trace);
    }
    CHECK(hipDeviceSynchronize() == hipSuccess, "sync");
}

static void check_release(void) {
    const size_t slack = (size_t)4 << 20;
    size_t free0 = 0, free1 = 0, free2 = 0, total = 0;
    /* a first round, released, so the baseline holds what the runtime keeps once it has run these
     * kernels at all (code objects, the scratch of spilling kernels, kernel-argument pools,
     * per-thread streams): only what the library itself caches is measured below */
    commit_three_sizes();
    CHECK(bj_release_tables() == BJ_OK && bj_release_workspace() == BJ_OK, "first release: %s", bj_last_error());
    CHECK(hipMemGetInfo(&free0, &total) == hipSuccess, "hipMemGetInfo");
    commit_three_sizes();
    CHECK(hipMemGetInfo(&free1, &total) == hipSuccess, "hipMemGetInfo");
    CHECK(bj_release_tables() == BJ_OK, "bj_release_tables: %s", bj_last_error());
    CHECK(bj_release_workspace() == BJ_OK, "bj_release_workspace: %s", bj_last_error());
    CHECK(hipMemGetInfo(&free2, &total) == hipSuccess, "hipMemGetInfo");
    CHECK(free1 + ((size_t)16 << 20) < free0, "three commits cached less than 16 MiB (%zu -> %zu)", free0, free1);
    CHECK(free2 + slack >= free0, "device memory not returned: free %zu before, %zu cached, %zu after release", free0,
          free1, free2);
    printf("c_caller release ok: free %.1f MiB before, %.1f with caches, %.1f after release\n", free0 / 1048576.0,
           free1 / 1048576.0, free2 / 1048576.0);
}

int main(int argc, char** argv) {
    if (argc == 2 && strcmp(argv[1], "release") == 0) {
        check_release();
        return failures ? 1 : 0;
    }
    if (argc != 6 && argc != 7) {
        fprintf(stderr, "usage: %s LOG_N N_COLS LOG_LDE CAP THREADS [LOG_K]\n", argv[0]);
        return 2;
    }
    uint32_t log_n = atoi(argv[1]), n_cols = atoi(argv[2]), log_lde = atoi(argv[3]), cap = atoi(argv[4]);
    int threads = atoi(argv[5]);
    uint32_t log_k = argc == 7 ? (uint32_t)atoi(argv[6]) : log_lde;
    if (cap == 0 || cap > 4096 || (cap & (cap - 1)) || threads < 1 || log_k > log_lde) {
        fprintf(stderr, "cap must be a power of two <= 4096, threads >= 1, LOG_K <= LOG_LDE\n");
        return 2;
    }
    fprintf(stderr, "abi %u.%u\n", bj_abi_version() >> 16, bj_abi_version() & 0xffff);
    for (int round = 0; round < 3; round++) check_fft_seam(log_n, n_cols, threads);
    check_tree_hasher();
    u64 cap_out[4 * 4096];
    check_commit(log_n, n_cols, log_lde, log_k, cap, threads, cap_out);
    /* BJ_TEST_MOCK_RCCL=path: load the mock librccl.so.1 first, so the library's RCCL path runs
     * multi-rank on one GPU (the real RCCL refuses two ranks on one device) */
    const char* mock = getenv("BJ_TEST_MOCK_RCCL");
    if (mock && !dlopen(mock, RTLD_NOW | RTLD_GLOBAL)) {
        fprintf(stderr, "cannot load %s: %s\n", mock, dlerror());
        return 2;
    }
    int worlds_checked = 0;
    for (int world = 2; world <= 8; world *= 2)
        if (n_cols % world == 0 && ((size_t)1 << (log_n + log_k)) / world > (cap / world ? cap / world : 1)) {
            check_sharded(log_n, n_cols, log_lde, log_k, cap, world, 0, 0);
            if (mock) {
                /* the stand-in's ranks share this GPU: the world check must name the shared device;
                 * with distinct (stand-in) device numbers it must pass */
                check_sharded(log_n, n_cols, log_lde, log_k, cap, world, 1, -1);
                setenv("MOCK_RCCL_FAKE_DEVICES", "1", 1);
                check_sharded(log_n, n_cols, log_lde, log_k, cap, world, 1, 1);
                /* a rank whose transport record fails: every rank gets BJ_EINVAL, none waits */
                char fail_rank[16];
                snprintf(fail_rank, sizeof(fail_rank), "%d", world - 1);
                setenv("MOCK_RCCL_FAIL_INFO_RANK", fail_rank, 1);
                check_sharded(log_n, n_cols, log_lde, log_k, cap, world, 1, 2);
                unsetenv("MOCK_RCCL_FAIL_INFO_RANK");
                unsetenv("MOCK_RCCL_FAKE_DEVICES");
                worlds_checked |= world;
            }
        }
    check_errors();
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    if (mock)
        printf("rccl world check ok at world%s%s%s: ncclCommCount = world, ncclCommUserRank = rank, shared device "
               "rejected, distinct devices accepted, a failed record rejected on every rank; link probe at each\n", worlds_checked & 2 ? " 2" : "", worlds_checked & 4 ? " 4" : "",
               worlds_checked & 8 ? " 8" : "");
    printf("c_caller ok%s: 2^%u x %u, LDE x%u, %u cosets committed, cap %u, %d seam threads; "
           "cap[0] = %016llx %016llx %016llx %016llx\n",
           mock ? " (collective also over RCCL's API, mock librccl)" : "", log_n, n_cols, 1u << log_lde, 1u << log_k, cap,
           threads, (unsigned long long)canon(cap_out[0]),
           (unsigned long long)canon(cap_out[1]), (unsigned long long)canon(cap_out[2]),
           (unsigned long long)canon(cap_out[3]));
    return 0;
}
