/*
 * boojum_oracle.c -- CPU ORACLE (TEST INFRASTRUCTURE ONLY).
 *
 * A plain-C restatement of the reference's witness-commitment path, used as the
 * checker for the HIP product path and as the timed CPU baseline ("port") in
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library.  The product path (era-boojum_amd/) never calls it.
 *
 * Every function cites the reference file:line it restates (paths relative to the
 * reference root, distributed-lab/era-boojum @ v2).
 *
 * Parity pinning: the Poseidon2 permutation, the Overwrite sponge, node hashing and
 * the cap layout are pinned by the reference's own proof.json / vk.json fixture
 * (tests/golden/, checked by tests/test_oracle_golden.py).  The LDE is pinned by the
 * reference's own methodology (naive coset DFT with generator 7, fft/mod.rs:1591-1634)
 * and the closed form LDE[c][L] = p_c(7 * w_{nD}^{bitrev(L)}).
 *
 * Representation: as in the reference, intermediate values may be non-canonical
 * u64 (any value < 2^64, field/goldilocks/mod.rs:92-94); every value exported by
 * this library is canonical (< p), as the reference's serialisation and equality
 * are on canonical values (mod.rs:96-105, 257-261).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

typedef uint64_t u64;
typedef unsigned __int128 u128;

#define GL_P 0xFFFFFFFF00000001ULL
#define GL_EPS 0xFFFFFFFFULL /* 2^32 - 1, field/goldilocks/mod.rs:82 */

/* ---------------------------------------------------------------- field (a1) */

/* to_reduced_u64, field/goldilocks/mod.rs:146-153 */
static inline u64 gl_canon(u64 x) { return x >= GL_P ? x - GL_P : x; }

/* add_assign_impl, field/goldilocks/mod.rs:213-231 */
static inline u64 gl_add(u64 a, u64 b) {
    u64 s = a + b;
    u64 over = s < a;
    u64 t = s + over * GL_EPS;
    if (t < s) t += GL_EPS; /* double overflow (both > ORDER) */
    return t;
}

/* sub_assign, field/goldilocks/mod.rs:307-325 */
static inline u64 gl_sub(u64 a, u64 b) {
    u64 d = a - b;
    u64 under = a < b;
    u64 t = d - under * GL_EPS;
    if (t > d) t -= GL_EPS; /* double underflow */
    return t;
}

/* from_u128_with_reduction, field/goldilocks/mod.rs:186-199 */
static inline u64 gl_reduce128(u128 x) {
    u64 lo = (u64)x, hi = (u64)(x >> 64);
    u64 hi_hi = hi >> 32, hi_lo = hi & GL_EPS;
    u64 t0 = lo - hi_hi;
    if (lo < hi_hi) t0 -= GL_EPS;
    u64 t1 = hi_lo * GL_EPS;
    u64 t2 = t0 + t1;
    if (t2 < t0) t2 += GL_EPS; /* add_no_canonicalize_trashing_input */
    return t2;
}

/* mul_assign_impl, field/goldilocks/mod.rs:243-247 */
static inline u64 gl_mul(u64 a, u64 b) { return gl_reduce128((u128)a * b); }

static u64 gl_pow(u64 b, u64 e) {
    u64 r = 1;
    while (e) {
        if (e & 1) r = gl_mul(r, b);
        b = gl_mul(b, b);
        e >>= 1;
    }
    return r;
}

static u64 gl_inv(u64 a) { return gl_pow(a, GL_P - 2); }

u64 bjo_gl_add(u64 a, u64 b) { return gl_canon(gl_add(a, b)); }
u64 bjo_gl_sub(u64 a, u64 b) { return gl_canon(gl_sub(a, b)); }
u64 bjo_gl_mul(u64 a, u64 b) { return gl_canon(gl_mul(a, b)); }
u64 bjo_gl_pow(u64 b, u64 e) { return gl_canon(gl_pow(b, e)); }
u64 bjo_gl_inv(u64 a) { return gl_canon(gl_inv(a)); }

/* ------------------------------------------------------- domain & twiddles */

/* domain_generator_for_size, cs/implementations/utils.rs:13-28:
 * square the 2^32-th root (mod.rs:108) down to the requested size. */
u64 bjo_domain_generator(uint32_t log_n) {
    u64 w = 0x185629dcda58878cULL; /* RADIX_2_SUBGROUP_GENERATOR, mod.rs:108 */
    for (uint32_t i = log_n; i < 32; i++) w = gl_mul(w, w);
    return gl_canon(w);
}

static inline uint64_t bitrev(uint64_t x, uint32_t bits) {
    if (bits == 0) return 0;
    uint64_t r = 0;
    for (uint32_t i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

/* bitreverse_enumeration_inplace, fft/mod.rs:41-155 (semantics: index bit reversal) */
void bjo_bitreverse_inplace(u64* a, size_t n) {
    uint32_t bits = 0;
    while (((size_t)1 << bits) < n) bits++;
    for (size_t i = 0; i < n; i++) {
        size_t j = (size_t)bitrev(i, bits);
        if (i < j) { u64 t = a[i]; a[i] = a[j]; a[j] = t; }
    }
}

/* precompute_twiddles_for_fft, cs/implementations/utils.rs:88-125:
 * omega (or omega^-1) powers 0..n/2, then bit-reversed (utils.rs:122).
 * Writes n/2 canonical values (n >= 2). */
void bjo_precompute_twiddles(uint32_t log_n, int inverse, u64* out) {
    size_t n = (size_t)1 << log_n, half = n / 2;
    u64 w = bjo_domain_generator(log_n);
    if (inverse) w = gl_inv(w);
    u64 cur = 1;
    for (size_t i = 0; i < half; i++) { out[i] = gl_canon(cur); cur = gl_mul(cur, w); }
    bjo_bitreverse_inplace(out, half);
}

/* --------------------------------------------------------------------- FFT */

/* distribute_powers, fft/mod.rs:308-317 */
void bjo_distribute_powers(u64* a, size_t n, u64 element) {
    u64 s = 1;
    for (size_t i = 0; i < n; i++) { a[i] = gl_mul(a[i], s); s = gl_mul(s, element); }
}

/* serial_ct_ntt_natural_to_bitreversed, fft/mod.rs:659-734 */
static void serial_ct_ntt(u64* a, size_t n, const u64* tw) {
    if (n == 1) return;
    size_t pairs = n / 2, groups = 1, dist = n / 2;
    for (size_t j = 0; j < pairs; j++) { /* omega = 1 stage, :678-699 */
        u64 u = a[j], v = a[j + dist];
        a[j + dist] = gl_sub(u, v);
        a[j] = gl_add(u, v);
    }
    pairs /= 2; groups *= 2; dist /= 2;
    while (groups < n) { /* :701-733 */
        for (size_t k = 0; k < groups; k++) {
            size_t i1 = k * pairs * 2, i2 = i1 + pairs;
            u64 s = tw[k];
            for (size_t j = i1; j < i2; j++) {
                u64 u = a[j], v = gl_mul(a[j + dist], s);
                a[j + dist] = gl_sub(u, v);
                a[j] = gl_add(u, v);
            }
        }
        pairs /= 2; groups *= 2; dist /= 2;
    }
}

/* fft_natural_to_bitreversed, fft/mod.rs:398-411 (values left as computed) */
static void fft_nb_raw(u64* a, size_t n, u64 coset, const u64* tw) {
    if (gl_canon(coset) != 1) bjo_distribute_powers(a, n, coset);
    serial_ct_ntt(a, n, tw);
}

void bjo_fft_natural_to_bitreversed(u64* a, size_t n, u64 coset, const u64* tw) {
    fft_nb_raw(a, n, coset, tw);
    for (size_t i = 0; i < n; i++) a[i] = gl_canon(a[i]);
}

/* ifft_natural_to_natural, fft/mod.rs:464-491 */
static void ifft_nn_raw(u64* a, size_t n, u64 coset, const u64* inv_tw) {
    serial_ct_ntt(a, n, inv_tw);
    bjo_bitreverse_inplace(a, n);
    if (gl_canon(coset) != 1) bjo_distribute_powers(a, n, gl_inv(coset));
    if (n > 1) {
        u64 n_inv = gl_inv((u64)n);
        for (size_t i = 0; i < n; i++) a[i] = gl_mul(a[i], n_inv);
    }
}

void bjo_ifft_natural_to_natural(u64* a, size_t n, u64 coset, const u64* inv_tw) {
    ifft_nn_raw(a, n, coset, inv_tw);
    for (size_t i = 0; i < n; i++) a[i] = gl_canon(a[i]);
}

/* ------------------------------------------------------- threaded "Worker" */

/* Worker::scope, worker/mod.rs:34-66: ceil(work / threads) chunks, one per thread. */
typedef struct {
    void (*fn)(void* ctx, size_t begin, size_t end);
    void* ctx;
    size_t begin, end;
} job_t;

static void* job_run(void* p) {
    job_t* j = (job_t*)p;
    if (j->begin < j->end) j->fn(j->ctx, j->begin, j->end);
    return NULL;
}

static void worker_scope(int threads, size_t work, void (*fn)(void*, size_t, size_t), void* ctx) {
    if (threads <= 1 || work <= 1) { fn(ctx, 0, work); return; }
    size_t chunk = (work + threads - 1) / threads;
    int nt = (int)((work + chunk - 1) / chunk);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nt);
    job_t* jobs = (job_t*)malloc(sizeof(job_t) * nt);
    for (int t = 0; t < nt; t++) {
        jobs[t].fn = fn; jobs[t].ctx = ctx;
        jobs[t].begin = t * chunk;
        jobs[t].end = (t + 1) * chunk < work ? (t + 1) * chunk : work;
        pthread_create(&th[t], NULL, job_run, &jobs[t]);
    }
    for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
    free(th); free(jobs);
}

/* ----------------------------------------------------------------- LDE (a11) */

typedef struct {
    u64* cols; size_t n; const u64* tw; u64* lde; uint32_t n_cols, lde_degree; const u64* cosets;
} lde_ctx_t;

static void lde_ifft_job(void* c, size_t b, size_t e) {
    lde_ctx_t* x = (lde_ctx_t*)c;
    for (size_t i = b; i < e; i++) ifft_nn_raw(x->cols + i * x->n, x->n, 1, x->tw);
}

static void lde_fft_job(void* c, size_t b, size_t e) {
    lde_ctx_t* x = (lde_ctx_t*)c;
    for (size_t job = b; job < e; job++) {
        /* job order as utils.rs:355-379: all columns of coset 0, then coset 1, ... */
        size_t coset_idx = job / x->n_cols, col = job % x->n_cols;
        u64* dst = x->lde + (col * x->lde_degree + coset_idx) * x->n;
        memcpy(dst, x->cols + col * x->n, x->n * sizeof(u64));
        fft_nb_raw(dst, x->n, x->cosets[coset_idx], x->tw);
        for (size_t i = 0; i < x->n; i++) dst[i] = gl_canon(dst[i]);
    }
}

/* LDE cosets: 7 * w_{nD}^{bitrev_{log D}(i)}, utils.rs:334-347, 370-373 */
void bjo_lde_cosets(uint32_t log_n, uint32_t log_d, u64* out) {
    size_t d = (size_t)1 << log_d;
    u64 g = bjo_domain_generator(log_n + log_d);
    for (size_t i = 0; i < d; i++) out[i] = gl_canon(gl_mul(gl_pow(g, bitrev(i, log_d)), 7));
}

/* transform_raw_storages_to_lde, utils.rs:270-309 + transform_monomials_to_lde :311-403.
 * trace: n_cols columns of n values (column-major, contiguous).  Overwritten with the
 * (canonical) monomials.  lde: n_cols x D x n, i.e. LDE[col][coset][row]
 * (the reference's per-column Vec<coset> storage, polynomial/lde.rs:156-341). */
void bjo_lde(u64* trace, uint32_t n_cols, uint32_t log_n, uint32_t log_d, u64* lde, int threads) {
    size_t n = (size_t)1 << log_n, d = (size_t)1 << log_d;
    u64* tw = (u64*)malloc(sizeof(u64) * (n / 2 > 0 ? n / 2 : 1));
    u64* cosets = (u64*)malloc(sizeof(u64) * d);
    lde_ctx_t x = {trace, n, tw, lde, n_cols, (uint32_t)d, cosets};
    if (n >= 2) bjo_precompute_twiddles(log_n, 1, tw);
    worker_scope(threads, n_cols, lde_ifft_job, &x);
    if (n >= 2) bjo_precompute_twiddles(log_n, 0, tw);
    bjo_lde_cosets(log_n, log_d, cosets);
    worker_scope(threads, (size_t)n_cols * d, lde_fft_job, &x);
    for (size_t i = 0; i < n * n_cols; i++) trace[i] = gl_canon(trace[i]);
    free(tw); free(cosets);
}

/* ----------------------------------------------------------- Poseidon2 (a14) */

static const u64 RC[30][12] = {
#include "poseidon2_rc.inc"
};

/* block_mul (M4), implementations/suggested_mds.rs:19-55 */
static inline void m4(u64* x0, u64* x1, u64* x2, u64* x3) {
    u64 t0 = gl_add(*x0, *x1), t1 = gl_add(*x2, *x3);
    u64 t2 = gl_add(gl_add(*x1, *x1), t1);
    u64 t3 = gl_add(gl_add(*x3, *x3), t0);
    u64 t4 = gl_add(gl_add(gl_add(t1, t1), gl_add(t1, t1)), t3);
    u64 t5 = gl_add(gl_add(gl_add(t0, t0), gl_add(t0, t0)), t2);
    u64 t6 = gl_add(t3, t5), t7 = gl_add(t2, t4);
    *x0 = t6; *x1 = t5; *x2 = t7; *x3 = t4;
}

/* suggested_mds_mul: block-circulant(2*M4, M4, M4), suggested_mds.rs:57-97 */
static void mds_ext(u64* s) {
    u64 x[12];
    memcpy(x, s, sizeof(x));
    m4(&x[0], &x[1], &x[2], &x[3]);
    m4(&x[4], &x[5], &x[6], &x[7]);
    m4(&x[8], &x[9], &x[10], &x[11]);
    for (int i = 0; i < 4; i++) {
        s[i] = gl_add(gl_add(gl_add(x[i], x[i]), x[i + 4]), x[i + 8]);
        s[i + 4] = gl_add(gl_add(gl_add(x[i + 4], x[i + 4]), x[i]), x[i + 8]);
        s[i + 8] = gl_add(gl_add(gl_add(x[i + 8], x[i + 8]), x[i]), x[i + 4]);
    }
}

static inline u64 sbox(u64 x) { /* apply_non_linearity x^7, state_generic_impl.rs:141-147 */
    u64 x2 = gl_mul(x, x), x3 = gl_mul(x2, x), x4 = gl_mul(x2, x2);
    return gl_mul(x4, x3);
}

/* M_I = diag(2^sh) + 1 1^T, state_generic_impl.rs:71-84 (diagonal) and :166-202 (m_i_mul) */
static const int MI_SHIFT[12] = {4, 14, 11, 8, 0, 5, 2, 9, 13, 6, 3, 12};

static void mds_int(u64* s) {
    u64 sum = 0;
    for (int i = 0; i < 12; i++) sum = gl_add(sum, s[i]);
    for (int i = 0; i < 12; i++) s[i] = gl_add(gl_mul(s[i], 1ULL << MI_SHIFT[i]), sum);
}

/* poseidon2_permutation, state_generic_impl.rs:221-236 */
void bjo_poseidon2_permutation(u64* s) {
    mds_ext(s);
    int r = 0;
    for (int i = 0; i < 4; i++, r++) { /* full_round :150-160 */
        for (int j = 0; j < 12; j++) s[j] = sbox(gl_add(s[j], RC[r][j]));
        mds_ext(s);
    }
    for (int i = 0; i < 22; i++, r++) { /* partial_round_poseidon2 :204-219 */
        s[0] = sbox(gl_add(s[0], RC[r][0]));
        mds_int(s);
    }
    for (int i = 0; i < 4; i++, r++) {
        for (int j = 0; j < 12; j++) s[j] = sbox(gl_add(s[j], RC[r][j]));
        mds_ext(s);
    }
}

void bjo_poseidon2_permute_canonical(u64* s) {
    bjo_poseidon2_permutation(s);
    for (int i = 0; i < 12; i++) s[i] = gl_canon(s[i]);
}

/* ------------------------------------------------------ sponge / tree hasher */

/* TreeHasher::hash_into_leaf for GoldilocksPoseidon2Sponge<AbsorptionModeOverwrite>:
 * cs/oracle/mod.rs:141-151 -> algebraic_props/sponge.rs:224-239 (absorb_single),
 * :300-323 (finalize: overwrite state[0..filled], zero-pad to rate 8, permute iff
 * filled > 0), commitment = state[0..4] (poseidon2/mod.rs:157-165).
 * Elements are read as elems[i * stride]. */
static void leaf_hash_strided(const u64* elems, size_t count, size_t stride, u64* out4) {
    u64 s[12] = {0};
    size_t filled = 0;
    for (size_t i = 0; i < count; i++) {
        s[filled++] = elems[i * stride];
        if (filled == 8) { bjo_poseidon2_permutation(s); filled = 0; }
    }
    if (filled > 0) {
        for (size_t i = filled; i < 8; i++) s[i] = 0;
        bjo_poseidon2_permutation(s);
    }
    for (int i = 0; i < 4; i++) out4[i] = gl_canon(s[i]);
}

void bjo_hash_into_leaf(const u64* elems, size_t count, u64* out4) {
    leaf_hash_strided(elems, count, 1, out4);
}

/* hash_into_node, cs/oracle/mod.rs:162-168: absorb(l), absorb(r), finalize ->
 * exactly one permutation of [l0..l3, r0..r3, 0,0,0,0]. */
void bjo_hash_into_node(const u64* l, const u64* r, u64* out4) {
    u64 s[12] = {0};
    for (int i = 0; i < 4; i++) { s[i] = l[i]; s[4 + i] = r[i]; }
    bjo_poseidon2_permutation(s);
    for (int i = 0; i < 4; i++) out4[i] = gl_canon(s[i]);
}

/* ------------------------------------------- Blake2s256 tree hasher (a18') */

/* TreeHasher for blake2::Blake2s256 (cs/oracle/mod.rs:179-245), the tree hasher of the
 * non-recursive prover configs (gadgets/sha256/mod.rs:263-269).  Third-party crate
 * blake2 = "0.10" (Cargo.toml:23, resolved 0.10.6): Blake2s256 = BLAKE2s with a 32-byte
 * digest, no key, salt or personalisation, i.e. RFC 7693 (restated below).
 *   leaf: update(as_u64_reduced(x).to_le_bytes()) for each element, finalize (:190-231);
 *   node: update(left 32 B), update(right 32 B), finalize (:234-245).
 * Digests are 32 bytes, stored here as 4 little-endian u64 words. */
static const uint32_t B2S_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                   0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t B2S_SIGMA[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

static inline uint32_t rotr32(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

/* RFC 7693 section 3.2, function F (10 rounds of G over the 4x4 state) */
static void b2s_compress(uint32_t h[8], const uint32_t m[16], uint64_t t, int last) {
    uint32_t v[16];
    for (int i = 0; i < 8; i++) { v[i] = h[i]; v[8 + i] = B2S_IV[i]; }
    v[12] ^= (uint32_t)t;
    v[13] ^= (uint32_t)(t >> 32);
    if (last) v[14] = ~v[14];
#define B2S_G(a, b, c, d, x, y)                    \
    do {                                           \
        v[a] = v[a] + v[b] + x; v[d] = rotr32(v[d] ^ v[a], 16); \
        v[c] = v[c] + v[d];     v[b] = rotr32(v[b] ^ v[c], 12); \
        v[a] = v[a] + v[b] + y; v[d] = rotr32(v[d] ^ v[a], 8);  \
        v[c] = v[c] + v[d];     v[b] = rotr32(v[b] ^ v[c], 7);  \
    } while (0)
    for (int r = 0; r < 10; r++) {
        const uint8_t* s = B2S_SIGMA[r];
        B2S_G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        B2S_G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        B2S_G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        B2S_G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        B2S_G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        B2S_G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        B2S_G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        B2S_G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
#undef B2S_G
    for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[8 + i];
}

static inline uint32_t load_le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* BLAKE2s-256 of len bytes (RFC 7693 section 3.3): every block but the last is compressed
 * as more data follows; the last (zero-padded, possibly empty) carries the final flag and
 * the total byte count. */
void bjo_blake2s(const uint8_t* data, size_t len, uint8_t* out32) {
    uint32_t h[8];
    for (int i = 0; i < 8; i++) h[i] = B2S_IV[i];
    h[0] ^= 0x01010000u ^ 32u; /* depth 1, fanout 1, no key, 32-byte digest */
    uint32_t m[16];
    size_t off = 0;
    while (len - off > 64) {
        for (int i = 0; i < 16; i++) m[i] = load_le32(data + off + 4 * i);
        off += 64;
        b2s_compress(h, m, off, 0);
    }
    uint8_t last[64] = {0};
    memcpy(last, data + off, len - off);
    for (int i = 0; i < 16; i++) m[i] = load_le32(last + 4 * i);
    b2s_compress(h, m, len, 1);
    for (int i = 0; i < 8; i++) {
        out32[4 * i] = (uint8_t)h[i];
        out32[4 * i + 1] = (uint8_t)(h[i] >> 8);
        out32[4 * i + 2] = (uint8_t)(h[i] >> 16);
        out32[4 * i + 3] = (uint8_t)(h[i] >> 24);
    }
}

static void b2s_leaf_strided(const u64* elems, size_t count, size_t stride, u64* out4) {
    uint8_t stackbuf[8 * 64] = {0};
    uint8_t* buf = count <= 64 ? stackbuf : (uint8_t*)malloc(8 * count);
    for (size_t i = 0; i < count; i++) {
        u64 v = gl_canon(elems[i * stride]); /* as_u64_reduced().to_le_bytes() */
        for (int b = 0; b < 8; b++) buf[8 * i + b] = (uint8_t)(v >> (8 * b));
    }
    bjo_blake2s(buf, 8 * count, (uint8_t*)out4); /* little-endian host: bytes == LE words */
    if (buf != stackbuf) free(buf);
}

void bjo_blake2s_leaf(const u64* elems, size_t count, u64* out4) { b2s_leaf_strided(elems, count, 1, out4); }

/* One leaf's message continued over a column range (the multi-GPU column pipeline):
 * h_in = the chaining value after `before` elements (a multiple of 8; NULL when 0).  With
 * final == 0 (count a multiple of 8) every block is compressed as more data follows and
 * out4 = the new chaining value; with final != 0 the last block carries the final flag and
 * out4 = the digest.  Chaining ranges gives exactly bjo_blake2s_leaf of the whole message. */
void bjo_blake2s_leaf_partial(const u64* h_in, const u64* elems, size_t count, uint64_t before, int final_,
                              u64* out4) {
    uint32_t h[8], m[16];
    if (h_in) {
        for (int i = 0; i < 4; i++) { h[2 * i] = (uint32_t)h_in[i]; h[2 * i + 1] = (uint32_t)(h_in[i] >> 32); }
    } else {
        for (int i = 0; i < 8; i++) h[i] = B2S_IV[i];
        h[0] ^= 0x01010000u ^ 32u;
    }
    uint64_t bytes = 8 * before;
    size_t k = 0;
    size_t nonfinal = final_ ? (count ? (count - 1) / 8 : 0) : count / 8;
    for (size_t g = 0; g < nonfinal; g++, k += 8) {
        for (int i = 0; i < 8; i++) { u64 v = gl_canon(elems[k + i]); m[2 * i] = (uint32_t)v; m[2 * i + 1] = (uint32_t)(v >> 32); }
        bytes += 64;
        b2s_compress(h, m, bytes, 0);
    }
    if (final_) {
        size_t rem = count - k;
        for (int i = 0; i < 8; i++) {
            u64 v = (size_t)i < rem ? gl_canon(elems[k + i]) : 0;
            m[2 * i] = (uint32_t)v;
            m[2 * i + 1] = (uint32_t)(v >> 32);
        }
        bytes += 8 * rem;
        b2s_compress(h, m, bytes, 1);
    }
    for (int i = 0; i < 4; i++) out4[i] = ((u64)h[2 * i + 1] << 32) | h[2 * i];
}

void bjo_blake2s_node(const u64* l, const u64* r, u64* out4) {
    uint8_t buf[64];
    memcpy(buf, l, 32);
    memcpy(buf + 32, r, 32);
    bjo_blake2s(buf, 64, (uint8_t*)out4);
}

/* ------------------------------------------- Keccak256 tree hasher (a18'') */

/* TreeHasher for sha3::Keccak256 (cs/oracle/mod.rs:247-313).  Third-party crate sha3 (git
 * RustCrypto/hashes rev 7a187e93, Cargo.toml:15): Keccak256 = Keccak[c = 512] with the
 * original Keccak padding (pad10*1 with domain byte 0x01), 32-byte digest; restated from the
 * Keccak reference (FIPS 202 section 3 permutation, rate 136 bytes).  The same sponge with
 * domain byte 0x06 is SHA3-256, which pins the permutation against hashlib.sha3_256.
 *   leaf: update(as_u64_reduced(x).to_le_bytes()) per element, finalize (:258-299);
 *   node: update(left 32 B), update(right 32 B), finalize (:302-313). */
static const u64 KECCAK_RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
/* rho offsets r[x + 5 y] */
static const int KECCAK_RHO[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                                   25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

static inline u64 rotl64(u64 x, int r) { return r ? (x << r) | (x >> (64 - r)) : x; }

/* Keccak-f[1600], lanes A[x + 5 y] (FIPS 202 3.2: theta, rho, pi, chi, iota) */
void bjo_keccak_f1600(u64* A) {
    for (int round = 0; round < 24; round++) {
        u64 C[5], D[5], B[25];
        for (int x = 0; x < 5; x++) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
        for (int x = 0; x < 5; x++) D[x] = C[(x + 4) % 5] ^ rotl64(C[(x + 1) % 5], 1);
        for (int i = 0; i < 25; i++) A[i] ^= D[i % 5];
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(A[x + 5 * y], KECCAK_RHO[x + 5 * y]);
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++)
                A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        A[0] ^= KECCAK_RC[round];
    }
}

/* sponge with rate 136 bytes, 32-byte output; domain 0x01 = Keccak256, 0x06 = SHA3-256 */
void bjo_keccak256(const uint8_t* data, size_t len, uint8_t* out32, int domain) {
    u64 A[25] = {0};
    uint8_t block[136];
    size_t off = 0;
    for (;;) {
        size_t take = len - off < 136 ? len - off : 136;
        int last = take < 136;
        memset(block, 0, sizeof(block));
        memcpy(block, data + off, take);
        off += take;
        if (last) {
            block[take] ^= (uint8_t)domain;
            block[135] ^= 0x80;
        }
        for (int i = 0; i < 17; i++) {
            u64 w = 0;
            for (int b = 0; b < 8; b++) w |= (u64)block[8 * i + b] << (8 * b);
            A[i] ^= w;
        }
        bjo_keccak_f1600(A);
        if (last) break;
    }
    for (int i = 0; i < 4; i++)
        for (int b = 0; b < 8; b++) out32[8 * i + b] = (uint8_t)(A[i] >> (8 * b));
}

static void keccak_leaf_strided(const u64* elems, size_t count, size_t stride, u64* out4) {
    uint8_t stackbuf[8 * 64] = {0};
    uint8_t* buf = count <= 64 ? stackbuf : (uint8_t*)malloc(8 * count);
    for (size_t i = 0; i < count; i++) {
        u64 v = gl_canon(elems[i * stride]);
        for (int b = 0; b < 8; b++) buf[8 * i + b] = (uint8_t)(v >> (8 * b));
    }
    bjo_keccak256(buf, 8 * count, (uint8_t*)out4, 0x01);
    if (buf != stackbuf) free(buf);
}

void bjo_keccak_leaf(const u64* elems, size_t count, u64* out4) { keccak_leaf_strided(elems, count, 1, out4); }

void bjo_keccak_node(const u64* l, const u64* r, u64* out4) {
    uint8_t buf[64];
    memcpy(buf, l, 32);
    memcpy(buf + 32, r, 32);
    bjo_keccak256(buf, 64, (uint8_t*)out4, 0x01);
}

/* ------------------------------------------------------------ Merkle (a19) */

/* tree hashers: 0 = GoldilocksPoseidon2Sponge<AbsorptionModeOverwrite>, 1 = Blake2s256,
 * 2 = Keccak256 */
typedef struct {
    const u64* lde; size_t col_stride; uint32_t n_cols; u64* leaves;
    const u64* prev; u64* next; int hasher;
} mk_ctx_t;

static void hash_node_h(int hasher, const u64* l, const u64* r, u64* out4) {
    if (hasher == 1) bjo_blake2s_node(l, r, out4);
    else if (hasher == 2) bjo_keccak_node(l, r, out4);
    else bjo_hash_into_node(l, r, out4);
}

static void leaf_job(void* c, size_t b, size_t e) {
    mk_ctx_t* x = (mk_ctx_t*)c;
    for (size_t L = b; L < e; L++) {
        if (x->hasher == 1) b2s_leaf_strided(x->lde + L, x->n_cols, x->col_stride, x->leaves + 4 * L);
        else if (x->hasher == 2) keccak_leaf_strided(x->lde + L, x->n_cols, x->col_stride, x->leaves + 4 * L);
        else leaf_hash_strided(x->lde + L, x->n_cols, x->col_stride, x->leaves + 4 * L);
    }
}

static void node_job(void* c, size_t b, size_t e) {
    mk_ctx_t* x = (mk_ctx_t*)c;
    for (size_t i = b; i < e; i++) hash_node_h(x->hasher, x->prev + 8 * i, x->prev + 8 * i + 4, x->next + 4 * i);
}

/* MerkleTreeWithCap::construct, cs/oracle/merkle_tree.rs:78-172.
 * lde: n_cols columns, column c's leaf-domain values at lde[c * col_stride + L] with
 * the flat leaf index L = coset * n + row (the coset-major concatenation of
 * ArcGenericLdeStorage cosets, :112-141).  Leaves are hashed per coset and row
 * chunk as in the reference (the work split does not change the values).
 * leaves: n_leaves x 4.  nodes: all node levels from the leaves up to and including
 * the cap level, concatenated (n_leaves/2 + n_leaves/4 + ... + cap_size) x 4
 * (node_hashes_enumerated_from_leafs, :388-449).  Returns the number of node levels. */
/* The leaf hashes alone (the reference's leaf loop, :112-157) ... */
void bjo_merkle_leaves_with(const u64* lde, size_t col_stride, uint32_t n_cols, size_t n_leaves, u64* leaves,
                            int threads, int hasher) {
    mk_ctx_t x = {lde, col_stride, n_cols, leaves, NULL, NULL, hasher};
    worker_scope(threads, n_leaves, leaf_job, &x);
}

/* The same leaves absorbed over a column range (the sponge is sequential over the row's
 * elements, sponge.rs:224-239): cap_in holds the 4 capacity words per leaf after the columns
 * before this range (NULL: fresh sponge); n_cols must be a multiple of 8 unless final, so the
 * range starts and ends on a rate boundary.  final == 0: out = capacity words (state[8..12))
 * after this range; final != 0: out = the leaf digests as bjo_merkle_leaves_with.  Lets a
 * caller hash a trace too large to hold whole, a column chunk at a time. */
typedef struct {
    const u64* lde;
    size_t col_stride;
    uint32_t n_cols;
    const u64* cap_in;
    u64* out;
    int final_;
} lp_ctx_t;

static void leaf_partial_job(void* c, size_t b, size_t e) {
    lp_ctx_t* x = (lp_ctx_t*)c;
    for (size_t L = b; L < e; L++) {
        u64 s[12] = {0};
        if (x->cap_in)
            for (int i = 0; i < 4; i++) s[8 + i] = x->cap_in[4 * L + i];
        size_t filled = 0;
        for (uint32_t i = 0; i < x->n_cols; i++) {
            s[filled++] = x->lde[(size_t)i * x->col_stride + L];
            if (filled == 8) { bjo_poseidon2_permutation(s); filled = 0; }
        }
        if (x->final_) {
            if (filled > 0) {
                for (size_t i = filled; i < 8; i++) s[i] = 0;
                bjo_poseidon2_permutation(s);
            }
            for (int i = 0; i < 4; i++) x->out[4 * L + i] = gl_canon(s[i]);
        } else {
            for (int i = 0; i < 4; i++) x->out[4 * L + i] = s[8 + i];
        }
    }
}

int bjo_poseidon2_leaves_partial(const u64* lde, size_t col_stride, uint32_t n_cols, size_t n_leaves,
                                 const u64* cap_in, u64* out, int final_, int threads) {
    if (!final_ && n_cols % 8 != 0) return -1;
    lp_ctx_t x = {lde, col_stride, n_cols, cap_in, out, final_};
    worker_scope(threads, n_leaves, leaf_partial_job, &x);
    return 0;
}

/* ... and the node levels over them (continue_from_leaf_hashes, :388-449). */
int bjo_merkle_nodes_with(const u64* leaves, size_t n_leaves, uint32_t cap_size, u64* nodes, int threads,
                          int hasher) {
    mk_ctx_t x = {NULL, 0, 0, NULL, NULL, NULL, hasher};
    int levels = 0;
    const u64* prev = leaves;
    u64* out = nodes;
    for (size_t len = n_leaves; len > cap_size; len /= 2) {
        x.prev = prev; x.next = out;
        worker_scope(threads, len / 2, node_job, &x);
        prev = out; out += 4 * (len / 2); levels++;
    }
    return levels;
}

int bjo_merkle_construct_with(const u64* lde, size_t col_stride, uint32_t n_cols, size_t n_leaves,
                              uint32_t cap_size, u64* leaves, u64* nodes, int threads, int hasher) {
    bjo_merkle_leaves_with(lde, col_stride, n_cols, n_leaves, leaves, threads, hasher);
    return bjo_merkle_nodes_with(leaves, n_leaves, cap_size, nodes, threads, hasher);
}

int bjo_merkle_construct(const u64* lde, size_t col_stride, uint32_t n_cols, size_t n_leaves,
                         uint32_t cap_size, u64* leaves, u64* nodes, int threads) {
    return bjo_merkle_construct_with(lde, col_stride, n_cols, n_leaves, cap_size, leaves, nodes, threads, 0);
}

/* get_proof, merkle_tree.rs:462-480.  Writes `levels` sibling digests. */
void bjo_merkle_get_proof(const u64* leaves, const u64* nodes, size_t n_leaves, int levels,
                          size_t idx, u64* leaf_out4, u64* path_out) {
    for (int i = 0; i < 4; i++) leaf_out4[i] = leaves[4 * idx + i];
    const u64* layer = leaves;
    size_t len = n_leaves;
    const u64* next_base = nodes;
    for (int l = 0; l < levels; l++) {
        size_t sib = idx ^ 1;
        for (int i = 0; i < 4; i++) path_out[4 * l + i] = layer[4 * sib + i];
        layer = next_base; next_base += 4 * (len / 2); len /= 2; idx >>= 1;
    }
}

/* verify_proof_over_cap, merkle_tree.rs:482-504 (digests compared after normalize_output:
 * canonical field elements for Poseidon2, the raw bytes for Blake2s) */
int bjo_verify_proof_over_cap_with(const u64* path, int levels, const u64* cap, const u64* leaf4, size_t idx,
                                   int hasher) {
    u64 cur[4], tmp[4];
    for (int i = 0; i < 4; i++) cur[i] = leaf4[i];
    for (int l = 0; l < levels; l++) {
        if ((idx & 1) == 0) hash_node_h(hasher, cur, path + 4 * l, tmp);
        else hash_node_h(hasher, path + 4 * l, cur, tmp);
        memcpy(cur, tmp, sizeof(cur));
        idx >>= 1;
    }
    for (int i = 0; i < 4; i++) {
        u64 a = cap[4 * idx + i], b = cur[i];
        if (hasher == 0) { a = gl_canon(a); b = gl_canon(b); }
        if (a != b) return 0;
    }
    return 1;
}

int bjo_verify_proof_over_cap(const u64* path, int levels, const u64* cap, const u64* leaf4, size_t idx) {
    return bjo_verify_proof_over_cap_with(path, levels, cap, leaf4, idx, 0);
}

/* ---------------------------------------------------- whole commit (a21) */

/* Witness commit as prover.rs:313-353: the LDE of every column at D = 2^log_d
 * (used_lde_degree = max(fri_lde_factor, quotient_degree), prover.rs:313, via
 * WitnessStorage::from_base_trace_ext, prover.rs:316-323), then the Merkle tree over
 * subset_for_degree(fri_lde_factor) of every column (prover.rs:325-347): the first
 * k = 2^log_k cosets (polynomial/lde.rs:298-308), i.e. leaf L < k * n of column c is
 * lde[c * D * n + L].  trace is overwritten with the monomials.  lde: n_cols x D x n;
 * leaves: k*n x 4; nodes: (k*n - cap) x 4; cap_out: cap_size x 4. */
int bjo_lde_commit_subset(u64* trace, uint32_t n_cols, uint32_t log_n, uint32_t log_d, uint32_t log_k,
                          uint32_t cap_size, u64* lde, u64* leaves, u64* nodes, u64* cap_out, int threads) {
    size_t n = (size_t)1 << log_n, nd = n << log_d, nl = n << log_k;
    bjo_lde(trace, n_cols, log_n, log_d, lde, threads);
    int levels = bjo_merkle_construct(lde, nd, n_cols, nl, cap_size, leaves, nodes, threads);
    const u64* top = leaves;
    if (levels > 0) {
        size_t off = 0, len = nl;
        for (int l = 0; l < levels - 1; l++) { off += len / 2; len /= 2; }
        top = nodes + 4 * off;
    }
    memcpy(cap_out, top, sizeof(u64) * 4 * cap_size);
    return levels;
}

/* All D cosets committed (fri_lde_factor == lde degree). */
int bjo_lde_commit(u64* trace, uint32_t n_cols, uint32_t log_n, uint32_t log_d, uint32_t cap_size,
                   u64* lde, u64* leaves, u64* nodes, u64* cap_out, int threads) {
    return bjo_lde_commit_subset(trace, n_cols, log_n, log_d, log_d, cap_size, lde, leaves, nodes, cap_out, threads);
}

/* Brute-force search for the leaf index of a proof.json query (fixture tool):
 * tries every path-bit pattern of `levels` bits; returns idx or -1. */
long bjo_find_query_index(const u64* leaf4, const u64* path, int levels, const u64* cap, size_t cap_size) {
    size_t combos = (size_t)1 << levels;
    for (size_t bits = 0; bits < combos; bits++) {
        u64 cur[4], tmp[4];
        memcpy(cur, leaf4, sizeof(cur));
        for (int l = 0; l < levels; l++) {
            if (((bits >> l) & 1) == 0) bjo_hash_into_node(cur, path + 4 * l, tmp);
            else bjo_hash_into_node(path + 4 * l, cur, tmp);
            memcpy(cur, tmp, sizeof(cur));
        }
        for (size_t c = 0; c < cap_size; c++)
            if (cap[4 * c] == cur[0] && cap[4 * c + 1] == cur[1] && cap[4 * c + 2] == cur[2] && cap[4 * c + 3] == cur[3])
                return (long)((c << levels) | bits);
    }
    return -1;
}
