/*
 * AVX-512 leaf hashing and LDE for the CPU BASELINE leg of bench.py -- test/bench
 * infrastructure, not the checker and not product code.
 *
 * The reference selects its AVX-512 field and Poseidon2 paths on an AVX-512 host
 * (field/goldilocks/mod.rs:36-75, avx512_impl.rs:357-428, poseidon2/state_avx512.rs) when built
 * with -C target-cpu=native, as its bench scripts do.  The scalar C restatement (boojum_oracle.c)
 * would understate that CPU, so the baseline's leaf hashing runs here on 8 leaves per 512-bit
 * vector (and its LDE on 8 butterflies per vector, below): the same permutation (poseidon2_permutation,
 * state_generic_impl.rs:221-236; MDS suggested_mds.rs:19-97; M_I :166-202) and sponge
 * (Overwrite, zero padding, sponge.rs:224-323), lane i hashing leaf L + i.  The Goldilocks
 * multiply is the 4 x 32x32 product + reduction of avx512_impl.rs:357-428 (mod.rs:186-199).
 * tests/test_oracle_baseline.py checks it against the scalar oracle bit for bit.
 *
 * Built into liboracle.so with per-function AVX-512 target attributes; bjo_avx512_available()
 * tells the caller whether the host can run it.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;

#define AVX512 __attribute__((target("avx512f,avx512dq,avx512vl")))

static const u64 RC[30][12] = {
#include "poseidon2_rc.inc"
};
static const int MI_SHIFT[12] = {4, 14, 11, 8, 0, 5, 2, 9, 13, 6, 3, 12};
static const u64 EPS = 0xFFFFFFFFull;

int bjo_avx512_available(void) {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq");
}

/* a + b mod p for any u64 a, b (add_assign_impl, goldilocks/mod.rs:213-231) */
AVX512 static inline __m512i vadd(__m512i a, __m512i b) {
    const __m512i eps = _mm512_set1_epi64((long long)EPS);
    __m512i s = _mm512_add_epi64(a, b);
    __mmask8 c1 = _mm512_cmplt_epu64_mask(s, a);
    __m512i t = _mm512_mask_add_epi64(s, c1, s, eps);
    __mmask8 c2 = c1 & _mm512_cmplt_epu64_mask(t, s);
    return _mm512_mask_add_epi64(t, c2, t, eps);
}

/* (hi:lo) mod p (from_u128_with_reduction, mod.rs:186-199) */
AVX512 static inline __m512i vreduce(__m512i lo, __m512i hi) {
    const __m512i eps = _mm512_set1_epi64((long long)EPS);
    __m512i hi_hi = _mm512_srli_epi64(hi, 32);
    __m512i hi_lo = _mm512_and_si512(hi, eps);
    __mmask8 b = _mm512_cmplt_epu64_mask(lo, hi_hi);
    __m512i t0 = _mm512_sub_epi64(lo, hi_hi);
    t0 = _mm512_mask_sub_epi64(t0, b, t0, eps);
    __m512i t1 = _mm512_sub_epi64(_mm512_slli_epi64(hi_lo, 32), hi_lo);
    __m512i r = _mm512_add_epi64(t0, t1);
    __mmask8 c = _mm512_cmplt_epu64_mask(r, t0);
    return _mm512_mask_add_epi64(r, c, r, eps);
}

/* a * b mod p (mul_assign_impl via 4 x mul_epu32, avx512_impl.rs:357-428) */
AVX512 static inline __m512i vmul(__m512i a, __m512i b) {
    __m512i ah = _mm512_srli_epi64(a, 32), bh = _mm512_srli_epi64(b, 32);
    __m512i p00 = _mm512_mul_epu32(a, b), p01 = _mm512_mul_epu32(a, bh);
    __m512i p10 = _mm512_mul_epu32(ah, b), p11 = _mm512_mul_epu32(ah, bh);
    __m512i mid = _mm512_add_epi64(p01, p10);
    __mmask8 cm = _mm512_cmplt_epu64_mask(mid, p01);
    __m512i lo = _mm512_add_epi64(p00, _mm512_slli_epi64(mid, 32));
    __mmask8 cl = _mm512_cmplt_epu64_mask(lo, p00);
    __m512i hi = _mm512_add_epi64(p11, _mm512_srli_epi64(mid, 32));
    hi = _mm512_mask_add_epi64(hi, cm, hi, _mm512_set1_epi64(1ll << 32));
    hi = _mm512_mask_add_epi64(hi, cl, hi, _mm512_set1_epi64(1));
    return vreduce(lo, hi);
}

/* x * 2^k mod p, k < 32: (x >> (64 - k)) : (x << k) as a 96-bit value */
AVX512 static inline __m512i vmul_pow2(__m512i x, int k) {
    if (k == 0) return x;
    __m512i lo = _mm512_slli_epi64(x, (unsigned)k);
    __m512i hi = _mm512_srli_epi64(x, (unsigned)(64 - k));
    return vreduce(lo, hi);
}

AVX512 static inline __m512i vsbox(__m512i x) {
    __m512i x2 = vmul(x, x), x3 = vmul(x2, x), x4 = vmul(x2, x2);
    return vmul(x4, x3);
}

AVX512 static inline void vm4(__m512i* x0, __m512i* x1, __m512i* x2, __m512i* x3) {
    __m512i t0 = vadd(*x0, *x1), t1 = vadd(*x2, *x3);
    __m512i t2 = vadd(vadd(*x1, *x1), t1);
    __m512i t3 = vadd(vadd(*x3, *x3), t0);
    __m512i t4 = vadd(vadd(vadd(t1, t1), vadd(t1, t1)), t3);
    __m512i t5 = vadd(vadd(vadd(t0, t0), vadd(t0, t0)), t2);
    __m512i t6 = vadd(t3, t5), t7 = vadd(t2, t4);
    *x0 = t6; *x1 = t5; *x2 = t7; *x3 = t4;
}

AVX512 static void vmds_ext(__m512i* s) {
    __m512i x[12];
    memcpy(x, s, sizeof(x));
    vm4(&x[0], &x[1], &x[2], &x[3]);
    vm4(&x[4], &x[5], &x[6], &x[7]);
    vm4(&x[8], &x[9], &x[10], &x[11]);
    for (int i = 0; i < 4; i++) {
        s[i] = vadd(vadd(vadd(x[i], x[i]), x[i + 4]), x[i + 8]);
        s[i + 4] = vadd(vadd(vadd(x[i + 4], x[i + 4]), x[i]), x[i + 8]);
        s[i + 8] = vadd(vadd(vadd(x[i + 8], x[i + 8]), x[i]), x[i + 4]);
    }
}

AVX512 static void vmds_int(__m512i* s) {
    __m512i sum = s[0];
    for (int i = 1; i < 12; i++) sum = vadd(sum, s[i]);
    for (int i = 0; i < 12; i++) s[i] = vadd(vmul_pow2(s[i], MI_SHIFT[i]), sum);
}

AVX512 static void vpermute(__m512i* s) {
    vmds_ext(s);
    int r = 0;
    for (int i = 0; i < 4; i++, r++) {
        for (int j = 0; j < 12; j++) s[j] = vsbox(vadd(s[j], _mm512_set1_epi64((long long)RC[r][j])));
        vmds_ext(s);
    }
    for (int i = 0; i < 22; i++, r++) {
        s[0] = vsbox(vadd(s[0], _mm512_set1_epi64((long long)RC[r][0])));
        vmds_int(s);
    }
    for (int i = 0; i < 4; i++, r++) {
        for (int j = 0; j < 12; j++) s[j] = vsbox(vadd(s[j], _mm512_set1_epi64((long long)RC[r][j])));
        vmds_ext(s);
    }
}

/* canonical(x): x - p when x >= p */
AVX512 static inline __m512i vcanon(__m512i x) {
    const __m512i p = _mm512_set1_epi64((long long)0xFFFFFFFF00000001ull);
    return _mm512_mask_sub_epi64(x, _mm512_cmpge_epu64_mask(x, p), x, p);
}

/* 8 leaves L0 .. L0+7 of MerkleTreeWithCap::construct's leaf loop (merkle_tree.rs:112-157):
 * leaf L = hash_into_leaf(src[0][L], ..., src[n_cols-1][L]) */
AVX512 static void leaves8(const u64* src, size_t col_stride, uint32_t n_cols, size_t L0, u64* out) {
    __m512i s[12];
    for (int i = 0; i < 12; i++) s[i] = _mm512_setzero_si512();
    uint32_t filled = 0;
    for (uint32_t c = 0; c < n_cols; c++) {
        s[filled++] = _mm512_loadu_si512((const void*)(src + (size_t)c * col_stride + L0));
        if (filled == 8) {
            vpermute(s);
            filled = 0;
        }
    }
    if (filled > 0) {
        for (uint32_t i = filled; i < 8; i++) s[i] = _mm512_setzero_si512();
        vpermute(s);
    }
    u64 t[4][8];
    for (int j = 0; j < 4; j++) _mm512_storeu_si512((void*)t[j], vcanon(s[j]));
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 4; j++) out[4 * (L0 + i) + j] = t[j][i];
}

typedef struct {
    const u64* src;
    size_t col_stride;
    uint32_t n_cols;
    u64* out;
    size_t begin, end;  /* in groups of 8 leaves */
} vjob_t;

AVX512 static void* vjob_run(void* p) {
    vjob_t* j = (vjob_t*)p;
    for (size_t g = j->begin; g < j->end; g++) leaves8(j->src, j->col_stride, j->n_cols, 8 * g, j->out);
    return NULL;
}

/* The leaf hashes of n_leaves (a multiple of 8) leaves, Worker-style: ceil-chunked over
 * `threads` threads (worker/mod.rs:34-66).  Returns -1 when the host lacks AVX-512. */
int bjo_merkle_leaves_avx512(const u64* src, size_t col_stride, uint32_t n_cols, size_t n_leaves, u64* out,
                             int threads) {
    if (!bjo_avx512_available() || n_leaves % 8) return -1;
    size_t groups = n_leaves / 8;
    if (threads < 1) threads = 1;
    size_t chunk = (groups + threads - 1) / threads;
    int nt = (int)((groups + chunk - 1) / chunk);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nt);
    vjob_t* jobs = (vjob_t*)malloc(sizeof(vjob_t) * nt);
    for (int t = 0; t < nt; t++) {
        jobs[t] = (vjob_t){src, col_stride, n_cols, out, t * chunk, (t + 1) * chunk < groups ? (t + 1) * chunk : groups};
        pthread_create(&th[t], NULL, vjob_run, &jobs[t]);
    }
    for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    return 0;
}

/* ------------------------------------------------------------------ LDE (baseline) */
/* The baseline's coset LDE (transform_raw_storages_to_lde, utils.rs:270-403) with the CT
 * butterflies of serial_ct_ntt_natural_to_bitreversed (fft/mod.rs:659-734) run 8 pairs per
 * vector wherever a group has >= 8 pairs (the MixedGL path's idea, fft/mod.rs:852-1077); the
 * last three stages, the bit reversal and the twiddle tables stay scalar.  Same values as
 * bjo_lde (checked in tests/test_oracle_baseline.py). */
void bjo_precompute_twiddles(uint32_t log_n, int inverse, u64* out);
void bjo_bitreverse_inplace(u64* a, size_t n);
void bjo_lde_cosets(uint32_t log_n, uint32_t log_d, u64* out);
u64 bjo_gl_mul(u64 a, u64 b);
u64 bjo_gl_inv(u64 a);

AVX512 static inline __m512i vsub(__m512i a, __m512i b) {
    const __m512i eps = _mm512_set1_epi64((long long)EPS);
    __m512i d = _mm512_sub_epi64(a, b);
    __mmask8 b1 = _mm512_cmplt_epu64_mask(a, b);
    __m512i t = _mm512_mask_sub_epi64(d, b1, d, eps);
    __mmask8 b2 = b1 & _mm512_cmplt_epu64_mask(d, eps);
    return _mm512_mask_sub_epi64(t, b2, t, eps);
}

static inline u64 s_add(u64 a, u64 b) {
    u64 s = a + b;
    if (s < a) { u64 t = s + EPS; if (t < s) t += EPS; s = t; }
    return s;
}
static inline u64 s_sub(u64 a, u64 b) {
    u64 d = a - b;
    if (a < b) { u64 t = d - EPS; if (d < EPS) t -= EPS; d = t; }
    return d;
}

AVX512 static void vct_ntt(u64* a, size_t n, const u64* tw) {
    if (n == 1) return;
    size_t pairs = n / 2, groups = 1;
    while (groups < n) {
        for (size_t k = 0; k < groups; k++) {
            u64* lo = a + k * pairs * 2;
            u64* hi = lo + pairs;
            const u64 s = k == 0 ? 1 : tw[k];   /* the first stage's twiddle is 1 (:678-699) */
            if (pairs >= 8) {
                const __m512i w = _mm512_set1_epi64((long long)s);
                for (size_t j = 0; j < pairs; j += 8) {
                    __m512i u = _mm512_loadu_si512((const void*)(lo + j));
                    __m512i v = _mm512_loadu_si512((const void*)(hi + j));
                    if (groups > 1) v = vmul(v, w);
                    _mm512_storeu_si512((void*)(hi + j), vsub(u, v));
                    _mm512_storeu_si512((void*)(lo + j), vadd(u, v));
                }
            } else {
                for (size_t j = 0; j < pairs; j++) {
                    u64 u = lo[j], v = groups > 1 ? bjo_gl_mul(hi[j], s) : hi[j];
                    hi[j] = s_sub(u, v);
                    lo[j] = s_add(u, v);
                }
            }
        }
        pairs /= 2;
        groups *= 2;
    }
}

/* x[i] *= scale * e^i */
AVX512 static void vdistribute(u64* a, size_t n, u64 e, u64 scale) {
    if (n < 8) {
        u64 s = scale;
        for (size_t i = 0; i < n; i++) { a[i] = bjo_gl_mul(a[i], s); s = bjo_gl_mul(s, e); }
        return;
    }
    u64 p[8];
    p[0] = scale;
    for (int i = 1; i < 8; i++) p[i] = bjo_gl_mul(p[i - 1], e);
    __m512i pw = _mm512_loadu_si512((const void*)p);
    const __m512i step = _mm512_set1_epi64((long long)bjo_gl_mul(bjo_gl_mul(bjo_gl_mul(e, e), bjo_gl_mul(e, e)),
                                                                  bjo_gl_mul(bjo_gl_mul(e, e), bjo_gl_mul(e, e))));
    for (size_t i = 0; i < n; i += 8) {
        _mm512_storeu_si512((void*)(a + i), vmul(_mm512_loadu_si512((const void*)(a + i)), pw));
        pw = vmul(pw, step);
    }
}

AVX512 static void vcanon_all(u64* a, size_t n) {
    size_t i = 0;
    for (; i + 8 <= n; i += 8) _mm512_storeu_si512((void*)(a + i), vcanon(_mm512_loadu_si512((const void*)(a + i))));
    for (; i < n; i++) if (a[i] >= 0xFFFFFFFF00000001ull) a[i] -= 0xFFFFFFFF00000001ull;
}

typedef struct {
    u64* cols; size_t n; const u64* tw; u64* lde; uint32_t n_cols, d; const u64* cosets;
    int phase; size_t begin, end;
} vlde_t;

AVX512 static void* vlde_run(void* p) {
    vlde_t* x = (vlde_t*)p;
    for (size_t job = x->begin; job < x->end; job++) {
        if (x->phase == 0) {
            /* ifft_natural_to_natural (fft/mod.rs:464-491): CT with inverse twiddles, bit
             * reversal, times n^-1 */
            u64* c = x->cols + job * x->n;
            vct_ntt(c, x->n, x->tw);
            bjo_bitreverse_inplace(c, x->n);
            if (x->n > 1) vdistribute(c, x->n, 1, bjo_gl_inv((u64)x->n));
            vcanon_all(c, x->n);
        } else {
            /* fft_natural_to_bitreversed with coset i (utils.rs:355-379 job order) */
            size_t coset = job / x->n_cols, col = job % x->n_cols;
            u64* dst = x->lde + (col * x->d + coset) * x->n;
            memcpy(dst, x->cols + col * x->n, x->n * sizeof(u64));
            vdistribute(dst, x->n, x->cosets[coset], 1);
            vct_ntt(dst, x->n, x->tw);
            vcanon_all(dst, x->n);
        }
    }
    return NULL;
}

static void vscope(int threads, size_t work, vlde_t* proto) {
    if (threads < 1) threads = 1;
    size_t chunk = (work + threads - 1) / threads;
    int nt = chunk ? (int)((work + chunk - 1) / chunk) : 0;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (nt ? nt : 1));
    vlde_t* jobs = (vlde_t*)malloc(sizeof(vlde_t) * (nt ? nt : 1));
    for (int t = 0; t < nt; t++) {
        jobs[t] = *proto;
        jobs[t].begin = t * chunk;
        jobs[t].end = (t + 1) * chunk < work ? (t + 1) * chunk : work;
        pthread_create(&th[t], NULL, vlde_run, &jobs[t]);
    }
    for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
}

/* As bjo_lde (trace overwritten with the monomials; lde n_cols x D x n); -1 without AVX-512. */
int bjo_lde_avx512(u64* trace, uint32_t n_cols, uint32_t log_n, uint32_t log_d, u64* lde, int threads) {
    if (!bjo_avx512_available()) return -1;
    size_t n = (size_t)1 << log_n, d = (size_t)1 << log_d;
    u64* tw = (u64*)malloc(sizeof(u64) * (n / 2 > 0 ? n / 2 : 1));
    u64* cosets = (u64*)malloc(sizeof(u64) * d);
    bjo_lde_cosets(log_n, log_d, cosets);
    vlde_t x = {trace, n, tw, lde, n_cols, (uint32_t)d, cosets, 0, 0, 0};
    if (n >= 2) bjo_precompute_twiddles(log_n, 1, tw);
    vscope(threads, n_cols, &x);
    if (n >= 2) bjo_precompute_twiddles(log_n, 0, tw);
    x.phase = 1;
    vscope(threads, (size_t)n_cols * d, &x);
    free(tw);
    free(cosets);
    return 0;
}
