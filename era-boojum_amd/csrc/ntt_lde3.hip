// Three-pass coset LDE for 2^18 <= n <= 2^23 (R = log n - 13 = 5..10).
//
// The reference computes D coset FFTs of the same monomials (transform_monomials_to_lde,
// cs/implementations/utils.rs:311-403): per coset distribute_powers + the natural->bit-reversed
// CT network (fft/mod.rs:308-317, 659-734).  The two-pass form (ntt_ct.hip) runs every transform
// as a head of R stages and a tail of 13; the inverse tail writes the monomials, and the forward
// head gathers them back once per coset.  Here the inverse tail and the first 13 stages of all D
// forward transforms share one block:
//
//   block q of the inverse tail (positions [8192 q, 8192 (q+1)) of the bit-reversed monomial
//   array) holds c_j for j = bitrev_13(l) 2^R + bitrev_R(q), l < 8192: every j with the same low
//   R bits, and the forward network's stages 0..12 (pair distances 2^(log n - 1) .. 2^R) only
//   ever pair such j.  So one block runs the inverse's last 13 stages, keeps the monomials in
//   registers, and for each coset runs forward stages 0..12 on them.
//
// Pass 1  inverse head (ntt_ct.hip, launch_ct_inverse_head): trace -> scratch.
// Pass 2  lde3_mid_kernel: scratch block q -> inverse stages R..R+12 -> (optionally the canonical
//         monomials back to scratch: bj_lde_d's contract) -> per coset: forward stages 0..12
//         (phases A, B in the power-of-two form, C general) -> 2^R runs of W = 2^(13-R) words,
//         run T of block q written to [T 8192 + q' W, + W) of the coset's column, q' = (q mod 32)
//         2^(R-5) + (q >> 5) (a row rotation, so pass 3 loads its rows contiguously).
// Pass 3  lde3_final_kernel: region T (8192 contiguous words: rows q < 2^R of W values M =
//         T W + o) -> the last R forward stages on each M's 2^R values (rows in bit-reversed
//         order: r = bitrev_R(q)) -> the region in natural order, o 2^R + r.  In place.
//
// Same field operations as the reference network, so the canonical outputs are bit-identical.
// Per column: reads n + D n + D n, writes n (+ n monomials) + D n + D n words, against 4 n + 4 D n
// in the two-pass form.
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "gl_asm.hpp"
#include "ntt_pow2.hpp"
#include "ntt_ct_common.hpp"
#include "bj_internal.hpp"

namespace bj {

namespace {

// table of one coset shift s (launch_lde3_table), for log n = R + 13:
//   [L3_C, +8192)        sigma_10(G)^((n/8192) j) at 8 G + j                    (forward phase C)
//   [L3_HA, +32)         s^((n/32) k)                                  (forward phase A)
//   [L3_HB, +1024)       sigma_5(g)^((n/1024) k) at 32 g + k            (forward phase B)
//   [L3_F1, +2^18)       sigma_13(M)^(2^(R-5) k) at k 8192 + M          (final phase 1)
//   [L3_U, +2^R)         w_{2^R}^(bitrev_5(p) rl) at p 2^(R-5) + rl     (final phase 2, universal)
//   [L3_A, +n/32)        sigma_13(M)^rl at rl 8192 + M                  (final phase 2)
//   [L3_F2, +n) (R > 5)  sigma_18(32 M + p)^rl at (32 rl + p) 8192 + M  (final phase 2, tabulated)
// with sigma_u(g) = s w_n^bitrev_u(g), the coset of group g after u stages.  Phase 2's factor
// sigma_18(32 M + p)^rl = A[rl][M] U[p][rl], since sigma_18(32 M + p) = sigma_13(M) w_{2^R}^bitrev_5(p).
// F1, A and F2 are laid out M-fastest, so the W lanes of a final block that share a row read
// consecutive words.
constexpr size_t L3_C = 0;
constexpr size_t L3_HA = 8192;
constexpr size_t L3_HB = L3_HA + 32;
constexpr size_t L3_F1 = L3_HB + 1024;
constexpr size_t L3_U = L3_F1 + ((size_t)1 << 18);
constexpr size_t L3_A = L3_U + 1024;
constexpr size_t L3_F2 = L3_A + ((size_t)1 << 18);

__host__ __device__ constexpr uint32_t cbrev(uint32_t x, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; i++) r |= ((x >> i) & 1u) << (bits - 1 - i);
    return r;
}

__device__ __forceinline__ uint32_t brev(uint32_t x, int bits) {
    return bits == 0 ? 0u : (__builtin_bitreverse32(x) >> (32 - bits));
}

// y[k] = x[bitrev_5(k)] * f[k]: a prescale whose inputs sit in bit-reversed register order
// (general products, any u64 representative)
__device__ __forceinline__ void prescale32_brev(uint64_t* y, const uint64_t* x, const uint64_t* f) {
#pragma unroll
    for (int k = 0; k < PT; k += 4) {
        uint32_t z0[4], z1[4];
        const uint64_t a0 = x[cbrev(k, 5)], a1 = x[cbrev(k + 1, 5)], a2 = x[cbrev(k + 2, 5)], a3 = x[cbrev(k + 3, 5)];
        glasm::mul_x4((uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)f[k], (uint32_t)(f[k] >> 32), z0[0], z1[0],
                      (uint32_t)a1, (uint32_t)(a1 >> 32), (uint32_t)f[k + 1], (uint32_t)(f[k + 1] >> 32), z0[1], z1[1],
                      (uint32_t)a2, (uint32_t)(a2 >> 32), (uint32_t)f[k + 2], (uint32_t)(f[k + 2] >> 32), z0[2], z1[2],
                      (uint32_t)a3, (uint32_t)(a3 >> 32), (uint32_t)f[k + 3], (uint32_t)(f[k + 3] >> 32), z0[3],
                      z1[3]);
#pragma unroll
        for (int i = 0; i < 4; i++) y[k + i] = join2(z0[i], z1[i]);
    }
}

// A raw buffer descriptor whose base is provably wave-uniform (readfirstlane on both halves:
// otherwise every buffer access through it becomes a waterfall loop)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const uint64_t* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, (int)bytes, 0x00020000);
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x2 as_u32x2(uint64_t v) {
    u32x2 r;
    r.x = (uint32_t)v;
    r.y = (uint32_t)(v >> 32);
    return r;
}
__device__ __forceinline__ uint64_t from_u32x2(u32x2 v) { return ((uint64_t)v.y << 32) | v.x; }

// y[k] = x[bitrev_5(k)] * h[k] with h wave-uniform (the phase-A factors s^((n/32) k), one table per
// coset): the factors stay in SGPRs (scalar loads, mul_sb_x4), so they take no VGPRs next to the
// monomials, the phase's values and its output
__device__ __forceinline__ void prescale32_brev_uniform(uint64_t* y, const uint64_t* x, const uint64_t* __restrict__ h) {
    // the factors 8 at a time (one 64-byte scalar load): a scalar load's wait cannot be deferred
    // past the next one (lgkmcnt(0)), so fewer, wider loads halve the waits
#pragma unroll
    for (int k8 = 0; k8 < PT; k8 += 8) {
        uint64_t hf[8];
#pragma unroll
        for (int i = 0; i < 8; i++) hf[i] = h[k8 + i];
#pragma unroll
        for (int k = k8; k < k8 + 8; k += 4) {
            uint32_t z0[4], z1[4];
            const uint64_t a0 = x[cbrev(k, 5)], a1 = x[cbrev(k + 1, 5)], a2 = x[cbrev(k + 2, 5)], a3 = x[cbrev(k + 3, 5)];
            const uint64_t f0 = hf[k - k8], f1 = hf[k - k8 + 1], f2 = hf[k - k8 + 2], f3 = hf[k - k8 + 3];
            glasm::mul_sb_x4((uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)f0, (uint32_t)(f0 >> 32), z0[0], z1[0],
                             (uint32_t)a1, (uint32_t)(a1 >> 32), (uint32_t)f1, (uint32_t)(f1 >> 32), z0[1], z1[1],
                             (uint32_t)a2, (uint32_t)(a2 >> 32), (uint32_t)f2, (uint32_t)(f2 >> 32), z0[2], z1[2],
                             (uint32_t)a3, (uint32_t)(a3 >> 32), (uint32_t)f3, (uint32_t)(f3 >> 32), z0[3], z1[3]);
#pragma unroll
            for (int i = 0; i < 4; i++) y[k + i] = join2(z0[i], z1[i]);
        }
    }
}

// Phase C's factors of the middle pass, k = 8 g + j with j > 0 (j = 0 is 1): the e-th of the 28
// (e = 7 g + j - 1) loaded to f[k], for E0 <= e < E1
__device__ __forceinline__ constexpr int c_reg(int e) { return 8 * (e / 7) + e % 7 + 1; }
template <int E0, int E1>
__device__ __forceinline__ void load_c(uint64_t* f, const uint64_t* __restrict__ c) {
#pragma unroll
    for (int e = E0; e < E1; e++) f[c_reg(e)] = c[c_reg(e)];
}

// y[k] *= f[k] for the registers of the 28 with E0 <= e < E1 (groups of 4; general products)
template <int E0, int E1>
__device__ __forceinline__ void prescale_c(uint64_t* y, const uint64_t* f) {
#pragma unroll
    for (int q = E0 / 4; q < E1 / 4; q++) {
        int k[4];
#pragma unroll
        for (int i = 0; i < 4; i++) k[i] = c_reg(4 * q + i);
        uint32_t z0[4], z1[4];
        glasm::mul_x4((uint32_t)y[k[0]], (uint32_t)(y[k[0]] >> 32), (uint32_t)f[k[0]], (uint32_t)(f[k[0]] >> 32), z0[0],
                      z1[0], (uint32_t)y[k[1]], (uint32_t)(y[k[1]] >> 32), (uint32_t)f[k[1]],
                      (uint32_t)(f[k[1]] >> 32), z0[1], z1[1], (uint32_t)y[k[2]], (uint32_t)(y[k[2]] >> 32),
                      (uint32_t)f[k[2]], (uint32_t)(f[k[2]] >> 32), z0[2], z1[2], (uint32_t)y[k[3]],
                      (uint32_t)(y[k[3]] >> 32), (uint32_t)f[k[3]], (uint32_t)(f[k[3]] >> 32), z0[3], z1[3]);
#pragma unroll
        for (int i = 0; i < 4; i++) y[k[i]] = join2(z0[i], z1[i]);
    }
}

// Where coset i of a column starts: (i >> log_k) block_stride + (i mod 2^log_k) coset_stride, i.e.
// the cosets in blocks of 2^log_k (the collective commit's [block][c][m] layout, m = 2^log_k n);
// log_k >= log2(n_cosets) is the plain i coset_stride.  Wave-uniform (SGPRs).
__device__ __forceinline__ size_t coset_offset(uint32_t i, size_t coset_stride, size_t block_stride, uint32_t log_k) {
    return (size_t)(i >> log_k) * block_stride + (size_t)(i & ((1u << log_k) - 1)) * coset_stride;
}

// The inverse tail (ct_tail_kernel<., true>) on the registers of block q: local stages 0..12 of
// the block (the inverse's stages R..R+12), n^-1 in TA.  In: x[k] = the inverse head's output at
// block position t + 256 k; out: x[k] = c_j at block position l = 32 t + k, that is
// j = bitrev_13(l) 2^R + bitrev_R(q) (the monomials in bit-reversed order, any u64 representative).
template <int R>
__device__ __forceinline__ void inverse_tail13(uint64_t* x, const uint64_t* __restrict__ inv_tab, uint32_t q,
                                               uint32_t t, uint64_t* lds) {
    constexpr uint32_t LOGN = R + 13;
    const uint32_t ba = tail_base_a(t), bc = tail_base_c(t);
    const uint64_t* ext = inv_tab + ((size_t)1 << LOGN);
    uint64_t f[PT], wa[16], wb[16], wc[16];
    load32(f, ext + EXT_TA + (size_t)q * 32);
    prescale32(x, f);
    dft_p2<5, true, 0>(x);
    const uint32_t tlo = t & 7, thi = t >> 3;
    const uint32_t bb = tail_base_b(thi, tlo);
#pragma unroll
    for (int k = 0; k < PT; k++) lds[ba + tail_off_a(k)] = x[k];
    // the TB factors in quarters of 8 as the forward phase B's: two in flight, each landing
    // behind a quarter's products
    const uint64_t* tb = ext + ext_tb(R) + ((((size_t)q << 5) | thi) << 5);
#pragma unroll
    for (int k = 0; k < 16; k++) f[k] = tb[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++) x[k] = lds[bb + tail_off_b(k)];
    prescale_n<8>(x, f);
#pragma unroll
    for (int k = 16; k < 24; k++) f[k] = tb[k];
    prescale_n<8>(x + 8, f + 8);
#pragma unroll
    for (int k = 24; k < PT; k++) f[k] = tb[k];
    prescale_n<8>(x + 16, f + 16);
    prescale_n<8>(x + 24, f + 24);
    dft_p2<5, true, 0>(x);
    tw_ct_tailC<10>(wa, inv_tab, R, q, t);
    // same slots as the reads just made by this thread: no barrier needed before the writes
#pragma unroll
    for (int k = 0; k < PT; k++) lds[bb + tail_off_b(k)] = x[k];
    tw_ct_tailC<11>(wb, inv_tab, R, q, t);
    tw_ct_tailC<12>(wc, inv_tab, R, q, t);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++) x[k] = lds[bc + k];
    ct_stage<4>(x, wa);
    ct_stage<2>(x, wb);
    ct_stage<1>(x, wc);
}

// ------------------------------------------------------------------ middle pass
//
// LDS layouts of the forward exchanges (element m = position within the block after the
// forward stages, j = m 2^R + r; l = bitrev_13(m)), each bank-conflict free for its reads and
// writes (checked on the host, tests/test_lde3_layout.py):
//   phase A out, m = 256 k + bitrev_8(t)          l-padded: 33 t + bitrev_5(k)
//   phase B, m = 256 g + 8 k + b, g = bitrev_5(t & 31), b = bitrev_3(t >> 5)
//                                                 l-padded: 1056 (t >> 5) + (t & 31) + 33 bitrev_5(k)
//   phase C read, m = 32 t + k                    l-padded: s8 + (s8 >> 5) + 264 bitrev_5(k), s8 = bitrev_8(t)
//   phase C out, m = 32 t + k                     m-padded: 33 t + k
//   store, m = t + 256 k                          m-padded: t + (t >> 5) + 264 k
template <int R, bool INV_PART, bool MONO>
__global__ __launch_bounds__(NT, 2) void lde3_mid_kernel(const uint64_t* src, size_t src_stride, uint64_t* mono,
                                                         size_t mono_stride, uint64_t* lde, size_t col_stride,
                                                         size_t coset_stride, size_t block_stride, uint32_t log_k, uint32_t n_cols, uint32_t n_cosets,
                                                         const uint64_t* __restrict__ inv_tab,
                                                         const uint64_t* __restrict__ tabs, size_t tab_stride) {
    constexpr uint32_t LOGN = R + 13;
    constexpr int LW = 13 - R;
    constexpr uint32_t W = 1u << LW;
    __shared__ uint64_t lds[PAD_LDS];
    const uint32_t t = threadIdx.x;
    // columns fastest: the blocks of one q (same inverse-table slices) run together
    // (readfirstlane: the division runs on the VALU, and the block's bases belong in SGPRs)
    const uint32_t c = __builtin_amdgcn_readfirstlane(blockIdx.x % n_cols);
    const uint32_t q = __builtin_amdgcn_readfirstlane(blockIdx.x / n_cols);
    const uint64_t* blk = src + (size_t)c * src_stride + (size_t)q * TILE;
    const uint32_t ba = tail_base_a(t), bc = tail_base_c(t);
    uint64_t x[PT];
    {
        const auto rb = uniform_rsrc(blk, 8u * TILE);
#pragma unroll
        for (int k = 0; k < PT; k++)
            x[k] = from_u32x2(__builtin_amdgcn_raw_buffer_load_b64(rb, (int)(t * 8), k * 2048, 0));
    }
    if constexpr (INV_PART) {
        inverse_tail13<R>(x, inv_tab, q, t, lds);
    } else {
        // monomials already in bit-reversed order: re-deal the coalesced load to l = 32 t + k
#pragma unroll
        for (int k = 0; k < PT; k++) lds[ba + tail_off_a(k)] = x[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = lds[bc + k];
    }
    // x[k] = c_j at block position l = 32 t + k: j = bitrev_13(l) 2^R + bitrev_R(q)
    if constexpr (MONO) {
        // the canonical monomials back to the block (bj_lde_d's scratch contract), coalesced
        // through the tail's epilogue exchange (l-padded C writes, A reads)
#pragma unroll
        for (int k = 0; k < PT; k += 4) {
            uint64_t v[4] = {x[k], x[k + 1], x[k + 2], x[k + 3]};
            canon4(v);
#pragma unroll
            for (int i = 0; i < 4; i++) lds[bc + k + i] = v[i];
        }
        __syncthreads();
        const auto rm = uniform_rsrc(mono + (size_t)c * mono_stride + (size_t)q * TILE, 8u * TILE);
#pragma unroll
        for (int k = 0; k < PT; k++)
            __builtin_amdgcn_raw_buffer_store_b64(as_u32x2(lds[ba + tail_off_a(k)]), rm, (int)(t * 8), k * 2048, 0);
    }
    const uint32_t s8 = brev(t, 8);
    const uint32_t b1 = 33 * t;                                  // phase A out (l-padded)
    const uint32_t b2 = 1056 * (t >> 5) + (t & 31);              // phase B (l-padded)
    const uint32_t b3 = s8 + (s8 >> 5);                          // phase C read (l-padded)
    const uint32_t g5 = brev(t & 31, 5);                         // phase-B group of this thread
    // store: m = t + 256 k -> run T = (t >> LW) + k 2^(8-LW), word q W + (t & (W-1)) of it
    // rows in the region in rotated order, q' = (q mod 32) 2^(R-5) + (q >> 5): the final pass then
    // loads its phase-1 rows (q = 32 qh + k, k < 32, per thread) as the contiguous t + 256 k
    const uint32_t qrot = ((q & 31u) << (R - 5)) | (q >> 5);
    const uint32_t vo = ((t >> LW) << 13) + qrot * W + (t & (W - 1));
#pragma unroll 1
    for (uint32_t i = 0; i < n_cosets; i++) {
        const uint64_t* tab = tabs + (size_t)i * tab_stride;
        uint64_t y[PT], f[PT];
        // phase A (forward stages 0..4): register k holds m's top 5 bits bitrev_5(k)
        prescale32_brev_uniform(y, x, tab + L3_HA);
        dft_p2<5, false, 0>(y);
        __syncthreads();  // the previous coset's (or the monomial epilogue's) LDS reads are done
#pragma unroll
        for (int k = 0; k < PT; k++) lds[b1 + cbrev(k, 5)] = y[k];
        // phase B's factors in quarters of 8, two in flight (64 VGPRs of factors next to the
        // monomials and the phase's values spill): quarters 0, 1 ahead of the barrier, quarter
        // q + 2 issued once quarter q's products are formed, so each load has a quarter's
        // products to land behind
        const uint64_t* hb = tab + L3_HB + 32 * g5;
#pragma unroll
        for (int k = 0; k < 16; k++) f[k] = hb[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PT; k++) y[k] = lds[b2 + 33 * cbrev(k, 5)];
        // phase B (stages 5..9): group g5, coefficient distance n / 1024
        prescale_n<8>(y, f);
#pragma unroll
        for (int k = 16; k < 24; k++) f[k] = hb[k];
        prescale_n<8>(y + 8, f + 8);
#pragma unroll
        for (int k = 24; k < PT; k++) f[k] = hb[k];
        prescale_n<8>(y + 16, f + 16);
        prescale_n<8>(y + 24, f + 24);
        dft_p2<5, false, 0>(y);
#pragma unroll
        for (int k = 0; k < PT; k++) lds[b2 + 33 * cbrev(k, 5)] = y[k];
        // phase C's factors (28: the first of each group of 8 is 1): the first 16 issued before
        // the barrier (all 28 ahead of phase B's DFT spill 26 VGPRs), the other 12 once the
        // first 8 products are formed
        const uint64_t* fc = tab + L3_C + 32 * t;
        load_c<0, 16>(f, fc);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PT; k++) y[k] = lds[b3 + 264 * cbrev(k, 5)];
        // phase C (stages 10..12) as a power-of-two phase: the 8 elements m = 8 G + j of stage-10
        // group G = 4 t + (k >> 3) times sigma_10(G)^((n / 8192) j), then an 8-point DFT with w_8
        // (the CT network's twiddles CT13[2^u + (m >> (13 - u))] are these factors' powers
        // times 8th roots of unity)
        prescale_c<0, 8>(y, f);
        load_c<16, 28>(f, fc);
        prescale_c<8, 16>(y, f);
        prescale_c<16, 28>(y, f);
        dft_p2_groups<3, false>(y);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PT; k++) lds[bc + k] = y[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PT; k++) y[k] = lds[ba + tail_off_a(k)];
        // buffer stores: the coset column's base in the descriptor (SGPRs), the per-thread word
        // offset in voffset and each register's run offset k 2^(21 - LW) words in soffset (plain
        // stores made a 64-bit VGPR address per register)
        const auto rs = uniform_rsrc(lde + (size_t)c * col_stride + coset_offset(i, coset_stride, block_stride, log_k), 8u << LOGN);
#pragma unroll
        for (int k = 0; k < PT; k++)
            __builtin_amdgcn_raw_buffer_store_b64(as_u32x2(y[k]), rs, (int)(vo * 8), (int)((uint32_t)k << (24 - LW)),
                                                  0);
    }
}

// ------------------------------------------------------------- inverse tail + fold
//
// The collective commit's sender-side fold (collective.hip, G > D shards; shard.hip's
// fold_all_kernel on ct_tail_kernel<true, true>'s monomials) straight from the inverse tail's
// registers: for each target P < shards, h_u = sum_b c[u F + b] z[P F + b], u < n / F, canonical,
// at dst + P dst_shard_stride.  The F terms of an output are registers F i .. F i + F - 1 of one
// thread (block position l = 32 t + k), so the monomials never reach memory (C3 at G = 8: the
// inverse + fold 2.30 -> 1.95 ms per rank, profiles/r4u_probe_ab.log).  Each target's 8192 / F
// outputs of the block go out coalesced through one of two LDS halves (slot w + w / 32: the
// writes w = (32 / F) t + i and the reads w = t + 256 k are both conflict-free), one barrier per
// target.
constexpr uint32_t kInvFoldConsts = 256;
struct InvFoldZ {
    uint64_t z[kInvFoldConsts];  // z[P F + bitrev_F(a)] = (s_P^m)^a
};

// acc[i] (+)= x[F i + b] * zb for i < OUTS; with set, acc[i] = the product.
template <uint32_t OUTS, uint32_t F>
__device__ __forceinline__ void fold_term(uint64_t* acc, const uint64_t* x, uint32_t b, uint64_t zb, bool set) {
    const uint32_t z0 = (uint32_t)zb, z1 = (uint32_t)(zb >> 32);
#pragma unroll
    for (uint32_t i = 0; i < OUTS; i += 4) {
        uint32_t p0[4], p1[4], s0[4], s1[4];
        glasm::mul_sb_x4((uint32_t)x[F * i + b], (uint32_t)(x[F * i + b] >> 32), z0, z1, p0[0], p1[0],
                         (uint32_t)x[F * (i + 1) + b], (uint32_t)(x[F * (i + 1) + b] >> 32), z0, z1, p0[1], p1[1],
                         (uint32_t)x[F * (i + 2) + b], (uint32_t)(x[F * (i + 2) + b] >> 32), z0, z1, p0[2], p1[2],
                         (uint32_t)x[F * (i + 3) + b], (uint32_t)(x[F * (i + 3) + b] >> 32), z0, z1, p0[3], p1[3]);
        if (set) {
#pragma unroll
            for (int j = 0; j < 4; j++) acc[i + j] = join2(p0[j], p1[j]);
            continue;
        }
        glasm::add_x4((uint32_t)acc[i], (uint32_t)(acc[i] >> 32), p0[0], p1[0], s0[0], s1[0], (uint32_t)acc[i + 1],
                      (uint32_t)(acc[i + 1] >> 32), p0[1], p1[1], s0[1], s1[1], (uint32_t)acc[i + 2],
                      (uint32_t)(acc[i + 2] >> 32), p0[2], p1[2], s0[2], s1[2], (uint32_t)acc[i + 3],
                      (uint32_t)(acc[i + 3] >> 32), p0[3], p1[3], s0[3], s1[3]);
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i + j] = join2(s0[j], s1[j]);
    }
}

// (a, b) <- (a + b, a - b) on four pairs (any u64 in and out)
__device__ __forceinline__ void add_sub4(uint64_t* a, uint64_t* b) {
    uint32_t s0[4], s1[4], d0[4], d1[4];
    glasm::add_x4((uint32_t)a[0], (uint32_t)(a[0] >> 32), (uint32_t)b[0], (uint32_t)(b[0] >> 32), s0[0], s1[0],
                  (uint32_t)a[1], (uint32_t)(a[1] >> 32), (uint32_t)b[1], (uint32_t)(b[1] >> 32), s0[1], s1[1],
                  (uint32_t)a[2], (uint32_t)(a[2] >> 32), (uint32_t)b[2], (uint32_t)(b[2] >> 32), s0[2], s1[2],
                  (uint32_t)a[3], (uint32_t)(a[3] >> 32), (uint32_t)b[3], (uint32_t)(b[3] >> 32), s0[3], s1[3]);
    glasm::sub_x4((uint32_t)a[0], (uint32_t)(a[0] >> 32), (uint32_t)b[0], (uint32_t)(b[0] >> 32), d0[0], d1[0],
                  (uint32_t)a[1], (uint32_t)(a[1] >> 32), (uint32_t)b[1], (uint32_t)(b[1] >> 32), d0[1], d1[1],
                  (uint32_t)a[2], (uint32_t)(a[2] >> 32), (uint32_t)b[2], (uint32_t)(b[2] >> 32), d0[2], d1[2],
                  (uint32_t)a[3], (uint32_t)(a[3] >> 32), (uint32_t)b[3], (uint32_t)(b[3] >> 32), d0[3], d1[3]);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        a[j] = join2(s0[j], s1[j]);
        b[j] = join2(d0[j], d1[j]);
    }
}

// Target P's OUTS outputs of this thread (block positions OUTS t + i) out through LDS half P & 1,
// coalesced: one barrier per target (the other half's reads, a target earlier, are behind it).
template <uint32_t OUTS>
__device__ __forceinline__ void store_fold_target(const uint64_t* h, uint64_t* lds, uint32_t P, uint32_t t, uint64_t* dst,
                                                  size_t dst_col_stride, size_t dst_shard_stride, uint32_t c,
                                                  uint32_t q) {
    constexpr uint32_t BLK = NT * OUTS, HALF = PAD_LDS / 2;
    uint64_t* buf = lds + (P & 1) * HALF;
#pragma unroll
    for (uint32_t i = 0; i < OUTS; i++) {
        const uint32_t w = OUTS * t + i;
        buf[w + (w >> 5)] = h[i];
    }
    __syncthreads();
    const auto rs = uniform_rsrc(dst + (size_t)P * dst_shard_stride + (size_t)c * dst_col_stride + (size_t)q * BLK,
                                 8u * BLK);
#pragma unroll
    for (uint32_t k = 0; k < OUTS; k++) {
        const uint32_t w = t + NT * k;
        __builtin_amdgcn_raw_buffer_store_b64(as_u32x2(buf[w + (w >> 5)]), rs, (int)(t * 8), (int)(k * 2048), 0);
    }
}

template <int R, int LOG_F>
__global__ __launch_bounds__(NT, 2) void lde3_inv_fold_kernel(const uint64_t* src, size_t src_stride, uint64_t* dst,
                                                              size_t dst_col_stride, size_t dst_shard_stride,
                                                              uint32_t n_cols, uint32_t shards, uint32_t paired,
                                                              const uint64_t* __restrict__ inv_tab, InvFoldZ zc) {
    __shared__ uint64_t lds[PAD_LDS];
    const uint32_t t = threadIdx.x;
    // columns fastest, XCD-aware (as the final pass): blocks are dealt round-robin over the 8
    // XCDs, so the n_cols blocks of one q (the same inverse-tail factor slices, ~67 KB) sit at ids
    // 8 (q8 n_cols + c) + (q & 7), all on one XCD, and the slices reach that XCD's L2 once instead
    // of once per XCD (C3 at G = 8: 0.82 GB of factor reads per rank call with q spread over the
    // XCDs, profiles/r5zi_shard_pmc_summary.txt); 2^R, the number of q, is a multiple of 8
    const uint32_t rest = blockIdx.x >> 3;
    const uint32_t c = __builtin_amdgcn_readfirstlane(rest % n_cols);
    const uint32_t q = __builtin_amdgcn_readfirstlane(((rest / n_cols) << 3) | (blockIdx.x & 7));
    uint64_t x[PT];
    {
        const auto rb = uniform_rsrc(src + (size_t)c * src_stride + (size_t)q * TILE, 8u * TILE);
#pragma unroll
        for (int k = 0; k < PT; k++)
            x[k] = from_u32x2(__builtin_amdgcn_raw_buffer_load_b64(rb, (int)(t * 8), k * 2048, 0));
    }
    inverse_tail13<R>(x, inv_tab, q, t, lds);
    // x[k] = c_j at block position l = 32 t + k; output u = (8192 q + 32 t) / F + i of every target
    {
        constexpr uint32_t F = 1u << LOG_F, OUTS = PT / F, BLK = TILE / F, HALF = PAD_LDS / 2;
        static_assert(OUTS % 4 == 0 && BLK + BLK / 32 <= HALF, "fold layout");
        __syncthreads();  // the tail's last LDS reads are done before the halves are written
        if (paired) {
            // targets P and P + 1 (P even) fold with z and -z: their shifts s and s' differ by
            // w^(2^(ls-1)), and (s'/s)^m = -1 (tests/test_fold_pairing.py).  Register b carries
            // the exponent bitrev_F(b), odd exactly for b >= F/2, so with E = the even-exponent
            // terms and O = the odd ones, target P gets E + O and target P + 1 gets E - O: half the
            // products.  At F = 2 that is one CT butterfly per output pair, (c0 + z c1, c0 - z c1):
            // 26 instructions where two products and two sums took 44.
#pragma unroll 1
            for (uint32_t P = 0; P < shards; P += 2) {
                uint64_t h0[OUTS], h1[OUTS];
                if constexpr (F == 2) {
                    const uint64_t z = zc.z[P * F + 1];
#pragma unroll
                    for (uint32_t i = 0; i < OUTS; i++) {
                        h0[i] = x[2 * i];
                        h1[i] = x[2 * i + 1];
                    }
#pragma unroll
                    for (uint32_t i = 0; i < OUTS; i += 4)
                        ct_bfly_x4(h0[i], h1[i], h0[i + 1], h1[i + 1], h0[i + 2], h1[i + 2], h0[i + 3], h1[i + 3], z,
                                   z, z, z);
                } else {
                    uint64_t e[OUTS], o[OUTS];
#pragma unroll
                    for (uint32_t i = 0; i < OUTS; i++) e[i] = x[F * i];
#pragma unroll
                    for (uint32_t b = 1; b < F; b++)
                        fold_term<OUTS, F>(b < F / 2 ? e : o, x, b, zc.z[P * F + b], b == F / 2);
#pragma unroll
                    for (uint32_t i = 0; i < OUTS; i += 4)
                        for (int j = 0; j < 4; j++) {
                            h0[i + j] = e[i + j];
                            h1[i + j] = o[i + j];
                        }
#pragma unroll
                    for (uint32_t i = 0; i < OUTS; i += 4) add_sub4(h0 + i, h1 + i);
                }
#pragma unroll
                for (uint32_t i = 0; i < OUTS; i += 4) {
                    canon4(h0 + i);
                    canon4(h1 + i);
                }
                store_fold_target<OUTS>(h0, lds, P, t, dst, dst_col_stride, dst_shard_stride, c, q);
                store_fold_target<OUTS>(h1, lds, P + 1, t, dst, dst_col_stride, dst_shard_stride, c, q);
            }
            return;
        }
#pragma unroll 1
        for (uint32_t P = 0; P < shards; P++) {
            uint64_t h[OUTS];
#pragma unroll
            for (uint32_t i = 0; i < OUTS; i++) h[i] = x[F * i];
#pragma unroll
            for (uint32_t b = 1; b < F; b++) fold_term<OUTS, F>(h, x, b, zc.z[P * F + b], false);
#pragma unroll
            for (uint32_t i = 0; i < OUTS; i += 4) canon4(h + i);
            store_fold_target<OUTS>(h, lds, P, t, dst, dst_col_stride, dst_shard_stride, c, q);
        }
    }
}

// ------------------------------------------------------------------- final pass
//
// Region T of a coset's column: element (q, o) at q' W + o (q' the middle pass's row rotation),
// M = T W + o, r = bitrev_R(q).
// Phase 1 (stages 13..17, r's top 5 bits = q's low 5): thread (qh = t >> LW, o = t & (W-1)) holds
// q = 32 qh + k.  Phase 2 (stages 18..12+R, r's low R-5 bits): thread (o, pl = t >> LW) holds
// groups p = pl + 2^(R-5) h, register h 2^(R-5) + rl <-> r = 2^(R-5) p + rl.  Store: position
// P = t + 256 k = o 2^R + r.  LDS layouts (conflict-free or nearly, tests/test_lde3_layout.py):
// "r-order" slot(e) = e + (e >> 5), e = r W + o, for R >= 6; "P-order" e = o 2^R + r at R = 5.
template <int R>
__device__ __forceinline__ constexpr uint32_t fin_slot(uint32_t r, uint32_t o) {
    const uint32_t e = R == 5 ? (o << R) + r : r * (1u << (13 - R)) + o;
    return e + (e >> 5);
}
// (r, o) of the three access patterns for thread t, register k
template <int R>
__device__ __forceinline__ constexpr uint32_t fin_p1(uint32_t t, uint32_t k) {
    constexpr int LW = 13 - R;
    return fin_slot<R>((k << (R - 5)) + cbrev(t >> LW, R - 5), t & ((1u << LW) - 1));
}
template <int R>
__device__ __forceinline__ constexpr uint32_t fin_p2(uint32_t t, uint32_t k) {
    constexpr int LW = 13 - R;
    const uint32_t h = k >> (R - 5), rl = k & ((1u << (R - 5)) - 1);
    const uint32_t p = (t >> LW) + (h << (R - 5));
    return fin_slot<R>((p << (R - 5)) + rl, t & ((1u << LW) - 1));
}
template <int R>
__device__ __forceinline__ constexpr uint32_t fin_p3(uint32_t t, uint32_t k) {
    const uint32_t P = t + 256 * k;
    return fin_slot<R>(P & ((1u << R) - 1), P >> R);
}

// Phase factors: phase 1's sigma_13(M)^(2^(R-5) k) (F1) and phase 2's sigma_18(32 M + p)^rl.
// * F1: 32 W distinct words per block, each used by 2^(R-5) threads: for R >= 8 the block stages
//   its slice in LDS (W / 8 coalesced loads per thread instead of 32), else direct loads.
// * phase 2: F2MODE 0 (production) loads the tabulated F2 (one distinct word per element, 64 KiB
//   per block, shared by the columns in L2) at the kernel's start, so the loads overlap phase 1;
//   F2MODE 1 forms A[rl][M] U[p][rl] from slices staged in LDS (256 + 32 2^(R-5) words per block)
//   with one extra product per element.  C3 (tools/lde3_ablation.hip, profiles/r3d_lde3_ablation.log):
//   17.4 ms against 18.5; both loading F1 and F2 directly at their use: 21.0.
template <int R>
struct FinLds {
    static constexpr int LW = 13 - R, RL = R - 5;
    static constexpr uint32_t W = 1u << LW;
    static constexpr bool F1_LDS = R >= 8;
    static constexpr uint32_t F1 = F1_LDS ? 32 * W : 0;      // [k][o]
    static constexpr uint32_t A = (1u << RL) * W;             // [rl][o]
    static constexpr uint32_t UP = (1u << RL) + 1;            // padded row of U: [p][rl], p rows of UP
    static constexpr uint32_t U = 32 * UP;
};

template <int R, int F2MODE>
__global__ __launch_bounds__(NT, 2) void lde3_final_kernel(uint64_t* lde, size_t col_stride, size_t coset_stride, size_t block_stride, uint32_t log_k,
                                                           uint32_t n_cols, uint32_t n_cosets,
                                                           const uint64_t* __restrict__ tabs, size_t tab_stride) {
    using FL = FinLds<R>;
    constexpr int LW = FL::LW, RL = FL::RL;
    constexpr uint32_t W = FL::W;
    __shared__ uint64_t lds[PAD_LDS];
    __shared__ uint64_t lf1[FL::F1 ? FL::F1 : 1];
    __shared__ uint64_t la[R > 5 && F2MODE == 1 ? FL::A : 1];
    __shared__ uint64_t lu[R > 5 && F2MODE == 1 ? FL::U : 1];
    const uint32_t t = threadIdx.x;
    // columns fastest, XCD-aware: blocks are dealt round-robin over the 8 XCDs, so the n_cols
    // blocks of one (coset, region) pair sit at ids 8 (pair8 n_cols + c) + (pair & 7), all on one
    // XCD in one time window, and its table slices are fetched into that XCD's L2 once
    // (pairs = n_cosets 2^R, a multiple of 8)
    const uint32_t rest = blockIdx.x >> 3;
    const uint32_t c = __builtin_amdgcn_readfirstlane(rest % n_cols);
    const uint32_t pair = ((rest / n_cols) << 3) | (blockIdx.x & 7);
    const uint32_t i = __builtin_amdgcn_readfirstlane(pair % n_cosets);
    const uint32_t T = __builtin_amdgcn_readfirstlane(pair / n_cosets);
    uint64_t* d = lde + (size_t)c * col_stride + coset_offset(i, coset_stride, block_stride, log_k) + (size_t)T * TILE;
    const uint64_t* tab = tabs + (size_t)i * tab_stride;
    const uint32_t o = t & (W - 1);
    const uint32_t M0 = T * W, M = M0 + o;
    uint64_t x[PT], y[PT], f[PT];
    // region rows in the middle pass's rotated order (q' = (q mod 32) 2^(R-5) + (q >> 5)): word t + 256 k
    // is row q = 32 qh + k (qh = t >> LW), column o -- the phase-1 layout, loaded fully coalesced;
    // buffer loads (the region's base in SGPRs, 2 KiB steps in soffset): plain loads at
    // t + 256 k kept a 64-bit VGPR address per register and spilled
    const auto rd = uniform_rsrc(d, 8u * TILE);
    // the F1 slice (coalesced: consecutive threads, consecutive M) is loaded first and stored to
    // LDS after the region's and F2's loads are issued: loads retire in issue order for vmcnt, so
    // the LDS stores then wait for these few loads only, and the F2 loads leave with the region's
    // instead of after all of them have landed
    constexpr uint32_t NF1 = FL::F1_LDS ? FL::F1 / NT : 1;
    uint64_t f1v[NF1];
    if constexpr (FL::F1_LDS) {
#pragma unroll
        for (uint32_t j = 0; j < NF1; j++) {
            const uint32_t e = t + j * NT;
            f1v[j] = tab[L3_F1 + ((size_t)(e >> LW) << 13) + M0 + (e & (W - 1))];
        }
    }
#pragma unroll
    for (int k = 0; k < PT; k++) x[k] = from_u32x2(__builtin_amdgcn_raw_buffer_load_b64(rd, (int)(t * 8), k * 2048, 0));
    if constexpr (R > 5 && F2MODE == 1) {
        la[t] = tab[L3_A + ((size_t)(t >> LW) << 13) + M0 + (t & (W - 1))];
#pragma unroll
        for (uint32_t e = t; e < (32u << RL); e += NT) lu[(e >> RL) * FL::UP + (e & ((1u << RL) - 1))] = tab[L3_U + e];
    }
    uint64_t g2[F2MODE == 0 && R > 5 ? PT : 1];
    if constexpr (F2MODE == 0 && R > 5) {
        // tabulated phase-2 factors, issued early so their latency overlaps phase 1
        // buffer loads: the block's slice base in SGPRs, (32 rl + p) 8192 words in soffset
        const auto rf = uniform_rsrc(tab + L3_F2 + M0, 8u << (R + 13));
        const int vf = (int)((o + ((t >> LW) << 13)) * 8);
#pragma unroll
        for (int k = 0; k < PT; k++) {
            const uint32_t h = k >> RL, rl = k & ((1u << RL) - 1);
            g2[k] = from_u32x2(__builtin_amdgcn_raw_buffer_load_b64(rf, vf, (int)((rl * 32 + (h << RL)) << 16), 0));
        }
    }
    if constexpr (FL::F1_LDS) {
#pragma unroll
        for (uint32_t j = 0; j < NF1; j++) lf1[t + j * NT] = f1v[j];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PT; k++) f[k] = lf1[k * W + o];
    } else {
        const uint64_t* f1 = tab + L3_F1 + M;
#pragma unroll
        for (int k = 0; k < PT; k++) f[k] = f1[(size_t)k << 13];
    }
    // phase 1: prescale sigma_13(M)^(2^(R-5) k), DFT over r's top 5 bits
    prescale32_brev(y, x, f);
    dft_p2<5, false, 0>(y);
    const uint32_t b1 = fin_p1<R>(t, 0);
#pragma unroll
    for (int k = 0; k < PT; k++) lds[b1 + (fin_p1<R>(0, k) - fin_p1<R>(0, 0))] = y[k];
    if constexpr (R > 5) {
        // phase 2 factors for groups p = pl + 2^(R-5) h, register h 2^(R-5) + rl
        const uint32_t pl = t >> LW;
        if constexpr (F2MODE == 1) {
            if constexpr (!FL::F1_LDS) __syncthreads();  // la / lu written
            uint64_t a[PT];
#pragma unroll
            for (int k = 0; k < PT; k++) {
                const uint32_t h = k >> RL, rl = k & ((1u << RL) - 1);
                a[k] = la[rl * W + o];
                f[k] = lu[(pl + (h << RL)) * FL::UP + rl];
            }
            prescale32(f, a);
        } else {
#pragma unroll
            for (int k = 0; k < PT; k++) f[k] = g2[k];
        }
        __syncthreads();
        const uint32_t b2 = fin_p2<R>(t, 0);
#pragma unroll
        for (int k = 0; k < PT; k++) y[k] = lds[b2 + (fin_p2<R>(0, k) - fin_p2<R>(0, 0))];
        prescale32(y, f);
        dft_p2_groups<RL, false>(y);
        // same slots as this thread's reads: no barrier before the writes
#pragma unroll
        for (int k = 0; k < PT; k++) lds[b2 + (fin_p2<R>(0, k) - fin_p2<R>(0, 0))] = y[k];
    }
    __syncthreads();
    const uint32_t b3 = fin_p3<R>(t, 0);
#pragma unroll
    for (int k = 0; k < PT; k++) y[k] = lds[b3 + (fin_p3<R>(0, k) - fin_p3<R>(0, 0))];
#pragma unroll
    for (int k = 0; k < PT; k += 4) canon4(y + k);
#pragma unroll
    for (int k = 0; k < PT; k++) __builtin_amdgcn_raw_buffer_store_b64(as_u32x2(y[k]), rd, (int)(t * 8), k * 2048, 0);
}

// ------------------------------------------------------------------- table
__global__ void lde3_table_kernel(uint64_t* out, uint32_t log_n, uint64_t w_n, uint64_t s, size_t len) {
    const size_t n = (size_t)1 << log_n;
    const uint32_t R = log_n - 13;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < len;
         idx += (size_t)gridDim.x * blockDim.x) {
        uint64_t v;
        if (idx < L3_HA) {
            const uint32_t G = (uint32_t)idx >> 3, j = (uint32_t)idx & 7;
            const uint64_t sigma = gl::mul(s, gl::pow(w_n, gl::bitrev32(G, 10)));
            v = gl::pow(sigma, (n >> 13) * j);
        } else if (idx < L3_HB) {
            v = gl::pow(s, (n >> 5) * (idx - L3_HA));
        } else if (idx < L3_F1) {
            const uint32_t j = (uint32_t)(idx - L3_HB);
            const uint64_t sigma = gl::mul(s, gl::pow(w_n, gl::bitrev32(j >> 5, 5)));
            v = gl::pow(sigma, (n >> 10) * (j & 31));
        } else if (idx < L3_U) {
            const uint32_t j = (uint32_t)(idx - L3_F1);
            const uint32_t M = j & 8191, k = j >> 13;
            const uint64_t sigma = gl::mul(s, gl::pow(w_n, gl::bitrev32(M, 13)));
            v = gl::pow(sigma, (uint64_t)k << (R - 5));
        } else if (idx < L3_A) {
            // w_{2^R} = w_n^(2^13)
            const uint32_t j = (uint32_t)(idx - L3_U);
            const uint32_t p = j >> (R - 5), rl = j & ((1u << (R - 5)) - 1);
            v = (j >> R) ? 0 : gl::pow(gl::pow(w_n, 8192), (uint64_t)gl::bitrev32(p, 5) * rl);
        } else if (idx < L3_F2) {
            const uint32_t j = (uint32_t)(idx - L3_A);
            const uint32_t M = j & 8191, rl = j >> 13;
            const uint64_t sigma = gl::mul(s, gl::pow(w_n, gl::bitrev32(M, 13)));
            v = (rl >> (R - 5)) ? 0 : gl::pow(sigma, rl);
        } else {
            const size_t j = idx - L3_F2;
            const uint32_t M = (uint32_t)(j & 8191), rest = (uint32_t)(j >> 13);
            const uint32_t p = rest & 31, rl = rest >> 5;
            const uint64_t sigma = gl::mul(s, gl::pow(w_n, gl::bitrev32(M * 32 + p, 18)));
            v = gl::pow(sigma, rl);
        }
        out[idx] = gl::canon(v);
    }
}

template <int R>
void launch_lde3_R(uint64_t* lde, size_t col_stride, size_t coset_stride, size_t block_stride, uint32_t log_k, uint32_t n_cosets, const uint64_t* src,
                   size_t src_stride, uint64_t* mono, size_t mono_stride, uint32_t n_cols, const uint64_t* inv_tab,
                   const uint64_t* tabs, size_t tab_stride, hipStream_t st, uint32_t passes) {
    const dim3 gm(n_cols << R);
    if (!(passes & LDE3_MID))
        ;
    else if (inv_tab && mono)
        hipLaunchKernelGGL((lde3_mid_kernel<R, true, true>), gm, dim3(NT), 0, st, src, src_stride, mono, mono_stride,
                           lde, col_stride, coset_stride, block_stride, log_k, n_cols, n_cosets, inv_tab, tabs, tab_stride);
    else if (inv_tab)
        hipLaunchKernelGGL((lde3_mid_kernel<R, true, false>), gm, dim3(NT), 0, st, src, src_stride, mono,
                           mono_stride, lde, col_stride, coset_stride, block_stride, log_k, n_cols, n_cosets, inv_tab, tabs, tab_stride);
    else
        hipLaunchKernelGGL((lde3_mid_kernel<R, false, false>), gm, dim3(NT), 0, st, src, src_stride, mono,
                           mono_stride, lde, col_stride, coset_stride, block_stride, log_k, n_cols, n_cosets, inv_tab, tabs, tab_stride);
    const dim3 gf((n_cols * n_cosets) << R);
    if (passes & LDE3_FINAL)
        hipLaunchKernelGGL((lde3_final_kernel<R, 0>), gf, dim3(NT), 0, st, lde, col_stride, coset_stride, block_stride,
                           log_k, n_cols, n_cosets, tabs, tab_stride);
}

}  // namespace

bool lde3_supported(uint32_t log_n) { return log_n >= 18 && log_n <= 23; }

size_t lde3_table_len(uint32_t log_n) {
    return log_n > 18 ? L3_F2 + ((size_t)1 << log_n) : L3_F2;
}

hipError_t launch_lde3_table(uint64_t* out, uint32_t log_n, uint64_t shift, hipStream_t st) {
    if (!lde3_supported(log_n)) return hipErrorInvalidValue;
    const size_t len = lde3_table_len(log_n);
    size_t blocks = (len + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(lde3_table_kernel, dim3((unsigned)blocks), dim3(256), 0, st, out, log_n,
                       gl::domain_generator(log_n), gl::canon(shift), len);
    return hipGetLastError();
}

hipError_t launch_lde3(uint64_t* lde, size_t col_stride, size_t coset_stride, uint32_t n_cosets, const uint64_t* src,
                       size_t src_stride, uint64_t* mono, size_t mono_stride, uint32_t n_cols, uint32_t log_n,
                       const uint64_t* inv_tab, const uint64_t* tabs, size_t tab_stride, hipStream_t st,
                       uint32_t log_k, size_t block_stride, uint32_t passes) {
    if (n_cols == 0 || n_cosets == 0) return hipSuccess;
    if (log_k > 31) log_k = 31;
    if (!lde3_supported(log_n)) return hipErrorInvalidValue;
    // the final pass's grid: (n_cols n_cosets) 2^R blocks of NT threads, within 2^32 - 1 work-items
    if (((uint64_t)n_cols * n_cosets) << (log_n - 13) > (0xffffffffull / NT)) return hipErrorInvalidValue;
#define BJ_LDE3(RR)                                                                                              \
    launch_lde3_R<RR>(lde, col_stride, coset_stride, block_stride, log_k, n_cosets, src, src_stride, mono, mono_stride, n_cols, inv_tab, \
                      tabs, tab_stride, st, passes)
    switch (log_n - 13) {
        case 5: BJ_LDE3(5); break;
        case 6: BJ_LDE3(6); break;
        case 7: BJ_LDE3(7); break;
        case 8: BJ_LDE3(8); break;
        case 9: BJ_LDE3(9); break;
        default: BJ_LDE3(10); break;
    }
#undef BJ_LDE3
    return hipGetLastError();
}

namespace {
template <int R>
void launch_lde3_inv_fold_R(uint64_t* dst, size_t dst_col_stride, size_t dst_shard_stride, const uint64_t* src,
                            size_t src_stride, uint32_t n_cols, uint32_t log_f, uint32_t shards, uint32_t paired,
                            const uint64_t* inv_tab, const InvFoldZ& zc, hipStream_t st) {
    const dim3 g(n_cols << R);
#define BJ_INV(LF)                                                                                             \
    hipLaunchKernelGGL((lde3_inv_fold_kernel<R, LF>), g, dim3(NT), 0, st, src, src_stride, dst, dst_col_stride, \
                       dst_shard_stride, n_cols, shards, paired, inv_tab, zc)
    switch (log_f) {
        case 1: BJ_INV(1); break;
        case 2: BJ_INV(2); break;
        default: BJ_INV(3); break;
    }
#undef BJ_INV
}
}  // namespace

bool lde3_inv_fold_supported(uint32_t log_n, uint32_t log_f, uint32_t shards) {
    return lde3_supported(log_n) && log_f >= 1 && log_f <= 3 && shards >= 1 &&
           (size_t)shards << log_f <= kInvFoldConsts;
}

hipError_t launch_lde3_inv_fold(uint64_t* dst, size_t dst_col_stride, size_t dst_shard_stride, const uint64_t* src,
                                size_t src_stride, uint32_t n_cols, uint32_t log_n, uint32_t log_f, uint32_t shards,
                                const uint64_t* s_pow_m, const uint64_t* inv_tab, hipStream_t st) {
    if (n_cols == 0) return hipSuccess;
    if (!lde3_inv_fold_supported(log_n, log_f, shards)) return hipErrorInvalidValue;
    if (((uint64_t)n_cols << (log_n - 13)) > 0xffffffffull / NT) return hipErrorInvalidValue;
    InvFoldZ zc{};
    const uint32_t F = 1u << log_f;
    for (uint32_t P = 0; P < shards; P++) {
        uint64_t acc = 1;
        for (uint32_t a = 0; a < F; a++) {
            zc.z[P * F + gl::bitrev32(a, log_f)] = acc;
            acc = gl::mul(acc, s_pow_m[P]);
        }
    }
    // targets in pairs (2P', 2P' + 1) whose s^m are negatives of each other (the collective's
    // targets are, tests/test_fold_pairing.py): the even/odd form (at F = 2 the butterfly)
    uint32_t paired = shards % 2 == 0 && !knobs().inv_fold_unpaired;
    for (uint32_t P = 0; paired && P < shards; P += 2)
        paired = gl::canon(s_pow_m[P + 1]) == gl::canon(gl::sub(0, s_pow_m[P]));
#define BJ_INVR(RR) \
    launch_lde3_inv_fold_R<RR>(dst, dst_col_stride, dst_shard_stride, src, src_stride, n_cols, log_f, shards, paired, \
                               inv_tab, zc, st)
    switch (log_n - 13) {
        case 5: BJ_INVR(5); break;
        case 6: BJ_INVR(6); break;
        case 7: BJ_INVR(7); break;
        case 8: BJ_INVR(8); break;
        case 9: BJ_INVR(9); break;
        default: BJ_INVR(10); break;
    }
#undef BJ_INVR
    return hipGetLastError();
}

}  // namespace bj
