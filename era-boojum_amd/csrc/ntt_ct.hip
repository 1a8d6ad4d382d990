// Coset-folded Cooley-Tukey NTT passes for 2^13 <= n <= 2^26.
//
// The reference's transform is serial_ct_ntt_natural_to_bitreversed (fft/mod.rs:659-734):
// at the stage with 2^u groups, group k pairs (j, j + h) and does
//   (a, c) <- (a + mu_k c, a - mu_k c),   mu_k = omegas_bit_reversed[k] = w_{2^(u+1)}^bitrev_u(k).
// The coset FFT (fft/mod.rs:398-411) first multiplies x_j by s^j (distribute_powers,
// :308-317). That shift folds into the butterflies. After stage u, group k evaluates its
// half-size polynomial on the coset sigma_k <w_m> with sigma_k = s * w_n^bitrev_u(k). So the
// shifted transform is the same network with
//   mu_k(s) = s^(n >> (u+1)) * w_{2^(u+1)}^bitrev_u(k)
// and no per-element powers at all. Same field values, so outputs (canonicalised) are
// bit-identical to the reference's.
//
// Twiddle table per shift: CT[2^u + k] = mu_k(s), for u < log n, k < 2^u (n entries, CT[0]
// unused), followed by the prescale tables of the power-of-two register phases (below). The
// inverse transform returns the monomials themselves (utils.rs:295-304 after ifft's x n^-1),
// not n * monomials: n^-1 sits in the tail's TA table (2^13, 2^18..2^23), or in CT[1] with the
// general heads multiplying their stage-0 lower operands by it.
//
// Register phases of <= 5 stages (the tail's A and B, the 2^18..2^23 heads' A' and B') run as
// a prescale by powers of the group's coset shift and a DFT with twiddles +-2^e
// (csrc/ntt_pow2.hpp); the tail's phase C and the other heads keep mu_k(s).
//
// Tiling: each thread holds 32 elements in VGPRs and runs up to five
// stages in registers; LDS (XOR-swizzled) only re-deals elements between register phases.
// * head: the first R = log n - 13 stages on tiles of 2^R rows x 2^(13-R) adjacent columns.
//   Stage v's group index is the row's top v bits, so in phase A' the twiddles are
//   wave-uniform (scalar loads) and in phase B' a per-thread base + constant.
// * tail: the last 13 stages on contiguous 8192-element blocks, with the group index
//   (q << v) + (offset >> (13 - v)) for tile q. A tile reads its own 8191-entry slice of the
//   table, and all columns (blockIdx.x) of one tile share that slice in L2.
// MODE 1 heads gather a bit-reversed source (the iNTT output, c_j at bitrev_n(j)) in runs of
// 2^R words, so the iFFT's bit reversal (fft/mod.rs:481) never costs a pass of its own.
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "gl_asm.hpp"
#include "ntt_pow2.hpp"
#include "ntt_ct_common.hpp"
#include "bj_internal.hpp"

namespace bj {

namespace {

// ------------------------------------------------------------------- head

template <int LOGW>
__device__ __forceinline__ uint32_t swz_head(uint32_t e) {
    constexpr uint32_t m = LOGW >= 5 ? 0u : ((32u >> LOGW) - 1u);
    return e ^ (((e >> (5 + LOGW)) & m) << LOGW);
}

// LDS slot of the MODE 1 gather staging: XOR the low 4 bits of the 13-bit tile index with its
// top 4 bits (the top bits of the row). A 16-lane ds_write_b64 group writes one column of 16
// rows whose top bits are bitrev(sg) (all different), so its 16 slots are distinct mod 16;
// a 32-lane ds_read_b64 half reads an aligned run of 32 indices, which the XOR maps onto itself.
__device__ __forceinline__ uint32_t swz_gather(uint32_t e) { return e ^ ((e >> 9) & 15); }

// Phase A' twiddles of stage v (register distance 16 >> v): pair q's group is lo(q) >> (5 - v),
// the same for every thread.
// gbase = 1 for a whole column; (2^u0 + g) for sub-column g of a column whose first u0 stages
// are already done (the group index of global stage u0 + v is (g << v) + the local group).
template <int V>
__device__ __forceinline__ void tw_ct_headA(uint64_t* w, const uint64_t* __restrict__ ct, uint32_t gbase) {
    constexpr int HK = 16 >> V;
    const uint64_t* base = ct + ((size_t)gbase << V);
#pragma unroll
    for (int q = 0; q < 16; q++) w[q] = base[pair_lo(q, HK) >> (5 - V)];
}

// Phase B' twiddles of stage v >= 5 (rows 32 s + k, register distance 2^(R-1-v)):
// group (32 s + lo(q)) >> (R - v).
template <int R, int V>
__device__ __forceinline__ void tw_ct_headB(uint64_t* w, const uint64_t* __restrict__ ct, uint32_t s, uint32_t gbase) {
    constexpr int HK = 1 << (R - 1 - V);
    const uint64_t* base = ct + ((size_t)gbase << V) + ((32u * s) >> (R - V));
#pragma unroll
    for (int q = 0; q < 16; q++) w[q] = base[pair_lo(q, HK) >> (R - V)];
}

template <int R, int V>
__device__ __forceinline__ void head_b_stage(uint64_t* x, const uint64_t* __restrict__ ct, uint32_t s, uint32_t gbase) {
    if constexpr (V < R) {
        uint64_t w[16];
        tw_ct_headB<R, V>(w, ct, s, gbase);
        ct_stage<(1 << (R - 1 - V))>(x, w);
        head_b_stage<R, V + 1>(x, ct, s, gbase);
    }
}

// Block -> (coset, unit = column * tiles + tile). XCD-aware when the unit count is a multiple
// of 8: blocks are dealt round-robin over the 8 XCDs, so the n_cosets blocks of one unit sit
// at ids unit8 + 8 c within a run of 8 n_cosets ids and share an XCD (its L2) and a time
// window. Otherwise (small heads: few columns x 2^R tiles) the cosets of a unit are
// consecutive ids. Speed only: any placement gives the same result.
__device__ __forceinline__ void head_unit(uint32_t bid, uint32_t n_cosets, bool xcd, uint32_t& coset,
                                          uint32_t& unit) {
    if (xcd) {
        const uint32_t rest = bid >> 3;
        coset = rest % n_cosets;
        unit = ((rest / n_cosets) << 3) | (bid & 7);
    } else {
        coset = bid % n_cosets;
        unit = bid / n_cosets;
    }
}

// MODE 0: natural source; MODE 1: bit-reversed source gathered in runs of 2^R words.
// KAPPA must be false: an inverse's n^-1 sits in its tail's TA table here (the small heads
// still scale their own stage 0 with CT[1] + mul4_by).
// Grid: one dimension (head_unit): with the XCD-aware placement the source tile is fetched
// from HBM once and re-read from L2 by the other cosets.
// SUB (log_sub > 0): stages log_sub .. log_sub + R - 1 of columns of 2^(log_n + log_sub) words
// whose first log_sub stages are done (launch_ct past 2^23): "column" c of the grid is
// sub-column g = c mod 2^log_sub (2^log_n words at g 2^log_n) of column c >> log_sub, read at
// src + column * src_stride + coset * src_coset_stride (in place on the coset outputs).
// P2 (whole columns, 5 <= R <= 10, no KAPPA): the power-of-two form of both phases, with the
// prescale tables after the CT table (INV: the inverse root; n^-1 then sits in the tail's TA).
template <int R, int MODE, bool KAPPA, bool SUB = false, bool P2 = false, bool INV = false>
__global__ __launch_bounds__(NT, 2) void ct_head_kernel(uint64_t* dst, size_t dst_col_stride, size_t coset_stride,
                                                        const uint64_t* src, size_t src_stride, uint32_t log_n,
                                                        const uint64_t* __restrict__ tab, size_t tab_stride,
                                                        uint64_t kappa, uint32_t n_cosets, uint32_t log_tiles,
                                                        int xcd, uint32_t log_sub, size_t src_coset_stride) {
    constexpr int LOGW = 13 - R;
    constexpr uint32_t W = 1u << LOGW;
    constexpr uint32_t T = 1u << (R - 5);
    __shared__ uint64_t lds[PAD_LDS];
    const uint32_t tid = threadIdx.x;
    const size_t n = (size_t)1 << log_n;
    const size_t S = n >> R;
    uint32_t coset, unit;
    head_unit(blockIdx.x, n_cosets, xcd != 0, coset, unit);
    const uint32_t colv = unit >> log_tiles;
    const uint32_t col = SUB ? colv >> log_sub : colv, sub = SUB ? colv & ((1u << log_sub) - 1) : 0;
    const uint32_t gbase = SUB ? (1u << log_sub) + sub : 1;  // compile-time 1 for whole columns
    const size_t o0 = (size_t)(unit & ((1u << log_tiles) - 1)) * W;
    const uint64_t* sc =
        src + (size_t)col * src_stride + (SUB ? (size_t)coset * src_coset_stride + ((size_t)sub << log_n) : 0);
    const uint64_t* ct = tab + (size_t)coset * tab_stride;
    const uint32_t w = tid & (W - 1);
    const uint32_t s = tid >> LOGW;
    const size_t o = o0 + w;
    uint64_t x[PT];
    uint64_t f[P2 ? PT : 1];
    // phase A' prescale factors (wave-uniform) first: after the gather's barrier they were
    // waited for one by one
    if constexpr (P2) load32(f, ct + n);
    if constexpr (MODE == 0) {
        // row s + T k of the tile: a wave-uniform row base (scalar) plus a per-thread 32-bit
        // index, so each load is one instruction with no address VALU
        const uint32_t vi = (uint32_t)(s * S + o);
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = (sc + (size_t)T * k * S)[vi];
    } else {
        const uint32_t wg = tid / T, sg = tid % T;
        const size_t run = (size_t)gl::bitrev32((uint32_t)(o0 + wg), log_n - R) << R;
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = sc[run + sg + T * k];
        if constexpr (R == 9) {
            // bitrev_R(sg + T k) = bitrev_{R-5}(sg) * 32 + bitrev_5(k) (sg < T = 2^(R-5)); at R = 9
            // the swizzle's bits 9..12 are bitrev_4(sg) and its XOR stays inside wg's 4 bits
            // (W = 16), so the slot is a per-thread base plus bitrev_5(k) W, a compile-time offset
            const uint32_t brs = gl::bitrev32(sg, R - 5);
            const uint32_t base = (brs << 5) * W + (wg ^ (brs & 15));
#pragma unroll
            for (int k = 0; k < PT; k++) lds[base + gl::bitrev32((uint32_t)k, 5) * W] = x[k];
        } else {
#pragma unroll
            for (int k = 0; k < PT; k++) lds[swz_gather(gl::bitrev32(sg + T * k, R) * W + wg)] = x[k];
        }
        __syncthreads();
        if constexpr (R >= 7 && R <= 9) {
            // swz_gather((s + T k) W + w): bits 9..12 are (k >> 1) & 15 and the XOR stays inside w
            // (R <= 9); at R = 5, 6 the compiler's own indexing is a little cheaper
            const uint32_t sw = s * W;
#pragma unroll
            for (int k = 0; k < PT; k++) x[k] = lds[sw + 256 * k + (w ^ ((k >> 1) & 15))];
        } else {
#pragma unroll
            for (int k = 0; k < PT; k++) x[k] = lds[swz_gather((s + T * k) * W + w)];
        }
    }
    static_assert(!KAPPA, "n^-1 sits in the tail's TA table (power-of-two heads) or CT[1] + the small heads");
    static_assert(!P2 || !SUB, "the power-of-two head takes whole columns");
    // phase A': rows s + T k, stages 0..4
    if constexpr (P2) {
        // coefficient distance n/32 between the rows: prescale s^((n/32) k)
        prescale32(x, f);
        dft_p2<5, INV, 0>(x);
    } else {
        uint64_t wa[16], wb[16];
        tw_ct_headA<0>(wa, ct, gbase);
        tw_ct_headA<1>(wb, ct, gbase);
        ct_stage<16>(x, wa);
        tw_ct_headA<2>(wa, ct, gbase);
        ct_stage<8>(x, wb);
        tw_ct_headA<3>(wb, ct, gbase);
        ct_stage<4>(x, wa);
        tw_ct_headA<4>(wa, ct, gbase);
        ct_stage<2>(x, wb);
        ct_stage<1>(x, wa);
    }
    if constexpr (MODE == 1) __syncthreads();  // gather reads of lds done
    // phase A' -> B' exchange in the padded layout: writes e = tid + 256 k at
    // (tid + (tid >> 5)) + 264 k, reads e = (32 s + k) W + w at 33 W s + w + (w >> 5) + kW + (kW >> 5):
    // per-thread bases, compile-time offsets, conflict free for every R
    const uint32_t pa = tid + (tid >> 5);
    const uint32_t pd = 33 * W * s + w + (w >> 5);
#pragma unroll
    for (int k = 0; k < PT; k++) lds[pa + 264 * k] = x[k];
    // phase B' factors in quarters of 8, two in flight: quarters 0, 1 ahead of the barrier,
    // quarter q + 2 once quarter q's products are formed (ntt_lde3.hip's phase B)
    const uint64_t* hb = ct + n + EXT_HB + 32 * s;
    if constexpr (P2 && R > 5) {
#pragma unroll
        for (int k = 0; k < 16; k++) f[k] = hb[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++) x[k] = lds[pd + k * W + ((k * W) >> 5)];
    if constexpr (P2) {
        // rows 32 s + k: groups of 2^(R-5) rows after phase A', coefficient distance n >> R
        if constexpr (R > 5) {
            prescale_n<8>(x, f);
#pragma unroll
            for (int k = 16; k < 24; k++) f[k] = hb[k];
            prescale_n<8>(x + 8, f + 8);
#pragma unroll
            for (int k = 24; k < PT; k++) f[k] = hb[k];
            prescale_n<8>(x + 16, f + 16);
            prescale_n<8>(x + 24, f + 24);
            dft_p2_groups<R - 5, INV>(x);
        }
    } else {
        head_b_stage<R, 5>(x, ct, s, gbase);
    }
    uint64_t* dc =
        dst + (size_t)col * dst_col_stride + (size_t)coset * coset_stride + (SUB ? ((size_t)sub << log_n) : 0);
    const uint32_t vo = (uint32_t)(32 * s * S + o);
#pragma unroll
    for (int k = 0; k < PT; k++) (dc + (size_t)k * S)[vo] = x[k];
}

// --------------------------------------------------------- small heads (R <= 4)

// 2^13 <= n <= 2^17: the head's R = log n - 13 stages fit in registers. A tile is 2^R rows
// x 2^(13-R) columns as above, and each thread holds all 2^R rows of C = 2^(5-R) columns
// (columns t + 256 i), so every butterfly is thread-local and needs no LDS; the group index
// of stage v is the row's top v bits, a compile-time register property, so every twiddle is
// a wave-uniform (scalar) load. R = 0 (n = 2^13) is the load / gather step alone.
// x[r * C + i] holds row r of column i; the pairs of stage v are (r, r + 2^(R-1-v)), i.e.
// registers k and k + 2^(R-1-v) C.
template <int R, int V>
__device__ __forceinline__ void tw_ct_small(uint64_t* w, const uint64_t* __restrict__ ct) {
    constexpr int C = 32 >> R;
    constexpr int HK = (1 << (R - 1 - V)) * C;
#pragma unroll
    for (int q = 0; q < 16; q++) w[q] = ct[(1 << V) + ((pair_lo(q, HK) / C) >> (R - V))];
}

template <int R, int V>
__device__ __forceinline__ void small_stage(uint64_t* x, const uint64_t* __restrict__ ct) {
    if constexpr (V < R) {
        uint64_t w[16];
        tw_ct_small<R, V>(w, ct);
        ct_stage<(1 << (R - 1 - V)) * (32 >> R)>(x, w);
        small_stage<R, V + 1>(x, ct);
    }
}

template <int R, int MODE, bool KAPPA>
__global__ __launch_bounds__(NT, 2) void ct_head_small_kernel(uint64_t* dst, size_t dst_col_stride,
                                                              size_t coset_stride, const uint64_t* src,
                                                              size_t src_stride, uint32_t log_n,
                                                              const uint64_t* __restrict__ tab, size_t tab_stride,
                                                              uint64_t kappa, uint32_t n_cosets, uint32_t log_tiles,
                                                              int xcd) {
    constexpr int C = 32 >> R;          // columns per thread
    constexpr uint32_t W = 1u << (13 - R);
    const uint32_t t = threadIdx.x;
    const size_t S = (size_t)1 << (log_n - R);
    uint32_t coset, unit;
    head_unit(blockIdx.x, n_cosets, xcd != 0, coset, unit);
    const uint32_t col = unit >> log_tiles;
    const size_t o0 = (size_t)(unit & ((1u << log_tiles) - 1)) * W;
    const uint64_t* sc = src + (size_t)col * src_stride;
    const uint64_t* ct = tab + (size_t)coset * tab_stride;
    uint64_t x[PT];
#pragma unroll
    for (int i = 0; i < C; i++) {
        const size_t o = o0 + t + NT * i;
        if constexpr (MODE == 0) {
#pragma unroll
            for (int r = 0; r < (1 << R); r++) x[r * C + i] = sc[r * S + o];
        } else {
            // c_j at bitrev_n(j), j = r S + o: the 2^R rows of column o are one contiguous run
            const size_t run = (size_t)gl::bitrev32((uint32_t)o, log_n - R) << R;
#pragma unroll
            for (int r = 0; r < (1 << R); r++) x[r * C + i] = sc[run + gl::bitrev32(r, R)];
        }
    }
    // R = 0 has no stage of its own: an inverse's n^-1 then sits in the tail's TA table
    // (kappa_in_tail), and launch_ct never passes kappa here
    if constexpr (KAPPA && R > 0) {
        // stage-0 lower operands: rows below 2^(R-1), registers 0..15
#pragma unroll
        for (int k = 0; k < 16; k += 4) mul4_by(x[k], x[k + 1], x[k + 2], x[k + 3], kappa);
    }
    small_stage<R, 0>(x, ct);
    uint64_t* dc = dst + (size_t)col * dst_col_stride + (size_t)coset * coset_stride;
#pragma unroll
    for (int i = 0; i < C; i++) {
        const size_t o = o0 + t + NT * i;
#pragma unroll
        for (int r = 0; r < (1 << R); r++) dc[r * S + o] = x[r * C + i];
    }
}

// ------------------------------------------------------------------- tail

// CANON: canonicalise the output (a template parameter: a run-time branch per element made the
// compiler wait on each epilogue LDS read separately). INV: the inverse root (the table is an
// inverse table). Phases A and B (local stages 0..4 and 5..9) run in the power-of-two form:
// block q's polynomial is evaluated on sigma_u0(q) <w_8192>, so phase A prescales element
// t + 256 k by TA[q][k] = sigma_u0(q)^(256 k) and phase B element (thi, 8 k + tlo) by
// TB[(q << 5) | thi][k]; phase C (3 stages) keeps the coset-folded general twiddles.
template <bool CANON, bool INV>
__global__ __launch_bounds__(NT, 2) void ct_tail_kernel(uint64_t* dst, size_t dst_col_stride, size_t coset_stride,
                                                        uint32_t log_n, const uint64_t* __restrict__ tab,
                                                        size_t tab_stride) {
    __shared__ uint64_t lds[PAD_LDS];
    const uint32_t t = threadIdx.x;
    const size_t q = blockIdx.y;
    const uint32_t u0 = log_n - 13;
    uint64_t* d = dst + (size_t)blockIdx.x * dst_col_stride + (size_t)blockIdx.z * coset_stride + q * TILE;
    const uint64_t* ct = tab + (size_t)blockIdx.z * tab_stride;
    const uint64_t* ext = ct + ((size_t)1 << log_n);
    uint64_t x[PT], f[PT], wa[16], wb[16];
#pragma unroll
    for (int k = 0; k < PT; k++) x[k] = d[t + NT * k];
    load32(f, ext + EXT_TA + q * 32);
    prescale32(x, f);
    dft_p2<5, INV, 0>(x);
    const uint32_t tlo = t & 7, thi = t >> 3;
    const uint32_t ba = tail_base_a(t), bb = tail_base_b(thi, tlo), bc = tail_base_c(t);
#pragma unroll
    for (int k = 0; k < PT; k++) lds[ba + tail_off_a(k)] = x[k];
    load32(f, ext + ext_tb(u0) + (((q << 5) | thi) << 5));
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++) x[k] = lds[bb + tail_off_b(k)];
    prescale32(x, f);
    dft_p2<5, INV, 0>(x);
    uint64_t wc[16];
    tw_ct_tailC<10>(wa, ct, u0, q, t);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++) lds[bb + tail_off_b(k)] = x[k];
    // phase C's other twiddles ahead of the barrier (x is in LDS), as the prescale factors
    tw_ct_tailC<11>(wb, ct, u0, q, t);
    tw_ct_tailC<12>(wc, ct, u0, q, t);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++) x[k] = lds[bc + k];
    ct_stage<4>(x, wa);
    ct_stage<2>(x, wb);
    ct_stage<1>(x, wc);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++) lds[bc + k] = x[k];
    __syncthreads();
    // all 32 reads first, then the canonicalisations four at a time, then the stores
#pragma unroll
    for (int k = 0; k < PT; k++) x[k] = lds[ba + tail_off_a(k)];
    if constexpr (CANON) {
#pragma unroll
        for (int k = 0; k < PT; k += 4) canon4(x + k);
    }
#pragma unroll
    for (int k = 0; k < PT; k++) d[t + NT * k] = x[k];
}

// ------------------------------------------------------------ table, scale

struct ShiftPowers {
    uint64_t sp[33];  // sp[u] = s^(n >> (u + 1))
};

// CT[2^u + k] = s^(n >> (u+1)) * w_n^(bitrev_u(k) * (n >> (u+1))); CT[1] *= scale1.
__global__ void ct_table_kernel(uint64_t* out, uint32_t log_n, uint64_t w_n, ShiftPowers spw, uint64_t scale1) {
    const size_t n = (size_t)1 << log_n;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if (i == 0) {
            out[0] = 0;
            continue;
        }
        const uint32_t u = 63 - __builtin_clzll(i);
        const uint32_t k = (uint32_t)(i - ((size_t)1 << u));
        const uint64_t e = (uint64_t)gl::bitrev32(k, u) << (log_n - u - 1);
        uint64_t v = gl::mul(gl::pow(w_n, e), spw.sp[u]);
        if (i == 1) v = gl::mul(v, scale1);
        out[i] = gl::canon(v);
    }
}

// The prescale tables after the CT table (layout at EXT_HB / EXT_TA / ext_tb above). w_n is the
// transform's root (inverted for the inverse), s its shift; ta_scale multiplies TA (n^-1 for the
// inverse transforms whose head runs in the power-of-two form, 1 otherwise).
__global__ void ct_ext_kernel(uint64_t* ext, uint32_t log_n, uint64_t w_n, uint64_t s, uint64_t ta_scale, size_t len) {
    const size_t n = (size_t)1 << log_n;
    const uint32_t u0 = log_n - 13, R = u0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < len; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t v;
        if (i < EXT_HB) {
            v = gl::pow(s, (n >> 5) * i);
        } else if (i < EXT_TA) {
            const size_t j = i - EXT_HB;
            if (R >= 5 && j < ((size_t)1 << R)) {
                const uint32_t g = (uint32_t)(j >> (R - 5));
                const uint64_t m = j & (((size_t)1 << (R - 5)) - 1);
                const uint64_t sigma = gl::mul(s, gl::pow(w_n, gl::bitrev32(g, 5)));
                v = gl::pow(sigma, (n >> R) * m);
            } else {
                v = 0;
            }
        } else if (i < ext_tb(u0)) {
            const size_t j = i - EXT_TA;
            const uint64_t sigma = gl::mul(s, gl::pow(w_n, gl::bitrev32((uint32_t)(j >> 5), u0)));
            v = gl::mul(gl::pow(sigma, 256 * (j & 31)), ta_scale);
        } else {
            const size_t j = i - ext_tb(u0);
            const uint64_t sigma = gl::mul(s, gl::pow(w_n, gl::bitrev32((uint32_t)(j >> 5), u0 + 5)));
            v = gl::pow(sigma, 8 * (j & 31));
        }
        ext[i] = gl::canon(v);
    }
}

__global__ __launch_bounds__(256) void scale_kernel(uint64_t* cols, size_t stride, size_t n, uint64_t k) {
    uint64_t* c = cols + (size_t)blockIdx.y * stride;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        c[i] = gl::canon(gl::mul(c[i], k));
}

// the heads of 2^18 .. 2^23 run in the power-of-two form (n^-1 of an inverse then in the tail)
constexpr bool p2_head(uint32_t log_n) { return log_n >= 18 && log_n <= 23; }
// where an inverse's n^-1 sits in the tail's TA table: the power-of-two heads, and 2^13, whose
// head (R = 0) has no stage of its own (the general heads scale their own stage 0)
constexpr bool kappa_in_tail(uint32_t log_n) { return p2_head(log_n) || log_n == 13; }

template <int R>
void launch_head_R(int mode, bool kappa_on, dim3 g, uint64_t* dst, size_t dst_col_stride, size_t coset_stride,
                   const uint64_t* src, size_t src_stride, uint32_t log_n, const uint64_t* tab, size_t tab_stride,
                   uint64_t kappa, hipStream_t st) {
    const uint32_t log_tiles = log_n - 13;
    const dim3 g1(g.x * g.y * g.z);
    const int xcd = ((g.x * g.y) % 8) == 0 ? 1 : 0;  // units (column x tile) in whole runs of 8
    if constexpr (R >= 5) {
        // whole columns of 2^18 .. 2^23 (p2_head): the power-of-two form; an inverse (kappa != 0)
        // has n^-1 in its tail's TA table
#define BJ_CT_HEAD_P2(M, I)                                                                                    \
    hipLaunchKernelGGL((ct_head_kernel<R, M, false, false, true, I>), g1, dim3(NT), 0, st, dst, dst_col_stride, \
                       coset_stride, src, src_stride, log_n, tab, tab_stride, (uint64_t)0, g.z, log_tiles, xcd, \
                       0u, (size_t)0)
        if (mode == 0) {
            if (kappa_on) BJ_CT_HEAD_P2(0, true);
            else BJ_CT_HEAD_P2(0, false);
        } else {
            if (kappa_on) BJ_CT_HEAD_P2(1, true);
            else BJ_CT_HEAD_P2(1, false);
        }
#undef BJ_CT_HEAD_P2
    } else {
#define BJ_CT_HEAD(M, K)                                                                                 \
    hipLaunchKernelGGL((ct_head_small_kernel<R, M, K>), g1, dim3(NT), 0, st, dst, dst_col_stride, coset_stride, \
                       src, src_stride, log_n, tab, tab_stride, kappa, g.z, log_tiles, xcd)
        if (mode == 0) {
            if (kappa_on) BJ_CT_HEAD(0, true);
            else BJ_CT_HEAD(0, false);
        } else {
            if (kappa_on) BJ_CT_HEAD(1, true);
            else BJ_CT_HEAD(1, false);
        }
#undef BJ_CT_HEAD
    }
}

}  // namespace

// 2^13..2^23: head (log n - 13 stages) + tail (13).  2^24..2^26: a small head runs the first
// log n - 23 stages over the whole column, the R = 10 head the next 10 on each 2^23-word
// sub-column in place, then the tail.
bool ct_ntt_supported(uint32_t log_n) { return log_n >= 13 && log_n <= 26; }

size_t ct_table_len(uint32_t log_n) {
    const size_t n = (size_t)1 << log_n;
    if (!ct_ntt_supported(log_n)) return n;
    const uint32_t u0 = log_n - 13;
    return n + ext_tb(u0) + ((size_t)32 << (u0 + 5));
}

hipError_t launch_ct_table(uint64_t* out, uint32_t log_n, bool inverse, uint64_t shift, uint64_t scale1,
                           hipStream_t st) {
    uint64_t w = gl::domain_generator(log_n);
    if (inverse) w = gl::canon(gl::inv(w));
    ShiftPowers spw{};
    for (uint32_t u = 0; u < log_n; u++) spw.sp[u] = gl::pow(gl::canon(shift), (uint64_t)1 << (log_n - u - 1));
    const size_t n = (size_t)1 << log_n;
    size_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(ct_table_kernel, dim3((unsigned)blocks), dim3(256), 0, st, out, log_n, w, spw,
                       gl::canon(scale1));
    if (ct_ntt_supported(log_n)) {
        const size_t len = ct_table_len(log_n) - n;
        const uint64_t ta_scale = inverse && kappa_in_tail(log_n) ? gl::canon(scale1) : 1;
        size_t eb = (len + 255) / 256;
        if (eb > 8192) eb = 8192;
        hipLaunchKernelGGL(ct_ext_kernel, dim3((unsigned)eb), dim3(256), 0, st, out + n, log_n, w, gl::canon(shift),
                           ta_scale, len);
    }
    return hipGetLastError();
}

// The first log n - 13 stages of the inverse transform alone (the power-of-two head, 2^18..2^23):
// pass 1 of the three-pass LDE (ntt_lde3.hip), whose middle pass runs the inverse tail fused
// with the forward transforms.  inv_tab: the inverse CT table with n^-1 (launch_ct_table).
hipError_t launch_ct_inverse_head(uint64_t* dst, size_t dst_col_stride, const uint64_t* src, size_t src_stride,
                                  uint32_t n_cols, uint32_t log_n, const uint64_t* inv_tab, hipStream_t st) {
    if (n_cols == 0) return hipSuccess;
    if (!p2_head(log_n)) return hipErrorInvalidValue;
    const dim3 g(n_cols, (unsigned)(((size_t)1 << log_n) / TILE), 1);
    switch (log_n - 13) {
        case 5: launch_head_R<5>(0, true, g, dst, dst_col_stride, 0, src, src_stride, log_n, inv_tab, 0, 0, st); break;
        case 6: launch_head_R<6>(0, true, g, dst, dst_col_stride, 0, src, src_stride, log_n, inv_tab, 0, 0, st); break;
        case 7: launch_head_R<7>(0, true, g, dst, dst_col_stride, 0, src, src_stride, log_n, inv_tab, 0, 0, st); break;
        case 8: launch_head_R<8>(0, true, g, dst, dst_col_stride, 0, src, src_stride, log_n, inv_tab, 0, 0, st); break;
        case 9: launch_head_R<9>(0, true, g, dst, dst_col_stride, 0, src, src_stride, log_n, inv_tab, 0, 0, st); break;
        default: launch_head_R<10>(0, true, g, dst, dst_col_stride, 0, src, src_stride, log_n, inv_tab, 0, 0, st); break;
    }
    return hipGetLastError();
}

hipError_t launch_scale(uint64_t* cols, size_t stride, uint32_t n_cols, size_t n, uint64_t k, hipStream_t st) {
    if (n_cols == 0 || n == 0) return hipSuccess;
    size_t bx = (n + 255) / 256;
    if (bx > 4096) bx = 4096;
    hipLaunchKernelGGL(scale_kernel, dim3((unsigned)bx, n_cols), dim3(256), 0, st, cols, stride, n, k);
    return hipGetLastError();
}

// Coset-folded CT transform(s), natural -> bit-reversed, for n_cosets twiddle tables at
// tab + i * tab_stride. Output (c, i, r) at dst + c * dst_col_stride + i * coset_stride + r.
// src_bitrev: source holds c_j at bitrev_n(j) (never in place); otherwise natural (in place
// allowed when dst == src and n_cosets == 1). kappa != 0 marks an inverse transform scaled by
// kappa: the tables must be inverse tables made with scale1 = kappa (launch_ct_table), which
// carry it (CT[1] for the general heads, TA for the power-of-two ones). Tables are
// ct_table_len(log_n) entries each.
hipError_t launch_ct(uint64_t* dst, size_t dst_col_stride, size_t coset_stride, uint32_t n_cosets,
                     const uint64_t* src, size_t src_stride, bool src_bitrev, uint32_t n_cols, uint32_t log_n,
                     const uint64_t* tab, size_t tab_stride, uint64_t kappa, bool canon_out, hipStream_t st) {
    if (n_cols == 0 || n_cosets == 0) return hipSuccess;
    if (!ct_ntt_supported(log_n)) return hipErrorInvalidValue;
    const size_t n = (size_t)1 << log_n;
    const unsigned tiles = (unsigned)(n / TILE);
    const dim3 g(n_cols, tiles, n_cosets);
    const int mode = src_bitrev ? 1 : 0;
    const bool k_on = kappa != 0;
    if (log_n > 23) {
        const uint32_t r1 = log_n - 23;
        switch (r1) {
            case 1: launch_head_R<1>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
            case 2: launch_head_R<2>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
            default: launch_head_R<3>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
        }
        // stages r1 .. r1 + 9 on the 2^r1 sub-columns of every column and coset, in place
        const uint32_t sub_tiles_log = 23 - 13;
        const size_t units = (size_t)n_cols * n_cosets << (r1 + sub_tiles_log);
        hipLaunchKernelGGL((ct_head_kernel<10, 0, false, true>), dim3((unsigned)units), dim3(NT), 0, st, dst,
                           dst_col_stride, coset_stride, dst, dst_col_stride, 23u, tab, tab_stride, (uint64_t)0,
                           n_cosets, sub_tiles_log, 1, r1, coset_stride);
    } else switch (log_n - 13) {
        case 0: launch_head_R<0>(mode, false, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
        case 1: launch_head_R<1>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
        case 2: launch_head_R<2>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
        case 3: launch_head_R<3>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
        case 4: launch_head_R<4>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
        case 5: launch_head_R<5>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
        case 6: launch_head_R<6>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
        case 7: launch_head_R<7>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
        case 8: launch_head_R<8>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
        case 9: launch_head_R<9>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
        default: launch_head_R<10>(mode, k_on, g, dst, dst_col_stride, coset_stride, src, src_stride, log_n, tab, tab_stride, kappa, st); break;
    }
#define BJ_CT_TAIL(C, I) \
    hipLaunchKernelGGL((ct_tail_kernel<C, I>), g, dim3(NT), 0, st, dst, dst_col_stride, coset_stride, log_n, tab, tab_stride)
    if (canon_out) {
        if (k_on) BJ_CT_TAIL(true, true);
        else BJ_CT_TAIL(true, false);
    } else {
        if (k_on) BJ_CT_TAIL(false, true);
        else BJ_CT_TAIL(false, false);
    }
#undef BJ_CT_TAIL
    return hipGetLastError();
}

}  // namespace bj
