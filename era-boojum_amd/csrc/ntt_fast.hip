// Register-resident DIF NTT passes for the large LDE sizes (2^18 <= n <= 2^23).
//
// Same transform and the same butterflies as ntt_dif.hip (DIF, natural in, bit-reversed
// out, TW[m/2 + j] = w_m^j pyramid); only the schedule differs: every thread keeps 32
// tile elements in VGPRs and runs up to five consecutive stages on them without touching
// LDS, so LDS is used only to re-deal elements between register phases (XOR-swizzled,
// conflict-free ds_read/write_b64), and each stage's 16 twiddles per thread are loaded one
// stage ahead.
//
// head pass: the first R stages (R = log_n - 13, 5 <= R <= 10) on tiles of 2^R rows x
//   W = 2^(13-R) adjacent columns (row stride S = n >> R).  Thread (s, w) first holds rows
//   s + T*k (T = 2^(R-5) threads per column, k < 32) -> stages of row distance 2^(R-1)..T;
//   then rows 32 s' + k -> the remaining R - 5 stages.  Output rows are stored straight
//   from registers (runs of W words).
// tail pass: the last 13 stages on contiguous 8192-element blocks: phase A (element
//   t + 256 k, distances 4096..256), phase B ((t>>3)<<8 | k<<3 | t&7, distances 128..8),
//   phase C (32 t + k, distances 4, 2, 1), then back to A order for a coalesced store.
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "gl_asm.hpp"
#include "bj_internal.hpp"

namespace bj {

namespace {

constexpr int NT = 256;  // threads per block
constexpr int PT = 32;   // elements per thread
constexpr int TILE = NT * PT;

__device__ __forceinline__ void split2(uint64_t x, uint32_t& lo, uint32_t& hi) {
    lo = (uint32_t)x;
    hi = (uint32_t)(x >> 32);
}
__device__ __forceinline__ uint64_t join2(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

// Butterflies (x[a_q], x[b_q]) <- (x_a + x_b, (x_a - x_b) * w_q) for q < 4.
template <bool MUL>
__device__ __forceinline__ void bfly_x4(uint64_t& xa0, uint64_t& xb0, uint64_t& xa1, uint64_t& xb1, uint64_t& xa2,
                                        uint64_t& xb2, uint64_t& xa3, uint64_t& xb3, uint64_t w0, uint64_t w1,
                                        uint64_t w2, uint64_t w3) {
    uint32_t a0[4], a1[4], c0[4], c1[4], s0[4], s1[4], d0[4], d1[4];
    split2(xa0, a0[0], a1[0]); split2(xb0, c0[0], c1[0]);
    split2(xa1, a0[1], a1[1]); split2(xb1, c0[1], c1[1]);
    split2(xa2, a0[2], a1[2]); split2(xb2, c0[2], c1[2]);
    split2(xa3, a0[3], a1[3]); split2(xb3, c0[3], c1[3]);
    glasm::add_x4(a0[0], a1[0], c0[0], c1[0], s0[0], s1[0], a0[1], a1[1], c0[1], c1[1], s0[1], s1[1],
                  a0[2], a1[2], c0[2], c1[2], s0[2], s1[2], a0[3], a1[3], c0[3], c1[3], s0[3], s1[3]);
    glasm::sub_x4(a0[0], a1[0], c0[0], c1[0], d0[0], d1[0], a0[1], a1[1], c0[1], c1[1], d0[1], d1[1],
                  a0[2], a1[2], c0[2], c1[2], d0[2], d1[2], a0[3], a1[3], c0[3], c1[3], d0[3], d1[3]);
    xa0 = join2(s0[0], s1[0]); xa1 = join2(s0[1], s1[1]);
    xa2 = join2(s0[2], s1[2]); xa3 = join2(s0[3], s1[3]);
    if (MUL) {
        uint32_t v0[4], v1[4], z0[4], z1[4];
        split2(w0, v0[0], v1[0]); split2(w1, v0[1], v1[1]);
        split2(w2, v0[2], v1[2]); split2(w3, v0[3], v1[3]);
        glasm::mul_x4(d0[0], d1[0], v0[0], v1[0], z0[0], z1[0], d0[1], d1[1], v0[1], v1[1], z0[1], z1[1],
                      d0[2], d1[2], v0[2], v1[2], z0[2], z1[2], d0[3], d1[3], v0[3], v1[3], z0[3], z1[3]);
        xb0 = join2(z0[0], z1[0]); xb1 = join2(z0[1], z1[1]);
        xb2 = join2(z0[2], z1[2]); xb3 = join2(z0[3], z1[3]);
    } else {
        xb0 = join2(d0[0], d1[0]); xb1 = join2(d0[1], d1[1]);
        xb2 = join2(d0[2], d1[2]); xb3 = join2(d0[3], d1[3]);
    }
}

// Index of the q-th (q < 16) lower element of the pairs at register distance hk.
__device__ __forceinline__ constexpr int pair_lo(int q, int hk) { return (q / hk) * 2 * hk + (q % hk); }

// One register stage on x[32] with pairs (k, k + HK); w[q] is the twiddle of pair q.
template <int HK, bool MUL>
__device__ __forceinline__ void reg_stage(uint64_t* x, const uint64_t* w) {
#pragma unroll
    for (int b = 0; b < 4; b++) {
        constexpr int dummy = 0;
        (void)dummy;
        const int q0 = 4 * b;
        bfly_x4<MUL>(x[pair_lo(q0, HK)], x[pair_lo(q0, HK) + HK], x[pair_lo(q0 + 1, HK)],
                     x[pair_lo(q0 + 1, HK) + HK], x[pair_lo(q0 + 2, HK)], x[pair_lo(q0 + 2, HK) + HK],
                     x[pair_lo(q0 + 3, HK)], x[pair_lo(q0 + 3, HK) + HK], w[q0], w[q0 + 1], w[q0 + 2], w[q0 + 3]);
    }
}

__device__ __forceinline__ uint64_t canon_u64(uint64_t v) {
    uint32_t a0, a1, z0, z1;
    split2(v, a0, a1);
    glasm::canon_x1(a0, a1, z0, z1);
    return join2(z0, z1);
}

__device__ __forceinline__ uint64_t mul_u64(uint64_t a, uint64_t b) {
    uint32_t a0, a1, b0, b1, z0, z1;
    split2(a, a0, a1);
    split2(b, b0, b1);
    glasm::mul_x1(a0, a1, b0, b1, z0, z1);
    return join2(z0, z1);
}

// ------------------------------------------------------------------ tail pass

__device__ __forceinline__ uint32_t swz_tail(uint32_t e) { return e ^ ((e >> 5) & 31); }

// Twiddles of one phase-A stage (distance h = 256 * HK elements): pair q has lower
// element t + 256 * lo(q), offset (t + 256 * (lo(q) mod HK)) in its half block.
template <int HK>
__device__ __forceinline__ void tw_phaseA(uint64_t* w, const uint64_t* __restrict__ tw, uint32_t t) {
    const uint32_t h = 256u * HK;
#pragma unroll
    for (int q = 0; q < 16; q++) w[q] = tw[h + t + 256u * (pair_lo(q, HK) % HK)];
}

// phase B: element (t>>3)<<8 | k<<3 | t&7, distance h = 8 * HK.
template <int HK>
__device__ __forceinline__ void tw_phaseB(uint64_t* w, const uint64_t* __restrict__ tw, uint32_t tlo) {
    const uint32_t h = 8u * HK;
#pragma unroll
    for (int q = 0; q < 16; q++) w[q] = tw[h + ((uint32_t)(pair_lo(q, HK) % HK) << 3) + tlo];
}

// Last 13 stages on contiguous 8192-element blocks (src -> dst, may alias).
__global__ __launch_bounds__(NT, 2) void dif_tail_kernel(uint64_t* dst, size_t dst_stride, const uint64_t* src,
                                                         size_t src_stride, const uint64_t* __restrict__ tw,
                                                         int canon_out) {
    __shared__ uint64_t lds[TILE];
    const uint32_t t = threadIdx.x;
    const size_t off = (size_t)blockIdx.x * TILE;
    const uint64_t* s = src + (size_t)blockIdx.y * src_stride + off;
    uint64_t* d = dst + (size_t)blockIdx.y * dst_stride + off;
    uint64_t x[PT], wa[16], wb[16];
#pragma unroll
    for (int k = 0; k < PT; k++) x[k] = s[t + NT * k];
    // phase A: distances 4096, 2048, 1024, 512, 256 (register distance 16..1)
    tw_phaseA<16>(wa, tw, t);
    tw_phaseA<8>(wb, tw, t);
    reg_stage<16, true>(x, wa);
    tw_phaseA<4>(wa, tw, t);
    reg_stage<8, true>(x, wb);
    tw_phaseA<2>(wb, tw, t);
    reg_stage<4, true>(x, wa);
    tw_phaseA<1>(wa, tw, t);
    reg_stage<2, true>(x, wb);
    const uint32_t tlo = t & 7, thi = t >> 3;
    tw_phaseB<16>(wb, tw, tlo);
    reg_stage<1, true>(x, wa);
#pragma unroll
    for (int k = 0; k < PT; k++) lds[swz_tail(t + NT * k)] = x[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++) x[k] = lds[swz_tail((thi << 8) | ((uint32_t)k << 3) | tlo)];
    // phase B: distances 128, 64, 32, 16, 8
    tw_phaseB<8>(wa, tw, tlo);
    reg_stage<16, true>(x, wb);
    tw_phaseB<4>(wb, tw, tlo);
    reg_stage<8, true>(x, wa);
    tw_phaseB<2>(wa, tw, tlo);
    reg_stage<4, true>(x, wb);
    tw_phaseB<1>(wb, tw, tlo);
    reg_stage<2, true>(x, wa);
    reg_stage<1, true>(x, wb);
    __syncthreads();  // every phase-B read of lds is done
#pragma unroll
    for (int k = 0; k < PT; k++) lds[swz_tail((thi << 8) | ((uint32_t)k << 3) | tlo)] = x[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++) x[k] = lds[swz_tail(t * PT + k)];
    // phase C: distances 4, 2, 1 inside each group of 8 consecutive elements
    {
        uint64_t w4[16], w2[16];
#pragma unroll
        for (int q = 0; q < 16; q++) {
            w4[q] = tw[4 + (pair_lo(q, 4) % 4)];
            w2[q] = tw[2 + (pair_lo(q, 2) % 2)];
        }
        reg_stage<4, true>(x, w4);
        reg_stage<2, true>(x, w2);
        reg_stage<1, false>(x, w2);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++) lds[swz_tail(t * PT + k)] = x[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; k++) {
        uint64_t v = lds[swz_tail(t + NT * k)];
        d[t + NT * k] = canon_out ? canon_u64(v) : v;
    }
}

// ------------------------------------------------------------------ head pass

// Swizzle of tile element e = row * W + w for the head exchange (see file comment).
template <int LOGW>
__device__ __forceinline__ uint32_t swz_head(uint32_t e) {
    constexpr uint32_t m = LOGW >= 5 ? 0u : ((32u >> LOGW) - 1u);
    return e ^ (((e >> (5 + LOGW)) & m) << LOGW);
}

// Head-pass twiddles, phase A' (row distance h_r = T * HK, stage block half = h_r * S):
// lower row of pair q is s + T * lo(q); offset in the half block (s + T*(lo(q) mod HK))*S + o.
template <int HK, int T>
__device__ __forceinline__ void tw_headA(uint64_t* w, const uint64_t* __restrict__ tw, size_t hm, size_t S,
                                         uint32_t s, size_t o) {
#pragma unroll
    for (int q = 0; q < 16; q++) w[q] = tw[hm + (size_t)(s + T * (pair_lo(q, HK) % HK)) * S + o];
}

// phase B': rows 32 s' + k, row distance HK (<= 16): offset (lo(q) mod HK) * S + o.
template <int HK>
__device__ __forceinline__ void tw_headB(uint64_t* w, const uint64_t* __restrict__ tw, size_t hm, size_t S,
                                         size_t o) {
#pragma unroll
    for (int q = 0; q < 16; q++) w[q] = tw[hm + (size_t)(pair_lo(q, HK) % HK) * S + o];
}

// Stages of phase A' for register distances 16..1 (R >= 5 rows bits; first 5 stages).
template <int T>
__device__ __forceinline__ void head_phaseA(uint64_t* x, const uint64_t* __restrict__ tw, uint32_t log_n, size_t S,
                                            uint32_t s, size_t o) {
    // stage v (0..4) has row distance T * 2^(4-v) and block half hm = n >> (v+1)
    uint64_t wa[16], wb[16];
    const size_t n = (size_t)1 << log_n;
    tw_headA<16, T>(wa, tw, n >> 1, S, s, o);
    tw_headA<8, T>(wb, tw, n >> 2, S, s, o);
    reg_stage<16, true>(x, wa);
    tw_headA<4, T>(wa, tw, n >> 3, S, s, o);
    reg_stage<8, true>(x, wb);
    tw_headA<2, T>(wb, tw, n >> 4, S, s, o);
    reg_stage<4, true>(x, wa);
    tw_headA<1, T>(wa, tw, n >> 5, S, s, o);
    reg_stage<2, true>(x, wb);
    reg_stage<1, true>(x, wa);
}

// Phase B' stages: register distances T/2 .. 1 (R - 5 stages), row halves hm = n >> (6 + j).
template <int T>
__device__ __forceinline__ void head_phaseB(uint64_t* x, const uint64_t* __restrict__ tw, uint32_t log_n, size_t S,
                                            size_t o) {
    const size_t n = (size_t)1 << log_n;
    uint64_t w[16];
    if constexpr (T >= 32) { tw_headB<16>(w, tw, n >> 6, S, o); reg_stage<16, true>(x, w); }
    if constexpr (T >= 16) { tw_headB<8>(w, tw, n >> (T >= 32 ? 7 : 6), S, o); reg_stage<8, true>(x, w); }
    if constexpr (T >= 8) {
        tw_headB<4>(w, tw, n >> (T >= 32 ? 8 : T >= 16 ? 7 : 6), S, o);
        reg_stage<4, true>(x, w);
    }
    if constexpr (T >= 4) {
        tw_headB<2>(w, tw, n >> (T >= 32 ? 9 : T >= 16 ? 8 : T >= 8 ? 7 : 6), S, o);
        reg_stage<2, true>(x, w);
    }
    if constexpr (T >= 2) {
        tw_headB<1>(w, tw, n >> (T >= 32 ? 10 : T >= 16 ? 9 : T >= 8 ? 8 : T >= 4 ? 7 : 6), S, o);
        reg_stage<1, true>(x, w);
    }
}

// MODE 0: plain (natural load, no scaling, one output); MODE 1: bit-reversed gather of the
// raw iNTT + per-coset scaling (multi-coset); MODE 2: natural load + per-coset scaling.
template <int R, int MODE>
__global__ __launch_bounds__(NT, 2) void dif_head_kernel(uint64_t* dst, size_t dst_col_stride, size_t coset_stride,
                                                         uint32_t n_cosets, const uint64_t* src, size_t src_stride,
                                                         uint32_t log_n, const uint64_t* __restrict__ tw,
                                                         const uint64_t* __restrict__ pw, size_t pw_stride) {
    constexpr int LOGW = 13 - R;
    constexpr uint32_t W = 1u << LOGW;
    constexpr uint32_t T = 1u << (R - 5);  // threads per column
    __shared__ uint64_t lds[TILE];
    const uint32_t tid = threadIdx.x;
    const size_t n = (size_t)1 << log_n;
    const size_t S = n >> R;
    const size_t o0 = (size_t)blockIdx.x * W;
    const uint64_t* sc = src + (size_t)blockIdx.y * src_stride;
    // phase A' / store mapping: w = tid % W, s = tid / W
    const uint32_t w = tid & (W - 1);
    const uint32_t s = tid >> LOGW;
    const size_t o = o0 + w;
    uint64_t x[PT];
    // gather mapping (MODE 1): column wg = tid / T, run position q = sg + T * k
    const uint32_t wg = tid / T, sg = tid % T;
    // One coset per block (blockIdx.z): the source tile is re-read per coset (L2 / MALL
    // resident after the first).  A coset loop inside the block would keep the hoisted
    // twiddle addresses and a cached source tile live beside x[] and spill.
    const uint32_t i = blockIdx.z;
    (void)n_cosets;
    {
        if (MODE == 0) {
#pragma unroll
            for (int k = 0; k < PT; k++) x[k] = sc[(size_t)(s + T * k) * S + o];
        } else if (MODE == 1) {
            // gather runs of the bit-reversed source, scale, deal through LDS to phase-A' order
            const uint64_t* lo = pw + i * pw_stride;
            const uint64_t* hi = lo + 4096;
            const size_t run = (size_t)gl::bitrev32((uint32_t)(o0 + wg), log_n - R) << R;
#pragma unroll
            for (int k = 0; k < PT; k++) x[k] = sc[run + sg + T * k];
#pragma unroll
            for (int k = 0; k < PT; k++) {
                const uint32_t row = gl::bitrev32(sg + T * k, R);
                const size_t j = (size_t)row * S + o0 + wg;
                lds[swz_head<LOGW>(row * W + wg)] = mul_u64(x[k], mul_u64(hi[j >> 12], lo[j & 4095]));
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < PT; k++) x[k] = lds[swz_head<LOGW>((s + T * k) * W + w)];
        } else {
            const uint64_t* lo = pw + i * pw_stride;
            const uint64_t* hi = lo + 4096;
#pragma unroll
            for (int k = 0; k < PT; k++) {
                const size_t j = (size_t)(s + T * k) * S + o;
                x[k] = mul_u64(sc[j], mul_u64(hi[j >> 12], lo[j & 4095]));
            }
        }
        head_phaseA<T>(x, tw, log_n, S, s, o);
        __syncthreads();  // LDS free (MODE 1 reads done)
#pragma unroll
        for (int k = 0; k < PT; k++) lds[swz_head<LOGW>((s + T * k) * W + w)] = x[k];
        __syncthreads();
        // phase B': thread (s', w) holds rows 32 s' + k
#pragma unroll
        for (int k = 0; k < PT; k++) x[k] = lds[swz_head<LOGW>((32 * s + k) * W + w)];
        head_phaseB<T>(x, tw, log_n, S, o);
        uint64_t* dc = dst + (size_t)blockIdx.y * dst_col_stride + (size_t)i * coset_stride;
#pragma unroll
        for (int k = 0; k < PT; k++) dc[(size_t)(32 * s + k) * S + o] = x[k];
    }
}

}  // namespace

bool fast_ntt_supported(uint32_t log_n) { return log_n >= 18 && log_n <= 23; }

template <int R>
static void launch_head_R(int mode, uint64_t* dst, size_t dst_col_stride, size_t coset_stride, uint32_t n_cosets,
                          const uint64_t* src, size_t src_stride, uint32_t n_cols, uint32_t log_n, const uint64_t* tw,
                          const uint64_t* pw, size_t pw_stride, hipStream_t st) {
    const size_t n = (size_t)1 << log_n;
    const unsigned blocks = (unsigned)((n >> R) >> (13 - R));
    dim3 g(blocks, n_cols, mode == 0 ? 1u : n_cosets);
    if (mode == 0)
        hipLaunchKernelGGL((dif_head_kernel<R, 0>), g, dim3(NT), 0, st, dst, dst_col_stride, coset_stride, n_cosets,
                           src, src_stride, log_n, tw, pw, pw_stride);
    else if (mode == 1)
        hipLaunchKernelGGL((dif_head_kernel<R, 1>), g, dim3(NT), 0, st, dst, dst_col_stride, coset_stride, n_cosets,
                           src, src_stride, log_n, tw, pw, pw_stride);
    else
        hipLaunchKernelGGL((dif_head_kernel<R, 2>), g, dim3(NT), 0, st, dst, dst_col_stride, coset_stride, n_cosets,
                           src, src_stride, log_n, tw, pw, pw_stride);
}

static void launch_head(int mode, uint64_t* dst, size_t dst_col_stride, size_t coset_stride, uint32_t n_cosets,
                        const uint64_t* src, size_t src_stride, uint32_t n_cols, uint32_t log_n, const uint64_t* tw,
                        const uint64_t* pw, size_t pw_stride, hipStream_t st) {
    switch (log_n - 13) {
        case 5: launch_head_R<5>(mode, dst, dst_col_stride, coset_stride, n_cosets, src, src_stride, n_cols, log_n, tw, pw, pw_stride, st); break;
        case 6: launch_head_R<6>(mode, dst, dst_col_stride, coset_stride, n_cosets, src, src_stride, n_cols, log_n, tw, pw, pw_stride, st); break;
        case 7: launch_head_R<7>(mode, dst, dst_col_stride, coset_stride, n_cosets, src, src_stride, n_cols, log_n, tw, pw, pw_stride, st); break;
        case 8: launch_head_R<8>(mode, dst, dst_col_stride, coset_stride, n_cosets, src, src_stride, n_cols, log_n, tw, pw, pw_stride, st); break;
        case 9: launch_head_R<9>(mode, dst, dst_col_stride, coset_stride, n_cosets, src, src_stride, n_cols, log_n, tw, pw, pw_stride, st); break;
        default: launch_head_R<10>(mode, dst, dst_col_stride, coset_stride, n_cosets, src, src_stride, n_cols, log_n, tw, pw, pw_stride, st); break;
    }
}

// Full natural->bit-reversed DIF transform (head + tail), src -> dst (may alias).
hipError_t launch_dif_fast(uint64_t* dst, size_t dst_stride, const uint64_t* src, size_t src_stride, uint32_t n_cols,
                           uint32_t log_n, const uint64_t* tw_pyr, bool canon_out, hipStream_t st) {
    if (n_cols == 0) return hipSuccess;
    launch_head(0, dst, dst_stride, 0, 1, src, src_stride, n_cols, log_n, tw_pyr, nullptr, 0, st);
    const size_t n = (size_t)1 << log_n;
    hipLaunchKernelGGL(dif_tail_kernel, dim3((unsigned)(n / TILE), n_cols), dim3(NT), 0, st, dst, dst_stride, dst,
                       dst_stride, tw_pyr, canon_out ? 1 : 0);
    return hipGetLastError();
}

// Forward LDE over all D cosets from the raw bit-reversed iNTT output (raw_bitrev) or from
// natural monomials; lde layout [c][i][r] with lde_col_stride = D * n.
hipError_t launch_lde_forward_fast(uint64_t* lde, size_t lde_col_stride, uint32_t n_cosets, const uint64_t* raw,
                                   size_t raw_stride, bool raw_bitrev, uint32_t n_cols, uint32_t log_n,
                                   const uint64_t* tw_pyr, const uint64_t* pw, size_t pw_stride, hipStream_t st) {
    if (n_cols == 0) return hipSuccess;
    const size_t n = (size_t)1 << log_n;
    launch_head(raw_bitrev ? 1 : 2, lde, lde_col_stride, n, n_cosets, raw, raw_stride, n_cols, log_n, tw_pyr, pw,
                pw_stride, st);
    hipLaunchKernelGGL(dif_tail_kernel, dim3((unsigned)(n / TILE), n_cols * n_cosets), dim3(NT), 0, st, lde, n, lde,
                       n, tw_pyr, 1);
    return hipGetLastError();
}

}  // namespace bj
