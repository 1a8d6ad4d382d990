// Multi-column Gentleman-Sande (DIF) NTT passes for gfx950.
//
// Computes the same transform as the reference's natural->bit-reversed NTT
// (fft/mod.rs:659-734): out[r] = sum_j x_j w^(j * bitrev(r)).  Radix-2 DIF gives exactly
// that ordering: stage u (block m = n >> u, half h = m/2) maps (a, c) at (j, j+h) of each
// block to (a + c, (a - c) * w_m^j).  Results are the same field elements; outputs are
// canonicalised, so they are bit-identical to the reference's.
//
// A pass runs R consecutive stages [u0, u0+R) on LDS tiles.  After stage u0 the column
// splits into 2^u0 independent blocks; inside a block the R stages couple the 2^R elements
// {base + t*S + o}, S = n >> (u0 + R).  A tile = 2^R rows (t) x W adjacent columns (o),
// tile size 2^(R + logW) <= 8192 (64 KiB LDS, two blocks per CU), so every HBM access is a
// run of W contiguous u64 (the last pass: whole contiguous 8192-element blocks).
// For n = 2^22: two passes (9 + 13 stages).
//
// Twiddles: one natural-order "pyramid" table per direction, TW[m/2 + j] = w_m^j
// (j < m/2, m = 2..n), so the butterflies of a stage read consecutive entries.
//
// The LDE's forward pass 1 (MULTI_COSET) reads the iNTT's raw bit-reversed output with a
// coalesced gather (index bitrev(j): runs of 2^R contiguous words per tile column), so the
// iFFT's bit reversal costs no pass of its own; it applies n^-1 * coset^j through two-level
// power tables and reuses the raw tile (kept in registers) for all D cosets.
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "gl_asm.hpp"
#include "bj_internal.hpp"

namespace bj {

constexpr int DIF_THREADS = 256;
constexpr int DIF_TILE_LOG = 13;
constexpr int DIF_TILE = 1 << DIF_TILE_LOG;

__device__ __forceinline__ void split(uint64_t x, uint32_t& lo, uint32_t& hi) {
    lo = (uint32_t)x;
    hi = (uint32_t)(x >> 32);
}
__device__ __forceinline__ uint64_t join(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

__device__ __forceinline__ uint64_t mul1(uint64_t a, uint64_t b) {
    uint32_t a0, a1, b0, b1, z0, z1;
    split(a, a0, a1);
    split(b, b0, b1);
    glasm::mul_x1(a0, a1, b0, b1, z0, z1);
    return join(z0, z1);
}

__device__ __forceinline__ uint64_t canon1(uint64_t a) {
    uint32_t a0, a1, z0, z1;
    split(a, a0, a1);
    glasm::canon_x1(a0, a1, z0, z1);
    return join(z0, z1);
}

// Four DIF butterflies: (x[i], y[i]) <- (x + y, (x - y) * w), or without the multiply.
template <bool MUL>
__device__ __forceinline__ void bfly4(uint64_t* x, uint64_t* y, const uint64_t* w) {
    uint32_t a0[4], a1[4], c0[4], c1[4], s0[4], s1[4], d0[4], d1[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        split(x[i], a0[i], a1[i]);
        split(y[i], c0[i], c1[i]);
    }
    glasm::add_x4(a0[0], a1[0], c0[0], c1[0], s0[0], s1[0], a0[1], a1[1], c0[1], c1[1], s0[1], s1[1],
                  a0[2], a1[2], c0[2], c1[2], s0[2], s1[2], a0[3], a1[3], c0[3], c1[3], s0[3], s1[3]);
    glasm::sub_x4(a0[0], a1[0], c0[0], c1[0], d0[0], d1[0], a0[1], a1[1], c0[1], c1[1], d0[1], d1[1],
                  a0[2], a1[2], c0[2], c1[2], d0[2], d1[2], a0[3], a1[3], c0[3], c1[3], d0[3], d1[3]);
#pragma unroll
    for (int i = 0; i < 4; i++) x[i] = join(s0[i], s1[i]);
    if (MUL) {
        uint32_t w0[4], w1[4], z0[4], z1[4];
#pragma unroll
        for (int i = 0; i < 4; i++) split(w[i], w0[i], w1[i]);
        glasm::mul_x4(d0[0], d1[0], w0[0], w1[0], z0[0], z1[0], d0[1], d1[1], w0[1], w1[1], z0[1], z1[1],
                      d0[2], d1[2], w0[2], w1[2], z0[2], z1[2], d0[3], d1[3], w0[3], w1[3], z0[3], z1[3]);
#pragma unroll
        for (int i = 0; i < 4; i++) y[i] = join(z0[i], z1[i]);
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) y[i] = join(d0[i], d1[i]);
    }
}

// R DIF stages on the LDS tile (tile_n = 2^(R+logW) elements, row-major [t][w]).
// Global stage index of the first stage u0; the tile's outer block index b (stage-u0 block)
// does not enter the twiddles (w_m^j depends on the offset inside the stage-u block only).
template <int NT>
__device__ __forceinline__ void dif_stages(uint64_t* tile, uint32_t log_n, uint32_t u0, uint32_t R, uint32_t logW,
                                           size_t o0, const uint64_t* __restrict__ tw) {
    if (R == 0) return;  // n = 1: the transform is the identity
    const uint32_t tid = threadIdx.x;
    const uint32_t W = 1u << logW;
    const uint32_t half_tile = 1u << (R + logW - 1);
    const size_t S = (size_t)1 << (log_n - u0 - R);
    for (uint32_t v = 0; v < R; v++) {
        const uint32_t lh = R - 1 - v;              // log2(half block) in rows
        const uint32_t u = u0 + v;                  // global stage
        const size_t hm = (size_t)1 << (log_n - u - 1);  // m/2: twiddle base index
        const bool mul = hm > 1;                    // the m = 2 stage has twiddle 1
        if (half_tile >= 4 * NT) {
#pragma unroll 1
            for (uint32_t k0 = 0; k0 < half_tile / NT; k0 += 4) {
                uint64_t x[4], y[4], w[4];
                uint32_t i1[4], i2[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t p = (k0 + q) * NT + tid;
                    const uint32_t ww = p & (W - 1);
                    const uint32_t pp = p >> logW;
                    const uint32_t g = pp >> lh;
                    const uint32_t within = pp & ((1u << lh) - 1);
                    const uint32_t t1 = (g << (lh + 1)) + within;
                    i1[q] = (t1 << logW) + ww;
                    i2[q] = i1[q] + ((1u << lh) << logW);
                    x[q] = tile[i1[q]];
                    y[q] = tile[i2[q]];
                    if (mul) w[q] = tw[hm + (size_t)within * S + o0 + ww];
                }
                if (mul) bfly4<true>(x, y, w);
                else bfly4<false>(x, y, w);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    tile[i1[q]] = x[q];
                    tile[i2[q]] = y[q];
                }
            }
        } else {
            for (uint32_t p = tid; p < half_tile; p += NT) {
                const uint32_t ww = p & (W - 1);
                const uint32_t pp = p >> logW;
                const uint32_t g = pp >> lh;
                const uint32_t within = pp & ((1u << lh) - 1);
                const uint32_t t1 = (g << (lh + 1)) + within;
                const uint32_t i1 = (t1 << logW) + ww;
                const uint32_t i2 = i1 + ((1u << lh) << logW);
                uint32_t a0, a1, c0, c1, s0, s1, d0, d1;
                split(tile[i1], a0, a1);
                split(tile[i2], c0, c1);
                glasm::add_x1(a0, a1, c0, c1, s0, s1);
                glasm::sub_x1(a0, a1, c0, c1, d0, d1);
                tile[i1] = join(s0, s1);
                uint64_t d = join(d0, d1);
                if (mul) d = mul1(d, tw[hm + (size_t)within * S + o0 + ww]);
                tile[i2] = d;
            }
        }
        __syncthreads();
    }
}

// Tile geometry shared by the kernels.
struct TileGeo {
    size_t base;   // global index of tile element (t = 0, w = 0)
    size_t S;      // row stride
    size_t o0;     // first column offset inside the stage-u0 block
};

__device__ __forceinline__ TileGeo tile_geo(uint32_t log_n, uint32_t u0, uint32_t R, uint32_t logW) {
    const size_t n = (size_t)1 << log_n;
    const size_t S = n >> (u0 + R);
    const size_t oblocks = S >> logW;
    const size_t q = blockIdx.x;
    const size_t b = q / oblocks;
    const size_t ob = q - b * oblocks;
    TileGeo g;
    g.S = S;
    g.o0 = ob << logW;
    g.base = b * (n >> u0) + g.o0;
    return g;
}

// Plain pass: src -> dst (may alias), natural order both sides.
__global__ __launch_bounds__(DIF_THREADS, 2) void dif_pass_kernel(uint64_t* dst, size_t dst_stride,
                                                                  const uint64_t* src, size_t src_stride,
                                                                  uint32_t log_n, uint32_t u0, uint32_t R,
                                                                  uint32_t logW, const uint64_t* __restrict__ tw,
                                                                  int canon_out) {
    __shared__ uint64_t tile[DIF_TILE];
    const uint32_t tid = threadIdx.x;
    const uint32_t tile_n = 1u << (R + logW);
    const uint32_t W = 1u << logW;
    const TileGeo geo = tile_geo(log_n, u0, R, logW);
    const uint64_t* s = src + (size_t)blockIdx.y * src_stride;
    uint64_t* d = dst + (size_t)blockIdx.y * dst_stride;
    for (uint32_t e = tid; e < tile_n; e += DIF_THREADS) {
        const uint32_t t = e >> logW, w = e & (W - 1);
        tile[e] = s[geo.base + (size_t)t * geo.S + w];
    }
    __syncthreads();
    dif_stages<DIF_THREADS>(tile, log_n, u0, R, logW, geo.o0, tw);
    for (uint32_t e = tid; e < tile_n; e += DIF_THREADS) {
        const uint32_t t = e >> logW, w = e & (W - 1);
        uint64_t v = tile[e];
        d[geo.base + (size_t)t * geo.S + w] = canon_out ? canon1(v) : v;
    }
}

// First forward pass of the LDE over all D cosets (u0 = 0).
// BITREV_SRC: src = iNTT output in bit-reversed order (y[r] = monomial[bitrev(r)]),
//   read with a coalesced gather (tile column w is the contiguous run of 2^R words at
//   bitrev(o) << R); otherwise src = monomials in natural order (runs of W words).
// Element j of coset i is src_j * pw_i(j), pw_i(j) = scale * s_i^j from the two-level
// table pw + i * pw_stride: lo[0..4096) then hi[j >> 12]; the raw tile is loaded once
// (registers) and reused for every coset.  Coset i goes to dst + i * coset_stride.
constexpr int LDE1_THREADS = 512;
constexpr int LDE1_PER_THREAD = DIF_TILE / LDE1_THREADS;  // 16 raw words cached per thread

template <bool BITREV_SRC>
__global__ __launch_bounds__(LDE1_THREADS, 2) void dif_lde_first_kernel(
    uint64_t* dst, size_t dst_col_stride, size_t coset_stride, uint32_t n_cosets, const uint64_t* src,
    size_t src_stride, uint32_t log_n, uint32_t R, uint32_t logW, const uint64_t* __restrict__ tw,
    const uint64_t* __restrict__ pw, size_t pw_stride, int canon_out) {
    __shared__ uint64_t tile[DIF_TILE];
    const uint32_t tid = threadIdx.x;
    const uint32_t tile_n = 1u << (R + logW);
    const uint32_t W = 1u << logW;
    const uint32_t Rm = (1u << R) - 1;
    const TileGeo geo = tile_geo(log_n, 0, R, logW);
    const uint64_t* s = src + (size_t)blockIdx.y * src_stride;
    uint64_t raw[LDE1_PER_THREAD];
#pragma unroll
    for (int k = 0; k < LDE1_PER_THREAD; k++) {
        const uint32_t e = k * LDE1_THREADS + tid;
        if (e < tile_n) {
            if (BITREV_SRC) {
                const uint32_t w = e >> R, q = e & Rm;
                raw[k] = s[((size_t)gl::bitrev32((uint32_t)(geo.o0 + w), log_n - R) << R) + q];
            } else {
                const uint32_t t = e >> logW, w = e & (W - 1);
                raw[k] = s[geo.base + (size_t)t * geo.S + w];
            }
        }
    }
    for (uint32_t i = 0; i < n_cosets; i++) {
        const uint64_t* lo = pw + i * pw_stride;
        const uint64_t* hi = lo + 4096;
#pragma unroll
        for (int k = 0; k < LDE1_PER_THREAD; k++) {
            const uint32_t e = k * LDE1_THREADS + tid;
            if (e < tile_n) {
                uint32_t t, w;
                if (BITREV_SRC) {
                    w = e >> R;
                    t = gl::bitrev32(e & Rm, R);
                } else {
                    t = e >> logW;
                    w = e & (W - 1);
                }
                const size_t j = (size_t)t * geo.S + geo.o0 + w;  // natural monomial index
                tile[(t << logW) + w] = mul1(raw[k], mul1(hi[j >> 12], lo[j & 4095]));
            }
        }
        __syncthreads();
        dif_stages<LDE1_THREADS>(tile, log_n, 0, R, logW, geo.o0, tw);
        uint64_t* d = dst + (size_t)blockIdx.y * dst_col_stride + i * coset_stride;
        for (uint32_t e = tid; e < tile_n; e += LDE1_THREADS) {
            const uint32_t t = e >> logW, w = e & (W - 1);
            uint64_t v = tile[e];
            d[geo.base + (size_t)t * geo.S + w] = canon_out ? canon1(v) : v;
        }
        __syncthreads();
    }
}

// Twiddle pyramid: TW[m/2 + j] = w_m^j, m = 2^s, j < m/2, entries [1, n); TW[0] unused.
__global__ void twiddle_pyramid_kernel(uint64_t* out, uint32_t log_n, uint64_t w_n) {
    const size_t n = (size_t)1 << log_n;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if (i == 0) { out[0] = 1; continue; }
        const uint32_t s = 63 - __builtin_clzll(i);  // m/2 = 2^s
        const size_t j = i - ((size_t)1 << s);
        // w_m = w_n^(n/m), m = 2^(s+1)
        out[i] = gl::canon(gl::pow(w_n, (uint64_t)j << (log_n - s - 1)));
    }
}

hipError_t launch_twiddle_pyramid(uint64_t* out, uint32_t log_n, bool inverse, hipStream_t st) {
    uint64_t w = gl::domain_generator(log_n);
    if (inverse) w = gl::canon(gl::inv(w));
    const size_t n = (size_t)1 << log_n;
    size_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(twiddle_pyramid_kernel, dim3((unsigned)blocks), dim3(256), 0, st, out, log_n, w);
    return hipGetLastError();
}

// Pass plan for a column of 2^log_n: the last pass runs min(log_n, 13) stages on contiguous
// tiles; the stages before it are split into passes of <= 10 stages with W = 2^(13 - R).
int dif_plan(uint32_t log_n, uint32_t* Rs, uint32_t* u0s) {
    const uint32_t last = log_n < (uint32_t)DIF_TILE_LOG ? log_n : (uint32_t)DIF_TILE_LOG;
    const uint32_t front = log_n - last;
    const uint32_t nf = (front + 9) / 10;
    uint32_t u = 0;
    int np = 0;
    for (uint32_t p = 0; p < nf; p++) {
        const uint32_t R = (front - u + (nf - p) - 1) / (nf - p);
        Rs[np] = R;
        u0s[np] = u;
        np++;
        u += R;
    }
    Rs[np] = last;
    u0s[np] = u;
    return np + 1;
}

// Natural -> bit-reversed DIF transform of n_cols columns, src -> dst (may alias).
hipError_t launch_dif(uint64_t* dst, size_t dst_stride, const uint64_t* src, size_t src_stride, uint32_t n_cols,
                      uint32_t log_n, const uint64_t* tw_pyr, bool canon_out, hipStream_t st) {
    if (n_cols == 0) return hipSuccess;
    uint32_t Rs[8], u0s[8];
    const int np = dif_plan(log_n, Rs, u0s);
    const uint64_t* cs = src;
    size_t css = src_stride;
    for (int p = 0; p < np; p++) {
        const uint32_t R = Rs[p], u0 = u0s[p];
        const bool last = p == np - 1;
        const uint32_t logW = last ? 0 : DIF_TILE_LOG - R;
        const size_t tiles = ((size_t)1 << log_n) >> (R + logW);
        hipLaunchKernelGGL(dif_pass_kernel, dim3((unsigned)tiles, n_cols), dim3(DIF_THREADS), 0, st, dst,
                           dst_stride, cs, css, log_n, u0, R, logW, tw_pyr, (last && canon_out) ? 1 : 0);
        cs = dst;
        css = dst_stride;
    }
    return hipGetLastError();
}

// Forward coset LDE from a raw (bit-reversed, unscaled) iNTT output: all D cosets.
// lde element (c, i, r) at lde + c * lde_col_stride + i * n + r.
hipError_t launch_lde_forward(uint64_t* lde, size_t lde_col_stride, uint32_t n_cosets, const uint64_t* raw,
                              size_t raw_stride, bool raw_bitrev, uint32_t n_cols, uint32_t log_n,
                              const uint64_t* tw_pyr, const uint64_t* pw, size_t pw_stride, hipStream_t st) {
    if (n_cols == 0) return hipSuccess;
    uint32_t Rs[8], u0s[8];
    const int np = dif_plan(log_n, Rs, u0s);
    const size_t n = (size_t)1 << log_n;
    {
        const uint32_t R = Rs[0];
        const bool last = np == 1;
        const uint32_t logW = last ? 0 : DIF_TILE_LOG - R;
        const size_t tiles = n >> (R + logW);
        if (raw_bitrev)
            hipLaunchKernelGGL(dif_lde_first_kernel<true>, dim3((unsigned)tiles, n_cols), dim3(LDE1_THREADS), 0, st,
                               lde, lde_col_stride, n, n_cosets, raw, raw_stride, log_n, R, logW, tw_pyr, pw,
                               pw_stride, last ? 1 : 0);
        else
            hipLaunchKernelGGL(dif_lde_first_kernel<false>, dim3((unsigned)tiles, n_cols), dim3(LDE1_THREADS), 0,
                               st, lde, lde_col_stride, n, n_cosets, raw, raw_stride, log_n, R, logW, tw_pyr, pw,
                               pw_stride, last ? 1 : 0);
    }
    for (int p = 1; p < np; p++) {
        const uint32_t R = Rs[p], u0 = u0s[p];
        const bool last = p == np - 1;
        const uint32_t logW = last ? 0 : DIF_TILE_LOG - R;
        const size_t tiles = n >> (R + logW);
        // all cosets of all columns as one grid: column index = c * D + i, stride n
        hipLaunchKernelGGL(dif_pass_kernel, dim3((unsigned)tiles, n_cols * n_cosets), dim3(DIF_THREADS), 0, st,
                           lde, n, lde, n, log_n, u0, R, logW, tw_pyr, last ? 1 : 0);
    }
    return hipGetLastError();
}

}  // namespace bj
