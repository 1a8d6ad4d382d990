// NTT kernels (gfx950): batched multi-column radix-2 Cooley-Tukey natural->bit-reversed
// transforms, the iFFT bit-reverse/scale pass, coset power tables and twiddles.
//
// Algorithm = the reference's serial_ct_ntt_natural_to_bitreversed (fft/mod.rs:659-734):
// stage s has 2^s groups; group k is the contiguous block [k*n/2^s, (k+1)*n/2^s) whose
// butterflies pair j with j + n/2^(s+1) and multiply the upper input by tw[k], tw the
// bit-reversed table of omega powers (utils.rs:88-125).  The stages are grouped into
// passes; one pass runs R consecutive stages on LDS tiles.  After stage s0 the column
// splits into 2^s0 independent blocks, and inside a block stages s0..s0+R-1 only couple
// the 2^R elements {base + t*stride + o}, stride = n >> (s0+R).  A tile holds 2^R rows
// (t) x W adjacent sub-problems (o), so every global access is a run of W contiguous
// u64 (W*8 bytes) and every butterfly is done in LDS.  Same butterflies, same twiddles,
// same order of operations per element as the reference => same field values.
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "bj_internal.hpp"

namespace bj {

constexpr int NTT_THREADS = 256;
constexpr int TILE_LOG = 12;  // 4096 u64 = 32 KiB of LDS per block

// --------------------------------------------------------------- twiddles
// tw[i] = w^bitrev_{log_n - 1}(i), i < n/2 (utils.rs:117-122: powers, then bitreverse).
__global__ void twiddles_kernel(uint64_t* out, uint32_t log_n, uint64_t w) {
    size_t half = (size_t)1 << (log_n - 1);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < half;
         i += (size_t)gridDim.x * blockDim.x) {
        uint32_t e = gl::bitrev32((uint32_t)i, log_n - 1);
        out[i] = gl::canon(gl::pow(w, e));
    }
}

// tw[i] = w^i, i < n/2: precompute_twiddles_for_fft_natural (utils.rs:127-155).
__global__ void twiddles_natural_kernel(uint64_t* out, uint32_t log_n, uint64_t w) {
    size_t half = (size_t)1 << (log_n - 1);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < half;
         i += (size_t)gridDim.x * blockDim.x)
        out[i] = gl::canon(gl::pow(w, i));
}

// In-place bit-reversal permutation of each column (bitreverse_enumeration_inplace,
// fft/mod.rs:41-155): the pair (i, bitrev(i)), i < bitrev(i), is swapped by the thread of i;
// values are moved, not re-represented.
__global__ void bitrev_inplace_kernel(uint64_t* cols, size_t col_stride, uint32_t log_n) {
    uint64_t* c = cols + (size_t)blockIdx.y * col_stride;
    const size_t n = (size_t)1 << log_n;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = log_n ? (size_t)gl::bitrev32((uint32_t)i, log_n) : 0;
        if (i < r) {
            const uint64_t a = c[i];
            c[i] = c[r];
            c[r] = a;
        }
    }
}

// Power tables for e^j = hi[j >> 12] * lo[j & 4095]: lo[t] = e^t (t < 4096),
// hi[t] = e^(4096 t) (t < n_hi).  Optional factor `scale` folded into lo.
__global__ void power_tables_kernel(uint64_t* lo, uint64_t* hi, uint32_t n_hi, uint64_t e, uint64_t scale) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 4096) lo[i] = gl::canon(gl::mul(gl::pow(e, i), scale));
    if (i < n_hi) hi[i] = gl::canon(gl::pow(e, (uint64_t)i * 4096));
}

// ----------------------------------------------------------------- NTT pass
// Grid: x = tiles per column, y = columns.  src may alias dst (in place).
// pw_lo/pw_hi (nullable): multiply element j by pw_hi[j>>12]*pw_lo[j&4095] on load
// (distribute_powers, fused into the first pass).
__global__ __launch_bounds__(NTT_THREADS) void ntt_pass_kernel(
    uint64_t* dst, size_t dst_stride, const uint64_t* src, size_t src_stride, uint32_t log_n,
    uint32_t s0, uint32_t R, uint32_t logW, const uint64_t* __restrict__ tw,
    const uint64_t* __restrict__ pw_lo, const uint64_t* __restrict__ pw_hi, int canon_out) {
    __shared__ uint64_t tile[1 << TILE_LOG];
    const uint32_t tid = threadIdx.x;
    const size_t col = blockIdx.y;
    const uint32_t tile_log = R + logW;
    const uint32_t tile_n = 1u << tile_log;
    const uint32_t W = 1u << logW;
    const size_t n = (size_t)1 << log_n;
    const size_t stride = n >> (s0 + R);
    const size_t oblocks = stride >> logW;
    const size_t q = blockIdx.x;
    const size_t b = q / oblocks;
    const size_t ob = q - b * oblocks;
    const size_t base = b * (n >> s0) + (ob << logW);
    const uint64_t* s = src + col * src_stride;
    uint64_t* d = dst + col * dst_stride;

    for (uint32_t e = tid; e < tile_n; e += NTT_THREADS) {
        const uint32_t t = e >> logW, w = e & (W - 1);
        const size_t j = base + (size_t)t * stride + w;
        uint64_t v = s[j];
        if (pw_lo) v = gl::mul(v, gl::mul(pw_hi[j >> 12], pw_lo[j & 4095]));
        tile[e] = v;
    }
    __syncthreads();
    for (uint32_t u = 0; u < R; u++) {
        const uint32_t lh = R - 1 - u;  // log2(half) in rows
        const uint32_t half = 1u << lh;
        for (uint32_t p = tid; p < tile_n / 2; p += NTT_THREADS) {
            const uint32_t w = p & (W - 1);
            const uint32_t pp = p >> logW;
            const uint32_t g = pp >> lh;
            const uint32_t within = pp & (half - 1);
            const uint32_t t1 = (g << (lh + 1)) + within;
            const uint32_t i1 = (t1 << logW) + w;
            const uint32_t i2 = i1 + (half << logW);
            const uint64_t x = tile[i1];
            const uint64_t y = gl::mul(tile[i2], tw[(b << u) + g]);
            tile[i1] = gl::add(x, y);
            tile[i2] = gl::sub(x, y);
        }
        __syncthreads();
    }
    for (uint32_t e = tid; e < tile_n; e += NTT_THREADS) {
        const uint32_t t = e >> logW, w = e & (W - 1);
        const size_t j = base + (size_t)t * stride + w;
        uint64_t v = tile[e];
        d[j] = canon_out ? gl::canon(v) : v;
    }
}

// ------------------------------------------------------- bit-reverse + scale
// dst[bitrev(i)] = src[i] * scale (canonical).  i = (a | m | b) with a, b of A bits:
// a 2^A x 2^A tile for fixed m is read with rows a (contiguous b) and written with rows
// bitrev(b) (contiguous bitrev(a)), transposed through LDS: both sides are runs of 2^A.
__global__ __launch_bounds__(256) void bitrev_scale_kernel(uint64_t* dst, size_t dst_stride, const uint64_t* src,
                                                           size_t src_stride, uint32_t log_n, uint32_t A,
                                                           uint64_t scale) {
    __shared__ uint64_t t[32 * 33];
    const size_t col = blockIdx.y;
    const uint32_t M = log_n - 2 * A;  // middle bits
    const uint32_t m = blockIdx.x;     // < 2^M
    const uint32_t side = 1u << A;
    const uint32_t mrev = gl::bitrev32(m, M);
    const uint64_t* s = src + col * src_stride;
    uint64_t* d = dst + col * dst_stride;
    for (uint32_t e = threadIdx.x; e < side * side; e += blockDim.x) {
        const uint32_t a = e >> A, bb = e & (side - 1);
        const size_t i = ((size_t)a << (M + A)) | ((size_t)m << A) | bb;
        t[a * 33 + bb] = s[i];
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < side * side; e += blockDim.x) {
        // output index o = (rb | mrev | ra), rb = bitrev(b) row, ra = bitrev(a) contiguous
        const uint32_t rb = e >> A, ra = e & (side - 1);
        const uint32_t a = gl::bitrev32(ra, A), bb = gl::bitrev32(rb, A);
        const size_t o = ((size_t)rb << (M + A)) | ((size_t)mrev << A) | ra;
        d[o] = gl::canon(gl::mul(t[a * 33 + bb], scale));
    }
}

// Small or degenerate sizes: elementwise copy with optional scale/canon.
__global__ void scale_copy_kernel(uint64_t* dst, size_t dst_stride, const uint64_t* src, size_t src_stride,
                                  size_t n, uint64_t scale) {
    const size_t col = blockIdx.y;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[col * dst_stride + i] = gl::canon(gl::mul(src[col * src_stride + i], scale));
}

// distribute_powers with tables (fft/mod.rs:308-317).
__global__ void distribute_kernel(uint64_t* cols, size_t col_stride, size_t n, const uint64_t* __restrict__ lo,
                                  const uint64_t* __restrict__ hi) {
    const size_t col = blockIdx.y;
    for (size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x; j < n; j += (size_t)gridDim.x * blockDim.x) {
        uint64_t* p = cols + col * col_stride + j;
        *p = gl::canon(gl::mul(*p, gl::mul(hi[j >> 12], lo[j & 4095])));
    }
}

// ------------------------------------------------------------------ launchers

static inline dim3 grid2(size_t x, uint32_t y) { return dim3((unsigned)x, y, 1); }

// Full natural->bit-reversed transform of n_cols columns (src -> dst; src may == dst),
// with optional coset power tables applied on load.
hipError_t launch_ntt_nb(uint64_t* dst, size_t dst_stride, const uint64_t* src, size_t src_stride,
                         uint32_t n_cols, uint32_t log_n, const uint64_t* tw, const uint64_t* pw_lo,
                         const uint64_t* pw_hi, bool canon_out, hipStream_t st) {
    if (n_cols == 0) return hipSuccess;
    if (log_n == 0) {
        // n == 1: transform is the identity (fft/mod.rs:666-668); coset power is e^0 = 1.
        hipLaunchKernelGGL(scale_copy_kernel, grid2(1, n_cols), dim3(64), 0, st, dst, dst_stride, src, src_stride,
                           (size_t)1, (uint64_t)1);
        return hipGetLastError();
    }
    // Plan: a last pass of min(log_n, 12) stages on contiguous tiles; the stages before it
    // split into passes of <= 8 stages (W = 2^(12-R) adjacent sub-problems per tile).
    const uint32_t last = log_n < (uint32_t)TILE_LOG ? log_n : (uint32_t)TILE_LOG;
    const uint32_t front = log_n - last;
    const uint32_t npass_front = (front + 7) / 8;
    uint32_t s0 = 0;
    const uint64_t* cur_src = src;
    size_t cur_stride = src_stride;
    for (uint32_t p = 0; p < npass_front; p++) {
        const uint32_t R = (front - s0 + (npass_front - p) - 1) / (npass_front - p);
        const uint32_t logW = TILE_LOG - R;
        const size_t tiles = ((size_t)1 << log_n) >> TILE_LOG;
        hipLaunchKernelGGL(ntt_pass_kernel, grid2(tiles, n_cols), dim3(NTT_THREADS), 0, st, dst, dst_stride,
                           cur_src, cur_stride, log_n, s0, R, logW, tw, p == 0 ? pw_lo : nullptr,
                           p == 0 ? pw_hi : nullptr, 0);
        s0 += R;
        cur_src = dst;
        cur_stride = dst_stride;
    }
    {
        const size_t tiles = ((size_t)1 << log_n) >> last;
        hipLaunchKernelGGL(ntt_pass_kernel, grid2(tiles, n_cols), dim3(NTT_THREADS), 0, st, dst, dst_stride,
                           cur_src, cur_stride, log_n, s0, last, 0u, tw, npass_front == 0 ? pw_lo : nullptr,
                           npass_front == 0 ? pw_hi : nullptr, canon_out ? 1 : 0);
    }
    return hipGetLastError();
}

hipError_t launch_bitrev_scale(uint64_t* dst, size_t dst_stride, const uint64_t* src, size_t src_stride,
                               uint32_t n_cols, uint32_t log_n, uint64_t scale, hipStream_t st) {
    if (n_cols == 0) return hipSuccess;
    if (log_n < 2) {  // bit reversal of 1 or 2 elements is the identity
        hipLaunchKernelGGL(scale_copy_kernel, grid2(1, n_cols), dim3(64), 0, st, dst, dst_stride, src, src_stride,
                           (size_t)1 << log_n, scale);
        return hipGetLastError();
    }
    uint32_t A = log_n / 2;
    if (A > 5) A = 5;
    const uint32_t M = log_n - 2 * A;
    hipLaunchKernelGGL(bitrev_scale_kernel, grid2((size_t)1 << M, n_cols), dim3(256), 0, st, dst, dst_stride, src,
                       src_stride, log_n, A, scale);
    return hipGetLastError();
}

hipError_t launch_twiddles(uint64_t* out, uint32_t log_n, bool inverse, hipStream_t st) {
    if (log_n == 0) return hipSuccess;
    uint64_t w = gl::domain_generator(log_n);
    if (inverse) w = gl::canon(gl::inv(w));
    size_t half = (size_t)1 << (log_n - 1);
    size_t blocks = (half + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(twiddles_kernel, dim3((unsigned)blocks), dim3(256), 0, st, out, log_n, w);
    return hipGetLastError();
}

hipError_t launch_twiddles_natural(uint64_t* out, uint32_t log_n, bool inverse, hipStream_t st) {
    if (log_n == 0) return hipSuccess;
    uint64_t w = gl::domain_generator(log_n);
    if (inverse) w = gl::canon(gl::inv(w));
    size_t half = (size_t)1 << (log_n - 1);
    size_t blocks = (half + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(twiddles_natural_kernel, dim3((unsigned)blocks), dim3(256), 0, st, out, log_n, w);
    return hipGetLastError();
}

hipError_t launch_bitrev_inplace(uint64_t* cols, size_t col_stride, uint32_t n_cols, uint32_t log_n, hipStream_t st) {
    if (n_cols == 0 || log_n < 2) return hipSuccess;
    size_t n = (size_t)1 << log_n;
    size_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(bitrev_inplace_kernel, dim3((unsigned)blocks, n_cols), dim3(256), 0, st, cols, col_stride,
                       log_n);
    return hipGetLastError();
}

hipError_t launch_power_tables(uint64_t* lo, uint64_t* hi, uint32_t log_n, uint64_t e, uint64_t scale,
                               hipStream_t st) {
    uint32_t n_hi = log_n > 12 ? (1u << (log_n - 12)) : 1u;
    uint32_t total = n_hi > 4096 ? n_hi : 4096;
    hipLaunchKernelGGL(power_tables_kernel, dim3((total + 255) / 256), dim3(256), 0, st, lo, hi, n_hi, e, scale);
    return hipGetLastError();
}

hipError_t launch_distribute(uint64_t* cols, size_t col_stride, uint32_t n_cols, uint32_t log_n,
                             const uint64_t* lo, const uint64_t* hi, hipStream_t st) {
    if (n_cols == 0) return hipSuccess;
    size_t n = (size_t)1 << log_n;
    size_t blocks = (n + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(distribute_kernel, grid2(blocks, n_cols), dim3(256), 0, st, cols, col_stride, n, lo, hi);
    return hipGetLastError();
}

}  // namespace bj

namespace bj {

// Synthetic trace: x = splitmix64(seed + c*n + r), reduced once mod p.
// A bench/test utility: the reference fills its trace from witness generation.
__global__ void synthetic_kernel(uint64_t* dst, size_t col_stride, uint32_t log_n, uint64_t seed, uint64_t col0) {
    const size_t n = (size_t)1 << log_n;
    const size_t col = blockIdx.y;
    for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < n; r += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (col0 + col) * n + r + 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z = z ^ (z >> 31);
        dst[col * col_stride + r] = z >= gl::P ? z - gl::P : z;
    }
}

hipError_t launch_synthetic(uint64_t* dst, size_t col_stride, uint32_t n_cols, uint32_t log_n, uint64_t seed,
                            uint64_t col0, hipStream_t st) {
    if (n_cols == 0) return hipSuccess;
    size_t n = (size_t)1 << log_n;
    size_t blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(synthetic_kernel, dim3((unsigned)blocks, n_cols), dim3(256), 0, st, dst, col_stride, log_n,
                       seed, col0);
    return hipGetLastError();
}

}  // namespace bj
