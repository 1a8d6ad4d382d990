// NTT support kernels (gfx950): the iFFT bit-reverse/scale pass, the in-place bit reversal,
// coset power tables, distribute_powers, twiddle tables (bit-reversed and natural order) and
// the synthetic trace generator.  The transforms themselves are ntt_ct.hip (2^13..2^23) and
// ntt_dif.hip (smaller sizes).
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "bj_internal.hpp"

namespace bj {


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
