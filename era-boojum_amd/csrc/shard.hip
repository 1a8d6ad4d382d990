// Sub-coset fold for the coset-sharded LDE, used when the number of shards G
// exceeds the LDE degree D and a shard owns m = n*D/G < n consecutive leaves of one coset.
//
// Those leaves are p(s' * w_m^{bitrev_m(u)}), u < m, with s' = 7 * w_{nD}^{bitrev_{log G}(P)}:
// an m-point coset evaluation of  h(Y) = sum_t h_t Y^t,  h_t = sum_{a<F} c_{t+a m} (s'^m)^a,
// F = n / m, followed by the usual s'^t scaling.  The coefficient buffer is bit-reversed
// (c_j at bitrev_n(j)), so the F terms of h_t sit next to each other:
//   bitrev_n(t + a m) = bitrev_m(t) * F + bitrev_F(a)
// and the folded buffer comes out bit-reversed too (h_t at bitrev_m(t)) - the layout the
// LDE head pass gathers from.  One coalesced read of n, one write of m per column.
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "bj_internal.hpp"

namespace bj {

namespace {

// z[bitrev_F(a)] = (s'^m)^a, so out[u] = sum_b src[u F + b] * z[b].
struct FoldConsts {
    uint64_t z[kMaxFold];
};

__global__ __launch_bounds__(256) void fold_kernel(uint64_t* dst, size_t dst_stride, const uint64_t* src,
                                                   size_t src_stride, size_t m, uint32_t log_f, FoldConsts zc) {
    const uint64_t* s = src + (size_t)blockIdx.y * src_stride;
    uint64_t* d = dst + (size_t)blockIdx.y * dst_stride;
    const uint32_t F = 1u << log_f;
    for (size_t u = (size_t)blockIdx.x * blockDim.x + threadIdx.x; u < m; u += (size_t)gridDim.x * blockDim.x) {
        const uint64_t* row = s + (u << log_f);
        uint64_t acc = row[0];  // z[0] = 1
        for (uint32_t b = 1; b < F; b++) acc = gl::add(acc, gl::mul(row[b], zc.z[b]));
        d[u] = acc;
    }
}

// Sender-side fold for every shard at once (the all-to-all exchange): one read of the F
// adjacent terms of h_t, G outputs.  z[P * F + b] = (s_P^m)^a at b = bitrev_F(a).
constexpr uint32_t kMaxFoldConsts = 256;
struct FoldAllConsts {
    uint64_t z[kMaxFoldConsts];
};

template <uint32_t LOG_F>
__global__ __launch_bounds__(256) void fold_all_kernel(uint64_t* dst, size_t dst_col_stride,
                                                       size_t dst_shard_stride, const uint64_t* src,
                                                       size_t src_stride, size_t m, uint32_t shards,
                                                       FoldAllConsts zc) {
    constexpr uint32_t F = 1u << LOG_F;
    const uint64_t* s = src + (size_t)blockIdx.y * src_stride;
    uint64_t* d = dst + (size_t)blockIdx.y * dst_col_stride;
    for (size_t u = (size_t)blockIdx.x * blockDim.x + threadIdx.x; u < m; u += (size_t)gridDim.x * blockDim.x) {
        const uint64_t* row = s + (u << LOG_F);
        uint64_t r[F];
#pragma unroll
        for (uint32_t b = 0; b < F; b++) r[b] = row[b];
        for (uint32_t P = 0; P < shards; P++) {
            const uint64_t* z = zc.z + P * F;
            uint64_t acc = r[0];
#pragma unroll
            for (uint32_t b = 1; b < F; b++) acc = gl::add(acc, gl::mul(r[b], z[b]));
            d[(size_t)P * dst_shard_stride + u] = acc;
        }
    }
}

}  // namespace

hipError_t launch_fold(uint64_t* dst, size_t dst_stride, const uint64_t* src, size_t src_stride, uint32_t n_cols,
                       uint32_t log_m, uint32_t log_f, uint64_t s_pow_m, hipStream_t st) {
    if (n_cols == 0) return hipSuccess;
    if (log_f == 0 || (1u << log_f) > kMaxFold) return hipErrorInvalidValue;
    FoldConsts zc;
    const uint32_t F = 1u << log_f;
    uint64_t acc = 1;
    for (uint32_t a = 0; a < F; a++) {
        zc.z[gl::bitrev32(a, log_f)] = acc;
        acc = gl::mul(acc, s_pow_m);
    }
    const size_t m = (size_t)1 << log_m;
    size_t blocks = (m + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(fold_kernel, dim3((unsigned)blocks, n_cols), dim3(256), 0, st, dst, dst_stride, src,
                       src_stride, m, log_f, zc);
    return hipGetLastError();
}

hipError_t launch_fold_all(uint64_t* dst, size_t dst_col_stride, size_t dst_shard_stride, const uint64_t* src,
                           size_t src_stride, uint32_t n_cols, uint32_t log_m, uint32_t log_f, uint32_t shards,
                           const uint64_t* s_pow_m, hipStream_t st) {
    if (n_cols == 0 || shards == 0) return hipSuccess;
    if (log_f == 0 || (1u << log_f) > kMaxFold) return hipErrorInvalidValue;
    const uint32_t F = 1u << log_f;
    const size_t m = (size_t)1 << log_m;
    if ((size_t)shards * F > kMaxFoldConsts || log_f > 3) {
        // too many constants for one launch: one single-shard fold per target
        for (uint32_t P = 0; P < shards; P++) {
            hipError_t e = launch_fold(dst + (size_t)P * dst_shard_stride, dst_col_stride, src, src_stride, n_cols,
                                       log_m, log_f, s_pow_m[P], st);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    FoldAllConsts zc;
    for (uint32_t P = 0; P < shards; P++) {
        uint64_t acc = 1;
        for (uint32_t a = 0; a < F; a++) {
            zc.z[P * F + gl::bitrev32(a, log_f)] = acc;
            acc = gl::mul(acc, s_pow_m[P]);
        }
    }
    size_t blocks = (m + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    const dim3 grid((unsigned)blocks, n_cols);
    if (log_f == 1)
        hipLaunchKernelGGL(fold_all_kernel<1>, grid, dim3(256), 0, st, dst, dst_col_stride, dst_shard_stride, src,
                           src_stride, m, shards, zc);
    else if (log_f == 2)
        hipLaunchKernelGGL(fold_all_kernel<2>, grid, dim3(256), 0, st, dst, dst_col_stride, dst_shard_stride, src,
                           src_stride, m, shards, zc);
    else
        hipLaunchKernelGGL(fold_all_kernel<3>, grid, dim3(256), 0, st, dst, dst_col_stride, dst_shard_stride, src,
                           src_stride, m, shards, zc);
    return hipGetLastError();
}

}  // namespace bj
