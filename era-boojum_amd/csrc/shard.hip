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

}  // namespace bj
