// FRI folding by 2 of a GoldilocksExt2 codeword held as two base columns (c0, c1).
//
// fold_multiple (cs/implementations/fri/mod.rs:362-474), as used by
// interpolate_independent_cosets (:476-585) and interpolate_flattened_cosets (:587-682):
// the codeword is bit-reversed, so f(x) and f(-x) are neighbours (2i, 2i + 1), and
//   out_i = f(x) + f(-x) + alpha * (f(x) - f(-x)) * roots[i] * coset_inverse,
// with alpha = (ch0, ch1) in GoldilocksExt2 (u^2 = 7, field/goldilocks/extension.rs:14-40,
// product as field/traits/field.rs:407-424) and roots the INVERSED bit-reversed twiddles of the
// full domain (precompute_twiddles_for_fft::<true>, fri/mod.rs:191-192). Over several cosets
// stored one after another the root index is the flat pair index, which is what both
// reference loops use. Outputs are canonical.
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "bj_internal.hpp"

namespace bj {

namespace {

constexpr uint64_t EXT2_NON_RESIDUE = 7;  // GoldilocksExt2::NON_RESIDUE (extension.rs:14-16)

__global__ __launch_bounds__(256) void fri_fold_kernel(const uint64_t* __restrict__ c0, const uint64_t* __restrict__ c1,
                                                       size_t n_out, const uint64_t* __restrict__ roots,
                                                       uint64_t coset_inverse, uint64_t ch0, uint64_t ch1,
                                                       uint64_t* __restrict__ d0, uint64_t* __restrict__ d1) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_out; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t x0 = c0[2 * i], mx0 = c0[2 * i + 1];
        const uint64_t x1 = c1[2 * i], mx1 = c1[2 * i + 1];
        const uint64_t r = gl::mul(roots[i], coset_inverse);
        const uint64_t a0 = gl::mul(gl::sub(x0, mx0), r);
        const uint64_t a1 = gl::mul(gl::sub(x1, mx1), r);
        // (a0 + a1 u) (ch0 + ch1 u), u^2 = 7
        const uint64_t v0 = gl::mul(a0, ch0);
        const uint64_t v1 = gl::mul(a1, ch1);
        const uint64_t m = gl::mul(gl::add(a0, a1), gl::add(ch0, ch1));
        const uint64_t e1 = gl::sub(gl::sub(m, v0), v1);
        const uint64_t e0 = gl::add(v0, gl::mul(v1, EXT2_NON_RESIDUE));
        d0[i] = gl::canon(gl::add(gl::add(e0, x0), mx0));
        d1[i] = gl::canon(gl::add(gl::add(e1, x1), mx1));
    }
}

}  // namespace

hipError_t launch_fri_fold(const uint64_t* c0, const uint64_t* c1, size_t n_out, const uint64_t* roots,
                           uint64_t coset_inverse, uint64_t ch0, uint64_t ch1, uint64_t* d0, uint64_t* d1,
                           hipStream_t st) {
    if (n_out == 0) return hipSuccess;
    size_t blocks = (n_out + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(fri_fold_kernel, dim3((unsigned)blocks), dim3(256), 0, st, c0, c1, n_out, roots,
                       gl::canon(coset_inverse), gl::canon(ch0), gl::canon(ch1), d0, d1);
    return hipGetLastError();
}

}  // namespace bj
