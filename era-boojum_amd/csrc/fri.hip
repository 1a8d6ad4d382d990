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
#include "gl_asm.hpp"
#include "bj_internal.hpp"

namespace bj {

namespace {

constexpr uint64_t EXT2_NON_RESIDUE = 7;  // GoldilocksExt2::NON_RESIDUE (extension.rs:14-16)
static_assert(EXT2_NON_RESIDUE == (1u << 3) - 1, "the fold multiplies by the non-residue as 2^3 v - v");

__device__ __forceinline__ void halves(uint64_t x, uint32_t& lo, uint32_t& hi) {
    lo = (uint32_t)x;
    hi = (uint32_t)(x >> 32);
}
__device__ __forceinline__ uint64_t join(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

// beta = alpha * coset_inverse (an Ext2 times a base element, folded on the host) and
// bsum = beta0 + beta1, so each output costs six products: (d0, d1) * roots[i] (2), the Karatsuba
// Ext2 product by beta (3) and the non-residue multiple (1), as interleaved gfx950 asm products
// (glasm, 14 instructions each).  Pairs (x, -x) are one 16-byte load per column when both
// columns are 16-byte aligned (V16), two 8-byte loads otherwise.
template <bool V16>
__device__ __forceinline__ ulonglong2 load_pair(const uint64_t* __restrict__ c, size_t i) {
    if constexpr (V16) return reinterpret_cast<const ulonglong2*>(c)[i];
    return make_ulonglong2(c[2 * i], c[2 * i + 1]);
}

template <bool V16>
__global__ __launch_bounds__(256) void fri_fold_kernel(const uint64_t* __restrict__ c0,
                                                       const uint64_t* __restrict__ c1, size_t n_out,
                                                       const uint64_t* __restrict__ roots, uint64_t beta0,
                                                       uint64_t beta1, uint64_t bsum, uint64_t* __restrict__ d0,
                                                       uint64_t* __restrict__ d1) {
    uint32_t b0l, b0h, b1l, b1h, bsl, bsh;
    halves(beta0, b0l, b0h);
    halves(beta1, b1l, b1h);
    halves(bsum, bsl, bsh);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_out; i += (size_t)gridDim.x * blockDim.x) {
        const ulonglong2 p0 = load_pair<V16>(c0, i), p1 = load_pair<V16>(c1, i);  // (f(x), f(-x))
        const uint64_t r = roots[i];
        uint32_t s0l, s0h, s1l, s1h, rl, rh;
        halves(gl::sub(p0.x, p0.y), s0l, s0h);
        halves(gl::sub(p1.x, p1.y), s1l, s1h);
        halves(r, rl, rh);
        uint32_t a0l, a0h, a1l, a1h;
        glasm::mul_x2(s0l, s0h, rl, rh, a0l, a0h, s1l, s1h, rl, rh, a1l, a1h);
        uint32_t sal, sah;
        halves(gl::add(join(a0l, a0h), join(a1l, a1h)), sal, sah);
        // (a0 + a1 u) (beta0 + beta1 u), u^2 = 7 (field/traits/field.rs:407-424)
        uint32_t v0l, v0h, v1l, v1h, ml, mh;
        glasm::mul_x3(a0l, a0h, b0l, b0h, v0l, v0h, a1l, a1h, b1l, b1h, v1l, v1h, sal, sah, bsl, bsh, ml, mh);
        const uint64_t v0 = join(v0l, v0h), v1 = join(v1l, v1h);
        const uint64_t e1 = gl::sub(gl::sub(join(ml, mh), v0), v1);
        const uint64_t e0 = gl::add(v0, gl::sub(gl::mul_pow2_small(v1, 3), v1));  // v0 + 7 v1
        d0[i] = gl::canon(gl::add(gl::add(e0, p0.x), p0.y));
        d1[i] = gl::canon(gl::add(gl::add(e1, p1.x), p1.y));
    }
}

}  // namespace

hipError_t launch_fri_fold(const uint64_t* c0, const uint64_t* c1, size_t n_out, const uint64_t* roots,
                           uint64_t coset_inverse, uint64_t ch0, uint64_t ch1, uint64_t* d0, uint64_t* d1,
                           hipStream_t st) {
    if (n_out == 0) return hipSuccess;
    if (((uintptr_t)c0 | (uintptr_t)c1) % 8) return hipErrorInvalidValue;  // u64 elements
    size_t blocks = (n_out + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    const uint64_t beta0 = gl::canon(gl::mul(ch0, coset_inverse)), beta1 = gl::canon(gl::mul(ch1, coset_inverse));
    const uint64_t bsum = gl::canon(gl::add(beta0, beta1));
    if (((uintptr_t)c0 | (uintptr_t)c1) % 16 == 0)
        hipLaunchKernelGGL(fri_fold_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, c0, c1, n_out, roots,
                           beta0, beta1, bsum, d0, d1);
    else
        hipLaunchKernelGGL(fri_fold_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, c0, c1, n_out, roots,
                           beta0, beta1, bsum, d0, d1);
    return hipGetLastError();
}

}  // namespace bj
