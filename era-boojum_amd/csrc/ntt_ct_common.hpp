// Register-level building blocks shared by the CT NTT passes (ntt_ct.hip) and the three-pass
// LDE (ntt_lde3.hip): the CT butterfly on four pairs, register stages, the power-of-two register
// phases (prescale + DFT), the prescale-table offsets and the padded LDS
// exchange layouts.  Everything is in an anonymous namespace: each translation unit gets its
// own copy, inlined.
#pragma once
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "gl_asm.hpp"
#include "ntt_pow2.hpp"

namespace bj {
namespace {

constexpr int NT = 256;
constexpr int PT = 32;
constexpr int TILE = NT * PT;

__device__ __forceinline__ void split2(uint64_t x, uint32_t& lo, uint32_t& hi) {
    lo = (uint32_t)x;
    hi = (uint32_t)(x >> 32);
}
__device__ __forceinline__ uint64_t join2(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

// CT butterflies on four pairs: t = c * mu; (a, c) <- (a + t, a - t)
// (glasm::ct_bfly_x4: t canonicalised, then one correcting 64-bit mad per output).
__device__ __forceinline__ void ct_bfly_x4(uint64_t& xa0, uint64_t& xc0, uint64_t& xa1, uint64_t& xc1,
                                           uint64_t& xa2, uint64_t& xc2, uint64_t& xa3, uint64_t& xc3, uint64_t w0,
                                           uint64_t w1, uint64_t w2, uint64_t w3) {
    uint64_t A[4], C[4];
    glasm::ct_bfly_x4((uint32_t)xa0, (uint32_t)(xa0 >> 32), (uint32_t)xc0, (uint32_t)(xc0 >> 32), (uint32_t)w0,
                      (uint32_t)(w0 >> 32), A[0], C[0],
                      (uint32_t)xa1, (uint32_t)(xa1 >> 32), (uint32_t)xc1, (uint32_t)(xc1 >> 32), (uint32_t)w1,
                      (uint32_t)(w1 >> 32), A[1], C[1],
                      (uint32_t)xa2, (uint32_t)(xa2 >> 32), (uint32_t)xc2, (uint32_t)(xc2 >> 32), (uint32_t)w2,
                      (uint32_t)(w2 >> 32), A[2], C[2],
                      (uint32_t)xa3, (uint32_t)(xa3 >> 32), (uint32_t)xc3, (uint32_t)(xc3 >> 32), (uint32_t)w3,
                      (uint32_t)(w3 >> 32), A[3], C[3]);
    xa0 = A[0]; xc0 = C[0];
    xa1 = A[1]; xc1 = C[1];
    xa2 = A[2]; xc2 = C[2];
    xa3 = A[3]; xc3 = C[3];
}

__device__ __forceinline__ void mul4_by(uint64_t& x0, uint64_t& x1, uint64_t& x2, uint64_t& x3, uint64_t k) {
    uint32_t a0[4], a1[4], z0[4], z1[4], k0, k1;
    split2(k, k0, k1);
    split2(x0, a0[0], a1[0]); split2(x1, a0[1], a1[1]);
    split2(x2, a0[2], a1[2]); split2(x3, a0[3], a1[3]);
    glasm::mul_x4(a0[0], a1[0], k0, k1, z0[0], z1[0], a0[1], a1[1], k0, k1, z0[1], z1[1],
                  a0[2], a1[2], k0, k1, z0[2], z1[2], a0[3], a1[3], k0, k1, z0[3], z1[3]);
    x0 = join2(z0[0], z1[0]); x1 = join2(z0[1], z1[1]);
    x2 = join2(z0[2], z1[2]); x3 = join2(z0[3], z1[3]);
}

__device__ __forceinline__ constexpr int pair_lo(int q, int hk) { return (q / hk) * 2 * hk + (q % hk); }

// One register stage on x[32], pairs (k, k + HK); w[q] = twiddle of pair q.
template <int HK>
__device__ __forceinline__ void ct_stage(uint64_t* x, const uint64_t* w) {
#pragma unroll
    for (int b = 0; b < 4; b++) {
        const int q0 = 4 * b;
        ct_bfly_x4(x[pair_lo(q0, HK)], x[pair_lo(q0, HK) + HK], x[pair_lo(q0 + 1, HK)], x[pair_lo(q0 + 1, HK) + HK],
                   x[pair_lo(q0 + 2, HK)], x[pair_lo(q0 + 2, HK) + HK], x[pair_lo(q0 + 3, HK)],
                   x[pair_lo(q0 + 3, HK) + HK], w[q0], w[q0 + 1], w[q0 + 2], w[q0 + 3]);
    }
}

__device__ __forceinline__ void canon4(uint64_t* x) {
    uint32_t z0[4], z1[4];
    glasm::canon_x4((uint32_t)x[0], (uint32_t)(x[0] >> 32), z0[0], z1[0], (uint32_t)x[1], (uint32_t)(x[1] >> 32), z0[1],
                    z1[1], (uint32_t)x[2], (uint32_t)(x[2] >> 32), z0[2], z1[2], (uint32_t)x[3], (uint32_t)(x[3] >> 32),
                    z0[3], z1[3]);
#pragma unroll
    for (int i = 0; i < 4; i++) x[i] = join2(z0[i], z1[i]);
}

__device__ __forceinline__ uint64_t canon_u64(uint64_t v) {
    uint32_t a0, a1, z0, z1;
    split2(v, a0, a1);
    glasm::canon_x1(a0, a1, z0, z1);
    return join2(z0, z1);
}

// ------------------------------------------------- power-of-two register phases (round 2)
//
// A register phase of r <= 5 stages acts on 2^r elements of one group of the network, whose
// polynomial Q is evaluated on a coset sigma <w>: with the elements at coefficient distance M,
// the phase is a 2^r-point DFT of (q_k sigma^(M k)) with the root w_{2^r}. So
// each phase multiplies its inputs by a prescale table once (one general product per element)
// and runs a DFT whose twiddles are +-2^e (csrc/ntt_pow2.hpp): 5 stages cost ~15% fewer
// instructions than the coset-folded general stages (tools/pow2_bench.hip).
//
// Table extension (after the n-entry CT table of a shift s, ct_table_len):
//   [0, 32)              HA[k] = s^((n/32) k)                       head phase A' (rows s + T k)
//   [32, 32 + 2^R)       HB[r] = sigma5_(r >> (R-5))^((n >> R) (r & (2^(R-5) - 1)))   phase B'
//   [EXT_TA, +32 2^u0)   TA[q][k] = sigma_u0(q)^(256 k) (x n^-1 for the inverse, 18 <= log n <= 23)
//   [ext_tb, +32 2^(u0+5)) TB[g][k] = sigma_(u0+5)(g)^(8 k)
// with sigma_u(g) = s w_n^bitrev_u(g), the coset of group g after u stages.
constexpr size_t EXT_HB = 32;
constexpr size_t EXT_TA = 32 + 1024;
__host__ __device__ __forceinline__ size_t ext_tb(uint32_t u0) { return EXT_TA + ((size_t)32 << u0); }

template <int LOG, bool INV, int B>
__device__ __forceinline__ void dft_p2(uint64_t* x) {
    using namespace p2dft;
    if constexpr (LOG == 1) { if constexpr (INV) dft2_inv<B>(x); else dft2_fwd<B>(x); }
    if constexpr (LOG == 2) { if constexpr (INV) dft4_inv<B>(x); else dft4_fwd<B>(x); }
    if constexpr (LOG == 3) { if constexpr (INV) dft8_inv<B>(x); else dft8_fwd<B>(x); }
    if constexpr (LOG == 4) { if constexpr (INV) dft16_inv<B>(x); else dft16_fwd<B>(x); }
    if constexpr (LOG == 5) { if constexpr (INV) dft32_inv<B>(x); else dft32_fwd<B>(x); }
}

// the 32 / 2^LOG register groups of a phase, each a 2^LOG-point DFT
template <int LOG, bool INV, int G = 0>
__device__ __forceinline__ void dft_p2_groups(uint64_t* x) {
    if constexpr (G < (32 >> LOG)) {
        dft_p2<LOG, INV, (G << LOG)>(x);
        dft_p2_groups<LOG, INV, G + 1>(x);
    }
}

// the 32 factors of a prescale into registers, issued ahead of the phase that uses them (before
// an exchange's barrier, so their latency overlaps it: the scheduler does not move loads across
// the barrier, and after it they sat right before each product)
__device__ __forceinline__ void load32(uint64_t* r, const uint64_t* __restrict__ f) {
#pragma unroll
    for (int k = 0; k < PT; k++) r[k] = f[k];
}

// x[k] *= f[k] for k < K (K a multiple of 4)
template <int K>
__device__ __forceinline__ void prescale_n(uint64_t* x, const uint64_t* f) {
#pragma unroll
    for (int k = 0; k < K; k += 4) {
        uint32_t z0[4], z1[4];
        glasm::mul_x4((uint32_t)x[k], (uint32_t)(x[k] >> 32), (uint32_t)f[k], (uint32_t)(f[k] >> 32), z0[0], z1[0],
                      (uint32_t)x[k + 1], (uint32_t)(x[k + 1] >> 32), (uint32_t)f[k + 1], (uint32_t)(f[k + 1] >> 32),
                      z0[1], z1[1], (uint32_t)x[k + 2], (uint32_t)(x[k + 2] >> 32), (uint32_t)f[k + 2],
                      (uint32_t)(f[k + 2] >> 32), z0[2], z1[2], (uint32_t)x[k + 3], (uint32_t)(x[k + 3] >> 32),
                      (uint32_t)f[k + 3], (uint32_t)(f[k + 3] >> 32), z0[3], z1[3]);
#pragma unroll
        for (int i = 0; i < 4; i++) x[k + i] = join2(z0[i], z1[i]);
    }
}

// x[k] *= f[k] for k < 32 (general products; outputs any u64 representative)
__device__ __forceinline__ void prescale32(uint64_t* x, const uint64_t* f) {
#pragma unroll
    for (int k = 0; k < PT; k += 4) {
        uint32_t z0[4], z1[4];
        glasm::mul_x4((uint32_t)x[k], (uint32_t)(x[k] >> 32), (uint32_t)f[k], (uint32_t)(f[k] >> 32), z0[0], z1[0],
                      (uint32_t)x[k + 1], (uint32_t)(x[k + 1] >> 32), (uint32_t)f[k + 1], (uint32_t)(f[k + 1] >> 32),
                      z0[1], z1[1], (uint32_t)x[k + 2], (uint32_t)(x[k + 2] >> 32), (uint32_t)f[k + 2],
                      (uint32_t)(f[k + 2] >> 32), z0[2], z1[2], (uint32_t)x[k + 3], (uint32_t)(x[k + 3] >> 32),
                      (uint32_t)f[k + 3], (uint32_t)(f[k + 3] >> 32), z0[3], z1[3]);
#pragma unroll
        for (int i = 0; i < 4; i++) x[k + i] = join2(z0[i], z1[i]);
    }
}

// Padded LDS layout shared by the head exchange and the tail: element e at slot e + (e >> 5).
constexpr int PAD_LDS = TILE + TILE / 32;

// Tail LDS layout: element e at slot e + (e >> 5) (one pad word per 32). For the three
// exchange patterns the slot splits into a per-thread base plus a compile-time offset per
// register k, so every ds_read / ds_write takes its k-part as an immediate offset and needs no
// address VALU:
//   A: e = t + 256 k                         -> (t + (t >> 5)) + 264 k
//   B: e = (thi << 8) | (k << 3) | tlo       -> (264 thi + tlo) + 8 k + (k >> 2)
//   C: e = 32 t + k                          -> 33 t + k
// and each is bank-conflict free for ds_read_b64 / ds_write_b64 (32 consecutive lanes hit 32
// distinct 8-byte slots mod 32, up to one pad skip in pattern A).
__device__ __forceinline__ uint32_t tail_base_a(uint32_t t) { return t + (t >> 5); }
__device__ __forceinline__ uint32_t tail_base_b(uint32_t thi, uint32_t tlo) { return 264 * thi + tlo; }
__device__ __forceinline__ uint32_t tail_base_c(uint32_t t) { return 33 * t; }
__device__ __forceinline__ constexpr uint32_t tail_off_a(int k) { return 264 * k; }
__device__ __forceinline__ constexpr uint32_t tail_off_b(int k) { return 8 * k + (k >> 2); }

// phase C (element 32 t + k, v = 10..12): (q << v) + (t << (v-8)) + (lo >> (13-v)).
template <int V>
__device__ __forceinline__ void tw_ct_tailC(uint64_t* w, const uint64_t* __restrict__ ct, uint32_t u0, size_t q,
                                            uint32_t t) {
    constexpr int HK = 4 >> (V - 10);
    const uint64_t* base = ct + ((size_t)1 << (u0 + V)) + (q << V) + ((size_t)t << (V - 8));
#pragma unroll
    for (int p = 0; p < 16; p++) w[p] = base[pair_lo(p, HK) >> (13 - V)];
}

}  // namespace
}  // namespace bj
