// Poseidon2 (width 12) with one permutation spread over the four lanes of a quad, for the tree
// levels with too few nodes to fill the chip: there a level costs one permutation's latency
// (~20 us with the whole state in one lane), and this form cuts the instructions on that
// dependency chain by ~2.5x.  Same permutation and field values as p2::permute
// (implementations/poseidon2/state_generic_impl.rs:221-236).
//
// Lane p (= lane & 3) holds the state elements p, p + 4, p + 8: position p of the three blocks
// of the external MDS (block-circulant(2 M4, M4, M4), implementations/suggested_mds.rs:19-97).
// * external MDS: M4 mixes the positions of a block, so lane p forms row p of M4 from its own
//   value and its three quad neighbours' (DPP quad permutes, no LDS); the block sums are lane-local;
// * full rounds: each lane adds its three round constants (staged in LDS by the kernel) and
//   applies three S-boxes;
// * partial rounds: every lane runs the S-box on its block-0 element and only lane 0 keeps it
//   (element 0); M_I = diag(2^sh) + 1 1^T needs the sum of all twelve: a lane-local sum of three
//   and a two-step quad butterfly;
// * linear layers on limbs (L = sum c lo, H = sum c hi, 64-bit, carry-free) and the 4-instruction
//   reduction, as in poseidon2.hpp.
#pragma once
#include "poseidon2.hpp"

namespace p2q {

// quad_perm controls: lane p reads lane p ^ 1, p ^ 2, p ^ 3 of its quad
constexpr int QP_X1 = 0xB1, QP_X2 = 0x4E, QP_X3 = 0x1B;

template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t qperm64(uint64_t v) {
    return ((uint64_t)qperm<CTRL>((uint32_t)(v >> 32)) << 32) | qperm<CTRL>((uint32_t)v);
}

// per-lane constants: row p of M4 as seen from the lane's neighbours (M4[p][p], M4[p][p ^ 1],
// M4[p][p ^ 3]; M4[p][p ^ 2] = 1 for every p), and 2^sh of the lane's three elements
struct Consts {
    uint32_t c0, c1, c3;
    uint32_t d[3];
    bool lead;  // the quad's lane 0 (element 0 takes the partial S-box)
};

__device__ __forceinline__ Consts consts(uint32_t p) {
    Consts k;
    const bool odd = p & 1;
    k.c0 = odd ? 6 : 5;
    k.c1 = odd ? 4 : 7;
    k.c3 = odd ? 1 : 3;
    // sh = [4,14,11,8, 0,5,2,9, 13,6,3,12] (state_generic_impl.rs:71-84), byte p of block b
    constexpr uint32_t SHB[3] = {4u | 14u << 8 | 11u << 16 | 8u << 24, 0u | 5u << 8 | 2u << 16 | 9u << 24,
                                 13u | 6u << 8 | 3u << 16 | 12u << 24};
#pragma unroll
    for (int b = 0; b < 3; b++) k.d[b] = 1u << ((SHB[b] >> (8 * p)) & 0xFF);
    k.lead = p == 0;
    return k;
}

// x^7 for the lane's three elements
__device__ __forceinline__ void sbox_x3(uint32_t* lo, uint32_t* hi) {
    uint32_t a0[3], a1[3], e0[3], e1[3], i0[3], i1[3];
    glasm::mul_x3(lo[0], hi[0], lo[0], hi[0], a0[0], a1[0], lo[1], hi[1], lo[1], hi[1], a0[1], a1[1],
                  lo[2], hi[2], lo[2], hi[2], a0[2], a1[2]);
    glasm::mul_x3(a0[0], a1[0], lo[0], hi[0], e0[0], e1[0], a0[1], a1[1], lo[1], hi[1], e0[1], e1[1],
                  a0[2], a1[2], lo[2], hi[2], e0[2], e1[2]);
    glasm::mul_x3(a0[0], a1[0], a0[0], a1[0], i0[0], i1[0], a0[1], a1[1], a0[1], a1[1], i0[1], i1[1],
                  a0[2], a1[2], a0[2], a1[2], i0[2], i1[2]);
    glasm::mul_x3(e0[0], e1[0], i0[0], i1[0], lo[0], hi[0], e0[1], e1[1], i0[1], i1[1], lo[1], hi[1],
                  e0[2], e1[2], i0[2], i1[2], lo[2], hi[2]);
}

// external MDS of one limb (v = the lane's three 32-bit limbs) into 64-bit limb sums X (< 2^38)
__device__ __forceinline__ void mds_limb(const uint32_t* v, uint64_t* X, const Consts& k) {
    uint64_t m[3];
#pragma unroll
    for (int b = 0; b < 3; b++) {
        const uint32_t a = v[b];
        const uint32_t n1 = qperm<QP_X1>(a), n2 = qperm<QP_X2>(a), n3 = qperm<QP_X3>(a);
        m[b] = (uint64_t)a * k.c0 + (uint64_t)n1 * k.c1 + (uint64_t)n3 * k.c3 + n2;
    }
    const uint64_t s = m[0] + m[1] + m[2];
#pragma unroll
    for (int b = 0; b < 3; b++) X[b] = s + m[b];
}

__device__ __forceinline__ void reduce3(const uint64_t* L, const uint64_t* H, uint32_t* lo, uint32_t* hi) {
    uint64_t z[3];
    glasm::reduce_x3(L[0], (uint32_t)H[0], (uint32_t)(H[0] >> 32), z[0], L[1], (uint32_t)H[1], (uint32_t)(H[1] >> 32),
                     z[1], L[2], (uint32_t)H[2], (uint32_t)(H[2] >> 32), z[2]);
#pragma unroll
    for (int b = 0; b < 3; b++) {
        lo[b] = (uint32_t)z[b];
        hi[b] = (uint32_t)(z[b] >> 32);
    }
}

// full round: pending limbs (L, H) + RC, reduce, S-boxes, external MDS into new limbs.
// rc: the lane's three round constants of this round
__device__ __forceinline__ void full_round(uint32_t* lo, uint32_t* hi, uint64_t* L, uint64_t* H, const uint64_t* rc,
                                           const Consts& k) {
#pragma unroll
    for (int b = 0; b < 3; b++) {
        L[b] += (uint32_t)rc[b];
        H[b] += rc[b] >> 32;
    }
    reduce3(L, H, lo, hi);
    sbox_x3(lo, hi);
    mds_limb(lo, L, k);
    mds_limb(hi, H, k);
}

// partial round r on the reduced state
__device__ __forceinline__ void partial_round(uint32_t* lo, uint32_t* hi, int r, const Consts& k) {
    // element 0: + RC[r][0], x^7 (every lane computes it on its block-0 element; lane 0 keeps it)
    const uint64_t L0 = p2::add_lo_u64(lo[0], p2::RCL.lo[r][0]);
    const uint64_t H0 = p2::add_lo_u64(hi[0], p2::RCL.hi[r][0]);
    uint64_t y;
    glasm::reduce_x1(L0, (uint32_t)H0, (uint32_t)(H0 >> 32), y);
    uint32_t tl = (uint32_t)y, th = (uint32_t)(y >> 32);
    p2::sbox_x1(tl, th);
    lo[0] = k.lead ? tl : lo[0];
    hi[0] = k.lead ? th : hi[0];
    // M_I: y_e = 2^sh_e x_e + sum of all twelve
    uint64_t SL = (uint64_t)lo[0] + lo[1] + lo[2];
    uint64_t SH = (uint64_t)hi[0] + hi[1] + hi[2];
    SL += qperm64<QP_X1>(SL);
    SH += qperm64<QP_X1>(SH);
    SL += qperm64<QP_X2>(SL);
    SH += qperm64<QP_X2>(SH);
    uint64_t L[3], H[3];
#pragma unroll
    for (int b = 0; b < 3; b++) {
        L[b] = (uint64_t)lo[b] * k.d[b] + SL;
        H[b] = (uint64_t)hi[b] * k.d[b] + SH;
    }
    reduce3(L, H, lo, hi);
}

// The permutation (state_generic_impl.rs:221-236) on the quad's state; rcf[8][12]: the round
// constants of the 8 full rounds (rows 0..3, 26..29) in LDS.
__device__ __forceinline__ void permute(uint32_t* lo, uint32_t* hi, const uint64_t* rcf, uint32_t p, const Consts& k) {
    uint64_t L[3], H[3];
    mds_limb(lo, L, k);
    mds_limb(hi, H, k);
#pragma unroll 1
    for (int r = 0; r < 8; r++) {
        if (r == 4) {
            reduce3(L, H, lo, hi);
#pragma unroll 1
            for (int q = 4; q < 26; q++) partial_round(lo, hi, q, k);
#pragma unroll
            for (int b = 0; b < 3; b++) {
                L[b] = lo[b];
                H[b] = hi[b];
            }
        }
        uint64_t rc[3];
#pragma unroll
        for (int b = 0; b < 3; b++) rc[b] = rcf[12 * r + p + 4 * b];
        full_round(lo, hi, L, H, rc, k);
    }
    reduce3(L, H, lo, hi);
}

}  // namespace p2q
