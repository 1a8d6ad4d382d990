// Poseidon2 over Goldilocks, width 12 / rate 8 / capacity 4, for gfx950 device code.
//
// Same permutation as the reference's State::poseidon2_permutation
// (implementations/poseidon2/state_generic_impl.rs:221-236):
//   external MDS; 4 full rounds (RC[r][i], x^7, external MDS); 22 partial rounds
//   (state[0] += RC[r][0], x^7 on state[0], internal M_I); 4 full rounds.
// External MDS = block-circulant(2*M4, M4, M4) (implementations/suggested_mds.rs:19-97),
// M_I = diag(2^sh) + 1 1^T with sh = [4,14,11,8,0,5,2,9,13,6,3,12]
// (state_generic_impl.rs:71-84, 166-202).  Round constants: poseidon2_rc.inc (data
// extracted by tools/gen_poseidon2_constants.py from poseidon_goldilocks_params.rs).
//
// gfx950 formulation (same field values; every result is compared canonically):
// * state element = (lo, hi) 32-bit halves of a u64 representative, one permutation per lane;
// * linear layers run on "limbs": L = sum c_j lo_j and H = sum c_j hi_j in 64-bit lanes,
//   so a linear combination never carries (coefficients here stay < 2^16), and one
//   4-instruction reduction (glasm::reduce_xN) turns (L, H) back into a u64 per element;
// * a full round's constant is one 64-bit add into L (the reduction takes any L < 2^64 - 2^40
//   plus H < 2^40); a partial round's constant costs nothing or one add per limb (Sched);
// * S-box multiplies are the interleaved inline-asm products of gl_asm.hpp.
#pragma once
#include "gl.hpp"
#include "gl_asm.hpp"

namespace p2 {

// Round constants split into 64-bit (value, 0) pairs so a scalar load yields an SGPR pair
// that v_lshl_add_u64 adds to a limb directly (the quad-lane node form, poseidon2_quad.hpp).
struct RcLimbs {
    uint64_t lo[30][12];
    uint64_t hi[30][12];
};

constexpr uint64_t RC_FLAT[30][12] = {
#include "poseidon2_rc.inc"
};

constexpr RcLimbs make_rc_limbs() {
    RcLimbs r{};
    for (int i = 0; i < 30; i++)
        for (int j = 0; j < 12; j++) {
            r.lo[i][j] = RC_FLAT[i][j] & 0xFFFFFFFFull;
            r.hi[i][j] = RC_FLAT[i][j] >> 32;
        }
    return r;
}

__device__ __constant__ static const RcLimbs RCL = make_rc_limbs();

// ---- The constant schedule (field values; every entry canonical, computed at compile time) ----
//
// The reference adds RC_r before round r's S-boxes (state_generic_impl.rs:131-138, 55-64).
// * Full rounds: the limbs after an external MDS are L, H < 2^39; L + RC_r stays below
//   2^64 - 2^40 for every full-round constant (checked below), where the reduction is still
//   exact (reduce_stream: W = Hhi EPS + L < 2^64), so RC_r is one 64-bit add into L instead of
//   a 32-bit limb add into each of L and H.
// * Partial rounds run in pairs (partial_round_pair).  The first M_I of a pair adds a constant
//   K to every element (its first limb-sum chain starts at K instead of 0, so K is free) and
//   the second adds D to element 0 only (one add per limb).  The state then differs from the
//   reference's by an offset vector f known at compile time; K and D are chosen so that f_0 is
//   exactly the next partial round's constant whenever element 0 enters its S-box, and the
//   first full round after the partial rounds adds RC_26 - f (rc26) instead of RC_26.
//   RC_4 (the first partial constant) is added to element 0 before the reduction that ends the
//   first full rounds.
// tests/test_poseidon2_sched.py restates this derivation and checks it against the reference's
// known answers.
namespace sched {
constexpr uint64_t P = 0xFFFFFFFF00000001ull;
constexpr uint64_t addm(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a + b) % P); }
constexpr uint64_t subm(uint64_t a, uint64_t b) { return addm(a, P - b % P); }
constexpr uint64_t mulm(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) % P); }
constexpr int SH[12] = {4, 14, 11, 8, 0, 5, 2, 9, 13, 6, 3, 12};
// A 64-bit constant added into L: L < 2^39 after an external MDS, so L + c < 2^64 - 2^40
// whenever c < 2^64 - 2^41.
constexpr uint64_t FULL_RC_BOUND = ~0ull - (1ull << 41) + 1;
// After the last partial round L < 2^60.1 and H < 2^61.1 (mi_layer_b_limbs on mi_layer_a_g's limbs,
// tests/test_poseidon2_sched.py::test_partial_pair_limb_bounds), so W = Hhi EPS + L + c < 2^64
// whenever c < 2^64 - 2^62; larger entries of rc26 go in as 32-bit limbs.
constexpr uint64_t LIMB_RC_BOUND = (1ull << 63) + (1ull << 62);
struct Values {
    uint64_t k[11];     // per partial pair: first M_I's constant (every element)
    uint64_t d[10];     // per partial pair but the last: second M_I's constant (element 0)
    uint64_t rc26[12];  // RC_26 - f
};
constexpr Values derive() {
    Values v{};
    // the offset f of the state against the reference's, entering each pair: f_0 = rc_r
    uint64_t f[12] = {RC_FLAT[4][0]};
    for (int q = 0; q < 11; q++) {
        const int r = 4 + 2 * q;
        uint64_t s = 0;  // element 0 leaves its S-box exact: offset only on 1..11
        for (int i = 1; i < 12; i++) s = addm(s, f[i]);
        v.k[q] = subm(RC_FLAT[r + 1][0], s);
        f[0] = 0;
        for (int i = 0; i < 12; i++) f[i] = addm(addm(mulm(f[i], 1ull << SH[i]), s), v.k[q]);
        s = 0;
        for (int i = 1; i < 12; i++) s = addm(s, f[i]);
        f[0] = 0;
        for (int i = 0; i < 12; i++) f[i] = addm(mulm(f[i], 1ull << SH[i]), s);
        if (q < 10) {
            v.d[q] = subm(RC_FLAT[r + 2][0], f[0]);
            f[0] = RC_FLAT[r + 2][0];
        }
    }
    for (int i = 0; i < 12; i++) v.rc26[i] = subm(RC_FLAT[26][i], f[i]);
    return v;
}
constexpr Values V = derive();
constexpr bool full_rcs_fit() {
    for (int r : {0, 1, 2, 3, 27, 28, 29})
        for (int i = 0; i < 12; i++)
            if (RC_FLAT[r][i] >= FULL_RC_BOUND) return false;
    return RC_FLAT[4][0] < FULL_RC_BOUND;
}
static_assert(full_rcs_fit(), "a full-round constant is too large for the one-add form");
}  // namespace sched

// The schedule's device tables: full words, and (value, 0) limb pairs for the asm layers.
struct Sched {
    // RC_FLAT as 64-bit words (full rounds, RC_4[0]), elements 0..7 and 8..11 in tables of their
    // own: one 64-byte and one 32-byte scalar load per round, each from its own base, so both are
    // in flight together (one table of 12 had the second load's address formed after the first
    // load's wait)
    uint64_t rcw8[30][8];
    uint64_t rcw4[30][4];
    uint64_t k_lo[11], k_hi[11];
    uint64_t d_lo[10], d_hi[10];
    uint64_t rc26_w[12], rc26_lo[12], rc26_hi[12];
};
constexpr Sched make_sched() {
    Sched s{};
    for (int r = 0; r < 30; r++)
        for (int i = 0; i < 12; i++) (i < 8 ? s.rcw8[r][i] : s.rcw4[r][i - 8]) = RC_FLAT[r][i];
    for (int q = 0; q < 11; q++) { s.k_lo[q] = sched::V.k[q] & 0xFFFFFFFFull; s.k_hi[q] = sched::V.k[q] >> 32; }
    for (int q = 0; q < 10; q++) { s.d_lo[q] = sched::V.d[q] & 0xFFFFFFFFull; s.d_hi[q] = sched::V.d[q] >> 32; }
    for (int i = 0; i < 12; i++) {
        s.rc26_w[i] = sched::V.rc26[i];
        s.rc26_lo[i] = sched::V.rc26[i] & 0xFFFFFFFFull;
        s.rc26_hi[i] = sched::V.rc26[i] >> 32;
    }
    return s;
}
__device__ __constant__ static const Sched SCH = make_sched();

struct State {
    uint32_t lo[12], hi[12];
};

// x^7 for 4 independent elements: x2 = x^2; x3 = x2*x, x4 = x2^2; x7 = x3*x4.
__device__ __forceinline__ void sbox_x4(uint32_t* lo, uint32_t* hi) {
    uint32_t a0, a1, b0, b1, c0, c1, d0, d1;  // x2 of the four
    glasm::mul_x4(lo[0], hi[0], lo[0], hi[0], a0, a1, lo[1], hi[1], lo[1], hi[1], b0, b1,
                  lo[2], hi[2], lo[2], hi[2], c0, c1, lo[3], hi[3], lo[3], hi[3], d0, d1);
    uint32_t e0, e1, f0, f1, g0, g1, h0, h1;  // x3 of the four
    glasm::mul_x4(a0, a1, lo[0], hi[0], e0, e1, b0, b1, lo[1], hi[1], f0, f1,
                  c0, c1, lo[2], hi[2], g0, g1, d0, d1, lo[3], hi[3], h0, h1);
    uint32_t i0, i1, j0, j1, k0, k1, l0, l1;  // x4 of the four
    glasm::mul_x4(a0, a1, a0, a1, i0, i1, b0, b1, b0, b1, j0, j1,
                  c0, c1, c0, c1, k0, k1, d0, d1, d0, d1, l0, l1);
    glasm::mul_x4(e0, e1, i0, i1, lo[0], hi[0], f0, f1, j0, j1, lo[1], hi[1],
                  g0, g1, k0, k1, lo[2], hi[2], h0, h1, l0, l1, lo[3], hi[3]);
}

__device__ __forceinline__ void sbox_x1(uint32_t& lo, uint32_t& hi) {
    uint32_t a0, a1, e0, e1, i0, i1;
    glasm::mul_x1(lo, hi, lo, hi, a0, a1);
    glasm::mul_x2(a0, a1, lo, hi, e0, e1, a0, a1, a0, a1, i0, i1);
    glasm::mul_x1(e0, e1, i0, i1, lo, hi);
}

// Limb form of the external MDS (suggested_mds_mul) applied to (lo, hi): outputs L[i], H[i]
// with L, H < 64 * 2^32.
__device__ __forceinline__ void m4_limbs(uint64_t& x0, uint64_t& x1, uint64_t& x2, uint64_t& x3) {
    uint64_t t0 = x0 + x1;
    uint64_t t1 = x2 + x3;
    uint64_t t2 = (x1 << 1) + t1;
    uint64_t t3 = (x3 << 1) + t0;
    uint64_t t4 = (t1 << 2) + t3;
    uint64_t t5 = (t0 << 2) + t2;
    uint64_t t6 = t3 + t5;
    uint64_t t7 = t2 + t4;
    x0 = t6; x1 = t5; x2 = t7; x3 = t4;
}

// lo + b as a 64-bit limb in one v_mad_u64_u32 (lo * 1 + b): no zero-extended register pair
// for lo.  b is wave-uniform (a round-constant limb in an SGPR pair).
__device__ __forceinline__ uint64_t add_lo_u64(uint32_t lo, uint64_t b) {
    uint64_t r;
    asm volatile("v_mad_u64_u32 %0, vcc, %1, 1, %2" : "=v"(r) : "v"(lo), "s"(b) : "vcc");
    return r;
}

// Which outputs of a permutation its caller reads: all 12 (bj_poseidon2_permute), the capacity
// words 8..11 (a sponge absorption followed by another: the Overwrite sponge replaces words 0..7,
// sponge.rs:241-323), or the digest words 0..3 (the last absorption of a leaf, a node).  The
// last round's external MDS and the final reduction then form only those outputs.
enum Out { OUT_ALL = 0, OUT_CAP = 1, OUT_DIGEST = 2 };

template <int OUT = OUT_ALL>
__device__ __forceinline__ void mds_ext_limbs(const uint32_t* v, uint64_t* X) {
#pragma unroll
    for (int i = 0; i < 12; i++) X[i] = v[i];
    m4_limbs(X[0], X[1], X[2], X[3]);
    m4_limbs(X[4], X[5], X[6], X[7]);
    m4_limbs(X[8], X[9], X[10], X[11]);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint64_t a = X[i], b = X[i + 4], c = X[i + 8];
        if constexpr (OUT == OUT_ALL) {
            uint64_t s = a + b + c;
            X[i] = s + a;
            X[i + 4] = s + b;
            X[i + 8] = s + c;
        } else if constexpr (OUT == OUT_CAP) {
            X[i + 8] = (c << 1) + a + b;
        } else {
            X[i] = (a << 1) + b + c;
        }
    }
}

__device__ __forceinline__ void split(uint64_t z, uint32_t& lo, uint32_t& hi) {
    lo = (uint32_t)z;
    hi = (uint32_t)(z >> 32);
}

// (L, H) -> reduced (lo, hi) for all 12 elements.  The reductions write 64-bit register pairs;
// lo / hi are their halves (sub-registers, no moves).
template <int OUT = OUT_ALL>
__device__ __forceinline__ void reduce12(const uint64_t* L, const uint64_t* H, uint32_t* lo, uint32_t* hi) {
#pragma unroll
    for (int q = 0; q < 3; q++) {
        if constexpr (OUT == OUT_CAP) { if (q != 2) continue; }
        if constexpr (OUT == OUT_DIGEST) { if (q != 0) continue; }
        const int i = 4 * q;
        uint64_t z[4];
        glasm::reduce_x4(L[i], (uint32_t)H[i], (uint32_t)(H[i] >> 32), z[0],
                         L[i + 1], (uint32_t)H[i + 1], (uint32_t)(H[i + 1] >> 32), z[1],
                         L[i + 2], (uint32_t)H[i + 2], (uint32_t)(H[i + 2] >> 32), z[2],
                         L[i + 3], (uint32_t)H[i + 3], (uint32_t)(H[i + 3] >> 32), z[3]);
#pragma unroll
        for (int j = 0; j < 4; j++) split(z[j], lo[i + j], hi[i + j]);
    }
}

// Full round r on the pending limbs (L, H) of the state (the external MDS of the previous
// step not yet reduced): reduce(L + RC_r, H) (Sched: one 64-bit add per element), x^7, then
// the external MDS into new pending limbs.  Leaves the reduced S-box output in s.
template <int OUT = OUT_ALL, bool RC = true>
__device__ __forceinline__ void full_round(State& s, uint64_t* L, uint64_t* H, int r) {
    if constexpr (RC) {
#pragma unroll
        for (int i = 0; i < 12; i++) L[i] += i < 8 ? SCH.rcw8[r][i] : SCH.rcw4[r][i - 8];
    }
    reduce12(L, H, s.lo, s.hi);
#pragma unroll
    for (int q = 0; q < 3; q++) sbox_x4(s.lo + 4 * q, s.hi + 4 * q);
    mds_ext_limbs<OUT>(s.lo, L);
    mds_ext_limbs<OUT>(s.hi, H);
}

// Two partial rounds (pair q: rounds 4 + 2q, 5 + 2q).  The state enters as element 0 reduced
// (z0, a 64-bit register pair already holding its round constant) and elements 1..11 either
// reduced (W[i]; pair 0, after the full rounds) or half-reduced (HALF: W[i] + G[i] 2^32, as the
// previous pair's mi_layer_b_half + eps_fold_x11 left them).  M_I of the first round leaves
// elements 1..11 as unreduced limbs (< 2^47); only s0, the next S-box input, is reduced.  The
// second M_I consumes the limbs (sums < 2^48, shifted terms < 2^61.1), reduces element 0 and
// hands elements 1..11 on half-reduced: W = Hhi EPS + L (one mad) and G = Hlo, where the full
// reduction took four instructions; the next first M_I takes G as a third limb (two mads more
// per element), so a pair costs 11 instructions fewer (glasm::mi_layer_a_g / mi_layer_b_half,
// tools/gen_gl_asm.py).  Same field values as two reduced rounds plus the schedule's offsets.
// The constants are read before the asm blocks (which the compiler does not move loads across),
// so their scalar loads land during the first S-box.
struct Partial {
    uint64_t z0;
    uint64_t W[12];  // 1..11
    uint32_t G[12];  // 1..11 (HALF)
};

template <bool HALF>
__device__ __forceinline__ void partial_first(const Partial& P, int q, uint64_t* L, uint64_t* H, uint32_t& lo0,
                                              uint32_t& hi0) {
    uint64_t z0;
    uint32_t lo[12], hi[12];
    const uint64_t kl = SCH.k_lo[q], kh = SCH.k_hi[q];
    split(P.z0, lo[0], hi[0]);
#pragma unroll
    for (int i = 1; i < 12; i++) split(P.W[i], lo[i], hi[i]);
    sbox_x1(lo[0], hi[0]);
    if constexpr (HALF) glasm::mi_layer_a_g(lo, hi, P.G, kl, kh, L, H, z0);
    else glasm::mi_layer_a(lo, hi, kl, kh, L, H, z0);
    split(z0, lo0, hi0);
    sbox_x1(lo0, hi0);
}

template <bool HALF>
__device__ __forceinline__ void partial_round_pair(Partial& P, int q) {
    uint64_t L[12], H[12], Lo[12], Ho[12];
    uint32_t lo0, hi0, hh[12];
    const uint64_t dl = SCH.d_lo[q], dh = SCH.d_hi[q];
    partial_first<HALF>(P, q, L, H, lo0, hi0);
    glasm::mi_layer_b_half(lo0, hi0, L, H, dl, dh, Lo, Ho, P.z0);
#pragma unroll
    for (int i = 1; i < 12; i++) split(Ho[i], P.G[i], hh[i]);
    glasm::eps_fold_x11(hh, Lo, P.W);
}

// The last pair (rounds 24, 25): the second M_I hands its limbs to the first full round.
__device__ __forceinline__ void partial_round_pair_last(const Partial& P, uint64_t* Lo, uint64_t* Ho) {
    uint64_t L[12], H[12];
    uint32_t lo0, hi0;
    partial_first<true>(P, 10, L, H, lo0, hi0);
    glasm::mi_layer_b_limbs(lo0, hi0, L, H, Lo, Ho);
}

// RC_26 - f into the limbs the last partial round left: one 64-bit add where the value allows
// it (sched::LIMB_RC_BOUND), else one 32-bit limb add into each of L and H.
template <int I = 0>
__device__ __forceinline__ void add_rc26(uint64_t* L, uint64_t* H) {
    if constexpr (sched::V.rc26[I] < sched::LIMB_RC_BOUND) {
        L[I] += SCH.rc26_w[I];
    } else {
        L[I] += SCH.rc26_lo[I];
        H[I] += SCH.rc26_hi[I];
    }
    if constexpr (I + 1 < 12) add_rc26<I + 1>(L, H);
}

// The permutation (state_generic_impl.rs:221-236): MDS; 4 x (RC, S-box, MDS);
// 22 partial rounds; 4 x (RC, S-box, MDS), with the round constants placed by Sched.
// OUT: the outputs the caller reads (the others are left unspecified); the last full round is
// peeled so that its MDS forms only those.
template <int OUT = OUT_ALL>
__device__ __forceinline__ void permute(State& s) {
    uint64_t L[12], H[12], Z[12];
    Partial P;
    mds_ext_limbs(s.lo, L);
    mds_ext_limbs(s.hi, H);
#pragma unroll 1
    for (int r = 0; r < 4; r++) full_round(s, L, H, r);
    L[0] += SCH.rcw8[4][0];
#pragma unroll
    for (int q = 0; q < 3; q++) {
        const int i = 4 * q;
        glasm::reduce_x4(L[i], (uint32_t)H[i], (uint32_t)(H[i] >> 32), Z[i],
                         L[i + 1], (uint32_t)H[i + 1], (uint32_t)(H[i + 1] >> 32), Z[i + 1],
                         L[i + 2], (uint32_t)H[i + 2], (uint32_t)(H[i + 2] >> 32), Z[i + 2],
                         L[i + 3], (uint32_t)H[i + 3], (uint32_t)(H[i + 3] >> 32), Z[i + 3]);
    }
    P.z0 = Z[0];
#pragma unroll
    for (int i = 1; i < 12; i++) P.W[i] = Z[i];
    partial_round_pair<false>(P, 0);
#pragma unroll 1
    for (int q = 1; q < 10; q++) partial_round_pair<true>(P, q);
    partial_round_pair_last(P, L, H);
    add_rc26(L, H);
    full_round<OUT_ALL, false>(s, L, H, 26);
#pragma unroll 1
    for (int r = 27; r < 29; r++) full_round(s, L, H, r);
    full_round<OUT>(s, L, H, 29);
    reduce12<OUT>(L, H, s.lo, s.hi);
}

__device__ __forceinline__ void permute(uint64_t v[12]) {
    State s;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        s.lo[i] = (uint32_t)v[i];
        s.hi[i] = (uint32_t)(v[i] >> 32);
    }
    permute(s);
#pragma unroll
    for (int i = 0; i < 12; i++) v[i] = ((uint64_t)s.hi[i] << 32) | s.lo[i];
}

}  // namespace p2
