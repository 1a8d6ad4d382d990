// Poseidon2 leaf / node hashing kernels (gfx950).
//
// Leaf: MerkleTreeWithCap::construct (cs/oracle/merkle_tree.rs:78-172) hashes, for each
// flat leaf index L = coset * n + row, the elements src[0][L], ..., src[C-1][L] with the
// Overwrite sponge (algebraic_props/sponge.rs:224-323): every 8 elements overwrite
// state[0..8] and permute; a partial last group is zero-padded to 8 and permuted; the
// digest is state[0..4].  One leaf per lane, state in VGPRs; lanes read consecutive L
// of one column at a time, so each wave load is 512 contiguous bytes.
//
// Node: hash_into_node (cs/oracle/mod.rs:162-168) = permute([l, r, 0,0,0,0])[0..4], one
// node per lane, level by level (continue_from_leaf_hashes, merkle_tree.rs:388-449);
// the last levels (<= 256 nodes) run in one workgroup through LDS.
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "poseidon2.hpp"
#include "poseidon2_quad.hpp"
#include "bj_internal.hpp"

namespace bj {

constexpr int LEAF_THREADS = 256;

// Store the first `n` state words canonicalised (to_reduced_u64, goldilocks/mod.rs:146-153).
__device__ __forceinline__ void store_canon4(const p2::State& s, uint64_t* o) {
    uint32_t z0[4], z1[4];
    glasm::canon_x4(s.lo[0], s.hi[0], z0[0], z1[0], s.lo[1], s.hi[1], z0[1], z1[1],
                    s.lo[2], s.hi[2], z0[2], z1[2], s.lo[3], s.hi[3], z0[3], z1[3]);
#pragma unroll
    for (int i = 0; i < 4; i++) o[i] = ((uint64_t)z1[i] << 32) | z0[i];
}

__device__ __forceinline__ void store_canon4_at(const p2::State& s, int q, uint64_t* o) {
    const int b = 4 * q;
    uint32_t z0[4], z1[4];
    glasm::canon_x4(s.lo[b], s.hi[b], z0[0], z1[0], s.lo[b + 1], s.hi[b + 1], z0[1], z1[1],
                    s.lo[b + 2], s.hi[b + 2], z0[2], z1[2], s.lo[b + 3], s.hi[b + 3], z0[3], z1[3]);
#pragma unroll
    for (int i = 0; i < 4; i++) o[i] = ((uint64_t)z1[i] << 32) | z0[i];
}

__device__ __forceinline__ void load8(p2::State& s, const uint64_t* q, size_t stride, uint32_t count) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t v = (uint32_t)i < count ? q[(size_t)i * stride] : 0;
        s.lo[i] = (uint32_t)v;
        s.hi[i] = (uint32_t)(v >> 32);
    }
}

// HAS_IN: the sponge continues from carried capacity words cap_in[L][0..4] = state[8..12]
// (the Overwrite sponge's rate words are overwritten by the next absorption, so the
// capacity is the whole carried state between 8-element groups).  FINAL: write the digest
// state[0..4]; otherwise write the capacity state[8..12] for the next column range.
// REM: n_cols is not a multiple of 8 (a zero-padded last group); without it the kernel carries no
// code, registers or branches for that case (C3's 256 columns, every 8-column chunk of the
// collective's pipeline), and a FINAL absorption's last permutation is always the digest form.
template <bool HAS_IN, bool FINAL, bool REM>
__device__ __forceinline__ void leaf_hash_body(const uint64_t* __restrict__ src, size_t col_stride, uint32_t n_cols,
                                               size_t n_leaves, const uint64_t* cap_in, uint64_t* out) {
    const size_t L = blockIdx.x * (size_t)LEAF_THREADS + threadIdx.x;
    if (L >= n_leaves) return;
    const uint64_t* p = src + L;
    p2::State s;
#pragma unroll
    for (int i = 0; i < 12; i++) s.lo[i] = s.hi[i] = 0;
    if (HAS_IN) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint64_t v = cap_in[4 * L + i];
            s.lo[8 + i] = (uint32_t)v;
            s.hi[8 + i] = (uint32_t)(v >> 32);
        }
    }
    const uint32_t full = n_cols >> 3;
    const uint32_t rem = REM ? n_cols & 7 : 0;
    // software prefetch: the next group's 8 loads are issued before this group's permute
    uint64_t nxt[8];
    if (full > 0) {
#pragma unroll
        for (int i = 0; i < 8; i++) nxt[i] = p[(size_t)i * col_stride];
    }
    // every absorption but the leaf's last is followed by another, which overwrites words 0..7:
    // it needs the capacity words only; the last needs the digest (FINAL) or the capacity.  The
    // last full group is peeled out of the loop (no prefetch live across its permutation).
    if (full > 0) {
        for (uint32_t g = 0; g + 1 < full; g++) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                s.lo[i] = (uint32_t)nxt[i];
                s.hi[i] = (uint32_t)(nxt[i] >> 32);
            }
            const uint64_t* q = p + (size_t)(g + 1) * 8 * col_stride;
#pragma unroll
            for (int i = 0; i < 8; i++) nxt[i] = q[(size_t)i * col_stride];
            p2::permute<p2::OUT_CAP>(s);
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            s.lo[i] = (uint32_t)nxt[i];
            s.hi[i] = (uint32_t)(nxt[i] >> 32);
        }
        if (FINAL && !REM)
            p2::permute<p2::OUT_DIGEST>(s);
        else
            p2::permute<p2::OUT_CAP>(s);
    }
    if (FINAL && REM) {
        load8(s, p + (size_t)full * 8 * col_stride, col_stride, rem);
        p2::permute<p2::OUT_DIGEST>(s);
    }
    if (FINAL) store_canon4(s, out + 4 * L);
    else store_canon4_at(s, 2, out + 4 * L);
}

// Three waves per SIMD (<= 168 VGPRs) is what keeps the permutation at its issue rate.  Without
// the ragged-group code (REM) every instantiation fits in 131-141 VGPRs on its own; a forced
// amdgpu_waves_per_eu(3, 3) made the compiler serialise each full round's two constant loads
// (one SGPR window for both), 0.4% of the leaves.
template <bool HAS_IN, bool FINAL, bool REM>
__global__ __launch_bounds__(LEAF_THREADS) void leaf_hash_kernel(const uint64_t* __restrict__ src,
                                                                 size_t col_stride, uint32_t n_cols,
                                                                 size_t n_leaves, const uint64_t* cap_in,
                                                                 uint64_t* out) {
    leaf_hash_body<HAS_IN, FINAL, REM>(src, col_stride, n_cols, n_leaves, cap_in, out);
}

// Leaf hashing of MerkleTreeWithCap::construct_by_chunking (merkle_tree.rs:176-306) and
// construct_by_chunking_from_flat_sources (:308-386): leaf L absorbs, for each source column
// c in order, the E = 2^log_e consecutive elements src[c][L*E .. (L+1)*E).  Used by the FRI
// oracles (fri/mod.rs:179-187, 258-266: c0 and c1 of the Ext2 codeword, E = 2^r).  One leaf
// per lane; element k of the leaf's sequence is (c = k >> log_e, t = k & (E-1)).
__global__ __launch_bounds__(LEAF_THREADS) void leaf_chunk_kernel(const uint64_t* __restrict__ src,
                                                                  size_t col_stride, uint32_t n_cols,
                                                                  uint32_t log_e, size_t n_leaves,
                                                                  uint64_t* __restrict__ out) {
    const size_t L = blockIdx.x * (size_t)LEAF_THREADS + threadIdx.x;
    if (L >= n_leaves) return;
    const uint32_t E = 1u << log_e;
    const uint64_t* p = src + (L << log_e);
    p2::State s;
#pragma unroll
    for (int i = 0; i < 12; i++) s.lo[i] = s.hi[i] = 0;
    const uint32_t total = n_cols << log_e;
    // every group but the last is followed by another (capacity words only); the last, full or
    // zero-padded, gives the digest
    uint32_t k = 0;
    for (; k + 8 < total; k += 8) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t e = k + i;
            const uint64_t v = p[(size_t)(e >> log_e) * col_stride + (e & (E - 1))];
            s.lo[i] = (uint32_t)v;
            s.hi[i] = (uint32_t)(v >> 32);
        }
        p2::permute<p2::OUT_CAP>(s);
    }
    if (k < total) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t e = k + i;
            const uint64_t v = e < total ? p[(size_t)(e >> log_e) * col_stride + (e & (E - 1))] : 0;
            s.lo[i] = (uint32_t)v;
            s.hi[i] = (uint32_t)(v >> 32);
        }
        p2::permute<p2::OUT_DIGEST>(s);
    }
    store_canon4(s, out + 4 * L);
}

__device__ __forceinline__ void node_hash(const uint64_t* l, const uint64_t* r, uint64_t* o) {
    p2::State s;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        s.lo[i] = (uint32_t)l[i];
        s.hi[i] = (uint32_t)(l[i] >> 32);
        s.lo[4 + i] = (uint32_t)r[i];
        s.hi[4 + i] = (uint32_t)(r[i] >> 32);
        s.lo[8 + i] = s.hi[8 + i] = 0;
    }
    p2::permute<p2::OUT_DIGEST>(s);
    store_canon4(s, o);
}

__global__ __launch_bounds__(256) void node_level_kernel(const uint64_t* __restrict__ prev,
                                                         uint64_t* __restrict__ next, size_t m) {
    const size_t i = blockIdx.x * (size_t)256 + threadIdx.x;
    if (i >= m) return;
    uint64_t lr[8];
#pragma unroll
    for (int k = 0; k < 8; k++) lr[k] = prev[8 * i + k];
    node_hash(lr, lr + 4, next + 4 * i);
}

// One node per quad of lanes (poseidon2_quad.hpp): for the levels too small to fill the chip,
// where a level costs one permutation's latency and the quad form shortens it ~2.5x.
__global__ __launch_bounds__(256) void node_level_q4_kernel(const uint64_t* __restrict__ prev,
                                                            uint64_t* __restrict__ next, size_t m) {
    // round constants of the 8 full rounds (rows 0..3, 26..29), each lane reads its own three
    __shared__ uint64_t rcf[8 * 12];
    const uint32_t t = threadIdx.x;
    if (t < 8 * 12) {
        const uint32_t r = t / 12, e = t % 12, row = r < 4 ? r : r + 22;
        rcf[t] = p2::RCL.lo[row][e] | (p2::RCL.hi[row][e] << 32);
    }
    __syncthreads();
    const size_t i = (blockIdx.x * (size_t)256 + t) >> 2;
    const uint32_t p = t & 3;
    if (i >= m) return;  // whole quads: 4 m lanes
    const p2q::Consts k = p2q::consts(p);
    const uint64_t l = prev[8 * i + p], r = prev[8 * i + 4 + p];
    uint32_t lo[3] = {(uint32_t)l, (uint32_t)r, 0}, hi[3] = {(uint32_t)(l >> 32), (uint32_t)(r >> 32), 0};
    p2q::permute(lo, hi, rcf, p, k);
    uint32_t z0, z1;
    glasm::canon_x1(lo[0], hi[0], z0, z1);
    next[4 * i + p] = ((uint64_t)z1 << 32) | z0;
}

// Levels of at most 2^15 nodes (below one wave per SIMD), several per launch (round 6): block w
// takes the 2^b consecutive digests [w 2^b, (w + 1) 2^b) of the level below and runs `lv`
// levels over them, one node per quad of lanes (p2q::permute), the digests between levels in
// LDS.  Every level's nodes are stored where per-level launches would put them (levels
// concatenated upward from `out`, node_hashes_enumerated_from_leafs; merkle_tree.rs:388-449),
// so a block's subtree is the reference's.  One launch replaces lv per-level grids of ~17 us
// each; the levels inside still run one permutation latency apart (a block barrier between).
constexpr uint32_t NODE_FUSED_THREADS = 512;  // 128 quads: level 1 of a 2^8-digest block in one pass
constexpr uint32_t NODE_FUSED_LOG_DIGESTS = 8;
__global__ __launch_bounds__(NODE_FUSED_THREADS) void node_levels_q4_kernel(const uint64_t* __restrict__ prev,
                                                                           uint64_t* __restrict__ out, size_t len,
                                                                           uint32_t b, uint32_t lv) {
    __shared__ uint64_t rcf[8 * 12];
    __shared__ uint64_t buf[2][(NODE_FUSED_THREADS / 4) * 4];
    const uint32_t t = threadIdx.x;
    if (t < 8 * 12) {
        const uint32_t r = t / 12, e = t % 12, row = r < 4 ? r : r + 22;
        rcf[t] = p2::RCL.lo[row][e] | (p2::RCL.hi[row][e] << 32);
    }
    __syncthreads();
    const uint32_t q = t >> 2, p = t & 3;
    const p2q::Consts k = p2q::consts(p);
    size_t base = 0, level_len = len >> 1;  // level j: level_len nodes from out + 4 base
    uint32_t nodes = 1u << (b - 1);         // this block's nodes of level j
    for (uint32_t j = 0; j < lv; j++) {
        if (q < nodes) {  // whole quads (and whole waves once nodes >= 16)
            uint64_t l, r;
            if (j == 0) {
                const size_t i = (size_t)blockIdx.x * nodes + q;
                l = prev[8 * i + p];
                r = prev[8 * i + 4 + p];
            } else {
                l = buf[(j - 1) & 1][8 * q + p];
                r = buf[(j - 1) & 1][8 * q + 4 + p];
            }
            uint32_t lo[3] = {(uint32_t)l, (uint32_t)r, 0}, hi[3] = {(uint32_t)(l >> 32), (uint32_t)(r >> 32), 0};
            p2q::permute(lo, hi, rcf, p, k);
            uint32_t z0, z1;
            glasm::canon_x1(lo[0], hi[0], z0, z1);
            const uint64_t z = ((uint64_t)z1 << 32) | z0;
            out[4 * (base + (size_t)blockIdx.x * nodes + q) + p] = z;
            buf[j & 1][4 * q + p] = z;
        }
        __syncthreads();
        base += level_len;
        level_len >>= 1;
        nodes >>= 1;
    }
}

// Remaining levels from `len` digests (len <= 4096; launch_nodes hands over len <= 512) down to
// cap_size, one workgroup.
__global__ __launch_bounds__(256) void node_tail_kernel(const uint64_t* __restrict__ prev, uint64_t* next,
                                                        uint32_t len, uint32_t cap_size) {
    __shared__ uint64_t buf[2][2048 * 4];
    int cur = 0;
    uint64_t* outp = next;
    uint32_t m = len / 2;
    for (uint32_t i = threadIdx.x; i < m; i += 256) {
        uint64_t lr[8];
        for (int k = 0; k < 8; k++) lr[k] = prev[8 * (size_t)i + k];
        uint64_t o[4];
        node_hash(lr, lr + 4, o);
        for (int k = 0; k < 4; k++) { buf[cur][4 * i + k] = o[k]; outp[4 * (size_t)i + k] = o[k]; }
    }
    outp += 4 * (size_t)m;
    __syncthreads();
    while (m > cap_size) {
        uint32_t m2 = m / 2;
        for (uint32_t i = threadIdx.x; i < m2; i += 256) {
            uint64_t o[4];
            node_hash(&buf[cur][8 * i], &buf[cur][8 * i + 4], o);
            for (int k = 0; k < 4; k++) { buf[cur ^ 1][4 * i + k] = o[k]; outp[4 * (size_t)i + k] = o[k]; }
        }
        outp += 4 * (size_t)m2;
        cur ^= 1;
        m = m2;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void permute_kernel(uint64_t* states, size_t count) {
    const size_t i = blockIdx.x * (size_t)256 + threadIdx.x;
    if (i >= count) return;
    p2::State s;
#pragma unroll
    for (int k = 0; k < 12; k++) {
        uint64_t v = states[12 * i + k];
        s.lo[k] = (uint32_t)v;
        s.hi[k] = (uint32_t)(v >> 32);
    }
    p2::permute(s);
#pragma unroll
    for (int q = 0; q < 3; q++) store_canon4_at(s, q, states + 12 * i + 4 * q);
}

hipError_t launch_leaves(const uint64_t* src, size_t col_stride, uint32_t n_cols, size_t n_leaves, uint64_t* out,
                         hipStream_t st) {
    return launch_leaves_partial(src, col_stride, n_cols, n_leaves, nullptr, out, true, st);
}

hipError_t launch_leaves_partial(const uint64_t* src, size_t col_stride, uint32_t n_cols, size_t n_leaves,
                                 const uint64_t* cap_in, uint64_t* out, bool final_, hipStream_t st) {
    if (n_leaves == 0) return hipSuccess;
    const dim3 g((unsigned)((n_leaves + LEAF_THREADS - 1) / LEAF_THREADS));
#define BJ_LEAF(IN, FIN, REM) \
    hipLaunchKernelGGL((leaf_hash_kernel<IN, FIN, REM>), g, dim3(LEAF_THREADS), 0, st, src, col_stride, n_cols, \
                       n_leaves, cap_in, out)
#define BJ_LEAF_R(IN, FIN) \
    do {                     \
        if (n_cols & 7)      \
            BJ_LEAF(IN, FIN, true); \
        else                 \
            BJ_LEAF(IN, FIN, false); \
    } while (0)
    if (cap_in) {
        if (final_) BJ_LEAF_R(true, true);
        else BJ_LEAF_R(true, false);
    } else {
        if (final_) BJ_LEAF_R(false, true);
        else BJ_LEAF_R(false, false);
    }
#undef BJ_LEAF_R
#undef BJ_LEAF
    return hipGetLastError();
}

hipError_t launch_leaves_chunked(const uint64_t* src, size_t col_stride, uint32_t n_cols, uint32_t log_e,
                                 size_t n_leaves, uint64_t* out, hipStream_t st) {
    if (n_leaves == 0) return hipSuccess;
    hipLaunchKernelGGL(leaf_chunk_kernel, dim3((unsigned)((n_leaves + LEAF_THREADS - 1) / LEAF_THREADS)),
                       dim3(LEAF_THREADS), 0, st, src, col_stride, n_cols, log_e, n_leaves, out);
    return hipGetLastError();
}

static size_t node_q4_max() { return (size_t)knobs().node_q4_max; }

hipError_t launch_nodes(const uint64_t* leaves, size_t n_leaves, uint32_t cap_size, uint64_t* nodes,
                        hipStream_t st) {
    const uint64_t* prev = leaves;
    uint64_t* out = nodes;
    size_t len = n_leaves;
    // every level above 512 digests as its own grid: a level costs one permutation's latency
    // (~20 us at one wave per SIMD) when every lane hashes one node, while one workgroup
    // would run a 2048-node level as 8 permutations in sequence.  Levels of <= q4max nodes
    // (default 2^15: below one wave per SIMD) hash one node per quad of lanes, each level its
    // own grid down to the cap; BJ_NODE_Q4_MAX=0 keeps one node per lane and the one-workgroup
    // tail for the last levels.
    const size_t q4max = node_q4_max();
    const auto pow2 = [](size_t x) { return x && !(x & (x - 1)); };
    const bool fuse = knobs().node_fused && pow2(n_leaves) && pow2(cap_size);
    while (len > cap_size && (q4max || len > 512)) {
        size_t m = len / 2;
        if (m <= q4max && fuse) {
            // up to 8 levels per launch (node_levels_q4_kernel): blocks of 2^b digests
            uint32_t L = 0, C = 0;
            while (((size_t)1 << L) < len) L++;
            while (((size_t)1 << C) < cap_size) C++;
            const uint32_t b = std::min(NODE_FUSED_LOG_DIGESTS, L), lv = std::min(b, L - C);
            hipLaunchKernelGGL(node_levels_q4_kernel, dim3((unsigned)(len >> b)), dim3(NODE_FUSED_THREADS), 0, st,
                               prev, out, len, b, lv);
            prev = out + 4 * (len - (len >> (lv - 1)));
            out += 4 * (len - (len >> lv));
            len >>= lv;
            continue;
        }
        if (m <= q4max)
            hipLaunchKernelGGL(node_level_q4_kernel, dim3((unsigned)((m + 63) / 64)), dim3(256), 0, st, prev, out, m);
        else
            hipLaunchKernelGGL(node_level_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, prev, out, m);
        prev = out;
        out += 4 * m;
        len = m;
    }
    if (len > cap_size) {
        hipLaunchKernelGGL(node_tail_kernel, dim3(1), dim3(256), 0, st, prev, out, (uint32_t)len, cap_size);
    }
    return hipGetLastError();
}

hipError_t launch_permute(uint64_t* states, size_t count, hipStream_t st) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(permute_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, states, count);
    return hipGetLastError();
}

}  // namespace bj
