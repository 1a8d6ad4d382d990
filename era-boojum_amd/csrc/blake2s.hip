// Blake2s256 tree hashing kernels (gfx950): the TreeHasher impl for blake2::Blake2s256
// (cs/oracle/mod.rs:179-245), the tree hasher of the non-recursive prover configs
// (gadgets/sha256/mod.rs:263-269).  Blake2s256 = BLAKE2s, 32-byte digest, no key (RFC 7693).
//
// Leaf (hash_into_leaf, :203-215): the message is the canonical little-endian bytes of the
// leaf's elements, 8 elements = one 64-byte block; every block but the last is compressed
// as more data follows, the last (zero-padded; one zero block for an empty leaf) carries
// the final flag and the byte count.  Node (:234-245): one block, left || right, final,
// 64 bytes.  Digests are 32 bytes, held as 4 little-endian u64 words in the same (N, 4)
// buffers as the Poseidon2 digests.
//
// One leaf per lane, as the Poseidon2 leaf kernel: lanes read consecutive L of one column,
// so each wave load is 512 contiguous bytes.  BLAKE2s is 32-bit add / xor / rotate: all
// full-rate VALU (v_add3_u32, v_xor_b32, v_alignbit_b32), about 1000 issue slots per block,
// against ~21000 for a Poseidon2 permutation absorbing the same 64 bytes, so these trees
// are bound by HBM reads rather than by VALU issue.
#include <hip/hip_runtime.h>
#include "gl.hpp"
#include "bj_internal.hpp"

namespace bj {

namespace {

constexpr int B2S_THREADS = 256;

constexpr uint32_t B2S_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                              0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};

// RFC 7693 section 2.7 message schedule
constexpr uint8_t SIGMA[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t r) { return __builtin_amdgcn_alignbit(x, x, r); }

#define B2S_G(a, b, c, d, x, y)         \
    do {                                \
        a = a + b + (x);                \
        d = rotr(d ^ a, 16);            \
        c = c + d;                      \
        b = rotr(b ^ c, 12);            \
        a = a + b + (y);                \
        d = rotr(d ^ a, 8);             \
        c = c + d;                      \
        b = rotr(b ^ c, 7);             \
    } while (0)

// RFC 7693 section 3.2 F: h <- compress(h, m, t, last)
__device__ __forceinline__ void compress(uint32_t* h, const uint32_t* m, uint32_t t_lo, uint32_t t_hi, bool last) {
    uint32_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
    uint32_t v8 = B2S_IV[0], v9 = B2S_IV[1], v10 = B2S_IV[2], v11 = B2S_IV[3];
    uint32_t v12 = B2S_IV[4] ^ t_lo, v13 = B2S_IV[5] ^ t_hi;
    uint32_t v14 = last ? ~B2S_IV[6] : B2S_IV[6], v15 = B2S_IV[7];
#pragma unroll
    for (int r = 0; r < 10; r++) {
        B2S_G(v0, v4, v8, v12, m[SIGMA[r][0]], m[SIGMA[r][1]]);
        B2S_G(v1, v5, v9, v13, m[SIGMA[r][2]], m[SIGMA[r][3]]);
        B2S_G(v2, v6, v10, v14, m[SIGMA[r][4]], m[SIGMA[r][5]]);
        B2S_G(v3, v7, v11, v15, m[SIGMA[r][6]], m[SIGMA[r][7]]);
        B2S_G(v0, v5, v10, v15, m[SIGMA[r][8]], m[SIGMA[r][9]]);
        B2S_G(v1, v6, v11, v12, m[SIGMA[r][10]], m[SIGMA[r][11]]);
        B2S_G(v2, v7, v8, v13, m[SIGMA[r][12]], m[SIGMA[r][13]]);
        B2S_G(v3, v4, v9, v14, m[SIGMA[r][14]], m[SIGMA[r][15]]);
    }
    h[0] ^= v0 ^ v8;
    h[1] ^= v1 ^ v9;
    h[2] ^= v2 ^ v10;
    h[3] ^= v3 ^ v11;
    h[4] ^= v4 ^ v12;
    h[5] ^= v5 ^ v13;
    h[6] ^= v6 ^ v14;
    h[7] ^= v7 ^ v15;
}
#undef B2S_G

__device__ __forceinline__ void init_h(uint32_t* h) {
#pragma unroll
    for (int i = 0; i < 8; i++) h[i] = B2S_IV[i];
    h[0] ^= 0x01010000u ^ 32u;  // parameter block: digest 32, no key, fanout 1, depth 1
}

// element -> two message words: as_u64_reduced().to_le_bytes() (cs/oracle/mod.rs:190-193)
__device__ __forceinline__ void put(uint32_t* m, int i, uint64_t v) {
    v = gl::canon(v);
    m[2 * i] = (uint32_t)v;
    m[2 * i + 1] = (uint32_t)(v >> 32);
}

__device__ __forceinline__ void store_digest(const uint32_t* h, uint64_t* o) {
#pragma unroll
    for (int i = 0; i < 4; i++) o[i] = ((uint64_t)h[2 * i + 1] << 32) | h[2 * i];
}

// Leaf L = elements src[c][L], c < n_cols, continuing a message of which `cols_before`
// elements (a multiple of 8) were absorbed earlier (HAS_IN: chaining value h from
// state_in[L]).  FINAL: the last block is the message's last (final flag, byte count
// 8 * (cols_before + n_cols)) and the digest is written; otherwise n_cols is a multiple of
// 8, every block is non-final and the chaining value h goes to out[L] for the next range.
template <bool HAS_IN, bool FINAL>
__global__ __launch_bounds__(B2S_THREADS) void b2s_leaf_kernel(const uint64_t* __restrict__ src, size_t col_stride,
                                                               uint32_t n_cols, size_t n_leaves, uint64_t cols_before,
                                                               const uint64_t* state_in, uint64_t* out) {
    const size_t L = blockIdx.x * (size_t)B2S_THREADS + threadIdx.x;
    if (L >= n_leaves) return;
    const uint64_t* p = src + L;
    uint32_t h[8];
    if (HAS_IN) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint64_t v = state_in[4 * L + i];
            h[2 * i] = (uint32_t)v;
            h[2 * i + 1] = (uint32_t)(v >> 32);
        }
    } else {
        init_h(h);
    }
    // blocks of this range; with FINAL the last one carries the flag (an empty message is
    // one zero block)
    const uint32_t full = n_cols >> 3;
    const uint32_t rem = n_cols & 7;
    const uint32_t nonfinal_full = (FINAL && rem == 0 && full > 0) ? full - 1 : full;
    uint64_t bytes = 8 * cols_before;
    uint32_t m[16];
    uint64_t nxt[8];
    if (nonfinal_full > 0) {
#pragma unroll
        for (int i = 0; i < 8; i++) nxt[i] = p[(size_t)i * col_stride];
    }
    for (uint32_t g = 0; g < nonfinal_full; g++) {
#pragma unroll
        for (int i = 0; i < 8; i++) put(m, i, nxt[i]);
        if (g + 1 < nonfinal_full) {
            const uint64_t* q = p + (size_t)(g + 1) * 8 * col_stride;
#pragma unroll
            for (int i = 0; i < 8; i++) nxt[i] = q[(size_t)i * col_stride];
        }
        bytes += 64;
        compress(h, m, (uint32_t)bytes, (uint32_t)(bytes >> 32), false);
    }
    if (FINAL) {
        // the last block: the remaining 8 (rem == 0, full > 0) or rem elements, zero padded
        const uint32_t first = nonfinal_full * 8;
        const uint32_t cnt = n_cols - first;
        const uint64_t* q = p + (size_t)first * col_stride;
#pragma unroll
        for (int i = 0; i < 8; i++) put(m, i, (uint32_t)i < cnt ? q[(size_t)i * col_stride] : 0);
        bytes += 8 * (uint64_t)cnt;
        compress(h, m, (uint32_t)bytes, (uint32_t)(bytes >> 32), true);
    }
    store_digest(h, out + 4 * L);
}

// construct_by_chunking leaves (merkle_tree.rs:176-386): leaf L absorbs, for each source
// column c in order, the E = 2^log_e consecutive elements src[c][L*E .. (L+1)*E).
__global__ __launch_bounds__(B2S_THREADS) void b2s_leaf_chunk_kernel(const uint64_t* __restrict__ src,
                                                                     size_t col_stride, uint32_t n_cols,
                                                                     uint32_t log_e, size_t n_leaves,
                                                                     uint64_t* __restrict__ out) {
    const size_t L = blockIdx.x * (size_t)B2S_THREADS + threadIdx.x;
    if (L >= n_leaves) return;
    const uint32_t E = 1u << log_e;
    const uint64_t* p = src + (L << log_e);
    uint32_t h[8];
    init_h(h);
    const uint32_t total = n_cols << log_e;
    uint32_t m[16];
    uint32_t k = 0;
    for (; k + 8 < total; k += 8) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t e = k + i;
            put(m, i, p[(size_t)(e >> log_e) * col_stride + (e & (E - 1))]);
        }
        const uint64_t bytes = 8 * (uint64_t)(k + 8);
        compress(h, m, (uint32_t)bytes, (uint32_t)(bytes >> 32), false);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t e = k + i;
        put(m, i, e < total ? p[(size_t)(e >> log_e) * col_stride + (e & (E - 1))] : 0);
    }
    const uint64_t bytes = 8 * (uint64_t)total;
    compress(h, m, (uint32_t)bytes, (uint32_t)(bytes >> 32), true);
    store_digest(h, out + 4 * L);
}

__device__ __forceinline__ void node_hash(const uint64_t* l, const uint64_t* r, uint64_t* o) {
    uint32_t h[8], m[16];
    init_h(h);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        m[2 * i] = (uint32_t)l[i];
        m[2 * i + 1] = (uint32_t)(l[i] >> 32);
        m[8 + 2 * i] = (uint32_t)r[i];
        m[8 + 2 * i + 1] = (uint32_t)(r[i] >> 32);
    }
    compress(h, m, 64, 0, true);
    store_digest(h, o);
}

__global__ __launch_bounds__(256) void b2s_node_level_kernel(const uint64_t* __restrict__ prev,
                                                             uint64_t* __restrict__ next, size_t m) {
    const size_t i = blockIdx.x * (size_t)256 + threadIdx.x;
    if (i >= m) return;
    uint64_t lr[8];
#pragma unroll
    for (int k = 0; k < 8; k++) lr[k] = prev[8 * i + k];
    node_hash(lr, lr + 4, next + 4 * i);
}

// Remaining levels from `len` digests (len <= 4096) down to cap_size, one workgroup.
__global__ __launch_bounds__(256) void b2s_node_tail_kernel(const uint64_t* __restrict__ prev, uint64_t* next,
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
        for (int k = 0; k < 4; k++) {
            buf[cur][4 * i + k] = o[k];
            outp[4 * (size_t)i + k] = o[k];
        }
    }
    outp += 4 * (size_t)m;
    __syncthreads();
    while (m > cap_size) {
        const uint32_t m2 = m / 2;
        for (uint32_t i = threadIdx.x; i < m2; i += 256) {
            uint64_t o[4];
            node_hash(&buf[cur][8 * i], &buf[cur][8 * i + 4], o);
            for (int k = 0; k < 4; k++) {
                buf[cur ^ 1][4 * i + k] = o[k];
                outp[4 * (size_t)i + k] = o[k];
            }
        }
        outp += 4 * (size_t)m2;
        cur ^= 1;
        m = m2;
        __syncthreads();
    }
}

// one whole message per lane (the host seam bj_blake2s_leaf_h and its tests)
__global__ void b2s_bytes_kernel(const uint64_t* __restrict__ words, uint32_t n_words, uint64_t* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint32_t h[8], m[16];
    init_h(h);
    uint32_t k = 0;
    for (; k + 8 < n_words; k += 8) {
        for (int i = 0; i < 8; i++) put(m, i, words[k + i]);
        const uint64_t bytes = 8 * (uint64_t)(k + 8);
        compress(h, m, (uint32_t)bytes, (uint32_t)(bytes >> 32), false);
    }
    for (int i = 0; i < 8; i++) put(m, i, k + i < n_words ? words[k + i] : 0);
    const uint64_t bytes = 8 * (uint64_t)n_words;
    compress(h, m, (uint32_t)bytes, (uint32_t)(bytes >> 32), true);
    store_digest(h, out);
}

}  // namespace

hipError_t launch_b2s_leaves(const uint64_t* src, size_t col_stride, uint32_t n_cols, size_t n_leaves,
                             uint64_t cols_before, const uint64_t* state_in, uint64_t* out, bool final_,
                             hipStream_t st) {
    if (n_leaves == 0) return hipSuccess;
    const dim3 g((unsigned)((n_leaves + B2S_THREADS - 1) / B2S_THREADS));
#define BJ_B2S_LEAF(IN, FIN)                                                                                  \
    hipLaunchKernelGGL((b2s_leaf_kernel<IN, FIN>), g, dim3(B2S_THREADS), 0, st, src, col_stride, n_cols, n_leaves, \
                       cols_before, state_in, out)
    if (state_in) {
        if (final_) BJ_B2S_LEAF(true, true);
        else BJ_B2S_LEAF(true, false);
    } else {
        if (final_) BJ_B2S_LEAF(false, true);
        else BJ_B2S_LEAF(false, false);
    }
#undef BJ_B2S_LEAF
    return hipGetLastError();
}

hipError_t launch_b2s_leaves_chunked(const uint64_t* src, size_t col_stride, uint32_t n_cols, uint32_t log_e,
                                     size_t n_leaves, uint64_t* out, hipStream_t st) {
    if (n_leaves == 0) return hipSuccess;
    hipLaunchKernelGGL(b2s_leaf_chunk_kernel, dim3((unsigned)((n_leaves + B2S_THREADS - 1) / B2S_THREADS)),
                       dim3(B2S_THREADS), 0, st, src, col_stride, n_cols, log_e, n_leaves, out);
    return hipGetLastError();
}

hipError_t launch_b2s_nodes(const uint64_t* leaves, size_t n_leaves, uint32_t cap_size, uint64_t* nodes,
                            hipStream_t st) {
    const uint64_t* prev = leaves;
    uint64_t* out = nodes;
    size_t len = n_leaves;
    while (len > cap_size && len > 4096) {
        const size_t m = len / 2;
        hipLaunchKernelGGL(b2s_node_level_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, prev, out, m);
        prev = out;
        out += 4 * m;
        len = m;
    }
    if (len > cap_size)
        hipLaunchKernelGGL(b2s_node_tail_kernel, dim3(1), dim3(256), 0, st, prev, out, (uint32_t)len, cap_size);
    return hipGetLastError();
}

hipError_t launch_b2s_words(const uint64_t* words, uint32_t n_words, uint64_t* out, hipStream_t st) {
    hipLaunchKernelGGL(b2s_bytes_kernel, dim3(1), dim3(64), 0, st, words, n_words, out);
    return hipGetLastError();
}

}  // namespace bj
