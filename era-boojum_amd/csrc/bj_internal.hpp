// Internal launcher declarations shared by the .hip translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

namespace bj {

// Experiment knobs (round 6).  The A/B switches of the kernel schedule -- BJ_LEAVES_DEFER and
// BJ_LEAVES_GROUP and BJ_LDE_OWN_FUSED (collective.hip), BJ_INV_FOLD_UNPAIRED (ntt_lde3.hip), BJ_LDE_PASSES (capi.hip) and
// BJ_NODE_Q4_MAX and BJ_NODE_FUSED (merkle.hip) -- are read from the environment only when BJ_EXPERIMENTS=1 is
// set, once per process, at the first call that needs one; otherwise each has its production
// value, so a prover's environment cannot change the schedule (the reference's
// transform_raw_storages_to_lde, utils.rs:270-403, is a pure function of its inputs).
// bj_experiment_knob (ABI 2.6) reports the values in effect.
struct Knobs {
    bool enabled;
    uint64_t leaves_defer;       // 0: chunk k's leaves right after its own LDE
    uint64_t leaves_group;       // 0: one chunk per leaf grid (collective.hip leaves_group())
    uint64_t inv_fold_unpaired;  // 0: the paired even/odd sender fold where the constants pair
    uint64_t lde_passes;         // 3: the three-pass LDE for 2^18..2^23 (2: head + tail per transform)
    uint64_t node_q4_max;        // 2^15: levels of at most this many digests use quad-lane permutations
    uint64_t node_fused;         // 1: those levels run up to 8 per launch (node_levels_q4_kernel)
    uint64_t lde_own_fused;      // 1: G <= D ranks fuse their own columns' inverse tail into the forward
};
inline Knobs read_knobs() {
    Knobs k{false, 0, 0, 0, 3, (uint64_t)1 << 15, 1, 1};
    const char* g = getenv("BJ_EXPERIMENTS");
    k.enabled = g && strcmp(g, "1") == 0;
    if (!k.enabled) return k;
    const char* e;
    if ((e = getenv("BJ_LEAVES_DEFER"))) k.leaves_defer = strtoull(e, nullptr, 0);
    if ((e = getenv("BJ_LEAVES_GROUP"))) k.leaves_group = strtoull(e, nullptr, 0);
    if ((e = getenv("BJ_INV_FOLD_UNPAIRED"))) k.inv_fold_unpaired = e[0] == '1';
    if ((e = getenv("BJ_LDE_PASSES"))) k.lde_passes = e[0] == '2' ? 2 : 3;
    if ((e = getenv("BJ_NODE_Q4_MAX"))) k.node_q4_max = strtoull(e, nullptr, 0);
    if ((e = getenv("BJ_NODE_FUSED"))) k.node_fused = e[0] != '0';
    if ((e = getenv("BJ_LDE_OWN_FUSED"))) k.lde_own_fused = e[0] != '0';
    return k;
}
// one instance per shared library (an inline function's static is merged across its TUs)
inline const Knobs& knobs() {
    static const Knobs k = read_knobs();
    return k;
}

hipError_t launch_bitrev_scale(uint64_t* dst, size_t dst_stride, const uint64_t* src, size_t src_stride,
                               uint32_t n_cols, uint32_t log_n, uint64_t scale, hipStream_t st);
hipError_t launch_twiddles(uint64_t* out, uint32_t log_n, bool inverse, hipStream_t st);
hipError_t launch_twiddles_natural(uint64_t* out, uint32_t log_n, bool inverse, hipStream_t st);
hipError_t launch_bitrev_inplace(uint64_t* cols, size_t col_stride, uint32_t n_cols, uint32_t log_n, hipStream_t st);
hipError_t launch_power_tables(uint64_t* lo, uint64_t* hi, uint32_t log_n, uint64_t e, uint64_t scale,
                               hipStream_t st);
hipError_t launch_distribute(uint64_t* cols, size_t col_stride, uint32_t n_cols, uint32_t log_n,
                             const uint64_t* lo, const uint64_t* hi, hipStream_t st);

hipError_t launch_leaves(const uint64_t* src, size_t col_stride, uint32_t n_cols, size_t n_leaves, uint64_t* out,
                         hipStream_t st);
hipError_t launch_leaves_partial(const uint64_t* src, size_t col_stride, uint32_t n_cols, size_t n_leaves,
                                 const uint64_t* cap_in, uint64_t* out, bool final_, hipStream_t st);
hipError_t launch_leaves_chunked(const uint64_t* src, size_t col_stride, uint32_t n_cols, uint32_t log_e,
                                 size_t n_leaves, uint64_t* out, hipStream_t st);
hipError_t launch_nodes(const uint64_t* leaves, size_t n_leaves, uint32_t cap_size, uint64_t* nodes,
                        hipStream_t st);
hipError_t launch_permute(uint64_t* states, size_t count, hipStream_t st);
hipError_t launch_synthetic(uint64_t* dst, size_t col_stride, uint32_t n_cols, uint32_t log_n, uint64_t seed,
                            uint64_t col0, hipStream_t st);

hipError_t launch_gl_op(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n, hipStream_t st);

hipError_t launch_twiddle_pyramid(uint64_t* out, uint32_t log_n, bool inverse, hipStream_t st);
hipError_t launch_dif(uint64_t* dst, size_t dst_stride, const uint64_t* src, size_t src_stride, uint32_t n_cols,
                      uint32_t log_n, const uint64_t* tw_pyr, bool canon_out, hipStream_t st);
hipError_t launch_lde_forward(uint64_t* lde, size_t lde_col_stride, uint32_t n_cosets, const uint64_t* raw,
                              size_t raw_stride, bool raw_bitrev, uint32_t n_cols, uint32_t log_n,
                              const uint64_t* tw_pyr, const uint64_t* pw, size_t pw_stride, hipStream_t st);

// power table sizes for a column of 2^log_n: lo 4096, hi max(1, n / 4096)
inline size_t pw_hi_len(uint32_t log_n) { return log_n > 12 ? ((size_t)1 << (log_n - 12)) : 1; }

}  // namespace bj

namespace bj {
// blake2s.hip: Blake2s256 tree hasher (cs/oracle/mod.rs:179-245)
hipError_t launch_b2s_leaves(const uint64_t* src, size_t col_stride, uint32_t n_cols, size_t n_leaves,
                             uint64_t cols_before, const uint64_t* state_in, uint64_t* out, bool final_,
                             hipStream_t st);
hipError_t launch_b2s_leaves_chunked(const uint64_t* src, size_t col_stride, uint32_t n_cols, uint32_t log_e,
                                     size_t n_leaves, uint64_t* out, hipStream_t st);
hipError_t launch_b2s_nodes(const uint64_t* leaves, size_t n_leaves, uint32_t cap_size, uint64_t* nodes,
                            hipStream_t st);
hipError_t launch_b2s_words(const uint64_t* words, uint32_t n_words, uint64_t* out, hipStream_t st);

// keccak.hip: Keccak256 tree hasher (cs/oracle/mod.rs:247-313)
hipError_t launch_kc_leaves(const uint64_t* src, size_t col_stride, uint32_t n_cols, size_t n_leaves, uint64_t* out,
                            hipStream_t st);
hipError_t launch_kc_leaves_chunked(const uint64_t* src, size_t col_stride, uint32_t n_cols, uint32_t log_e,
                                    size_t n_leaves, uint64_t* out, hipStream_t st);
hipError_t launch_kc_nodes(const uint64_t* leaves, size_t n_leaves, uint32_t cap_size, uint64_t* nodes,
                           hipStream_t st);

// shard.hip: sub-coset fold of the bit-reversed coefficients (G > D shards)
constexpr uint32_t kMaxFold = 64;
hipError_t launch_fold(uint64_t* dst, size_t dst_stride, const uint64_t* src, size_t src_stride, uint32_t n_cols,
                       uint32_t log_m, uint32_t log_f, uint64_t s_pow_m, hipStream_t st);
// the same fold for `shards` targets at once: dst + P * dst_shard_stride + c * dst_col_stride
// receives column c folded with s_pow_m[P]
hipError_t launch_fold_all(uint64_t* dst, size_t dst_col_stride, size_t dst_shard_stride, const uint64_t* src,
                           size_t src_stride, uint32_t n_cols, uint32_t log_m, uint32_t log_f, uint32_t shards,
                           const uint64_t* s_pow_m, hipStream_t st);

}  // namespace bj

namespace bj {
// ntt_ct.hip: coset-folded Cooley-Tukey passes for 2^13 <= n <= 2^23
bool ct_ntt_supported(uint32_t log_n);
// entries of one CT table (the coset-folded table + the power-of-two phases' prescale tables)
size_t ct_table_len(uint32_t log_n);
hipError_t launch_ct_table(uint64_t* out, uint32_t log_n, bool inverse, uint64_t shift, uint64_t scale1,
                           hipStream_t st);
hipError_t launch_ct(uint64_t* dst, size_t dst_col_stride, size_t coset_stride, uint32_t n_cosets,
                     const uint64_t* src, size_t src_stride, bool src_bitrev, uint32_t n_cols, uint32_t log_n,
                     const uint64_t* tab, size_t tab_stride, uint64_t kappa, bool canon_out, hipStream_t st);
hipError_t launch_scale(uint64_t* cols, size_t stride, uint32_t n_cols, size_t n, uint64_t k, hipStream_t st);
hipError_t launch_ct_inverse_head(uint64_t* dst, size_t dst_col_stride, const uint64_t* src, size_t src_stride,
                                  uint32_t n_cols, uint32_t log_n, const uint64_t* inv_tab, hipStream_t st);

// ntt_lde3.hip: the three-pass LDE for 2^18 <= n <= 2^23 (inverse head; inverse tail fused with
// the first 13 forward stages of every coset; the last log n - 13 forward stages)
bool lde3_supported(uint32_t log_n);
size_t lde3_table_len(uint32_t log_n);
hipError_t launch_lde3_table(uint64_t* out, uint32_t log_n, uint64_t shift, hipStream_t st);
// middle + final passes.  src: inv_tab != NULL -> the inverse head's output (natural order after
// its log n - 13 stages), and mono (if non-NULL) receives the canonical monomials in bit-reversed
// order; inv_tab == NULL -> src holds the monomials in bit-reversed order already.  `passes`
// selects the middle pass (stages 0..12 of every coset), the final pass (the last log n - 13, in
// place on the middle pass's output), or both.  Output coset
// i (table tabs + i * tab_stride) of column c at lde + c * col_stride + i * coset_stride; with
// log_k < log2(n_cosets) the cosets come in blocks of 2^log_k, coset i at
// lde + c * col_stride + (i >> log_k) * block_stride + (i mod 2^log_k) * coset_stride.
constexpr uint32_t LDE3_MID = 1, LDE3_FINAL = 2, LDE3_BOTH = 3;
hipError_t launch_lde3(uint64_t* lde, size_t col_stride, size_t coset_stride, uint32_t n_cosets, const uint64_t* src,
                       size_t src_stride, uint64_t* mono, size_t mono_stride, uint32_t n_cols, uint32_t log_n,
                       const uint64_t* inv_tab, const uint64_t* tabs, size_t tab_stride, hipStream_t st,
                       uint32_t log_k = 31, size_t block_stride = 0, uint32_t passes = LDE3_BOTH);
// the inverse tail on the inverse head's output src, folded by F = 2^log_f (1..3) for `shards`
// targets: dst + P * dst_shard_stride + c * dst_col_stride receives column c's monomials folded
// with s_pow_m[P] (launch_fold_all's output), the monomials themselves never written
bool lde3_inv_fold_supported(uint32_t log_n, uint32_t log_f, uint32_t shards);
hipError_t launch_lde3_inv_fold(uint64_t* dst, size_t dst_col_stride, size_t dst_shard_stride, const uint64_t* src,
                                size_t src_stride, uint32_t n_cols, uint32_t log_n, uint32_t log_f, uint32_t shards,
                                const uint64_t* s_pow_m, const uint64_t* inv_tab, hipStream_t st);
}  // namespace bj

namespace bj {
// fri.hip: one FRI fold by 2 of a GoldilocksExt2 codeword (c0, c1)
hipError_t launch_fri_fold(const uint64_t* c0, const uint64_t* c1, size_t n_out, const uint64_t* roots,
                           uint64_t coset_inverse, uint64_t ch0, uint64_t ch1, uint64_t* d0, uint64_t* d1,
                           hipStream_t st);
}  // namespace bj

namespace bj {
// capi.hip: set the calling thread's bj_last_error() message; returns code
int set_error(int code, const char* msg);
// capi.hip: stream-ordered allocation from the library's private pool of the current device
// (free with hipFreeAsync); the process's default pool is never reconfigured
hipError_t pool_alloc(void** p, size_t bytes, hipStream_t st);
hipError_t pool_trim_all();
// capi.hip: LDE coset shift 7 * w_{nD}^{bitrev_{log D}(i)} (utils.rs:334-347, 370-373) and the
// shift of leaf range `shard` of 2^log_shards over the n*D domain, 7 * w_{nD}^{bitrev(shard)}
uint64_t shard_shift(uint32_t log_n, uint32_t log_lde, uint32_t log_shards, uint32_t shard);
// capi.hip: the fused three-pass LDE of the trace (bj_lde_ex_d's kernels, no monomial write-back)
// with the D cosets laid out in blocks of 2^log_k: coset i of column c at
// lde + (i >> log_k) * block_stride + c * col_stride + (i mod 2^log_k) * 2^log_n.  scratch holds
// n_cols * 2^log_n words.  False (nothing launched) when log_n is outside the three-pass range.
bool lde_fused_supported(uint32_t log_n);
int lde_fused_blocks(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n, uint32_t log_lde,
                     uint32_t log_k, uint64_t* scratch, uint64_t* lde, size_t col_stride, size_t block_stride,
                     hipStream_t st);
// capi.hip: the sender-side fold of the trace's monomials for `targets` shards without writing the
// monomials (the inverse head into scratch, n_cols * 2^log_n words, then launch_lde3_inv_fold): target
// T of column c at dst + T * dst_shard_stride + c * dst_col_stride, folded with s_pow_m[T] --
// launch_fold_all's output.  inverse_fold_supported false: use bj_lde_coeffs_d + launch_fold_all.
bool inverse_fold_supported(uint32_t log_n, uint32_t log_f, uint32_t targets);
// capi.hip: a rank's own columns at G <= D (whole cosets [P per, (P + 1) per), per = D / G): the
// inverse head of the trace into mono, then the inverse tail fused with forward stages 0..12 of
// the rank's cosets (lde3_mid_kernel<R, true, true>), which writes the canonical monomials back
// to mono (the exchange format, c_j at bitrev_n(j)) and the cosets' middle-pass output to lde
// (column c at lde + c * col_stride, coset i at + i * 2^log_n); passes LDE3_FINAL then runs the
// last stages in place.  The monomials are written once and never read back for these columns.
int lde_own_shard(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n, uint32_t log_lde,
                  uint32_t log_shards, uint32_t shard, uint64_t* mono, size_t mono_stride, uint64_t* lde,
                  size_t col_stride, uint32_t passes, hipStream_t st);
int inverse_fold_all(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n, uint32_t log_f,
                     uint32_t targets, const uint64_t* s_pow_m, uint64_t* scratch, size_t scratch_stride,
                     uint64_t* dst, size_t dst_col_stride, size_t dst_shard_stride, hipStream_t st);
}  // namespace bj
