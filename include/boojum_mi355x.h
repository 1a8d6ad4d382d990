/*
 * boojum_mi355x.h -- C ABI of the MI355X-native witness-commitment hot path
 * (coset LDE over Goldilocks + Poseidon2 Merkle tree with cap).
 *
 * Library: era-boojum_amd/boojum_amd/libboojum_mi355x.so (hipcc, gfx950).
 * Plain C types only: pointers, sizes, u64 field elements.  All field elements
 * crossing this boundary are u64; outputs are canonical (< p = 2^64 - 2^32 + 1),
 * inputs may be any u64 representative (as the reference's GoldilocksField,
 * field/goldilocks/mod.rs:92-94).
 *
 * Return value: 0 on success, a negative errno-style code on failure
 * (BJ_EINVAL for violated preconditions -- the reference asserts/panics on these,
 * fft/mod.rs:399-402, utils.rs:284-287, merkle_tree.rs:83-96 -- BJ_EHIP for a HIP
 * runtime error).  bj_last_error() gives a message for the calling thread.
 * A Rust/ctypes shim maps non-zero to panic!/raise, keeping reference semantics.
 *
 * Two families:
 *   *_d   device-resident batched entry points.  Pointers are device (HBM)
 *         pointers; `stream` is a hipStream_t (NULL = default stream).  Calls are
 *         asynchronous on the stream and never synchronise the device.  These are
 *         what a batched GPU prover calls once per commitment.
 *   *_h   host-pointer entry points with exactly the reference seam's per-call
 *         semantics (in place, synchronous), for drop-in replacement of the
 *         reference functions named in each comment.
 *
 * Thread safety: all entry points are re-entrant (the reference calls its FFT seam
 * concurrently from rayon workers, cs/implementations/utils.rs:295-304,363-379).
 * The only global state is a per-device cache of twiddle tables, filled under a
 * lock on first use of a size (bj_prepare fills it ahead of time; bj_release_tables, which must
 * not run concurrently with other calls, empties it).
 */
#ifndef BOOJUM_MI355X_H
#define BOOJUM_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BJ_OK 0
#define BJ_EINVAL (-22)
#define BJ_ENOMEM (-12)
#define BJ_EHIP (-5)

/* Message for the last failure on the calling thread ("" if none). */
const char* bj_last_error(void);
/* ABI version (major << 16 | minor). */
uint32_t bj_abi_version(void);

/* The value in effect of one experiment knob (ABI 2.6; no reference counterpart).  The library's
 * same-binary A/B switches -- BJ_LEAVES_DEFER (default 0), BJ_LEAVES_GROUP (0: one chunk per
 * leaf grid), BJ_INV_FOLD_UNPAIRED (0),
 * BJ_LDE_PASSES (3), BJ_NODE_Q4_MAX (32768), BJ_NODE_FUSED (1) and BJ_LDE_OWN_FUSED (1) -- are read from the environment only when
 * BJ_EXPERIMENTS=1 is set, once per process at the first call that needs one; otherwise each
 * keeps its production value, so a prover's environment cannot change the kernel schedule (the
 * reference's transform_raw_storages_to_lde, cs/implementations/utils.rs:270-403, is a pure
 * function of its inputs).  Every setting gives the same outputs.  name "BJ_EXPERIMENTS" reports
 * the gate (0 / 1).  BJ_EINVAL for an unknown name.  Host-only: touches no device. */
int bj_experiment_knob(const char* name, uint64_t* value);

/* Fill the device twiddle cache for FFT size 2^log_n (forward + inverse tables) on the
 * current device, synchronously.  Twiddle precompute is outside the timed region in
 * the reference's own accounting (prover.rs:313-353 precomputes before "LDE taken").
 * Cached tables stay until bj_release_tables; for 2^13 <= n <= 2^26 a table of one coset shift
 * is n + 1056 (1 + n / 2^13) u64 (36 MiB at 2^22), and an LDE at degree D keeps D of them. */
int bj_prepare(uint32_t log_n);

/* Return the library's cached device workspace to the system (ABI 2.1; no reference
 * counterpart: the reference's Vec workspaces are freed when dropped).  The *_h calls, the
 * host-buffer commit, the collective commit and the LDE's own temporaries take their device
 * workspace from a stream-ordered pool private to the library (one per device); freed blocks
 * stay mapped for the next call (re-mapping C2's 5 GB after every call cost ~20 ms), so after a
 * large call the pool keeps that much reserved -- e.g. ~8.5 GB after a native C3 commit at N = 1.
 * This trims every device's pool to the blocks still in use (hipMemPoolTrimTo(pool, 0)); blocks
 * whose stream-ordered free has not completed yet are released by a later call.  Call it when a
 * long-running prover goes idle.  Twiddle tables (bj_prepare) are not affected. */
int bj_release_workspace(void);

/* Free every cached table (twiddles, coset powers, the LDE passes' factor tables) on every device
 * (ABI 2.3; no reference counterpart: the reference's twiddles are Vecs the caller drops).  The
 * cache only grows: an LDE of 2^22 rows at degree 4 keeps ~180 MiB, one of 2^23 at degree 8
 * ~600 MiB, and a prover that commits many sizes keeps the tables of each.  Each device with
 * tables is synchronised first, so work already queued there has finished with them; no other
 * library call may run concurrently with this one, and a HIP graph captured over library calls
 * holds table addresses, so it must be captured again afterwards.  Later calls rebuild what they
 * need (as on first use; bj_prepare rebuilds ahead of time). */
int bj_release_tables(void);

/* ---------------------------------------------------------------- FFT seam */

/* precompute_twiddles_for_fft::<INVERSED> (cs/implementations/utils.rs:88-125,
 * wrapper fft/mod.rs:625-641): omega_n^i (or omega_n^-i), i < n/2, bit-reversed order.
 * out_d: n/2 u64 (device). */
int bj_precompute_twiddles_d(uint32_t log_n, int inverse, uint64_t* out_d, void* stream);
int bj_precompute_twiddles_h(uint32_t log_n, int inverse, uint64_t* out_h);

/* precompute_twiddles_for_fft_natural (cs/implementations/utils.rs:127-155, wrapper
 * fft/mod.rs:640-657): w^i (or w^-i) for i < n/2 in natural order, canonical; out_d has n/2
 * u64 on the device. */
int bj_precompute_twiddles_natural_d(uint32_t log_n, int inverse, uint64_t* out_d, void* stream);

/* bitreverse_enumeration_inplace (fft/mod.rs:41-155): the bit-reversal permutation of each of
 * n_cols columns of n = 2^log_n, in place; values are moved unchanged. */
int bj_bitreverse_enumeration_d(uint64_t* cols, uint32_t n_cols, size_t col_stride, uint32_t log_n, void* stream);

/* distribute_powers (fft/mod.rs:308-317): col[j] *= element^j, for n_cols columns of
 * 2^log_n elements, column c at cols + c * col_stride. */
int bj_distribute_powers_d(uint64_t* cols, uint32_t n_cols, size_t col_stride, uint32_t log_n,
                           uint64_t element, void* stream);
int bj_distribute_powers_h(uint64_t* col, size_t len, uint64_t element);

/* fft_natural_to_bitreversed (fft/mod.rs:398-411; PrimeFieldLikeVectorized seam
 * field/traits/field_like.rs:111-162): distribute_powers(coset) if coset != 1, then the
 * radix-2 natural->bit-reversed transform (fft/mod.rs:659-734).  In place.
 * twiddles may be NULL (the device cache is used); if given it must be the
 * bj_precompute_twiddles output for this size (it is used as is). */
int bj_fft_natural_to_bitreversed_d(uint64_t* cols, uint32_t n_cols, size_t col_stride, uint32_t log_n,
                                    uint64_t coset, const uint64_t* twiddles_d, void* stream);
int bj_fft_natural_to_bitreversed_h(uint64_t* col, size_t len, uint64_t coset);

/* ifft_natural_to_natural (fft/mod.rs:464-491): inverse transform, bit-reverse, times
 * coset^-j if coset != 1, times n^-1.  In place. */
int bj_ifft_natural_to_natural_d(uint64_t* cols, uint32_t n_cols, size_t col_stride, uint32_t log_n,
                                 uint64_t coset, const uint64_t* inv_twiddles_d, void* stream);
int bj_ifft_natural_to_natural_h(uint64_t* col, size_t len, uint64_t coset);

/* ------------------------------------------------------------------- LDE */

/* transform_raw_storages_to_lde (cs/implementations/utils.rs:270-309 + :311-403, as
 * driven by WitnessStorage::from_base_trace*, witness_storage.rs:18-116):
 *   monomials[c] = ifft_natural_to_natural(trace[c])
 *   lde[c][i]    = fft_natural_to_bitreversed(monomials[c], 7 * w_{nD}^{bitrev(i)})
 * trace:   n_cols columns of n = 2^log_n at trace + c * trace_stride (read only)
 * scratch: n_cols x n device workspace (on return it holds the monomials in bit-reversed
 *          order, c_j at bitrev_n(j) -- the format of bj_lde_coeffs_d)
 * lde:     n_cols x D x n, element (c, i, r) at lde + (c * D + i) * n + r
 *          (the reference's per-column Vec<coset> of ArcGenericLdeStorage)
 * D = 2^log_lde. */
int bj_lde_d(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n,
             uint32_t log_lde, uint64_t* scratch, uint64_t* lde, void* stream);

/* bj_lde_d with flags (ABI 2.2).  Without BJ_LDE_KEEP_MONOMIALS, scratch is workspace only and
 * its contents on return are unspecified -- the reference's transform_raw_storages_to_lde
 * (utils.rs:270-403) returns the LDE alone and drops the monomials, and the three-pass path
 * (2^18 <= n <= 2^23) then skips writing them (one pass over n words per column less).
 * bj_lde_d == bj_lde_ex_d(..., BJ_LDE_KEEP_MONOMIALS, ...).  Unknown flags: BJ_EINVAL. */
#define BJ_LDE_KEEP_MONOMIALS 1u
int bj_lde_ex_d(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n,
                uint32_t log_lde, uint64_t* scratch, uint64_t* lde, uint32_t flags, void* stream);

/* Coset LDE of already-monomial columns (transform_monomials_to_lde, utils.rs:311-403;
 * also the quotient commit path prover.rs:1471-1482).  monomials read only. */
int bj_monomials_to_lde_d(const uint64_t* monomials, uint32_t n_cols, size_t mono_stride, uint32_t log_n,
                          uint32_t log_lde, uint64_t* lde, void* stream);

/* ------------------------------------------------ coset-sharded LDE (8(e)) */
/* The multi-GPU split of transform_raw_storages_to_lde (utils.rs:270-403) over G = 2^log_shards
 * ranks: the flat leaf domain L = coset * n + row (merkle_tree.rs:112-157 leaf order) is cut
 * into G contiguous ranges of m = n*D/G leaves; rank P owns [P*m, (P+1)*m).
 *
 * Step 1 (every rank, its own trace columns): bj_lde_coeffs_d writes the inverse transform
 *   in the exchange format: column c holds c_j at position bitrev_n(j), where c_j are the
 *   monomials of ifft_natural_to_natural (utils.rs:295-304), canonical.  Ranks all-gather
 *   these columns.
 * Step 2 (every rank, all columns): bj_lde_shard_d evaluates its leaf range:
 *   G <= D: cosets [P*D/G, (P+1)*D/G), each as in bj_lde_d;
 *   G >  D: rows [q*m, (q+1)*m) of coset i = P / (G/D), q = P mod (G/D), as an m-point coset
 *           FFT of the coefficients folded mod Y^m - s'^m, s' = 7 * w_{nD}^{bitrev_{log G}(P)}.
 *   lde: n_cols x m, element (c, L - P*m) at lde + c * m + (L - P*m), identical to the slice
 *   of bj_lde_d's output for those leaves.  work: n_cols x m device scratch (G > D only;
 *   may be NULL when G <= D).  Requires log_shards <= log_n + log_lde and, for G > D,
 *   G / D <= 64. */
int bj_lde_coeffs_d(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n,
                    uint64_t* coeffs, size_t coeffs_stride, void* stream);
int bj_lde_shard_d(const uint64_t* coeffs, uint32_t n_cols, size_t coeffs_stride, uint32_t log_n,
                   uint32_t log_lde, uint32_t log_shards, uint32_t shard, uint64_t* work, uint64_t* lde,
                   void* stream);

/* G > D with the fold moved to the sender (all-to-all exchange of m-length columns instead of
 * an all-gather of n-length ones: n/m = G/D times fewer bytes on the wire).
 * bj_lde_fold_shards_d (every rank, its own columns in the bj_lde_coeffs_d format): for every
 *   shard P < G, out + P * out_shard_stride + c * m receives column c folded mod
 *   Y^m - s_P^m, bit-reversed (the h of bj_lde_shard_d's fold step); out_shard_stride >=
 *   n_cols * m.
 * bj_lde_shard_folded_d (rank P, every column folded for P, gathered from all ranks): the
 *   m-point coset transform of the folded columns, the same leaf range and layout as
 *   bj_lde_shard_d.  folded read only. */
int bj_lde_fold_shards_d(const uint64_t* coeffs, uint32_t n_cols, size_t coeffs_stride, uint32_t log_n,
                         uint32_t log_lde, uint32_t log_shards, uint64_t* out, size_t out_shard_stride,
                         void* stream);
int bj_lde_shard_folded_d(const uint64_t* folded, uint32_t n_cols, size_t folded_stride, uint32_t log_n,
                          uint32_t log_lde, uint32_t log_shards, uint32_t shard, uint64_t* lde, void* stream);

/* ---------------------------------------------------------- Poseidon2 / Merkle */

/* poseidon2_permutation (implementations/poseidon2/state_generic_impl.rs:221-249) on
 * `count` independent 12-element states, in place. */
int bj_poseidon2_permute_d(uint64_t* states, size_t count, void* stream);
int bj_poseidon2_permute_h(uint64_t* state12);

/* TreeHasher::hash_into_leaf for GoldilocksPoseidon2Sponge<AbsorptionModeOverwrite>
 * (cs/oracle/mod.rs:141-151, algebraic_props/sponge.rs:224-323) of n_elems elements. */
int bj_hash_into_leaf_h(const uint64_t* elems, size_t n_elems, uint64_t* out4);
/* TreeHasher::hash_into_node (cs/oracle/mod.rs:162-168). */
int bj_hash_into_node_h(const uint64_t* left4, const uint64_t* right4, uint64_t* out4);

/* Leaf hashing of MerkleTreeWithCap::construct (cs/oracle/merkle_tree.rs:78-172):
 * leaf L (flat index coset * n + row) = hash_into_leaf(src[0][L], ..., src[n_cols-1][L]),
 * column c's leaf-domain values at src + c * col_stride.  leaves: n_leaves x 4. */
int bj_merkle_leaves_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                       uint64_t* leaves, void* stream);

/* Leaf hashing of MerkleTreeWithCap::construct_by_chunking (merkle_tree.rs:176-306) and
 * construct_by_chunking_from_flat_sources (:308-386), the FRI oracles' trees (fri/mod.rs:179-187,
 * 258-266): leaf L = hash_into_leaf of, for each column c in order, the elems_per_leaf
 * consecutive elements src[c * col_stride + L * elems_per_leaf + t].  elems_per_leaf is a power
 * of two.  With a [c][coset][row] LDE the flat leaf index runs over the cosets in order, as the
 * reference's per-coset chunks do.  leaves: n_leaves x 4. */
int bj_merkle_leaves_chunked_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                               uint32_t elems_per_leaf, uint64_t* out, void* stream);

/* Leaf hashing over a column range, continuing a sponge (the column-pipelined multi-GPU
 * commit absorbs column chunks as they arrive).  The Overwrite sponge replaces the rate words
 * with each 8-element group, so between groups its whole carried state is the capacity
 * state[8..12].  cap_in: NULL for a fresh sponge (zero state), else n_leaves x 4 capacity words
 * from a previous non-final call.  final_ == 0: n_cols must be a multiple of 8; out receives
 * the capacity words (n_leaves x 4, canonical).  final_ != 0: the remaining columns are
 * absorbed with the reference's padding (sponge.rs:300-323) and out receives the digests, as
 * bj_merkle_leaves_d.  cap_in == out is allowed.  Chaining calls over columns [0, k), [k, C)
 * gives exactly bj_merkle_leaves_d over [0, C). */
int bj_merkle_leaves_partial_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                               const uint64_t* cap_in, uint64_t* out, int final_, void* stream);

/* continue_from_leaf_hashes (merkle_tree.rs:388-449): node levels from n_leaves leaves
 * up to cap_size nodes.  nodes: (n_leaves - cap_size) x 4, the levels concatenated from
 * the leaves upward (node_hashes_enumerated_from_leafs); the cap is the last cap_size
 * digests (get_cap, merkle_tree.rs:451-460, canonical).  Requires n_leaves > cap_size,
 * both powers of two. */
int bj_merkle_nodes_d(const uint64_t* leaves, size_t n_leaves, uint32_t cap_size, uint64_t* nodes,
                      void* stream);

/* ------------------------------------------------ Blake2s256 tree hasher */
/* MerkleTreeWithCap<GoldilocksField, blake2::Blake2s256>: the TreeHasher impl of
 * cs/oracle/mod.rs:179-245, used by the non-recursive prover configs
 * (gadgets/sha256/mod.rs:263-269).  Leaf = BLAKE2s-256 (RFC 7693, no key) of the canonical
 * little-endian bytes of the leaf's elements (as_u64_reduced().to_le_bytes(), :194-197);
 * node = BLAKE2s-256(left || right) (:233-245).  A digest is 32 bytes, stored as 4
 * little-endian u64 words, so leaves / nodes use the same (N x 4) layout as the Poseidon2
 * tree.  Same arguments, layouts and preconditions as the bj_merkle_* calls above. */
int bj_blake2s_leaves_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                        uint64_t* leaves, void* stream);
int bj_blake2s_leaves_chunked_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                                uint32_t elems_per_leaf, uint64_t* out, void* stream);
int bj_blake2s_nodes_d(const uint64_t* leaves, size_t n_leaves, uint32_t cap_size, uint64_t* nodes,
                       void* stream);
/* Column-range continuation (the column pipeline): the carried state is the 32-byte chaining
 * value h plus the byte count, which is 8 * cols_before (a multiple of 64).  state_in: NULL iff
 * cols_before == 0.  final_ == 0: n_cols a multiple of 8, out = chaining values (n_leaves x 4);
 * final_ != 0: out = digests, and n_cols > 0 when cols_before > 0 (the message's last block
 * must be in this range). */
int bj_blake2s_leaves_partial_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                                uint64_t cols_before, const uint64_t* state_in, uint64_t* out, int final_,
                                void* stream);
/* host seams (TreeHasher::hash_into_leaf / hash_into_node) */
int bj_blake2s_leaf_h(const uint64_t* elems, size_t n_elems, uint64_t* out4);
int bj_blake2s_node_h(const uint64_t* left4, const uint64_t* right4, uint64_t* out4);

/* ---------------------------------------------- Keccak256 tree hasher */
/* MerkleTreeWithCap<GoldilocksField, sha3::Keccak256>: the TreeHasher impl of
 * cs/oracle/mod.rs:247-313.  Leaf = Keccak256 (rate 136 bytes, domain byte 0x01) of the
 * canonical little-endian bytes of the leaf's elements; node = Keccak256(left || right).
 * Digests are 32 bytes as 4 little-endian u64 words.  Same arguments, layouts and
 * preconditions as the bj_merkle_* calls. */
int bj_keccak256_leaves_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                          uint64_t* leaves, void* stream);
int bj_keccak256_leaves_chunked_d(const uint64_t* src, uint32_t n_cols, size_t col_stride, size_t n_leaves,
                                  uint32_t elems_per_leaf, uint64_t* out, void* stream);
int bj_keccak256_nodes_d(const uint64_t* leaves, size_t n_leaves, uint32_t cap_size, uint64_t* nodes,
                         void* stream);
int bj_keccak256_leaf_h(const uint64_t* elems, size_t n_elems, uint64_t* out4);
int bj_keccak256_node_h(const uint64_t* left4, const uint64_t* right4, uint64_t* out4);

/* ------------------------------------------------------- whole commitment */

/* Witness commitment, the batched hot path (prover.rs:313-353): the LDE of every column at
 * D = 2^log_lde (used_lde_degree = max(fri_lde_factor, quotient_degree), prover.rs:313), then
 * MerkleTreeWithCap::construct over the first k = 2^log_commit_cosets cosets only
 * (source = subset_for_degree(fri_lde_factor), prover.rs:325-347, polynomial/lde.rs:298-308):
 * leaf L = coset * n + row < k * n, node levels to the cap.  log_commit_cosets <= log_lde; the
 * reference's own proof.json is D = 8 (quotient degree), k = 2 (fri_lde_factor).
 *   scratch  n_cols x n (monomials, as bj_lde_d)
 *   lde      n_cols x D x n, all D cosets (as bj_lde_d)
 *   leaves   k*n x 4;  nodes (k*n - cap_size) x 4, the cap being the last cap_size digests
 * All pointers device; cap additionally copied to cap_h (host, cap_size x 4) if non-NULL
 * (this synchronises the stream).  Requires power-of-two cap_size < k * n. */
int bj_lde_commit_d(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n,
                    uint32_t log_lde, uint32_t log_commit_cosets, uint32_t cap_size, uint64_t* scratch,
                    uint64_t* lde, uint64_t* leaves, uint64_t* nodes, uint64_t* cap_h, void* stream);

/* bj_lde_commit_d with flags (ABI 2.4): with BJ_LDE_KEEP_MONOMIALS scratch receives the
 * monomials (bj_lde_d's contract); without it scratch is workspace only, as
 * transform_raw_storages_to_lde drops them (utils.rs:270-403), and the middle LDE pass skips
 * their write-back.  bj_lde_commit_d == bj_lde_commit_ex_d(..., BJ_LDE_KEEP_MONOMIALS, ...).
 * Unknown flags: BJ_EINVAL. */
int bj_lde_commit_ex_d(const uint64_t* trace, uint32_t n_cols, size_t trace_stride, uint32_t log_n,
                       uint32_t log_lde, uint32_t log_commit_cosets, uint32_t cap_size, uint64_t* scratch,
                       uint64_t* lde, uint64_t* leaves, uint64_t* nodes, uint64_t* cap_h, uint32_t flags,
                       void* stream);

/* Host-buffer variant (drop-in for a Rust prover that owns host Vecs): the trace goes in,
 * bj_lde_commit_d's pipeline runs column chunk by column chunk, every output comes back (lde_h
 * n_cols x D x n, leaves_h k*n x 4, nodes_h, cap_h).  Any output pointer may be NULL to skip its
 * copy.  Device workspace comes from the library's own stream-ordered pool (the process's default
 * pool is not touched); pinned staging (3 x 64 MiB + 3 streams per set) comes from a per-device
 * pool of at most 4 sets shared by all calling threads.  PCIe-inclusive; never the headline. */
int bj_lde_commit_h(const uint64_t* trace_h, uint32_t n_cols, uint32_t log_n, uint32_t log_lde,
                    uint32_t log_commit_cosets, uint32_t cap_size, uint64_t* lde_h, uint64_t* leaves_h,
                    uint64_t* nodes_h, uint64_t* cap_h);

/* ------------------------------------- collective sharded commit (8(b), 8(e)) */
/* The whole G-rank witness commitment as one collective call per rank: one process (or
 * thread) per GPU, each calling bj_sharded_commit_d on its own column shard with its own
 * communicator.  It runs the column pipeline of DESIGN.md section 7 natively: local iNTTs,
 * per-chunk exchange on a high-priority stream (G <= D: all-gather of coefficients; G > D:
 * sender-side fold + all-to-all), this rank's coset/sub-coset LDE, the chained leaf sponge,
 * the subtree and the cap all-gather.  It replaces MerkleTreeWithCap::construct over
 * transform_raw_storages_to_lde (utils.rs:270-403, merkle_tree.rs:78-172, prover.rs:313-353)
 * with the leaf domain split over the ranks.
 *
 * Communicators (opaque bj_comm):
 *   bj_comm_rccl_unique_id  ncclGetUniqueId (128 bytes); rank 0 creates it and the caller
 *                           broadcasts it by its own means (torch.distributed, MPI, a file);
 *   bj_comm_init_rccl       ncclCommInitRank on the current device (collective, blocking);
 *   bj_comm_wrap_rccl       an ncclComm_t the caller already owns (not destroyed by us);
 *   bj_comm_local_*         in-process ranks that share one device (threads; device-to-device
 *                           copies through a host barrier): a rehearsal transport that runs the
 *                           same pipeline multi-rank on one GPU.  Not for performance.  If a rank
 *                           fails mid-collective the group is aborted: its peers return an error
 *                           instead of waiting, and the group must be destroyed;
 *   bj_comm_init_callback   the caller's own exchange (gloo, MPI, a test double), called for
 *                           every data exchange from the thread that called the collective.
 *                           kind BJ_XCHG_ALL_GATHER: recv (world x bytes) <- concat over ranks of
 *                           send (bytes); BJ_XCHG_ALL_TO_ALL: recv block p (bytes) <- block `rank`
 *                           of rank p's send (world x bytes).  host_staged != 0: send / recv are
 *                           host buffers (the library synchronises, copies out, calls, copies
 *                           back; stream is NULL).  host_staged == 0: device pointers, and the
 *                           exchange must be ordered on `stream`.  Returns 0 on success.
 * RCCL is resolved at run time (dlopen of librccl.so.1, reusing an already loaded copy), so the
 * library loads without it.  All ranks must call collectives in the same order. */
typedef struct bj_comm bj_comm;
#define BJ_XCHG_ALL_GATHER 0
#define BJ_XCHG_ALL_TO_ALL 1
typedef int (*bj_exchange_fn)(void* user, int kind, const void* send, void* recv, size_t bytes, void* stream);
int bj_comm_rccl_unique_id(uint8_t* id_out128);
int bj_comm_init_rccl(const uint8_t* id128, int world, int rank, bj_comm** out);
int bj_comm_wrap_rccl(void* nccl_comm, int world, int rank, bj_comm** out);
int bj_comm_local_group_create(int world, void** group_out);
int bj_comm_local_group_destroy(void* group);
int bj_comm_init_local(void* group, int rank, bj_comm** out);
int bj_comm_init_callback(int world, int rank, bj_exchange_fn exchange, void* user, int host_staged, bj_comm** out);
int bj_comm_destroy(bj_comm* comm);
/* What a communicator's transport sees (ABI 2.5; no reference counterpart: the reference has no
 * collectives).  kind: BJ_COMM_RCCL / BJ_COMM_LOCAL / BJ_COMM_CALLBACK; world, rank: as the
 * communicator was made; transport_count, transport_rank, device: RCCL's own ncclCommCount,
 * ncclCommUserRank and ncclCommCuDevice (the other transports: world, rank and the device current
 * when the communicator was made); pci_bus_id: hipDeviceGetPCIBusId of that device ("" when this
 * process cannot open it); host: gethostname.  128 bytes. */
#define BJ_COMM_RCCL 0
#define BJ_COMM_LOCAL 1
#define BJ_COMM_CALLBACK 2
#define BJ_COMM_INVALID (-1) /* bj_comm_check_world: the rank could not read its record; reserved[0] = its error */
typedef struct bj_comm_info_t {
    int32_t kind;
    int32_t world, rank;
    int32_t transport_count, transport_rank;
    int32_t device;
    char pci_bus_id[32];
    char host[64];
    int32_t reserved[2];
} bj_comm_info_t;
int bj_comm_info(bj_comm* comm, bj_comm_info_t* out);
/* Collective over `comm` (ordered on `stream`, as bj_comm_exchange_d): all-gathers every rank's
 * bj_comm_info_t into all_out[world] and checks the world the transport formed: slot p holds rank
 * p, and every rank's transport count and rank equal the communicator's world and rank; for RCCL
 * also that no two ranks drive one device (same host and PCI bus id, or same device number where
 * the bus id is unknown).  BJ_EINVAL naming the ranks otherwise (all_out is filled either way once
 * the gather ran).  The local and callback transports may share a device by design.  A rank whose
 * own bj_comm_info fails still enters the gather with a record of kind BJ_COMM_INVALID, so every
 * rank returns BJ_EINVAL; only a failed device allocation (128 * (world + 1) bytes) returns before
 * the gather, and then the peers wait in the transport's collective. */
int bj_comm_check_world(bj_comm* comm, bj_comm_info_t* all_out, void* stream);
/* One data exchange of bj_sharded_commit_d's kinds (BJ_XCHG_ALL_GATHER / BJ_XCHG_ALL_TO_ALL, the
 * layouts above) over `comm`, ordered on `stream`: the transport alone, so a caller can check its
 * communicator before a commit.  Collective; bytes per rank block, a multiple of 8.  An RCCL
 * communicator issues the RCCL call even at world 1 (ncclAllGather; grouped ncclSend/ncclRecv). */
int bj_comm_exchange_d(bj_comm* comm, int kind, const void* send, void* recv, size_t bytes, void* stream);
/* Phase timing of bj_sharded_commit_d on this communicator (no reference counterpart: the
 * reference logs its phase times, merkle_tree.rs:162-167, prover.rs:345).  on != 0: every later
 * call records HIP events on its compute stream around the inverse transforms (+ folds), the
 * LDE evaluations, the leaf hashing and the subtree + cap; waits for the exchange are outside
 * every interval.  Each call first sums the intervals of earlier calls that have completed and
 * frees their events, so the events held are those of calls still in flight.  bj_comm_phase_ms
 * waits for the recorded calls, writes the summed milliseconds {inverse, lde, leaves, nodes} to
 * ms_out[4] and their count to *calls_out, and starts a new sum.  The events cost a little time
 * on the compute stream: time production steps with timing off. */
int bj_comm_set_timing(bj_comm* comm, int on);
int bj_comm_phase_ms(bj_comm* comm, float* ms_out4, int* calls_out);

#define BJ_HASHER_POSEIDON2 0
#define BJ_HASHER_BLAKE2S 1
#define BJ_HASHER_KECCAK256 2

/* Which global trace columns rank `shard` of G = 2^log_shards holds, in the order of its
 * trace_shard rows: the column pipeline deals chunk k (G * c_k consecutive columns, u = 8 /
 * gcd(8, G), c = u, u, then 3/2 (G <= 4) or 2 (G >= 8) times the previous rounded down to u but
 * at least u more, capped at 32 rounded to u) as G runs of c_k; when n_cols / G
 * is not a multiple of u, or the hasher cannot be continued over column ranges (Keccak256),
 * rank P holds columns [P * n_cols / G, (P + 1) * n_cols / G).  cols_out: n_cols / G entries.
 * Host only (no device call). */
int bj_sharded_columns(uint32_t n_cols, uint32_t log_shards, uint32_t shard, int hasher, uint32_t* cols_out);

/* Rank P's part of the G-way commit (G = the communicator's world, a power of two; P its rank).
 * The LDE is at D = 2^log_lde, the tree over the first k = 2^log_commit_cosets cosets
 * (bj_lde_commit_d; prover.rs:313-347).  The committed domain of m_k = k * n leaves is cut into
 * G ranges of m = k * n / G; rank P owns leaf range [P * m, (P + 1) * m) and, so that the LDE
 * work stays balanced, the same range of every other block of k cosets: block j (cosets
 * [j*k, (j+1)*k), j < B = D / k) of the D-coset LDE is itself a k-coset LDE with an extra shift,
 * and rank P holds its part [P * m, (P + 1) * m).
 * trace_shard: n_cols / G columns of n = 2^log_n in bj_sharded_columns order at
 *              trace_shard + j * trace_stride (device, read only).
 * Outputs (device):
 *   lde    B x n_cols x m: block j, global column c at lde + (j * n_cols + c) * m; block 0 is the
 *          committed one, equal to lde_full[c][P*m .. (P+1)*m) of bj_lde_commit_d's flat
 *          coset * n + row index; block j to lde_full[c][j*k*n + P*m ..];
 *   leaves m x 4;
 *   nodes  (m - cap_local) x 4, the subtree levels, cap_local = max(1, cap_size / G);
 *   cap    cap_size x 4, the full gathered cap (identical on every rank).
 * Exchange: G <= D all-gather of the coefficients (8 n n_cols bytes in total); G > D the sender
 * folds its columns for every (block, rank) and all-to-alls deliver them (8 n D / G n_cols bytes
 * received per rank).  Requires n_cols % G == 0, log_lde >= 1, log_commit_cosets <= log_lde,
 * G <= k * n, G / k <= 64, power-of-two cap_size < k * n, m > cap_local.  Asynchronous on
 * `stream`; workspace comes from the library's stream-ordered pool. */
int bj_sharded_commit_d(bj_comm* comm, const uint64_t* trace_shard, size_t trace_stride, uint32_t n_cols,
                        uint32_t log_n, uint32_t log_lde, uint32_t log_commit_cosets, uint32_t cap_size,
                        int hasher, uint64_t* lde, uint64_t* leaves, uint64_t* nodes, uint64_t* cap, void* stream);

/* OracleQuery::construct (proof.rs:65-97) on a bj_sharded_commit_d commit: tree index idx < k * n
 * (flat leaf index coset * n + row of the committed cosets) of the global tree.  The owning rank
 * reads the row of every column and its subtree path; when cap_size < G the top levels over the
 * gathered subtree roots finish the path on every rank.  Collective: every rank passes its own
 * commit outputs and the same idx, and every rank receives, in host memory, leaf_elements
 * (n_cols), leaf_hash (4) and proof (depth x 4, depth = log2(k * n / cap_size),
 * MerkleTreeWithCap::get_proof order, merkle_tree.rs:462-480).  Synchronous. */
int bj_sharded_query_h(bj_comm* comm, const uint64_t* lde, const uint64_t* leaves, const uint64_t* nodes,
                       uint32_t n_cols, uint32_t log_n, uint32_t log_lde, uint32_t log_commit_cosets,
                       uint32_t cap_size, int hasher, uint64_t idx, uint64_t* leaf_elements_h,
                       uint64_t* leaf_hash_h, uint64_t* proof_h, void* stream);

/* ------------------------------------------------------------------- FRI */

/* One FRI fold by 2 of a GoldilocksExt2 codeword stored as base columns c0, c1 of n_src
 * bit-reversed values (fold_multiple, cs/implementations/fri/mod.rs:362-474, as driven by
 * interpolate_independent_cosets :476-585 and interpolate_flattened_cosets :587-682):
 *   dst_i = f(x) + f(-x) + alpha * (f(x) - f(-x)) * roots[i] * coset_inverse,  i < n_src / 2,
 * f(x) = (c0[2i], c1[2i]), f(-x) = (c0[2i+1], c1[2i+1]), alpha = (ch0, ch1), u^2 = 7.
 * roots: the INVERSED bit-reversed twiddles of the full FRI domain (bj_precompute_twiddles_d
 * with inverse = 1), indexed by the flat pair index.  Device pointers; outputs canonical.
 * c0 / c1 at 16-byte-aligned addresses load each (f(x), f(-x)) pair as one 16-byte load; any
 * other 8-byte-aligned address runs the same fold with 8-byte loads. */
int bj_fri_fold_d(const uint64_t* c0, const uint64_t* c1, size_t n_src, const uint64_t* roots,
                  uint64_t coset_inverse, uint64_t ch0, uint64_t ch1, uint64_t* dst_c0, uint64_t* dst_c1,
                  void* stream);

/* ------------------------------------------------------------- utility */

/* Batched field arithmetic through the device field layer (utility for parity tests of
 * the Goldilocks primitives, field/goldilocks/mod.rs:186-325): out[i] = canonical(a[i] op b[i]),
 * op 0 = mul, 1 = add, 2 = sub, 3 = a + b * 2^32 (a < 2^63, b < 2^63 with b >> 32 < 2^31),
 * 4 = canonical(a).  Device pointers. */
int bj_gl_op_d(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n, void* stream);

/* Bench/test input (not a reference entry point): column-major synthetic trace,
 * x = splitmix64(seed + (first_col + c) * n + r) reduced once mod p. */
int bj_fill_synthetic_d(uint64_t* dst, uint32_t n_cols, size_t col_stride, uint32_t log_n, uint64_t seed,
                        uint64_t first_col, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* BOOJUM_MI355X_H */
