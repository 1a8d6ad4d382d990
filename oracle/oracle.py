"""ctypes wrapper over oracle/liboracle.so -- CPU ORACLE, TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module.  The product (era-boojum_amd/boojum_amd) never imports it.

All arrays are numpy uint64; all outputs are canonical Goldilocks values.
See boojum_oracle.c for the reference file:line each function restates.
"""
import ctypes
import os

import numpy as np

P = 0xFFFFFFFF00000001
_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_u64p = ctypes.POINTER(ctypes.c_uint64)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle` "
                               "(or __graft_entry__.build())")
        L = ctypes.CDLL(path)
        u64, sz, u32, i = ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int
        for name in ("bjo_gl_add", "bjo_gl_sub", "bjo_gl_mul", "bjo_gl_pow"):
            getattr(L, name).restype = u64
            getattr(L, name).argtypes = [u64, u64]
        L.bjo_gl_inv.restype = u64
        L.bjo_gl_inv.argtypes = [u64]
        L.bjo_domain_generator.restype = u64
        L.bjo_domain_generator.argtypes = [u32]
        L.bjo_bitreverse_inplace.argtypes = [_u64p, sz]
        L.bjo_precompute_twiddles.argtypes = [u32, i, _u64p]
        L.bjo_distribute_powers.argtypes = [_u64p, sz, u64]
        L.bjo_fft_natural_to_bitreversed.argtypes = [_u64p, sz, u64, _u64p]
        L.bjo_ifft_natural_to_natural.argtypes = [_u64p, sz, u64, _u64p]
        L.bjo_lde_cosets.argtypes = [u32, u32, _u64p]
        L.bjo_lde.argtypes = [_u64p, u32, u32, u32, _u64p, i]
        L.bjo_poseidon2_permute_canonical.argtypes = [_u64p]
        L.bjo_hash_into_leaf.argtypes = [_u64p, sz, _u64p]
        L.bjo_hash_into_node.argtypes = [_u64p, _u64p, _u64p]
        L.bjo_merkle_construct.restype = i
        L.bjo_merkle_construct.argtypes = [_u64p, sz, u32, sz, u32, _u64p, _u64p, i]
        L.bjo_merkle_get_proof.argtypes = [_u64p, _u64p, sz, i, sz, _u64p, _u64p]
        L.bjo_verify_proof_over_cap.restype = i
        L.bjo_verify_proof_over_cap.argtypes = [_u64p, i, _u64p, _u64p, sz]
        L.bjo_lde_commit.restype = i
        L.bjo_lde_commit.argtypes = [_u64p, u32, u32, u32, u32, _u64p, _u64p, _u64p, _u64p, i]
        L.bjo_lde_commit_subset.restype = i
        L.bjo_lde_commit_subset.argtypes = [_u64p, u32, u32, u32, u32, u32, _u64p, _u64p, _u64p, _u64p, i]
        L.bjo_blake2s.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p]
        L.bjo_blake2s_leaf.argtypes = [_u64p, sz, _u64p]
        L.bjo_blake2s_node.argtypes = [_u64p, _u64p, _u64p]
        L.bjo_blake2s_leaf_partial.argtypes = [_u64p, _u64p, sz, u64, i, _u64p]
        L.bjo_keccak256.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, i]
        L.bjo_keccak_leaf.argtypes = [_u64p, sz, _u64p]
        L.bjo_keccak_node.argtypes = [_u64p, _u64p, _u64p]
        L.bjo_merkle_leaves_with.argtypes = [_u64p, sz, u32, sz, _u64p, i, i]
        L.bjo_avx512_available.restype = i
        L.bjo_avx512_available.argtypes = []
        L.bjo_lde_avx512.restype = i
        L.bjo_lde_avx512.argtypes = [_u64p, u32, u32, u32, _u64p, i]
        L.bjo_merkle_leaves_avx512.restype = i
        L.bjo_merkle_leaves_avx512.argtypes = [_u64p, sz, u32, sz, _u64p, i]
        L.bjo_merkle_nodes_with.restype = i
        L.bjo_merkle_nodes_with.argtypes = [_u64p, sz, u32, _u64p, i, i]
        L.bjo_merkle_construct_with.restype = i
        L.bjo_merkle_construct_with.argtypes = [_u64p, sz, u32, sz, u32, _u64p, _u64p, i, i]
        L.bjo_verify_proof_over_cap_with.restype = i
        L.bjo_verify_proof_over_cap_with.argtypes = [_u64p, i, _u64p, _u64p, sz, i]
        L.bjo_poseidon2_leaves_partial.restype = i
        L.bjo_poseidon2_leaves_partial.argtypes = [_u64p, sz, u32, sz, _u64p, _u64p, i, i]
        L.bjo_find_query_index.restype = ctypes.c_long
        L.bjo_find_query_index.argtypes = [_u64p, _u64p, i, _u64p, sz]
        _LIB = L
    return _LIB


def _p(a):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data_as(_u64p)


def _u64(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.uint64))


def gl_mul(a, b):
    return lib().bjo_gl_mul(a, b)


def gl_add(a, b):
    return lib().bjo_gl_add(a, b)


def gl_sub(a, b):
    return lib().bjo_gl_sub(a, b)


def gl_pow(a, e):
    return lib().bjo_gl_pow(a, e)


def gl_inv(a):
    return lib().bjo_gl_inv(a)


def domain_generator(log_n):
    return lib().bjo_domain_generator(log_n)


def precompute_twiddles(log_n, inverse=False):
    out = np.zeros(max(1, (1 << log_n) // 2), dtype=np.uint64)
    lib().bjo_precompute_twiddles(log_n, 1 if inverse else 0, _p(out))
    return out[: (1 << log_n) // 2]


def bitreverse(a):
    a = _u64(a).copy()
    lib().bjo_bitreverse_inplace(_p(a), a.size)
    return a


def distribute_powers(a, element):
    a = _u64(a).copy()
    lib().bjo_distribute_powers(_p(a), a.size, element)
    return a


def fft_natural_to_bitreversed(a, coset=1):
    a = _u64(a).copy()
    log_n = a.size.bit_length() - 1
    tw = precompute_twiddles(log_n, False) if a.size > 1 else np.zeros(1, np.uint64)
    tw = np.ascontiguousarray(tw if tw.size else np.zeros(1, np.uint64))
    lib().bjo_fft_natural_to_bitreversed(_p(a), a.size, coset, _p(tw))
    return a


def ifft_natural_to_natural(a, coset=1):
    a = _u64(a).copy()
    log_n = a.size.bit_length() - 1
    tw = precompute_twiddles(log_n, True) if a.size > 1 else np.zeros(1, np.uint64)
    tw = np.ascontiguousarray(tw if tw.size else np.zeros(1, np.uint64))
    lib().bjo_ifft_natural_to_natural(_p(a), a.size, coset, _p(tw))
    return a


def lde_cosets(log_n, log_d):
    out = np.zeros(1 << log_d, dtype=np.uint64)
    lib().bjo_lde_cosets(log_n, log_d, _p(out))
    return out


def lde(trace, log_d, threads=1):
    """trace: (C, n) uint64 -> (monomials (C, n), lde (C, D, n))"""
    tr = _u64(trace).copy()
    c, n = tr.shape
    log_n = n.bit_length() - 1
    out = np.zeros((c, 1 << log_d, n), dtype=np.uint64)
    lib().bjo_lde(_p(tr), c, log_n, log_d, _p(out), threads)
    return tr, out


def poseidon2_permutation(state):
    s = _u64(state).copy()
    assert s.size == 12
    lib().bjo_poseidon2_permute_canonical(_p(s))
    return s


def hash_into_leaf(elems):
    e = _u64(elems)
    if e.size == 0:
        e = np.zeros(1, np.uint64)
        n = 0
    else:
        n = e.size
    out = np.zeros(4, dtype=np.uint64)
    lib().bjo_hash_into_leaf(_p(e), n, _p(out))
    return out


def hash_into_node(left, right):
    l, r = _u64(left), _u64(right)
    out = np.zeros(4, dtype=np.uint64)
    lib().bjo_hash_into_node(_p(l), _p(r), _p(out))
    return out


HASHERS = {"poseidon2": 0, "blake2s": 1, "keccak256": 2}


def blake2s(data):
    """BLAKE2s-256 (RFC 7693) of a bytes object: the blake2 crate's Blake2s256."""
    data = bytes(data)
    out = ctypes.create_string_buffer(32)
    lib().bjo_blake2s(data, len(data), out)
    return out.raw


def blake2s_leaf(elems):
    """TreeHasher::hash_into_leaf for Blake2s256 (cs/oracle/mod.rs:203-215): the canonical
    little-endian bytes of each element.  Digest as 4 little-endian u64 words."""
    e = _u64(elems)
    n = e.size
    if n == 0:
        e = np.zeros(1, np.uint64)
    out = np.zeros(4, dtype=np.uint64)
    lib().bjo_blake2s_leaf(_p(e), n, _p(out))
    return out


def blake2s_leaf_partial(h_in, elems, before, final):
    """One leaf's Blake2s message continued over a column range (bjo_blake2s_leaf_partial)."""
    e = _u64(elems)
    n = e.size
    if n == 0:
        e = np.zeros(1, np.uint64)
    out = np.zeros(4, dtype=np.uint64)
    hp = None if h_in is None else _p(_u64(h_in))
    lib().bjo_blake2s_leaf_partial(hp, _p(e), n, before, 1 if final else 0, _p(out))
    return out


def blake2s_node(left, right):
    """TreeHasher::hash_into_node for Blake2s256 (cs/oracle/mod.rs:234-245)."""
    out = np.zeros(4, dtype=np.uint64)
    lib().bjo_blake2s_node(_p(_u64(left)), _p(_u64(right)), _p(out))
    return out


def keccak256(data, domain=0x01):
    """Keccak256 (domain 0x01, the sha3 crate's Keccak256) or SHA3-256 (domain 0x06) of bytes."""
    data = bytes(data)
    out = ctypes.create_string_buffer(32)
    lib().bjo_keccak256(data, len(data), out, domain)
    return out.raw


def keccak_leaf(elems):
    """TreeHasher::hash_into_leaf for Keccak256 (cs/oracle/mod.rs:271-283)."""
    e = _u64(elems)
    n = e.size
    if n == 0:
        e = np.zeros(1, np.uint64)
    out = np.zeros(4, dtype=np.uint64)
    lib().bjo_keccak_leaf(_p(e), n, _p(out))
    return out


def keccak_node(left, right):
    """TreeHasher::hash_into_node for Keccak256 (cs/oracle/mod.rs:302-313)."""
    out = np.zeros(4, dtype=np.uint64)
    lib().bjo_keccak_node(_p(_u64(left)), _p(_u64(right)), _p(out))
    return out


def num_node_levels(n_leaves, cap_size):
    return (n_leaves.bit_length() - 1) - (cap_size.bit_length() - 1)


def merkle_construct(lde_flat, cap_size, threads=1, hasher="poseidon2"):
    """lde_flat: (C, n_leaves) uint64 (column c's values over the flat leaf index).
    Returns (leaves (n_leaves, 4), nodes (sum of levels, 4), levels, cap (cap_size, 4)).
    hasher: "poseidon2" (GoldilocksPoseidon2Sponge) or "blake2s" (Blake2s256, digests as
    4 little-endian u64 words)."""
    src = _u64(lde_flat)
    c, nl = src.shape
    levels = num_node_levels(nl, cap_size)
    leaves = np.zeros((nl, 4), dtype=np.uint64)
    n_nodes = nl - cap_size if levels > 0 else 0
    nodes = np.zeros((max(n_nodes, 1), 4), dtype=np.uint64)
    got = lib().bjo_merkle_construct_with(_p(src), nl, c, nl, cap_size, _p(leaves), _p(nodes), threads,
                                          HASHERS[hasher])
    assert got == levels
    cap = nodes[n_nodes - cap_size: n_nodes].copy() if levels > 0 else leaves.copy()
    return leaves, nodes[:n_nodes], levels, cap


def lde_avx512(trace, log_d, threads=1):
    """The CPU baseline's AVX-512 LDE (oracle/baseline_avx512.c): same values as lde().  None when
    the host has no AVX-512."""
    tr = _u64(trace).copy()
    c, n = tr.shape
    log_n = n.bit_length() - 1
    out = np.zeros((c, 1 << log_d, n), dtype=np.uint64)
    if lib().bjo_lde_avx512(_p(tr), c, log_n, log_d, _p(out), threads) != 0:
        return None
    return tr, out


def avx512_available():
    return bool(lib().bjo_avx512_available())


def merkle_leaves_avx512(lde_flat, threads=1):
    """The CPU baseline's 8-leaf AVX-512 Poseidon2 leaf hashing (oracle/baseline_avx512.c):
    same leaves as merkle_construct's.  None when the host has no AVX-512."""
    src = _u64(lde_flat)
    c, nl = src.shape
    leaves = np.zeros((nl, 4), dtype=np.uint64)
    if lib().bjo_merkle_leaves_avx512(_p(src), nl, c, nl, _p(leaves), threads) != 0:
        return None
    return leaves


def merkle_construct_timed(lde_flat, cap_size, threads=1, hasher="poseidon2", simd=False):
    """merkle_construct with the reference's own phase split (merkle_tree.rs:162-167 leaf timing,
    :438-442 node timing): returns (leaves, nodes, levels, cap, {"leaves": s, "nodes": s}).
    simd: hash the leaves with the AVX-512 baseline path (Poseidon2, host permitting)."""
    import time
    src = _u64(lde_flat)
    c, nl = src.shape
    levels = num_node_levels(nl, cap_size)
    leaves = np.zeros((nl, 4), dtype=np.uint64)
    n_nodes = nl - cap_size if levels > 0 else 0
    nodes = np.zeros((max(n_nodes, 1), 4), dtype=np.uint64)
    t0 = time.perf_counter()
    if not (simd and hasher == "poseidon2" and nl % 8 == 0 and
            lib().bjo_merkle_leaves_avx512(_p(src), nl, c, nl, _p(leaves), threads) == 0):
        lib().bjo_merkle_leaves_with(_p(src), nl, c, nl, _p(leaves), threads, HASHERS[hasher])
    t1 = time.perf_counter()
    got = lib().bjo_merkle_nodes_with(_p(leaves), nl, cap_size, _p(nodes), threads, HASHERS[hasher])
    t2 = time.perf_counter()
    assert got == levels
    cap = nodes[n_nodes - cap_size: n_nodes].copy() if levels > 0 else leaves.copy()
    return leaves, nodes[:n_nodes], levels, cap, {"leaves": t1 - t0, "nodes": t2 - t1}


def merkle_construct_by_chunking(sources_flat, elements_per_leaf, cap_size, threads=1, hasher="poseidon2"):
    """MerkleTreeWithCap::construct_by_chunking / construct_by_chunking_from_flat_sources
    (merkle_tree.rs:176-386): leaf L hashes, for each source c in order, the E consecutive
    elements sources[c][L*E .. (L+1)*E).  Restated as an ordinary tree over C*E rows, row
    c*E + t holding sources[c][L*E + t] for leaf L."""
    src = _u64(sources_flat)
    c, total = src.shape
    e = elements_per_leaf
    nl = total // e
    rows = np.ascontiguousarray(src.reshape(c, nl, e).transpose(0, 2, 1).reshape(c * e, nl))
    return merkle_construct(rows, cap_size, threads=threads, hasher=hasher)


def merkle_get_proof(leaves, nodes, levels, idx):
    nl = leaves.shape[0]
    leaf = np.zeros(4, dtype=np.uint64)
    path = np.zeros((max(levels, 1), 4), dtype=np.uint64)
    nd = nodes if nodes.size else np.zeros((1, 4), np.uint64)
    lib().bjo_merkle_get_proof(_p(_u64(leaves)), _p(_u64(nd)), nl, levels, idx, _p(leaf), _p(path))
    return leaf, path[:levels]


def verify_proof_over_cap(path, cap, leaf, idx, hasher="poseidon2"):
    path = _u64(path).reshape(-1, 4)
    pp = path if path.size else np.zeros((1, 4), np.uint64)
    return bool(lib().bjo_verify_proof_over_cap_with(_p(pp), path.shape[0], _p(_u64(cap)), _p(_u64(leaf)), idx,
                                                     HASHERS[hasher]))


def lde_commit(trace, log_d, cap_size, threads=1, log_k=None, in_place=False):
    """Full witness commit (oracle, prover.rs:313-347): LDE at 2^log_d, tree over the first
    2^log_k cosets (subset_for_degree; default all).  Returns dict with monomials, lde (C, D, n),
    leaves (k n, 4), nodes, cap.  in_place: the trace array itself becomes the monomials."""
    tr = _u64(trace) if in_place else _u64(trace).copy()
    c, n = tr.shape
    log_n = n.bit_length() - 1
    log_k = log_d if log_k is None else log_k
    nl = n << log_k
    lde_out = np.zeros((c, 1 << log_d, n), dtype=np.uint64)
    leaves = np.zeros((nl, 4), dtype=np.uint64)
    n_nodes = nl - cap_size
    nodes = np.zeros((max(n_nodes, 1), 4), dtype=np.uint64)
    cap = np.zeros((cap_size, 4), dtype=np.uint64)
    lib().bjo_lde_commit_subset(_p(tr), c, log_n, log_d, log_k, cap_size, _p(lde_out), _p(leaves), _p(nodes),
                                _p(cap), threads)
    return {"monomials": tr, "lde": lde_out, "leaves": leaves, "nodes": nodes[:n_nodes], "cap": cap}


def poseidon2_leaves_partial(lde_cols, cap_in, final, threads=1):
    """Leaf sponges over a column range (bjo_poseidon2_leaves_partial): lde_cols (C, N) the
    range's columns in leaf order, cap_in (N, 4) the capacity words after the previous columns
    or None.  final: (N, 4) digests; else (N, 4) capacity words to carry on."""
    src = _u64(lde_cols)
    c, nl = src.shape
    out = np.zeros((nl, 4), dtype=np.uint64)
    cin = None if cap_in is None else _u64(cap_in)
    rc = lib().bjo_poseidon2_leaves_partial(_p(src), nl, c, nl, None if cin is None else _p(cin), _p(out),
                                            1 if final else 0, threads)
    if rc != 0:
        raise ValueError("a non-final column range must be a multiple of 8 columns")
    return out


def merkle_nodes(leaves, cap_size, threads=1, hasher="poseidon2"):
    """Node levels over given leaf digests (bjo_merkle_nodes_with); returns (nodes, cap)."""
    lv = _u64(leaves).reshape(-1, 4)
    nl = lv.shape[0]
    nodes = np.zeros((max(nl - cap_size, 1), 4), dtype=np.uint64)
    levels = lib().bjo_merkle_nodes_with(_p(lv), nl, cap_size, _p(nodes), threads, HASHERS[hasher])
    cap = lv[:cap_size] if levels == 0 else nodes[nl - 2 * cap_size:nl - cap_size]
    return nodes[:nl - cap_size], cap.copy()


def find_query_index(leaf, path, cap):
    path = _u64(path).reshape(-1, 4)
    cap = _u64(cap).reshape(-1, 4)
    return lib().bjo_find_query_index(_p(_u64(leaf)), _p(path), path.shape[0], _p(cap), cap.shape[0])


# ----------------------------------------------------------- pure-python helpers

def splitmix64(x):
    """splitmix64 finaliser on a uint64 numpy array (synthetic inputs)."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def synthetic_trace(n_cols, log_n, seed=42, col_offset=0):
    """Column-major canonical trace: x = splitmix64(seed + c*n + r), reduced once."""
    n = 1 << log_n
    idx = (np.arange(col_offset, col_offset + n_cols, dtype=np.uint64)[:, None] * np.uint64(n)
           + np.arange(n, dtype=np.uint64)[None, :] + np.uint64(seed))
    x = splitmix64(idx)
    return np.where(x >= np.uint64(P), x - np.uint64(P), x)


def naive_coset_lde_column(col, log_d):
    """Closed form: LDE[L] = p(7 * w_{nD}^{bitrev_{log nD}(L)}), p the
    interpolant of `col` over <w_n>.  Pure python, tiny n only (reference test
    methodology fft/mod.rs:1591-1634)."""
    n = len(col)
    log_n = n.bit_length() - 1
    mono = [int(v) for v in ifft_natural_to_natural(col)]
    nd = n << log_d
    bits = log_n + log_d
    g = domain_generator(bits)
    out = []
    for L in range(nd):
        r = int(format(L, "0%db" % bits)[::-1], 2) if bits else 0
        x = (7 * pow(g, r, P)) % P
        acc = 0
        for c in reversed(mono):
            acc = (acc * x + c) % P
        out.append(acc)
    return out


def fri_fold(c0, c1, roots, coset_inverse, challenge):
    """fold_multiple (cs/implementations/fri/mod.rs:362-474) in Python ints (test sizes only):
    out_i = f(x) + f(-x) + alpha * (f(x) - f(-x)) * roots[i] * coset_inverse over GoldilocksExt2
    (u^2 = 7, field/traits/field.rs:407-424), f(x) at 2i, f(-x) at 2i + 1."""
    ch0, ch1 = int(challenge[0]) % P, int(challenge[1]) % P
    n = len(c0) // 2
    d0 = np.zeros(n, dtype=np.uint64)
    d1 = np.zeros(n, dtype=np.uint64)
    for i in range(n):
        x0, mx0, x1, mx1 = int(c0[2 * i]), int(c0[2 * i + 1]), int(c1[2 * i]), int(c1[2 * i + 1])
        r = int(roots[i]) * coset_inverse % P
        a0 = (x0 - mx0) * r % P
        a1 = (x1 - mx1) * r % P
        e0 = (a0 * ch0 + 7 * a1 * ch1) % P
        e1 = (a0 * ch1 + a1 * ch0) % P
        d0[i] = (e0 + x0 + mx0) % P
        d1[i] = (e1 + x1 + mx1) % P
    return d0, d1
