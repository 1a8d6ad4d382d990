"""MerkleTreeWithCap / TreeHasher over the Poseidon2 Overwrite sponge, Blake2s256 or Keccak256.

Mirrors cs/oracle/merkle_tree.rs (construct :78-172, continue_from_leaf_hashes
:388-449, get_cap :451-460, get_proof :462-480, verify_proof_over_cap :482-504) and the
TreeHasher impls for GoldilocksPoseidon2Sponge<AbsorptionModeOverwrite>
(cs/oracle/mod.rs:114-175; digests [u64; 4], canonical) and blake2::Blake2s256
(:179-245) and sha3::Keccak256 (:247-313), whose digests [u8; 32] are held as 4 little-endian
u64 words.  `hasher` selects one: "poseidon2" (the default, the recursive-mode tree),
"blake2s" (the non-recursive one) or "keccak256".

Device layout: leaf_hashes (n_leaves, 4); node levels concatenated from the leaves up
to the cap, (n_leaves - cap_size, 4) -- the reference's node_hashes_enumerated_from_leafs
as one buffer (level l starts at sum_{i<l} n_leaves / 2^(i+1)).
"""
import ctypes

import numpy as np
import torch

from ._lib import call
from .field import as_u64_host, stream_of, to_host

_u64p = ctypes.POINTER(ctypes.c_uint64)


def _hp(a):
    return a.ctypes.data_as(_u64p)


class Poseidon2Sponge:
    """TreeHasher<GoldilocksField> for GoldilocksPoseidon2Sponge<AbsorptionModeOverwrite>
    (host-call forms; the batched device forms are the tree kernels)."""

    @staticmethod
    def hash_into_leaf(elements):
        e = as_u64_host(elements)
        out = np.zeros(4, dtype=np.uint64)
        call("bj_hash_into_leaf_h", _hp(e) if e.size else None, e.size, _hp(out))
        return out

    @staticmethod
    def hash_into_node(left, right, depth=0):
        out = np.zeros(4, dtype=np.uint64)
        call("bj_hash_into_node_h", _hp(as_u64_host(left)), _hp(as_u64_host(right)), _hp(out))
        return out

    @staticmethod
    def poseidon2_permutation(state):
        s = as_u64_host(state).copy()
        if s.size != 12:
            raise ValueError("state must have 12 elements")
        call("bj_poseidon2_permute_h", _hp(s))
        return s


class Blake2s256:
    """TreeHasher<GoldilocksField> for blake2::Blake2s256 (host-call forms). Digests are 32
    bytes as 4 little-endian u64 words (`digest_bytes` gives the bytes)."""

    @staticmethod
    def hash_into_leaf(elements):
        e = as_u64_host(elements)
        out = np.zeros(4, dtype=np.uint64)
        call("bj_blake2s_leaf_h", _hp(e) if e.size else None, e.size, _hp(out))
        return out

    @staticmethod
    def hash_into_node(left, right, depth=0):
        out = np.zeros(4, dtype=np.uint64)
        call("bj_blake2s_node_h", _hp(as_u64_host(left)), _hp(as_u64_host(right)), _hp(out))
        return out

    @staticmethod
    def digest_bytes(words):
        return np.asarray(words, dtype=np.uint64).astype("<u8").tobytes()


class Keccak256:
    """TreeHasher<GoldilocksField> for sha3::Keccak256 (host-call forms), cs/oracle/mod.rs:247-313.
    Digests are 32 bytes as 4 little-endian u64 words."""

    @staticmethod
    def hash_into_leaf(elements):
        e = as_u64_host(elements)
        out = np.zeros(4, dtype=np.uint64)
        call("bj_keccak256_leaf_h", _hp(e) if e.size else None, e.size, _hp(out))
        return out

    @staticmethod
    def hash_into_node(left, right, depth=0):
        out = np.zeros(4, dtype=np.uint64)
        call("bj_keccak256_node_h", _hp(as_u64_host(left)), _hp(as_u64_host(right)), _hp(out))
        return out

    digest_bytes = Blake2s256.digest_bytes


# hasher name -> (host TreeHasher, leaves, chunked leaves, nodes entry points)
HASHERS = {
    "poseidon2": (Poseidon2Sponge, "bj_merkle_leaves_d", "bj_merkle_leaves_chunked_d", "bj_merkle_nodes_d"),
    "blake2s": (Blake2s256, "bj_blake2s_leaves_d", "bj_blake2s_leaves_chunked_d", "bj_blake2s_nodes_d"),
    "keccak256": (Keccak256, "bj_keccak256_leaves_d", "bj_keccak256_leaves_chunked_d", "bj_keccak256_nodes_d"),
}


def _hasher(name):
    if name not in HASHERS:
        raise ValueError("unknown tree hasher %r (expected one of %s)" % (name, sorted(HASHERS)))
    return HASHERS[name]


def _log2(n):
    if n <= 0 or n & (n - 1):
        raise ValueError("size must be a power of two, got %d" % n)
    return n.bit_length() - 1


def _leaf_sources(leafs_sources, num_cosets=None):
    """-> (tensor ptr base view, n_cols, col_stride, n_leaves).  Accepts a (C, D, n)
    LDE tensor (optionally only its first `num_cosets` cosets, as
    subset_for_degree, prover.rs:325-343) or a (C, L) tensor of flat leaf-domain rows."""
    t = leafs_sources
    if t.dim() == 3:
        c, d, n = t.shape
        k = d if num_cosets is None else num_cosets
        if k > d or k < 1:
            raise ValueError("num_cosets out of range")
        if t.stride(2) != 1 or t.stride(1) != n:
            raise ValueError("LDE tensor must be (C, D, n) with contiguous cosets")
        return t, c, t.stride(0), k * n
    if t.dim() == 2:
        if t.stride(1) != 1:
            raise ValueError("rows must be contiguous")
        c, L = t.shape
        return t, c, (t.stride(0) if c > 1 else L), L
    raise ValueError("expected (C, D, n) or (C, L) tensor")


class MerkleTreeWithCap:
    def __init__(self, cap_size, leaf_hashes, nodes, hasher="poseidon2"):
        _hasher(hasher)
        self.cap_size = cap_size
        self.leaf_hashes = leaf_hashes            # (n_leaves, 4) int64 CUDA tensor
        self.nodes = nodes                        # (n_leaves - cap_size, 4)
        self.hasher = hasher

    @classmethod
    def construct(cls, leafs_sources, cap_size, num_cosets=None, leaf_out=None, node_out=None, hasher="poseidon2"):
        _, f_leaves, _, f_nodes = _hasher(hasher)
        src, c, stride, nl = _leaf_sources(leafs_sources, num_cosets)
        _log2(nl)
        _log2(cap_size)
        if nl <= cap_size:
            raise ValueError("tree size must exceed cap size (merkle_tree.rs:97)")
        dev = src.device
        leaves = leaf_out if leaf_out is not None else torch.empty((nl, 4), dtype=torch.int64, device=dev)
        nodes = node_out if node_out is not None else torch.empty((nl - cap_size, 4), dtype=torch.int64, device=dev)
        st = stream_of(src)
        call(f_leaves, src.data_ptr(), c, stride, nl, leaves.data_ptr(), st)
        call(f_nodes, leaves.data_ptr(), nl, cap_size, nodes.data_ptr(), st)
        return cls(cap_size, leaves, nodes, hasher)

    @classmethod
    def construct_by_chunking(cls, leafs_sources, elements_to_take_per_leaf, cap_size, hasher="poseidon2"):
        """merkle_tree.rs:176-306 (the FRI base oracle, fri/mod.rs:179-187): leaf j of the flat
        tree hashes, for each source in order, elements [j*E, (j+1)*E) of its flat LDE (cosets
        in order). leafs_sources: (C, D, n) LDE tensor or (C, L) flat rows."""
        src, c, stride, total = _leaf_sources(leafs_sources)
        e = elements_to_take_per_leaf
        _log2(e)
        _log2(cap_size)
        if total % e:
            raise ValueError("source length must be a multiple of elements_to_take_per_leaf")
        nl = total // e
        if leafs_sources.dim() == 3 and leafs_sources.shape[2] % e:
            raise ValueError("each coset must hold whole leaves (merkle_tree.rs:197-198)")
        if nl <= cap_size:
            raise ValueError("tree size must exceed cap size (merkle_tree.rs:207)")
        return cls._chunked(src, c, stride, nl, e, cap_size, hasher)

    @classmethod
    def construct_by_chunking_from_flat_sources(cls, leafs_sources, elements_to_take_per_leaf, cap_size,
                                                hasher="poseidon2"):
        """merkle_tree.rs:308-386 (FRI intermediate oracles, fri/mod.rs:258-266): as
        construct_by_chunking over flat (C, N) sources; tree_size == cap_size is allowed (the
        cap is then the leaf layer)."""
        src, c, stride, total = _leaf_sources(leafs_sources)
        e = elements_to_take_per_leaf
        _log2(e)
        _log2(cap_size)
        if total % e:
            raise ValueError("poly size must be a multiple of elements_to_take_per_leaf")
        nl = total // e
        if nl < cap_size:
            raise ValueError("trying to make tree of size %d with cap %d" % (nl, cap_size))
        return cls._chunked(src, c, stride, nl, e, cap_size, hasher)

    @classmethod
    def _chunked(cls, src, c, stride, nl, e, cap_size, hasher):
        _, _, f_chunked, f_nodes = _hasher(hasher)
        _log2(nl)
        dev = src.device
        leaves = torch.empty((nl, 4), dtype=torch.int64, device=dev)
        nodes = torch.empty((nl - cap_size, 4), dtype=torch.int64, device=dev)
        st = stream_of(src)
        call(f_chunked, src.data_ptr(), c, stride, nl, e, leaves.data_ptr(), st)
        if nl > cap_size:
            call(f_nodes, leaves.data_ptr(), nl, cap_size, nodes.data_ptr(), st)
        return cls(cap_size, leaves, nodes, hasher)

    @property
    def n_leaves(self):
        return self.leaf_hashes.shape[0]

    def num_levels(self):
        return _log2(self.n_leaves) - _log2(self.cap_size)

    def level(self, l):
        """Node level l (1 = parents of the leaves), as a device tensor view."""
        if l == 0:
            return self.leaf_hashes
        off, ln = 0, self.n_leaves
        for _ in range(l - 1):
            ln //= 2
            off += ln
        return self.nodes[off: off + ln // 2]

    def get_cap(self):
        """merkle_tree.rs:451-460 -> numpy (cap_size, 4) canonical."""
        if self.n_leaves == self.cap_size:
            return to_host(self.leaf_hashes)
        return to_host(self.nodes[-self.cap_size:])

    def get_proof(self, idx):
        """merkle_tree.rs:462-480 -> (leaf_hash (4,), path (depth, 4))."""
        depth = self.num_levels()
        leaf = to_host(self.leaf_hashes[idx])
        path = []
        for i in range(depth):
            path.append(to_host(self.level(i)[idx ^ 1]))
            idx >>= 1
        return leaf, np.array(path, dtype=np.uint64).reshape(depth, 4)

    @staticmethod
    def verify_proof_over_cap(proof, cap, leaf_hash, idx, hasher="poseidon2"):
        """merkle_tree.rs:482-504 (host; one node hash per level through the library)."""
        H = _hasher(hasher)[0]
        cur = as_u64_host(leaf_hash)
        for el in np.asarray(proof, dtype=np.uint64).reshape(-1, 4):
            if idx & 1 == 0:
                cur = H.hash_into_node(cur, el)
            else:
                cur = H.hash_into_node(el, cur)
            idx >>= 1
        cap = np.asarray(cap, dtype=np.uint64).reshape(-1, 4)
        return bool(np.array_equal(cap[idx], cur))
