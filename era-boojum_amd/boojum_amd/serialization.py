"""MemcopySerializable wire format for handing LDEs and trees back to a Rust prover.

Restates the reference's byte layout (cs/implementations/fast_serialization.rs), all
integers little-endian u64:
* Vec<F> / GenericPolynomial (polynomial/mod.rs:101-120, fast_serialization.rs:142-207):
  length in base elements, then the elements' u64 words. Goldilocks has
  CAN_CAST_VECTOR_TO_U64_LE_VECTOR = true (field/goldilocks/mod.rs:539), so the words are the
  in-memory representation.
* ArcGenericLdeStorage (polynomial/lde.rs:174-217): the number of cosets, then one Vec<F>
  per coset (each bit-reversed, in the [coset][row] order of the LDE).
* Vec<[F; 4]> digests (fast_serialization.rs:269-341): length in base elements (4 per
  digest), then the words.
* Vec<[u8; 32]> digests of the byte-output tree hashers (Blake2s256 / Keccak256,
  H::Output = [u8; 32]; fast_serialization.rs:343-358): length in BYTES (32 per digest), then
  the raw bytes.  This library keeps such a digest as 4 little-endian u64 words, whose bytes
  are exactly the digest's bytes in order.
* MerkleTreeWithCap (merkle_tree.rs:36-73): cap_size, the leaf hashes as Vec<H::Output>, then
  write_vec_into_buffer of node_hashes_enumerated_from_leafs: the number of levels, then each
  level as Vec<H::Output> (fast_serialization.rs:17-47).
Every value this library writes is canonical. The reference writes its in-memory words, which
may be non-canonical representatives of the same elements; readers compare canonically
(goldilocks/mod.rs:257-261).
"""
import struct

import numpy as np
import torch

from .field import to_host

_U64 = struct.Struct("<Q")


def _write_u64(f, v):
    f.write(_U64.pack(int(v)))


def _read_u64(f):
    b = f.read(8)
    if len(b) != 8:
        raise EOFError("truncated MemcopySerializable stream")
    return _U64.unpack(b)[0]


def _write_words(f, arr):
    a = np.ascontiguousarray(np.asarray(arr, dtype=np.uint64))
    _write_u64(f, a.size)
    f.write(a.astype("<u8", copy=False).tobytes())


def _read_words(f):
    n = _read_u64(f)
    b = f.read(8 * n)
    if len(b) != 8 * n:
        raise EOFError("truncated MemcopySerializable stream")
    return np.frombuffer(b, dtype="<u8").astype(np.uint64)


def _host(t):
    return to_host(t) if isinstance(t, torch.Tensor) else np.asarray(t, dtype=np.uint64)


def write_lde_storage(f, column_lde):
    """One column's ArcGenericLdeStorage: column_lde is (D, n) (device or host)."""
    cos = _host(column_lde)
    _write_u64(f, cos.shape[0])
    for c in cos:
        _write_words(f, c)


def read_lde_storage(f):
    """-> numpy (D, n)."""
    d = _read_u64(f)
    if d & (d - 1) or d == 0:
        raise ValueError("coset count must be a power of two (lde.rs:196)")
    cos = [_read_words(f) for _ in range(d)]
    return np.stack(cos)


# tree hashers whose digest (H::Output) is [u8; 32] rather than [F; 4]
BYTE_HASHERS = ("blake2s", "keccak256")


def _check_hasher(hasher):
    if hasher not in ("poseidon2",) + BYTE_HASHERS:
        raise ValueError("unknown tree hasher %r" % (hasher,))
    return hasher in BYTE_HASHERS


def write_digests(f, digests, hasher="poseidon2"):
    """Vec<H::Output>: [F; 4] digests as Vec<[F; 4]> (length in field elements), [u8; 32]
    digests as Vec<[u8; 32]> (length in bytes, fast_serialization.rs:343-358)."""
    words = np.ascontiguousarray(_host(digests).reshape(-1), dtype=np.uint64)
    if not _check_hasher(hasher):
        _write_words(f, words)
        return
    _write_u64(f, 8 * words.size)
    f.write(words.astype("<u8", copy=False).tobytes())


def read_digests(f, hasher="poseidon2"):
    if not _check_hasher(hasher):
        w = _read_words(f)
        if w.size % 4:
            raise ValueError("digest vector length must be a multiple of 4")
        return w.reshape(-1, 4)
    nbytes = _read_u64(f)
    if nbytes % 32:
        raise ValueError("byte-digest vector length must be a multiple of 32")
    b = f.read(nbytes)
    if len(b) != nbytes:
        raise EOFError("truncated MemcopySerializable stream")
    return np.frombuffer(b, dtype="<u8").astype(np.uint64).reshape(-1, 4)


def write_merkle_tree(f, tree):
    """MerkleTreeWithCap::write_into_buffer for a boojum_amd.merkle.MerkleTreeWithCap (its
    digests written per its tree hasher's H::Output)."""
    hasher = getattr(tree, "hasher", "poseidon2")
    _write_u64(f, tree.cap_size)
    write_digests(f, tree.leaf_hashes, hasher)
    levels = tree.num_levels()
    _write_u64(f, levels)
    for lvl in range(1, levels + 1):
        write_digests(f, tree.level(lvl), hasher)


def read_merkle_tree(f, hasher="poseidon2"):
    """-> (cap_size, leaf_hashes (N, 4), [level_1, ..., level_k]) as numpy."""
    cap_size = _read_u64(f)
    leaves = read_digests(f, hasher)
    n = _read_u64(f)
    levels = [read_digests(f, hasher) for _ in range(n)]
    return cap_size, leaves, levels


# ------------------------------------------------------------- serde JSON (proof format)
# The prover's Proof is serde-serialised (cs/implementations/proof.rs:118-160); the parts this
# path produces are caps (MerkleTreeCap = Vec<[F; 4]>) and OracleQuery {leaf_elements: Vec<F>,
# proof: Vec<[F; 4]>} (proof.rs:48-63).  GoldilocksField serialises as its u64 (canonical here),
# so proof.json holds plain integers: a cap is [[u64; 4], ...], a query
# {"leaf_elements": [...], "proof": [[u64; 4], ...]}.

def _canon_list(a):
    a = _host(a).astype(np.uint64)
    p = np.uint64(0xFFFFFFFF00000001)
    a = np.where(a >= p, a - p, a)
    return a.tolist()


def _digests_to_json(d, hasher):
    """[F; 4] digests as canonical u64 lists; [u8; 32] digests as serde writes a byte array:
    32 ints each, the raw bytes (no canonicalisation: they are not field elements)."""
    d = np.ascontiguousarray(np.asarray(_host(d), dtype=np.uint64).reshape(-1, 4))
    if not _check_hasher(hasher):
        return _canon_list(d)
    return d.astype("<u8", copy=False).view(np.uint8).reshape(-1, 32).astype(int).tolist()


def _digests_from_json(obj, hasher):
    a = np.asarray(obj, dtype=np.uint64)
    if not _check_hasher(hasher):
        if a.ndim != 2 or a.shape[1] != 4:
            raise ValueError("a [F; 4] digest list is a list of 4-element lists")
        return a
    if a.ndim != 2 or a.shape[1] != 32 or (a > 255).any():
        raise ValueError("a [u8; 32] digest list is a list of 32-byte lists")
    return np.ascontiguousarray(a.astype(np.uint8)).view("<u8").astype(np.uint64).reshape(-1, 4)


def cap_to_json(cap, hasher="poseidon2"):
    """MerkleTreeCap -> the serde JSON of Vec<H::Output> (as in proof.json's *_oracle_cap for
    Poseidon2: 4-lists of canonical ints)."""
    return _digests_to_json(cap, hasher)


def cap_from_json(obj, hasher="poseidon2"):
    return _digests_from_json(obj, hasher)


def oracle_query_to_json(leaf_elements, proof, hasher="poseidon2"):
    """OracleQuery -> {"leaf_elements": [...], "proof": [...]} (serde field order); the leaf
    elements are field elements (canonical), the proof is Vec<H::Output>."""
    return {"leaf_elements": _canon_list(np.asarray(_host(leaf_elements)).reshape(-1)),
            "proof": _digests_to_json(proof, hasher)}


def oracle_query_from_json(obj, hasher="poseidon2"):
    """-> (leaf_elements (k,), proof (depth, 4)) as numpy uint64."""
    leaf = np.asarray(obj["leaf_elements"], dtype=np.uint64).reshape(-1)
    return leaf, _digests_from_json(obj["proof"], hasher)


def dumps(obj):
    """serde_json::to_string layout: no whitespace."""
    import json
    return json.dumps(obj, separators=(",", ":"))
