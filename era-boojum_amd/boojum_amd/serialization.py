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
* MerkleTreeWithCap (merkle_tree.rs:36-73): cap_size, the leaf hashes as Vec<[F; 4]>, then
  write_vec_into_buffer of node_hashes_enumerated_from_leafs: the number of levels, then each
  level as Vec<[F; 4]> (fast_serialization.rs:17-47).
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


def write_digests(f, digests):
    _write_words(f, _host(digests).reshape(-1))


def read_digests(f):
    w = _read_words(f)
    if w.size % 4:
        raise ValueError("digest vector length must be a multiple of 4")
    return w.reshape(-1, 4)


def write_merkle_tree(f, tree):
    """MerkleTreeWithCap::write_into_buffer for a boojum_amd.merkle.MerkleTreeWithCap."""
    _write_u64(f, tree.cap_size)
    write_digests(f, tree.leaf_hashes)
    levels = tree.num_levels()
    _write_u64(f, levels)
    for lvl in range(1, levels + 1):
        write_digests(f, tree.level(lvl))


def read_merkle_tree(f):
    """-> (cap_size, leaf_hashes (N, 4), [level_1, ..., level_k]) as numpy."""
    cap_size = _read_u64(f)
    leaves = read_digests(f)
    n = _read_u64(f)
    levels = [read_digests(f) for _ in range(n)]
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


def cap_to_json(cap):
    """MerkleTreeCap -> list of 4-lists of canonical ints (as in proof.json's *_oracle_cap)."""
    return _canon_list(np.asarray(_host(cap)).reshape(-1, 4))


def cap_from_json(obj):
    a = np.asarray(obj, dtype=np.uint64)
    if a.ndim != 2 or a.shape[1] != 4:
        raise ValueError("a cap is a list of 4-element digests")
    return a


def oracle_query_to_json(leaf_elements, proof):
    """OracleQuery -> {"leaf_elements": [...], "proof": [[...], ...]} (serde field order)."""
    return {"leaf_elements": _canon_list(np.asarray(_host(leaf_elements)).reshape(-1)),
            "proof": _canon_list(np.asarray(_host(proof)).reshape(-1, 4))}


def oracle_query_from_json(obj):
    """-> (leaf_elements (k,), proof (depth, 4)) as numpy uint64."""
    leaf = np.asarray(obj["leaf_elements"], dtype=np.uint64).reshape(-1)
    proof = np.asarray(obj["proof"], dtype=np.uint64).reshape(-1, 4)
    return leaf, proof


def dumps(obj):
    """serde_json::to_string layout: no whitespace."""
    import json
    return json.dumps(obj, separators=(",", ":"))
