"""MemcopySerializable byte layout (fast_serialization.rs, lde.rs:174-217, merkle_tree.rs:36-73),
checked on host data: exact bytes for small cases and round trips."""
import io
import struct

import numpy as np
import pytest

from boojum_amd import serialization as S


def le(*vals):
    return b"".join(struct.pack("<Q", v) for v in vals)


def test_lde_storage_bytes_and_roundtrip():
    lde = np.array([[1, 2, 3, 4], [5, 6, 7, 0xFFFFFFFF00000000]], dtype=np.uint64)   # D = 2, n = 4
    f = io.BytesIO()
    S.write_lde_storage(f, lde)
    assert f.getvalue() == le(2, 4, 1, 2, 3, 4, 4, 5, 6, 7, 0xFFFFFFFF00000000)
    f.seek(0)
    assert np.array_equal(S.read_lde_storage(f), lde)


class _Tree:
    """Host stand-in with the MerkleTreeWithCap mirror's accessors."""

    def __init__(self, cap_size, leaves, levels):
        self.cap_size, self.leaf_hashes, self._levels = cap_size, leaves, levels

    def num_levels(self):
        return len(self._levels)

    def level(self, i):
        return self.leaf_hashes if i == 0 else self._levels[i - 1]


def test_merkle_tree_bytes_and_roundtrip():
    leaves = np.arange(16, dtype=np.uint64).reshape(4, 4)
    l1 = np.arange(100, 108, dtype=np.uint64).reshape(2, 4)
    t = _Tree(2, leaves, [l1])
    f = io.BytesIO()
    S.write_merkle_tree(f, t)
    assert f.getvalue() == le(2, 16, *range(16), 1, 8, *range(100, 108))
    f.seek(0)
    cap, lv, levels = S.read_merkle_tree(f)
    assert cap == 2 and np.array_equal(lv, leaves) and len(levels) == 1 and np.array_equal(levels[0], l1)


def test_truncated_stream_raises():
    with pytest.raises(EOFError):
        S.read_lde_storage(io.BytesIO(le(2, 4, 1, 2)))
    with pytest.raises(ValueError):
        S.read_lde_storage(io.BytesIO(le(3)))


def test_serde_json_round_trips_the_reference_proof_parts():
    """proof.json's caps and OracleQuery objects (tests/golden, extracted from the reference's
    proof.json) read and re-serialise to the same JSON, and the parsed query still opens against
    the parsed cap (the oracle's verify_proof_over_cap, merkle_tree.rs:482-504)."""
    import json
    import os
    import oracle as O
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "proof_queries.json")))
    cap = S.cap_from_json(fx["caps"]["witness"])
    assert S.cap_to_json(cap) == fx["caps"]["witness"]
    for q in fx["queries"][:4]:
        leaf_elems, proof = S.oracle_query_from_json(q["witness"])
        assert S.oracle_query_to_json(leaf_elems, proof) == q["witness"]
        assert json.loads(S.dumps(S.oracle_query_to_json(leaf_elems, proof))) == q["witness"]
        leaf = O.hash_into_leaf(leaf_elems)
        assert O.verify_proof_over_cap(proof, cap, leaf, q["index"])


def test_serde_json_is_canonical_and_compact():
    p = 0xFFFFFFFF00000001
    q = S.oracle_query_to_json(np.array([p, p + 5, 3], dtype=np.uint64), np.arange(8, dtype=np.uint64))
    assert q == {"leaf_elements": [0, 5, 3], "proof": [[0, 1, 2, 3], [4, 5, 6, 7]]}
    assert S.dumps(q) == '{"leaf_elements":[0,5,3],"proof":[[0,1,2,3],[4,5,6,7]]}'
    with pytest.raises(ValueError):
        S.cap_from_json([[1, 2, 3]])


def test_byte_digest_tree_layout_blake2s():
    """MerkleTreeWithCap<F, Blake2s256>: H::Output = [u8; 32], so leaf hashes and node levels go
    out as Vec<[u8; 32]> (fast_serialization.rs:343-358): the length prefix counts BYTES (32 per
    digest) and the payload is the raw digest bytes -- here the 4 little-endian words of each."""
    import hashlib
    digests = [hashlib.blake2s(bytes([i])).digest() for i in range(6)]
    words = np.frombuffer(b"".join(digests), dtype="<u8").astype(np.uint64).reshape(6, 4)
    t = _Tree(2, words[:4], [words[4:]])
    t.hasher = "blake2s"
    f = io.BytesIO()
    S.write_merkle_tree(f, t)
    want = le(2) + le(128) + b"".join(digests[:4]) + le(1) + le(64) + b"".join(digests[4:])
    assert f.getvalue() == want
    f.seek(0)
    cap, lv, levels = S.read_merkle_tree(f, "blake2s")
    assert cap == 2 and np.array_equal(lv, words[:4]) and np.array_equal(levels[0], words[4:])


def test_byte_digest_json_is_raw_bytes():
    """serde writes a [u8; 32] digest as 32 integers: no reduction mod p (a word >= p survives)."""
    w = np.array([[0xFFFFFFFFFFFFFFFF, 1, 2, 0xFFFFFFFF00000001]], dtype=np.uint64)
    j = S.cap_to_json(w, "keccak256")
    assert len(j) == 1 and len(j[0]) == 32 and j[0][:8] == [255] * 8 and j[0][8] == 1
    assert np.array_equal(S.cap_from_json(j, "keccak256"), w)
    q = S.oracle_query_to_json(np.array([5, 0xFFFFFFFF00000002], dtype=np.uint64), w, "blake2s")
    assert q["leaf_elements"] == [5, 1] and len(q["proof"][0]) == 32
    leaf, proof = S.oracle_query_from_json(q, "blake2s")
    assert np.array_equal(proof, w)
    with pytest.raises(ValueError):
        S.cap_to_json(w, "sha256")
