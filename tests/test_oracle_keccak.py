"""The oracle's Keccak256 tree hasher (oracle/boojum_oracle.c, restating Keccak-f[1600] and the
TreeHasher impl of cs/oracle/mod.rs:247-313) pinned by an independent implementation and known
answers: the same sponge with the SHA3 domain byte (0x06) against CPython's hashlib.sha3_256
(pins the permutation, the rate and multi-block absorption), and Keccak256 itself against its
well-known digests of "" and "abc".  The reference's dependency (sha3, git RustCrypto/hashes
rev 7a187e93, Cargo.toml:15) is absent here."""
import hashlib

import numpy as np
import pytest

import oracle as O


def le_bytes(elems):
    return b"".join(int(x % O.P).to_bytes(8, "little") for x in elems)


def words(d):
    return np.frombuffer(d, dtype="<u8").astype(np.uint64)


def test_keccak256_known_answers():
    assert O.keccak256(b"").hex() == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"
    assert O.keccak256(b"abc").hex() == "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45"


@pytest.mark.parametrize("n", [0, 1, 7, 135, 136, 137, 271, 272, 273, 1000, 4096])
def test_sponge_matches_hashlib_sha3_256(n):
    data = np.random.default_rng(n).integers(0, 256, size=n, dtype=np.uint8).tobytes()
    assert O.keccak256(data, 0x06) == hashlib.sha3_256(data).digest()


@pytest.mark.parametrize("n", [0, 1, 16, 17, 18, 33, 34, 35, 93])
def test_leaf_is_keccak_of_canonical_le_bytes(n):
    e = np.random.default_rng(50 + n).integers(0, 2**64 - 1, size=n, dtype=np.uint64, endpoint=True)
    assert np.array_equal(O.keccak_leaf(e), words(O.keccak256(le_bytes(e))))


def test_tree_and_proofs():
    src = np.random.default_rng(5).integers(0, O.P, size=(20, 64), dtype=np.uint64)
    leaves, nodes, levels, cap = O.merkle_construct(src, 4, hasher="keccak256")
    layer = [O.keccak256(le_bytes(src[:, L])) for L in range(64)]
    assert np.array_equal(leaves, np.stack([words(d) for d in layer]))
    while len(layer) > 4:
        layer = [O.keccak256(layer[2 * i] + layer[2 * i + 1]) for i in range(len(layer) // 2)]
    assert np.array_equal(cap, np.stack([words(d) for d in layer]))
    leaf, path = O.merkle_get_proof(leaves, nodes, levels, 37)
    assert O.verify_proof_over_cap(path, cap, leaf, 37, hasher="keccak256")
