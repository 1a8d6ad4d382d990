"""The oracle's Blake2s256 tree hasher (oracle/boojum_oracle.c, restating RFC 7693 and the
TreeHasher impl of cs/oracle/mod.rs:179-245) pinned against an independent implementation:
CPython's hashlib.blake2s (the BLAKE2 authors' reference code), plus the RFC 7693 Appendix B
vector.  The reference's own dependency (blake2 = "0.10", Cargo.toml:23) is a third-party
crate absent here; Blake2s256 is BLAKE2s-256 with no key, which hashlib.blake2s() is."""
import hashlib

import numpy as np
import pytest

import oracle as O


def le_bytes(elems):
    return b"".join(int(x % O.P).to_bytes(8, "little") for x in elems)


def digest_words(d):
    return np.frombuffer(d, dtype="<u8").astype(np.uint64)


def test_rfc7693_appendix_b():
    assert O.blake2s(b"abc").hex() == "508c5e8c327c14e2e1a72ba34eeb452f37458b209ed63a294d999b4c86675982"


@pytest.mark.parametrize("n", [0, 1, 3, 63, 64, 65, 127, 128, 129, 1000, 4096])
def test_blake2s_matches_hashlib(n):
    data = np.random.default_rng(n).integers(0, 256, size=n, dtype=np.uint8).tobytes()
    assert O.blake2s(data) == hashlib.blake2s(data).digest()


@pytest.mark.parametrize("n", [0, 1, 2, 7, 8, 9, 15, 16, 17, 93, 256])
def test_leaf_is_blake2s_of_canonical_le_bytes(n):
    rng = np.random.default_rng(100 + n)
    e = rng.integers(0, 2**64 - 1, size=n, dtype=np.uint64, endpoint=True)  # non-canonical too
    got = O.blake2s_leaf(e)
    assert np.array_equal(got, digest_words(hashlib.blake2s(le_bytes(e)).digest()))


def test_node_is_blake2s_of_concatenation():
    rng = np.random.default_rng(7)
    l, r = rng.integers(0, 2**63, size=4, dtype=np.uint64), rng.integers(0, 2**63, size=4, dtype=np.uint64)
    want = hashlib.blake2s(l.astype("<u8").tobytes() + r.astype("<u8").tobytes()).digest()
    assert np.array_equal(O.blake2s_node(l, r), digest_words(want))


@pytest.mark.parametrize("c,nl,cap", [(5, 64, 4), (16, 128, 1), (9, 32, 16)])
def test_tree_against_python_blake2s_tree(c, nl, cap):
    src = np.random.default_rng(c * nl).integers(0, O.P, size=(c, nl), dtype=np.uint64)
    leaves, nodes, levels, cap_out = O.merkle_construct(src, cap, hasher="blake2s")
    layer = [hashlib.blake2s(le_bytes(src[:, L])).digest() for L in range(nl)]
    assert np.array_equal(leaves, np.stack([digest_words(d) for d in layer]))
    allnodes = []
    while len(layer) > cap:
        layer = [hashlib.blake2s(layer[2 * i] + layer[2 * i + 1]).digest() for i in range(len(layer) // 2)]
        allnodes += layer
    assert np.array_equal(nodes, np.stack([digest_words(d) for d in allnodes]))
    assert np.array_equal(cap_out, np.stack([digest_words(d) for d in layer]))
    for idx in (0, nl - 1, nl // 3):
        leaf, path = O.merkle_get_proof(leaves, nodes, levels, idx)
        assert O.verify_proof_over_cap(path, cap_out, leaf, idx, hasher="blake2s")
        bad = leaf.copy()
        bad[0] ^= np.uint64(1)
        assert not O.verify_proof_over_cap(path, cap_out, bad, idx, hasher="blake2s")


def test_chunked_tree_blake2s():
    src = np.random.default_rng(3).integers(0, O.P, size=(2, 64), dtype=np.uint64)
    leaves, _, _, _ = O.merkle_construct_by_chunking(src, 4, 2, hasher="blake2s")
    for L in range(16):
        elems = np.concatenate([src[0, 4 * L:4 * L + 4], src[1, 4 * L:4 * L + 4]])
        assert np.array_equal(leaves[L], digest_words(hashlib.blake2s(le_bytes(elems)).digest()))
