"""Pin the CPU oracle (oracle/boojum_oracle.c) before trusting it as the checker.

* Poseidon2 / Overwrite sponge / node hashing / cap layout: the reference's own
  proof.json + vk.json (tests/golden/proof_queries.json, made by make_fixtures.py):
  every leaf hash + 16-level path must reproduce the committed cap for the witness,
  stage-2, quotient and setup oracles of each query, all at one leaf index
  (verifier.rs:2062-2091, merkle_tree.rs:482-504).
* LDE: the reference's test methodology (naive coset DFT with generator 7,
  fft/mod.rs:1591-1634; roundtrips :1539-1589, 1636-1709) and the closed form
  LDE[c][L] = p_c(7 * w_{nD}^{bitrev(L)}).
* SURVEY Appendix A/B known-answer vectors.
"""
import json
import os

import numpy as np
import pytest

import oracle as O

P = O.P
HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "proof_queries.json")))


@pytest.fixture(scope="module", autouse=True)
def _lib():
    O.lib()


def h(xs):
    return [int(x) for x in xs]


# ------------------------------------------------------------ proof.json pins

@pytest.mark.parametrize("qi", range(len(FIX["queries"])))
@pytest.mark.parametrize("oracle_name", ["witness", "stage_2", "quotient", "setup"])
def test_proof_json_base_oracle_paths(qi, oracle_name):
    q = FIX["queries"][qi]
    e = q[oracle_name]
    leaf = O.hash_into_leaf(e["leaf_elements"])
    assert len(e["proof"]) == 16  # log2(2^20 * 2) - log2(32)
    assert O.verify_proof_over_cap(e["proof"], FIX["caps"][oracle_name], leaf, q["index"])
    # a flipped element must break it
    bad = list(e["leaf_elements"])
    bad[0] = (bad[0] + 1) % P
    assert not O.verify_proof_over_cap(e["proof"], FIX["caps"][oracle_name], O.hash_into_leaf(bad), q["index"])


def test_proof_json_leaf_lengths_cover_padding_cases():
    # 156, 58, 16, 167 elements: lengths = 4, 2, 0, 7 mod 8 exercise the zero-padded
    # finalize and the exact-multiple case (sponge.rs:300-323).
    q = FIX["queries"][0]
    assert [len(q[k]["leaf_elements"]) % 8 for k in ("witness", "stage_2", "quotient", "setup")] == [4, 2, 0, 7]


def test_proof_json_fri_base_oracle_path():
    # FRI base oracle (construct_by_chunking, 16 elements per leaf): same hasher.
    for q in FIX["queries"]:
        f = q["fri_base"]
        leaf = O.hash_into_leaf(f["leaf_elements"])
        assert O.verify_proof_over_cap(f["proof"], FIX["caps"]["fri_base"], leaf, f["index"])
        assert f["index"] == q["index"] >> 3


# ----------------------------------------------------------- Appendix A KATs

def test_poseidon2_kats():
    assert h(O.poseidon2_permutation(np.arange(12))[:4]) == [
        0x5d82c16b87f07f98, 0x3655af22bb2f037d, 0x82c1535dfb4bdf90, 0x4d318cfdafd2378e]
    assert h(O.poseidon2_permutation(np.zeros(12))[:4]) == [
        0x78e86c27e831c353, 0xc4c13a505ffd93b8, 0xc3a6d7d7f7971adc, 0xf6ff8f53ab94d8c7]
    assert h(O.hash_into_node([1, 2, 3, 4], [5, 6, 7, 8])) == [
        0x49ed75d52f4148d7, 0xb15e7420024e9275, 0x0706da62b08023fa, 0xad3e507a5ffad5f1]
    assert h(O.hash_into_leaf(np.arange(256))) == [
        0x9460f151ad087234, 0x42329be1e9b89e20, 0xa6b9b6c68d1f9e2b, 0x90edda90e50faa32]
    assert h(O.hash_into_leaf([0, 1, 2])) == [
        0x54ea9039ce5495e2, 0xf500c918575fe14b, 0x88038222f9c57c39, 0xc992f62d5c99322e]


def test_empty_leaf_is_zero_state():
    # finalize with filled == 0 runs no permutation (sponge.rs:300-323)
    assert h(O.hash_into_leaf([])) == [0, 0, 0, 0]


def test_leaf_multiple_of_rate_has_no_extra_permutation():
    x = list(range(1, 9))
    s = np.zeros(12, dtype=np.uint64)
    s[:8] = x
    assert h(O.hash_into_leaf(x)) == h(O.poseidon2_permutation(s)[:4])


def test_noncanonical_inputs_hash_like_canonical():
    x = np.array([P + 5, 2**64 - 1, 3], dtype=np.uint64)
    y = np.array([5, (2**64 - 1) - P, 3], dtype=np.uint64)
    assert h(O.hash_into_leaf(x)) == h(O.hash_into_leaf(y))


# --------------------------------------------------------- Appendix B + LDE

def test_domain_generators_and_twiddles():
    assert O.domain_generator(3) == 0xfffffffeff000001
    assert O.domain_generator(4) == 0xefffffff00000001
    assert O.domain_generator(22) == 0x4b2a18ade67246b5
    assert h(O.precompute_twiddles(3)) == [1, 0x1000000000000, 0xfffffffeff000001, 0xfffffeff00000101]
    for log_n in range(1, 12):
        w = O.domain_generator(log_n)
        assert pow(w, 1 << log_n, P) == 1 and (log_n == 0 or pow(w, 1 << (log_n - 1), P) != 1)


def test_appendix_b_lde_vector():
    mono, l = O.lde(np.arange(8)[None, :], 1)
    assert " ".join("%016x" % x for x in l[0].reshape(-1)) == (
        "f868a66099900b7c 3c37599c666e1f6b 07d9062e0621772f c386f9d2f9e04b38 "
        "b7390621061fb4db 1426f9dff9de88ca 3c37599c66632092 f868a660999eb49b "
        "770b6c1aa730220d 815ef218f7047dfb 855bd9d54fcba706 6f77c7f511ffb902 "
        "0ff884606f908122 fb343f6a50a3bce6 e44d7088d9259efb 2347cbaa66a6230d")
    assert " ".join("%016x" % x for x in mono[0]) == (
        "7fffffff80000004 80007f7f7f800080 80007fff80000000 7fff7f7f7f800080 "
        "7fffffff80000000 8000807f807fff80 7fff7fff80000000 7fff807f807fff80")


@pytest.mark.parametrize("log_n,log_d", [(1, 1), (2, 1), (3, 2), (4, 1), (4, 2), (5, 3), (6, 2)])
def test_lde_matches_naive_coset_evaluation(log_n, log_d):
    rng = np.random.default_rng(log_n * 10 + log_d)
    col = rng.integers(0, P, size=1 << log_n, dtype=np.uint64)
    _, l = O.lde(col[None, :], log_d)
    assert h(l[0].reshape(-1)) == O.naive_coset_lde_column(col, log_d)


def test_fft_matches_naive_dft_with_coset():
    # fft/mod.rs:1591-1634: X[bitrev(k)] = sum_j x_j (7 w^k)^j
    rng = np.random.default_rng(7)
    for log_n in range(0, 7):
        n = 1 << log_n
        x = rng.integers(0, P, size=n, dtype=np.uint64)
        out = O.fft_natural_to_bitreversed(x, 7)
        w = O.domain_generator(log_n)
        for r in range(n):
            k = int(format(r, "0%db" % log_n)[::-1], 2) if log_n else 0
            pt = 7 * pow(w, k, P) % P
            assert int(out[r]) == sum(int(x[j]) * pow(pt, j, P) for j in range(n)) % P


def test_fft_ifft_roundtrip_with_coset():
    rng = np.random.default_rng(3)
    for log_n in (1, 5, 10, 13):
        x = rng.integers(0, P, size=1 << log_n, dtype=np.uint64)
        y = O.fft_natural_to_bitreversed(x, 1)
        z = O.ifft_natural_to_natural(O.bitreverse(y), 1)
        assert np.array_equal(z, x)
        # coset variant: ifft(coset) undoes distribute_powers(coset) + ntt
        y = O.bitreverse(O.fft_natural_to_bitreversed(x, 7))
        assert np.array_equal(O.ifft_natural_to_natural(y, 7), x)


def test_merkle_tree_small_consistency():
    rng = np.random.default_rng(11)
    src = rng.integers(0, P, size=(13, 64), dtype=np.uint64)
    leaves, nodes, levels, cap = O.merkle_construct(src, 4)
    assert levels == 4 and cap.shape == (4, 4)
    for L in range(64):
        assert np.array_equal(leaves[L], O.hash_into_leaf(src[:, L]))
    for idx in (0, 17, 63):
        leaf, path = O.merkle_get_proof(leaves, nodes, levels, idx)
        assert O.verify_proof_over_cap(path, cap, leaf, idx)


def test_threaded_oracle_equals_single_thread():
    tr = O.synthetic_trace(9, 8)
    a = O.lde_commit(tr, 2, 8, threads=1)
    b = O.lde_commit(tr, 2, 8, threads=4)
    for k in ("monomials", "lde", "leaves", "nodes", "cap"):
        assert np.array_equal(a[k], b[k]), k
