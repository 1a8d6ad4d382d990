"""The reference's own proof.json pins the LDE evaluation domain and the FRI fold, not only the
Merkle/Poseidon2 layer: oracle/transcript.py replays the verifier's Poseidon2 transcript
(transcript.rs:48-141, verifier.rs:924-1984) over tests/golden/proof_fri.json and checks, for
the first six queries of proof.json, everything Verifier::verify checks at a query
(verifier.rs:2050-2518) apart from the constraint evaluation at z:

  * the query indices drawn from the transcript equal the ones recovered from the Merkle
    paths by brute force (tests/golden/proof_queries.json) -- transcript, challenge order and
    BoolsBuffer bit order are right;
  * the DEEP combination of the witness / stage-2 / quotient / setup leaf values at
    x = 7 w_{nD}^{bitrev(idx)} equals the FRI base oracle's committed value -- the leaves are
    the LDE on the bit-reversed coset domain of SURVEY 0's closed form (a natural-order x fails);
  * every FRI step's fold of its committed leaf equals the next oracle's committed value, and the
    last one equals final_fri_monomials at the folded point -- the fold (fold_multiple,
    fri/mod.rs:362-474) as the oracle's fri_fold restates it (three folds by 2 per leaf of 8),
    with the full-domain inverse twiddles indexed by the flat pair index.
"""
import json
import os

import numpy as np
import pytest

import oracle as O
import transcript as T

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def fx():
    return json.load(open(os.path.join(HERE, "golden", "proof_fri.json")))


@pytest.fixture(scope="module")
def replayed(fx):
    return T.replay(fx)


def test_transcript_derives_the_fixture_query_indices(replayed):
    want = [q["index"] for q in json.load(open(os.path.join(HERE, "golden", "proof_queries.json")))["queries"]]
    assert [q["index"] for q in replayed["queries"]] == want
    assert replayed["schedule"] == [3, 3, 3, 3, 3, 1] and replayed["num_queries"] == 100


def test_deep_value_is_the_fri_base_leaf_value(replayed):
    for q in replayed["queries"]:
        assert q["steps"][0]["expected"] == q["deep"]


def test_natural_order_domain_is_rejected(fx, replayed):
    with pytest.raises(AssertionError):
        T.replay_with(fx, replayed["geometry"], "natural")


def fold_leaf_with_oracle(step, roots):
    """The oracle's fri_fold (test restatement of fold_multiple) applied to one committed leaf of
    2^d Ext2 values: d folds by 2, each with the full-domain inverse twiddles at the flat pair
    indices of the leaf and the coset inverse squared after each fold."""
    leaf = [int(v) for v in step["leaf"]]
    deg = len(leaf) // 2
    c0, c1 = np.array(leaf[:deg], dtype=np.uint64), np.array(leaf[deg:], dtype=np.uint64)
    base = step["tree_idx"] * deg // 2
    ci = step["coset_inverse"]
    for ch in step["challenges"]:
        r = roots[base: base + len(c0) // 2]
        c0, c1 = O.fri_fold(c0, c1, r, ci, ch)
        base //= 2
        ci = ci * ci % O.P
    return int(c0[0]), int(c1[0])


def test_fri_chain_with_the_oracle_fold(fx, replayed):
    n = fx["vk"]["domain_size"] * fx["proof_config"]["fri_lde_factor"]
    roots = O.precompute_twiddles(n.bit_length() - 1, True)
    for q in replayed["queries"]:
        steps = q["steps"]
        for k, st in enumerate(steps):
            got = fold_leaf_with_oracle(st, roots)
            want = steps[k + 1]["expected"] if k + 1 < len(steps) else q["final"]
            assert got == want, "query %d step %d" % (q["index"], k)
