#!/usr/bin/env python3
"""Generate tests/golden/proof_queries.json from the reference's own fixture files.

Inputs (data files the reference holds, read as JSON -- nothing executed):
  /root/reference/proof.json  (GoldilocksPoseidon2Sponge<AbsorptionModeOverwrite> tree hasher,
                                per recursive_verifier.rs:2214-2222; fri_lde_factor 2, cap 32)
  /root/reference/vk.json      (setup_merkle_tree_cap)

Output: a small JSON with the four base-oracle caps (witness, stage-2, quotient, setup),
the FRI base-oracle cap, and the first N_QUERIES queries' leaf elements + Merkle paths,
plus each query's leaf index.  proof.json does not store the index (the verifier derives
it from the transcript), so it is recovered here by brute force over the path-bit
patterns with the CPU oracle (idx = (cap_idx << depth) | path_bits, merkle_tree.rs:482-504).
The index is a label only: tests check leaf-hash + path -> cap at that index, and that
all four base oracles of a query agree on it (verifier.rs:2062-2091).

Run in the build container (the reference is absent on the GPU box):
    python tests/golden/make_fixtures.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

N_QUERIES = 6


def main():
    proof = json.load(open("/root/reference/proof.json"))
    vk = json.load(open("/root/reference/vk.json"))
    caps = {
        "witness": proof["witness_oracle_cap"],
        "stage_2": proof["stage_2_oracle_cap"],
        "quotient": proof["quotient_oracle_cap"],
        "setup": vk["setup_merkle_tree_cap"],
        "fri_base": proof["fri_base_oracle_cap"],
    }
    queries = []
    for qi in range(N_QUERIES):
        q = proof["queries_per_fri_repetition"][qi]
        w = q["witness_query"]
        idx = oracle.find_query_index(oracle.hash_into_leaf(w["leaf_elements"]), w["proof"], caps["witness"])
        assert idx >= 0, "witness query %d did not verify against the cap" % qi
        entry = {"index": int(idx)}
        for name in ("witness", "stage_2", "quotient", "setup"):
            qq = q[name + "_query"]
            leaf = oracle.hash_into_leaf(qq["leaf_elements"])
            assert oracle.verify_proof_over_cap(qq["proof"], caps[name], leaf, idx), (qi, name)
            entry[name] = {"leaf_elements": qq["leaf_elements"], "proof": qq["proof"]}
        fq = q["fri_queries"][0]
        fidx = oracle.find_query_index(oracle.hash_into_leaf(fq["leaf_elements"]), fq["proof"], caps["fri_base"])
        assert fidx >= 0
        entry["fri_base"] = {"index": int(fidx), "leaf_elements": fq["leaf_elements"], "proof": fq["proof"]}
        queries.append(entry)
        print("query", qi, "index", idx, "fri_base index", fidx)
    out = {
        "source": "distributed-lab/era-boojum proof.json + vk.json (reference repo root)",
        "proof_config": proof["proof_config"],
        "domain_size": vk["fixed_parameters"]["domain_size"],
        "caps": caps,
        "queries": queries,
    }
    path = os.path.join(HERE, "proof_queries.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
