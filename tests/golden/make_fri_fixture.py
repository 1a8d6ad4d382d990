#!/usr/bin/env python3
"""Generate tests/golden/proof_fri.json from the reference's own fixture files (JSON data only,
nothing executed): everything the verifier's transcript and FRI query checks read for the first
N_QUERIES queries of /root/reference/proof.json under /root/reference/vk.json
(cs/implementations/verifier.rs:888-2523):

  * the VK parameters the verifier reads (circuit geometry, lookup parameters, domain size,
    total_tables_len, public input locations, quotient degree) and the setup cap;
  * proof_config, public_inputs, the witness / stage-2 / quotient caps, values_at_z,
    values_at_z_omega, values_at_0, the FRI base and intermediate caps, final_fri_monomials,
    pow_challenge;
  * per query: the four base-oracle openings and every FRI step's opening (fri_queries).

tests/test_oracle_transcript.py replays the Poseidon2 transcript over these (oracle/transcript.py)
and checks the derived query indices, the DEEP combination at x = 7 w^bitrev(idx) and the whole
FRI folding chain down to final_fri_monomials.

Run in the build container (the reference is absent on the GPU box):
    python tests/golden/make_fri_fixture.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
N_QUERIES = 6


def ext_list(vals):
    return [v["coeffs"] for v in vals]


def main():
    proof = json.load(open("/root/reference/proof.json"))
    vk = json.load(open("/root/reference/vk.json"))
    fp = vk["fixed_parameters"]
    out = {
        "source": "distributed-lab/era-boojum proof.json + vk.json (reference repo root), first %d queries" % N_QUERIES,
        "vk": {
            "parameters": fp["parameters"],
            "lookup_parameters": fp["lookup_parameters"],
            "domain_size": fp["domain_size"],
            "total_tables_len": fp["total_tables_len"],
            "public_inputs_locations": fp["public_inputs_locations"],
            "extra_constant_polys_for_selectors": fp["extra_constant_polys_for_selectors"],
            "quotient_degree": fp["quotient_degree"],
            "fri_lde_factor": fp["fri_lde_factor"],
            "cap_size": fp["cap_size"],
            "setup_merkle_tree_cap": vk["setup_merkle_tree_cap"],
        },
        "proof_config": proof["proof_config"],
        "public_inputs": proof["public_inputs"],
        "witness_oracle_cap": proof["witness_oracle_cap"],
        "stage_2_oracle_cap": proof["stage_2_oracle_cap"],
        "quotient_oracle_cap": proof["quotient_oracle_cap"],
        "values_at_z": ext_list(proof["values_at_z"]),
        "values_at_z_omega": ext_list(proof["values_at_z_omega"]),
        "values_at_0": ext_list(proof["values_at_0"]),
        "fri_base_oracle_cap": proof["fri_base_oracle_cap"],
        "fri_intermediate_oracles_caps": proof["fri_intermediate_oracles_caps"],
        "final_fri_monomials": proof["final_fri_monomials"],
        "pow_challenge": proof["pow_challenge"],
        "queries": proof["queries_per_fri_repetition"][:N_QUERIES],
    }
    path = os.path.join(HERE, "proof_fri.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
