"""The golden caps bench.py verifies against (tests/golden/bench_caps.json,
tools/make_bench_golden.py) are the oracle's caps of the bench configs' synthetic traces:
recompute the small ones here."""
import json
import os

import numpy as np
import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("key,cfg", [("C1/poseidon2", (32, 16, 1, 16)), ("C5/poseidon2", (93, 16, 3, 16))])
def test_golden_caps_are_the_oracle_caps(key, cfg):
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_caps.json")))["caps"]
    assert "C3/poseidon2" in g, "the headline config's golden cap is missing"
    n_cols, log_n, log_lde, cap = cfg
    ref = O.lde_commit(O.synthetic_trace(n_cols, log_n), log_lde, cap, threads=os.cpu_count() or 1)
    want = [["%016x" % int(x) for x in row] for row in ref["cap"].astype(np.uint64)]
    assert g[key]["cap"] == want


def test_bench_reads_the_golden_cap():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    c3 = bench.golden_cap("C3", "poseidon2")
    assert c3 is not None and len(c3) == 16 and all(len(d) == 4 for d in c3)
    assert bench.golden_cap("C3", "keccak256") is None


@pytest.mark.parametrize("n_cols,chunk", [(40, 16), (32, 8), (13, 8)])
def test_chunked_oracle_commit_matches_one_shot(n_cols, chunk):
    """tools/make_bench_golden.py --chunk-cols (how the C4 cap is made): the LDE of a column
    chunk, then the leaf sponges carried over it by their capacity words, equals the one-shot
    commit (the sponge is sequential over the row; 8-column boundaries are rate boundaries)."""
    log_n, log_d, cap = 9, 2, 8
    threads = os.cpu_count() or 1
    ref = O.lde_commit(O.synthetic_trace(n_cols, log_n), log_d, cap, threads=threads)
    state = None
    for c0 in range(0, n_cols, chunk):
        k = min(chunk, n_cols - c0)
        _, lde = O.lde(O.synthetic_trace(k, log_n, col_offset=c0), log_d, threads=threads)
        state = O.poseidon2_leaves_partial(lde.reshape(k, -1), state, c0 + k == n_cols, threads=threads)
    nodes, capv = O.merkle_nodes(state, cap, threads=threads)
    assert (state == ref["leaves"]).all() and (nodes == ref["nodes"]).all() and (capv == ref["cap"]).all()


def test_partial_leaves_reject_a_ragged_middle_chunk():
    lde = O.synthetic_trace(5, 6)
    with pytest.raises(ValueError):
        O.poseidon2_leaves_partial(lde, None, False)
