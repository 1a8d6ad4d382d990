"""Launch a G-rank sharded commit (gloo) and check every rank's outputs against the oracle's
single-process commit of the same synthetic trace.  Shared by the CPU and GPU tests."""
import os

import numpy as np

import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PATHS = [HERE, ROOT, os.path.join(ROOT, "era-boojum_amd"), os.path.join(ROOT, "oracle")]


def run_and_check(world, cfg, tmp_path, device):
    import torch.multiprocessing as mp
    import shard_worker
    mp.start_processes(shard_worker.run, args=(world, cfg, str(tmp_path), device, PATHS), nprocs=world,
                       join=True, start_method="spawn")
    n_cols, log_n, log_lde, cap = cfg[:4]
    hasher = cfg[6] if len(cfg) > 6 and cfg[6] else "poseidon2"
    log_k = cfg[7] if len(cfg) > 7 and cfg[7] is not None else log_lde
    n, nd, nl = 1 << log_n, 1 << (log_n + log_lde), 1 << (log_n + log_k)
    m = nl // world
    if hasher == "poseidon2":
        ref = O.lde_commit(O.synthetic_trace(n_cols, log_n), log_lde, cap, threads=4, log_k=log_k)
    else:
        _, lde = O.lde(O.synthetic_trace(n_cols, log_n), log_lde, threads=4)
        leaves, nodes, _, cap_ref = O.merkle_construct(np.ascontiguousarray(lde.reshape(n_cols, nd)[:, :nl]), cap,
                                                       threads=4, hasher=hasher)
        ref = {"lde": lde, "leaves": leaves, "nodes": nodes, "cap": cap_ref}
    lde_flat = ref["lde"].reshape(n_cols, nd)
    # global node levels: level k (k >= 1) holds nl >> k digests
    offs, o = [], 0
    k = 1
    while (nl >> k) >= cap:
        offs.append(o)
        o += nl >> k
        k += 1
    for P in range(world):
        r = np.load(os.path.join(str(tmp_path), "rank%d.npz" % P))
        # block j of rank P: range j G + P of the D-coset domain (cosets [j k, (j+1) k))
        for j in range(nd // nl):
            lo = j * nl + P * m
            assert np.array_equal(r["lde"][j], lde_flat[:, lo:lo + m]), "rank %d lde block %d" % (P, j)
        assert np.array_equal(r["leaves"], ref["leaves"][P * m:(P + 1) * m]), "rank %d leaves" % P
        assert np.array_equal(r["cap"], ref["cap"]), "rank %d cap" % P
        # local subtree level k == slice of global level k
        lo, k = 0, 1
        while (m >> k) >= max(1, cap // world):
            cnt = m >> k
            want = ref["nodes"][offs[k - 1] + P * cnt: offs[k - 1] + (P + 1) * cnt]
            assert np.array_equal(r["nodes"][lo:lo + cnt], want), "rank %d node level %d" % (P, k)
            lo += cnt
            k += 1
        assert lo == r["nodes"].shape[0]
        # openings (OracleQuery::construct): identical on every rank, equal to the full tree's
        levels = (nl.bit_length() - 1) - (cap.bit_length() - 1)
        for j, idx in enumerate(r["qidx"]):
            idx = int(idx)
            leaf, path = O.merkle_get_proof(ref["leaves"], ref["nodes"], levels, idx)
            assert np.array_equal(r["q_elems"][j], lde_flat[:, idx]), "rank %d query %d elements" % (P, idx)
            assert np.array_equal(r["q_leaf"][j], leaf), "rank %d query %d leaf" % (P, idx)
            assert np.array_equal(r["q_path"][j], path), "rank %d query %d path" % (P, idx)
            assert O.verify_proof_over_cap(r["q_path"][j], ref["cap"], r["q_leaf"][j], idx, hasher=hasher)
