"""Full-size GPU checks at the BASELINE configurations.

* C2 (2^20 x 128, LDE x2, cap 16): bit-exact against the CPU oracle end to end (LDE,
  leaves, nodes, cap). This is BASELINE.json configs[1] "bit-exact vs CPU LDE + caps".
* C3 (2^22 x 256, LDE x4, cap 16, the bench workload) and C4 (2^23 x 256, LDE x8, the 8-GPU
  sizing case, 164 GB of HBM on one GPU): the oracle would need minutes, so the checks are
  size-independent properties of the same commit:
  - three whole columns (first, middle, last) equal the oracle's LDE of those columns;
  - 256 sampled leaves are re-hashed on the CPU from the GPU's LDE rows;
  - every node level is spot-checked: sampled parents re-hashed from their two children;
  - the cap recomputed from the level below it;
  - Merkle paths of sampled leaves verify against the cap (verify_proof_over_cap,
    merkle_tree.rs:482-504).
"""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def bj():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import boojum_amd
    from boojum_amd import commit, field
    boojum_amd.load()
    return type("BJ", (), dict(torch=torch, commit=commit, field=field))


def eq(a, b, what):
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    bad = np.argwhere(a != b)
    assert bad.size == 0, "%s: first mismatches at %s" % (what, bad[:5].tolist())


def test_c2_bit_exact(bj):
    c, log_n, log_d, cap = 128, 20, 1, 16
    tr = bj.commit.synthetic_trace(c, log_n)
    ws = bj.commit.witness_commit(tr, 1 << log_d, cap)
    bj.torch.cuda.synchronize()
    ref = O.lde_commit(O.synthetic_trace(c, log_n), log_d, cap, threads=THREADS)
    eq(bj.field.to_host(ws.cap), ref["cap"], "cap")
    eq(bj.field.to_host(ws.leaves), ref["leaves"], "leaves")
    eq(bj.field.to_host(ws.nodes), ref["nodes"], "nodes")
    eq(bj.field.to_host(ws.lde), ref["lde"], "lde")


@pytest.mark.parametrize("cfg", [(256, 22, 2, 16), (256, 23, 3, 16)], ids=["C3", "C4"])
def test_fullsize_properties(bj, cfg):
    torch = bj.torch
    c, log_n, log_d, cap = cfg
    n, D = 1 << log_n, 1 << log_d
    nl = n * D
    torch.cuda.empty_cache()
    tr = bj.commit.synthetic_trace(c, log_n)
    ws = bj.commit.witness_commit(tr, D, cap)
    torch.cuda.synchronize()
    rng = np.random.default_rng(3)

    # whole columns against the oracle's LDE of the same columns
    cols = [0, c // 2, c - 1]
    x = np.stack([O.synthetic_trace(1, log_n, col_offset=k)[0] for k in cols])
    eq(bj.field.to_host(tr[cols]), x, "trace")
    _, l_ref = O.lde(x, log_d, threads=THREADS)
    eq(bj.field.to_host(ws.lde[cols]), l_ref, "lde columns")

    # sampled leaves re-hashed from the GPU LDE rows
    flat = ws.lde.view(c, nl)
    idx = np.concatenate([[0, nl - 1, n - 1, n], rng.integers(0, nl, size=252)])
    rows = bj.field.to_host(flat[:, torch.as_tensor(idx, device=flat.device)])
    leaves = bj.field.to_host(ws.leaves)
    for j, L in enumerate(idx):
        eq(leaves[L], O.hash_into_leaf(np.ascontiguousarray(rows[:, j])), "leaf %d" % L)

    # node levels: sampled parents from their children; cap from the level below
    nodes = bj.field.to_host(ws.nodes)
    below, off, ln = leaves, 0, nl
    while ln > cap:
        ln //= 2
        level = nodes[off: off + ln]
        for i in np.unique(np.concatenate([[0, ln - 1], rng.integers(0, ln, size=32)])):
            eq(level[i], O.hash_into_node(below[2 * i], below[2 * i + 1]), "node (%d, %d)" % (ln, i))
        below, off = level, off + ln
    assert off == nl - cap
    eq(below, nodes[-cap:], "cap level")
    prev = nodes[-3 * cap: -cap]
    eq(np.stack([O.hash_into_node(prev[2 * i], prev[2 * i + 1]) for i in range(cap)]), nodes[-cap:], "cap")

    # Merkle paths against the cap
    levels = log_n + log_d - (cap.bit_length() - 1)
    for L in idx[:16]:
        leaf, path = O.merkle_get_proof(leaves, nodes, levels, int(L))
        assert O.verify_proof_over_cap(path, nodes[-cap:], leaf, int(L))
