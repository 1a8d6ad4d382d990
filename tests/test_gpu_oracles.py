"""GPU parity of the prover's other commitments: the same kernels with other
column sets, an LDE degree above the committed coset count (subset_for_degree), Ext2 columns
as (c0, c1) base pairs, quotient chunks in monomial form, and the sha256 circuit's shape (C5).
Every output is compared bit for bit with the CPU oracle."""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def bj():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import boojum_amd
    from boojum_amd import commit, field
    boojum_amd.load()
    return type("BJ", (), dict(torch=torch, commit=commit, field=field))


def rand(shape, seed):
    return np.random.default_rng(seed).integers(0, O.P, size=shape, dtype=np.uint64)


def eq(a, b, what=""):
    a, b = np.asarray(a, dtype=np.uint64), np.asarray(b, dtype=np.uint64)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    bad = np.argwhere(a != b)
    assert bad.size == 0, "%s: first mismatches at %s" % (what, bad[:5].tolist())


def ref_commit(lde, k, cap):
    c, d, n = lde.shape
    return O.merkle_construct(np.ascontiguousarray(lde[:, :k, :]).reshape(c, k * n), cap, threads=THREADS)


@pytest.mark.parametrize("c,log_n,log_d,k,cap", [(7, 10, 3, 2, 16), (16, 12, 2, 1, 8), (3, 9, 3, 8, 4)])
def test_commit_subset_of_cosets(bj, c, log_n, log_d, k, cap):
    """LDE at used_lde_degree, tree over the first fri_lde_factor cosets (prover.rs:313-347)."""
    x = rand((c, 1 << log_n), c + log_n)
    oc = bj.commit.commit_trace_columns(bj.field.to_device(x), 1 << log_d, k, cap)
    _, l_ref = O.lde(x, log_d, threads=THREADS)
    eq(bj.field.to_host(oc.lde), l_ref, "lde")
    leaves, nodes, _, cap_ref = ref_commit(l_ref, k, cap)
    eq(bj.field.to_host(oc.tree.leaf_hashes), leaves, "leaves")
    eq(oc.get_cap(), cap_ref, "cap")


def test_second_stage_ext2_pairs(bj):
    """Stage-2 oracle: Ext2 polys as (c0, c1) base pairs in the prover's leaf order."""
    n = 1 << 11
    z = rand((2, n), 1)
    inter = rand((3, 2, n), 2)
    lw = rand((2, 2, n), 3)
    mu = rand((1, 2, n), 4)
    to = bj.field.to_device
    oc = bj.commit.second_stage_commit((to(z[0]), to(z[1])), [(to(a), to(b)) for a, b in inter],
                                       [(to(a), to(b)) for a, b in lw], [(to(a), to(b)) for a, b in mu], 8, 4, 16)
    base = np.concatenate([z, inter.reshape(-1, n), lw.reshape(-1, n), mu.reshape(-1, n)])
    _, l_ref = O.lde(base, 3, threads=THREADS)
    _, _, _, cap_ref = ref_commit(l_ref, 4, 16)
    eq(oc.get_cap(), cap_ref, "stage-2 cap")


def test_quotient_from_monomials(bj):
    """Quotient oracle: monomial chunks -> LDE at fri_lde_factor -> tree (prover.rs:1454-1495)."""
    c, log_n, log_d, cap = 16, 10, 1, 16
    mono = rand((c, 1 << log_n), 9)
    oc = bj.commit.quotient_commit(bj.field.to_device(mono), 1 << log_d, cap)
    cos = O.lde_cosets(log_n, log_d)
    l_ref = np.stack([np.stack([O.fft_natural_to_bitreversed(mono[i], int(s)) for s in cos]) for i in range(c)])
    eq(bj.field.to_host(oc.lde), l_ref, "quotient lde")
    _, _, _, cap_ref = ref_commit(l_ref, 1 << log_d, cap)
    eq(oc.get_cap(), cap_ref, "quotient cap")


def test_c5_sha256_shape_witness_commit(bj):
    """C5: the sha256 test circuit's witness oracle shape (sha256/mod.rs:309-360): n = 2^16,
    60 copy-permutation + 8 x 4 lookup + 1 multiplicity = 93 columns, LDE x8, cap 16."""
    c, log_n, log_d, cap = 93, 16, 3, 16
    tr = bj.commit.synthetic_trace(c, log_n)
    ws = bj.commit.witness_commit(tr, 1 << log_d, cap)
    ref = O.lde_commit(O.synthetic_trace(c, log_n), log_d, cap, threads=THREADS)
    eq(bj.field.to_host(ws.cap), ref["cap"], "cap")
    eq(bj.field.to_host(ws.leaves), ref["leaves"], "leaves")


@pytest.mark.parametrize("hasher", ["poseidon2", "blake2s"])
def test_commit_graph_replay(bj, hasher):
    """commit.CommitGraph: the commit captured once as a HIP graph; refilling the trace buffer in
    place and replaying commits the new contents (not a cached result)."""
    torch = bj.torch
    c, log_n, log_d, cap = 24, 14, 2, 16
    tr = bj.commit.synthetic_trace(c, log_n)
    g = bj.commit.CommitGraph(tr, 1 << log_d, cap, hasher=hasher)
    for seed in (42, 7):
        bj.commit.synthetic_trace(c, log_n, seed=seed, out=tr)
        ws = g.replay()
        torch.cuda.synchronize()
        x = O.synthetic_trace(c, log_n, seed=seed)
        _, l_ref = O.lde(x, log_d, threads=THREADS)
        leaves, _, _, cap_ref = O.merkle_construct(l_ref.reshape(c, -1), cap, threads=THREADS, hasher=hasher)
        eq(bj.field.to_host(ws.leaves), leaves, "graph leaves seed %d" % seed)
        eq(bj.field.to_host(ws.cap), cap_ref, "graph cap seed %d" % seed)


def test_memcopy_serialization_roundtrip(bj):
    """A GPU tree and LDE written in the reference's MemcopySerializable layout read back equal."""
    import io
    from boojum_amd import merkle, serialization as S
    x = rand((3, 1 << 9), 12)
    oc = bj.commit.commit_trace_columns(bj.field.to_device(x), 4, 4, 8)
    f = io.BytesIO()
    S.write_lde_storage(f, oc.lde[1])
    S.write_merkle_tree(f, oc.tree)
    f.seek(0)
    eq(S.read_lde_storage(f), bj.field.to_host(oc.lde[1]), "lde")
    cap, leaves, levels = S.read_merkle_tree(f)
    assert cap == 8 and len(levels) == oc.tree.num_levels()
    eq(leaves, bj.field.to_host(oc.tree.leaf_hashes), "leaves")
    eq(levels[-1], oc.get_cap(), "cap level")
    path = np.stack([lvl[(5 >> i) ^ 1] for i, lvl in enumerate([leaves] + levels[:-1])])
    assert merkle.MerkleTreeWithCap.verify_proof_over_cap(path, oc.get_cap(), leaves[5], 5)
