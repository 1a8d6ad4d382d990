"""GPU parity of the Keccak256 tree hasher (csrc/keccak.hip, cs/oracle/mod.rs:247-313) against
the oracle (pinned to hashlib.sha3_256 and known answers, tests/test_oracle_keccak.py): leaves
of every block-padding case (17 elements per 136-byte block), non-canonical inputs, node levels
to several caps, chunked (FRI) leaves, host seams and a whole commit."""
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
    from boojum_amd import commit, field, merkle
    from boojum_amd._lib import call
    boojum_amd.load()
    return type("BJ", (), dict(torch=torch, commit=commit, field=field, merkle=merkle, call=staticmethod(call)))


def rand(shape, seed, full_range=False):
    hi = 2**64 - 1 if full_range else O.P - 1
    return np.random.default_rng(seed).integers(0, hi, size=shape, dtype=np.uint64, endpoint=True)


def eq(a, b, what=""):
    a, b = np.asarray(a, dtype=np.uint64), np.asarray(b, dtype=np.uint64)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    bad = np.argwhere(a != b)
    assert bad.size == 0, "%s: first mismatches at %s" % (what, bad[:5].tolist())


@pytest.mark.parametrize("c", [0, 1, 15, 16, 17, 18, 33, 34, 35, 93])
def test_leaves_every_padding_case(bj, c):
    nl = 256
    x = rand((max(c, 1), nl), 40 + c, full_range=True)[:c]
    src = bj.field.to_device(x if c else np.zeros((1, nl), np.uint64))
    out = bj.torch.empty((nl, 4), dtype=bj.torch.int64, device="cuda")
    bj.call("bj_keccak256_leaves_d", src.data_ptr(), c, nl, nl, out.data_ptr(), 0)
    eq(bj.field.to_host(out), np.stack([O.keccak_leaf(x[:, L]) for L in range(nl)]), "leaves c=%d" % c)


@pytest.mark.parametrize("nl,cap", [(2, 1), (1024, 16), (8192, 2048), (1 << 14, 4)])
def test_tree_matches_oracle(bj, nl, cap):
    x = rand((9, nl), nl + cap)
    t = bj.merkle.MerkleTreeWithCap.construct(bj.field.to_device(x), cap, hasher="keccak256")
    leaves, nodes, _, cap_ref = O.merkle_construct(x, cap, threads=THREADS, hasher="keccak256")
    eq(bj.field.to_host(t.leaf_hashes), leaves, "leaves")
    eq(bj.field.to_host(t.nodes), nodes, "nodes")
    eq(t.get_cap(), cap_ref, "cap")
    leaf, path = t.get_proof(nl // 3)
    assert bj.merkle.MerkleTreeWithCap.verify_proof_over_cap(path, cap_ref, leaf, nl // 3, hasher="keccak256")


def test_host_seams(bj):
    H = bj.merkle.Keccak256
    for n in (0, 1, 17, 40):
        e = rand(n, 500 + n, full_range=True)
        eq(H.hash_into_leaf(e), O.keccak_leaf(e), "leaf %d" % n)
    l, r = rand(4, 1), rand(4, 2)
    eq(H.hash_into_node(l, r), O.keccak_node(l, r), "node")


@pytest.mark.parametrize("c,e,cap", [(2, 4, 4), (2, 16, 8), (3, 8, 1)])
def test_chunked_leaves(bj, c, e, cap):
    x = rand((c, 1 << 12), c * e + 1)
    t = bj.merkle.MerkleTreeWithCap.construct_by_chunking(bj.field.to_device(x), e, cap, hasher="keccak256")
    leaves, _, _, cap_ref = O.merkle_construct_by_chunking(x, e, cap, threads=THREADS, hasher="keccak256")
    eq(bj.field.to_host(t.leaf_hashes), leaves, "chunked leaves")
    eq(t.get_cap(), cap_ref, "chunked cap")


def test_witness_commit_keccak(bj):
    c, log_n, log_d, cap = 40, 14, 2, 16
    ws = bj.commit.witness_commit(bj.commit.synthetic_trace(c, log_n), 1 << log_d, cap, hasher="keccak256")
    bj.torch.cuda.synchronize()
    _, l_ref = O.lde(O.synthetic_trace(c, log_n), log_d, threads=THREADS)
    leaves, _, _, cap_ref = O.merkle_construct(l_ref.reshape(c, -1), cap, threads=THREADS, hasher="keccak256")
    eq(bj.field.to_host(ws.leaves), leaves, "leaves")
    eq(bj.field.to_host(ws.cap), cap_ref, "cap")
