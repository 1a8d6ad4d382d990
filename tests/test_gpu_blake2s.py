"""GPU parity of the Blake2s256 tree hasher (csrc/blake2s.hip, cs/oracle/mod.rs:179-245),
the tree of the non-recursive prover configs (C5: gadgets/sha256/mod.rs:263-269), against the
oracle (itself pinned to hashlib.blake2s, tests/test_oracle_blake2s.py): leaves of every
block-padding case, non-canonical inputs, node levels to caps of 1..2048, chunked (FRI)
leaves, the column-range continuation, host seams, and the C5 witness and stage-2 commits."""
import hashlib
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


@pytest.mark.parametrize("c", [0, 1, 2, 7, 8, 9, 15, 16, 17, 24, 93, 130])
def test_leaves_every_padding_case(bj, c):
    nl = 512
    x = rand((max(c, 1), nl), 10 + c, full_range=True)[:c]
    src = bj.field.to_device(x if c else np.zeros((1, nl), np.uint64))
    out = bj.torch.empty((nl, 4), dtype=bj.torch.int64, device="cuda")
    bj.call("bj_blake2s_leaves_d", src.data_ptr(), c, nl, nl, out.data_ptr(), 0)
    got = bj.field.to_host(out)
    want = np.stack([O.blake2s_leaf(x[:, L]) for L in range(nl)])
    eq(got, want, "leaves c=%d" % c)


@pytest.mark.parametrize("nl,cap", [(2, 1), (64, 1), (1024, 16), (8192, 2048), (1 << 14, 16), (1 << 14, 4096)])
def test_tree_matches_oracle(bj, nl, cap):
    c = 11
    x = rand((c, nl), nl + cap)
    t = bj.merkle.MerkleTreeWithCap.construct(bj.field.to_device(x), cap, hasher="blake2s")
    leaves, nodes, levels, cap_ref = O.merkle_construct(x, cap, threads=THREADS, hasher="blake2s")
    eq(bj.field.to_host(t.leaf_hashes), leaves, "leaves")
    eq(bj.field.to_host(t.nodes), nodes, "nodes")
    eq(t.get_cap(), cap_ref, "cap")
    for idx in (0, nl - 1, nl // 3):
        leaf, path = t.get_proof(idx)
        assert bj.merkle.MerkleTreeWithCap.verify_proof_over_cap(path, cap_ref, leaf, idx, hasher="blake2s")
        assert O.verify_proof_over_cap(path, cap_ref, leaf, idx, hasher="blake2s")


def test_host_seams_match_hashlib(bj):
    H = bj.merkle.Blake2s256
    for n in (0, 1, 8, 9, 40):
        e = rand(n, 300 + n, full_range=True)
        want = hashlib.blake2s(b"".join(int(v % O.P).to_bytes(8, "little") for v in e)).digest()
        assert H.digest_bytes(H.hash_into_leaf(e)) == want, n
    l, r = rand(4, 1), rand(4, 2)
    assert H.digest_bytes(H.hash_into_node(l, r)) == hashlib.blake2s(H.digest_bytes(l) + H.digest_bytes(r)).digest()


@pytest.mark.parametrize("c,e,cap", [(2, 4, 4), (2, 1, 16), (4, 8, 1), (2, 16, 8)])
def test_chunked_leaves(bj, c, e, cap):
    total = 1 << 12
    x = rand((c, total), c * e)
    t = bj.merkle.MerkleTreeWithCap.construct_by_chunking(bj.field.to_device(x), e, cap, hasher="blake2s")
    leaves, _, _, cap_ref = O.merkle_construct_by_chunking(x, e, cap, threads=THREADS, hasher="blake2s")
    eq(bj.field.to_host(t.leaf_hashes), leaves, "chunked leaves")
    eq(t.get_cap(), cap_ref, "chunked cap")


@pytest.mark.parametrize("splits", [(8, 13), (16, 16), (8, 8, 8, 1), (24, 0 + 8)])
def test_partial_ranges_equal_one_shot(bj, splits):
    torch = bj.torch
    c, nl = sum(splits), 1024
    x = rand((c, nl), c)
    src = bj.field.to_device(x)
    want = torch.empty((nl, 4), dtype=torch.int64, device="cuda")
    bj.call("bj_blake2s_leaves_d", src.data_ptr(), c, nl, nl, want.data_ptr(), 0)
    state = torch.empty((nl, 4), dtype=torch.int64, device="cuda")
    out = torch.empty((nl, 4), dtype=torch.int64, device="cuda")
    before = 0
    for i, k in enumerate(splits):
        last = i == len(splits) - 1
        bj.call("bj_blake2s_leaves_partial_d", src[before].data_ptr(), k, nl, nl, before,
                state.data_ptr() if before else None, (out if last else state).data_ptr(), 1 if last else 0, 0)
        before += k
    eq(bj.field.to_host(out), bj.field.to_host(want), "partial")


def test_partial_errors(bj):
    from boojum_amd import BoojumError
    with pytest.raises(BoojumError):
        bj.call("bj_blake2s_leaves_partial_d", None, 7, 16, 16, 0, None, None, 0, None)     # non-final, 7 cols
    with pytest.raises(BoojumError):
        bj.call("bj_blake2s_leaves_partial_d", None, 8, 16, 16, 4, None, None, 1, None)     # cols_before % 8
    with pytest.raises(BoojumError):
        bj.call("bj_blake2s_leaves_partial_d", None, 8, 16, 16, 8, None, None, 1, None)     # no state_in
    with pytest.raises(BoojumError):
        bj.call("bj_blake2s_nodes_d", None, 16, 16, None, None)                              # n_leaves == cap


def test_c5_non_recursive_witness_commit(bj):
    """C5 with the tree hasher the non-recursive sha256 prover uses (Blake2s256,
    gadgets/sha256/mod.rs:263-269): 93 witness columns of 2^16 rows, LDE x8, cap 16."""
    c, log_n, log_d, cap = 93, 16, 3, 16
    tr = bj.commit.synthetic_trace(c, log_n)
    ws = bj.commit.witness_commit(tr, 1 << log_d, cap, hasher="blake2s")
    bj.torch.cuda.synchronize()
    x = O.synthetic_trace(c, log_n)
    _, l_ref = O.lde(x, log_d, threads=THREADS)
    leaves, nodes, _, cap_ref = O.merkle_construct(l_ref.reshape(c, -1), cap, threads=THREADS, hasher="blake2s")
    eq(bj.field.to_host(ws.leaves), leaves, "leaves")
    eq(bj.field.to_host(ws.nodes), nodes, "nodes")
    eq(bj.field.to_host(ws.cap), cap_ref, "cap")


def test_c5_stage2_ext2_blake2s(bj):
    """Stage-2 (prover.rs:505-554) under the Blake2s tree: Ext2 (c0, c1) pairs, LDE x8, the
    first 8 cosets committed."""
    n = 1 << 12
    z = rand((2, n), 21)
    inter = rand((4, 2, n), 22)
    to = bj.field.to_device
    oc = bj.commit.second_stage_commit((to(z[0]), to(z[1])), [(to(a), to(b)) for a, b in inter], [], [], 8, 8, 16,
                                       hasher="blake2s")
    base = np.concatenate([z, inter.reshape(-1, n)])
    _, l_ref = O.lde(base, 3, threads=THREADS)
    _, _, _, cap_ref = O.merkle_construct(l_ref.reshape(base.shape[0], -1), 16, threads=THREADS, hasher="blake2s")
    eq(oc.get_cap(), cap_ref, "stage-2 cap")
