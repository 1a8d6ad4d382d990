"""GPU parity: the HIP path (through the C ABI) against the CPU oracle, bit-exact.

Sizes are ones the oracle finishes in seconds.  Full-size (BASELINE configs) checks are
in test_gpu_fullsize.py.  Edge cases follow what the reference's tests and asserts
cover: ragged column counts (leaf lengths not multiples of the rate 8), n = 1 and 2,
non-canonical inputs, all-zero / all-(p-1) / impulse columns, every LDE degree used.
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

P = O.P


@pytest.fixture(scope="module")
def bj():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import boojum_amd
    from boojum_amd import commit, fft, field, lde, merkle
    boojum_amd.load()
    return type("BJ", (), dict(torch=torch, fft=fft, field=field, lde=lde, merkle=merkle, commit=commit))


def rand(shape, seed):
    return np.random.default_rng(seed).integers(0, P, size=shape, dtype=np.uint64)


def eq(a, b):
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    assert a.shape == b.shape, (a.shape, b.shape)
    bad = np.argwhere(a != b)
    assert bad.size == 0, "first mismatches at %s" % bad[:5].tolist()


# -------------------------------------------------------------- Poseidon2

def test_permutation_kats(bj):
    s = bj.merkle.Poseidon2Sponge.poseidon2_permutation(np.arange(12))
    assert [int(x) for x in s[:4]] == [0x5d82c16b87f07f98, 0x3655af22bb2f037d, 0x82c1535dfb4bdf90,
                                       0x4d318cfdafd2378e]


def test_permutation_batch_random_and_edge(bj):
    st = rand((4096, 12), 1)
    st[0] = 0
    st[1] = P - 1
    st[2] = np.uint64(2**64 - 1)  # non-canonical representative
    st[3, :] = np.arange(12, dtype=np.uint64) + np.uint64(P)
    t = bj.field.to_device(st)
    from boojum_amd._lib import call
    call("bj_poseidon2_permute_d", t.data_ptr(), st.shape[0], bj.field.stream_of(t))
    got = bj.field.to_host(t)
    want = np.stack([O.poseidon2_permutation(np.array([int(x) % P for x in row], dtype=np.uint64)) for row in st])
    eq(got, want)


@pytest.mark.parametrize("n", [0, 1, 3, 7, 8, 9, 16, 58, 156, 167, 256, 257])
def test_hash_into_leaf(bj, n):
    x = rand(n, n + 100)
    eq(bj.merkle.Poseidon2Sponge.hash_into_leaf(x), O.hash_into_leaf(x))


def test_hash_into_node(bj):
    l, r = rand(4, 1), rand(4, 2)
    eq(bj.merkle.Poseidon2Sponge.hash_into_node(l, r), O.hash_into_node(l, r))


def test_proof_json_paths_verify_on_gpu(bj):
    import json
    import os
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "proof_queries.json")))
    T = bj.merkle.MerkleTreeWithCap
    for q in fx["queries"][:3]:
        for name in ("witness", "stage_2", "quotient", "setup"):
            e = q[name]
            leaf = bj.merkle.Poseidon2Sponge.hash_into_leaf(e["leaf_elements"])
            assert T.verify_proof_over_cap(e["proof"], fx["caps"][name], leaf, q["index"])


# -------------------------------------------------------------------- FFT

@pytest.mark.parametrize("log_n", [1, 2, 3, 5, 8, 12, 13, 16, 17])
def test_twiddles(bj, log_n):
    for inv in (False, True):
        t = bj.fft.precompute_twiddles_for_fft(1 << log_n, inverse=inv)
        eq(bj.field.to_host(t), O.precompute_twiddles(log_n, inv))


@pytest.mark.parametrize("log_n", [0, 1, 2, 4, 7, 11, 12, 13, 14, 15, 16, 17, 18, 20, 21, 23])
def test_fft_natural_to_bitreversed_batch(bj, log_n):
    c = 3 if log_n < 18 else 1
    x = rand((c, 1 << log_n), log_n)
    x[0, 0] = np.uint64(2**64 - 1)  # non-canonical input
    for coset in (1, 7, 0x1234567):
        t = bj.field.to_device(x)
        bj.fft.fft_natural_to_bitreversed(t, coset)
        want = np.stack([O.fft_natural_to_bitreversed(x[i], coset) for i in range(c)])
        eq(bj.field.to_host(t), want)


@pytest.mark.parametrize("log_n", [0, 1, 2, 3, 6, 10, 12, 13, 14, 15, 16, 17, 18, 19, 22, 23])
def test_ifft_natural_to_natural_batch(bj, log_n):
    x = rand((2, 1 << log_n), 50 + log_n)
    for coset in (1, 7):
        t = bj.field.to_device(x)
        bj.fft.ifft_natural_to_natural(t, coset)
        want = np.stack([O.ifft_natural_to_natural(x[i], coset) for i in range(2)])
        eq(bj.field.to_host(t), want)


@pytest.mark.parametrize("log_n", [1, 2, 5, 12, 20])
def test_twiddles_natural_and_bitreverse(bj, log_n):
    """precompute_twiddles_for_fft_natural = the bit-reversed table put back in natural order
    (utils.rs:117-122 vs :127-155); bitreverse_enumeration_inplace is a pure permutation
    (non-canonical values are moved unchanged)."""
    n = 1 << log_n
    for inv in (False, True):
        nat = bj.field.to_host(bj.fft.precompute_twiddles_for_fft_natural(n, inv))
        ref_br = O.precompute_twiddles(log_n, inv)
        eq(nat, O.bitreverse(ref_br) if log_n > 1 else ref_br)
    x = np.random.default_rng(log_n).integers(0, 2**64 - 1, size=(3, n), dtype=np.uint64, endpoint=True)
    t = bj.field.to_device(x)
    bj.fft.bitreverse_enumeration_inplace(t)
    eq(bj.field.to_host(t), np.stack([O.bitreverse(r) for r in x]))


def test_distribute_powers(bj):
    x = rand((2, 1 << 14), 5)
    t = bj.field.to_device(x)
    bj.fft.distribute_powers(t, 0xdeadbeef)
    eq(bj.field.to_host(t), np.stack([O.distribute_powers(x[i], 0xdeadbeef) for i in range(2)]))


def test_host_seam_in_place(bj):
    x = rand(1 << 10, 9)
    y = x.copy()
    bj.fft.fft_natural_to_bitreversed_host(y, 7)
    eq(y, O.fft_natural_to_bitreversed(x, 7))
    z = x.copy()
    bj.fft.ifft_natural_to_natural_host(z, 1)
    eq(z, O.ifft_natural_to_natural(x, 1))
    w = x.copy()
    bj.fft.distribute_powers_host(w, 11)
    eq(w, O.distribute_powers(x, 11))
    eq(bj.fft.precompute_twiddles_for_fft_host(1 << 10, True), O.precompute_twiddles(10, True))


def test_host_seams_concurrent_threads(bj):
    """The PrimeFieldLikeVectorized seam is driven from rayon worker threads, one column per
    call, in place and concurrently (utils.rs:295-304, 363-379). 8 host threads call the
    per-column seams at once (ctypes drops the GIL), on sizes 2^10..2^19 and both NTT paths,
    with first-use table creation racing; every result must equal the oracle's."""
    from concurrent.futures import ThreadPoolExecutor
    jobs = []
    for k in range(24):
        log_n = (10, 14, 18, 19)[k % 4]
        x = rand(1 << log_n, 1000 + k)
        coset = (1, 7, 11, 0x1234567)[k % 4]
        jobs.append((k, x, coset))

    def run(job):
        k, x, coset = job
        y = x.copy()
        if k % 2 == 0:
            bj.fft.fft_natural_to_bitreversed_host(y, coset)
            return y, O.fft_natural_to_bitreversed(x, coset)
        bj.fft.ifft_natural_to_natural_host(y, coset)
        return y, O.ifft_natural_to_natural(x, coset)

    with ThreadPoolExecutor(8) as ex:
        for got, want in ex.map(run, jobs):
            eq(got, want)


# -------------------------------------------------------------------- LDE

@pytest.mark.parametrize("c,log_n,log_d", [(1, 0, 1), (2, 1, 1), (3, 3, 2), (5, 6, 3), (4, 12, 1), (3, 13, 2),
                                           (3, 14, 3), (5, 15, 1), (1, 16, 2), (7, 13, 3),
                                           (2, 16, 3), (1, 17, 1), (2, 18, 2), (1, 19, 3), (1, 20, 1),
                                           (2, 22, 2)])
def test_lde_batch(bj, c, log_n, log_d):
    x = rand((c, 1 << log_n), c * 100 + log_n)
    t = bj.field.to_device(x)
    l = bj.lde.transform_raw_storages_to_lde(t, 1 << log_d)
    m_ref, l_ref = O.lde(x, log_d, threads=4)
    eq(bj.field.to_host(l), l_ref)
    # monomials path: iFFT natural->natural then monomials -> LDE
    m = bj.field.to_device(x)
    bj.fft.ifft_natural_to_natural(m, 1)
    eq(bj.field.to_host(m), m_ref)
    eq(bj.field.to_host(bj.lde.transform_monomials_to_lde(m, 1 << log_d)), l_ref)


@pytest.mark.parametrize("c,log_n,log_d", [(2, 10, 4), (1, 14, 4), (1, 13, 5), (1, 12, 5), (1, 15, 5)])
def test_lde_high_degree(bj, c, log_n, log_d):
    """LDE factors 16 and 32 (used_lde_degree = max(fri_lde_factor, quotient_degree),
    prover.rs:313, is not bounded by 8), on both NTT paths."""
    x = rand((c, 1 << log_n), 7 * log_d + log_n)
    l = bj.lde.transform_raw_storages_to_lde(bj.field.to_device(x), 1 << log_d)
    eq(bj.field.to_host(l), O.lde(x, log_d, threads=4)[1])


@pytest.mark.slow
@pytest.mark.parametrize("log_n", [24, 25, 26])
def test_transforms_past_2_23(bj, log_n):
    """Columns longer than 2^23: the CT passes run a small head over the whole column, the
    R = 10 head on each 2^23-word sub-column, then the tail (launch_ct): forward with a coset,
    inverse, and an LDE x2, one column each."""
    x = rand((1, 1 << log_n), 300 + log_n)
    t = bj.field.to_device(x)
    bj.fft.fft_natural_to_bitreversed(t, 7)
    eq(bj.field.to_host(t)[0], O.fft_natural_to_bitreversed(x[0], 7))
    t = bj.field.to_device(x)
    bj.fft.ifft_natural_to_natural(t, 1)
    eq(bj.field.to_host(t)[0], O.ifft_natural_to_natural(x[0], 1))
    if log_n == 24:
        l = bj.lde.transform_raw_storages_to_lde(bj.field.to_device(x), 2)
        eq(bj.field.to_host(l), O.lde(x, 1, threads=8)[1])


@pytest.mark.slow
@pytest.mark.parametrize("log_n", [27, 28])
def test_transforms_past_2_26(bj, log_n):
    """Columns of 2^27 and 2^28 words (the multi-pass DIF network, ntt_dif.hip), where the oracle
    does not finish in seconds, checked by closed forms and a round trip: x = e_1 + 5 e_3 gives
    X_k = c w^k + 5 (c w^k)^3 at bit-reversed position bitrev(k) (4096 sampled positions, coset
    c = 7), and a device-made random column goes forward (coset 7), back to natural order and
    through the inverse (coset 7) to itself, bit-exact."""
    torch = bj.torch
    n, c = 1 << log_n, 7
    w = O.domain_generator(log_n)
    x = torch.zeros((1, n), dtype=torch.int64, device="cuda")
    x[0, 1], x[0, 3] = 1, 5
    bj.fft.fft_natural_to_bitreversed(x, c)
    pos = np.random.default_rng(log_n).integers(0, n, 4096)
    got = bj.field.to_host(x[0, torch.from_numpy(pos).cuda()])
    want = []
    for i in pos.tolist():
        k = int(format(i, "0%db" % log_n)[::-1], 2)
        y = O.gl_mul(c, O.gl_pow(w, k))
        want.append(O.gl_add(y, O.gl_mul(5, O.gl_pow(y, 3))))
    eq(got, np.array(want, dtype=np.uint64))
    del x
    t = bj.commit.synthetic_trace(1, log_n, seed=log_n)
    ref = t.clone()
    bj.fft.fft_natural_to_bitreversed(t, c)
    bj.fft.bitreverse_enumeration_inplace(t)
    bj.fft.ifft_natural_to_natural(t, c)
    assert torch.equal(t, ref), "round trip differs"


@pytest.mark.parametrize("log_n", [0, 1, 5, 12, 17, 18, 21])
def test_lde_coeffs_exchange_format(bj, log_n):
    """bj_lde_coeffs_d: monomials c_j at bitrev_n(j), canonical (the multi-GPU exchange format)."""
    from boojum_amd._lib import call
    c = 2
    x = rand((c, 1 << log_n), 900 + log_n)
    x[0, 0] = np.uint64(2**64 - 1)
    t = bj.field.to_device(x)
    out = bj.torch.empty_like(t)
    call("bj_lde_coeffs_d", t.data_ptr(), c, 1 << log_n, log_n, out.data_ptr(), 1 << log_n, bj.field.stream_of(out))
    want = np.stack([O.bitreverse(O.ifft_natural_to_natural(x[i])) for i in range(c)])
    eq(bj.field.to_host(out), want)


@pytest.mark.parametrize("log_n,log_d", [(18, 1), (18, 3), (22, 2), (23, 1)])
def test_lde_edge_columns_large(bj, log_n, log_d):
    """Zero / p-1 / impulse / non-canonical columns on the register-resident NTT sizes."""
    n = 1 << log_n
    x = np.zeros((4, n), dtype=np.uint64)
    x[1, :] = P - 1
    x[2, n - 1] = 1
    x[3, :] = np.uint64(2**64 - 1)
    t = bj.field.to_device(x)
    l = bj.field.to_host(bj.lde.transform_raw_storages_to_lde(t, 1 << log_d))
    m_ref, l_ref = O.lde(x, log_d, threads=8)
    eq(l, l_ref)
    assert not l[0].any()


def test_lde_edge_columns(bj):
    n = 1 << 10
    x = np.zeros((4, n), dtype=np.uint64)
    x[1, :] = P - 1
    x[2, 5] = 1
    x[3, :] = np.uint64(2**64 - 1)  # all non-canonical (== 2^32 - 2 mod p)
    t = bj.field.to_device(x)
    l = bj.lde.transform_raw_storages_to_lde(t, 4)
    m_ref, l_ref = O.lde(x, 2)
    eq(bj.field.to_host(l), l_ref)
    assert not bj.field.to_host(l)[0].any()


def test_lde_with_strided_trace(bj):
    # trace columns inside a wider buffer (col_stride > n)
    x = rand((3, 1 << 11), 77)
    big = np.zeros((3, 3 << 11), dtype=np.uint64)
    big[:, : 1 << 11] = x
    t = bj.field.to_device(big)[:, : 1 << 11]
    l = bj.lde.transform_raw_storages_to_lde(t, 2)
    m_ref, l_ref = O.lde(x, 1)
    eq(bj.field.to_host(l), l_ref)


# ------------------------------------------------------------------ Merkle

@pytest.mark.parametrize("c,nl,cap", [(1, 2, 1), (5, 64, 4), (8, 1024, 16), (13, 4096, 1), (33, 1 << 13, 16),
                                      (16, 1 << 14, 2048), (7, 1 << 9, 1), (3, 1 << 16, 256), (4, 1 << 17, 16),
                                      (2, 1 << 18, 1)])
def test_merkle_tree(bj, c, nl, cap):
    src = rand((c, nl), c + nl)
    t = bj.field.to_device(src)
    tree = bj.merkle.MerkleTreeWithCap.construct(t, cap)
    leaves, nodes, levels, capr = O.merkle_construct(src, cap, threads=4)
    eq(bj.field.to_host(tree.leaf_hashes), leaves)
    eq(bj.field.to_host(tree.nodes), nodes)
    eq(tree.get_cap(), capr)
    for idx in (0, nl - 1, nl // 3):
        leaf, path = tree.get_proof(idx)
        assert bj.merkle.MerkleTreeWithCap.verify_proof_over_cap(path, tree.get_cap(), leaf, idx)


@pytest.mark.parametrize("knob,value", [("BJ_NODE_Q4_MAX", "0"), ("BJ_NODE_FUSED", "0")])
def test_node_levels_one_per_lane(bj, knob, value):
    """BJ_NODE_Q4_MAX=0 keeps one node per lane for every level and the one-workgroup tail (the
    form the quad kernel replaces on small levels, poseidon2_quad.hpp); BJ_NODE_FUSED=0 runs each
    small level as its own quad-lane grid instead of up to 8 levels per launch
    (node_levels_q4_kernel).  Every form must give the reference's tree.  A child process, since
    the library reads the variables once (and only under BJ_EXPERIMENTS=1)."""
    import os
    import subprocess
    import sys
    code = (
        "import numpy as np, oracle as O\n"
        "from boojum_amd import field, merkle\n"
        "src = np.random.default_rng(5).integers(0, O.P, size=(9, 1 << 15), dtype=np.uint64)\n"
        "import ctypes; from boojum_amd._lib import load\n"
        "v = ctypes.c_uint64(9); assert load().bj_experiment_knob(%r, ctypes.byref(v)) == 0\n"
        "assert v.value == 0, v.value\n"
        "for cap in (1, 16, 512):\n"
        "    tree = merkle.MerkleTreeWithCap.construct(field.to_device(src), cap)\n"
        "    leaves, nodes, levels, capr = O.merkle_construct(src, cap, threads=4)\n"
        "    assert np.array_equal(field.to_host(tree.nodes), nodes), cap\n"
        "    assert np.array_equal(tree.get_cap(), capr), cap\n"
        "print('lane-form tree ok')\n") % knob.encode()
    env = dict(os.environ, BJ_EXPERIMENTS="1", **{knob: value})
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(root, "era-boojum_amd"), os.path.join(root, "oracle"),
                                         env.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "lane-form tree ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("c,splits", [(16, [8]), (37, [8, 24]), (256, [64, 128, 192]), (9, [8]), (24, [16])])
def test_leaves_partial_chain_equals_full(bj, c, splits):
    """bj_merkle_leaves_partial_d over column ranges, carrying the capacity, == bj_merkle_leaves_d."""
    from boojum_amd._lib import call
    nl = 1000
    src = rand((c, nl), c * 7 + len(splits))
    t = bj.field.to_device(src)
    st = bj.field.stream_of(t)
    full = bj.torch.empty((nl, 4), dtype=bj.torch.int64, device=t.device)
    call("bj_merkle_leaves_d", t.data_ptr(), c, nl, nl, full.data_ptr(), st)
    state = bj.torch.empty((nl, 4), dtype=bj.torch.int64, device=t.device)
    out = bj.torch.empty((nl, 4), dtype=bj.torch.int64, device=t.device)
    bounds = [0] + splits + [c]
    for i in range(len(bounds) - 1):
        a, b = bounds[i], bounds[i + 1]
        last = i == len(bounds) - 2
        call("bj_merkle_leaves_partial_d", t[a:b].data_ptr(), b - a, nl, nl, None if i == 0 else state.data_ptr(),
             (out if last else state).data_ptr(), 1 if last else 0, st)
    eq(bj.field.to_host(out), bj.field.to_host(full))
    want = np.stack([O.hash_into_leaf(np.ascontiguousarray(src[:, r])) for r in (0, 1, nl - 1)])
    eq(bj.field.to_host(out)[[0, 1, nl - 1]], want)


def test_leaves_partial_rejects_ragged_middle(bj):
    from boojum_amd import BoojumError
    from boojum_amd._lib import call
    with pytest.raises(BoojumError):
        call("bj_merkle_leaves_partial_d", None, 7, 1, 1, None, None, 0, None)


@pytest.mark.parametrize("c,total,e,cap", [(2, 1 << 12, 8, 32), (2, 1 << 10, 16, 1), (3, 1 << 9, 1, 4), (1, 64, 2, 8),
                                           (2, 256, 8, 32), (5, 1 << 11, 4, 16)])
def test_construct_by_chunking_flat(bj, c, total, e, cap):
    """FRI oracles' trees (fri/mod.rs:179-187, 258-266), incl. tree_size == cap_size."""
    src = rand((c, total), c * 31 + e)
    t = bj.field.to_device(src)
    T = bj.merkle.MerkleTreeWithCap
    nl = total // e
    tree = T.construct_by_chunking_from_flat_sources(t, e, cap)
    leaves, nodes, levels, capr = O.merkle_construct_by_chunking(src, e, cap, threads=4)
    eq(bj.field.to_host(tree.leaf_hashes), leaves)
    eq(tree.get_cap(), capr)
    if nl > cap:
        eq(bj.field.to_host(tree.nodes), nodes)
        tree2 = T.construct_by_chunking(t, e, cap)
        eq(tree2.get_cap(), capr)
        leaf, path = tree.get_proof(nl - 1)
        assert T.verify_proof_over_cap(path, tree.get_cap(), leaf, nl - 1)


def test_construct_by_chunking_over_lde_cosets(bj):
    """construct_by_chunking over a (C, D, n) LDE: the flat leaf index runs over the cosets."""
    x = rand((2, 1 << 10), 55)
    t = bj.field.to_device(x)
    l = bj.lde.transform_raw_storages_to_lde(t, 4)
    tree = bj.merkle.MerkleTreeWithCap.construct_by_chunking(l, 8, 16)
    _, l_ref = O.lde(x, 2)
    leaves, nodes, levels, capr = O.merkle_construct_by_chunking(l_ref.reshape(2, -1), 8, 16)
    eq(bj.field.to_host(tree.leaf_hashes), leaves)
    eq(tree.get_cap(), capr)


def test_fri_base_oracle_leaves_from_fixture_on_gpu(bj):
    """The proof.json FRI base-oracle leaves (8 elements of c0 then 8 of c1) hashed by the
    chunked leaf kernel verify against the committed FRI cap."""
    import json
    import os
    from boojum_amd._lib import call
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "proof_queries.json")))
    T = bj.merkle.MerkleTreeWithCap
    for q in fx["queries"]:
        f = q["fri_base"]
        el = np.array(f["leaf_elements"], dtype=np.uint64).reshape(2, 8)   # sources c0, c1
        t = bj.field.to_device(el)
        out = bj.torch.empty((1, 4), dtype=bj.torch.int64, device=t.device)
        call("bj_merkle_leaves_chunked_d", t.data_ptr(), 2, 8, 1, 8, out.data_ptr(), bj.field.stream_of(t))
        leaf = bj.field.to_host(out)[0]
        assert T.verify_proof_over_cap(f["proof"], fx["caps"]["fri_base"], leaf, f["index"])


# --------------------------------------------------------------- commit

@pytest.mark.parametrize("c,log_n,log_d,cap,log_k", [
    (32, 16, 1, 16, 1), (7, 10, 2, 8, 2), (9, 9, 3, 16, 3), (1, 4, 1, 2, 1),
    # LDE at D, tree over the first k < D cosets through one call (prover.rs:313-347)
    (16, 14, 3, 32, 1),   # proof.json's ratio: D = 8 (quotient degree), k = 2 (fri_lde_factor), cap 32
    (12, 13, 2, 16, 0),   # D = 4, k = 1
])
def test_witness_commit_matches_oracle(bj, c, log_n, log_d, cap, log_k):
    """Config 1 (2^16 x 32, LDE 2, cap 16) end to end, plus ragged shapes and k < D."""
    tr_np = O.synthetic_trace(c, log_n)
    tr = bj.commit.synthetic_trace(c, log_n)
    eq(bj.field.to_host(tr), tr_np)
    ws = bj.commit.witness_commit(tr, 1 << log_d, cap, fri_lde_factor=1 << log_k)
    ref = O.lde_commit(tr_np, log_d, cap, threads=8, log_k=log_k)
    eq(bj.field.to_host(ws.lde), ref["lde"])
    eq(bj.field.to_host(ws.leaves), ref["leaves"])
    eq(bj.field.to_host(ws.nodes), ref["nodes"])
    eq(bj.field.to_host(ws.cap), ref["cap"])


@pytest.mark.parametrize("c,log_n,log_d,log_k", [(24, 18, 2, 1), (5, 12, 1, 1)])
def test_lde_commit_ex_flags(bj, c, log_n, log_d, log_k):
    """bj_lde_commit_ex_d (ABI 2.4): flags 0 commits like bj_lde_commit_d without writing the
    monomials back (three-pass size and a two-pass one); BJ_LDE_KEEP_MONOMIALS leaves them in
    scratch as bj_lde_d does; unknown flags are refused."""
    import ctypes
    from boojum_amd._lib import call, load
    torch = bj.torch
    cap = 16
    n, D = 1 << log_n, 1 << log_d
    nl = n << log_k
    tr_np = O.synthetic_trace(c, log_n)
    tr = bj.commit.synthetic_trace(c, log_n)
    ref = O.lde_commit(tr_np, log_d, cap, threads=8, log_k=log_k)
    st = bj.field.stream_of(tr)
    for flags in (0, 1):
        scratch = torch.zeros((c, n), dtype=torch.int64, device="cuda")
        lde = torch.empty((c, D, n), dtype=torch.int64, device="cuda")
        leaves = torch.empty((nl, 4), dtype=torch.int64, device="cuda")
        nodes = torch.empty((nl - cap, 4), dtype=torch.int64, device="cuda")
        capo = np.zeros((cap, 4), dtype=np.uint64)
        call("bj_lde_commit_ex_d", tr.data_ptr(), c, n, log_n, log_d, log_k, cap, scratch.data_ptr(), lde.data_ptr(),
             leaves.data_ptr(), nodes.data_ptr(), capo.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), flags, st)
        torch.cuda.synchronize()
        eq(bj.field.to_host(lde), ref["lde"])
        eq(bj.field.to_host(leaves), ref["leaves"])
        eq(bj.field.to_host(nodes), ref["nodes"])
        eq(capo, ref["cap"])
        if flags:
            m_ref, _ = O.lde(tr_np, log_d, threads=8)
            eq(bj.field.to_host(scratch), np.stack([O.bitreverse(m_ref[i]) for i in range(c)]))
    assert load().bj_lde_commit_ex_d(tr.data_ptr(), c, n, log_n, log_d, log_k, cap, scratch.data_ptr(),
                                     lde.data_ptr(), leaves.data_ptr(), nodes.data_ptr(), None, 2, st) == -22


@pytest.mark.parametrize("c,log_n,log_d,cap,log_k", [(5, 8, 2, 4, 2), (70, 10, 1, 16, 1), (64, 12, 2, 8, 2),
                                                     (33, 14, 3, 16, 3), (40, 14, 3, 32, 1), (20, 12, 2, 16, 0)])
def test_commit_host_abi_matches(bj, c, log_n, log_d, cap, log_k):
    """bj_lde_commit_h: the column-chunked host pipeline (32-column chunks: one ragged, several
    full, and a 1-column tail) equals the oracle's one-shot commit, also with the tree over the
    first k < D cosets (D = 8 / k = 2 / cap 32, proof.json's ratio; D = 4 / k = 1)."""
    import ctypes
    from boojum_amd._lib import call
    tr = O.synthetic_trace(c, log_n)
    nl = 1 << (log_n + log_k)
    lde = np.zeros((c, 1 << log_d, 1 << log_n), dtype=np.uint64)
    leaves = np.zeros((nl, 4), dtype=np.uint64)
    nodes = np.zeros((nl - cap, 4), dtype=np.uint64)
    capo = np.zeros((cap, 4), dtype=np.uint64)
    p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))  # noqa: E731
    call("bj_lde_commit_h", p(np.ascontiguousarray(tr)), c, log_n, log_d, log_k, cap, p(lde), p(leaves), p(nodes),
         p(capo))
    ref = O.lde_commit(tr, log_d, cap, threads=8, log_k=log_k)
    eq(lde, ref["lde"])
    eq(leaves, ref["leaves"])
    eq(nodes, ref["nodes"])
    eq(capo, ref["cap"])


def test_release_workspace_between_host_commits(bj):
    """bj_release_workspace (ABI 2.1) trims the library's pool after a host commit; the next
    commit re-allocates its workspace and is still bit-exact."""
    import ctypes
    from boojum_amd._lib import call, load
    assert load().bj_abi_version() == (2 << 16) | 6
    c, log_n, log_d, cap = 40, 14, 2, 16
    tr = O.synthetic_trace(c, log_n)
    ref = O.lde_commit(tr, log_d, cap, threads=8)
    p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))  # noqa: E731
    for _ in range(2):
        nl = 1 << (log_n + log_d)
        lde = np.zeros((c, 1 << log_d, 1 << log_n), dtype=np.uint64)
        leaves = np.zeros((nl, 4), dtype=np.uint64)
        nodes = np.zeros((nl - cap, 4), dtype=np.uint64)
        capo = np.zeros((cap, 4), dtype=np.uint64)
        call("bj_lde_commit_h", p(np.ascontiguousarray(tr)), c, log_n, log_d, log_d, cap, p(lde), p(leaves),
             p(nodes), p(capo))
        call("bj_release_workspace")
        eq(lde, ref["lde"])
        eq(capo, ref["cap"])


def test_release_tables_then_rebuild(bj):
    """bj_release_tables (ABI 2.3) frees every cached table; the next calls rebuild them: the LDE
    of both forms (three-pass at 2^18, two-pass CT at 2^14) and a commit stay bit-exact."""
    from boojum_amd._lib import call
    from boojum_amd import commit, field
    for c, log_n, log_d in ((3, 18, 2), (5, 14, 1)):
        ref = O.lde_commit(O.synthetic_trace(c, log_n), log_d, 16, threads=8)
        for _ in range(2):
            tr = commit.synthetic_trace(c, log_n)
            ws = commit.witness_commit(tr, 1 << log_d, 16)
            bj.torch.cuda.synchronize()
            eq(field.to_host(ws.lde), ref["lde"])
            eq(field.to_host(ws.cap), ref["cap"])
            del ws, tr
            call("bj_release_tables")


def test_errors_are_loud(bj):
    from boojum_amd import BoojumError
    t = bj.torch.zeros((2, 24), dtype=bj.torch.int64, device="cuda")
    with pytest.raises((BoojumError, ValueError)):
        bj.fft.fft_natural_to_bitreversed(t, 1)
    with pytest.raises((BoojumError, ValueError)):
        bj.lde.transform_raw_storages_to_lde(bj.torch.zeros((2, 16), dtype=bj.torch.int64, device="cuda"), 1)
    with pytest.raises((BoojumError, ValueError)):
        bj.merkle.MerkleTreeWithCap.construct(bj.torch.zeros((2, 16), dtype=bj.torch.int64, device="cuda"), 16)
