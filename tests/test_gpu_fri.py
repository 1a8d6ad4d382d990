"""GPU FRI folding (fri/mod.rs:362-682) against the oracle's restatement, bit-exact, and the
low-degree property the reference debug-asserts after every fold (fri/mod.rs:556-571): folding
the coset LDE of a degree-< n polynomial gives, after interpolation on the squared coset, zeros
above n / 2^k."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bj():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import boojum_amd
    from boojum_amd import field, fri
    boojum_amd.load()
    return type("BJ", (), dict(torch=torch, field=field, fri=fri))


def rand(shape, seed):
    return np.random.default_rng(seed).integers(0, O.P, size=shape, dtype=np.uint64)


@pytest.mark.parametrize("log_n", [1, 4, 11])
def test_single_fold_matches_oracle(bj, log_n):
    n = 1 << log_n
    c0, c1 = rand(n, 1), rand(n, 2)
    roots = O.precompute_twiddles(log_n, True)
    ci, ch = O.gl_inv(7), (int(rand(1, 3)[0]), int(rand(1, 4)[0]))
    d0, d1 = bj.fri.fold(bj.field.to_device(c0), bj.field.to_device(c1), bj.field.to_device(roots), ci, ch)
    w0, w1 = O.fri_fold(c0, c1, roots, ci, ch)
    assert np.array_equal(bj.field.to_host(d0), w0)
    assert np.array_equal(bj.field.to_host(d1), w1)


def test_folding_schedule_keeps_low_degree(bj):
    """A degree < n Ext2 polynomial's LDE (D = 4) folded 3 times is a degree < n/8 polynomial
    on the coset (7^-1)^(-8) ... i.e. the reference's debug check passes."""
    log_n, log_d = 8, 2
    n = 1 << log_n
    full = n << log_d
    x0, x1 = rand(n, 5), rand(n, 6)
    _, l0 = O.lde(x0[None, :], log_d)
    _, l1 = O.lde(x1[None, :], log_d)
    c0, c1 = l0.reshape(-1), l1.reshape(-1)
    roots_h = O.precompute_twiddles(log_n + log_d, True)
    chs = bj.fri.challenge_powers((123456789, 987654321), 3)
    roots = bj.fri.precompute_roots(full)
    assert np.array_equal(bj.field.to_host(roots), roots_h)
    g0, g1, ci = bj.fri.interpolate(bj.field.to_device(c0), bj.field.to_device(c1), chs, roots)
    # oracle chain
    w0, w1, cio = c0, c1, O.gl_inv(7)
    for ch in chs:
        w0, w1 = O.fri_fold(w0, w1, roots_h, cio, ch)
        cio = cio * cio % O.P
    assert ci == cio
    assert np.array_equal(bj.field.to_host(g0), w0)
    assert np.array_equal(bj.field.to_host(g1), w1)
    # the reference's debug assertion: bitreverse + iFFT on coset 1/ci leaves degree < len / D
    for w in (w0, w1):
        mono = O.ifft_natural_to_natural(O.bitreverse(w), O.gl_inv(ci))
        assert not mono[len(mono) >> log_d:].any()


def test_gpu_fold_reproduces_proof_json_fri_chain(bj):
    """bj_fri_fold_d on the reference's own FRI data: for the first six queries of proof.json,
    every committed FRI leaf (8 Ext2 values) folded three times by 2 on the GPU -- with the
    transcript-derived challenges (oracle/transcript.py replays the verifier's Poseidon2
    transcript), the full-domain inverse twiddles at the leaf's flat pair indices and the coset
    inverse of that step -- equals the value the next oracle commits, and the last step's equals
    final_fri_monomials at the folded point (verifier.rs:2396-2518)."""
    import json
    import os
    import transcript as T
    torch = bj.torch
    fx = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "proof_fri.json")))
    rep = T.replay(fx)
    n = fx["vk"]["domain_size"] * fx["proof_config"]["fri_lde_factor"]
    roots = bj.fri.precompute_roots(n)
    for q in rep["queries"]:
        steps = q["steps"]
        for k, st in enumerate(steps):
            leaf = [int(v) for v in st["leaf"]]
            deg = len(leaf) // 2
            c0 = bj.field.to_device(np.array(leaf[:deg], dtype=np.uint64))
            c1 = bj.field.to_device(np.array(leaf[deg:], dtype=np.uint64))
            base, ci = st["tree_idx"] * deg // 2, st["coset_inverse"]
            for ch in st["challenges"]:
                c0, c1 = bj.fri.fold(c0, c1, roots[base:], ci, ch)
                base //= 2
                ci = ci * ci % O.P
            got = (int(bj.field.to_host(c0)[0]), int(bj.field.to_host(c1)[0]))
            want = steps[k + 1]["expected"] if k + 1 < len(steps) else q["final"]
            assert got == want, "query %d step %d" % (q["index"], k)
