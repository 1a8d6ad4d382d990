"""GPU parity of the three-pass LDE (csrc/ntt_lde3.hip, 2^18 <= n <= 2^23) against the CPU oracle.

The path the reference takes (utils.rs:270-403: iFFT, then D coset FFTs of the same monomials,
fft/mod.rs:398-411, 659-734) must come out bit for bit: every size the three-pass form serves,
LDE degrees 2..32, ragged column counts, strided traces, non-canonical inputs, the monomial
scratch contract of bj_lde_d (c_j at bitrev_n(j), canonical), the monomial-source forward pass
(bj_lde_shard_d, G <= D) and the single-shift pass on folded sub-cosets (G > D).  The two-pass CT
path (BJ_LDE_PASSES=2, same binary) must agree with it."""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu
P = O.P


@pytest.fixture(scope="module")
def bj():
    return make_bj()


def make_bj():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    import boojum_amd
    from boojum_amd import field, lde
    boojum_amd.load()
    return type("BJ", (), dict(torch=torch, field=field, lde=lde))


def rand(shape, seed):
    return np.random.default_rng(seed).integers(0, P, size=shape, dtype=np.uint64)


def eq(a, b):
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    assert a.shape == b.shape, (a.shape, b.shape)
    bad = np.argwhere(a != b)
    assert bad.size == 0, "first mismatches at %s of %d" % (bad[:5].tolist(), len(bad))


def lde_d(bj, x, log_d, stride=None):
    """bj_lde_d on host array x (c, n); returns (lde (c, D, n), scratch (c, n))."""
    from boojum_amd._lib import call
    c, n = x.shape
    log_n = n.bit_length() - 1
    stride = stride or n
    big = np.zeros((c, stride), dtype=np.uint64)
    big[:, :n] = x
    t = bj.field.to_device(big)
    scratch = bj.torch.empty((c, n), dtype=bj.torch.int64, device="cuda")
    out = bj.torch.empty((c, 1 << log_d, n), dtype=bj.torch.int64, device="cuda")
    call("bj_lde_d", t.data_ptr(), c, stride, log_n, log_d, scratch.data_ptr(), out.data_ptr(), bj.field.stream_of(t))
    bj.torch.cuda.synchronize()
    return bj.field.to_host(out), bj.field.to_host(scratch)


@pytest.mark.parametrize("c,log_n,log_d", [(3, 18, 1), (1, 18, 4), (2, 19, 2), (3, 20, 3), (1, 21, 1), (2, 21, 2),
                                           (1, 22, 2), (1, 23, 1), (5, 18, 2), (1, 18, 5)])
def test_lde3_matches_oracle_and_keeps_monomials(bj, c, log_n, log_d):
    x = rand((c, 1 << log_n), 4000 + 10 * log_n + log_d)
    x[0, 0] = np.uint64(2**64 - 1)            # a non-canonical representative
    got, scratch = lde_d(bj, x, log_d)
    m_ref, l_ref = O.lde(x, log_d, threads=8)
    eq(got, l_ref.reshape(got.shape))
    # bj_lde_d's contract: the canonical monomials, c_j at bitrev_n(j)
    eq(scratch, np.stack([O.bitreverse(m_ref[i]) for i in range(c)]))


def test_lde3_strided_trace(bj):
    x = rand((3, 1 << 19), 4100)
    got, _ = lde_d(bj, x, 2, stride=(1 << 19) + 3 * 8192)
    eq(got, O.lde(x, 2, threads=8)[1].reshape(got.shape))


@pytest.mark.parametrize("log_n,log_d", [(20, 1), (22, 2)])
def test_lde3_equals_two_pass_path(bj, log_n, log_d):
    """Same binary, BJ_LDE_PASSES=2 (head + tail per transform) against the default three passes.
    The library reads its experiment knobs once per process and only under BJ_EXPERIMENTS=1
    (bj_internal.hpp), so the two-pass form runs in a child process and writes its LDE to a file."""
    import subprocess
    import sys
    import tempfile
    x = rand((4, 1 << log_n), 4200 + log_n)
    a, ma = lde_d(bj, x, log_d)
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    with tempfile.TemporaryDirectory() as td:
        np.save(os.path.join(td, "x.npy"), x)
        code = "\n".join([
            "import sys; sys.path[:0] = [%r, %r, %r, %r]" % (os.path.join(root, "oracle"),
                                                            os.path.join(root, "era-boojum_amd"), root, here),
            "import ctypes, numpy as np, test_gpu_lde3 as T",
            "bj = T.make_bj()",
            "from boojum_amd._lib import load",
            "v = ctypes.c_uint64(0); assert load().bj_experiment_knob(b'BJ_LDE_PASSES', ctypes.byref(v)) == 0",
            "assert v.value == 2, v.value",
            "l, m = T.lde_d(bj, np.load(%r), %d)" % (os.path.join(td, "x.npy"), log_d),
            "np.save(%r, l); np.save(%r, m)" % (os.path.join(td, "l.npy"), os.path.join(td, "m.npy")),
            "print('two-pass ok')"])
        env = dict(os.environ, BJ_EXPERIMENTS="1", BJ_LDE_PASSES="2")
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=200)
        assert r.returncode == 0 and "two-pass ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
        b, mb = np.load(os.path.join(td, "l.npy")), np.load(os.path.join(td, "m.npy"))
    eq(a, b)
    eq(ma, mb)


@pytest.mark.parametrize("log_n,log_d,log_g", [(18, 2, 0), (19, 3, 2), (21, 2, 1), (20, 1, 1), (19, 1, 3),
                                               (20, 2, 4)])
def test_lde3_shards(bj, log_n, log_d, log_g):
    """bj_lde_shard_d from bit-reversed monomials: whole cosets (G <= D, the monomial-source pass)
    and folded sub-cosets (G > D, one shift per shard, sizes down to 2^18)."""
    from boojum_amd._lib import call
    c, n = 3, 1 << log_n
    x = rand((c, n), 4300 + log_n)
    _, l_ref = O.lde(x, log_d, threads=8)
    l_ref = l_ref.reshape(c, -1)
    mono = bj.torch.empty((c, n), dtype=bj.torch.int64, device="cuda")
    t = bj.field.to_device(x)
    st = bj.field.stream_of(t)
    call("bj_lde_coeffs_d", t.data_ptr(), c, n, log_n, mono.data_ptr(), n, st)
    G = 1 << log_g
    m = (n << log_d) // G
    work = bj.torch.empty((c, m), dtype=bj.torch.int64, device="cuda") if G > (1 << log_d) else None
    for P_ in range(G):
        out = bj.torch.empty((c, m), dtype=bj.torch.int64, device="cuda")
        call("bj_lde_shard_d", mono.data_ptr(), c, n, log_n, log_d, log_g, P_,
             work.data_ptr() if work is not None else None, out.data_ptr(), st)
        bj.torch.cuda.synchronize()
        eq(bj.field.to_host(out), l_ref[:, P_ * m:(P_ + 1) * m])


def test_lde3_edge_columns(bj):
    """Zero / p-1 / impulse / all non-canonical columns through the three passes at D = 8."""
    n = 1 << 20
    x = np.zeros((4, n), dtype=np.uint64)
    x[1, :] = P - 1
    x[2, n // 2 + 1] = 1
    x[3, :] = np.uint64(2**64 - 1)
    got, scratch = lde_d(bj, x, 3)
    m_ref, l_ref = O.lde(x, 3, threads=8)
    eq(got, l_ref.reshape(got.shape))
    assert not got[0].any() and not scratch[0].any()


@pytest.mark.parametrize("log_n,log_d", [(18, 1), (20, 2), (22, 2), (23, 1), (17, 2)])
def test_lde_ex_without_monomials(bj, log_n, log_d):
    """bj_lde_ex_d without BJ_LDE_KEEP_MONOMIALS: the same LDE as bj_lde_d (the three-pass
    path then skips writing the monomials; other sizes keep their path); unknown flags refused."""
    from boojum_amd._lib import call, load
    c, n = 2, 1 << log_n
    x = rand((c, n), 4400 + log_n)
    want, _ = lde_d(bj, x, log_d)
    t = bj.field.to_device(x)
    scratch = bj.torch.empty((c, n), dtype=bj.torch.int64, device="cuda")
    out = bj.torch.empty((c, 1 << log_d, n), dtype=bj.torch.int64, device="cuda")
    call("bj_lde_ex_d", t.data_ptr(), c, n, log_n, log_d, scratch.data_ptr(), out.data_ptr(), 0,
         bj.field.stream_of(t))
    bj.torch.cuda.synchronize()
    eq(bj.field.to_host(out), want)
    assert load().bj_lde_ex_d(t.data_ptr(), c, n, log_n, log_d, scratch.data_ptr(), out.data_ptr(), 2,
                              bj.field.stream_of(t)) == -22
