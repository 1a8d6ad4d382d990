"""The CPU baseline's AVX-512 leaf hashing (oracle/baseline_avx512.c, bench.py cpu_baseline) gives
exactly the scalar oracle's leaves -- every sponge padding case and non-canonical inputs."""
import numpy as np
import pytest

import oracle as O


@pytest.mark.parametrize("n_cols", [0, 1, 7, 8, 9, 16, 19, 32])
def test_avx512_leaves_equal_scalar(n_cols):
    if not O.avx512_available():
        pytest.skip("host without AVX-512")
    rng = np.random.default_rng(n_cols)
    x = rng.integers(0, 2 ** 64 - 1, size=(max(n_cols, 1), 64), dtype=np.uint64, endpoint=True)[:n_cols]
    x[:, :3] = np.uint64(0xFFFFFFFFFFFFFFFF)     # non-canonical words
    if n_cols == 0:
        x = np.zeros((0, 64), dtype=np.uint64)
    got = O.merkle_leaves_avx512(x if n_cols else np.zeros((1, 64), np.uint64)[:0].reshape(0, 64), threads=3)
    want = np.stack([O.hash_into_leaf(np.ascontiguousarray(x[:, r])) for r in range(64)])
    assert np.array_equal(got, want)


def test_timed_construct_with_simd_equals_plain():
    if not O.avx512_available():
        pytest.skip("host without AVX-512")
    tr = O.synthetic_trace(24, 9)
    _, lde = O.lde(tr, 1, threads=2)
    flat = lde.reshape(24, -1)
    a = O.merkle_construct(flat, 16, threads=2)
    b = O.merkle_construct_timed(flat, 16, threads=2, simd=True)
    for u, v in zip(a[:2], b[:2]):
        assert np.array_equal(u, v)
    assert np.array_equal(a[3], b[3])


@pytest.mark.parametrize("log_n,log_d", [(0, 1), (2, 1), (3, 2), (4, 3), (10, 2), (13, 1)])
def test_avx512_lde_equals_scalar(log_n, log_d):
    if not O.avx512_available():
        pytest.skip("host without AVX-512")
    x = np.random.default_rng(log_n).integers(0, 2 ** 64 - 1, size=(5, 1 << log_n), dtype=np.uint64, endpoint=True)
    m0, l0 = O.lde(x, log_d, threads=2)
    m1, l1 = O.lde_avx512(x, log_d, threads=3)
    assert np.array_equal(m0, m1) and np.array_equal(l0, l1)
