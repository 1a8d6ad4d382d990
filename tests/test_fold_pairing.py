"""The constants the sender fold pairs (ntt_lde3.hip lde3_inv_fold_kernel, F = 2; CPU only).

Shard T's sub-coset shift is s_T = 7 w^bitrev_ls(T), w the generator of the n D domain
(capi.hip shard_shift; the reference's coset order, utils.rs:311-403), and its fold constant is
z_T = s_T^m.  At F = G / k = 2 the targets T and T ^ 1 are the two halves of one coset, so
z_(T^1) = -z_T and the kernel forms both outputs as one butterfly (c0 + z c1, c0 - z c1); the host
checks exactly this on the constants before choosing that form.  The pairing holds at every F
(bitrev_ls(T ^ 1) differs from bitrev_ls(T) by 2^(ls-1), and w^(2^(ls-1) m) = -1), and the kernel
uses it at F = 2, 4 and 8: a butterfly at F = 2 (C3 at G = 8), E +- O at F = 4 and 8 (E the
even-exponent terms, O the odd ones).  The per-target loop runs only under the experiment knob
BJ_INV_FOLD_UNPAIRED=1 (with BJ_EXPERIMENTS=1), which
tests/test_gpu_native_sharded.py::test_native_sharded_commit_env_knobs checks gives the same
commitment.
"""
import pytest

import oracle as O

P = 0xFFFFFFFF00000001


def _bitrev(x, bits):
    return int(format(x, "0%db" % bits)[::-1], 2) if bits else 0


def fold_constants(log_n, log_lde, log_g, log_k):
    """z_T for every target T = j G + p of the collective commit at G = 2^log_g > D."""
    ls = log_g + log_lde - log_k
    m = 1 << (log_n + log_k - log_g)
    g = O.domain_generator(log_n + log_lde)
    return [O.gl_pow(O.gl_mul(O.gl_pow(g, _bitrev(T, ls)), 7), m) % P for T in range(1 << ls)]


@pytest.mark.parametrize("log_n,log_lde,log_g,log_k", [
    (22, 2, 3, 2),   # C3 at G = 8: F = 2, 8 targets
    (18, 2, 3, 2),
    (19, 1, 2, 1),   # D = 2 at G = 4
    (18, 3, 3, 2),   # k < D: B = 2 blocks of 8 targets
    (20, 2, 3, 2),
])
def test_f2_targets_pair_as_negatives(log_n, log_lde, log_g, log_k):
    assert log_g - log_k == 1  # F = 2
    z = fold_constants(log_n, log_lde, log_g, log_k)
    for T in range(0, len(z), 2):
        assert z[T + 1] == (P - z[T]) % P, T
        assert z[T] not in (0, 1)


@pytest.mark.parametrize("log_n,log_lde,log_g,log_k", [
    (18, 2, 3, 1),   # F = 4
    (18, 1, 3, 0),   # F = 8
])
def test_wider_folds_pair_too(log_n, log_lde, log_g, log_k):
    z = fold_constants(log_n, log_lde, log_g, log_k)
    for T in range(0, len(z), 2):
        assert z[T + 1] == (P - z[T]) % P, T
