"""The middle LDE pass's phase C (forward stages 10..12 of a block, csrc/ntt_lde3.hip) in its
power-of-two form equals the coset-folded CT network it replaced, on the CPU: for a stage-10
group G, the 8 elements m = 8 G + j through three CT stages with the twiddles
CT13[2^u + (m >> (13 - u))] = s^(n >> (u+1)) w_n^(bitrev_u(.) (n >> (u+1))) (fft/mod.rs:659-734
with the shift folded in) are the 8-point DFT (root w_8 = w_n^(n/8), natural in, bit-reversed
out) of x_j sigma_10(G)^((n / 8192) j), sigma_10(G) = s w_n^bitrev_10(G): the factors
lde3_table_kernel writes at [L3_C + 8 G + j].  Pure-Python field arithmetic over the oracle's
domain generators."""
import random

import oracle as O

P = O.P


def bitrev(x, bits):
    return int(format(x, "0%db" % bits)[::-1], 2) if bits else 0


def ct13(u, g, log_n, w_n, s):
    n = 1 << log_n
    return pow(w_n, bitrev(g, u) << (log_n - u - 1), P) * pow(s, n >> (u + 1), P) % P


def network(x, G, log_n, w_n, s):
    """Stages 10, 11, 12 of the block's natural -> bit-reversed CT network on m = 8 G + j."""
    y = list(x)
    for u, half in ((10, 4), (11, 2), (12, 1)):
        for j in range(8):
            if j & half:
                continue
            m = 8 * G + j
            w = ct13(u, m >> (13 - u), log_n, w_n, s)
            a, c = y[j], y[j + half]
            t = w * c % P
            y[j], y[j + half] = (a + t) % P, (a - t) % P
    return y


def pow2_phase(x, G, log_n, w_n, s):
    n = 1 << log_n
    sigma = s * pow(w_n, bitrev(G, 10), P) % P
    f = [pow(sigma, (n >> 13) * j, P) for j in range(8)]   # the factor table's row G
    y = [x[j] * f[j] % P for j in range(8)]
    w8 = pow(w_n, n // 8, P)
    return [sum(y[i] * pow(w8, i * bitrev(j, 3), P) for i in range(8)) % P for j in range(8)]


def test_phase_c_pow2_form_equals_ct_network():
    rng = random.Random(7)
    for log_n in (18, 20, 22, 23):
        w_n = int(O.domain_generator(log_n))
        for _ in range(6):
            # a coset shift as the LDE uses (7 w^i) or a random one, and a random stage-10 group
            s = rng.choice([7, 7 * pow(w_n, rng.randrange(1 << log_n), P) % P, rng.randrange(1, P)])
            G = rng.randrange(1024)
            x = [rng.randrange(P) for _ in range(8)]
            assert network(x, G, log_n, w_n, s) == pow2_phase(x, G, log_n, w_n, s), (log_n, G)

