"""The power-of-two register DFTs of the NTT (tools/gen_ntt_pow2.py -> csrc/ntt_pow2.hpp,
DESIGN.md 4.3), on the CPU: the root exponents against the oracle's domain generators, the
committed header against a fresh generation, and each butterfly class's word-level steps
(the same carries and corrections the gfx950 sequence takes) against exact arithmetic."""
import importlib.util
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
P = (1 << 64) - (1 << 32) + 1
EPS = (1 << 32) - 1
M64 = (1 << 64) - 1


def gen():
    spec = importlib.util.spec_from_file_location("gen_ntt_pow2", os.path.join(ROOT, "tools", "gen_ntt_pow2.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_root_exponents_match_the_domain_generators():
    import oracle as O
    g = gen()
    for j in range(1, 6):
        w = O.domain_generator(j)
        assert pow(2, g.FWD_EXP[j], P) == w, j
        assert pow(2, g.INV_EXP[j], P) == pow(w, P - 2, P), j


def test_header_is_current(tmp_path):
    g = gen()
    committed = open(g.OUT).read()
    g.OUT = str(tmp_path / "ntt_pow2.hpp")
    g.main()
    assert open(g.OUT).read() == committed, "csrc/ntt_pow2.hpp is stale: run tools/gen_ntt_pow2.py"


def shifted_product(c, e):
    """t = c * 2^e as a u64 representative, following the generated sequence of e's class."""
    c0, c1 = c & 0xFFFFFFFF, c >> 32
    if e == 0:
        return c
    cls = 1 if e < 32 else (2 if e < 64 else 3)
    f = e - 32 * (cls - 1)
    r0 = (c0 << f) & 0xFFFFFFFF
    r1 = ((c1 << f) | (c0 >> (32 - f))) & 0xFFFFFFFF      # v_alignbit_b32 c1, c0, 32 - f
    r2 = c1 >> (32 - f)
    if cls == 1:
        z = r2 * EPS + ((r1 << 32) | r0)                    # v_mad_u64_u32, carry out
        u = z & M64
        if z >> 64:
            u += EPS
            assert u <= M64
        return u
    if cls == 2:
        z = r1 * EPS + (r0 << 32)
        u, carry = z & M64, z >> 64
        d = u - r2
        borrow = d < 0
        u = d & M64
        if borrow:
            u -= EPS                                        # v_mad_i64_i32 by -65537 * 65535
            assert u >= 0
        if carry:
            u += EPS
            assert u <= M64
        return u
    z = r0 * EPS                                            # < 2^64
    d = z - ((r2 << 32) | r1)
    u = d & M64
    if d < 0:
        u -= EPS
        assert u >= 0
    return u


def butterfly(a, c, te):
    """(a + c w, a - c w) for w = 2^te with the generated tail: t canonicalised, one
    correction per output."""
    te %= 192
    neg = te >= 96
    t = shifted_product(c, te - 96 if neg else te)
    t = t - P if t >= P else t
    s, d = a + t, a - t
    A = s - (1 << 64) + EPS if s > M64 else s
    C = d + (1 << 64) - EPS if d < 0 else d
    assert 0 <= A <= M64 and 0 <= C <= M64
    return (C, A) if neg else (A, C)


def test_butterfly_classes_exact():
    rng = random.Random(5)
    edge = [0, 1, 2, EPS, 1 << 32, P - 1, P, P + 1, M64 - 1, M64, 1 << 63]
    values = edge + [rng.getrandbits(64) for _ in range(300)]
    for te in range(0, 192, 3):   # every root of order <= 64 is 2^(3 j)
        w = pow(2, te, P)
        for a in values[:40]:
            for c in values:
                A, C = butterfly(a, c, te)
                assert A % P == (a + c * w) % P and C % P == (a - c * w) % P, (te, a, c)
