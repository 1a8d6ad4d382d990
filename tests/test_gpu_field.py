"""Device field layer (inline-asm Goldilocks primitives) vs the reference semantics.

Every op is checked against exact Python integer arithmetic mod p on adversarial
operands: 0, 1, p-1, p, p+1, 2^64-1, 2^32-1, 2^32, powers of two (a*b = 2^96 style
products exercise the r1 = r2 = 0 borrow path of the reduction), values just below
and above p, plus random u64 (non-canonical included).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001
M64 = (1 << 64) - 1


def edge_values():
    v = {0, 1, 2, P - 1, P, P + 1, M64, M64 - 1, (1 << 32) - 1, 1 << 32, (1 << 32) + 1, 1 << 63, (1 << 63) - 1,
         P - (1 << 32), 0xFFFFFFFE00000002, 0x00000000FFFFFFFF, 0xFFFFFFFF00000000, 0xFFFFFFFF7FFFFFFF}
    for k in range(64):
        v.add(1 << k)
        v.add(M64 ^ (1 << k))
    return sorted(v)


@pytest.fixture(scope="module")
def run():
    import torch
    from boojum_amd import field
    from boojum_amd._lib import call

    def go(op, a, b):
        a = np.asarray(a, dtype=np.uint64)
        b = np.asarray(b, dtype=np.uint64)
        ta, tb = field.to_device(a), field.to_device(b)
        out = torch.empty_like(ta)
        call("bj_gl_op_d", op, ta.data_ptr(), tb.data_ptr(), out.data_ptr(), a.size, field.stream_of(ta))
        return [int(x) for x in field.to_host(out)]
    return go


def pairs(n_random=200000, seed=1):
    e = edge_values()
    a = [x for x in e for _ in e]
    b = [y for _ in e for y in e]
    rng = np.random.default_rng(seed)
    ra = rng.integers(0, 2**64, size=n_random, dtype=np.uint64)
    rb = rng.integers(0, 2**64, size=n_random, dtype=np.uint64)
    return np.concatenate([np.array(a, dtype=np.uint64), ra]), np.concatenate([np.array(b, dtype=np.uint64), rb])


@pytest.mark.parametrize("op,name", [(0, "mul"), (1, "add"), (2, "sub")])
def test_binary_ops_exact(run, op, name):
    a, b = pairs()
    got = run(op, a, b)
    ai, bi = [int(x) for x in a], [int(x) for x in b]
    if op == 0:
        want = [(x * y) % P for x, y in zip(ai, bi)]
    elif op == 1:
        want = [(x + y) % P for x, y in zip(ai, bi)]
    else:
        want = [(x - y) % P for x, y in zip(ai, bi)]
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, "%s: %d mismatches, first %s" % (name, len(bad), [(hex(ai[i]), hex(bi[i])) for i in bad[:3]])


def test_products_with_zero_middle_words(run):
    # a*b = r3*2^96 + r0 (r1 = r2 = 0, r3 > r0): the B2 repair path of the reduction
    a, b = [], []
    for i in range(32, 64):
        for j in range(32, 64):
            if i + j >= 96:
                a.append(1 << i)
                b.append(1 << j)
                a.append((1 << i) + 1)
                b.append(1 << j)
    got = run(0, a, b)
    for x, y, g in zip(a, b, got):
        assert g == (x * y) % P, (hex(x), hex(y))


def test_limb_reduction(run):
    rng = np.random.default_rng(5)
    L = rng.integers(0, 2**63, size=100000, dtype=np.uint64)
    H = rng.integers(0, 2**63 - 2**62, size=100000, dtype=np.uint64) >> np.uint64(rng.integers(0, 40))
    L[:4] = [0, 2**63 - 1, 1, 2**40]
    H[:4] = [2**62 + 5, 2**62 - 1, (2**31 - 1) << 32 | 0xFFFFFFFF, 0xFFFFFFFF]
    got = run(3, L, H)
    for l, h, g in zip(L.tolist(), H.tolist(), got):
        assert g == (l + (h << 32)) % P


def test_canonicalise(run):
    e = np.array(edge_values(), dtype=np.uint64)
    got = run(4, e, e)
    assert got == [int(x) % P for x in e]
