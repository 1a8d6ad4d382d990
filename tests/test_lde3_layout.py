"""Host checks of the three-pass LDE's LDS exchanges (csrc/ntt_lde3.hip): every access pattern
is a bijection onto the block's 8192 elements, splits into a per-thread base plus a per-register
compile-time offset (the kernels rely on that to use immediate ds offsets), and the bank
conflicts are what the kernel comments claim.  Model of gfx950 LDS banking
(MI355X_MICROARCH.md, LDS): ds_read_b64 serves 32-lane groups, ds_write_b64 16-lane groups,
one cycle per group when the 8-byte slots are distinct mod 32 (reads) / mod 16 (writes)."""
import pytest


def brev(x, b):
    r = 0
    for i in range(b):
        r = (r << 1) | ((x >> i) & 1)
    return r


def pad(e):
    return e + (e >> 5)


def extra_cycles(slot_of, write):
    grp, mod = (16, 16) if write else (32, 32)
    extra = 0
    for k in range(32):
        for g0 in range(0, 256, grp):
            banks = {}
            for t in range(g0, g0 + grp):
                s = slot_of(t, k)
                banks.setdefault(s % mod, set()).add(s)
            extra += max(len(v) for v in banks.values()) - 1
    return extra


def decomposes(slot_of):
    return all(slot_of(t, k) == slot_of(t, 0) + slot_of(0, k) - slot_of(0, 0) for t in range(256) for k in range(32))


def bijective(elem_of):
    return sorted(elem_of(t, k) for t in range(256) for k in range(32)) == list(range(8192))


# ------------------------------------------------------------ middle pass (element m)
lpad = lambda m: pad(brev(m, 13))  # noqa: E731
MID = {
    # name: (element m of thread t register k, layout, slot formula used by the kernel, write?)
    "phaseA_out": (lambda t, k: 256 * k + brev(t, 8), lpad, lambda t, k: 33 * t + brev(k, 5), True),
    "phaseB_read": (lambda t, k: 256 * brev(t & 31, 5) + 8 * k + brev(t >> 5, 3), lpad,
                    lambda t, k: 1056 * (t >> 5) + (t & 31) + 33 * brev(k, 5), False),
    "phaseB_write": (lambda t, k: 256 * brev(t & 31, 5) + 8 * k + brev(t >> 5, 3), lpad,
                     lambda t, k: 1056 * (t >> 5) + (t & 31) + 33 * brev(k, 5), True),
    "phaseC_read": (lambda t, k: 32 * t + k, lpad,
                    lambda t, k: brev(t, 8) + (brev(t, 8) >> 5) + 264 * brev(k, 5), False),
    "phaseC_out": (lambda t, k: 32 * t + k, pad, lambda t, k: 33 * t + k, True),
    "store_read": (lambda t, k: t + 256 * k, pad, lambda t, k: t + (t >> 5) + 264 * k, False),
}


@pytest.mark.parametrize("name", sorted(MID))
def test_mid_exchanges(name):
    elem, layout, formula, write = MID[name]
    assert bijective(elem)
    slot = lambda t, k: layout(elem(t, k))  # noqa: E731
    assert all(slot(t, k) == formula(t, k) for t in range(256) for k in range(32)), "kernel formula != layout"
    assert decomposes(slot)
    assert extra_cycles(slot, write) == 0


def test_mid_phase_roles():
    """Phase A's registers are m's top 5 bits (bit-reversed register order after the inverse's
    phase C: l = 32 t + k, m = bitrev_13(l)); phase B's thread holds one 5-bit group g and low bits
    b; phase C's thread 32 consecutive m (4 groups of 8)."""
    for t in range(256):
        for k in range(32):
            m = brev(32 * t + k, 13)
            assert m >> 8 == brev(k, 5) and m & 255 == brev(t, 8)


# -------------------------------------------------------------- final pass (element (r, o))
def fin_slot(R, r, o):
    e = (o << R) + r if R == 5 else r * (1 << (13 - R)) + o
    return pad(e)


def fin_patterns(R):
    LW = 13 - R
    W = 1 << LW
    RL = R - 5

    def p1(t, k):
        return (k << RL) + brev(t >> LW, RL), t & (W - 1)

    def p2(t, k):
        h, rl = k >> RL, k & ((1 << RL) - 1)
        p = (t >> LW) + (h << RL)
        return (p << RL) + rl, t & (W - 1)

    def p3(t, k):
        P = t + 256 * k
        return P & ((1 << R) - 1), P >> R
    return p1, p2, p3


# extra LDS cycles per block accepted for each R (phase-1 write, phase-2 read, phase-2 write,
# store read): the r-order layout is conflict-free except where listed
FIN_EXTRA = {5: (0, None, None, 0), 6: (0, 0, 0, 768), 7: (0, 0, 0, 256), 8: (0, 0, 0, 0), 9: (0, 256, 0, 0),
             10: (512, 0, 0, 0)}


@pytest.mark.parametrize("R", range(5, 11))
def test_final_exchanges(R):
    p1, p2, p3 = fin_patterns(R)
    W = 1 << (13 - R)
    for p in (p1, p2, p3):
        assert bijective(lambda t, k: (lambda ro: ro[0] * W + ro[1])(p(t, k)))
    want = FIN_EXTRA[R]
    for (pat, write), w in zip(((p1, True), (p2, False), (p2, True), (p3, False)), want):
        if w is None:
            continue
        slot = lambda t, k: fin_slot(R, *pat(t, k))  # noqa: E731
        assert decomposes(slot)
        assert extra_cycles(slot, write) == w
