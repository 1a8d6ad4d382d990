"""The generated partial-round asm of csrc/gl_asm.hpp, executed on the CPU (no GPU).

tools/gen_gl_asm.py emits the Poseidon2 partial-round layers (mi_layer_a, mi_layer_a_g,
mi_layer_b, mi_layer_b_half, mi_layer_b_limbs, eps_fold_x11) as gfx950 inline asm.  This test
parses the committed header's asm text and interprets it, one lane, with the instruction
semantics the layers use (v_mad_u64_u32, v_lshl_add_u64, v_lshlrev_b64, v_add_co_u32,
v_cndmask_b32_e64), asserting that no 64-bit intermediate wraps where the code discards the
carry.  Chained as csrc/poseidon2.hpp chains them (pair 0 from reduced words, pairs 1..9 and the
last pair from the half-reduced hand-off), the partial rounds must give the field values of the
restated schedule (tests/test_poseidon2_sched.py, itself checked against the reference's
permutation, state_generic_impl.rs:166-202, 221-249), on random states and on the all-ones
limbs that bound every intermediate from above.
"""
import os
import random
import re

import pytest

from test_poseidon2_sched import D, K, P, _mi, _sbox

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M32, M64 = (1 << 32) - 1, (1 << 64) - 1


def _functions():
    txt = open(os.path.join(ROOT, "era-boojum_amd", "csrc", "gl_asm.hpp")).read()
    out = {}
    for m in re.finditer(r"void (\w+)\((.*?)\) \{\n(.*?)\n\}\n", txt, re.S):
        body = m.group(3)
        instrs = re.findall(r'^\s+"([^"]*)\\n"', body, re.M)
        out[m.group(1)] = instrs
    return out


FN = _functions()


class Lane:
    """One lane's registers: fixed VGPRs v<N>, compiler operands by name (64-bit operands as
    ints < 2^64, 32-bit ones < 2^32), carries as 0/1."""

    def __init__(self, operands):
        self.v = {}
        self.op = dict(operands)

    def _pair_regs(self, t):
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", t)
        return (int(m.group(1)), int(m.group(2))) if m else None

    def get32(self, t):
        if t.startswith("%["):
            return self.op[t[2:-1]] & M32
        if re.fullmatch(r"v\d+", t):
            return self.v[int(t[1:])]
        x = int(t, 0)
        return x & M32

    def get64(self, t):
        r = self._pair_regs(t)
        if r:
            return self.v[r[0]] | (self.v[r[1]] << 32)
        if t.startswith("%["):
            return self.op[t[2:-1]]
        return int(t, 0) & M64

    def set64(self, t, x):
        assert 0 <= x <= M64
        r = self._pair_regs(t)
        if r:
            self.v[r[0]], self.v[r[1]] = x & M32, x >> 32
        else:
            self.op[t[2:-1]] = x

    def set32(self, t, x):
        if t.startswith("%["):
            self.op[t[2:-1]] = x & M32
        else:
            self.v[int(t[1:])] = x & M32

    def run(self, instrs):
        for ins in instrs:
            mn, _, rest = ins.partition(" ")
            a = [x.strip() for x in rest.split(",")] if rest else []
            if mn in ("s_nop",):
                continue
            if mn == "s_mov_b32":
                self.op[a[0][2:-1]] = int(a[1], 0)
            elif mn == "v_mad_u64_u32":
                d, c, x, y, s = a
                r = self.get32(x) * self.get32(y) + self.get64(s)
                assert r <= M64, "v_mad_u64_u32 wrapped: %s" % ins
                self.set64(d, r)
            elif mn == "v_lshl_add_u64":
                d, x, sh, y = a
                r = (self.get64(x) << int(sh)) + self.get64(y)
                assert r <= M64, "v_lshl_add_u64 wrapped: %s" % ins
                self.set64(d, r)
            elif mn == "v_lshlrev_b64":
                d, sh, x = a
                r = self.get64(x) << int(sh)
                assert r <= M64, "v_lshlrev_b64 dropped bits: %s" % ins
                self.set64(d, r)
            elif mn == "v_add_co_u32":
                d, c, x, y = a
                r = self.get32(x) + self.get32(y)
                self.set32(d, r)
                self.op[c[2:-1]] = r >> 32
            elif mn == "v_cndmask_b32_e64":
                d, x, y, c = a
                self.set32(d, self.get32(y) if self.op[c[2:-1]] else self.get32(x))
            else:
                raise AssertionError("instruction not modelled: " + ins)


def call(name, **operands):
    lane = Lane(operands)
    lane.run(FN[name])
    return lane.op


def layer_a(lo, hi, k, g=None):
    ops = {"KL": k & M32, "KH": k >> 32}
    ops.update({"lo%d" % i: lo[i] for i in range(12)})
    ops.update({"hi%d" % i: hi[i] for i in range(12)})
    if g is not None:
        ops.update({"g%d" % i: g[i] for i in range(1, 12)})
    r = call("mi_layer_a_g" if g is not None else "mi_layer_a", **ops)
    return r["z0"], {i: r["L%d" % i] for i in range(1, 12)}, {i: r["H%d" % i] for i in range(1, 12)}


def layer_b_half(lo0, hi0, L, H, d):
    ops = {"lo0": lo0, "hi0": hi0, "DL": d & M32, "DH": d >> 32}
    ops.update({"L%d" % i: L[i] for i in range(1, 12)})
    ops.update({"H%d" % i: H[i] for i in range(1, 12)})
    r = call("mi_layer_b_half", **ops)
    return r["z0"], {i: r["Lo%d" % i] for i in range(1, 12)}, {i: r["Ho%d" % i] for i in range(1, 12)}


def layer_b_limbs(lo0, hi0, L, H):
    ops = {"lo0": lo0, "hi0": hi0}
    ops.update({"L%d" % i: L[i] for i in range(1, 12)})
    ops.update({"H%d" % i: H[i] for i in range(1, 12)})
    r = call("mi_layer_b_limbs", **ops)
    return {i: r["Lo%d" % i] for i in range(12)}, {i: r["Ho%d" % i] for i in range(12)}


def eps_fold(hh, L):
    ops = {"hh%d" % i: hh[i] for i in range(1, 12)}
    ops.update({"L%d" % i: L[i] for i in range(1, 12)})
    r = call("eps_fold_x11", **ops)
    return {i: r["W%d" % i] for i in range(1, 12)}


def sbox_any(z):
    """glasm's S-box products return some u64 representative; the worst case for the bounds is
    any word < 2^64, so the model returns the canonical value or, with `high`, value + p when
    that still fits."""
    return _sbox(z % P)


def device_partial_rounds(z, high=False):
    """csrc/poseidon2.hpp's partial rounds on the 12 reduced words z (element 0 holding RC_4):
    pair 0 (reduced in), pairs 1..9 (half-reduced in), the last pair (limbs out).  Returns the
    field values of the limbs the last pair hands to the first full round."""
    up = (lambda v: v + P if high and v + P <= M64 else v)
    z0, W, G = z[0], {i: z[i] for i in range(1, 12)}, None
    for q in range(11):
        s0 = up(sbox_any(z0))
        lo = [s0 & M32] + [W[i] & M32 for i in range(1, 12)]
        hi = [s0 >> 32] + [W[i] >> 32 for i in range(1, 12)]
        a0, L, H = layer_a(lo, hi, K[q], G)
        s1 = up(sbox_any(a0))
        if q == 10:
            Lo, Ho = layer_b_limbs(s1 & M32, s1 >> 32, L, H)
            return [(Lo[i] + (Ho[i] << 32)) % P for i in range(12)], Lo, Ho
        z0, Lo, Ho = layer_b_half(s1 & M32, s1 >> 32, L, H, D[q])
        G = {i: Ho[i] & M32 for i in range(1, 12)}
        W = eps_fold({i: Ho[i] >> 32 for i in range(1, 12)}, Lo)


def restated_partial_rounds(x):
    """The same segment in field arithmetic (tests/test_poseidon2_sched.py::scheduled_permutation)."""
    x = list(x)
    for q in range(11):
        x[0] = _sbox(x[0])
        x = [(v + K[q]) % P for v in _mi(x)]
        x[0] = _sbox(x[0])
        x = _mi(x)
        if q < 10:
            x[0] = (x[0] + D[q]) % P
    return x


def test_layers_present():
    for name in ("mi_layer_a", "mi_layer_a_g", "mi_layer_b", "mi_layer_b_half", "mi_layer_b_limbs", "eps_fold_x11"):
        assert FN.get(name), name


@pytest.mark.parametrize("seed", range(6))
def test_partial_rounds_asm_equal_schedule(seed):
    rng = random.Random(seed)
    x = [rng.randrange(P) for _ in range(12)]
    got, _, _ = device_partial_rounds(x)
    assert got == restated_partial_rounds(x)


def test_partial_rounds_asm_edge_words():
    # non-canonical inputs (the full rounds' reductions return any u64 representative)
    for x in ([M64] * 12, [P - 1] * 12, [0] * 12, [P + 5] * 12):
        got, _, _ = device_partial_rounds(x, high=True)
        assert got == restated_partial_rounds([v % P for v in x])


def test_partial_pair_limb_bounds():
    """All-ones limbs bound every intermediate (every op is a monotone mad / shift / add): no
    wrap anywhere in the chained layers (the interpreter asserts it), and the limbs handed to
    the first full round fit its one-add constant form (poseidon2.hpp LIMB_RC_BOUND:
    Hhi EPS + L < 2^62)."""
    ones = {i: M32 for i in range(12)}
    # worst-case layer_a_g limbs from all-ones inputs, then the layers downstream of them
    a0, L, H = layer_a([M32] * 12, [M32] * 12, M64 >> 1, ones)
    assert max(L.values()) < 2 ** 46.01 and max(H.values()) < 2 ** 47.01
    z0, Lo, Ho = layer_b_half(M32, M32, L, H, M64 >> 1)
    assert max(Lo.values()) < 2 ** 60.01 and max(Ho.values()) < 2 ** 61.01
    W = eps_fold({i: Ho[i] >> 32 for i in range(1, 12)}, Lo)
    assert max(W.values()) < 2 ** 62
    Lo, Ho = layer_b_limbs(M32, M32, L, H)
    assert max((Ho[i] >> 32) * M32 + Lo[i] for i in range(12)) < 2 ** 62
