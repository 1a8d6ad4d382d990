"""The Poseidon2 constant schedule of csrc/poseidon2.hpp (CPU, no GPU).

The device permutation places the reference's round constants differently
(state_generic_impl.rs:131-138 full rounds, :55-64 partial rounds): a full round's constant is
one 64-bit add into the L limb, and each pair of partial rounds carries an offset vector whose
constants K (every element, first M_I of the pair) and D (element 0, second M_I) keep element 0
exact at every S-box; the first full round after the partial rounds adds RC_26 - f.

This file restates that schedule independently in Python, checks that the field values it
produces equal the reference permutation's (known answers of SURVEY Appendix A, the C oracle on
random and edge states), and that the compile-time values the C++ header derives (dumped by
tools/sched_dump.hip, host code only) are the same numbers.  The limb bounds the one-add forms
rely on are checked against the constants themselves.
"""
import json
import os
import random
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0xFFFFFFFF00000001
SH = [4, 14, 11, 8, 0, 5, 2, 9, 13, 6, 3, 12]
M4 = [[5, 7, 1, 3], [4, 6, 1, 1], [1, 3, 5, 7], [1, 1, 4, 6]]


def _rc():
    txt = open(os.path.join(ROOT, "era-boojum_amd", "csrc", "poseidon2_rc.inc")).read()
    vals = [int(x) for x in re.findall(r"(\d+)ULL", txt)]
    assert len(vals) == 360
    return [vals[12 * r:12 * r + 12] for r in range(30)]


RC = _rc()


def _mds(x):
    out = []
    for i in range(12):
        bi, ii = divmod(i, 4)
        acc = 0
        for j in range(12):
            bj, jj = divmod(j, 4)
            acc += (2 if bi == bj else 1) * M4[ii][jj] * x[j]
        out.append(acc % P)
    return out


def _mi(x):
    s = sum(x)
    return [(x[i] * (1 << SH[i]) + s) % P for i in range(12)]


def _sbox(v):
    return pow(v, 7, P)


def reference_permutation(x):
    """state_generic_impl.rs:221-236 as written: MDS; 4 full; 22 partial; 4 full."""
    x = _mds(list(x))
    for r in range(4):
        x = _mds([_sbox((x[i] + RC[r][i]) % P) for i in range(12)])
    for r in range(4, 26):
        x[0] = _sbox((x[0] + RC[r][0]) % P)
        x = _mi(x)
    for r in range(26, 30):
        x = _mds([_sbox((x[i] + RC[r][i]) % P) for i in range(12)])
    return x


def derive_schedule():
    """K, D and RC_26 - f, derived independently of the C++ header's code."""
    f = [RC[4][0]] + [0] * 11
    k, d = [], []
    for q in range(11):
        r = 4 + 2 * q
        kq = (RC[r + 1][0] - sum(f[1:])) % P
        k.append(kq)
        ft = [0] + f[1:]
        f = [(v + kq) % P for v in _mi(ft)]
        assert f[0] == RC[r + 1][0]
        f = _mi([0] + f[1:])
        if q < 10:
            d.append((RC[r + 2][0] - f[0]) % P)
            f[0] = RC[r + 2][0]
    rc26 = [(RC[26][i] - f[i]) % P for i in range(12)]
    return k, d, rc26


K, D, RC26 = derive_schedule()


def scheduled_permutation(x):
    """The device schedule's field values (poseidon2.hpp permute)."""
    x = _mds(list(x))
    for r in range(4):
        x = _mds([_sbox((x[i] + RC[r][i]) % P) for i in range(12)])
    x[0] = (x[0] + RC[4][0]) % P
    for q in range(11):
        x[0] = _sbox(x[0])
        x = [(v + K[q]) % P for v in _mi(x)]
        x[0] = _sbox(x[0])
        x = _mi(x)
        if q < 10:
            x[0] = (x[0] + D[q]) % P
    x = [(x[i] + RC26[i]) % P for i in range(12)]
    x = _mds([_sbox(v) for v in x])
    for r in range(27, 30):
        x = _mds([_sbox((x[i] + RC[r][i]) % P) for i in range(12)])
    return x


def test_reference_restatement_matches_known_answers():
    # SURVEY Appendix A (derived from the proof.json-pinned oracle)
    assert [hex(v) for v in reference_permutation(list(range(12)))[:4]] == [
        "0x5d82c16b87f07f98", "0x3655af22bb2f037d", "0x82c1535dfb4bdf90", "0x4d318cfdafd2378e"]
    assert [hex(v) for v in reference_permutation([0] * 12)[:4]] == [
        "0x78e86c27e831c353", "0xc4c13a505ffd93b8", "0xc3a6d7d7f7971adc", "0xf6ff8f53ab94d8c7"]


def test_schedule_gives_the_reference_permutation():
    import oracle as O
    rng = random.Random(5)
    states = [list(range(12)), [0] * 12, [P - 1] * 12, [1] + [0] * 11]
    states += [[rng.randrange(P) for _ in range(12)] for _ in range(60)]
    for x in states:
        want = reference_permutation(x)
        assert scheduled_permutation(x) == want
        got = O.poseidon2_permutation(np.array(x, dtype=np.uint64))
        assert [int(v) for v in got] == want


def test_one_add_bounds_hold_for_the_constants():
    # full rounds: L < 2^39 after an MDS (row sums <= 64 over 32-bit limbs); L + c must stay
    # below 2^64 - 2^40 so that W = Hhi * EPS + L (Hhi < 2^7) cannot wrap
    full_bound = 2 ** 64 - 2 ** 41
    for r in (0, 1, 2, 3, 27, 28, 29):
        assert max(RC[r]) < full_bound
    assert RC[4][0] < full_bound
    assert 64 * 2 ** 32 + full_bound + (2 ** 7) * (2 ** 32 - 1) < 2 ** 64


@pytest.fixture(scope="module")
def cxx_schedule(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("sched") / "sched_dump")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O1", "-std=c++17", "--offload-arch=gfx950", "-o", exe,
                    os.path.join(ROOT, "tools", "sched_dump.hip")], check=True)
    return json.loads(subprocess.run([exe], check=True, capture_output=True, text=True).stdout)


def test_header_schedule_equals_restatement(cxx_schedule):
    assert [int(v) for v in cxx_schedule["k"]] == K
    assert [int(v) for v in cxx_schedule["d"]] == D
    assert [int(v) for v in cxx_schedule["rc26"]] == RC26
    assert int(cxx_schedule["full_rc_bound"]) == 2 ** 64 - 2 ** 41
    assert int(cxx_schedule["limb_rc_bound"]) == 2 ** 63 + 2 ** 62
