#!/usr/bin/env python3
"""Generate era-boojum_amd/csrc/ntt_pow2.hpp: register DFTs of 2..32 points whose twiddles are
powers of two, for the NTT's register phases (csrc/ntt_ct.hip).

Why: in Goldilocks, 2 has order 192, so every root of unity of order <= 64 is +-2^e
(the reference's w_32 = 2^78, w_16 = 2^156, w_8 = 2^120, w_4 = 2^48, w_2 = 2^96 = -1;
their inverses 2^114, 2^36, 2^72, 2^144).  A register phase of r <= 5 stages of the
natural -> bit-reversed CT network is, after a prescale of its inputs by powers of its group's
coset shift, a plain 2^r-point DFT, so its twiddles are shifts: c * 2^e is
5-8 instructions instead of the 14 of a general product.

Butterfly (A, C) <- (a + c 2^e, a - c 2^e), e in [0, 96) (a twiddle -2^e swaps A and C), by the
class of e; t = c 2^e as any u64 representative, then the ct butterfly's tail (t canonicalised,
one correcting mad per output, tools/gen_gl_asm.py ct_bfly_stream):
  class 0, e = 0:        t = c
  class 1, 0 < e < 32:   c 2^e = h 2^64 + L, h = c >> (64 - e) < 2^e, L = c << e (64 bits):
                         t = h EPS + L (one mad, carry -> + EPS)
  class 2, 32 <= e < 64: with f = e - 32, c 2^f = (r2 : r1 : r0) (96 bits) and
                         c 2^e = r0 2^32 + r1 2^64 + r2 2^96 == (r0 : 0) + r1 EPS - r2
  class 3, 64 <= e < 96: with f = e - 64, c 2^e == r0 2^64 + r1 2^96 + r2 2^128
                         == r0 EPS - (r2 : r1)                      (2^96 = -1, 2^128 = -2^32)
Every exponent used here is a multiple of 3, so f = 0 (a 32-bit shift, which the shifters
take mod 32) never occurs; the generator checks it.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_gl_asm import BFLY_SCONST, JUNK, NEG_EPS_S, NEG_EPS_V, SGPR_BASE, merge, pad, sgpr_operandize, sp  # noqa: E402,E501

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "era-boojum_amd", "csrc", "ntt_pow2.hpp")

# log2 of the power of two equal to w_{2^j} (forward) and its inverse: verified against the
# oracle's domain generators (tests/test_ntt_pow2_gen.py)
FWD_EXP = {1: 96, 2: 48, 3: 120, 4: 156, 5: 78}
INV_EXP = {1: 96, 2: 144, 3: 72, 4: 36, 5: 114}


def tail(k, vb, vconst, src):
    """Canonicalise t (src pair halves, result in U), then C = a - t and A = a + t."""
    P0, P1, U0, U1, W0, W1, V6 = ["v%d" % (vb + i) for i in range(7)]
    P, W = "v[%d:%d]" % (vb, vb + 1), "v[%d:%d]" % (vb + 4, vb + 5)
    p0, p1 = sp(3 * k), sp(3 * k + 1)
    a0, a1, A, C = ["%%[%s%d]" % (n, k) for n in ("a0", "a1", "A", "C")]
    s0, s1 = src
    return [
        ("v_add_co_u32 %s, %s, %s, -1" % (P0, p0, s0), set(), {p0}),
        ("v_addc_co_u32 %s, %s, %s, 0, %s" % (P1, p0, s1, p0), {p0}, {p0}),
        ("v_cndmask_b32_e64 %s, %s, %s, %s" % (U0, s0, P0, p0), {p0}, set()),
        ("v_cndmask_b32_e64 %s, %s, %s, %s" % (U1, s1, P1, p0), {p0}, set()),
        ("v_sub_co_u32 %s, %s, %s, %s" % (P0, p1, a0, U0), set(), {p1}),
        ("v_subb_co_u32 %s, %s, %s, %s, %s" % (P1, p1, a1, U1, p1), {p1}, {p1}),
        ("v_cndmask_b32_e64 %s, 0, %s, %s" % (V6, vconst, p1), {p1}, set()),
        ("v_mad_i64_i32 %s, %s, %s, %s, %s" % (C, JUNK, V6, BFLY_SCONST, P), set(), {JUNK}),
        ("v_add_co_u32 %s, %s, %s, %s" % (W0, p0, a0, U0), set(), {p0}),
        ("v_addc_co_u32 %s, %s, %s, %s, %s" % (W1, p0, a1, U1, p0), {p0}, {p0}),
        ("v_cndmask_b32_e64 %s, 0, -1, %s" % (U0, p0), {p0}, set()),
        ("v_mad_u64_u32 %s, %s, %s, 1, %s" % (A, JUNK, U0, W), set(), {JUNK}),
    ]


def p2_stream(k, vb, vconst, cls):
    U0, U1, W0, W1, V6, V7, V8, V9 = ["v%d" % (vb + i) for i in range(2, 10)]
    U, W = "v[%d:%d]" % (vb + 2, vb + 3), "v[%d:%d]" % (vb + 4, vb + 5)
    p0, p1 = sp(3 * k), sp(3 * k + 1)
    c0, c1, e, r = ["%%[%s%d]" % (n, k) for n in ("c0", "c1", "e", "r")]
    I = []
    if cls == 0:
        return tail(k, vb, vconst, (c0, c1))
    if cls == 1:
        I += [("v_lshlrev_b32 %s, %s, %s" % (W0, e, c0), set(), set()),
              ("v_alignbit_b32 %s, %s, %s, %s" % (W1, c1, c0, r), set(), set()),
              ("v_lshrrev_b32 %s, %s, %s" % (V7, r, c1), set(), set()),
              ("v_mad_u64_u32 %s, %s, %s, -1, %s" % (U, p0, V7, W), set(), {p0}),
              ("v_cndmask_b32_e64 %s, 0, -1, %s" % (V6, p0), {p0}, set()),
              ("v_mad_u64_u32 %s, %s, %s, 1, %s" % (U, JUNK, V6, U), set(), {JUNK})]
    elif cls == 2:
        # U = r1 EPS + (r0 : 0) (carry p0), minus r2 (borrow p1); -EPS on the borrow, then
        # +EPS on the carry (in that order: no intermediate wrap)
        I += [("v_mov_b32 %s, 0" % W0, set(), set()),
              ("v_lshlrev_b32 %s, %s, %s" % (W1, e, c0), set(), set()),
              ("v_alignbit_b32 %s, %s, %s, %s" % (V6, c1, c0, r), set(), set()),
              ("v_lshrrev_b32 %s, %s, %s" % (V7, r, c1), set(), set()),
              ("v_mad_u64_u32 %s, %s, %s, -1, %s" % (U, p0, V6, W), set(), {p0}),
              ("v_sub_co_u32 %s, %s, %s, %s" % (U0, p1, U0, V7), set(), {p1}),
              ("v_subb_co_u32 %s, %s, %s, 0, %s" % (U1, p1, U1, p1), {p1}, {p1}),
              ("v_cndmask_b32_e64 %s, 0, %s, %s" % (V8, vconst, p1), {p1}, set()),
              ("v_mad_i64_i32 %s, %s, %s, %s, %s" % (U, JUNK, V8, BFLY_SCONST, U), set(), {JUNK}),
              ("v_cndmask_b32_e64 %s, 0, -1, %s" % (V9, p0), {p0}, set()),
              ("v_mad_u64_u32 %s, %s, %s, 1, %s" % (U, JUNK, V9, U), set(), {JUNK})]
    else:
        # U = r0 EPS - (r2 : r1) (borrow p1), -EPS on the borrow
        I += [("v_lshlrev_b32 %s, %s, %s" % (V8, e, c0), set(), set()),
              ("v_alignbit_b32 %s, %s, %s, %s" % (W0, c1, c0, r), set(), set()),
              ("v_lshrrev_b32 %s, %s, %s" % (W1, r, c1), set(), set()),
              ("v_mad_u64_u32 %s, %s, %s, -1, 0" % (U, JUNK, V8), set(), {JUNK}),
              ("v_sub_co_u32 %s, %s, %s, %s" % (U0, p1, U0, W0), set(), {p1}),
              ("v_subb_co_u32 %s, %s, %s, %s, %s" % (U1, p1, U1, W1, p1), {p1}, {p1}),
              ("v_cndmask_b32_e64 %s, 0, %s, %s" % (V9, vconst, p1), {p1}, set()),
              ("v_mad_i64_i32 %s, %s, %s, %s, %s" % (U, JUNK, V9, BFLY_SCONST, U), set(), {JUNK})]
    return I + tail(k, vb, vconst, (U0, U1))


def emit_p2(cls, n):
    vconst = "v%d" % (10 * n)
    streams = [p2_stream(k, 10 * k, vconst, cls) for k in range(n)]
    pro = [("v_mov_b32 %s, 0x%x" % (vconst, NEG_EPS_V), set(), set()),
           ("s_mov_b32 %s, 0x%x" % (BFLY_SCONST, NEG_EPS_S), set(), set())]
    body = pad(pro + merge(streams))
    args, outs, ins = [], [], []
    for k in range(n):
        args += ["uint32_t a0%d" % k, "uint32_t a1%d" % k, "uint32_t c0%d" % k, "uint32_t c1%d" % k,
                 "uint64_t& A%d" % k, "uint64_t& C%d" % k]
        outs += ['[%s%d] "=&v"(%s%d)' % (nm, k, nm, k) for nm in ("A", "C")]
        ins += ['[%s%d] "v"(%s%d)' % (nm, k, nm, k) for nm in ("a0", "a1", "c0", "c1")]
        if cls:
            ins += ['[e%d] "n"(S%d)' % (k, k), '[r%d] "n"(32 - S%d)' % (k, k)]
    clob = ['"v%d"' % i for i in range(10 * n + 1)] + ['"s%d"' % i for i in range(SGPR_BASE, SGPR_BASE + 27)]
    n_v = sum(1 for t in body if t.startswith("v_"))
    head = "template <%s>\n" % ", ".join("int S%d" % k for k in range(n)) if cls else ""
    lines = ["// %d butterflies (A, C) <- (a + c 2^e, a - c 2^e), class %d (%d VALU instructions)" % (n, cls, n_v),
             head + "__device__ __forceinline__ void p2c%d_x%d(%s) {" % (cls, n, ", ".join(args)), "    asm volatile("]
    lines += ['        "%s\\n"' % t for t in body]
    lines += ["        : %s" % ", ".join(outs), "        : %s" % ", ".join(ins), "        : %s);" % ", ".join(clob),
              "}"]
    return "\n".join(lines) + "\n"


def bitrev(x, bits):
    r = 0
    for _ in range(bits):
        r = (r << 1) | (x & 1)
        x >>= 1
    return r


def classify(te):
    """Twiddle 2^te (te mod 192) -> (class, shift, negated)."""
    te %= 192
    neg = te >= 96
    e = te - 96 if neg else te
    if e == 0:
        return 0, 0, neg
    cls = 1 if e < 32 else (2 if e < 64 else 3)
    f = e - 32 * (cls - 1)
    assert 0 < f < 32, "shift %d of 2^%d is not supported" % (f, te)
    return cls, f, neg


def dft_body(log_n, inverse):
    """Calls of one natural -> bit-reversed CT DFT of 2^log_n points on x[B .. B + 2^log_n),
    stage u pairing (i, i + h) with twiddle w_{2^(u+1)}^bitrev_u(group) = 2^te; the butterflies
    of a stage are grouped by class into calls of up to four."""
    E = INV_EXP if inverse else FWD_EXP
    n = 1 << log_n
    lines = []
    for u in range(log_n):
        h = n >> (u + 1)
        by_cls = {}
        for g in range(1 << u):
            cls, f, neg = classify(E[u + 1] * bitrev(g, u))
            for j in range(h):
                lo = g * 2 * h + j
                by_cls.setdefault(cls, []).append((lo, lo + h, f, neg))
        for cls in sorted(by_cls):
            items = by_cls[cls]
            for i in range(0, len(items), 4):
                chunk = items[i:i + 4]
                m = len(chunk)
                targs = "<%s>" % ", ".join(str(f) for _, _, f, _ in chunk) if cls else ""
                call_args = ["LO(x[B + %d]), HI(x[B + %d]), LO(x[B + %d]), HI(x[B + %d]), ta%d, tc%d"
                             % (a, a, c, c, idx, idx) for idx, (a, c, _, _) in enumerate(chunk)]
                lines.append("    {")
                lines.append("        uint64_t %s;" % ", ".join("ta%d, tc%d" % (i2, i2) for i2 in range(m)))
                lines.append("        glasm::p2c%d_x%d%s(%s);" % (cls, m, targs, ", ".join(call_args)))
                for idx, (a, c, _, neg) in enumerate(chunk):
                    # a twiddle -2^e: a + t = C', a - t = A'
                    ra, rc = ("tc%d" % idx, "ta%d" % idx) if neg else ("ta%d" % idx, "tc%d" % idx)
                    lines.append("        x[B + %d] = %s; x[B + %d] = %s;" % (a, ra, c, rc))
                lines.append("    }")
    return lines


def emit_dft(log_n, inverse):
    name = "dft%d_%s" % (1 << log_n, "inv" if inverse else "fwd")
    lines = ["// %d-point natural -> bit-reversed DFT with w%s_%d on x[B ..] (power-of-two twiddles)"
             % (1 << log_n, "^-1" if inverse else "", 1 << log_n),
             "template <int B>", "__device__ __forceinline__ void %s(uint64_t* x) {" % name]
    lines += dft_body(log_n, inverse)
    lines.append("}")
    return "\n".join(lines) + "\n"


def main():
    parts = ['''// GENERATED by tools/gen_ntt_pow2.py -- do not edit.
// Register DFTs with power-of-two twiddles for the NTT register phases (DESIGN.md 4.3).
#pragma once
#include <stdint.h>

namespace glasm {
''']
    for cls in range(4):
        for n in (1, 2, 3, 4):
            parts.append(emit_p2(cls, n))
    parts.append("}  // namespace glasm\n\nnamespace bj {\nnamespace p2dft {\n"
                 "#define LO(v) ((uint32_t)(v))\n#define HI(v) ((uint32_t)((v) >> 32))\n")
    for inverse in (False, True):
        for log_n in range(1, 6):
            parts.append(emit_dft(log_n, inverse))
    parts.append("#undef LO\n#undef HI\n}  // namespace p2dft\n}  // namespace bj\n")
    parts = [sgpr_operandize(x) for x in parts]
    with open(OUT, "w") as f:
        f.write("\n".join(parts))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
