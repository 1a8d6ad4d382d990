#!/usr/bin/env python3
"""Generate era-boojum_amd/csrc/gl_asm.hpp: gfx950 inline-asm Goldilocks primitives.

Why asm: on gfx950 every carry-producing / 64-bit / multiply VALU op issues at half
rate while 32-bit logic is full rate (tools/microbench_isa.hip), so the multiply is
priced by its instruction count.  hipcc materialises carries through v_cmp_lt_u64 +
v_cndmask + v_mov pairs (~31 instructions per multiply); the sequences
below keep every carry in an SGPR pair and use 14 instructions per multiply.

Each primitive is emitted in N-way interleaved forms (N independent operations,
round-robin) so a carry consumer sits >= 2 instructions after its producer: gfx950
needs 2 wait states between a VALU write of an SGPR and a VALU read of it (hipcc pads
exactly that).  Where the interleave leaves fewer, the generator inserts s_nop.

Scratch: fixed VGPR pairs v[0:K) and SGPR pairs s[40:66) are declared clobbered; all
other operands are compiler-allocated 32-bit registers (no 64-bit operand halves are
ever needed, which inline asm cannot address).

Field semantics: p = 2^64 - 2^32 + 1, EPS = 2^32 - 1; inputs any u64, outputs any u64
representative of the right residue (never canonicalised here).
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "era-boojum_amd", "csrc", "gl_asm.hpp")

SGPR_BASE = 40


def sp(i):
    return "s[%d:%d]" % (SGPR_BASE + 2 * i, SGPR_BASE + 2 * i + 1)


JUNK = sp(12)  # carry-out sink (never read)


class Stream:
    """One operation's instruction list; operands as format fields."""

    def __init__(self, instrs):
        self.instrs = instrs  # list of (text, reads_sgprs set, writes_sgprs set)


def mul_stream(k, vbase, out=None):
    """z = a * b mod p in 14 instructions.  Inputs a0,a1,b0,b1; outputs z0,z1.
    Scratch pairs P,U,W,V at vbase..vbase+7, m at vbase+8; carries cA, cB, cW.

    a*b = P + (a0 b1 + a1 b0) 2^32 + V 2^64 with P = a0 b0, V = a1 b1.  The cross sum is
    one mad, W = a0 b1 + U (U = a1 b0), whose carry-out cw is worth 2^96 = 2^32 * 2^64,
    i.e. it adds to the top word r3.  Columns: r0 = P0, r1 = P1 + W0, r2 = W1 + V0 + c,
    r3 = V1 + cw + c'.  Reduction (2^64 = EPS, 2^96 = -1): x = (r1:r0) - r3 with borrow B
    (r3's own carry c' enters as the borrow-in), r2' = r2 - B (borrow B2),
    z = r2' * EPS + x, + EPS on overflow, + B2 (the r2 = 0, B = 1 case, where r2 - B wraps
    to 2^32 - 1 and the product is short by exactly one)."""
    P0, P1, U0, U1, W0, W1, V0, V1, M = ["v%d" % (vbase + i) for i in range(9)]
    P, U, W, V = ["v[%d:%d]" % (vbase + 2 * i, vbase + 2 * i + 1) for i in range(4)]
    cA, cB, cW = sp(3 * k), sp(3 * k + 1), sp(3 * k + 2)
    a0, a1, b0, b1, z0, z1 = ["%%[%s%d]" % (n, k) for n in ("a0", "a1", "b0", "b1", "z0", "z1")]
    if out is not None:
        z0, z1 = out
    I = []
    I.append(("v_mad_u64_u32 %s, %s, %s, %s, 0" % (U, JUNK, a1, b0), set(), {JUNK}))
    I.append(("v_mad_u64_u32 %s, %s, %s, %s, 0" % (P, JUNK, a0, b0), set(), {JUNK}))
    I.append(("v_mad_u64_u32 %s, %s, %s, %s, %s" % (W, cW, a0, b1, U), set(), {cW}))
    I.append(("v_mad_u64_u32 %s, %s, %s, %s, 0" % (V, JUNK, a1, b1), set(), {JUNK}))
    I.append(("v_add_co_u32 %s, %s, %s, %s" % (P1, cA, P1, W0), set(), {cA}))            # r1
    I.append(("v_addc_co_u32 %s, %s, %s, 0, %s" % (V1, JUNK, V1, cW), {cW}, {JUNK}))     # V1 + cw
    I.append(("v_addc_co_u32 %s, %s, %s, %s, %s" % (W1, cB, W1, V0, cA), {cA}, {cB}))    # r2, c'
    I.append(("v_subb_co_u32 %s, %s, %s, %s, %s" % (P0, cA, P0, V1, cB), {cB}, {cA}))    # r0 - r3
    I.append(("v_subb_co_u32 %s, %s, %s, 0, %s" % (P1, cA, P1, cA), {cA}, {cA}))         # B
    I.append(("v_subb_co_u32 %s, %s, %s, 0, %s" % (W1, cA, W1, cA), {cA}, {cA}))         # r2', B2
    I.append(("v_mad_u64_u32 %s, %s, %s, -1, %s" % (U, cB, W1, P), set(), {cB}))         # C
    I.append(("v_cndmask_b32_e64 %s, 0, -1, %s" % (M, cB), {cB}, set()))
    I.append(("v_addc_co_u32 %s, %s, %s, %s, %s" % (z0, cB, U0, M, cA), {cA}, {cB}))
    I.append(("v_addc_co_u32 %s, %s, %s, 0, %s" % (z1, JUNK, U1, cB), {cB}, {JUNK}))
    return I


def reduce_stream(k, vbase, pair_out=False):
    """z = L + H * 2^32 mod p for a 64-bit pair L and H = (Hhi:Hlo) given as two 32-bit
    operands, with L < 2^63 and Hhi < 2^31 (so Hhi * EPS + L < 2^64).  These bounds hold
    for every lazily accumulated linear-layer limb in poseidon2.hpp (< 2^48).
    Scratch pair W at vbase, m at vbase+2."""
    W = "v[%d:%d]" % (vbase, vbase + 1)
    W0, W1, M = "v%d" % vbase, "v%d" % (vbase + 1), "v%d" % (vbase + 2)
    cA = sp(2 * k)
    L, Hlo, Hhi, z0, z1 = ["%%[%s%d]" % (n, k) for n in ("L", "Hlo", "Hhi", "z0", "z1")]
    I = []
    # value = L + Hlo*2^32 + Hhi*2^64 == (Hhi*EPS + L) + Hlo*2^32
    I.append(("v_mad_u64_u32 %s, %s, %s, -1, %s" % (W, JUNK, Hhi, L), set(), {JUNK}))
    I.append(("v_add_co_u32 %s, %s, %s, %s" % (W1, cA, W1, Hlo), set(), {cA}))
    # a carry out of the high word is 2^64 == EPS; W then < 2^48 so W + EPS cannot overflow
    I.append(("v_cndmask_b32_e64 %s, 0, -1, %s" % (M, cA), {cA}, set()))
    if pair_out:
        # z = M * 1 + W in one 64-bit mad (z is a compiler-allocated VGPR pair)
        I.append(("v_mad_u64_u32 %%[z%d], %s, %s, 1, %s" % (k, JUNK, M, W), set(), {JUNK}))
    else:
        I.append(("v_add_co_u32 %s, %s, %s, %s" % (z0, cA, W0, M), set(), {cA}))
        I.append(("v_addc_co_u32 %s, %s, %s, 0, %s" % (z1, JUNK, W1, cA), {cA}, {JUNK}))
    return I


def addsub_stream(k, vbase, op):
    """z = a +/- b mod p for any u64 a, b (a0,a1,b0,b1 -> z0,z1)."""
    M = "v%d" % vbase
    cA = sp(2 * k)
    a0, a1, b0, b1, z0, z1 = ["%%[%s%d]" % (n, k) for n in ("a0", "a1", "b0", "b1", "z0", "z1")]
    I = []
    if op == "add":
        # a + b = s + c*2^64 == s + c*EPS; a second overflow can only follow the first
        I.append(("v_add_co_u32 %s, %s, %s, %s" % (z0, cA, a0, b0), set(), {cA}))
        I.append(("v_addc_co_u32 %s, %s, %s, %s, %s" % (z1, cA, a1, b1, cA), {cA}, {cA}))
        for _ in range(2):
            I.append(("v_cndmask_b32_e64 %s, 0, -1, %s" % (M, cA), {cA}, set()))
            I.append(("v_add_co_u32 %s, %s, %s, %s" % (z0, cA, z0, M), set(), {cA}))
            I.append(("v_addc_co_u32 %s, %s, %s, 0, %s" % (z1, cA, z1, cA), {cA}, {cA}))
    else:
        # a - b = d - c*2^64 == d - c*EPS
        I.append(("v_sub_co_u32 %s, %s, %s, %s" % (z0, cA, a0, b0), set(), {cA}))
        I.append(("v_subb_co_u32 %s, %s, %s, %s, %s" % (z1, cA, a1, b1, cA), {cA}, {cA}))
        for _ in range(2):
            I.append(("v_cndmask_b32_e64 %s, 0, -1, %s" % (M, cA), {cA}, set()))
            I.append(("v_sub_co_u32 %s, %s, %s, %s" % (z0, cA, z0, M), set(), {cA}))
            I.append(("v_subb_co_u32 %s, %s, %s, 0, %s" % (z1, cA, z1, cA), {cA}, {cA}))
    return I


# VGPR / SGPR holding the two factors of -EPS = -65537 * 65535 (EPS = (2^16 + 1)(2^16 - 1)) for
# the butterfly's signed-mad subtract correction; set once per asm block
NEG_EPS_V = 0xFFFEFFFF  # -65537 as i32
NEG_EPS_S = 0xFFFF      # 65535
BFLY_SCONST = "s%d" % (SGPR_BASE + 26)


def ct_bfly_stream(k, vbase, vconst):
    """Cooley-Tukey butterfly: (A, C) <- (a + c w, a - c w), 26 instructions.
    t = c * w (mul_stream, result left in its U pair), canonicalised (t + EPS overflows iff
    t >= p).  With t < p, a - t borrows at most once and a + t wraps 2^64 at most once, so each
    needs a single EPS correction, applied by one 64-bit mad into the output pair:
      a - t = d - borrow * 2^64 == d - borrow * EPS:  C = M * 65535 + d (v_mad_i64_i32),
          M = borrow ? -65537 : 0, since -65537 * 65535 = -EPS; no underflow (d > EPS when the
          subtraction borrowed);
      a + t = s + carry * 2^64 == s + carry * EPS:    A = M' * 1 + s (v_mad_u64_u32),
          M' = carry ? EPS : 0; no overflow (s <= p - 2 when the addition carried).
    Operands: a0,a1,c0,c1,w0,w1 read; A, C written (64-bit pairs, early clobber).
    vconst holds -65537; BFLY_SCONST holds 65535."""
    P0, P1, U0, U1, W0, W1, V0 = ["v%d" % (vbase + i) for i in range(7)]
    P, W = "v[%d:%d]" % (vbase, vbase + 1), "v[%d:%d]" % (vbase + 4, vbase + 5)
    p0, p1 = sp(3 * k), sp(3 * k + 1)
    a0, a1, A, C = ["%%[%s%d]" % (n, k) for n in ("a0", "a1", "A", "C")]
    I = []
    for t, r, w in mul_stream(k, vbase, out=(U0, U1)):
        t = t.replace("%%[b0%d]" % k, "%%[w0%d]" % k).replace("%%[b1%d]" % k, "%%[w1%d]" % k)
        t = t.replace("%%[a0%d]" % k, "%%[c0%d]" % k).replace("%%[a1%d]" % k, "%%[c1%d]" % k)
        I.append((t, r, w))
    # canonical t: X = t + EPS (into the dead P pair); carry => t >= p => t = X
    I.append(("v_add_co_u32 %s, %s, %s, -1" % (P0, p0, U0), set(), {p0}))
    I.append(("v_addc_co_u32 %s, %s, %s, 0, %s" % (P1, p0, U1, p0), {p0}, {p0}))
    I.append(("v_cndmask_b32_e64 %s, %s, %s, %s" % (U0, U0, P0, p0), {p0}, set()))
    I.append(("v_cndmask_b32_e64 %s, %s, %s, %s" % (U1, U1, P1, p0), {p0}, set()))
    # C = a - t (into P), then the borrow's -EPS
    I.append(("v_sub_co_u32 %s, %s, %s, %s" % (P0, p1, a0, U0), set(), {p1}))
    I.append(("v_subb_co_u32 %s, %s, %s, %s, %s" % (P1, p1, a1, U1, p1), {p1}, {p1}))
    I.append(("v_cndmask_b32_e64 %s, 0, %s, %s" % (V0, vconst, p1), {p1}, set()))
    I.append(("v_mad_i64_i32 %s, %s, %s, %s, %s" % (C, JUNK, V0, BFLY_SCONST, P), set(), {JUNK}))
    # A = a + t (into W), then the wrap's +EPS
    I.append(("v_add_co_u32 %s, %s, %s, %s" % (W0, p0, a0, U0), set(), {p0}))
    I.append(("v_addc_co_u32 %s, %s, %s, %s, %s" % (W1, p0, a1, U1, p0), {p0}, {p0}))
    I.append(("v_cndmask_b32_e64 %s, 0, -1, %s" % (U0, p0), {p0}, set()))
    I.append(("v_mad_u64_u32 %s, %s, %s, 1, %s" % (A, JUNK, U0, W), set(), {JUNK}))
    return I


def emit_ct_bfly(n):
    vconst = "v%d" % (10 * n)
    streams = [ct_bfly_stream(k, 10 * k, vconst) for k in range(n)]  # 64-bit tuples even-aligned
    pro = [("v_mov_b32 %s, 0x%x" % (vconst, NEG_EPS_V), set(), set()),
           ("s_mov_b32 %s, 0x%x" % (BFLY_SCONST, NEG_EPS_S), set(), set())]
    body = pad(pro + merge(streams))
    args, outs, ins = [], [], []
    for k in range(n):
        args += ["uint32_t a0%d" % k, "uint32_t a1%d" % k, "uint32_t c0%d" % k, "uint32_t c1%d" % k,
                 "uint32_t w0%d" % k, "uint32_t w1%d" % k, "uint64_t& A%d" % k, "uint64_t& C%d" % k]
        outs += ['[%s%d] "=&v"(%s%d)' % (nm, k, nm, k) for nm in ("A", "C")]
        ins += ['[%s%d] "v"(%s%d)' % (nm, k, nm, k) for nm in ("a0", "a1", "c0", "c1", "w0", "w1")]
    clob = ['"v%d"' % i for i in range(10 * n + 1)] + ['"s%d"' % i for i in range(SGPR_BASE, SGPR_BASE + 27)]
    n_v = sum(1 for t in body if t.startswith("v_"))
    lines = ["// %d Cooley-Tukey butterflies (A, C) <- (a + c w, a - c w) (%d VALU instructions)" % (n, n_v),
             "__device__ __forceinline__ void ct_bfly_x%d(%s) {" % (n, ", ".join(args)), "    asm volatile("]
    lines += ['        "%s\\n"' % t for t in body]
    lines += ["        : %s" % ", ".join(outs), "        : %s" % ", ".join(ins), "        : %s);" % ", ".join(clob),
              "}"]
    return "\n".join(lines) + "\n"


def canon_stream(k, vbase):
    """z = canonical(x): x + EPS overflows iff x >= p, and then x + EPS - 2^64 = x - p."""
    T0, T1 = "v%d" % vbase, "v%d" % (vbase + 1)
    cA = sp(2 * k)
    a0, a1, z0, z1 = ["%%[%s%d]" % (n, k) for n in ("a0", "a1", "z0", "z1")]
    I = []
    I.append(("v_add_co_u32 %s, %s, %s, -1" % (T0, cA, a0), set(), {cA}))
    I.append(("v_addc_co_u32 %s, %s, %s, 0, %s" % (T1, cA, a1, cA), {cA}, {cA}))
    I.append(("v_cndmask_b32_e64 %s, %s, %s, %s" % (z0, a0, T0, cA), {cA}, set()))
    I.append(("v_cndmask_b32_e64 %s, %s, %s, %s" % (z1, a1, T1, cA), {cA}, set()))
    return I


def merge(streams):
    merged = []
    idx = [0] * len(streams)
    while any(i < len(s) for i, s in zip(idx, streams)):
        for j, s in enumerate(streams):
            if idx[j] < len(s):
                merged.append(s[idx[j]])
                idx[j] += 1
    return merged


def interleave(streams):
    """Round-robin merge, then pad SGPR write->read distances to >= 2 wait states."""
    return pad(merge(streams))


def pad(merged):
    out = []
    last_write = {}  # sgpr -> position in out (counting only instructions)
    pos = 0
    for text, reads, writes in merged:
        need = 0
        for r in reads:
            if r in last_write:
                gap = pos - last_write[r] - 1  # instructions in between
                need = max(need, 2 - gap)
        if need > 0:
            out.append("s_nop %d" % (need - 1))
            pos += need
        out.append(text)
        for w in writes:
            last_write[w] = pos
        pos += 1
    return out


def emit_fn(name, n, stream_fn, vper, in_names, out_names, in_kinds=None, doc="", out_kinds=None, in_cons=None):
    streams = [stream_fn(k, vper * k) for k in range(n)]
    body = interleave(streams)
    n_v = vper * n
    args = []
    for k in range(n):
        for nm in in_names:
            kind = (in_kinds or {}).get(nm, "uint32_t")
            args.append("%s %s%d" % (kind, nm, k))
        for nm in out_names:
            args.append("%s& %s%d" % ((out_kinds or {}).get(nm, "uint32_t"), nm, k))
    outs = ", ".join('[%s%d] "=&v"(%s%d)' % (nm, k, nm, k) for k in range(n) for nm in out_names)
    ins = ", ".join('[%s%d] "%s"(%s%d)' % (nm, k, (in_cons or {}).get(nm, "v"), nm, k) for k in range(n)
                    for nm in in_names)
    clob = ['"v%d"' % i for i in range(n_v)] + ['"s%d"' % i for i in range(SGPR_BASE, SGPR_BASE + 26)]
    lines = []
    if doc:
        lines.append("// " + doc)
    lines.append("__device__ __forceinline__ void %s(%s) {" % (name, ", ".join(args)))
    lines.append("    asm volatile(")
    for t in body:
        lines.append('        "%s\\n"' % t)
    lines.append("        : %s" % outs)
    lines.append("        : %s" % ins)
    lines.append("        : %s);" % ", ".join(clob))
    lines.append("}")
    return "\n".join(lines) + "\n"


SH = [4, 14, 11, 8, 0, 5, 2, 9, 13, 6, 3, 12]  # M_I diagonal exponents, state_generic_impl.rs:71-84


# v_lshl_add_u64 shift amounts verified on gfx950 hardware (tools/isa_probe.hip)
MAX_LSHL_ADD_SHIFT = 4


def reduce_limbs(Lp, Hp, Wp, M, c, z):
    """The 4-instruction limb reduction (reduce_stream, pair_out) on register pairs Lp, Hp ->
    the 64-bit output operand z."""
    H0, H1 = Hp.split("[")[1].rstrip("]").split(":")
    H0, H1 = "v" + H0, "v" + H1
    W0, W1 = Wp.split("[")[1].rstrip("]").split(":")
    W0, W1 = "v" + W0, "v" + W1
    return [
        ("v_mad_u64_u32 %s, %s, %s, -1, %s" % (Wp, JUNK, H1, Lp), set(), {JUNK}),
        ("v_add_co_u32 %s, %s, %s, %s" % (W1, c, W1, H0), set(), {c}),
        ("v_cndmask_b32_e64 %s, 0, -1, %s" % (M, c), {c}, set()),
        ("v_mad_u64_u32 %s, %s, %s, 1, %s" % (z, JUNK, M, Wp), set(), {JUNK}),
    ]


def _consts(pro):
    consts = {}
    sreg = SGPR_BASE + 26
    for k in sorted(set(SH)):
        if k > 6:
            consts[k] = "s%d" % sreg
            pro.append(("s_mov_b32 s%d, %d" % (sreg, 1 << k), set(), set()))
            sreg += 1
    return consts, sreg


# limb-sum chains per limb in the M_I layers (ILP against instruction count: k chains cost k - 1
# combining adds).  One chain each measured fastest with tools/leaf_bench.hip (C3 leaf shape,
# 2^22 leaves, alternated on one box, profiles/r5d_leaf_variants.log): 3 + 2 chains 33.70 ms,
# 2 + 1 33.62, 1 + 1 33.57; three waves per SIMD cover the chains' latency.
LAYER_A_CHAINS = 1
LAYER_B_CHAINS = 1


def emit_mi_layer_a(with_g=False):
    """First partial round of a pair: M_I with elements 1..11 left as unreduced limbs.
    L_i = lo_i 2^SH[i] + sum lo_j + K_lo, H_i likewise (one mad each, < 2^46.6); only element
    0, the next S-box input, is reduced (into the 64-bit z0).  The pair's second round
    (mi_layer_b*) reduces all.  K (K_lo, K_hi: wave-uniform 64-bit SGPR pairs holding 32-bit
    values) starts the first sum chain in place of 0, so it costs nothing: it adds the field
    constant K_lo + K_hi 2^32 to every output.  poseidon2.hpp chooses K so that element 0 gets
    the next partial round's constant and carries the offset the other elements pick up
    (p2::Sched).

    with_g (mi_layer_a_g, round 6): elements 1..11 arrive half-reduced from the previous pair's
    mi_layer_b_half, as value = lo + hi 2^32 + G 2^32 with a third 32-bit limb G of the same
    weight as hi.  G joins the H sum (11 more mads) and each H_i (one more mad: H_i =
    G_i 2^SH[i] + (hi_i 2^SH[i] + Hs)), 22 instructions against the 33 the producer no longer
    spends finishing its reductions.  Bounds: Ls < 13 * 2^32, Hs < 24 * 2^32, L_i < 2^46.0,
    H_i < 2^47.0 (tests/test_poseidon2_sched.py::test_partial_pair_limb_bounds)."""
    pro = []
    consts, sreg = _consts(pro)
    NC = LAYER_A_CHAINS
    SUM = {("L", c): "v[%d:%d]" % (2 * c, 2 * c + 1) for c in range(NC)}
    SUM.update({("H", c): "v[%d:%d]" % (6 + 2 * c, 7 + 2 * c) for c in range(NC)})
    members = [[i for i in range(12) if i % NC == c] for c in range(NC)]
    chains = []
    for limb, src in (("L", "lo"), ("H", "hi")):
        for c in range(NC):
            ch = []
            for t, i in enumerate(members[c]):
                acc = SUM[(limb, c)]
                start = ("%%[K%s]" % limb) if c == 0 else "0"
                ch.append(("v_mad_u64_u32 %s, %s, %%[%s%d], 1, %s" % (acc, JUNK, src, i, start if t == 0 else acc),
                           set(), {JUNK}))
                if with_g and limb == "H" and i > 0:
                    ch.append(("v_mad_u64_u32 %s, %s, %%[g%d], 1, %s" % (acc, JUNK, i, acc), set(), {JUNK}))
            chains.append(ch)
    body = pro + merge(chains)
    for limb in ("L", "H"):
        a = SUM[(limb, 0)]
        for c in range(1, NC):
            body.append(("v_lshl_add_u64 %s, %s, 0, %s" % (a, SUM[(limb, c)], a), set(), set()))
    Ls, Hs = SUM[("L", 0)], SUM[("H", 0)]
    for i in range(1, 12):
        K = consts.get(SH[i], str(1 << SH[i]))
        body.append(("v_mad_u64_u32 %%[L%d], %s, %%[lo%d], %s, %s" % (i, JUNK, i, K, Ls), set(), {JUNK}))
        body.append(("v_mad_u64_u32 %%[H%d], %s, %%[hi%d], %s, %s" % (i, JUNK, i, K, Hs), set(), {JUNK}))
    if with_g:
        for i in range(1, 12):
            K = consts.get(SH[i], str(1 << SH[i]))
            body.append(("v_mad_u64_u32 %%[H%d], %s, %%[g%d], %s, %%[H%d]" % (i, JUNK, i, K, i), set(), {JUNK}))
    body.append(("v_mad_u64_u32 v[12:13], %s, %%[lo0], %d, %s" % (JUNK, 1 << SH[0], Ls), set(), {JUNK}))
    body.append(("v_mad_u64_u32 v[14:15], %s, %%[hi0], %d, %s" % (JUNK, 1 << SH[0], Hs), set(), {JUNK}))
    body += reduce_limbs("v[12:13]", "v[14:15]", "v[16:17]", "v18", sp(0), "%[z0]")
    text = pad(body)
    name = "mi_layer_a_g" if with_g else "mi_layer_a"
    args = "const uint32_t* lo, const uint32_t* hi, %suint64_t KL, uint64_t KH, uint64_t* L, uint64_t* H, uint64_t& z0" % (
        "const uint32_t* g, " if with_g else "")
    outs = ['[z0] "=&v"(z0)']
    outs += ['[L%d] "=&v"(L[%d]), [H%d] "=&v"(H[%d])' % (i, i, i, i) for i in range(1, 12)]
    ins = ['[lo%d] "v"(lo[%d]), [hi%d] "v"(hi[%d])' % (i, i, i, i) for i in range(12)]
    if with_g:
        ins += ['[g%d] "v"(g[%d])' % (i, i) for i in range(1, 12)]
    ins += ['[KL] "s"(KL)', '[KH] "s"(KH)']
    clob = ['"v%d"' % i for i in range(20)] + ['"s%d"' % i for i in range(SGPR_BASE, sreg)]
    n_v = sum(1 for t in text if t.startswith("v_"))
    what = ("elements 1..11 half-reduced in, " if with_g else "") + "elements 1..11 as limbs L, H"
    lines = ["// Poseidon2 partial round M_I + K, first of a pair: %s (%d VALU instructions)" % (what, n_v),
             "__device__ __forceinline__ void %s(%s) {" % (name, args), "    asm volatile("]
    lines += ['        "%s\\n"' % t for t in text]
    lines += ["        : %s" % ", ".join(outs), "        : %s" % ", ".join(ins), "        : %s);" % ", ".join(clob), "}"]
    return "\n".join(lines) + "\n"


def _layer_b_sums(body):
    """The limb sums of mi_layer_b*: element 0 (lo0, hi0) and the limbs L_i, H_i, i = 1..11,
    into v[0:1] / v[2:3]; two chains per limb for ILP: (0, 1..5) and (6..11)."""
    Ls, Hs = "v[0:1]", "v[2:3]"
    Ls2, Hs2 = "v[4:5]", "v[6:7]"
    chains = []
    for acc, acc2, src, lim in ((Ls, Ls2, "lo", "L"), (Hs, Hs2, "hi", "H")):
        ch = [("v_mad_u64_u32 %s, %s, %%[%s0], 1, %%[%s1]" % (acc, JUNK, src, lim), set(), {JUNK})]
        if LAYER_B_CHAINS == 1:
            for j in range(2, 12):
                ch.append(("v_lshl_add_u64 %s, %%[%s%d], 0, %s" % (acc, lim, j, acc), set(), set()))
            chains.append(ch)
            continue
        for j in range(2, 6):
            ch.append(("v_lshl_add_u64 %s, %%[%s%d], 0, %s" % (acc, lim, j, acc), set(), set()))
        ch2 = [("v_lshl_add_u64 %s, %%[%s6], 0, %%[%s7]" % (acc2, lim, lim), set(), set())]
        for j in range(8, 12):
            ch2.append(("v_lshl_add_u64 %s, %%[%s%d], 0, %s" % (acc2, lim, j, acc2), set(), set()))
        chains += [ch, ch2]
    body += merge(chains)
    if LAYER_B_CHAINS == 2:
        body.append(("v_lshl_add_u64 %s, %s, 0, %s" % (Ls, Ls2, Ls), set(), set()))
        body.append(("v_lshl_add_u64 %s, %s, 0, %s" % (Hs, Hs2, Hs), set(), set()))
    return Ls, Hs


def _layer_b_term(i, Lp, Hp, Ls, Hs, corr=False):
    """L_i' = L_i << SH[i] + sum (element 0: lo0 2^SH[0] + sum), H_i' likewise; with corr,
    element 0 also gets the SGPR constant pair D (DL, DH)."""
    st = []
    if i == 0:
        st.append(("v_mad_u64_u32 %s, %s, %%[lo0], %d, %s" % (Lp, JUNK, 1 << SH[0], Ls), set(), {JUNK}))
        st.append(("v_mad_u64_u32 %s, %s, %%[hi0], %d, %s" % (Hp, JUNK, 1 << SH[0], Hs), set(), {JUNK}))
        if corr:
            st.append(("v_lshl_add_u64 %s, %s, 0, %%[DL]" % (Lp, Lp), set(), set()))
            st.append(("v_lshl_add_u64 %s, %s, 0, %%[DH]" % (Hp, Hp), set(), set()))
    else:
        for P, lim, S in ((Lp, "L", Ls), (Hp, "H", Hs)):
            if SH[i] <= MAX_LSHL_ADD_SHIFT:
                st.append(("v_lshl_add_u64 %s, %%[%s%d], %d, %s" % (P, lim, i, SH[i], S), set(), set()))
            else:
                st.append(("v_lshlrev_b64 %s, %d, %%[%s%d]" % (P, SH[i], lim, i), set(), set()))
                st.append(("v_lshl_add_u64 %s, %s, 0, %s" % (P, P, S), set(), set()))
    return st


def emit_mi_layer_b():
    """Second partial round of a pair: M_I on element 0 (reduced lo0, hi0) and elements 1..11
    as the limbs L_i, H_i < 2^46.6 left by mi_layer_a.  Sums over limbs < 2^50.2;
    L_i' = L_i << SH[i] + sum < 2^61 (one v_lshl_add_u64 when SH[i] <= MAX_LSHL_ADD_SHIFT,
    else shift + add); element 0 also gets the constant D (the next pair's first round
    constant, less the offset the others carry: p2::Sched); then the 4-instruction reduction of
    every element into the 64-bit z[i]."""
    pro = []
    consts, sreg = _consts(pro)
    body = list(pro)
    Ls, Hs = _layer_b_sums(body)
    for g in range(3):
        streams = []
        for j in range(4):
            i = 4 * g + j
            base = 8 + 8 * j
            Lp = "v[%d:%d]" % (base, base + 1)
            Hp = "v[%d:%d]" % (base + 2, base + 3)
            Wp = "v[%d:%d]" % (base + 4, base + 5)
            M = "v%d" % (base + 6)
            st = _layer_b_term(i, Lp, Hp, Ls, Hs, corr=True)
            st += reduce_limbs(Lp, Hp, Wp, M, sp(j), "%%[z%d]" % i)
            streams.append(st)
        body += merge(streams)
    text = pad(body)
    args = "uint32_t lo0, uint32_t hi0, const uint64_t* L, const uint64_t* H, uint64_t DL, uint64_t DH, uint64_t* z"
    outs = ['[z%d] "=&v"(z[%d])' % (i, i) for i in range(12)]
    ins = ['[lo0] "v"(lo0)', '[hi0] "v"(hi0)']
    ins += ['[L%d] "v"(L[%d]), [H%d] "v"(H[%d])' % (i, i, i, i) for i in range(1, 12)]
    ins += ['[DL] "s"(DL)', '[DH] "s"(DH)']
    clob = ['"v%d"' % i for i in range(8 + 32)] + ['"s%d"' % i for i in range(SGPR_BASE, sreg)]
    n_v = sum(1 for t in text if t.startswith("v_"))
    lines = ["// Poseidon2 partial round M_I + D e_0, second of a pair: reduces every element (%d VALU instructions)" % n_v,
             "__device__ __forceinline__ void mi_layer_b(%s) {" % args, "    asm volatile("]
    lines += ['        "%s\\n"' % t for t in text]
    lines += ["        : %s" % ", ".join(outs), "        : %s" % ", ".join(ins), "        : %s);" % ", ".join(clob), "}"]
    return "\n".join(lines) + "\n"


def emit_mi_layer_b_limbs():
    """The last partial round (the second of the last pair): M_I as in mi_layer_b, but the
    outputs stay limbs (L_i' < 2^61, H_i' likewise): the first full round after the partial
    rounds adds its constants to them and reduces, so the pair's own 12 reductions (and the
    moves that re-split reduced words into limbs) are not needed."""
    pro = []
    consts, sreg = _consts(pro)
    body = list(pro)
    Ls, Hs = _layer_b_sums(body)
    for g in range(3):
        streams = []
        for j in range(4):
            i = 4 * g + j
            streams.append(_layer_b_term(i, "%%[Lo%d]" % i, "%%[Ho%d]" % i, Ls, Hs))
        body += merge(streams)
    text = pad(body)
    args = "uint32_t lo0, uint32_t hi0, const uint64_t* L, const uint64_t* H, uint64_t* Lo, uint64_t* Ho"
    outs = ['[Lo%d] "=&v"(Lo[%d]), [Ho%d] "=&v"(Ho[%d])' % (i, i, i, i) for i in range(12)]
    ins = ['[lo0] "v"(lo0)', '[hi0] "v"(hi0)']
    ins += ['[L%d] "v"(L[%d]), [H%d] "v"(H[%d])' % (i, i, i, i) for i in range(1, 12)]
    clob = ['"v%d"' % i for i in range(8)] + ['"s%d"' % i for i in range(SGPR_BASE, sreg)]
    n_v = sum(1 for t in text if t.startswith("v_"))
    lines = ["// Poseidon2 last partial round M_I, outputs as limbs (%d VALU instructions)" % n_v,
             "__device__ __forceinline__ void mi_layer_b_limbs(%s) {" % args, "    asm volatile("]
    lines += ['        "%s\\n"' % t for t in text]
    lines += ["        : %s" % ", ".join(outs), "        : %s" % ", ".join(ins), "        : %s);" % ", ".join(clob), "}"]
    return "\n".join(lines) + "\n"


def emit_mi_layer_b_half():
    """Second partial round of a pair, half-reduced hand-off (round 6): element 0 as in mi_layer_b
    (+ D, reduced into the 64-bit z0: the next pair's S-box input), elements 1..11 left as the
    limbs L_i', H_i' (< 2^60.1, < 2^61.1) of mi_layer_b_limbs.  eps_fold_x11 then forms
    W_i = Hhi_i EPS + L_i' (< 2^62), and the next pair's mi_layer_a_g reads element i as
    W_i + Hlo_i 2^32: one mad per element where the full reduction took four (the carry of
    Hlo into W's high word, its EPS correction and the final mad are gone).  Hlo_i and Hhi_i are
    the halves of the 64-bit output Ho[i]; the consumers take them as 32-bit operands, which the
    compiler maps to the pair's sub-registers (inline asm cannot name a sub-register of its own
    64-bit operand, hence the two blocks)."""
    pro = []
    consts, sreg = _consts(pro)
    body = list(pro)
    Ls, Hs = _layer_b_sums(body)
    for g in range(3):
        streams = []
        for j in range(4):
            i = 4 * g + j
            if i == 0:
                st = _layer_b_term(0, "v[8:9]", "v[10:11]", Ls, Hs, corr=True)
                st += reduce_limbs("v[8:9]", "v[10:11]", "v[12:13]", "v14", sp(0), "%[z0]")
            else:
                st = _layer_b_term(i, "%%[Lo%d]" % i, "%%[Ho%d]" % i, Ls, Hs)
            streams.append(st)
        body += merge(streams)
    text = pad(body)
    args = ("uint32_t lo0, uint32_t hi0, const uint64_t* L, const uint64_t* H, uint64_t DL, uint64_t DH, "
            "uint64_t* Lo, uint64_t* Ho, uint64_t& z0")
    outs = ['[z0] "=&v"(z0)']
    outs += ['[Lo%d] "=&v"(Lo[%d]), [Ho%d] "=&v"(Ho[%d])' % (i, i, i, i) for i in range(1, 12)]
    ins = ['[lo0] "v"(lo0)', '[hi0] "v"(hi0)']
    ins += ['[L%d] "v"(L[%d]), [H%d] "v"(H[%d])' % (i, i, i, i) for i in range(1, 12)]
    ins += ['[DL] "s"(DL)', '[DH] "s"(DH)']
    clob = ['"v%d"' % i for i in range(15)] + ['"s%d"' % i for i in range(SGPR_BASE, sreg)]
    n_v = sum(1 for t in text if t.startswith("v_"))
    lines = ["// Poseidon2 partial round M_I + D e_0, second of a pair: element 0 reduced, 1..11 as limbs (%d VALU instructions)" % n_v,
             "__device__ __forceinline__ void mi_layer_b_half(%s) {" % args, "    asm volatile("]
    lines += ['        "%s\\n"' % t for t in text]
    lines += ["        : %s" % ", ".join(outs), "        : %s" % ", ".join(ins), "        : %s);" % ", ".join(clob), "}"]
    return "\n".join(lines) + "\n"


def emit_eps_fold():
    """W_i = Hhi_i EPS + L_i for i = 1..11: the first step of the limb reduction, as mi_layer_b_half's
    hand-off (Hhi_i the high half of its 64-bit H_i', passed as a 32-bit operand)."""
    body = [("v_mad_u64_u32 %%[W%d], %s, %%[hh%d], -1, %%[L%d]" % (i, JUNK, i, i), set(), {JUNK}) for i in range(1, 12)]
    text = pad(body)
    args = "const uint32_t* hh, const uint64_t* L, uint64_t* W"
    outs = ['[W%d] "=&v"(W[%d])' % (i, i) for i in range(1, 12)]
    ins = ['[hh%d] "v"(hh[%d]), [L%d] "v"(L[%d])' % (i, i, i, i) for i in range(1, 12)]
    lines = ["// W_i = Hhi_i * EPS + L_i, i = 1..11 (11 VALU instructions)",
             "__device__ __forceinline__ void eps_fold_x11(%s) {" % args, "    asm volatile("]
    lines += ['        "%s\\n"' % t for t in text]
    lines += ["        : %s" % ", ".join(outs), "        : %s" % ", ".join(ins), "        : \"s%d\", \"s%d\");" % (SGPR_BASE + 24, SGPR_BASE + 25), "}"]
    return "\n".join(lines) + "\n"


SGPR_OPERANDS = True  # carry / constant SGPRs as compiler-allocated operands (False: fixed s40..)


def sgpr_operandize(fn_text):
    """Turn the fixed SGPRs of one generated asm function into compiler-allocated early-clobber
    outputs: every pair s[a:a+1] becomes a uint64_t "=&s" operand %[qa] and every single sN a
    uint32_t one %[kN]; their clobbers go.  The instruction order (and so the s_nop padding, which
    depends only on the distances between an SGPR's writer and its readers) is unchanged, and
    distinct operands get distinct registers, so the sequence computes the same values; what
    changes is that the compiler is no longer barred from s40..s66 around every asm block (with
    27 SGPRs clobbered, kernels that also need wave-uniform pointers ran short and kept them in
    VGPRs).  The VGPR scratch stays fixed: pairs whose halves are also used alone cannot be
    compiler operands (inline asm has no sub-register syntax)."""
    if not SGPR_OPERANDS:
        return fn_text
    import re
    lines = fn_text.split("\n")
    try:
        a = next(i for i, l in enumerate(lines) if l.strip() == "asm volatile(")
    except StopIteration:
        return fn_text
    b = next(i for i in range(a, len(lines)) if lines[i].strip().startswith(": ") or lines[i].strip() == ":")
    body = "\n".join(lines[a + 1:b])
    pairs = sorted({int(m.group(1)) for m in re.finditer(r"\bs\[(\d+):(\d+)\]", body)})
    singles = sorted({int(m.group(1)) for m in re.finditer(r"(?<![\w\[:])s(\d+)\b", body)})
    assert not any(x in pairs or x - 1 in pairs for x in singles), "single SGPR inside a pair"
    body = re.sub(r"\bs\[(\d+):(\d+)\]", lambda m: "%%[q%s]" % m.group(1), body)
    body = re.sub(r"(?<![\w\[:])s(\d+)\b", lambda m: "%%[k%s]" % m.group(1), body)
    outs_line = lines[b]
    extra = ['[q%d] "=&s"(q%d)' % (x, x) for x in pairs] + ['[k%d] "=&s"(k%d)' % (x, x) for x in singles]
    if extra:
        if outs_line.strip() == ":":
            outs_line = outs_line.rstrip() + " " + ", ".join(extra)
        else:
            outs_line = outs_line.rstrip() + ", " + ", ".join(extra)
    clob_i = b + 2
    clob = lines[clob_i]
    clob = re.sub(r',?\s*"s\d+"', "", clob).replace(":,", ":").replace(": ,", ":")
    decl = []
    if pairs:
        decl.append("    uint64_t %s;" % ", ".join("q%d" % x for x in pairs))
    if singles:
        decl.append("    uint32_t %s;" % ", ".join("k%d" % x for x in singles))
    out = lines[:a] + decl + [lines[a]] + body.split("\n") + [outs_line, lines[b + 1], clob] + lines[clob_i + 1:]
    return "\n".join(out)


def main():
    import argparse
    global LAYER_A_CHAINS, LAYER_B_CHAINS
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=OUT, help="output header (variants for A/B builds elsewhere)")
    ap.add_argument("--a-chains", type=int, default=LAYER_A_CHAINS, choices=(1, 2, 3))  # L sums in v0..v5, H in v6..v11
    ap.add_argument("--b-chains", type=int, default=LAYER_B_CHAINS, choices=(1, 2))
    args = ap.parse_args()
    LAYER_A_CHAINS, LAYER_B_CHAINS = args.a_chains, args.b_chains
    parts = ['''// GENERATED by tools/gen_gl_asm.py -- do not edit.
// gfx950 inline-asm Goldilocks primitives (see the generator's docstring for the
// design and the hazard rule).  p = 2^64 - 2^32 + 1.  All values are (lo, hi) 32-bit
// halves of u64 representatives; results are NOT canonicalised.
#pragma once
#include <stdint.h>

namespace glasm {
''']
    for n in (1, 2, 3, 4):
        parts.append(emit_fn("mul_x%d" % n, n, mul_stream, 10, ["a0", "a1", "b0", "b1"], ["z0", "z1"],
                             doc="%d independent products z = a * b mod p (14 instructions each)" % n))
    # the same products with a wave-uniform multiplier b in SGPRs (each mad reads one SGPR: gfx950's
    # constant-bus limit), so uniform factors need no VGPR copies
    parts.append(emit_fn("mul_sb_x4", 4, mul_stream, 10, ["a0", "a1", "b0", "b1"], ["z0", "z1"],
                         in_cons={"b0": "s", "b1": "s"},
                         doc="4 independent products z = a * b mod p, b wave-uniform in SGPRs (14 instructions each)"))
    for n in (1, 2, 3, 4):
        parts.append(emit_fn("reduce_x%d" % n, n, lambda k, vb: reduce_stream(k, vb, pair_out=True), 4,
                             ["L", "Hlo", "Hhi"], ["z"], in_kinds={"L": "uint64_t"}, out_kinds={"z": "uint64_t"},
                             doc="%d reductions z = L + (Hhi:Hlo) * 2^32 mod p, L and H < 2^63 "
                                 "(4 instructions each, z a 64-bit register pair)" % n))
    for n in (1, 2, 4):
        parts.append(emit_fn("add_x%d" % n, n, lambda k, vb: addsub_stream(k, vb, "add"), 2,
                             ["a0", "a1", "b0", "b1"], ["z0", "z1"], doc="%d general additions" % n))
        parts.append(emit_fn("sub_x%d" % n, n, lambda k, vb: addsub_stream(k, vb, "sub"), 2,
                             ["a0", "a1", "b0", "b1"], ["z0", "z1"], doc="%d general subtractions" % n))
    for n in (1, 4):
        parts.append(emit_ct_bfly(n))
    for n in (1, 2, 4):
        parts.append(emit_fn("canon_x%d" % n, n, canon_stream, 2, ["a0", "a1"], ["z0", "z1"],
                             doc="%d canonicalisations z = x mod p in [0, p)" % n))
    parts.append(emit_mi_layer_a())
    parts.append(emit_mi_layer_b())
    parts.append(emit_mi_layer_b_limbs())
    parts.append(emit_mi_layer_a(with_g=True))
    parts.append(emit_mi_layer_b_half())
    parts.append(emit_eps_fold())
    parts.append("}  // namespace glasm\n")
    parts = [sgpr_operandize(x) for x in parts]
    with open(args.out, "w") as f:
        f.write("\n".join(parts))
    print("wrote", args.out)


if __name__ == "__main__":
    main()
