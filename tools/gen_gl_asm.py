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


def reduce_stream(k, vbase):
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


def ct_bfly_stream(k, vbase):
    """Cooley-Tukey butterfly in place: (a, c) <- (a + c w, a - c w), 28 instructions.
    t = c * w (mul_stream, result left in its U pair), canonicalised (t + EPS overflows iff
    t >= p).  With t < p, a - t borrows at most once and a + t wraps 2^64 at most once, so each
    needs a single EPS correction (5 instructions instead of 8).  The difference goes into c's
    registers (c is dead after the products), then the sum into a's.
    Operands: a0,a1 and c0,c1 read-write; w0,w1 read."""
    P0, P1, U0, U1 = ["v%d" % (vbase + i) for i in range(4)]
    M = "v%d" % (vbase + 8)
    p0, p1, p2 = sp(3 * k), sp(3 * k + 1), sp(3 * k + 2)
    a0, a1, c0, c1 = ["%%[%s%d]" % (n, k) for n in ("a0", "a1", "c0", "c1")]
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
    # c = a - t: one borrow at most, worth -2^64 == -EPS
    I.append(("v_sub_co_u32 %s, %s, %s, %s" % (c0, p1, a0, U0), set(), {p1}))
    I.append(("v_subb_co_u32 %s, %s, %s, %s, %s" % (c1, p1, a1, U1, p1), {p1}, {p1}))
    I.append(("v_cndmask_b32_e64 %s, 0, -1, %s" % (M, p1), {p1}, set()))
    I.append(("v_sub_co_u32 %s, %s, %s, %s" % (c0, p2, c0, M), set(), {p2}))
    I.append(("v_subb_co_u32 %s, %s, %s, 0, %s" % (c1, JUNK, c1, p2), {p2}, {JUNK}))
    # a = a + t: one wrap at most, worth 2^64 == EPS
    I.append(("v_add_co_u32 %s, %s, %s, %s" % (a0, p0, a0, U0), set(), {p0}))
    I.append(("v_addc_co_u32 %s, %s, %s, %s, %s" % (a1, p0, a1, U1, p0), {p0}, {p0}))
    I.append(("v_cndmask_b32_e64 %s, 0, -1, %s" % (M, p0), {p0}, set()))
    I.append(("v_add_co_u32 %s, %s, %s, %s" % (a0, p1, a0, M), set(), {p1}))
    I.append(("v_addc_co_u32 %s, %s, %s, 0, %s" % (a1, JUNK, a1, p1), {p1}, {JUNK}))
    return I


def emit_ct_bfly(n):
    streams = [ct_bfly_stream(k, 10 * k) for k in range(n)]  # 64-bit tuples even-aligned
    body = interleave(streams)
    args, outs, ins = [], [], []
    for k in range(n):
        args += ["uint32_t& a0%d" % k, "uint32_t& a1%d" % k, "uint32_t& c0%d" % k, "uint32_t& c1%d" % k,
                 "uint32_t w0%d" % k, "uint32_t w1%d" % k]
        outs += ['[%s%d] "+v"(%s%d)' % (nm, k, nm, k) for nm in ("a0", "a1", "c0", "c1")]
        ins += ['[%s%d] "v"(%s%d)' % (nm, k, nm, k) for nm in ("w0", "w1")]
    clob = ['"v%d"' % i for i in range(10 * n - 1)] + ['"s%d"' % i for i in range(SGPR_BASE, SGPR_BASE + 26)]
    lines = ["// %d in-place Cooley-Tukey butterflies (a, c) <- (a + c w, a - c w) (28 instructions each)" % n,
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


def emit_fn(name, n, stream_fn, vper, in_names, out_names, in_kinds=None, doc=""):
    streams = [stream_fn(k, vper * k) for k in range(n)]
    body = interleave(streams)
    n_v = vper * n
    args = []
    for k in range(n):
        for nm in in_names:
            kind = (in_kinds or {}).get(nm, "uint32_t")
            args.append("%s %s%d" % (kind, nm, k))
        for nm in out_names:
            args.append("uint32_t& %s%d" % (nm, k))
    outs = ", ".join('[%s%d] "=&v"(%s%d)' % (nm, k, nm, k) for k in range(n) for nm in out_names)
    ins = ", ".join('[%s%d] "v"(%s%d)' % (nm, k, nm, k) for k in range(n) for nm in in_names)
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


def emit_mi_layer():
    """Partial-round internal linear layer on a reduced state (lo[i], hi[i] 32-bit):
    s_i' = s_i * 2^SH[i] + sum_j s_j  (M_I = diag(2^SH) + 1 1^T, state_generic_impl.rs:166-202).
    Limb form: Ls = sum lo_j, Hs = sum hi_j (mad chains, no zero-extension), then per element
    L = lo_i * 2^k + Ls, H = hi_i * 2^k + Hs (one mad each; < 2^47) and the 5-instruction
    limb reduction.  One asm block, 12 elements reduced 4 at a time."""
    SUM = {("L", c): "v[%d:%d]" % (2 * c, 2 * c + 1) for c in range(3)}
    SUM.update({("H", c): "v[%d:%d]" % (6 + 2 * c, 7 + 2 * c) for c in range(3)})
    consts = {}
    sreg = SGPR_BASE + 26
    pro = []
    for k in sorted(set(SH)):
        if k > 6:
            consts[k] = "s%d" % sreg
            pro.append(("s_mov_b32 s%d, %d" % (sreg, 1 << k), set(), set()))
            sreg += 1
    chains = []
    for limb, src in (("L", "lo"), ("H", "hi")):
        for c in range(3):
            ch = []
            for t in range(4):
                i = 4 * c + t
                acc = SUM[(limb, c)]
                ch.append(("v_mad_u64_u32 %s, %s, %%[%s%d], 1, %s" % (acc, JUNK, src, i, "0" if t == 0 else acc),
                           set(), {JUNK}))
            chains.append(ch)
    body = pro + merge(chains)
    for limb in ("L", "H"):
        a = SUM[(limb, 0)]
        body.append(("v_lshl_add_u64 %s, %s, 0, %s" % (a, SUM[(limb, 1)], a), set(), set()))
        body.append(("v_lshl_add_u64 %s, %s, 0, %s" % (a, SUM[(limb, 2)], a), set(), set()))
    Ls, Hs = SUM[("L", 0)], SUM[("H", 0)]
    for g in range(3):
        streams = []
        for j in range(4):
            i = 4 * g + j
            base = 12 + 8 * j
            Lp = "v[%d:%d]" % (base, base + 1)
            Hp = "v[%d:%d]" % (base + 2, base + 3)
            H0, H1 = "v%d" % (base + 2), "v%d" % (base + 3)
            Wp = "v[%d:%d]" % (base + 4, base + 5)
            W0, W1, M = "v%d" % (base + 4), "v%d" % (base + 5), "v%d" % (base + 6)
            K = consts.get(SH[i], str(1 << SH[i]))
            c = sp(j)
            st = [
                ("v_mad_u64_u32 %s, %s, %%[lo%d], %s, %s" % (Lp, JUNK, i, K, Ls), set(), {JUNK}),
                ("v_mad_u64_u32 %s, %s, %%[hi%d], %s, %s" % (Hp, JUNK, i, K, Hs), set(), {JUNK}),
                ("v_mad_u64_u32 %s, %s, %s, -1, %s" % (Wp, JUNK, H1, Lp), set(), {JUNK}),
                ("v_add_co_u32 %s, %s, %s, %s" % (W1, c, W1, H0), set(), {c}),
                ("v_cndmask_b32_e64 %s, 0, -1, %s" % (M, c), {c}, set()),
                ("v_add_co_u32 %%[lo%d], %s, %s, %s" % (i, c, W0, M), set(), {c}),
                ("v_addc_co_u32 %%[hi%d], %s, %s, 0, %s" % (i, JUNK, W1, c), {c}, {JUNK}),
            ]
            streams.append(st)
        body += merge(streams)
    text = pad(body)
    # in place: element i's result overwrites lo[i]/hi[i] only after every read of them
    # (the sums read all inputs first; element i's own mads read lo[i]/hi[i] before its write)
    args = ", ".join(["uint32_t* lo", "uint32_t* hi"])
    outs = ", ".join('[lo%d] "+v"(lo[%d]), [hi%d] "+v"(hi[%d])' % (i, i, i, i) for i in range(12))
    ins = ""
    clob = ['"v%d"' % i for i in range(12 + 32)] + ['"s%d"' % i for i in range(SGPR_BASE, sreg)]
    lines = ["// Poseidon2 partial-round M_I on a reduced state (%d VALU instructions)" % sum(1 for t in text if t.startswith("v_")),
             "__device__ __forceinline__ void mi_layer(%s) {" % args, "    asm volatile("]
    lines += ['        "%s\\n"' % t for t in text]
    lines += ["        : %s" % outs, "        : %s" % ins, "        : %s);" % ", ".join(clob), "}"]
    return "\n".join(lines) + "\n"


# v_lshl_add_u64 shift amounts verified on gfx950 hardware (tools/isa_probe.hip)
MAX_LSHL_ADD_SHIFT = 4


def reduce_limbs(Lp, Hp, Wp, M, c, z0, z1):
    """The 5-instruction limb reduction (reduce_stream) on register pairs Lp, Hp -> z0, z1."""
    H0, H1 = Hp.split("[")[1].rstrip("]").split(":")
    H0, H1 = "v" + H0, "v" + H1
    W0, W1 = Wp.split("[")[1].rstrip("]").split(":")
    W0, W1 = "v" + W0, "v" + W1
    return [
        ("v_mad_u64_u32 %s, %s, %s, -1, %s" % (Wp, JUNK, H1, Lp), set(), {JUNK}),
        ("v_add_co_u32 %s, %s, %s, %s" % (W1, c, W1, H0), set(), {c}),
        ("v_cndmask_b32_e64 %s, 0, -1, %s" % (M, c), {c}, set()),
        ("v_add_co_u32 %s, %s, %s, %s" % (z0, c, W0, M), set(), {c}),
        ("v_addc_co_u32 %s, %s, %s, 0, %s" % (z1, JUNK, W1, c), {c}, {JUNK}),
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


def emit_mi_layer_a():
    """First partial round of a pair: M_I with elements 1..11 left as unreduced limbs.
    L_i = lo_i 2^SH[i] + sum lo_j, H_i likewise (one mad each, < 2^46.6); only element 0,
    the next S-box input, is reduced.  The pair's second round (mi_layer_b) reduces all."""
    pro = []
    consts, sreg = _consts(pro)
    SUM = {("L", c): "v[%d:%d]" % (2 * c, 2 * c + 1) for c in range(3)}
    SUM.update({("H", c): "v[%d:%d]" % (6 + 2 * c, 7 + 2 * c) for c in range(3)})
    chains = []
    for limb, src in (("L", "lo"), ("H", "hi")):
        for c in range(3):
            ch = []
            for t in range(4):
                i = 4 * c + t
                acc = SUM[(limb, c)]
                ch.append(("v_mad_u64_u32 %s, %s, %%[%s%d], 1, %s" % (acc, JUNK, src, i, "0" if t == 0 else acc),
                           set(), {JUNK}))
            chains.append(ch)
    body = pro + merge(chains)
    for limb in ("L", "H"):
        a = SUM[(limb, 0)]
        body.append(("v_lshl_add_u64 %s, %s, 0, %s" % (a, SUM[(limb, 1)], a), set(), set()))
        body.append(("v_lshl_add_u64 %s, %s, 0, %s" % (a, SUM[(limb, 2)], a), set(), set()))
    Ls, Hs = SUM[("L", 0)], SUM[("H", 0)]
    for i in range(1, 12):
        K = consts.get(SH[i], str(1 << SH[i]))
        body.append(("v_mad_u64_u32 %%[L%d], %s, %%[lo%d], %s, %s" % (i, JUNK, i, K, Ls), set(), {JUNK}))
        body.append(("v_mad_u64_u32 %%[H%d], %s, %%[hi%d], %s, %s" % (i, JUNK, i, K, Hs), set(), {JUNK}))
    body.append(("v_mad_u64_u32 v[12:13], %s, %%[lo0], %d, %s" % (JUNK, 1 << SH[0], Ls), set(), {JUNK}))
    body.append(("v_mad_u64_u32 v[14:15], %s, %%[hi0], %d, %s" % (JUNK, 1 << SH[0], Hs), set(), {JUNK}))
    body += reduce_limbs("v[12:13]", "v[14:15]", "v[16:17]", "v18", sp(0), "%[lo0]", "%[hi0]")
    text = pad(body)
    args = "uint32_t* lo, uint32_t* hi, uint64_t* L, uint64_t* H"
    outs = ['[lo0] "+v"(lo[0])', '[hi0] "+v"(hi[0])']
    outs += ['[L%d] "=&v"(L[%d]), [H%d] "=&v"(H[%d])' % (i, i, i, i) for i in range(1, 12)]
    ins = ['[lo%d] "v"(lo[%d]), [hi%d] "v"(hi[%d])' % (i, i, i, i) for i in range(1, 12)]
    clob = ['"v%d"' % i for i in range(20)] + ['"s%d"' % i for i in range(SGPR_BASE, sreg)]
    n_v = sum(1 for t in text if t.startswith("v_"))
    lines = ["// Poseidon2 partial round M_I, first of a pair: elements 1..11 as limbs L, H (%d VALU instructions)" % n_v,
             "__device__ __forceinline__ void mi_layer_a(%s) {" % args, "    asm volatile("]
    lines += ['        "%s\\n"' % t for t in text]
    lines += ["        : %s" % ", ".join(outs), "        : %s" % ", ".join(ins), "        : %s);" % ", ".join(clob), "}"]
    return "\n".join(lines) + "\n"


def emit_mi_layer_b():
    """Second partial round of a pair: M_I on element 0 (reduced lo0, hi0) and elements 1..11
    as the limbs L_i, H_i < 2^46.6 left by mi_layer_a.  Sums over limbs < 2^50.2;
    L_i' = L_i << SH[i] + sum < 2^61 (one v_lshl_add_u64 when SH[i] <= MAX_LSHL_ADD_SHIFT,
    else shift + add); then the 5-instruction reduction of every element."""
    pro = []
    consts, sreg = _consts(pro)
    Ls, Hs = "v[0:1]", "v[2:3]"
    Ls2, Hs2 = "v[4:5]", "v[6:7]"
    body = list(pro)
    # two chains per limb for ILP: (0, 1..5) and (6..11)
    chains = []
    for acc, acc2, src, lim in ((Ls, Ls2, "lo", "L"), (Hs, Hs2, "hi", "H")):
        ch = [("v_mad_u64_u32 %s, %s, %%[%s0], 1, %%[%s1]" % (acc, JUNK, src, lim), set(), {JUNK})]
        for j in range(2, 6):
            ch.append(("v_lshl_add_u64 %s, %%[%s%d], 0, %s" % (acc, lim, j, acc), set(), set()))
        ch2 = [("v_lshl_add_u64 %s, %%[%s6], 0, %%[%s7]" % (acc2, lim, lim), set(), set())]
        for j in range(8, 12):
            ch2.append(("v_lshl_add_u64 %s, %%[%s%d], 0, %s" % (acc2, lim, j, acc2), set(), set()))
        chains += [ch, ch2]
    body += merge(chains)
    body.append(("v_lshl_add_u64 %s, %s, 0, %s" % (Ls, Ls2, Ls), set(), set()))
    body.append(("v_lshl_add_u64 %s, %s, 0, %s" % (Hs, Hs2, Hs), set(), set()))
    for g in range(3):
        streams = []
        for j in range(4):
            i = 4 * g + j
            base = 8 + 8 * j
            Lp = "v[%d:%d]" % (base, base + 1)
            Hp = "v[%d:%d]" % (base + 2, base + 3)
            Wp = "v[%d:%d]" % (base + 4, base + 5)
            M = "v%d" % (base + 6)
            c = sp(j)
            st = []
            if i == 0:
                st.append(("v_mad_u64_u32 %s, %s, %%[lo0], %d, %s" % (Lp, JUNK, 1 << SH[0], Ls), set(), {JUNK}))
                st.append(("v_mad_u64_u32 %s, %s, %%[hi0], %d, %s" % (Hp, JUNK, 1 << SH[0], Hs), set(), {JUNK}))
            else:
                for P, lim, S in ((Lp, "L", Ls), (Hp, "H", Hs)):
                    if SH[i] <= MAX_LSHL_ADD_SHIFT:
                        st.append(("v_lshl_add_u64 %s, %%[%s%d], %d, %s" % (P, lim, i, SH[i], S), set(), set()))
                    else:
                        st.append(("v_lshlrev_b64 %s, %d, %%[%s%d]" % (P, SH[i], lim, i), set(), set()))
                        st.append(("v_lshl_add_u64 %s, %s, 0, %s" % (P, P, S), set(), set()))
            st += reduce_limbs(Lp, Hp, Wp, M, c, "%%[lo%d]" % i, "%%[hi%d]" % i)
            streams.append(st)
        body += merge(streams)
    text = pad(body)
    args = "uint32_t* lo, uint32_t* hi, const uint64_t* L, const uint64_t* H"
    outs = ['[lo0] "+v"(lo[0])', '[hi0] "+v"(hi[0])']
    outs += ['[lo%d] "=&v"(lo[%d]), [hi%d] "=&v"(hi[%d])' % (i, i, i, i) for i in range(1, 12)]
    ins = ['[L%d] "v"(L[%d]), [H%d] "v"(H[%d])' % (i, i, i, i) for i in range(1, 12)]
    clob = ['"v%d"' % i for i in range(8 + 32)] + ['"s%d"' % i for i in range(SGPR_BASE, sreg)]
    n_v = sum(1 for t in text if t.startswith("v_"))
    lines = ["// Poseidon2 partial round M_I, second of a pair: reduces every element (%d VALU instructions)" % n_v,
             "__device__ __forceinline__ void mi_layer_b(%s) {" % args, "    asm volatile("]
    lines += ['        "%s\\n"' % t for t in text]
    lines += ["        : %s" % ", ".join(outs), "        : %s" % ", ".join(ins), "        : %s);" % ", ".join(clob), "}"]
    return "\n".join(lines) + "\n"


def main():
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
    for n in (1, 2, 3, 4):
        parts.append(emit_fn("reduce_x%d" % n, n, reduce_stream, 4, ["L", "Hlo", "Hhi"], ["z0", "z1"],
                             in_kinds={"L": "uint64_t"},
                             doc="%d reductions z = L + (Hhi:Hlo) * 2^32 mod p, L and H < 2^63" % n))
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
    parts.append(emit_mi_layer())
    parts.append(emit_mi_layer_a())
    parts.append(emit_mi_layer_b())
    parts.append("}  // namespace glasm\n")
    with open(OUT, "w") as f:
        f.write("\n".join(parts))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
