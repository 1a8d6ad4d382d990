#!/usr/bin/env python3
"""Static VALU census of one Poseidon2 permutation as compiled for gfx950.

The permutation (csrc/poseidon2.hpp) has three `#pragma unroll 1` round loops with fixed
trip counts: 4 full rounds, 9 pairs of partial rounds (pair 0, which takes reduced words, is peeled;
round 6) and 2 full rounds (peeled: the last pair
of partial rounds, which hands limbs to the first full round after it; that round, which takes
its constants from the schedule; and the last full round, so that its MDS forms only the outputs
the caller reads). The census kernels of
tools/census_perm.hip run exactly one permutation per lane in each output form (all 12
words, the capacity words, the digest), so their dynamic instruction stream is known
statically:
    straight-line code x1 + loop bodies x (4, 9, 2).
This tool disassembles the gfx950 code object and weights each VALU instruction by the
issue cost measured in profiles/r1_isa_rates.txt:
* 1 slot: full-rate 32-bit ops (v_add_u32, v_mov_b32, logic);
* 2 slots: carry, 64-bit and multiply ops.
The output is the issue-slot count per permutation, which bench.py uses for the leaf
kernel's VALU roofline.

usage: python tools/valu_census.py [--json out.json]
"""
import argparse
import json
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
HIPCC = "/opt/rocm/bin/hipcc"

# full rate on gfx950 (profiles/r1_isa_rates.txt, r1n_isa_rates_alu32.txt): VOP2 32-bit add /
# logic / shift / move and v_bitop3_b32; the VOP3-only 32-bit forms (v_add3, v_alignbit,
# v_perm, v_lshl_or, v_xad, v_or3, ...) issue at half rate like the carry / 64-bit ops
FULL_RATE = re.compile(r"^v_(add_u32_e32|sub_u32_e32|mov_b32|and_b32_e32|or_b32_e32|xor_b32_e32|lshlrev_b32_e32|"
                       r"lshrrev_b32_e32|not_b32|bitop3_b32)")


def disassemble(name="merkle", src=None):
    src = src or os.path.join(ROOT, "era-boojum_amd", "csrc", name + ".hip")
    dev = "/tmp/_census_%s_dev.o" % name
    co = "/tmp/_census_%s.co" % name
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-c", "-o", dev,
                    src], check=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + dev,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
    return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co], check=True, capture_output=True,
                          text=True).stdout


def kernel_lines(dis, name):
    out, on = [], False
    for line in dis.splitlines():
        if line.endswith(">:"):
            on = name in line
            continue
        if on and line.strip():
            out.append(line)
    return out


def parse(lines):
    """[(addr, mnemonic, branch_target_addr|None)]"""
    instrs = []
    for line in lines:
        m = re.match(r"\s+(\S+).*//\s*([0-9A-Fa-f]+):", line)
        if not m:
            continue
        mn, addr = m.group(1), int(m.group(2), 16)
        tgt = None
        t = re.search(r"<[^+>]+\+0x([0-9a-f]+)>", line)
        if mn.startswith("s_cbranch") or mn == "s_branch":
            if t:
                tgt = int(t.group(1), 16)
        instrs.append((addr, mn, tgt))
    return instrs


def census(instrs, trips=(4, 9, 2)):
    base = instrs[0][0]
    back = [(i, a, t) for i, (a, mn, t) in enumerate(instrs) if t is not None and base + t < a]
    if len(back) != len(trips):
        raise SystemExit("expected %d backward branches, found %d" % (len(trips), len(back)))
    weight = [1] * len(instrs)
    for (i_end, _, t), trip in zip(back, trips):
        start = next(k for k, (a, _, _) in enumerate(instrs) if a == base + t)
        for k in range(start, i_end + 1):
            weight[k] = trip
    valu = slots = 0
    hist = {}
    for (a, mn, _), w in zip(instrs, weight):
        if not mn.startswith("v_"):
            continue
        cost = 1 if FULL_RATE.match(mn) else 2
        valu += w
        slots += w * cost
        hist[mn] = hist.get(mn, 0) + w
    return valu, slots, hist


def straight_line(instrs):
    """(VALU instructions, issue slots) of a kernel without loops, every instruction once."""
    valu = slots = 0
    for _, mn, _ in instrs:
        if mn.startswith("v_"):
            valu += 1
            slots += 1 if FULL_RATE.match(mn) else 2
    return valu, slots


def ntt_census():
    """Per-wave VALU instructions and issue slots of the coset-folded CT passes (ntt_ct.hip):
    ct_head_kernel<R, MODE, KAPPA> for R = log n - 13 (forward: MODE 1, no kappa; inverse:
    MODE 0, inverse roots) and ct_tail_kernel<true, INV>. They are fully unrolled (no loops), so one wave
    executes each instruction once; bench.py multiplies by the launched waves for the NTT
    phase's VALU utilisation."""
    dis = disassemble("ntt_ct")
    out = {}
    for r in range(5, 11):
        # the power-of-two heads the LDE launches at 2^18 .. 2^23 (P2 = true; INV false / true)
        for key, tmpl in (("head_fwd", "ct_head_kernelILi%dELi1ELb0ELb0ELb1ELb0E" % r),
                          ("head_inv", "ct_head_kernelILi%dELi0ELb0ELb0ELb1ELb1E" % r)):
            ins = parse(kernel_lines(dis, tmpl))
            if ins:
                v, s = straight_line(ins)
                out.setdefault(key, {})[str(r)] = {"valu": v, "slots": s}
    # the LDE's tails canonicalise their output (ct_tail_kernel<true, INV>); match one
    # instantiation each (a name prefix alone matches several)
    v, s = straight_line(parse(kernel_lines(dis, "ct_tail_kernelILb1ELb0E")))
    out["tail"] = {"valu": v, "slots": s}
    v, s = straight_line(parse(kernel_lines(dis, "ct_tail_kernelILb1ELb1E")))
    out["tail_inv"] = {"valu": v, "slots": s}
    out["waves_per_block"] = 4
    out["elements_per_block"] = 8192
    return out


def lde3_census():
    """Per-wave issue slots of the three-pass LDE's kernels (ntt_lde3.hip) for R = log n - 13:
    the middle pass lde3_mid_kernel<R, true, false> (the inverse tail outside its coset loop, one
    forward stage 0..12 set per loop trip; the form bj_lde_ex_d runs without
    BJ_LDE_KEEP_MONOMIALS, as the bench and the commits do; "mid_mono" is the monomial-storing form) and the final pass
    lde3_final_kernel<R, 0> (no loops).  bench.py prices the LDE phase with them (plus the
    inverse head, head_inv above)."""
    dis = disassemble("ntt_lde3")
    out = {}
    for r in range(5, 11):
        for key, mono in (("mid", 0), ("mid_mono", 1)):
            ins = parse(kernel_lines(dis, "lde3_mid_kernelILi%dELb1ELb%dE" % (r, mono)))
            if ins:
                o, body = loop_census(ins)
                out.setdefault(key, {})[str(r)] = {"slots_outside_loop": o, "slots_per_coset": body}
        ins = parse(kernel_lines(dis, "lde3_final_kernelILi%dELi0E" % r))
        if ins:
            v, s = straight_line(ins)
            out.setdefault("final", {})[str(r)] = {"valu": v, "slots": s}
    out["waves_per_block"] = 4
    out["elements_per_block"] = 8192
    return out


def loop_census(instrs):
    """(slots outside the single loop, slots of one loop iteration) of a kernel with one loop."""
    base = instrs[0][0]
    back = [(i, a, t) for i, (a, mn, t) in enumerate(instrs) if t is not None and base + t < a]
    if not back:
        raise SystemExit("no loop found")
    # the loop is the widest backward edge; the others return from out-of-line blocks
    spans = []
    for i_end, a, t in back:
        start = next(k for k, (aa, _, _) in enumerate(instrs) if aa == base + t)
        spans.append((i_end - start, start, i_end))
    _, start, i_end = max(spans)
    out = body = 0
    for k, (_, mn, _) in enumerate(instrs):
        if not mn.startswith("v_"):
            continue
        cost = 1 if FULL_RATE.match(mn) else 2
        if start <= k <= i_end:
            body += cost
        else:
            out += cost
    return out, body


def blake2s_census():
    """Issue slots of the Blake2s256 leaf kernel (b2s_leaf_kernel<false, true>): a leaf of C
    columns (C % 8 == 0) runs the block loop C/8 - 1 times plus the final block outside it."""
    dis = disassemble("blake2s")
    ins = parse(kernel_lines(dis, "b2s_leaf_kernelILb0ELb1E"))
    out, body = loop_census(ins)
    return {"kernel": "b2s_leaf_kernel<false, true>", "slots_outside_loop": out, "slots_per_block": body}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json")
    args = ap.parse_args()
    # one permutation per lane in each output form (tools/census_perm.hip): the loads and stores
    # around it are a few instructions of 10k
    dis = disassemble("census_perm", os.path.join(ROOT, "tools", "census_perm.hip"))
    forms = {}
    for form in ("all", "cap", "digest"):
        valu, slots, hist = census(parse(kernel_lines(dis, "census_perm_" + form)))
        forms[form] = {"valu": valu, "slots": slots}
        if form == "all":
            top = dict(sorted(hist.items(), key=lambda kv: -kv[1])[:12])
    res = {"kernel": "census_perm_{all,cap,digest} (tools/census_perm.hip: one Poseidon2 permutation per lane)",
           "valu_instr_per_perm": forms["all"]["valu"], "issue_slots_per_perm": forms["all"]["slots"],
           "perm_forms": forms,
           "top": top,
           "ntt_ct": ntt_census(),
           "lde3": lde3_census(),
           "blake2s": blake2s_census()}
    print(json.dumps(res, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
