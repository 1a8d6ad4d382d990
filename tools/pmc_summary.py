#!/usr/bin/env python3
"""Per-launch HBM traffic and VALU counters from rocprofv3 PMC passes (scripts/profile_pass.sh).

Reads <dir>/fetch, <dir>/write and <dir>/sq run_counter_collection.csv files, averages each
counter per kernel over its dispatches and writes profiles/pmc_summary.json:
  {config: {kernel_key: {fetch_bytes, write_bytes, hbm_bytes_per_launch, sq_insts_valu, ...}}}

Units and gfx950 corrections (MI355X_MICROARCH.md, HBM section):
* FETCH_SIZE and WRITE_SIZE are in KiB.
* FETCH_SIZE reports half the bytes of every read shape these kernels use, calibrated
  independently of them on known byte counts (tools/fetch_calibration.hip, 2 GiB each,
  profiles/r2a_fetch_calibration.json): 8-byte-per-lane column loads (the leaf kernel's and the
  NTT tails' shape) 0.5000, 128-byte runs of 8-byte lanes (the NTT heads' strided rows) 0.5000,
  16-byte-per-lane streams 0.5000.  WRITE_SIZE equals the bytes of 8-byte-per-lane stores
  (1.0000).  So every read is doubled (the third field of KERNELS) and writes are taken as is.

usage: python tools/pmc_summary.py gpurun_out/prof_TAG [--config C3]
"""
import argparse
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# kernel-name prefix (after an optional "void ") -> (key, FETCH_SIZE read factor)
KERNELS = [
    ("bj::leaf_hash_kernel", "leaf_hash_kernel", 2.0),
    ("bj::node_level_kernel", "node_level_kernel", 1.0),
    # the small levels (<= 2^15 nodes), one node per quad of lanes: part of the node phase
    ("bj::node_level_q4_kernel", "node_level_q4_kernel", 1.0),
    ("bj::node_tail_kernel", "node_tail_kernel", 1.0),
    ("bj::(anonymous namespace)::ct_head_kernel<9, 1", "ct_head_fwd", 2.0),
    ("bj::(anonymous namespace)::ct_head_kernel<9, 0", "ct_head_inv", 2.0),
    ("bj::(anonymous namespace)::ct_tail_kernel", "ct_tail", 2.0),
    ("bj::(anonymous namespace)::lde3_mid_kernel<9", "lde3_mid", 2.0),
    ("bj::(anonymous namespace)::lde3_final_kernel<9", "lde3_final", 2.0),
    ("bj::(anonymous namespace)::dif_head_kernel<9, 1>", "dif_head_fwd", 2.0),
    ("bj::(anonymous namespace)::dif_head_kernel<9, 0>", "dif_head_inv", 2.0),
    ("bj::(anonymous namespace)::dif_tail_kernel", "dif_tail", 2.0),
]


def key_of(name):
    if name.startswith("void "):
        name = name[5:]
    for pre, key, fac in KERNELS:
        if name.startswith(pre):
            return key, fac
    return None, None


def load(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return acc
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        per[(r["Dispatch_Id"], r["Kernel_Name"])][r["Counter_Name"]] = float(r["Counter_Value"])
    for (_, name), ctrs in per.items():
        k, _ = key_of(name)
        if k:
            for c, v in ctrs.items():
                acc[k][c].append(v)
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--config", default="C3")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_summary.json"))
    args = ap.parse_args()
    data = {}
    for sub in ("fetch", "write", "sq"):
        for k, ctrs in load(os.path.join(args.dir, sub, "run_counter_collection.csv")).items():
            d = data.setdefault(k, {})
            for c, vals in ctrs.items():
                d[c] = sum(vals) / len(vals)
                d[c + "_dispatches"] = len(vals)
    # the source hashes of the library the passes ran (build_info.json, written by build()):
    # bench.py quotes an entry only while the built library's hash for its group is the same
    sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))
    from boojum_amd import srchash
    info = os.path.join(ROOT, "era-boojum_amd", "boojum_amd", "build_info.json")
    hashes = json.load(open(info))["src_hash"] if os.path.exists(info) else srchash.source_hashes()
    out = {}
    for k, d in data.items():
        fac = next(f for _, kk, f in KERNELS if kk == k)
        e = {"source": os.path.basename(os.path.normpath(args.dir)), "src_hash": hashes.get(srchash.group_of(k))}
        if "FETCH_SIZE" in d:
            e["fetch_bytes"] = d["FETCH_SIZE"] * 1024 * fac
        if "WRITE_SIZE" in d:
            e["write_bytes"] = d["WRITE_SIZE"] * 1024
        if "fetch_bytes" in e and "write_bytes" in e:
            e["hbm_bytes_per_launch"] = e["fetch_bytes"] + e["write_bytes"]
        for c in ("SQ_INSTS_VALU", "SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"):
            if c in d:
                e[c.lower()] = d[c]
        out[k] = e
    # the LDE phase as one unit: sum of its kernels per commit.  Three-pass form: one inverse head,
    # one middle and one final pass; two-pass form: one inverse head + tail, one forward head +
    # tail (tail launches alternate inverse / forward)
    l3 = [out.get(k) for k in ("ct_head_inv", "lde3_mid", "lde3_final")]
    ct = [out.get(k) for k in ("ct_head_inv", "ct_head_fwd", "ct_tail")]
    if all(x and "hbm_bytes_per_launch" in x for x in l3):
        out["lde"] = {"hbm_bytes_per_launch": sum(x["hbm_bytes_per_launch"] for x in l3),
                      "note": "three-pass LDE: inverse head + middle + final, one commit",
                      "src_hash": hashes.get("lde")}
    elif all(x and "hbm_bytes_per_launch" in x for x in ct):
        out["lde"] = {"hbm_bytes_per_launch": ct[0]["hbm_bytes_per_launch"] + ct[1]["hbm_bytes_per_launch"]
                      + 2 * ct[2]["hbm_bytes_per_launch"], "note": "iNTT + forward, one commit",
                      "src_hash": hashes.get("lde")}
    full = {}
    if os.path.exists(args.out):
        full = json.load(open(args.out))
    full[args.config] = out
    with open(args.out, "w") as f:
        json.dump(full, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
