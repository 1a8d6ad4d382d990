#!/usr/bin/env python3
"""Attribute the per-rank compute of the G-way commit (rocprofv3 kernel traces of
tools/shard_compute_probe.py, scripts/shard_trace.sh) to kernels and launch gaps.

The probe makes 1 warm-up + 3 + 3 calls of bj_sharded_commit_d per config (the last three with
the phase events on).  Per config this prints, per kernel name, the time per call, and the
call's span on the compute queue against the sum of its kernels (the difference is gaps between
launches: grid drains, host-side waits).  Against G = 1, the G = 4 / 8 rows show each kernel's
time x G, so what a rank pays above 1/G of the one-GPU commit is attributed kernel by kernel.

usage: python tools/shard_trace_summary.py gpurun_out/TAG [--json out.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

CALLS = 7


def short(name):
    name = re.sub(r"^void ", "", name)
    name = name.replace("bj::(anonymous namespace)::", "").replace("(anonymous namespace)::", "").replace("bj::", "")
    name = re.sub(r"\(.*$", "", name)
    return name


def load(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        return None
    rows = list(csv.DictReader(open(f[0])))
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    ks.sort()
    return ks


def calls_of(ks):
    """Split the trace into the probe's calls: a call starts with the inverse head of its first
    column chunk (ct_head_kernel) right after the previous call's last node level (or after the
    synthetic-trace fill); the last CALLS such starts are the probe's calls."""
    ks = [k for k in ks if not k[2].startswith("__amd_rocclr")]
    starts = [i for i, k in enumerate(ks)
              if k[2].startswith("ct_head_kernel") and (i == 0 or not ks[i - 1][2].startswith(("ct_", "lde3_", "leaf_")))]
    starts = starts[-CALLS:]
    return "ct_head_kernel", [ks[a:b] for a, b in zip(starts, starts[1:] + [len(ks)])]


def summarize(ks):
    first, calls = calls_of(ks)
    per = collections.defaultdict(float)
    spans, busy = [], []
    for c in calls[1:4]:  # the headline calls (phase events off), after the warm-up
        for s, e, n in c:
            per[n] += (e - s) / 1e6 / 3
        spans.append((c[-1][1] - c[0][0]) / 1e6)
        busy.append(sum(e - s for s, e, _ in c) / 1e6)
    return {"first_kernel": first, "per_kernel_ms": dict(sorted(per.items(), key=lambda x: -x[1])),
            "span_ms": sum(spans) / len(spans), "kernels_ms": sum(busy) / len(busy),
            "launches_per_call": len(calls[0]) if calls else 0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    args = ap.parse_args()
    res = {}
    for G in (1, 4, 8):
        ks = load(os.path.join(args.dir, "G%d" % G))
        if ks:
            res[G] = summarize(ks)
    base = res.get(1)
    for G, r in res.items():
        print("G = %d: span %.2f ms per call, kernels %.2f ms, gaps %.2f ms, %d launches (x G: span %.2f)" % (
            G, r["span_ms"], r["kernels_ms"], r["span_ms"] - r["kernels_ms"], r["launches_per_call"],
            r["span_ms"] * G))
        for n, ms in r["per_kernel_ms"].items():
            b = base["per_kernel_ms"].get(n, 0.0) if base else 0.0
            print("   %-60s %8.3f ms  x G %8.2f  (G = 1: %8.2f)" % (n[:60], ms, ms * G, b))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
