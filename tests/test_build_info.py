"""build_info.json (written by every library build: __graft_entry__.build() and the Makefile) must
describe the sources in the tree: bench.py quotes a committed PMC traffic figure only while its
source hash equals build_info's, so a build_info left behind by an older build would let a stale
figure through (host logic only, no device call)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "era-boojum_amd"))

from boojum_amd import srchash  # noqa: E402

INFO = os.path.join(ROOT, "era-boojum_amd", "boojum_amd", "build_info.json")


def test_build_info_matches_sources():
    assert json.load(open(INFO))["src_hash"] == srchash.source_hashes(), \
        "build_info.json is stale: rebuild the library (make -C era-boojum_amd)"


def test_lde_group_covers_every_ntt_source():
    csrc = os.path.join(ROOT, "era-boojum_amd", "csrc")
    ntt = {f for f in os.listdir(csrc) if f.startswith("ntt")}
    assert ntt <= set(srchash.GROUPS["lde"]), ntt - set(srchash.GROUPS["lde"])


def test_stale_traffic_is_withheld():
    import bench
    stats = {"pmc": {"C3": {"lde": {"hbm_bytes_per_launch": 1.0, "src_hash": "a"},
                            "leaf_hash_kernel": {"hbm_bytes_per_launch": 2.0, "src_hash": "b"}}},
             "build": {"src_hash": {"lde": "a", "leaf_hash_kernel": "c"}}}
    assert bench.pmc_traffic(stats, "C3", "lde") == (1.0, False)
    assert bench.pmc_traffic(stats, "C3", "leaf_hash_kernel") == (None, True)
    assert bench.pmc_traffic(stats, "C4", "lde") == (None, None)


def test_census_matches_sources():
    """valu_census.json (the static slot counts bench.py's VALU rooflines use) was made from the
    kernels in the tree: build() stamps it and regenerates it when a hash differs."""
    census = json.load(open(os.path.join(ROOT, "era-boojum_amd", "boojum_amd", "valu_census.json")))
    assert census.get("src_hash") == srchash.source_hashes(), \
        "valu_census.json is stale: run __graft_entry__.build()"
