"""integration/rust/ffi.rs (the raw Rust binding a Boojum maintainer adds) is generated from
include/boojum_mi355x.h and must stay current: every declared entry point, nothing else."""
import os
import re
import subprocess
import sys

from test_abi import ROOT, declared_functions


def test_rust_ffi_is_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_rust_ffi.py"), "--check"])
    assert r.returncode == 0, "integration/rust/ffi.rs is stale: run python tools/gen_rust_ffi.py"


def test_rust_ffi_covers_the_header():
    text = open(os.path.join(ROOT, "integration", "rust", "ffi.rs")).read()
    names = re.findall(r"pub fn (bj_[a-z0-9_]+)\(", text)
    assert sorted(names) == declared_functions()
