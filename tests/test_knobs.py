"""Experiment knobs stay out of the product path (CPU, no GPU; ABI 2.6).

The library's same-binary A/B switches (BJ_LEAVES_DEFER, BJ_LEAVES_GROUP, BJ_INV_FOLD_UNPAIRED, BJ_LDE_PASSES,
BJ_NODE_Q4_MAX, BJ_NODE_FUSED; csrc/bj_internal.hpp) are read from the environment only under BJ_EXPERIMENTS=1.
bj_experiment_knob is host-only, so a child process per environment loads the library and reads
the values in effect: without the gate every knob keeps its production value whatever the
environment says; with it the environment's values apply.  The reference's
transform_raw_storages_to_lde (cs/implementations/utils.rs:270-403) is a pure function of its
inputs, and the GPU tests check that every knob setting gives the same commitment
(tests/test_gpu_native_sharded.py::test_native_sharded_commit_env_knobs,
test_gpu_lde3.py::test_lde3_equals_two_pass_path, test_gpu_parity.py::test_node_levels_one_per_lane)."""
import json
import os
import subprocess
import sys

from test_abi import LIB

PRODUCTION = {"BJ_EXPERIMENTS": 0, "BJ_LEAVES_DEFER": 0, "BJ_LEAVES_GROUP": 0, "BJ_INV_FOLD_UNPAIRED": 0, "BJ_LDE_PASSES": 3,
              "BJ_NODE_Q4_MAX": 1 << 15, "BJ_NODE_FUSED": 1, "BJ_LDE_OWN_FUSED": 1}
SET = {"BJ_LEAVES_DEFER": "99", "BJ_LEAVES_GROUP": "3", "BJ_INV_FOLD_UNPAIRED": "1", "BJ_LDE_PASSES": "2", "BJ_NODE_Q4_MAX": "0",
       "BJ_NODE_FUSED": "0", "BJ_LDE_OWN_FUSED": "0"}

CODE = """
import ctypes, json, sys
L = ctypes.CDLL(sys.argv[1])
L.bj_experiment_knob.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]
out = {}
for k in %r:
    v = ctypes.c_uint64(12345)
    rc = L.bj_experiment_knob(k.encode(), ctypes.byref(v))
    out[k] = v.value if rc == 0 else rc
v = ctypes.c_uint64(0)
out["unknown_rc"] = L.bj_experiment_knob(b"BJ_NO_SUCH_KNOB", ctypes.byref(v))
print(json.dumps(out))
""" % (list(PRODUCTION),)


def knobs(extra):
    env = {k: v for k, v in os.environ.items() if not k.startswith("BJ_")}
    env.update(extra)
    r = subprocess.run([sys.executable, "-c", CODE, LIB], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def test_knobs_ignored_without_the_gate():
    got = knobs(dict(SET))
    assert {k: got[k] for k in PRODUCTION} == PRODUCTION
    assert got["unknown_rc"] == -22
    for gate in ("0", "yes", "11", ""):
        got = knobs(dict(SET, BJ_EXPERIMENTS=gate))
        assert {k: got[k] for k in PRODUCTION} == PRODUCTION, gate


def test_knobs_apply_under_the_gate():
    got = knobs(dict(SET, BJ_EXPERIMENTS="1"))
    assert got == {"BJ_EXPERIMENTS": 1, "BJ_LEAVES_DEFER": 99, "BJ_LEAVES_GROUP": 3, "BJ_INV_FOLD_UNPAIRED": 1, "BJ_LDE_PASSES": 2,
                   "BJ_NODE_Q4_MAX": 0, "BJ_NODE_FUSED": 0, "BJ_LDE_OWN_FUSED": 0, "unknown_rc": -22}
    # BJ_INV_FOLD_UNPAIRED is parsed, not only tested for presence
    got = knobs({"BJ_EXPERIMENTS": "1", "BJ_INV_FOLD_UNPAIRED": "0"})
    assert got["BJ_INV_FOLD_UNPAIRED"] == 0


def test_product_sources_read_no_knob_directly():
    # the one place that reads the environment for the schedule is bj_internal.hpp's read_knobs
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(root, "era-boojum_amd", "csrc")
    for name in os.listdir(csrc):
        text = open(os.path.join(csrc, name), errors="ignore").read()
        for knob in SET:
            if name != "bj_internal.hpp":
                assert 'getenv("%s")' % knob not in text, (name, knob)
