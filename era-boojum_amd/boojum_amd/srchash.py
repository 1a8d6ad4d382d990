"""Source hashes of the kernel groups the committed profiles measure.

Every library build (`__graft_entry__.build()` and `make -C era-boojum_amd`) writes them next to
the built library (build_info.json);
tools/pmc_summary.py stamps every PMC entry with the hash of its group, and bench.py uses a
committed traffic figure only while the two agree, so a profile can never be quoted for kernels
it did not measure (host logic only, no device call)."""
import hashlib
import json
import os

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")

_FIELD = ("gl.hpp", "gl_asm.hpp", "bj_internal.hpp")
GROUPS = {
    "leaf_hash_kernel": ("merkle.hip", "poseidon2.hpp", "poseidon2_rc.inc") + _FIELD,
    "node_level_kernel": ("merkle.hip", "poseidon2.hpp", "poseidon2_quad.hpp", "poseidon2_rc.inc") + _FIELD,
    "node_tail_kernel": ("merkle.hip", "poseidon2.hpp", "poseidon2_quad.hpp", "poseidon2_rc.inc") + _FIELD,
    "b2s_leaf_kernel": ("blake2s.hip",) + _FIELD,
    # the LDE phase: every NTT kernel source and the launch sequence that picks them
    "lde": ("ntt.hip", "ntt_ct.hip", "ntt_lde3.hip", "ntt_pow2.hpp", "ntt_dif.hip", "ntt_ct_common.hpp", "capi.hip") + _FIELD,
}


def group_of(kernel_key):
    """The hash group of a tools/pmc_summary.py kernel key."""
    if kernel_key == "lde" or kernel_key.startswith(("ct_", "dif_", "lde3_")):
        return "lde"
    if kernel_key == "node_level_q4_kernel":
        return "node_level_kernel"
    return kernel_key if kernel_key in GROUPS else None


def source_hashes(csrc=CSRC):
    out = {}
    for g, files in GROUPS.items():
        h = hashlib.sha256()
        for f in files:
            p = os.path.join(csrc, f)
            h.update(f.encode())
            if os.path.exists(p):
                with open(p, "rb") as fh:
                    h.update(fh.read())
        out[g] = h.hexdigest()[:16]
    return out


def write_build_info(path):
    with open(path, "w") as f:
        json.dump({"src_hash": source_hashes()}, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    import sys

    write_build_info(sys.argv[1])
