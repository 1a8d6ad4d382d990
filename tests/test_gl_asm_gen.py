"""The committed csrc/gl_asm.hpp is exactly what tools/gen_gl_asm.py emits (CPU, no GPU): the
generator is the source of the hand-scheduled primitives, its docstrings explain them, and a
hand edit of the header would otherwise drift from them silently."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gl_asm_header_is_generated(tmp_path):
    out = tmp_path / "gl_asm.hpp"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_gl_asm.py"), "--out", str(out)], check=True,
                   capture_output=True)
    committed = open(os.path.join(ROOT, "era-boojum_amd", "csrc", "gl_asm.hpp")).read()
    assert out.read_text() == committed, "csrc/gl_asm.hpp differs from tools/gen_gl_asm.py's output"


def test_mi_layers_use_one_sum_chain_per_limb():
    # the chain counts the leaf microbenchmark chose (gen_gl_asm.py LAYER_A_CHAINS / LAYER_B_CHAINS)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_gl_asm
    assert (gen_gl_asm.LAYER_A_CHAINS, gen_gl_asm.LAYER_B_CHAINS) == (1, 1)
