"""CPU checks of compile-time invariants of the join kernels (hipcc front end
only, -fsyntax-only: no GPU, ~1 s each)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "mlir-hashjoin_amd")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _instantiate(tmp_path, inst):
    src = tmp_path / "inst.hip"
    src.write_text('#include "hj_radix.hip"\nnamespace hj { namespace { ' + inst + " } }\n")
    return subprocess.run([HIPCC, "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only",
                           "-I", os.path.join(os.path.dirname(HERE), "include"), "-I", os.path.join(PKG, "csrc"),
                           str(src)], capture_output=True, text=True, timeout=300)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_join_round_must_load_every_row(tmp_path):
    """round 5's dropped int64 shape (512 threads over a
    2048-slot table) lost one build row in five of every deferred partition
    (16,986 of 20,942 pairs on a 1-bit plan): k_join loads RI = RCAP / NT
    rows per thread per round but steps its run cursor by RCAP / 64 runs, and
    RCAP = 1280 is no multiple of 512.  The kernel now refuses such a shape at
    compile time; the product shapes compile."""
    bad = _instantiate(tmp_path, "template __global__ void k_join<true, true, 11, 512, 0, kJoinItems, 4, 0, true>(JoinArgs);")
    assert bad.returncode != 0
    assert "a build round must load exactly RCAP rows" in bad.stderr
    good = _instantiate(tmp_path, "template __global__ void k_join<true, true, kTableLog, 512, 0, kJoinItems, 4, 0, true>(JoinArgs);")
    assert good.returncode == 0, good.stderr[-2000:]
