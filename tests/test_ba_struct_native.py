"""LocalBA's device-side structure build (round 6) against the host build, on the CPU.

tests/native/ba_struct_check.cpp runs the host half (csrc/ba_structure.h build_structure_counts) with an
emulation of the two fill kernels (orbba.hip ba_struct_slots_kernel, ba_struct_pairs_kernel) and
requires exactly build_structure's arrays (generic and point-sorted builds; the reference's
BlockSolver fill pattern, Thirdparty/g2o/g2o/core/block_solver.hpp:142-295) on 600 random point-sorted
graphs, and that unsorted edges or a point seeing a free pose twice are refused (the host build then
runs).  The GPU side of the same claim is tests/test_ba_gpu.py::test_local_ba_struct_forms_identical."""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_device_structure_build_matches_host(tmp_path):
    exe = tmp_path / "ba_struct_check"
    # (AddressSanitizer: an out-of-bounds store in the host build fails the run, not just its output)
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-I", str(ROOT / "orb_slam2_refactored_amd" / "csrc"),
                    str(ROOT / "tests" / "native" / "ba_struct_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "600"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "0 mismatches" in out.stdout, out.stdout + out.stderr
