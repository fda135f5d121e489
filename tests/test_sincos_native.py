"""describe_kernel's double sincos of the float angle (orb_slam2_refactored_amd/csrc/sincos_f.h; mode d the
fdlibm form sincos_f2d that describe uses, mode t the round-5 table form sincos_f2d_tab)
against glibc's (float)::sin / ::cos((double)x), the functions ComputeOrbDescriptor calls
(ORBextractor.cc:105-107).  The header is plain IEEE double arithmetic built with
-ffp-contract=off, as in the library, so host and device compute the same bits.  Here every 97th
float in [0, 6.2832] (11.2 M values, < 1 s); `sincos_check 8 1` covers all 1,086,918,649 floats
of the range (run once: 0 mismatches).  Mode f checks sincosf_glibc (the ORBX_TRIG=float path, the
float overloads cosf / sinf) against glibc's sinf / cosf the same way (`sincos_check 8 1 f`: 0
mismatches on all 1,086,918,649 floats, with and without -ffp-contract=fast -mfma)."""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


import pytest


@pytest.mark.parametrize("mode", ["d", "t", "f"])
def test_sincos_matches_glibc(tmp_path, mode):
    exe = tmp_path / "sincos_check"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-pthread", str(ROOT / "tests" / "native" / "sincos_check.cpp"),
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "4", "97", mode], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "0 mismatches" in out.stdout, out.stdout + out.stderr
