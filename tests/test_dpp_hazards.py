"""Build-time guard (CPU): no VALU-write -> DPP-read hazard in the device code.  The LocalBA solve's
diagonal-block pivots are generated inline asm (tools/gen_ba_diag.py) whose DPP broadcasts the
compiler's hazard recognizer does not see; a register-allocator copy placed right before one of
them silently corrupts the factorisation (found in round 3 with the split Linv registers).
tools/dpp_hazard_check.py scans the compiled listing."""
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "orb_slam2_refactored_amd" / "csrc"


@pytest.mark.parametrize("src", ["orbba.hip"])
def test_no_dpp_hazards(tmp_path, src):
    listing = tmp_path / (src + ".s")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
           f"-I{ROOT / 'include'}", f"-I{CSRC}", "--cuda-device-only", "-S", str(CSRC / src), "-o", str(listing)]
    if not Path(cmd[0]).exists():
        pytest.skip("hipcc not available")
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "dpp_hazard_check.py"), str(listing)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
