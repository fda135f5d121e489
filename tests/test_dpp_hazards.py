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


# the shipped build, plus the variants the A/B scripts build: SB_SPLIT_DEF (Schur-block parts) and a
# diagonal-pivot include generated with no Newton step after v_rcp_f64 (tools/gen_ba_diag.py 0)
VARIANTS = [("orbba.hip", []), ("orbba.hip", ["-DSB_SPLIT_DEF=8"]), ("orbba.hip", ["newton0"]), ("orbx.hip", []),
            ("orbm.hip", [])]
VGPR_FORM = ("orbx.hip", "orbm.hip")   # built with -amdgpu-mfma-vgpr-form, as the Makefile does


_LISTINGS = {}


def listing_of(tmp_dir, src, flags):
    """The device listing of src built as the Makefile builds it (plus flags), compiled once per session."""
    key = (src, tuple(flags))
    if key in _LISTINGS:
        return _LISTINGS[key]
    listing = tmp_dir / (src + "_".join(f.strip("-").replace("=", "") for f in flags) + ".s")
    extra = list(flags)
    if "newton0" in extra:
        inc = tmp_dir / "orbba_diag_n0.inc"
        subprocess.run([sys.executable, str(ROOT / "tools" / "gen_ba_diag.py"), "0", str(inc)], check=True,
                       capture_output=True, timeout=120)
        extra = [f'-DORBBA_DIAG_INC="{inc}"']
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
           f"-I{ROOT / 'include'}", f"-I{CSRC}", "--cuda-device-only", "-S", str(CSRC / src), "-o", str(listing)] + extra
    if src in VGPR_FORM:
        cmd += ["-mllvm", "-amdgpu-mfma-vgpr-form"]
    if not Path(cmd[0]).exists():
        pytest.skip("hipcc not available")
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    _LISTINGS[key] = listing
    return listing


@pytest.fixture(scope="module")
def lst_dir(tmp_path_factory):
    return tmp_path_factory.mktemp("listings")


@pytest.mark.parametrize("src,flags", VARIANTS, ids=["orbba", "orbba-sb8", "orbba-newton0", "orbx", "orbm"])
def test_no_dpp_hazards(lst_dir, src, flags):
    listing = listing_of(lst_dir, src, flags)
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "dpp_hazard_check.py"), str(listing)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr


@pytest.mark.parametrize("src,flags", [("orbx.hip", []), ("orbm.hip", []), ("orbba.hip", [])],
                         ids=["orbx", "orbm", "orbba"])
def test_no_mfma_hazards(lst_dir, src, flags):
    """Every shipped MFMA kernel: no read of an MFMA result inside its window (tools/mfma_raw_check.py)."""
    listing = listing_of(lst_dir, src, flags)
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "mfma_raw_check.py"), str(listing)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr


def test_describe_free_of_nondeterministic_pattern(lst_dir):
    """describe_kernel has no LDS load into a source register of an MFMA issued within 16 wait states:
    the schedule of both describe builds whose descriptors differed between identical runs on MI355X
    (DESC_ANGLE_MFMA=0 and DESC_ANGLE_FIRST=1: 1018-1024 differing rows per 64 frames; the shipped,
    keep-alive and fused-sincos builds: 0 and no such load).  A correlate, not a proven hazard (the i8
    matcher has it and is exact): DESIGN §4, describe round 5."""
    listing = listing_of(lst_dir, "orbx.hip", [])
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "mfma_raw_check.py"), str(listing), "describe_kernel",
                          "--war"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr


def test_mfma_checker_rejects_nondeterministic_describe(lst_dir):
    """The rule flags the build the determinism probe found nondeterministic (the LDS IC_Angle)."""
    listing = listing_of(lst_dir, "orbx.hip", ["-DDESC_ANGLE_MFMA=0"])
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "mfma_raw_check.py"), str(listing), "describe_kernel",
                          "--war"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 1 and "load(s) over the source of an MFMA in flight" in out.stdout, out.stdout


def test_mfma_overlap_checker(tmp_path):
    s = tmp_path / "t.s"
    s.write_text("k:\n\tv_mfma_i32_16x16x64_i8 v[2:5], v[2:5], v[18:21], 0\n"
                 "\tv_mfma_i32_16x16x64_i8 v[6:9], v[10:13], v[14:17], v[6:9]\n")
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "mfma_overlap.py"), str(s)], capture_output=True,
                         text=True, timeout=60)
    assert out.returncode == 1 and "overlaps: 1" in out.stdout, out.stdout


def test_checker_follows_branch_edges(tmp_path):
    """A VALU write 1 wait state before a branch reaches the DPP read at the target through the edge,
    even though the fall-through path pads it (the checker's round-3 blind spot)."""
    s = tmp_path / "t.s"
    s.write_text("kern:\n\tv_mov_b32 v2, v1\n\ts_cbranch_scc1 .L2\n\ts_nop 4\n.L2:\n"
                 "\tv_add_f64_dpp v[4:5], v[2:3], v[6:7] row_newbcast:1\n\ts_endpgm\n"
                 "ok:\n\tv_mov_b32 v2, v1\n\ts_cbranch_scc1 .L3\n\ts_nop 4\n.L3:\n\ts_nop 1\n"
                 "\tv_add_f64_dpp v[4:5], v[2:3], v[6:7] row_newbcast:1\n\ts_endpgm\n")
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "dpp_hazard_check.py"), str(s)], capture_output=True,
                         text=True, timeout=60)
    assert out.returncode == 1 and "kern:" in out.stdout and "ok:" not in out.stdout, out.stdout
