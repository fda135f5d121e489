#!/usr/bin/env python3
"""Per-work-unit instruction counts from rocprofv3 PMC passes (tools/gpu_pmc.sh output directory):
fast_cells per 30x30 cell (the reference's ComputeKeyPointsOctTree grid, ORBextractor.cc:599-621:
border 16, cells of W = 30 px, 8 levels of 1/1.2), describe per wavefront (= per selection slot).
usage: pmc_percell.py <pmc dir> <frames> [cols rows]"""
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import collect  # noqa: E402

d, frames = sys.argv[1], int(sys.argv[2])
cols, rows = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (1280, 720)
cells = 0
for lv in range(8):
    s = 1.2 ** lv
    w, h = int(round(cols / s)), int(round(rows / s))
    cells += int((w - 32) / 30) * int((h - 32) / 30)
acc = collect(d)
print(f"{cols}x{rows}: {cells} cells per frame, {frames} frames")
for k, unit, n in (("fast_cells_kernel", "cell", cells * frames), ("describe_kernel", "wavefront", None)):
    if k not in acc:
        continue
    cs = acc[k]
    den = n if n else cs.get("SQ_WAVES", float("nan"))
    print(f"{k} per {unit} ({den:.0f} units):")
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_LDS_BANK_CONFLICT",
              "SQ_WAIT_INST_LDS"):
        if c in cs:
            print(f"   {c:22s} {cs[c] / den:10.1f}")
