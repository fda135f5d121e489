#!/usr/bin/env python3
"""Extract the 256-pair rBRIEF sampling pattern (constant data) from the reference.

The reference holds the pattern as `bit_pattern_31_` in src/ORBextractor.cc:142-400
(the same table OpenCV's orb.cpp ships).  It is data, not code: 1024 small ints
(x0, y0, x1, y1 per pair).  This script parses the numbers out of that file and
writes them as a C include in our own layout, plus a checksum used by the tests.

Run in the build container (where /root/reference exists):
    python tools/extract_pattern.py
"""
import hashlib
import re
import sys
from pathlib import Path

REF = Path("/root/reference/src/ORBextractor.cc")
OUT = Path(__file__).resolve().parents[1] / "orb_slam2_refactored_amd" / "csrc" / "orb_pattern31.inc"


def parse(text: str):
    start = text.index("bit_pattern_31_[256 * 4]")
    body = text[text.index("{", start) + 1: text.index("};", start)]
    body = re.sub(r"/\*.*?\*/", " ", body, flags=re.S)
    vals = [int(v) for v in re.findall(r"-?\d+", body)]
    assert len(vals) == 1024, len(vals)
    return vals


def digest(vals):
    return hashlib.sha256(",".join(map(str, vals)).encode()).hexdigest()


def main():
    vals = parse(REF.read_text(errors="replace"))
    lines = ["// rBRIEF 31x31 sampling pattern: 256 pairs (x0,y0,x1,y1).",
             "// Data extracted by tools/extract_pattern.py from the reference",
             "// (src/ORBextractor.cc:142-400, bit_pattern_31_); sha256 of the",
             f"// comma-joined values: {digest(vals)}",
             "// Included inside an array initializer: { #include \"orb_pattern31.inc\" }"]
    for i in range(0, 1024, 16):
        lines.append("  " + ", ".join(f"{v:3d}" for v in vals[i:i + 16]) + ",")
    OUT.write_text("\n".join(lines) + "\n")
    print(OUT, digest(vals))


if __name__ == "__main__":
    sys.exit(main())
