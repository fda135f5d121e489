#!/usr/bin/env python3
"""Static check of a gfx950 assembly listing for the VALU-write -> DPP-read hazard (a DPP source
VGPR read within 2 wait states of a VALU write of it), which the compiler's hazard recognizer does
not see when the DPP instruction sits in inline asm (orbba.hip's generated diagonal-block pivots)
and the register allocator puts a copy of the operand right before it.

usage: dpp_hazard_check.py listing.s [kernel-name-substring]
Walks each function in fall-through order (conservative across labels); wait states: 1 per
instruction, N+1 per s_nop N.  Exit status 1 when a hazard is found."""
import re
import sys

path = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
reg = re.compile(r"v\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(op):
    out = []
    for m in reg.finditer(op):
        if m.group(1):
            out += list(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.append(int(m.group(3)))
    return out


bad = 0
fn = None
t = 0
last_w = {}
for line in open(path):
    s = line.strip()
    if re.match(r"^[A-Za-z_][\w.$]*:", s) and not s.startswith("."):
        fn = s[:-1]
        last_w = {}
        t = 0
        continue
    if fn is None or not s or s.startswith((";", ".")) or s.endswith(":"):
        continue
    if want and want not in fn:
        continue
    op = s.split()[0]
    args = s[len(op):].split(";")[0]
    parts = [a.strip() for a in args.split(",")]
    if op == "s_nop":
        t += int(parts[0], 0) + 1
        continue
    t += 1
    if op.startswith("v_") and "_dpp" in op and len(parts) >= 2:
        for r in regs(parts[1]):
            if r in last_w and t - last_w[r] < 3:   # fewer than 2 wait states between
                bad += 1
                print(f"{fn[:60]}: hazard at '{s[:90]}' (v{r} written {t - last_w[r] - 1} wait states before)")
                break
    if op.startswith("v_") and not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")) and parts and parts[0]:
        for r in regs(parts[0]):
            last_w[r] = t
print(f"{path}: {bad} DPP hazard(s)")
sys.exit(1 if bad else 0)
