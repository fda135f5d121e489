"""Scan device asm for MFMAs whose destination overlaps the srcA / srcB registers of the same MFMA or
of an MFMA issued shortly before it in the same listing (still in flight: its passes read A / B while
the later product writes D).  With -amdgpu-mfma-vgpr-form this compiler can assign D over a dying
A / B operand; on gfx950 v_mfma_i32_16x16x64_i8 then returns wrong values now and then
(describe_kernel, rounds 3 and 4).  Usage: mfma_overlap.py listing.s ... (exit 1 if any)."""
import re
import sys

WINDOW = 24   # instructions after an MFMA during which its A / B registers count as in flight


def rng(tok):
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return m.group(1), int(m.group(2)), int(m.group(3))
    m = re.match(r"([va])(\d+)$", tok)
    if m:
        return m.group(1), int(m.group(2)), int(m.group(2))
    return None


def overlap(a, b):
    return a and b and a[0] == b[0] and not (a[2] < b[1] or b[2] < a[1])


bad = 0
for path in sys.argv[1:]:
    fn = "?"
    recent = []   # (instruction index, [A, B]) of recent MFMAs
    idx = 0
    for ln in open(path):
        t = ln.strip()
        m = re.match(r"([A-Za-z_][\w.$]*):", t)
        if m:
            fn, recent = m.group(1), []
            continue
        if not t or t.startswith((";", ".")):
            continue
        idx += 1
        if not t.startswith("v_mfma"):
            continue
        ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
        d = rng(ops[0])
        srcs = [rng(o) for o in ops[1:3]]
        recent = [(i, s) for i, s in recent if idx - i <= WINDOW]
        hit = any(overlap(d, s) for s in srcs) or any(overlap(d, s) for _, ss in recent for s in ss)
        if hit:
            bad += 1
            print(f"{path}: {fn[:90]}: {t}")
        recent.append((idx, srcs))
print("overlaps:", bad)
sys.exit(1 if bad else 0)
