"""Scan device asm for MFMAs whose destination overlaps srcA / srcB (tools/kinfo-style .s files).
With -amdgpu-mfma-vgpr-form this compiler can assign D over a dying A / B operand; on gfx950
v_mfma_i32_16x16x64_i8 then returns wrong values (describe_kernel, round 3)."""
import re, sys


def rng(tok):
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return m.group(1), int(m.group(2)), int(m.group(3))
    m = re.match(r"([va])(\d+)$", tok)
    if m:
        return m.group(1), int(m.group(2)), int(m.group(2))
    return None


bad = 0
for path in sys.argv[1:]:
    fn = "?"
    for ln in open(path):
        t = ln.strip()
        if t.endswith(":") and not t.startswith((".", ";")):
            fn = t[:-1]
        if not t.startswith("v_mfma"):
            continue
        ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
        d = rng(ops[0])
        for src in ops[1:3]:
            s = rng(src)
            if d and s and d[0] == s[0] and not (d[2] < s[1] or s[2] < d[1]):
                bad += 1
                print(f"{path}: {fn}: {t}")
print("overlaps:", bad)
sys.exit(1 if bad else 0)
