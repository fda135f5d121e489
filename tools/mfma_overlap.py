"""Scan device asm for MFMAs whose destination overlaps the srcA / srcB registers of the same MFMA, or
the srcA / srcB / srcC registers of an MFMA issued shortly before it in the same listing (still in
flight: its passes read them while the later product writes D).  A diagnostic listing, not a gate: the
round-4 bisection (describe round 4) found these patterns benign -- the shipped describe and
matchers have them and are bit-deterministic -- while the empty-asm keep-alives that removed them made
describe's results differ between runs.  Usage: mfma_overlap.py listing.s ... (exit 1 if any)."""
import re
import sys

WINDOW = 16   # instructions after an MFMA during which its sources count as in flight (>= 4 cycles each: a
# 16-pass product, the longest here, is done 64 cycles after issue)


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
    recent = []   # (instruction index, [A, B, C], D, C written by an MFMA) of recent MFMAs
    wrote = []    # every MFMA D of the current function
    idx = 0
    for ln in open(path):
        t = ln.strip()
        m = re.match(r"([A-Za-z_][\w.$]*):", t)
        if m:
            fn, recent, wrote = m.group(1), [], []
            continue
        if not t or t.startswith((";", ".")):
            continue
        idx += 1
        if not t.startswith("v_mfma"):
            continue
        ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
        d = rng(ops[0])
        srcs = [rng(o) for o in ops[1:3]]
        c = rng(ops[3]) if len(ops) > 3 else None
        recent = [r for r in recent if idx - r[0] <= WINDOW]
        # D over its own A / B, or over the A / B / C of an earlier product still in flight (D == its
        # own C is the accumulate form and allowed)
        # (a product whose C is an earlier product's D waits for it: the chain is serialised, so the
        # earlier one and everything before it are no longer in flight)
        for k in range(len(recent) - 1, -1, -1):
            if overlap(c, recent[k][2]):
                recent = recent[k + 1:]
                break
        # (an in-flight C that an earlier product wrote is an accumulator chain the hardware orders:
        # the round-3 matchers run that pattern; a C from a VALU register, e.g. a shared initial value,
        # is flagged)
        hit = any(overlap(d, s) for s in srcs) or any(
            overlap(d, s) for _, ss, _, cw in recent for j, s in enumerate(ss) if not (j == 2 and cw))
        if hit:
            bad += 1
            print(f"{path}: {fn[:90]}: {t}")
        c_from_mfma = any(overlap(c, r[2]) for r in recent) or any(overlap(c, dd) for dd in wrote)
        recent.append((idx, srcs + [c], d, c_from_mfma))
        wrote.append(d)
print("overlaps:", bad)
sys.exit(1 if bad else 0)
