#!/usr/bin/env python3
"""Static check of a gfx950 assembly listing for the VALU-write -> DPP-read hazard (a DPP source
VGPR read within 2 wait states of a VALU write of it), which the compiler's hazard recognizer does
not see when the DPP instruction sits in inline asm (orbba.hip's generated diagonal-block pivots)
and the register allocator puts a copy of the operand right before it.

usage: dpp_hazard_check.py listing.s [kernel-name-substring]
Wait states: 1 per instruction, N+1 per s_nop N.  Control flow: straight-line order (a label reached
by fall-through keeps the writes before it) plus every branch edge -- the registers written within 2
wait states before an s_branch / s_cbranch_* are still pending at its target label, one wait state
later (the branch itself), for forward and backward (loop) targets alike.  Exit status 1
when a hazard is found."""
import re
import sys

path = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
reg = re.compile(r"v\[(\d+):(\d+)\]|\bv(\d+)\b")
label_re = re.compile(r"^([.\w$]+):")
func_re = re.compile(r"^[A-Za-z_][\w.$]*:")


def regs(op):
    out = []
    for m in reg.finditer(op):
        if m.group(1):
            out += list(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.append(int(m.group(3)))
    return out


def functions(lines):
    """[(name, [stripped lines])] per function of the listing."""
    fns, cur = [], None
    for line in lines:
        s = line.strip()
        if func_re.match(s) and not s.startswith("."):
            cur = (s[:-1], [])
            fns.append(cur)
            continue
        if cur is not None:
            cur[1].append(s)
    return fns


def walk(body, incoming, report):
    """One pass over a function body.  incoming: label -> {vgpr: wait states already elapsed}.  Returns
    the branch edges found: label -> {vgpr: wait states elapsed at the target}."""
    edges = {}
    t = 0
    last_w = {}
    bad = 0
    for s in body:
        if not s or s.startswith(";"):
            continue
        m = label_re.match(s)
        if m:
            for r, ws in incoming.get(m.group(1), {}).items():   # pending writes of branches to this label
                last_w[r] = max(last_w.get(r, -10 ** 9), t - ws)
            continue
        if s.startswith("."):
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
                    report(f"hazard at '{s[:90]}' (v{r} written {t - last_w[r] - 1} wait states before)")
                    break
        if op == "s_branch" or op.startswith("s_cbranch"):
            target = parts[0]
            pend = {r: t - w for r, w in last_w.items() if t - w < 3}   # wait states since the write, branch included
            if pend:
                e = edges.setdefault(target, {})
                for r, ws in pend.items():
                    e[r] = min(e.get(r, 10 ** 9), ws)
        if op.startswith("v_") and not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")) and parts and parts[0]:
            for r in regs(parts[0]):
                last_w[r] = t
    return edges, bad


def main():
    bad = 0
    for name, body in functions(open(path)):
        if want and want not in name:
            continue
        edges, _ = walk(body, {}, lambda msg: None)           # pass 1: the branch edges
        _, nb = walk(body, edges, lambda msg: print(f"{name[:60]}: {msg}"))   # pass 2: with them
        bad += nb
    print(f"{path}: {bad} DPP hazard(s)")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
