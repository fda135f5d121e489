#!/usr/bin/env python3
"""Static checks of a gfx950 listing around the MFMAs.

1. RAW: is every read of an MFMA's destination far enough behind the MFMA?  An XDL MFMA writes its D
   registers several cycles after issue; a VALU / memory / DPP / readlane read of D inside that window
   returns the OLD register contents (tools/probe/hazard_probe.hip, T5, measures the window on the
   hardware).  The compiler inserts the wait states itself -- except that it counts an inline asm
   statement as wait states even when the asm is empty, so an empty asm between an MFMA and the read
   of its result can leave the read inside the window.
   Wait states: 1 per instruction, N+1 per `s_nop N`; the empty-asm markers (`;;#ASMSTART` /
   `;;#ASMEND` with nothing between) count 0.  Control flow: straight-line order plus every branch edge
   (writes pending at a branch stay pending at its target, one wait state later), as
   tools/dpp_hazard_check.py does.  A VALU write of a pending register ends its window (later reads
   see the VALU's value).  Required wait states per MFMA shape: REQUIRED below.

2. LDS-load WAR (--war): an LDS load (ds_read / ds_load) whose destination overlaps a SrcA / SrcB /
   SrcC register of an MFMA issued within the previous WAR_WINDOW wait states.  This is the pattern of
   every describe build that gave different descriptor bits between identical runs (round 5,
   tools/diag/desc_determinism.py on 64 frames of 640 x 480, today's describe source):
     DESC_ANGLE_MFMA=0 (the LDS IC_Angle)   1022-1024 differing rows   3 loads at 0 / 5 / 10 wait states
     DESC_ANGLE_FIRST=1                     1018                        1 load at 0 wait states
     shipped, DESC_KEEPALIVE_DIAG, SINCOS_FMA_DIAG       0              none
   The register allocator reuses a source register of an MFMA it has just issued as the destination
   of the next fragment's LDS load (`v_mfma ... v[16:19] ...` then `ds_read_b128 v[18:21]`); the
   compiler's hazard recognizer inserts nothing, and the outcome depends on whether the load returns
   before the MFMA has read its operands.  The isolated hardware probe (hazard_probe T10 / T12, the
   exact angold sequence) did not reproduce it, and the i8 matcher (hamming_top2_mfma_kernel, the
   same pattern at 0-5 wait states) and the LocalBA solve (f64 MFMAs, 0-12) give exact, repeatable
   results (tools/diag/matcher_i8_war.py: 0 differences in 12 runs of 65536 x 2048 / 16384 x 4500).
   So the pattern is not by itself a hazard; it is a correlate of the two describe schedules that are,
   and describe is kept free of it as a precaution (tests/test_dpp_hazards.py).  Global loads
   (hundreds of cycles) are not counted.

usage: mfma_raw_check.py listing.s [kernel-substring] [--war]   (exit 1 on any finding)"""
import re
import sys

# wait states between an MFMA's issue and the first safe read of its D by (a VALU / DPP / readlane, a
# memory instruction).  The compiler's own spacing in this repository's listings, where no inline asm sits
# between (the smallest value for which its code has no violation): i8 and FP4 16x16 8, f64 16x16x4 19 / 18.
# hazard_probe T5 measures the hardware's window for the i8 shape.
REQUIRED = {
    "v_mfma_i32_16x16x64_i8": (8, 8),
    "v_mfma_scale_f32_16x16x128_f8f6f4": (8, 8),
    "v_mfma_f32_16x16x32_f16": (8, 8),
    "v_mfma_f64_16x16x4_f64": (19, 18),
}
DEFAULT_REQUIRED = (19, 19)
MEM_OPS = ("ds_", "buffer_", "global_", "flat_", "scratch_")
# an LDS load issued within this many wait states of an MFMA must not write that MFMA's sources
# (the nondeterministic builds have them at 0-10; the shipped kernels have none within 64)
WAR_WINDOW = 16

reg_re = re.compile(r"v\[(\d+):(\d+)\]|\bv(\d+)\b")
label_re = re.compile(r"^([.\w$]+):")
func_re = re.compile(r"^[A-Za-z_][\w.$]*:")


def regs(op):
    out = []
    for m in reg_re.finditer(op):
        if m.group(1):
            out += list(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.append(int(m.group(3)))
    return out


def functions(lines):
    fns, cur = [], None
    for line in lines:
        s = line.rstrip("\n")
        t = s.strip()
        if func_re.match(t) and not t.startswith("."):
            cur = (t[:-1], [])
            fns.append(cur)
            continue
        if cur is not None:
            cur[1].append(t)
    return fns


def ws_of(t):
    m = re.match(r"s_nop\s+(\d+)", t)
    return int(m.group(1)) + 1 if m else 1


def walk(body, incoming, report):
    """pending: vgpr -> (VALU wait states still required, mfma text, how many fewer a memory read needs).
    Returns the branch edges."""
    edges = {}
    pending = {}
    bad = 0
    in_asm, asm_count = False, 0
    for t in body:
        if t.startswith(";;#ASMSTART"):
            in_asm, asm_count = True, 0
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not t or t.startswith(";") or t.startswith("."):
            continue
        m = label_re.match(t)
        if m:
            for r, (need, src, d) in incoming.get(m.group(1), {}).items():
                if need > pending.get(r, (0, "", 0))[0]:
                    pending[r] = (need, src, d)
            continue
        code = t.split(";")[0].strip()
        if not code:
            continue
        op = code.split()[0]
        args = code[len(op):]
        parts = [p.strip() for p in args.split(",")] if args.strip() else []
        if op.startswith("v_mfma"):
            # an MFMA reading an in-flight D as A/B is a hazard too; as SrcC (same shape, chained) it is not
            srcs = parts[1:3]
            for p in srcs:
                for r in regs(p):
                    if r in pending:
                        if report:
                            print(f"  {code}  reads v{r} of `{pending[r][1]}` with {pending[r][0]} wait states left")
                        bad += 1
            step = ws_of(code)
            pending = {r: (n - step, s, d) for r, (n, s, d) in pending.items() if n - step > 0}
            need_valu, need_mem = REQUIRED.get(op, DEFAULT_REQUIRED)
            for r in regs(parts[0]) if parts else []:
                pending[r] = (need_valu, code, need_valu - need_mem)
            continue
        if pending and not op.startswith("s_"):
            # the first operand of a VALU op or a load is its destination; every operand of a store is read
            srcs = parts[1:] if op.startswith(("v_", "ds_read", "ds_load", "global_load", "buffer_load",
                                                "flat_load", "scratch_load")) else parts
            if op.startswith(("buffer_store", "global_store", "flat_store", "ds_write", "ds_store", "scratch_store")):
                srcs = parts
            mem = op.startswith(MEM_OPS)
            for p in srcs:
                for r in regs(p):
                    if r in pending:
                        left = pending[r][0] - (pending[r][2] if mem else 0)
                        if left <= 0:
                            continue
                        if report:
                            print(f"  {code}  reads v{r} of `{pending[r][1]}` with {left} wait states left")
                        bad += 1
        if pending and op.startswith("v_") and parts and not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
            for r in regs(parts[0]):   # a VALU result replaces the MFMA's value: later reads see it
                pending.pop(r, None)
        step = ws_of(code)
        pending = {r: (n - step, s, d) for r, (n, s, d) in pending.items() if n - step > 0}
        if op.startswith(("s_branch", "s_cbranch")) and parts:
            tgt = parts[-1]
            e = edges.setdefault(tgt, {})
            for r, (n, s, d) in pending.items():
                if n - 1 > e.get(r, (0, "", 0))[0]:
                    e[r] = (n - 1, s, d)
    return edges, bad


LOAD_OPS = ("ds_read", "ds_load")   # LDS loads: tens of cycles, inside an MFMA queue's operand reads


def war_loads(body, window, report):
    """LDS loads (asynchronous VGPR writes) whose destination overlaps a SrcA / SrcB / SrcC register of
    an MFMA issued within the previous `window` wait states (straight-line order; a label or branch ends
    the window).  Returns the count."""
    recent = []   # (wait states since issue, set of source vgprs, mfma text)
    bad = 0
    for t in body:
        if not t or t.startswith(";") or t.startswith("."):
            continue
        if label_re.match(t):
            recent = []
            continue
        code = t.split(";")[0].strip()
        if not code:
            continue
        op = code.split()[0]
        args = code[len(op):]
        parts = [p.strip() for p in args.split(",")] if args.strip() else []
        if op.startswith(LOAD_OPS) and parts:
            dst = set(regs(parts[0]))
            for age, srcs, txt in recent:
                hit = dst & srcs
                if hit:
                    bad += 1
                    if report:
                        print(f"  {code}  overwrites v{min(hit)} read by `{txt}` {age} wait states after its issue")
        step = ws_of(code)
        recent = [(a + step, s_, x) for a, s_, x in recent if a + step < window]
        if op.startswith("v_mfma") and len(parts) >= 4:
            srcs = set()
            for p in parts[1:4]:
                srcs |= set(regs(p))
            recent.append((0, srcs, code))
        if op.startswith(("s_branch", "s_cbranch", "s_setpc", "s_swappc")):
            recent = []
    return bad


def check(path, want="", war=False):
    total = 0
    for name, body in functions(open(path).read().splitlines()):
        if want and want not in name:
            continue
        incoming = {}
        for _ in range(4):   # propagate branch edges to a fixed point (loops)
            edges, _ = walk(body, incoming, False)
            if edges == incoming:
                break
            incoming = edges
        _, bad = walk(body, incoming, False)
        if bad:
            print(f"{name}: {bad} read(s) of an MFMA result inside its window")
            walk(body, incoming, True)
        wb = war_loads(body, WAR_WINDOW, False) if war else 0
        if wb:
            print(f"{name}: {wb} load(s) over the source of an MFMA in flight")
            war_loads(body, WAR_WINDOW, True)
        total += bad + wb
    return total


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--war"]
    n = check(args[0], args[1] if len(args) > 1 else "", "--war" in sys.argv)
    print(f"{n} MFMA-result read hazard(s)")
    sys.exit(1 if n else 0)
