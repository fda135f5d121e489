#!/usr/bin/env python3
"""Instruction stream of one kernel from a device .s listing (labels, directives and comments dropped):
tools/asm_body.py listing.s kernel_symbol_substring  -> prints the instructions.  Used to check that a
refactor leaves a kernel's code unchanged (diff two listings' bodies)."""
import sys


def body(path, name):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.split(":")[0] == name)
    out = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        t = l.split(";")[0].strip()
        if t and not t.startswith(".") and not t.endswith(":"):
            out.append(t)
    return out


def find_label(path, sub):
    for l in open(path):
        if not l.startswith((" ", "\t", ".", ";")) and ":" in l and sub in l.split(":")[0]:
            return l.split(":")[0]
    raise SystemExit(f"no kernel matching {sub} in {path}")


if __name__ == "__main__":
    lab = find_label(sys.argv[1], sys.argv[2])
    print("\n".join(body(sys.argv[1], lab)))
