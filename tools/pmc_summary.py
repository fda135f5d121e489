#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes: per kernel, the mean per-dispatch value of each counter."""
import re
import csv
import sys
from collections import defaultdict
from pathlib import Path


def collect(d):
    """{kernel: {counter: mean per-dispatch value}}"""
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(Path(d).rglob("run_counter_collection.csv")):
        per = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(f)):
            name = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].replace("orbamd::", "").replace("void ", ""))
            per[(name, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for (name, _), cs in per.items():
            for c, v in cs.items():
                acc[name][c].append(v)
    return {n: {c: sum(vs) / len(vs) for c, vs in cs.items()} for n, cs in acc.items()}


def main(d):
    for name, cs in sorted(collect(d).items()):
        print(name)
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {v:16.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
