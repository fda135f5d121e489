#!/usr/bin/env python3
"""Print the LocalBA kernel timeline of the last call in a rocprofv3 kernel trace directory."""
import re
import csv
import sys
from pathlib import Path

rows = []
for f in Path(sys.argv[1]).rglob("*kernel_trace.csv"):
    rows += list(csv.DictReader(open(f)))
rows = [r for r in rows if "ba_" in r["Kernel_Name"] or "copyBuffer" in r["Kernel_Name"] or "fillBuffer" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "ba_ctl_start" in r["Kernel_Name"]]
seq = rows[starts[-2]:] if len(starts) >= 2 else rows[-60:]
t0 = int(seq[0]["Start_Timestamp"])
prev = t0
tot = {}
for r in seq:
    n = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].replace("orbamd::", "").replace("void ", ""))
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if len(sys.argv) > 2:
        print(f"{n:28s} start {(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:7.1f}")
    tot[n] = tot.get(n, 0) + (e - s) / 1e3
    prev = e
print(f"span {(prev - t0) / 1e3:.1f} us")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {k:28s} {v:8.1f} us")
