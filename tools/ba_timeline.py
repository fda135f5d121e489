#!/usr/bin/env python3
"""Print the LocalBA GPU timeline (kernels, and memory copies when traced) of the last complete call in
a rocprofv3 trace directory.  Usage: ba_timeline.py <dir> [v]  (v: every event with its gap and duration).
A call starts at the first of its host-to-device copies (the problem upload)."""
import csv
import re
import sys
from pathlib import Path

ev = []
for f in Path(sys.argv[1]).rglob("*kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "ba_" in n or "copyBuffer" in n or "fillBuffer" in n:
            n = re.sub(r"<[^>]*>$", "", n.split("(")[0].replace("orbamd::", "").replace("void ", ""))
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
for f in Path(sys.argv[1]).rglob("*memory_copy_trace.csv"):
    for r in csv.DictReader(open(f)):
        d = r.get("Direction", "") or r.get("Operation", "")
        n = "copy H2D" if "HOST_TO_DEVICE" in d else "copy D2H" if "DEVICE_TO_HOST" in d else "copy " + d
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
ev.sort()
have_copies = any(n.startswith("copy") for _, _, n in ev)
if have_copies:
    starts = [i for i in range(1, len(ev)) if ev[i][2] == "copy H2D" and ev[i - 1][2] != "copy H2D"]
    seq = ev[starts[-2]:starts[-1]] if len(starts) >= 2 else ev[-120:]
else:
    starts = [i for i, e in enumerate(ev) if "ba_ctl_start" in e[2]]
    seq = ev[starts[-2]:] if len(starts) >= 2 else ev[-60:]
t0 = seq[0][0]
prev = t0
tot, gaps = {}, 0.0
for s, e, n in seq:
    if len(sys.argv) > 2:
        print(f"{n:28s} start {(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:7.1f}")
    gaps += max(0, s - prev) / 1e3
    tot[n] = tot.get(n, 0) + (e - s) / 1e3
    prev = max(prev, e)
print(f"span {(prev - t0) / 1e3:.1f} us, idle gaps {gaps:.1f} us")
for n, t in sorted(tot.items(), key=lambda x: -x[1])[:12]:
    print(f"   {n:28s} {t:8.1f} us")
