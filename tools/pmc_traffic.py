#!/usr/bin/env python3
"""Per-dispatch HBM-side traffic from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/gpu_traffic.sh).

FETCH_SIZE and WRITE_SIZE are reported in KiB.  The calibration program reads / writes a known
1 GiB per dispatch with 4-, 8- and 16-byte lane accesses; its ratios (counter bytes / true bytes)
are reported next to each extractor kernel's raw and calibration-corrected bytes per dispatch.
"""
import re
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

CALIB = 1 << 30


def per_dispatch(d, counter):
    acc = defaultdict(lambda: defaultdict(float))
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].replace("orbamd::", "").replace("void ", "")).replace("void ", "")
            acc[name][r["Dispatch_Id"]] += float(r["Counter_Value"]) * 1024.0   # KiB -> bytes
    return {k: sum(v.values()) / len(v) for k, v in acc.items()}


def main(src, dst, frames=128):
    src = Path(src)
    cf = per_dispatch(src / "calib_FETCH_SIZE", "FETCH_SIZE")
    cw = per_dispatch(src / "calib_WRITE_SIZE", "WRITE_SIZE")
    calib = {}
    for k, v in cf.items():
        if "read_kernel" in k:
            width = {"read_kernel<unsigned int>": 4, "read_kernel<HIP_vector_type<unsigned int, 2u> >": 8,
                     "read_kernel<HIP_vector_type<unsigned int, 4u> >": 16}.get(k, k)
            calib[f"fetch_ratio_{width}B"] = v / CALIB
    for k, v in cw.items():
        if "write_kernel" in k:
            calib["write_ratio_4B"] = v / CALIB
    kf = per_dispatch(src / "kb_FETCH_SIZE", "FETCH_SIZE")
    kw = per_dispatch(src / "kb_WRITE_SIZE", "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(kf) | set(kw)):
        if not any(s in k for s in ("pyramid", "fast_cells", "quadtree", "describe", "hamming")):
            continue
        kernels[k] = {"fetch_bytes": kf.get(k), "write_bytes": kw.get(k)}
    out = {"source": str(src), "calibration": calib, "kernels_per_dispatch": kernels,
           "workload": {"frames": int(frames), "width": 1280, "height": 720, "nfeatures": 2000,
                        "data": "tools/kbench.py --pan (bench.py's pan-sequence frames)" if int(frames) != 128
                        else "tools/kbench.py defaults (G frames)"}}
    Path(dst).write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(sys.argv[3:4]))
