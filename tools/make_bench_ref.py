"""profiles/<tag>_bench_ref.json: what bench.py reads from the round's committed profiles (the per-leg
rocprofv3 kernel summary and the k_select phase clocks) in one small JSON file. The GPU box's upload
skips profiles/*.csv and *.txt (.gpurunignore), so bench.py falls back to this file there.
usage: python3 tools/make_bench_ref.py <tag>   (reads profiles/<tag>_bench_kernel_stats.csv and
profiles/<tag>_select_stamps.txt)"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r05"
kfile = os.path.join("profiles", f"{tag}_bench_kernel_stats.csv")
sfile = os.path.join("profiles", f"{tag}_select_stamps.txt")
out = {"_what": "extract of " + kfile + " (the headline and roofline_kernel legs) and " + sfile + " (k_select cycles lines) for bench.py",
       "kernel_stats_source": kfile, "kernel_stats": [], "select_stamps_source": sfile, "select_stamps_lines": []}
with open(os.path.join(ROOT, kfile)) as fh:
    rows = list(csv.reader(l for l in fh if not l.startswith("#")))
for r in rows[1:]:
    if len(r) >= 4 and r[0] in ("fdbench:headline", "fdbench:roofline_kernel"):  # (the legs bench.py looks up)
        out["kernel_stats"].append([r[0], r[1], int(r[2]), float(r[3])])
with open(os.path.join(ROOT, sfile)) as fh:
    lines = fh.readlines()
for i, l in enumerate(lines):
    if l.startswith("k_select cycles:"):
        out["select_stamps_lines"] = [l.rstrip("\n")] + ([lines[i + 1].rstrip("\n")] if i + 1 < len(lines) else [])
        break
with open(os.path.join(ROOT, "profiles", f"{tag}_bench_ref.json"), "w") as fh:
    json.dump(out, fh, indent=1)
print(len(out["kernel_stats"]), "kernel rows,", len(out["select_stamps_lines"]), "stamp lines")
