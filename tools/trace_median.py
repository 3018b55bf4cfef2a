"""Median / min / max kernel durations (us) in a rocprofv3 kernel trace.

  python tools/trace_median.py DIR_OR_CSV [name-substring ...]"""
import csv
import glob
import os
import statistics
import sys

path = sys.argv[1]
if os.path.isdir(path):
    path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(path)))
names = sys.argv[2:] or sorted({r["Kernel_Name"].split("(")[0] for r in rows})
for n in names:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if n in r["Kernel_Name"]]
    if d:
        print(f"{n[:60]:60s} n {len(d):4d} median {statistics.median(d):9.2f} min {min(d):9.2f} max {max(d):9.2f} us")
