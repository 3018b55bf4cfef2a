"""Split a rocprofv3 kernel trace of `bench.py` by launch pattern (round 4,
verdict item 3): the packed linearize kernel's launches inside the drop-in
call (each followed by the solve's LLT launch) against the same kernel
launched back to back (neighbours are packed launches too), with the
gathering launch and the LLT beside them.

usage: python tools/prof_split.py DIR/.../run_kernel_trace.csv [bench.json]
(with the bench line, its in-call avg_launch_ms is printed beside the trace's)"""
import csv
import json
import statistics
import sys


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


rows = list(csv.DictReader(open(sys.argv[1])))
seq = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
seq = [s for s in seq if "at::" not in s[2] and "__amd_rocclr" not in s[2]]
groups = {"packed in-call": [], "packed back-to-back": [], "gather": [], "sparse_llt": []}
for i, (s, e, n) in enumerate(seq):
    d = (e - s) / 1e3
    if "linearize_packed_kernel" in n:
        prev_n = seq[i - 1][2] if i else ""
        next_n = seq[i + 1][2] if i + 1 < len(seq) else ""
        if "sparse_llt" in next_n:
            groups["packed in-call"].append(d)
        elif "linearize_packed_kernel" in prev_n and "linearize_packed_kernel" in next_n:
            groups["packed back-to-back"].append(d)
    elif "linearize_gather_kernel" in n:
        groups["gather"].append(d)
    elif "sparse_llt_kernel" in n:
        groups["sparse_llt"].append(d)
for k, v in groups.items():
    if v:
        print(f"{k:22s} launches {len(v):5d}  avg {statistics.mean(v):8.2f} us  median {statistics.median(v):8.2f}"
              f"  min {min(v):8.2f}  max {max(v):8.2f}")
if len(sys.argv) > 2:
    b = json.load(open(sys.argv[2]))
    r = b["roofline"]
    ic = statistics.mean(groups["packed in-call"]) if groups["packed in-call"] else float("nan")
    print(f"bench line: in-call avg_launch_ms {r['avg_launch_ms'] * 1e3:.2f} us (HIP events), back_to_back_ms "
          f"{r['back_to_back_ms'] * 1e3:.2f} us; trace in-call avg {ic:.2f} us "
          f"({(r['avg_launch_ms'] * 1e3 / ic - 1) * 100:+.1f}% events vs trace)")
