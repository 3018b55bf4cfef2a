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
incall_idx, first_b2b = [], None
for i, (s, e, n) in enumerate(seq):
    d = (e - s) / 1e3
    if "linearize_packed_kernel" in n:
        prev_n = seq[i - 1][2] if i else ""
        next_n = seq[i + 1][2] if i + 1 < len(seq) else ""
        if "sparse_llt" in next_n:
            groups["packed in-call"].append(d)
            incall_idx.append(i)
        elif "linearize_packed_kernel" in prev_n and "linearize_packed_kernel" in next_n:
            groups["packed back-to-back"].append(d)
            if first_b2b is None:
                first_b2b = i
    elif "linearize_gather_kernel" in n:
        groups["gather"].append(d)
    elif "sparse_llt_kernel" in n:
        groups["sparse_llt"].append(d)
for k, v in groups.items():
    if v:
        print(f"{k:22s} launches {len(v):5d}  avg {statistics.mean(v):8.2f} us  median {statistics.median(v):8.2f}"
              f"  min {min(v):8.2f}  max {max(v):8.2f}")
# bench.py's roofline leg: 1 warm-up + 5 timed calls (9 packed launches each)
# right before its back-to-back run; their 45 in-call launches
leg = [(seq[i][1] - seq[i][0]) / 1e3 for i in incall_idx if first_b2b is not None and i < first_b2b][-45:]
if leg:
    print(f"{'roofline-leg in-call':22s} launches {len(leg):5d}  avg {statistics.mean(leg):8.2f} us  median "
          f"{statistics.median(leg):8.2f}  min {min(leg):8.2f}  max {max(leg):8.2f}  (the 5 timed calls before the "
          f"back-to-back run)")
if len(sys.argv) > 2:
    b = json.load(open(sys.argv[2]))
    r = b["roofline"]
    ic = statistics.mean(leg) if leg else statistics.mean(groups["packed in-call"])
    print(f"bench line: in-call avg_launch_ms {r['avg_launch_ms'] * 1e3:.2f} us, back_to_back_ms "
          f"{r['back_to_back_ms'] * 1e3:.2f} us; trace, the same calls: {ic:.2f} us "
          f"({(r['avg_launch_ms'] * 1e3 / ic - 1) * 100:+.1f}% bench vs trace)")
