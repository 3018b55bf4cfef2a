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

# per drop-in call (round 6, verdict item 5): a call starts at its
# gn_prologue_kernel; its kernels' summed durations against its wall span
# (first kernel start -> last kernel end) and the idle gap before the next
# call, for the C3 calls (10 solves each)
calls, cur = [], None
for s, e, n in seq:
    if "gn_prologue_kernel" in n:
        if cur:
            calls.append(cur)
        cur = []
    if cur is not None:
        cur.append((s, e, n))
if cur:
    calls.append(cur)
c3 = [c for c in calls if sum("sparse_llt" in n for _, _, n in c) == 10]
if c3:
    busy = [sum(e - s for s, e, _ in c) / 1e3 for c in c3]
    span = [(c[-1][1] - c[0][0]) / 1e3 for c in c3]
    nxt = [(calls[calls.index(c) + 1][0][0] - c[-1][1]) / 1e3 for c in c3 if calls.index(c) + 1 < len(calls)]
    print(f"C3 calls {len(c3)}: kernel time per call avg {statistics.mean(busy):8.1f} us (median "
          f"{statistics.median(busy):.1f}), wall span {statistics.mean(span):8.1f} us, idle to next call median "
          f"{statistics.median(nxt) if nxt else 0:.1f} us")
    per = {}
    for c in c3:
        for s, e, n in c:
            k = n.split("<")[0]
            per.setdefault(k, []).append((e - s) / 1e3)
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k:28s} per call {sum(v) / len(c3):8.1f} us  ({len(v) / len(c3):.0f} launches, avg "
              f"{statistics.mean(v):.2f} us)")
    if len(sys.argv) > 2:
        print(f"bench ms_per_step {b['ms_per_step'] * 1e3:.1f} us; roofline line spans x launches: "
              f"{(r['gather_kernel']['avg_launch_ms'] + (b['config']['gn_iters_per_step'] - 1) * r['avg_launch_ms'] + b['config']['gn_iters_per_step'] * r['solve']['avg_ms']) * 1e3:.1f} us")
