"""Per-kernel averages of the GN launches in a rocprofv3 kernel trace (the
torch bookkeeping kernels are left out), plus the launch sequence of one solve
iteration that runs the sparse LLT."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
seq = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


ours = [(s, e, short(n)) for s, e, n in seq if "anonymous namespace" in n and "at::" not in n]
agg = defaultdict(list)
for s, e, n in ours:
    agg[n].append((e - s) / 1e3)
for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{n[:60]:60s} calls {len(v):5d} avg {sum(v) / len(v):9.2f} us")
for i, (s, e, n) in enumerate(ours):
    if ("sparse_llt" in n or "col_backsub" in n) and i > len(ours) // 2:
        j = i
        while j > 0 and "linearize" not in ours[j][2]:
            j -= 1
        t0 = ours[j][0]
        print("one iteration:")
        for s2, e2, n2 in ours[j:i + 1]:
            print(f"  +{(s2 - t0) / 1e3:8.1f} us  {(e2 - s2) / 1e3:8.1f} us  {n2[:70]}")
        break
