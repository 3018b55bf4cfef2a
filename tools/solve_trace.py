"""Launch-level timeline of GN solve iterations from a rocprofv3 kernel trace
(tools/prof_solve_small.sh): for each solve (the launches from an
assemble/finalize kernel, or df_factor_kernel, to the back-substitution that
ends it) the kernels' start offsets and durations, averaged over the traced
iterations, and the idle gaps between consecutive launches.

usage: python tools/solve_trace.py gpurun_out/X/run_kernel_trace.csv"""
import csv
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))


def short(n):
    return n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


seq = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
seq = [s for s in seq if not s[2].startswith("at::") and "elementwise" not in s[2]]
starts = ("assemble_slots_kernel", "finalize_edges_kernel", "df_factor_kernel")
ends = ("col_backsub_kernel", "sparse_llt_kernel")
iters, cur = [], None
for s, e, n in seq:
    if cur is None and n.startswith(starts):
        cur = [(s, e, n)]
    elif cur is not None:
        if cur[-1][2].startswith("tail_pair_kernel") and not n.startswith(ends):
            iters.append(cur)  # the tail launch ran the back-substitution too (knob gcomb)
            cur = [(s, e, n)] if n.startswith(starts) else None
            continue
        if n.startswith(starts) and not cur[-1][2].startswith(starts):
            cur = [(s, e, n)]
            continue
        cur.append((s, e, n))
        if n.startswith(ends):
            iters.append(cur)
            cur = None
print(f"{len(iters)} solve iterations traced")
by = defaultdict(lambda: defaultdict(list))
spans, gaps_all = [], defaultdict(list)
for it in iters:
    t0 = it[0][0]
    spans.append((it[-1][1] - t0) / 1e3)
    for k, (s, e, n) in enumerate(it):
        by[(k, n)]["start"].append((s - t0) / 1e3)
        by[(k, n)]["dur"].append((e - s) / 1e3)
        if k:
            gaps_all[(k, n)].append((s - it[k - 1][1]) / 1e3)
for (k, n), d in sorted(by.items()):
    g = gaps_all.get((k, n), [0.0])
    print(f"  {k:2d} {n[:48]:48s} start +{statistics.median(d['start']):7.1f} us  dur {statistics.median(d['dur']):7.1f} us"
          f"  gap before {statistics.median(g):5.1f} us")
if spans:
    print(f"solve span (first launch start -> last end): median {statistics.median(spans):.1f} us")
