"""Per-launch averages of the PMC passes of tools/pmc_bench.sh for one kernel
-> pmc/linearize_c3.json (bench.py reads hbm_bytes_per_launch as
roofline.traffic). Fabric read bytes = TCC_EA0_RDREQ_128B x 128 B + the other
(64 B) requests x 64 B, the gfx950 counting of MI355X_MICROARCH.md (a 128-B
request is tallied once); writes = TCC_EA0_WRREQ_64B x 64 B.

usage: python tools/pmc_summary.py gpurun_out/pmc [kernel-substring] [out.json] [kf] [merge-key]

With merge-key (e.g. "gather" for the first-iteration kernel "linearize_kernel": rocprofv3 reports names without template arguments, and "linearize_packed_kernel" does not contain it), the
summary is stored under that key of the existing out.json instead of replacing it.

The record carries the sha256 prefix of the library it was collected on and
the keyframe count; bench.py reports it as roofline.traffic only for that
same build and workload."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
kern = sys.argv[2] if len(sys.argv) > 2 else "linearize_packed_kernel"
out = sys.argv[3] if len(sys.argv) > 3 else "pmc/linearize_c3.json"
kf = int(sys.argv[4]) if len(sys.argv) > 4 else 32
merge = sys.argv[5] if len(sys.argv) > 5 else None
tot, disp = defaultdict(float), defaultdict(set)
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        c = r["Counter_Name"]
        tot[c] += float(r["Counter_Value"])
        disp[c].add((f, r["Dispatch_Id"]))
avg = {c: tot[c] / len(disp[c]) for c in tot}
rd128 = avg.get("TCC_EA0_RDREQ_128B_sum", 0.0)
rd = avg.get("TCC_EA0_RDREQ_sum", 0.0)
import hashlib  # noqa: E402

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
_lib = os.path.join(ROOT, "mast3r-slam-ysh_amd", "mast3r_slam_backends", "libm3s_gn.so")
res = {
    "lib_sha256_16": hashlib.sha256(open(_lib, "rb").read()).hexdigest()[:16],
    "kf": kf,
    "note": "C3 (calib, 98 directed edges x 262144 px). Per-launch averages from rocprofv3 --pmc passes over "
            "bench.py (tools/pmc_bench.sh, one counter group per run; tools/pmc_summary.py). Fabric bytes = "
            "TCC_EA0_RDREQ_128B_sum x 128 B + the 64-B requests x 64 B; writes = TCC_EA0_WRREQ_64B_sum x 64 B.",
    "kernel": kern,
    "hbm_bytes_per_launch": rd128 * 128 + (rd - rd128) * 64,
    "hbm_write_bytes_per_launch": avg.get("TCC_EA0_WRREQ_64B_sum", 0.0) * 64,
    "dispatches_per_counter": {c: len(v) for c, v in disp.items()},
    "counters": avg,
}
os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
if merge:
    base = json.load(open(out))
    base[merge] = res
    json.dump(base, open(out, "w"), indent=1)
else:
    json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: res[k] for k in ("hbm_bytes_per_launch", "hbm_write_bytes_per_launch")}))
