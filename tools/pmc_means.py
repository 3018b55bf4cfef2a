"""Per-kernel means of every counter in the rocprofv3 --pmc passes under a
directory (tools/pmc_kernel.sh), plus the derived figures: fabric read / write
bytes (gfx950 counting, MI355X_MICROARCH.md: a 128-B read request tallied
once), VALU instructions per wave, and the busy fractions.

usage: python tools/pmc_means.py gpurun_out/TAG"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
tot, disp = defaultdict(float), defaultdict(set)
names = set()
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        names.add(k)
        c = (k, r["Counter_Name"])
        tot[c] += float(r["Counter_Value"])
        disp[c].add((f, r["Dispatch_Id"]))
for k in sorted(names):
    avg = {c: tot[(kk, c)] / len(disp[(kk, c)]) for (kk, c) in tot if kk == k}
    print(k)
    for c in sorted(avg):
        print(f"  {c:32s} {avg[c]:.4e}   ({len(disp[(k, c)])} dispatches)")
    rd, rd128 = avg.get("TCC_EA0_RDREQ_sum"), avg.get("TCC_EA0_RDREQ_128B_sum")
    if rd is not None and rd128 is not None:
        print(f"  fabric read bytes                {rd128 * 128 + (rd - rd128) * 64:.4e}")
    if "TCC_EA0_WRREQ_64B_sum" in avg:
        print(f"  fabric write bytes               {avg['TCC_EA0_WRREQ_64B_sum'] * 64:.4e}")
    if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
        print(f"  VALU instructions per wave       {avg['SQ_INSTS_VALU'] / avg['SQ_WAVES']:.1f}")
    if "SQ_WAIT_INST_ANY" in avg and "SQ_WAVE_CYCLES" in avg:
        print(f"  wait-inst / wave cycles          {avg['SQ_WAIT_INST_ANY'] / avg['SQ_WAVE_CYCLES']:.3f}")
    if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
        print(f"  VALU-active / wave cycles        {avg['SQ_ACTIVE_INST_VALU'] / avg['SQ_WAVE_CYCLES']:.3f}")
    if "TA_BUSY_avr" in avg and "GRBM_GUI_ACTIVE" in avg:
        print(f"  TA busy (avr / GUI_ACTIVE)       {avg['TA_BUSY_avr'] / avg['GRBM_GUI_ACTIVE']:.3f}")
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        print(f"  L2 hit rate                      {avg['TCC_HIT_sum'] / (avg['TCC_HIT_sum'] + avg['TCC_MISS_sum']):.3f}")
