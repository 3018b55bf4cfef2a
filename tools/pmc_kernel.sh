#!/bin/bash
# PMC passes on one kernel (KREGEX) of a command: SQ instruction / wait /
# wave figures, TA and L1 (TCP) activity, L2 hits and fabric reads / writes.
# One counter group per rocprofv3 run; a group runs only if every counter of
# it is in rocprofv3's list on this box. Summaries: tools/pmc_summary.py-style
# means per counter (tools/pmc_means.py).
# usage: KREGEX=linearize_gather TAG=x bash tools/pmc_kernel.sh python tools/ab_linearize.py LIB
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-pmc_kernel}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" "TA_BUSY_avr TA_TA_BUSY_sum" ; do
  i=$((i+1))
  ok=1
  for c in $grp; do grep -q "\b${c%_sum}\b\|\b${c%_avr}\b\|\b$c\b" $OUT/avail.txt || ok=0; done
  if [ $ok = 0 ]; then echo "pass $i skipped (not offered): $grp"; continue; fi
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:?}" -T -d $OUT/p$i -o run --output-format csv -- "$@" > $OUT/p$i.txt 2> $OUT/p$i.err || { echo "pass $i failed: $grp"; tail -5 $OUT/p$i.err; exit 1; }
  echo "pass $i done: $grp"
done
python3 $R/tools/pmc_means.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
rm -f $OUT/avail.txt
