#!/bin/bash
# PMC passes on refine_f16_kernel (bench.py's 512x512 matching pair through
# tools/refine_time.py): SQ instruction / wave figures, L2 fabric reads, L2
# hit rate, and the L1 (TCP) / TA counters this box offers (a pass runs only
# if every counter of it is in rocprofv3's list). One group per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-pmc_refine}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TA_BUSY_avr TA_TA_BUSY_sum" ; do
  i=$((i+1))
  ok=1
  for c in $grp; do grep -q "\b${c%_sum}\b\|\b${c%_avr}\b\|\b$c\b" $OUT/avail.txt || ok=0; done
  if [ $ok = 0 ]; then echo "pass $i skipped (not offered): $grp"; continue; fi
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex refine -T -d $OUT/p$i -o run --output-format csv -- python $R/tools/refine_time.py > $OUT/p$i.txt 2> $OUT/p$i.err || { echo "pass $i failed: $grp"; tail -5 $OUT/p$i.err; exit 1; }
  echo "pass $i done: $grp"
done
