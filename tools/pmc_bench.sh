#!/bin/bash
# PMC passes on the linearize kernels (one counter group per rocprofv3 run),
# bench.py's roofline leg (packed kernel launches) plus its GN steps.
# BENCH_ARGS adds bench options (e.g. "--mode rays --kf-per-gpu 128"), TAG
# names the output directory.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 2 --warmup 1 --no-cpu --no-tracker --lin-reps 10 --cold-steps 0 ${BENCH_ARGS:-}"
i=0
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-linearize}" -T -d $OUT/p$i -o run --output-format csv -- python $R/bench.py $ARGS > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed: $grp"; tail -5 $OUT/p$i.err; exit 1; }
done
echo pmc done
