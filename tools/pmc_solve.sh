#!/bin/bash
# PMC passes on the solve kernels (bench run, few steps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_solve
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_BRANCH" \
           "GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "sparse_llt" -T -d $OUT/p$i -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --no-cpu --no-tracker --lin-reps 2 > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed"; tail -3 $OUT/p$i.err; }
done
