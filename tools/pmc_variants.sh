#!/bin/bash
# GPU-box: fabric read / write bytes of one linearize kernel for each library
# variant (tools/ab_linearize.py on ONE variant per rocprofv3 run, one counter
# group per run), summarised per variant. KREGEX picks the kernel
# (default the first-iteration gathering kernel).
# usage: bash tools/pmc_variants.sh variants/lib_A.so variants/lib_B.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-pmcvar}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  i=0
  for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    mkdir -p $OUT/$n
    timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-linearize_gather}" -d $OUT/$n/p$i -o run --output-format csv -- python $R/tools/ab_linearize.py $R/$lib > $OUT/$n/p$i.txt 2>&1 || { echo "pass $i of $n failed"; tail -5 $OUT/$n/p$i.txt; exit 1; }
  done
  python3 $R/tools/pmc_summary.py $OUT/$n "${KNAME:-linearize_gather_kernel}" $OUT/$n/summary.json 32 | sed "s/^/$n: /"
done
