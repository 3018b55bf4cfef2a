#!/bin/bash
# GPU-box: the default bench line (with the CPU leg), then single-GPU bench
# lines at 64 / 128 / 256 keyframes (the graph sizes of the N-GPU weak-scaling
# runs, solved on one GPU). Any failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python bench.py > $OUT/bench_full.json 2> $OUT/bench_full.err || { echo "bench failed"; tail -5 $OUT/bench_full.err; exit 1; }
cat $OUT/bench_full.json
for n in ${NS:-64 128 256}; do
  timeout -k 10 240 python bench.py --kf-per-gpu $n --steps 3 --warmup 1 --no-cpu --no-tracker > $OUT/bench_n$n.json 2> $OUT/bench_n$n.err || { echo "bench n=$n failed"; tail -5 $OUT/bench_n$n.err; exit 1; }
  python - "$OUT/bench_n$n.json" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["config"]
print(c["keyframes"], "KF", c["directed_edges"], "edges:", d["value"], "pair-it/s,", d["gn_iters_per_s"], "GN it/s,",
      d["ms_per_step"], "ms/step, linearize", d["roofline"]["avg_launch_ms"], "ms")
EOF
done
