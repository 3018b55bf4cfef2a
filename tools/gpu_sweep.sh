#!/bin/bash
# GPU-box: single-GPU bench lines at the weak-scaling graph sizes (64 / 128 /
# 256 keyframes = the graphs of the 2 / 4 / 8-GPU runs, solved on one GPU),
# MODE=calib|rays. Prints GN it/s, ms/step and the per-launch linearize and
# solve times. Any failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${TAG:-sweep}
mkdir -p $OUT
cd $R
for n in ${NS:-64 128 256}; do
  timeout -k 10 240 python bench.py --kf-per-gpu $n --steps 3 --warmup 1 --cold-steps 2 --no-cpu --no-tracker --mode ${MODE:-calib} ${BENCH_ARGS:-} > $OUT/${TAG}_n$n.json 2> $OUT/${TAG}_n$n.err || { echo "bench n=$n failed"; tail -5 $OUT/${TAG}_n$n.err; exit 1; }
  python - "$OUT/${TAG}_n$n.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c, r = d["config"], d["roofline"]
print(c["keyframes"], "KF", c["directed_edges"], "edges:", d["gn_iters_per_s"], "GN it/s,", d["ms_per_step"],
      "ms/step (cold", d["cold"]["ms_per_step"], "), linearize", r["avg_launch_ms"], "ms, gather",
      r["gather_kernel"]["avg_launch_ms"], "ms, solve", r["solve"]["avg_ms"], "ms")
PY
done
