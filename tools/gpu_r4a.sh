set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_backend.py -k "partial_trip or tiled or over_capacity or singular" -v -s --timeout 300 --timeout-method thread > $OUT/r4a_backend.log 2>&1 || { echo "backend tests failed"; tail -30 $OUT/r4a_backend.log; exit 1; }
tail -2 $OUT/r4a_backend.log
timeout -k 10 300 python bench.py --no-cpu --steps 10 > $OUT/r4a_bench.json 2> $OUT/r4a_bench.err || { echo "bench failed"; tail -30 $OUT/r4a_bench.err; exit 1; }
cat $OUT/r4a_bench.json
timeout -k 10 700 python -u -m pytest tests/test_gpu_large.py -k calib -v -s --timeout 650 --timeout-method thread > $OUT/r4a_large.log 2>&1 || { echo "large tests failed"; tail -30 $OUT/r4a_large.log; exit 1; }
grep -E "calib|PASS|FAIL" $OUT/r4a_large.log | tail -20
