set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_matching.py -x -q --timeout 200 --timeout-method thread > $OUT/r4k_match.log 2>&1 || { echo "match tests failed"; tail -30 $OUT/r4k_match.log; exit 1; }
tail -1 $OUT/r4k_match.log
M3S_REFINE_STAGED=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_matching.py -x -q --timeout 200 --timeout-method thread -k refine > $OUT/r4k_match0.log 2>&1 || { echo "match0 tests failed"; tail -30 $OUT/r4k_match0.log; exit 1; }
tail -1 $OUT/r4k_match0.log
for k in 4 0; do M3S_REFINE_STAGED=$k timeout -k 10 120 python -u tools/refine_time.py 2>&1 | grep -v amdgpu.ids; done
