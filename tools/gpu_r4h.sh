set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_matching.py -x -q --timeout 200 --timeout-method thread > $OUT/r4h_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/r4h_tests.log; exit 1; }
tail -2 $OUT/r4h_tests.log
M3S_REFINE_STAGED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_matching.py -x -q --timeout 200 --timeout-method thread -k refine > $OUT/r4h_tests1.log 2>&1 || { echo "tests1 failed"; tail -30 $OUT/r4h_tests1.log; exit 1; }
tail -1 $OUT/r4h_tests1.log
for k in 2 1 0; do M3S_REFINE_STAGED=$k timeout -k 10 120 python -u tools/refine_time.py 2>&1 | grep -v amdgpu.ids; done
N=256 M3S_SUBTREE=0 timeout -k 10 200 python -u tools/col_stamps.py variants/lib_colst.so > $OUT/r4h_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/r4h_stamps.txt; exit 1; }
grep -A60 "pair kernel, waves" $OUT/r4h_stamps.txt
timeout -k 5 60 ./variants/ubench_diag7
