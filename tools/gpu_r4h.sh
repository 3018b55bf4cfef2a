set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_matching.py -x -q --timeout 200 --timeout-method thread > $OUT/r4h_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/r4h_tests.log; exit 1; }
tail -2 $OUT/r4h_tests.log
timeout -k 10 120 python -u tools/refine_time.py 2>&1 | grep -v amdgpu.ids
M3S_REFINE_STAGED=0 timeout -k 10 120 python -u tools/refine_time.py 2>&1 | grep -v amdgpu.ids
