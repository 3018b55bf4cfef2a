set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_tracker.py -x -v --timeout 300 --timeout-method thread > $OUT/r4u_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/r4u_tests.log | head; tail -20 $OUT/r4u_tests.log; exit 1; }
tail -1 $OUT/r4u_tests.log
timeout -k 10 300 python -u tools/trk_ab.py variants/lib_sh8.so variants/lib_sh4.so variants/lib_sh16.so > $OUT/r4u_ab.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/r4u_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/r4u_ab.txt
