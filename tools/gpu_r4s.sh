set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_tracker.py -x -v --timeout 300 --timeout-method thread > $OUT/r4s_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/r4s_tests.log | head; tail -20 $OUT/r4s_tests.log; exit 1; }
tail -1 $OUT/r4s_tests.log
timeout -k 10 300 python -u tools/trk_ab.py variants/lib_trk_new3.so variants/lib_trk_new4.so > $OUT/r4s_ab.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/r4s_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/r4s_ab.txt
timeout -k 10 200 python -u tools/trk_stamps.py variants/lib_trkst.so > $OUT/r4s_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/r4s_stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/r4s_stamps.txt
