set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 5 60 ./variants/ubench_diag7 2>&1 | tee $OUT/r4i_ubench_diag7.txt
timeout -k 5 60 ./variants/ubench_icache 2>&1 | tee $OUT/r4i_ubench_icache.txt
AB_CASES="calib:32:512:512:10:16:1003,calib:32:128:128:10:16,rays:256:12:16:3:16" timeout -k 10 400 python -u tools/ab_calls.py variants/lib_pre.so variants/lib_rsq.so variants/lib_cur.so > $OUT/r4i_ab.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/r4i_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/r4i_ab.txt | tail -8
timeout -k 10 600 python -u -m pytest tests/test_gpu_backend.py -x -q --timeout 300 --timeout-method thread > $OUT/r4i_backend.log 2>&1 || { echo "backend tests failed"; grep -E "FAILED|Error" $OUT/r4i_backend.log | head; tail -20 $OUT/r4i_backend.log; exit 1; }
tail -1 $OUT/r4i_backend.log
timeout -k 10 200 python -u tools/llt_stamps.py variants/lib_lst.so > $OUT/r4i_llt_stamps.txt 2>&1 || { echo "llt stamps failed"; tail -20 $OUT/r4i_llt_stamps.txt; exit 1; }
head -4 $OUT/r4i_llt_stamps.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_matching.py -x -q --timeout 200 --timeout-method thread > $OUT/r4i_match.log 2>&1 || { echo "match tests failed"; tail -30 $OUT/r4i_match.log; exit 1; }
tail -1 $OUT/r4i_match.log
for k in 2 1 0; do M3S_REFINE_STAGED=$k timeout -k 10 120 python -u tools/refine_time.py 2>&1 | grep -v amdgpu.ids; done
N=256 M3S_SUBTREE=0 timeout -k 10 200 python -u tools/col_stamps.py variants/lib_colst.so > $OUT/r4i_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/r4i_stamps.txt; exit 1; }
grep -A60 "pair kernel, waves" $OUT/r4i_stamps.txt
