set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 5 60 ./variants/ubench_f64 > $OUT/r4j_ubench_f64.txt 2>&1; grep stores $OUT/r4j_ubench_f64.txt
AB_CASES="calib:32:512:512:10:16:1003,calib:32:128:128:10:16,rays:24:64:64:10:16,rays:256:12:16:3:16" timeout -k 10 500 python -u tools/ab_calls.py variants/lib_cur.so variants/lib_unroll.so variants/lib_early.so > $OUT/r4j_ab.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/r4j_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/r4j_ab.txt | tail -14
timeout -k 10 200 python -u tools/llt_stamps.py variants/lib_lst.so > $OUT/r4j_llt_stamps.txt 2>&1 || { echo "llt stamps failed"; tail -20 $OUT/r4j_llt_stamps.txt; exit 1; }
grep -v amdgpu $OUT/r4j_llt_stamps.txt | tail -26
timeout -k 10 600 python -u -m pytest tests/test_gpu_backend.py tests/test_gpu_ate.py -x -q --timeout 300 --timeout-method thread > $OUT/r4j_backend.log 2>&1 || { echo "backend tests failed"; grep -E "FAILED|Error" $OUT/r4j_backend.log | head; tail -20 $OUT/r4j_backend.log; exit 1; }
tail -1 $OUT/r4j_backend.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_matching.py -x -q --timeout 200 --timeout-method thread > $OUT/r4j_match.log 2>&1 || { echo "match tests failed"; tail -30 $OUT/r4j_match.log; exit 1; }
tail -1 $OUT/r4j_match.log
for k in 3 2 0; do M3S_REFINE_STAGED=$k timeout -k 10 120 python -u tools/refine_time.py 2>&1 | grep -v amdgpu.ids; done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r4j_prof -o run -- python3 bench.py --no-cpu > $OUT/r4j_prof_bench.json 2> $OUT/r4j_prof_bench.err || { echo "prof failed"; tail -5 $OUT/r4j_prof_bench.err; exit 1; }
python3 tools/prof_split.py $(find $OUT/r4j_prof -name "*kernel_trace.csv" | head -1) $OUT/r4j_prof_bench.json | tee $OUT/r4j_prof_split.txt
