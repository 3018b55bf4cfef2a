set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 5 60 ./variants/ubench_diag7 2>&1 | tee $OUT/r4i_ubench_diag7.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_matching.py -x -q --timeout 200 --timeout-method thread > $OUT/r4i_match.log 2>&1 || { echo "match tests failed"; tail -30 $OUT/r4i_match.log; exit 1; }
tail -1 $OUT/r4i_match.log
for k in 2 1 0; do M3S_REFINE_STAGED=$k timeout -k 10 120 python -u tools/refine_time.py 2>&1 | grep -v amdgpu.ids; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_backend.py -x -q --timeout 300 --timeout-method thread > $OUT/r4i_backend.log 2>&1 || { echo "backend tests failed"; grep -E "FAILED|Error" $OUT/r4i_backend.log | head; tail -20 $OUT/r4i_backend.log; exit 1; }
tail -1 $OUT/r4i_backend.log
timeout -k 10 200 python -u tools/llt_stamps.py variants/lib_lst.so > $OUT/r4i_llt_stamps.txt 2>&1 || { echo "llt stamps failed"; tail -20 $OUT/r4i_llt_stamps.txt; exit 1; }
head -4 $OUT/r4i_llt_stamps.txt
timeout -k 10 400 python bench.py --no-cpu > $OUT/r4i_bench.json 2> $OUT/r4i_bench.err || { echo "bench failed"; tail -20 $OUT/r4i_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/r4i_bench.json')); print('ms/step', d['ms_per_step'], 'solve', d['roofline']['solve'], 'pk', d['roofline']['avg_launch_ms'], 'gather', d['roofline']['gather_kernel']['avg_launch_ms'], 'refine', d.get('matching_512'))"
