set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_backend.py tests/test_gpu_matching.py -x -q --timeout 300 --timeout-method thread > $OUT/r4m_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/r4m_tests.log | head; tail -20 $OUT/r4m_tests.log; exit 1; }
tail -1 $OUT/r4m_tests.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r4m_prof -o run -- python3 bench.py --no-cpu > $OUT/r4m_prof_bench.json 2> $OUT/r4m_prof_bench.err || { echo "prof failed"; tail -5 $OUT/r4m_prof_bench.err; exit 1; }
python3 tools/prof_split.py $(find $OUT/r4m_prof -name "*kernel_trace.csv" | head -1) $OUT/r4m_prof_bench.json | tee $OUT/r4m_prof_split.txt
timeout -k 10 400 python bench.py --no-cpu > $OUT/r4m_bench.json 2> $OUT/r4m_bench.err || { echo "bench failed"; tail -5 $OUT/r4m_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/r4m_bench.json')); r=d['roofline']; print('ms/step', d['ms_per_step'], 'pk', r['avg_launch_ms'], r['in_call_ms_min_max'], 'b2b', r['back_to_back_ms'], 'frac', r['frac'], 'gather', r['gather_kernel']['avg_launch_ms'], 'solve', r['solve']['avg_ms'])"
timeout -k 10 400 python -u -m pytest tests/test_gpu_backend.py -k "tail or warmup or block_dataflow" -x -q --timeout 200 --timeout-method thread > $OUT/r4m_tail.log 2>&1 || { echo "tail tests failed"; tail -20 $OUT/r4m_tail.log; exit 1; }
tail -1 $OUT/r4m_tail.log
SOLVE_AB="tail_pair=1|tail_pair=0" timeout -k 10 300 python -u tools/solve_ab.py > $OUT/r4m_solve_ab.txt 2>&1 || { echo "solve_ab failed"; tail -20 $OUT/r4m_solve_ab.txt; exit 1; }
grep -v amdgpu $OUT/r4m_solve_ab.txt
N=256 timeout -k 10 200 python -u tools/col_stamps.py variants/lib_colst.so > $OUT/r4m_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/r4m_stamps.txt; exit 1; }
grep -A30 "dense tail" $OUT/r4m_stamps.txt | head -24
