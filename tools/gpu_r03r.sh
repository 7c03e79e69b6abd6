# round-3 GPU pass r: bench with the HBM-streaming leg; bench GPU tests; configs[4] end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03r_bench_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03r_bench_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r03r_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r03r_bench.log; exit 1; }
tail -1 gpurun_out/r03r_bench.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['bound'], d['roofline']['frac'], json.dumps(d.get('hbm_streaming')))"
timeout -k 10 600 python -u tools/bench_sim.py 1048576 LP118_2:BP > gpurun_out/r03r_sim_bp.jsonl 2>&1 || { tail -5 gpurun_out/r03r_sim_bp.jsonl; exit 1; }
grep shots_per_s gpurun_out/r03r_sim_bp.jsonl | cut -c1-160
