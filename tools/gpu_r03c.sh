# round-3 GPU pass c: HBM-resident kernel tests + throughput, then the full suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hbm.py -v --timeout 120 --timeout-method thread > gpurun_out/r03c_hbm.log 2>&1
rc=$?
tail -15 gpurun_out/r03c_hbm.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u tools/bench_configs.py --hbm > gpurun_out/r03c_hbm_bench.jsonl 2>&1
cat gpurun_out/r03c_hbm_bench.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 120 --timeout-method thread > gpurun_out/r03c_pytest_gpu.log 2>&1
tail -8 gpurun_out/r03c_pytest_gpu.log
