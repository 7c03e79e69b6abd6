# round-3 GPU pass: tests, smoke, per-config throughput, counter list
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 120 --timeout-method thread > gpurun_out/r03b_pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/r03b_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03b_smoke.log 2>&1
cat gpurun_out/r03b_smoke.log
timeout -k 10 300 python -u tools/bench_configs.py > gpurun_out/r03b_configs.jsonl 2>&1
cat gpurun_out/r03b_configs.jsonl
rocprofv3 --list-avail > gpurun_out/r03b_avail.txt 2>&1 || true
