# round-3 GPU pass ad: full GPU suite at HEAD, smoke, bench; configs[3] p = 0.1 end-to-end kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r03ad_pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r03ad_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ad_smoke.log 2>&1 || { tail -8 gpurun_out/r03ad_smoke.log; exit 1; }
tail -2 gpurun_out/r03ad_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r03ad_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r03ad_bench.log; exit 1; }
tail -1 gpurun_out/r03ad_bench.log | cut -c1-400
timeout -k 10 300 python -u tools/bench_configs.py --hbm > gpurun_out/r03ad_hbm.jsonl 2>&1 || { tail -5 gpurun_out/r03ad_hbm.jsonl; exit 1; }
