# round-3 GPU pass j (re-entry): full GPU suite, smoke, headline bench at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r03j_pytest_gpu.log 2>&1
rc=$?; tail -6 gpurun_out/r03j_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03j_smoke.log 2>&1 || { tail -8 gpurun_out/r03j_smoke.log; exit 1; }
tail -3 gpurun_out/r03j_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r03j_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r03j_bench.log; exit 1; }
tail -1 gpurun_out/r03j_bench.log
