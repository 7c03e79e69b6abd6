# round-1 evidence: full GPU test suite, smoke, headline bench with CPU baseline,
# rocprofv3 kernel trace + stats, separate FETCH_SIZE / WRITE_SIZE PMC passes.
# usage: bash tools/gpu_round1_full.sh TAG   (outputs under gpurun_out/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o trace -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_prof.log 2>&1 || exit $?
timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$TAG -o pmc -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/bench_pmc_fetch.log 2>&1 || exit $?
timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$TAG -o pmc -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/bench_pmc_write.log 2>&1 || exit $?
bash tools/gpu_counters.sh $TAG || exit $?
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err || exit $?
timeout -k 10 900 python tools/bench_sim.py > gpurun_out/sim_$TAG.jsonl 2> gpurun_out/sim_$TAG.err || exit $?
