# round-3 GPU pass e: full GPU suite (pair-major tanh table, lift-16 flood
# layout), config throughput, A/B of the flood layouts, counter profile, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 tools/probe/simd_probe > gpurun_out/r03e_probe.log 2>&1; cat gpurun_out/r03e_probe.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03e_pytest.log 2>&1
rc=$?
tail -15 gpurun_out/r03e_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_configs.py > gpurun_out/r03e_configs.jsonl 2>&1 || { tail -5 gpurun_out/r03e_configs.jsonl; exit 1; }
cat gpurun_out/r03e_configs.jsonl
QLDPC_FLOOD_PLAIN=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/r03e_bench_plain.log 2>&1 || exit 1
tail -1 gpurun_out/r03e_bench_plain.log
bash tools/gpu_profile_roofline.sh r03e flood "" || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r03e_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r03e_bench.log; exit 1; }
tail -1 gpurun_out/r03e_bench.log
