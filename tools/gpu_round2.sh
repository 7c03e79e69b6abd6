# Round-2 evidence on one GPU box: GPU test suite, smoke, headline bench (with
# the CPU baselines), then the counter profile bench.py's roofline reads.
# (+ configs table, simulate table, simulate kernel stats)
# usage: bash tools/gpu_round2.sh TAG [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu_$TAG.log
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; exit 1; }
fi
bash tools/gpu_profile_roofline.sh $TAG \
  flood "" \
  msl0 "--schedule L --batch 262144" \
  msl2 "--code LP118_2 --schedule L --p 0.05 --batch 262144" \
  bpf0 "--algo BP --iters 100 --batch 65536" \
  bpl2 "--code LP118_2 --algo BP --schedule L --iters 100 --p 0.05 --batch 131072" || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
# device OSD (configs[3] at p = 0.1): kernel stats of the block elimination
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/osd_$TAG -o t -- python3 tools/osd_bench.py LP118_2 MS L 50 0.1 131072 0 3 > gpurun_out/osd_$TAG.log 2>&1 || { echo "osd profile failed"; exit 1; }
tail -1 gpurun_out/osd_$TAG.log
# kernel-side configs table and end-to-end simulate_p table (device sampler + decode + OSD + counters)
timeout -k 10 400 python -u tools/bench_configs.py > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err || { echo "configs failed"; tail -5 gpurun_out/configs_$TAG.err; exit 1; }
timeout -k 10 600 python -u tools/bench_sim.py > gpurun_out/sim_$TAG.jsonl 2> gpurun_out/sim_$TAG.err || { echo "simulate failed"; tail -5 gpurun_out/sim_$TAG.err; exit 1; }
# kernel stats of the configs[3] simulate path (LP118_2 MS-L + OSD-0 p-sweep)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/simprof_$TAG -o t -- python3 tools/bench_sim.py 1048576 LP118_2:MS > gpurun_out/simprof_$TAG.log 2>&1 || { echo "simulate profile failed"; exit 1; }
echo "round evidence $TAG done"
