# device sampler / counter kernels: tests, phase profile, end-to-end simulate table
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-chan}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_simulator.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit $?
for B in 262144; do
timeout -k 10 120 python tools/prof_sim.py LP118_0 MS F -1 50 0.01 $B >> gpurun_out/prof_sim_$TAG.jsonl 2>> gpurun_out/prof_sim_$TAG.err || exit $?
done
timeout -k 10 120 python tools/prof_sim.py LP118_2 MS L 0 50 0.05 65536 >> gpurun_out/prof_sim_$TAG.jsonl 2>> gpurun_out/prof_sim_$TAG.err || exit $?
timeout -k 10 900 python tools/bench_sim.py 262144 > gpurun_out/sim_$TAG.jsonl 2> gpurun_out/sim_$TAG.err || exit $?
