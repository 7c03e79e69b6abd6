set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/prof_sim.jsonl
for c in "LP118_2 MS L 0 50 0.1" "LP118_2 MS L 0 50 0.05" "LP118_0 MS F 0 50 0.1"; do
  timeout -k 10 300 python tools/prof_sim.py $c >> gpurun_out/prof_sim.jsonl 2>> gpurun_out/prof_sim.err || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_simulator.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_osd.log 2>&1 || exit $?
# >> gpurun_out/prof_sim.jsonl 2>> gpurun_out/prof_sim.err || exit $?
