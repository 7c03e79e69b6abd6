# parity, then static vs dynamic half-shot scheduling on channel configs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_simulator.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || exit $?
: > gpurun_out/ab_queue.jsonl
for cfg in "LP118_0 MS F 0.01 50 1048576" "LP118_0 MS F 0.05 50 1048576" "LP118_0 MS F None 50 1048576" "LP118_2 MS L 0.05 50 262144" "LP118_0 BP F 0.05 100 262144"; do
  timeout -k 10 600 python tools/ab_variants.py $cfg 2 guided static:QLDPC_STATIC_SCHED=1 >> gpurun_out/ab_queue.jsonl 2>> gpurun_out/ab_queue.err || exit $?
done
