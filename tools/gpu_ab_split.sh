# layered MS: parity, then interleaved A/B of G lanes per check (default choice)
# against one lane per check (QLDPC_MS_LANES_PER_CHECK=1 = "on").
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "MS or layered" --timeout 120 --timeout-method thread > gpurun_out/pytest_split.log 2>&1 || exit $?
: > gpurun_out/ab_split.jsonl
for cfg in "LP118_2 MS L 0.05 50 262144" "LP118_2 MS L None 50 65536" "LP118_0 MS L None 50 65536" "LP118_2 MS L 0.01 50 262144" "LP118_2 MS S 0.05 50 16384" "LP04_0 MS L 0.05 50 262144"; do
  echo "$cfg" >> gpurun_out/ab_split.jsonl
  timeout -k 10 300 python tools/ab_env.py QLDPC_MS_LANES_PER_CHECK $cfg 3 >> gpurun_out/ab_split.jsonl 2>> gpurun_out/ab_split.err || exit $?
done
