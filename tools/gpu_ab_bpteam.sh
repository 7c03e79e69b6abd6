# parity (all GPU tests, default = BP team kernel W=4; BP tests again with W=8),
# then BP configs: team W=4 vs W=8 vs the one-wave kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || exit $?
QLDPC_BP_TEAM_W=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k BP --timeout 120 --timeout-method thread > gpurun_out/pytest_ab8.log 2>&1 || exit $?
: > gpurun_out/ab_bpteam.jsonl
for cfg in "LP118_0 BP F 0.05 100 262144" "LP118_0 BP F None 100 65536" "LP118_0 BP L 0.05 100 262144" "LP118_2 BP L 0.05 100 131072" "LP118_2 BP L 0.1 100 65536"; do
  timeout -k 10 900 python tools/ab_variants.py $cfg 2 team4 team8:QLDPC_BP_TEAM_W=8 wave:QLDPC_BP_WAVE=1 >> gpurun_out/ab_bpteam.jsonl 2>> gpurun_out/ab_bpteam.err || exit $?
done
