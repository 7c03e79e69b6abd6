# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab43
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "layered" --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
# row / adjacency tables in global memory (8 waves per CU on LP118_2) vs LDS (6)
for cfg in "LP118_2 MS L 0.05 50 262144" "LP118_2 MS L None 50 65536" "LP118_2 MS L 0.1 50 131072" "LP118_2 MS L 0.02 50 262144"; do
  timeout -k 10 300 python -u tools/ab_env.py QLDPC_MS_GT=1/0 $cfg 3 >> gpurun_out/${T}_gt.log 2>&1 || { tail -20 gpurun_out/${T}_gt.log; exit 1; }
done
grep "{" gpurun_out/${T}_gt.log
