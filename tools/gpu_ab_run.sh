# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab21
for c in "LP118_2 MS L 0 50 0.1 262144" "LP118_2 MS L 0 50 0.05 262144" "LP118_2 BP L 4 100 0.05 131072"; do
  timeout -k 10 300 python tools/prof_sim.py $c > gpurun_out/${T}_sim.log 2>&1 || { tail -5 gpurun_out/${T}_sim.log; exit 1; }
  tail -1 gpurun_out/${T}_sim.log
done
