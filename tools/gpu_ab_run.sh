# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab40
# lanes per check on 17-32 / 17-64-row layers (LP118_0 32-row, LP118_2 30/60-row layers)
for cfg in "LP118_2 MS L 0.05 50 262144" "LP118_0 MS L None 50 262144" "LP118_2 MS L None 50 65536"; do
  for v in 32 64; do
    timeout -k 10 300 python -u tools/ab_env.py QLDPC_MS_G2_ROWS=$v $cfg 3 >> gpurun_out/${T}_g2.log 2>&1 || { tail -20 gpurun_out/${T}_g2.log; exit 1; }
  done
done
cat gpurun_out/${T}_g2.log | grep "{"
# occupancy sensitivity of the layered kernel (waves per workgroup = waves per CU here)
for w in 3 4 5; do
  timeout -k 10 300 python -u tools/ab_env.py QLDPC_WAVES_PER_WG=$w LP118_2 MS L 0.05 50 262144 2 >> gpurun_out/${T}_occ.log 2>&1 || { tail -20 gpurun_out/${T}_occ.log; exit 1; }
done
cat gpurun_out/${T}_occ.log | grep "{"
