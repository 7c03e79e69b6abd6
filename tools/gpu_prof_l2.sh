set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for p in 0.01 0.02 0.05; do
timeout -k 10 120 python tools/prof_sim.py LP118_2 MS L 0 50 $p 262144 >> gpurun_out/prof_sim_l2.jsonl 2>> gpurun_out/prof_sim_l2.err || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_l2 -o trace -- python3 tools/prof_sim.py LP118_2 MS L 0 50 0.01 262144 > gpurun_out/prof_l2.log 2>&1 || exit $?
