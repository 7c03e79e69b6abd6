set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python tools/bench_sim.py 262144 > gpurun_out/sim_pipe.jsonl 2> gpurun_out/sim_pipe.err || exit $?
