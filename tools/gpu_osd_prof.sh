# OSD-heavy point: phase split and kernel durations (LP118_2 MS-L + OSD-0, p = 0.1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-osdprof}
mkdir -p gpurun_out
timeout -k 10 200 python tools/prof_sim.py LP118_2 MS L 0 50 0.1 65536 > gpurun_out/prof_sim_$TAG.jsonl 2> gpurun_out/prof_sim_$TAG.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o trace -- python3 tools/prof_sim.py LP118_2 MS L 0 50 0.1 65536 > gpurun_out/prof_$TAG.log 2>&1 || exit $?
