# kernel durations of the simulate loop phases (rocprofv3 kernel trace + stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-chanprof}
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o trace -- python3 tools/prof_sim.py LP118_0 MS F -1 50 0.01 262144 > gpurun_out/prof_$TAG.log 2>&1 || exit $?
