set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-osd2}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_simulator.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit $?
bash tools/gpu_osd_prof.sh $TAG
