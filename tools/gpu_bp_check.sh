# BP path after a libm change: GPU parity (bit-exact vs oracle), libm, configs table
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-bp}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_libm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit $?
timeout -k 10 600 python tools/bench_configs.py > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err || exit $?
