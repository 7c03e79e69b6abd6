# quick GPU iteration: parity tests + headline bench (no CPU baseline)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench.log 2>&1
