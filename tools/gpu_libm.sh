set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_libm.py -q -m gpu > gpurun_out/pytest_libm.log 2>&1
