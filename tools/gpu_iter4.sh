set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x --durations=5 > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
