set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_osd.py tests/test_gpu_simulator.py -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_configs.py --osd > gpurun_out/osd.jsonl 2> gpurun_out/osd.err
