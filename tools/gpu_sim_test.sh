set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_simulator.py tests/test_gpu_osd.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_sim.log 2>&1 || exit $?
timeout -k 10 900 python tools/bench_sim.py 262144 > gpurun_out/sim_pipe.jsonl 2> gpurun_out/sim_pipe.err || exit $?
