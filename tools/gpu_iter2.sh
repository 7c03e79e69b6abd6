# parity (MS flood subset) + headline bench with and without the register-table kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "MS and F" > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench.log 2>&1 || exit $?
QLDPC_NO_REGTAB=1 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_noreg.log 2>&1 || exit $?
