# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab49
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_simulator.py tests/test_oracle_golden.py -x -q -m gpu -k "BP or bp" --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
B=$PWD/qldpcsim_amd/_build
# flooding BP: the stop-test barrier doubles as the CN -> VN barrier (new) vs HEAD
timeout -k 10 600 python -u tools/ab_libs.py --rounds 3 --cfg "--algo BP --iters 100 --batch 65536" --cfg "--algo BP --iters 100 --p 0.05 --batch 262144" $B/var_base.so $B/libqldpc_hip.so > gpurun_out/${T}_ab.log 2>&1 || { tail -20 gpurun_out/${T}_ab.log; exit 1; }
grep "{" gpurun_out/${T}_ab.log
