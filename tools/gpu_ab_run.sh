# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab48
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_simulator.py tests/test_oracle_golden.py -x -q -m gpu -k "BP or bp" --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
B=$PWD/qldpcsim_amd/_build
# layered BP stop test: parity filters (new) vs per-flip parity atomics (HEAD)
timeout -k 10 600 python -u tools/ab_libs.py --rounds 3 --cfg "--code LP118_2 --algo BP --schedule L --iters 100 --p 0.05 --batch 131072" --cfg "--code LP118_2 --algo BP --schedule L --iters 100 --p 0.1 --batch 65536" --cfg "--algo BP --schedule L --iters 100 --p 0.05 --batch 262144" --cfg "--algo BP --schedule L --iters 100 --batch 32768" $B/var_base.so $B/libqldpc_hip.so > gpurun_out/${T}_ab.log 2>&1 || { tail -20 gpurun_out/${T}_ab.log; exit 1; }
grep "{" gpurun_out/${T}_ab.log
