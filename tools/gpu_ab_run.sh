# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab57
B=$PWD/qldpcsim_amd/_build
QLDPC_LIB=$B/var_lg6.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "global_row_table" --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
# layered BP teams compiled for 5 / 6 waves per SIMD (LP118_0: 5-6 teams per CU) vs 4
timeout -k 10 600 python -u tools/ab_libs.py --rounds 3 --cfg "--algo BP --schedule L --iters 100 --p 0.05 --batch 262144" --cfg "--algo BP --schedule L --iters 100 --batch 32768" --cfg "--code LP118_2 --algo BP --schedule L --iters 100 --p 0.05 --batch 131072" $B/libqldpc_hip.so $B/var_lg5.so $B/var_lg6.so > gpurun_out/${T}_ab.log 2>&1 || { tail -20 gpurun_out/${T}_ab.log; exit 1; }
grep "{" gpurun_out/${T}_ab.log
