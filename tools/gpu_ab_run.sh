# ad-hoc GPU session (edited per experiment)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=ab56
B=$PWD/qldpcsim_amd/_build
QLDPC_LIB=$B/var_msl4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "layered" --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
# layered MS compiled for 4 waves per SIMD (<= 128 VGPRs) vs the compiler's choice
timeout -k 10 600 python -u tools/ab_libs.py --rounds 3 --cfg "--schedule L --batch 262144" --cfg "--code LP118_2 --schedule L --p 0.05 --batch 262144" --cfg "--schedule L --p 0.05 --batch 262144" $B/libqldpc_hip.so $B/var_msl4.so > gpurun_out/${T}_ab.log 2>&1 || { tail -20 gpurun_out/${T}_ab.log; exit 1; }
grep "{" gpurun_out/${T}_ab.log
