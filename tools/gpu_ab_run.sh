# ad-hoc GPU A/B session (edited per experiment): parity subset, then tools/ab_libs.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "layered" > gpurun_out/ab4_pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/ab4_pytest.log; exit 1; }
tail -2 gpurun_out/ab4_pytest.log
B=qldpcsim_amd/_build
C1="--schedule L --batch 262144"; C2="--code LP118_2 --schedule L --p 0.05 --batch 262144"; C3="--code LP118_2 --schedule L --batch 65536"; C4="--code LP04_0 --schedule L --batch 262144"
timeout -k 10 900 python tools/ab_libs.py --rounds 3 --cfg "$C1" --cfg "$C2" --cfg "$C3" --cfg "$C4" $B/var_cur.so $B/var_lg.so 2>&1 | tee gpurun_out/ab4.jsonl || exit 1
