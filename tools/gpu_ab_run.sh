set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_simulator.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab1_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/ab1_pytest.log; exit 1; }
tail -2 gpurun_out/ab1_pytest.log
B=qldpcsim_amd/_build
timeout -k 10 600 python tools/ab_libs.py --rounds 3 --cfg "--schedule L --batch 262144" --cfg "--code LP118_2 --schedule L --p 0.05 --batch 262144" --cfg "--code LP118_2 --schedule L --batch 65536" --cfg "--schedule S --batch 65536" $B/var_base.so $B/var_filt.so 2>&1 | tee gpurun_out/ab1.jsonl || exit 1
for g in 2 4; do
QLDPC_MS_LANES_PER_CHECK=$g timeout -k 10 300 python tools/ab_libs.py --rounds 2 --cfg "--schedule L --batch 262144" --cfg "--code LP118_2 --schedule L --batch 65536" $B/var_filt.so 2>&1 | sed "s/^/G$g /" | tee -a gpurun_out/ab1.jsonl || exit 1
done
