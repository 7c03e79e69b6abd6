# round-3 GPU pass ae: layered VN four variables per lane (main vs var_h2) and BP team
# prologue/epilogue with batched loads (var_h2 vs var_head) — parity, interleaved A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bits.py tests/test_gpu_simulator.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03ae_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r03ae_parity.log; [ $rc -eq 0 ] || exit $rc
B=qldpcsim_amd/_build
timeout -k 10 900 python -u tools/ab_libs.py --rounds 3 --cfg "--code LP118_2 --schedule L --p 0.05 --batch 262144 --io bytes" --cfg "--code LP118_2 --schedule L --p 0.1 --batch 65536 --io bytes" --cfg "--schedule L --batch 262144" --cfg "--code LP118_2 --algo BP --schedule L --iters 100 --p 0.01 --batch 131072 --io bits" --cfg "--code LP118_2 --algo BP --schedule L --iters 100 --p 0.05 --batch 131072 --io bits" --cfg "--algo BP --iters 100 --batch 65536" $B/libqldpc_hip.so $B/var_h2.so $B/var_head.so > gpurun_out/r03ae_ab.json 2>&1 || { tail -5 gpurun_out/r03ae_ab.json; exit 1; }
cat gpurun_out/r03ae_ab.json
