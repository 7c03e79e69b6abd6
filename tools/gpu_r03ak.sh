# round-3 GPU pass ak: layered VN eight variables per lane on layers of more than 256 variables
# (main) vs four (var_h4); layered parity, interleaved A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bits.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03ak_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r03ak_parity.log; [ $rc -eq 0 ] || exit $rc
B=qldpcsim_amd/_build
timeout -k 10 600 python -u tools/ab_libs.py --rounds 3 --cfg "--code LP118_2 --schedule L --p 0.05 --batch 262144 --io bytes" --cfg "--code LP118_2 --schedule L --p 0.1 --batch 65536 --io bytes" --cfg "--schedule L --batch 262144" $B/libqldpc_hip.so $B/var_h4.so > gpurun_out/r03ak_ab.json 2>&1 || { tail -5 gpurun_out/r03ak_ab.json; exit 1; }
cat gpurun_out/r03ak_ab.json
