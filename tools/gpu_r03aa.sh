# round-3 GPU pass aa: flood kernel prologue/epilogue with batched loads — parity, interleaved A/B vs HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bits.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03aa_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r03aa_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/ab_libs.py --rounds 3 --cfg "" --cfg "--p 0.01" --cfg "--code LP04_0 --p 0.05" qldpcsim_amd/_build/libqldpc_hip.so qldpcsim_amd/_build/var_head.so > gpurun_out/r03aa_ab.json 2>&1 || { tail -5 gpurun_out/r03aa_ab.json; exit 1; }
cat gpurun_out/r03aa_ab.json
