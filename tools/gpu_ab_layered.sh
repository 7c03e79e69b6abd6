# MS kernels: parity, then interleaved A/B of two library builds on channel and fixed-work configs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
A=${1:-head}; B=${2:-new}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "MS" --timeout 120 --timeout-method thread > gpurun_out/pytest_abl.log 2>&1 || exit $?
V="$A:QLDPC_LIB=qldpcsim_amd/_build/var_$A.so $B:QLDPC_LIB=qldpcsim_amd/_build/var_$B.so"
for cfg in "LP118_0 MS F None 50 1048576" "LP118_0 MS F 0.01 50 1048576" "LP118_2 MS L 0.01 50 262144" "LP118_2 MS F None 50 262144"; do
timeout -k 10 600 python tools/ab_variants.py $cfg 3 $V >> gpurun_out/ab_layered.jsonl 2>> gpurun_out/ab_layered.err || exit $?
done
