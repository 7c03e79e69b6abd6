# layered MS: parity at the working tree, then interleaved A/B of two library builds
# (tools/build_variants.sh) on the layered configurations.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
A=${1:-head}; B=${2:-new}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "MS or layered" --timeout 120 --timeout-method thread > gpurun_out/pytest_l2.log 2>&1 || exit $?
: > gpurun_out/ab_l2.jsonl
V="$A:QLDPC_LIB=qldpcsim_amd/_build/var_$A.so $B:QLDPC_LIB=qldpcsim_amd/_build/var_$B.so"
for cfg in "LP118_2 MS L 0.05 50 262144" "LP118_2 MS L None 50 65536" "LP118_0 MS L None 50 65536" "LP118_2 MS L 0.01 50 262144" "LP118_2 MS S 0.05 50 16384" "LP04_0 MS L 0.05 50 262144" "LP118_2 MS L 0.1 50 65536"; do
  timeout -k 10 300 python tools/ab_variants.py $cfg 3 $V >> gpurun_out/ab_l2.jsonl 2>> gpurun_out/ab_l2.err || exit $?
done
