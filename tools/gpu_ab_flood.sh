# flooding MS: parity, then interleaved A/B of library builds (tools/build_variants.sh)
# usage: bash tools/gpu_ab_flood.sh name1 name2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench.py -x -q -k "MS or bench" --timeout 120 --timeout-method thread > gpurun_out/pytest_flood.log 2>&1 || exit $?
V=""
for n in "$@"; do V="$V $n:QLDPC_LIB=qldpcsim_amd/_build/var_$n.so"; done
: > gpurun_out/ab_flood.jsonl
for cfg in "LP118_0 MS F None 50 1048576" "LP118_0 MS F 0.01 50 1048576" "LP118_0 MS F 0.05 50 1048576" "LP04_0 MS F 0.05 50 1048576" "LP118_2 MS F None 50 262144" "LP118_2 MS F 0.01 50 1048576"; do
  timeout -k 10 300 python tools/ab_variants.py $cfg 3 $V >> gpurun_out/ab_flood.jsonl 2>> gpurun_out/ab_flood.err || exit $?
done
