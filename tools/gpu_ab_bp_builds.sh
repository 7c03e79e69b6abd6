# BP: parity, then interleaved A/B of library builds (tools/build_variants.sh)
# usage: bash tools/gpu_ab_bp_builds.sh name1 name2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "BP" --timeout 120 --timeout-method thread > gpurun_out/pytest_bp.log 2>&1 || exit $?
V=""
for n in "$@"; do V="$V $n:QLDPC_LIB=qldpcsim_amd/_build/var_$n.so"; done
: > gpurun_out/ab_bp.jsonl
for cfg in "LP118_2 BP L 0.05 100 131072" "LP118_2 BP L None 100 16384" "LP118_0 BP L 0.05 100 262144" "LP118_2 BP L 0.1 100 32768"; do
  timeout -k 10 300 python tools/ab_variants.py $cfg 3 $V >> gpurun_out/ab_bp.jsonl 2>> gpurun_out/ab_bp.err || exit $?
done
