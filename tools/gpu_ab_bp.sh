# parity (all GPU tests), then BP configs A/B of two library variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || exit $?
: > gpurun_out/ab_bp.jsonl
for cfg in "LP118_0 BP F 0.05 100 262144" "LP118_0 BP F None 100 65536" "LP118_0 BP L 0.05 100 262144"; do
  timeout -k 10 600 python tools/ab_variants.py $cfg 2 "$1:QLDPC_LIB=qldpcsim_amd/_build/var_$1.so" "$2:QLDPC_LIB=qldpcsim_amd/_build/var_$2.so" >> gpurun_out/ab_bp.jsonl 2>> gpurun_out/ab_bp.err || exit $?
done
