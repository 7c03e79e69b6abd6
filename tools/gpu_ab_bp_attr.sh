# BP team kernel: compile-time knock-out attribution (fixed work, random syndromes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=""
for n in "$@"; do V="$V $n:QLDPC_LIB=qldpcsim_amd/_build/var_$n.so"; done
: > gpurun_out/ab_bp_attr.jsonl
for cfg in "LP118_2 BP L None 100 16384" "LP118_0 BP F None 100 65536" "LP118_2 BP L 0.05 100 131072"; do
  timeout -k 10 300 python tools/ab_variants.py $cfg 2 $V >> gpurun_out/ab_bp_attr.jsonl 2>> gpurun_out/ab_bp_attr.err || exit $?
done
