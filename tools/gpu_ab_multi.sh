# interleaved A/B/C... of library builds (tools/build_variants.sh) on layered MS configs
# usage: bash tools/gpu_ab_multi.sh name1 name2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=""
for n in "$@"; do V="$V $n:QLDPC_LIB=qldpcsim_amd/_build/var_$n.so"; done
: > gpurun_out/ab_multi.jsonl
for cfg in "LP118_2 MS L 0.05 50 262144" "LP118_2 MS L None 50 65536" "LP118_0 MS L None 50 65536" "LP118_2 MS L 0.01 50 262144" "LP118_2 MS S 0.05 50 16384" "LP04_0 MS L 0.05 50 262144"; do
  timeout -k 10 300 python tools/ab_variants.py $cfg 2 $V >> gpurun_out/ab_multi.jsonl 2>> gpurun_out/ab_multi.err || exit $?
done
