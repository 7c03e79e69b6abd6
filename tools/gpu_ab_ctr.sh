# A/B of library variants + SQ counters of the first variant (headline config)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_ab_libs.sh --no-tests "$@" || exit $?
bash tools/gpu_counters.sh $1 QLDPC_LIB=qldpcsim_amd/_build/var_$1.so || exit $?
