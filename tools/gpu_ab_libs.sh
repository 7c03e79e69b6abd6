# parity of the default build (all MS paths), then interleaved A/B of library variants
# usage: bash tools/gpu_ab_libs.sh [--no-tests] name1 name2 ...  (qldpcsim_amd/_build/var_<name>.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$1" = "--no-tests" ]; then shift; else
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_simulator.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || exit $?
fi
B=qldpcsim_amd/_build
V=""
for n in "$@"; do V="$V $n:QLDPC_LIB=$B/var_$n.so"; done
timeout -k 10 900 python tools/ab_variants.py LP118_0 MS F None 50 1048576 3 $V > gpurun_out/ab_libs.jsonl 2> gpurun_out/ab_libs.err || exit $?
