# parity, then interleaved A/B of library variants on one config
# usage: bash tools/gpu_ab_cfg.sh CODE ALGO SCHED P ITERS BATCH name1 name2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_simulator.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || exit $?
C="$1 $2 $3 $4 $5 $6"; shift 6
V=""
for n in "$@"; do V="$V $n:QLDPC_LIB=qldpcsim_amd/_build/var_$n.so"; done
timeout -k 10 900 python tools/ab_variants.py $C 3 $V > gpurun_out/ab_cfg.jsonl 2> gpurun_out/ab_cfg.err || exit $?
