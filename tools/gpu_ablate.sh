set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in base 1 2; do
  if [ $v = base ]; then export QLDPC_LIB=$PWD/qldpcsim_amd/_build/libqldpc_hip.so; else export QLDPC_LIB=$PWD/qldpcsim_amd/_build/libqldpc_ablate$v.so; fi
  timeout -k 10 200 python bench.py --batch 262144 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/ablate_$v.log 2>&1 || exit $?
done
