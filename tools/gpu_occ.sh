set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "4 1" "6 1" "8 1" "12 1" "6 2" "4 3"; do
  set -- $cfg
  QLDPC_WAVES_PER_WG=$1 QLDPC_WG_PER_CU=$2 timeout -k 10 200 python bench.py --batch 1048576 --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/occ_$1_$2.log 2>&1 || exit $?
done
