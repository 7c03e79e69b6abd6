# Stall attribution of one bench.py decode kernel per library build (GPU box):
# one --pmc pass of SQ wave-state counters per build, the same workload each.
# usage: bash tools/stall_profile.sh TAG "BENCH ARGS" LIB [LIB ...]
#        LIB = main (the in-tree build) or a name of qldpcsim_amd/_build/var_<name>.so
#        then python tools/stall_summary.py TAG  ->  gpurun_out/stall_TAG/summary.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; ARGS=$2; shift 2
SET="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
SET2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM"
D=gpurun_out/stall_$TAG
mkdir -p $D
echo "$ARGS" > $D/config.txt
for l in "$@"; do
  mkdir -p $D/$l
  [ $l = main ] && P=qldpcsim_amd/_build/libqldpc_hip.so || P=qldpcsim_amd/_build/var_$l.so
  B="python3 bench.py --gpus 1 --steps 1 --warmup 1 --cpu-seconds 0 --sim-legs= --hbm-leg 0 $ARGS"
  for k in 1 2; do
    [ $k = 1 ] && S=$SET || S=$SET2
    echo "[$l] pass $k"
    QLDPC_LIB=$P timeout -k 10 -s KILL 240 rocprofv3 --pmc $S --output-format csv -d $D/$l/p$k -o c -- $B --worklog $D/$l/p$k.work.json > $D/$l/p$k.log 2>&1 || { echo "$l pass $k failed rc=$?"; tail -5 $D/$l/p$k.log; exit 1; }
  done
done
python3 tools/stall_summary.py $TAG > $D/summary.json 2> $D/summary.err || { cat $D/summary.err; exit 1; }
cat $D/summary.json
