# Counter profile for bench.py's roofline (GPU box). For each config: one
# kernel-trace --stats pass and one --pmc pass per counter set, each a separate
# short bench.py run (same seeds, so the same work) with its own worklog.
# usage: bash tools/gpu_profile_roofline.sh TAG NAME "BENCH ARGS" [NAME "BENCH ARGS" ...]
#        ("osd:ARGS" profiles tools/osd_bench.py ARGS instead of bench.py)
#        then (here or there) python tools/roofline_profile.py TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
PASSES=("FETCH_SIZE"
        "WRITE_SIZE"
        "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32"
        "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU"
        "SQ_INSTS_LDS_STORE SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE_BANDWIDTH SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS")
while [ $# -ge 2 ]; do
  NAME=$1; ARGS=$2; shift 2
  D=gpurun_out/roof_$TAG/$NAME
  mkdir -p $D
  echo "$ARGS" > $D/config.txt
  if [[ "$ARGS" == osd:* ]]; then
    BENCH="python3 tools/osd_bench.py ${ARGS#osd:}"
  else
    BENCH="python3 bench.py --gpus 1 --steps 2 --warmup 1 --cpu-seconds 0 $ARGS"
  fi
  echo "[$NAME] trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o t -- $BENCH --worklog $D/trace.work.json > $D/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 1; }
  i=0
  for set in "${PASSES[@]}"; do
    i=$((i+1))
    echo "[$NAME] pass $i: $set"
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $D/p$i -o c -- $BENCH --worklog $D/p$i.work.json > $D/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  done
done
python3 tools/roofline_profile.py $TAG > gpurun_out/roof_$TAG/summary.json 2> gpurun_out/roof_$TAG/summary.err || exit 1
